// Sanitizer driver for the host side of libwam_hip.so (no reference counterpart):
// host-only plans (wam_plan_create_host) over odd, tiny, huge and invalid shapes, every level
// count, filter length and mode, then every host query the library answers from a plan -- band
// layout, reconstruction shape, workspace sizes, kernel capability checks (which run the fused
// kernels' geometry / LDS / ring predicates) and the split-sigma workspace size -- with invariants
// checked. Built by tests/native/build_sanitized.sh with AddressSanitizer and UndefinedBehavior-
// Sanitizer on the host code only (no GPU needed; compute entry points must refuse host plans).
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../include/wam_hip.h"

static int fails = 0, made = 0, with_caps = 0;
#define CHECK(c)                                                      \
  do {                                                                \
    if (!(c)) {                                                       \
      std::fprintf(stderr, "check failed line %d: %s\n", __LINE__, #c); \
      ++fails;                                                        \
    }                                                                 \
  } while (0)

static uint64_t rng_state = 0x9E3779B97F4A7C15ull;
static uint64_t rnd() {
  rng_state ^= rng_state << 13;
  rng_state ^= rng_state >> 7;
  rng_state ^= rng_state << 17;
  return rng_state;
}

static void probe(int ndim, const int64_t* shape, int levels, int L, int mode, int flags) {
  std::vector<double> f(L > 0 ? L : 1, 0.25);
  wam_plan* p = nullptr;
  const int rc = wam_plan_create_host(&p, ndim, shape, levels, f.data(), f.data(), f.data(), f.data(), L, mode, flags);
  if (rc != WAM_OK) {
    CHECK(p == nullptr);
    CHECK(wam_strerror(rc) != nullptr);
    return;
  }
  ++made;
  const int nb = wam_plan_num_bands(p);
  CHECK(nb == 1 + levels * ((1 << ndim) - 1));
  int64_t prev = -1, dims[3];
  for (int b = 0; b < nb; ++b) {
    const int64_t off = wam_plan_band_offset(p, b);
    CHECK(off > prev);
    prev = off;
    CHECK(wam_plan_band_shape(p, b, dims) == WAM_OK);
    for (int a = 0; a < ndim; ++a) CHECK(dims[a] >= 1);
  }
  CHECK(wam_plan_band_shape(p, nb, dims) != WAM_OK);   // out of range
  CHECK(wam_plan_band_shape(p, -1, dims) != WAM_OK);
  CHECK(wam_plan_coeff_numel(p) > prev);
  CHECK(wam_plan_rec_shape(p, dims) == WAM_OK);
  for (int a = 0; a < ndim; ++a) CHECK(dims[a] >= shape[a] && dims[a] <= shape[a] + 1);
  for (int64_t batch : {int64_t(0), int64_t(1), int64_t(7), int64_t(4800)}) CHECK(wam_plan_workspace_bytes(p, batch) >= 0);
  const int caps = wam_plan_caps(p);  // the fused kernels' support predicates
  CHECK((caps & ~(WAM_CAP_NOISY_WAVEDEC | WAM_CAP_ADJOINT_MAPS | WAM_CAP_BF16_NHWC)) == 0);
  // the bf16 hand-off needs the fused maps pass
  CHECK(!(caps & WAM_CAP_BF16_NHWC) || (caps & WAM_CAP_ADJOINT_MAPS));
  with_caps += caps != 0;
  // compute entry points refuse a host-only plan before touching any buffer
  float dummy[4] = {0, 0, 0, 0};
  CHECK(wam_wavedec(p, 1, dummy, dummy, dummy, nullptr) == WAM_ERR_INVALID_ARG);
  CHECK(wam_waverec_bf16_nhwc(p, 3, dummy, nullptr, 1, 3, dummy, nullptr) == WAM_ERR_INVALID_ARG);
  CHECK(wam_waverec_adjoint_maps_bf16_nhwc(p, 1, 1, 3, dummy, dummy, dummy, nullptr) == WAM_ERR_INVALID_ARG);
  CHECK(wam_waverec(p, 1, dummy, nullptr, 1, dummy, dummy, nullptr) == WAM_ERR_INVALID_ARG);
  CHECK(wam_waverec_adjoint(p, 1, dummy, dummy, dummy, nullptr) == WAM_ERR_INVALID_ARG);
  wam_plan_destroy(p);
}

int main() {
  const int Ls[] = {2, 4, 6, 8, 10, 12, 16, 20, 40, 128, 0, 3, 130};
  const int64_t edge[] = {1, 2, 3, 4, 5, 7, 8, 15, 16, 17, 33, 63, 64, 65, 127, 224, 255, 256, 257, 511, 512, 513,
                          4095, 80000, 1 << 20, int64_t(1) << 30, (int64_t(1) << 31) - 1, int64_t(1) << 31,
                          int64_t(1) << 40, -1, 0};
  const int ne = sizeof(edge) / sizeof(edge[0]);
  int n = 0;
  for (int ndim = 0; ndim <= 4; ++ndim)
    for (int levels : {0, 1, 2, 3, 5, 8, 16, 17})
      for (int L : Ls)
        for (int mode = -1; mode <= 5; ++mode)
          for (int k = 0; k < 6; ++k) {
            int64_t shape[3];
            for (int a = 0; a < 3; ++a) shape[a] = (k < 2) ? edge[(k * 7 + a * 3 + levels) % ne] : edge[rnd() % ne];
            const int flags = (int)(rnd() % 64);
            probe(ndim, shape, levels, L, mode, flags);
            ++n;
          }
  // the benchmark configurations (c1/c2 224^2, c4 512^2 sym8 J=5, c3 80,000-sample db6 J=5, c5 128^3
  // haar J=2) under every flag combination: the fused kernels' predicates on real geometries
  const int64_t s224[2] = {224, 224}, s512[2] = {512, 512}, s1[1] = {80000}, s3[3] = {128, 128, 128};
  for (int fl = 0; fl < 64; ++fl)
    for (int mode = 0; mode <= 4; ++mode) {
      probe(2, s224, 3, 8, mode, fl);
      probe(2, s224, 3, 2, mode, fl);
      probe(2, s512, 5, 16, mode, fl);
      probe(1, s1, 5, 12, mode, fl);
      probe(3, s3, 2, 2, mode, fl);
    }
  // null / invalid arguments
  CHECK(wam_plan_create_host(nullptr, 2, nullptr, 1, nullptr, nullptr, nullptr, nullptr, 2, 0, 0) != WAM_OK);
  CHECK(wam_plan_num_bands(nullptr) < 0);
  CHECK(wam_plan_caps(nullptr) == 0);
  CHECK(wam_item_sigma_ws_bytes(0, 5) == 0);
  CHECK(wam_item_sigma_ws_bytes(64, 150528) > 0);
  CHECK(wam_item_sigma_ws_bytes(1, int64_t(1) << 40) > 0);
  std::printf("plan_fuzz: %d random plans probed, %d plans created, %d with fused-kernel caps, %d failed checks\n",
              n, made, with_caps, fails);
  return fails ? 1 : 0;
}

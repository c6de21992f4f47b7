// Fused 3D Haar transforms for gfx950 (config c5: haar J=2 on 128^3 volumes).
//
// With the 2-tap Haar filters and dimensions divisible by 2^J no boundary extension is involved
// (p = 0, no odd-length pad), so a J-level 3D transform is local to 2^J x 2^J x 2^J blocks: one
// thread owns one block, reads it with 16-byte loads (lanes = consecutive blocks along W, so a
// wave reads whole contiguous rows), runs every level in registers and writes each band's patch
// (float2 runs at level 1 for J = 2, single values at the coarsest level). The per-axis kernels
// need 3 passes per level with intermediate volumes in HBM; this is one pass over the data.
// Arithmetic follows the per-axis kernels exactly (W then H then D; fmaf chains starting at 0),
// so results are bit-identical to the generic path.
#include "kernels.hpp"
#include "rng.hpp"

namespace {

constexpr int kT3 = 256;

struct Haar3Geom {
  int J;
  int64_t D, H, W;           // input dims
  int64_t off_a;             // per-item band offsets (band-major buffer with `items` items)
  int64_t off[2][7];         // [level][key - 1]
  int64_t items;
};

// one analysis level along one axis for a pair (x0, x1) -> (lo, hi)
__device__ __forceinline__ void ana2(float x0, float x1, const float (&f)[4], float& lo, float& hi) {
  lo = fmaf(f[1], x1, fmaf(f[0], x0, 0.f));
  hi = fmaf(f[3], x1, fmaf(f[2], x0, 0.f));
}

// 2x2x2 block v[z][y][x] -> 8 subbands indexed by key = (D hi) 4 | (H hi) 2 | (W hi) 1
__device__ __forceinline__ void haar3_level(const float (&v)[2][2][2], const float (&f)[4], float (&out)[8]) {
  float w[2][2][2];  // [z][y][W part]
#pragma unroll
  for (int z = 0; z < 2; ++z)
#pragma unroll
    for (int y = 0; y < 2; ++y) ana2(v[z][y][0], v[z][y][1], f, w[z][y][0], w[z][y][1]);
  float h[2][2][2];  // [z][H part][W part]
#pragma unroll
  for (int z = 0; z < 2; ++z)
#pragma unroll
    for (int wp = 0; wp < 2; ++wp) ana2(w[z][0][wp], w[z][1][wp], f, h[z][0][wp], h[z][1][wp]);
#pragma unroll
  for (int hp = 0; hp < 2; ++hp)
#pragma unroll
    for (int wp = 0; wp < 2; ++wp) {
      float lo, hi;
      ana2(h[0][hp][wp], h[1][hp][wp], f, lo, hi);
      out[(hp << 1) | wp] = lo;
      out[4 | (hp << 1) | wp] = hi;
    }
}

// synthesis of one axis: (a, d) -> (y0, y1) = (rlo0 a + rhi0 d, rlo1 a + rhi1 d) in the
// per-axis kernel's order
__device__ __forceinline__ void syn2(float a, float d, const float (&r)[4], float& y0, float& y1) {
  y0 = fmaf(r[2], d, fmaf(r[0], a, 0.f));
  y1 = fmaf(r[3], d, fmaf(r[1], a, 0.f));
}

// 8 subbands (key order) -> 2x2x2 block; synthesis passes W, then H, then D
__device__ __forceinline__ void haar3_inv(const float (&c)[8], const float (&r)[4], float (&v)[2][2][2]) {
  float w[2][2][2];  // [D part][H part][x]
#pragma unroll
  for (int dp = 0; dp < 2; ++dp)
#pragma unroll
    for (int hp = 0; hp < 2; ++hp) syn2(c[(dp << 2) | (hp << 1)], c[(dp << 2) | (hp << 1) | 1], r, w[dp][hp][0],
                                        w[dp][hp][1]);
  float h[2][2][2];  // [D part][y][x]
#pragma unroll
  for (int dp = 0; dp < 2; ++dp)
#pragma unroll
    for (int x = 0; x < 2; ++x) syn2(w[dp][0][x], w[dp][1][x], r, h[dp][0][x], h[dp][1][x]);
#pragma unroll
  for (int y = 0; y < 2; ++y)
#pragma unroll
    for (int x = 0; x < 2; ++x) syn2(h[0][y][x], h[1][y][x], r, v[0][y][x], v[1][y][x]);
}

// NOISE: SmoothGrad sample generation fused into the load (single-channel volumes): output item
// s * images + i is the transform of x_i + sigma_i * N(0,1) with the Philox stream of
// wam_noise_add (counter (sample_base + s, image_base + i, element / 4)); a B-wide row of a block
// is one (B = 4) or half a (B = 2) group of 4 elements, so noise costs one Philox call per row.
// Work order (NOISE): workgroup w takes sample w % S of a 256-block chunk of image w / S, so the S
// samples of a chunk are consecutive (XCD-swizzled) workgroups and read the clean chunk from one L2.
template <int J, bool NOISE>
__global__ void __launch_bounds__(kT3) k_haar3_ana(const float* __restrict__ in, float* __restrict__ coeffs,
                                                  const float* __restrict__ filt, Haar3Geom g, int64_t blocks,
                                                  WamNoise nz, int64_t S) {
  constexpr int B = 1 << J;
  const int64_t bw = g.W / B, bh = g.H / B, bd = g.D / B;
  const int64_t nb = bw * bh * bd;  // blocks per volume
  int64_t t, item, src_item, smp = 0;
  float sg = 0.f;
  if constexpr (NOISE) {
    const int64_t nc = (nb + kT3 - 1) / kT3;  // workgroup chunks per volume
    const int64_t w = wam_xcd_block(blockIdx.x, gridDim.x);
    const int64_t s = w % S, rest = w / S, i = rest / nc;
    t = (rest % nc) * kT3 + threadIdx.x;
    if (t >= nb || i >= nz.images) return;
    src_item = i;
    item = s * nz.images + i;
    smp = nz.sample_base + s;
    sg = nz.sigma[i];
  } else {
    const int64_t tt = (int64_t)blockIdx.x * kT3 + threadIdx.x;
    if (tt >= blocks) return;
    t = tt % nb;
    item = src_item = tt / nb;
  }
  const int64_t bx = t % bw, by = (t / bw) % bh, bz = t / (bw * bh);
  float f[4] = {filt[0], filt[1], filt[2], filt[3]};  // lo0 lo1 hi0 hi1
  float v[B][B][B];
  const float* src = in + src_item * g.D * g.H * g.W + (bz * B * g.H + by * B) * g.W + bx * B;
#pragma unroll
  for (int z = 0; z < B; ++z)
#pragma unroll
    for (int y = 0; y < B; ++y) {
      const float* row = src + ((int64_t)z * g.H + y) * g.W;
      if constexpr (B == 4) {
        const float4 q = *reinterpret_cast<const float4*>(row);
        v[z][y][0] = q.x;
        v[z][y][1] = q.y;
        v[z][y][2] = q.z;
        v[z][y][3] = q.w;
      } else {
        const float2 q = *reinterpret_cast<const float2*>(row);
        v[z][y][0] = q.x;
        v[z][y][1] = q.y;
      }
    }
  if constexpr (NOISE) {
    // element group of row (z, y): ((bz B + z) H + by B + y) W / 4 + bx B / 4 (W % 4 == 0, host check)
    const uint32_t W4 = (uint32_t)(g.W / 4);
    const uint32_t g0 = (uint32_t)(bz * B * g.H + by * B) * W4 + (uint32_t)(bx * B / 4);
    const uint32_t img = (uint32_t)(nz.image_base + src_item), sm = (uint32_t)smp;
#pragma unroll
    for (int r = 0; r < B * B; r += 2) {
      const int z0 = r / B, y0 = r % B, z1 = (r + 1) / B, y1 = (r + 1) % B;
      float za[4], zb[4];
      wam_normal4_x2(g0 + (uint32_t)(z0 * g.H + y0) * W4, g0 + (uint32_t)(z1 * g.H + y1) * W4, img, sm, nz.k0, nz.k1,
                     za, zb);
      const int q = (int)((bx * B) & 3);  // B = 2: the half of the group this block holds
#pragma unroll
      for (int k = 0; k < B; ++k) {
        v[z0][y0][k] = fmaf(sg, za[q + k], v[z0][y0][k]);  // noisy = fma(sigma, z, x) (wam_noise_add)
        v[z1][y1][k] = fmaf(sg, zb[q + k], v[z1][y1][k]);
      }
    }
  }
  // level 1 (finest): B/2 x B/2 x B/2 blocks of 2^3
  constexpr int B1 = B / 2;
  float ll[B1][B1][B1];
  const int64_t d1 = g.D / 2, h1 = g.H / 2, w1 = g.W / 2;
  const int64_t n1 = d1 * h1 * w1;
  float c1[B1][B1][B1][8];
#pragma unroll
  for (int z = 0; z < B1; ++z)
#pragma unroll
    for (int y = 0; y < B1; ++y)
#pragma unroll
      for (int x = 0; x < B1; ++x) {
        float blk[2][2][2];
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int c = 0; c < 2; ++c) blk[a][b][c] = v[2 * z + a][2 * y + b][2 * x + c];
        haar3_level(blk, f, c1[z][y][x]);
        ll[z][y][x] = c1[z][y][x][0];
      }
  // level-1 details (level index 0 = finest)
#pragma unroll
  for (int k = 1; k < 8; ++k) {
    float* dst = coeffs + g.items * g.off[0][k - 1] + item * n1;
#pragma unroll
    for (int z = 0; z < B1; ++z)
#pragma unroll
      for (int y = 0; y < B1; ++y) {
        const int64_t o = ((bz * B1 + z) * h1 + (by * B1 + y)) * w1 + bx * B1;
        if constexpr (B1 == 2) *reinterpret_cast<float2*>(dst + o) = make_float2(c1[z][y][0][k], c1[z][y][1][k]);
        else dst[o] = c1[z][y][0][k];
      }
  }
  if constexpr (J == 1) {
    float* dst = coeffs + g.items * g.off_a + item * n1;
    dst[(bz * h1 + by) * w1 + bx] = ll[0][0][0];
  } else {
    float c2[8];
    haar3_level(ll, f, c2);
    const int64_t d2 = d1 / 2, h2 = h1 / 2, w2 = w1 / 2;
    const int64_t n2 = d2 * h2 * w2, o = (bz * h2 + by) * w2 + bx;
    coeffs[g.items * g.off_a + item * n2 + o] = c2[0];
#pragma unroll
    for (int k = 1; k < 8; ++k) coeffs[g.items * g.off[1][k - 1] + item * n2 + o] = c2[k];
  }
}

template <int J>
__global__ void __launch_bounds__(kT3) k_haar3_syn(const float* __restrict__ coeffs, float* __restrict__ out,
                                                  const float* __restrict__ filt, Haar3Geom g, int64_t blocks,
                                                  float s) {
  constexpr int B = 1 << J;
  constexpr int B1 = B / 2;
  const int64_t t = (int64_t)blockIdx.x * kT3 + threadIdx.x;
  if (t >= blocks) return;
  const int64_t bw = g.W / B, bh = g.H / B, bd = g.D / B;
  const int64_t bx = t % bw, by = (t / bw) % bh, bz = (t / (bw * bh)) % bd, item = t / (bw * bh * bd);
  const float r[4] = {filt[0], filt[1], filt[2], filt[3]};  // rec lo0 lo1, rec hi0 hi1
  const int64_t d1 = g.D / 2, h1 = g.H / 2, w1 = g.W / 2;
  const int64_t n1 = d1 * h1 * w1;
  float ll[B1][B1][B1];
  if constexpr (J == 1) {
    ll[0][0][0] = s * coeffs[g.items * g.off_a + item * n1 + (bz * h1 + by) * w1 + bx];
  } else {
    const int64_t h2 = h1 / 2, w2 = w1 / 2, n2 = (d1 / 2) * h2 * w2, o = (bz * h2 + by) * w2 + bx;
    float c2[8];
    c2[0] = s * coeffs[g.items * g.off_a + item * n2 + o];
#pragma unroll
    for (int k = 1; k < 8; ++k) c2[k] = s * coeffs[g.items * g.off[1][k - 1] + item * n2 + o];
    haar3_inv(c2, r, ll);  // the approximation is scaled once, on its load (as wam_waverec)
  }
  float c1[B1][B1][B1][8];
#pragma unroll
  for (int z = 0; z < B1; ++z)
#pragma unroll
    for (int y = 0; y < B1; ++y)
#pragma unroll
      for (int x = 0; x < B1; ++x) c1[z][y][x][0] = ll[z][y][x];
#pragma unroll
  for (int k = 1; k < 8; ++k) {
    const float* src = coeffs + g.items * g.off[0][k - 1] + item * n1;
#pragma unroll
    for (int z = 0; z < B1; ++z)
#pragma unroll
      for (int y = 0; y < B1; ++y) {
        const int64_t o = ((bz * B1 + z) * h1 + (by * B1 + y)) * w1 + bx * B1;
        if constexpr (B1 == 2) {
          const float2 q = *reinterpret_cast<const float2*>(src + o);
          c1[z][y][0][k] = s * q.x;
          c1[z][y][1][k] = s * q.y;
        } else {
          c1[z][y][0][k] = s * src[o];
        }
      }
  }
  float v[B][B][B];
#pragma unroll
  for (int z = 0; z < B1; ++z)
#pragma unroll
    for (int y = 0; y < B1; ++y)
#pragma unroll
      for (int x = 0; x < B1; ++x) {
        float blk[2][2][2];
        haar3_inv(c1[z][y][x], r, blk);
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int c = 0; c < 2; ++c) v[2 * z + a][2 * y + b][2 * x + c] = blk[a][b][c];
      }
  float* dst = out + item * g.D * g.H * g.W + (bz * B * g.H + by * B) * g.W + bx * B;
#pragma unroll
  for (int z = 0; z < B; ++z)
#pragma unroll
    for (int y = 0; y < B; ++y) {
      float* row = dst + ((int64_t)z * g.H + y) * g.W;
      if constexpr (B == 4) wam_st4(row, v[z][y][0], v[z][y][1], v[z][y][2], v[z][y][3]);
      else wam_st(reinterpret_cast<wam_f2v*>(row), wam_f2v{v[z][y][0], v[z][y][1]});
    }
}

Haar3Geom make_geom3(const wam_plan* p, int64_t items) {
  Haar3Geom g{};
  g.J = p->levels;
  g.D = p->lin[0][0];
  g.H = p->lin[0][1];
  g.W = p->lin[0][2];
  g.off_a = p->band_off[0];
  for (int l = 0; l < p->levels; ++l)
    for (int k = 0; k < 7; ++k) g.off[l][k] = p->band_off[wam_band_of(p, l, k)];
  g.items = items;
  return g;
}

}  // namespace

bool dwt3_haar_supported(const wam_plan* p) {
  if (p->ndim != 3 || p->L != 2 || p->levels < 1 || p->levels > 2) return false;
  const int B = 1 << p->levels;
  for (int a = 0; a < 3; ++a)
    if (p->lin[0][a] % B) return false;
  return true;  // no padding for even sizes: every boundary mode gives the same coefficients
}

int launch_dwt3_haar_analysis(const wam_plan* p, int64_t batch, const float* in, float* coeffs, bool adjoint,
                              hipStream_t st) {
  if (!dwt3_haar_supported(p) || ((uintptr_t)in & 15)) return WAM_ERR_UNSUPPORTED;
  const Haar3Geom g = make_geom3(p, batch);
  const int B = 1 << p->levels;
  const int64_t blocks = batch * (g.D / B) * (g.H / B) * (g.W / B);
  const int64_t grid = (blocks + kT3 - 1) / kT3;
  if (grid > 0x7fffffff) return WAM_ERR_UNSUPPORTED;
  const float* filt = p->d_filt + (adjoint ? WAM_F_ADJ_LO : WAM_F_ANA_LO) * p->L;  // lo0 lo1 hi0 hi1
  WamTimer tm(st, "k_haar3_ana", 4.0 * (double)batch * ((double)g.D * g.H * g.W + (double)p->band_off[p->nbands]));
  const WamNoise none{nullptr, 1, 1, 0, 0, 0, 0};
  if (p->levels == 1)
    hipLaunchKernelGGL((k_haar3_ana<1, false>), dim3((unsigned)grid), dim3(kT3), 0, st, in, coeffs, filt, g, blocks,
                       none, (int64_t)1);
  else
    hipLaunchKernelGGL((k_haar3_ana<2, false>), dim3((unsigned)grid), dim3(kT3), 0, st, in, coeffs, filt, g, blocks,
                       none, (int64_t)1);
  WAM_LAUNCH_CHECK();
  return WAM_OK;
}

int launch_dwt3_haar_analysis_noisy(const wam_plan* p, int64_t batch, const float* in, float* coeffs,
                                    const WamNoise* nz, int64_t n_samples, hipStream_t st) {
  if (!dwt3_haar_supported(p) || ((uintptr_t)in & 15) || !nz) return WAM_ERR_UNSUPPORTED;
  if (nz->channels != 1 || batch != n_samples * nz->images) return WAM_ERR_UNSUPPORTED;
  const Haar3Geom g = make_geom3(p, batch);
  if (g.W % 4 || g.D * g.H * g.W >= (int64_t(1) << 34)) return WAM_ERR_UNSUPPORTED;  // 32-bit element groups
  const int B = 1 << p->levels;
  const int64_t nb = (g.D / B) * (g.H / B) * (g.W / B);
  const int64_t grid = n_samples * nz->images * ((nb + kT3 - 1) / kT3);
  if (grid > 0x7fffffff) return WAM_ERR_UNSUPPORTED;
  const float* filt = p->d_filt + WAM_F_ANA_LO * p->L;
  const double vol = (double)g.D * g.H * g.W;
  // algorithmic bytes: the clean volumes once, every sample's coefficients
  WamTimer tm(st, "k_haar3_ana<noise>", 4.0 * ((double)nz->images * vol + (double)batch * p->band_off[p->nbands]));
  if (p->levels == 1)
    hipLaunchKernelGGL((k_haar3_ana<1, true>), dim3((unsigned)grid), dim3(kT3), 0, st, in, coeffs, filt, g, batch * nb,
                       *nz, n_samples);
  else
    hipLaunchKernelGGL((k_haar3_ana<2, true>), dim3((unsigned)grid), dim3(kT3), 0, st, in, coeffs, filt, g, batch * nb,
                       *nz, n_samples);
  WAM_LAUNCH_CHECK();
  return WAM_OK;
}

int launch_dwt3_haar_synthesis(const wam_plan* p, int64_t batch, const float* coeffs, const float* alpha, int n_alpha,
                               float* out, hipStream_t st) {
  if (!dwt3_haar_supported(p) || ((uintptr_t)out & 15)) return WAM_ERR_UNSUPPORTED;
  const Haar3Geom g = make_geom3(p, batch);
  const int B = 1 << p->levels;
  const int64_t blocks = batch * (g.D / B) * (g.H / B) * (g.W / B);
  const int64_t grid = (blocks + kT3 - 1) / kT3;
  if (grid > 0x7fffffff) return WAM_ERR_UNSUPPORTED;
  const float* filt = p->d_filt + WAM_F_SYN_LO * p->L;  // rec lo0 lo1 hi0 hi1
  const int64_t vol = g.D * g.H * g.W;
  for (int ai = 0; ai < n_alpha; ++ai) {
    const float s = alpha ? alpha[ai] : 1.0f;
    float* o = out + (int64_t)ai * batch * vol;
    WamTimer tm(st, "k_haar3_syn", 4.0 * (double)batch * ((double)vol + (double)p->band_off[p->nbands]));
    if (p->levels == 1)
      hipLaunchKernelGGL(k_haar3_syn<1>, dim3((unsigned)grid), dim3(kT3), 0, st, coeffs, o, filt, g, blocks, s);
    else
      hipLaunchKernelGGL(k_haar3_syn<2>, dim3((unsigned)grid), dim3(kT3), 0, st, coeffs, o, filt, g, blocks, s);
    WAM_LAUNCH_CHECK();
  }
  return WAM_OK;
}

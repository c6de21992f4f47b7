// Streaming-copy ceiling sweep on gfx950 (not part of the library): which
// load/store form of a 2 GiB fp32 device copy gets closest to the 6.29 TB/s float4 copy of
// /opt/skills/guides/MI355X_MICROARCH.md. Variables: cache policy (plain / nontemporal loads and
// stores), bytes in flight per lane (U float4 loads issued before the first store), grid (one-shot:
// every thread a U-float4 run, no loop; or grid-stride over a capped grid), block size, and the
// XCD-aware block order. Each variant: 3 warm-up + 20 timed launches, HIP events, read + write bytes.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/ubench_copy.hip -o scripts/ubench_copy
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef float f4 __attribute__((ext_vector_type(4)));

template <int U, bool NTL, bool NTS>
__global__ void k_copy_stride(int64_t n4, const f4* __restrict__ src, f4* __restrict__ dst) {
  const int64_t step = (int64_t)gridDim.x * blockDim.x * U;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x * U + threadIdx.x; t + (U - 1) * (int64_t)blockDim.x < n4;
       t += step) {
    f4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      v[u] = NTL ? __builtin_nontemporal_load(src + t + u * (int64_t)blockDim.x) : src[t + u * (int64_t)blockDim.x];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (NTS) __builtin_nontemporal_store(v[u], dst + t + u * (int64_t)blockDim.x);
      else dst[t + u * (int64_t)blockDim.x] = v[u];
    }
  }
}

// one-shot: block b copies its own contiguous U * blockDim float4 run; n4 a multiple of that
template <int U, bool NTL, bool NTS, bool XCD>
__global__ void k_copy_once(int64_t n4, const f4* __restrict__ src, f4* __restrict__ dst) {
  int64_t b = blockIdx.x;
  if (XCD) {  // consecutive logical blocks on one XCD (bijective for grids divisible by 8)
    const int64_t q = gridDim.x / 8;
    b = (b % 8) * q + b / 8;
  }
  const int64_t t = b * blockDim.x * U + threadIdx.x;
  f4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u)
    v[u] = NTL ? __builtin_nontemporal_load(src + t + u * (int64_t)blockDim.x) : src[t + u * (int64_t)blockDim.x];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (NTS) __builtin_nontemporal_store(v[u], dst + t + u * (int64_t)blockDim.x);
    else dst[t + u * (int64_t)blockDim.x] = v[u];
  }
}

static const f4* g_src;
static f4* g_dst;
static int64_t g_n4;

template <class F>
static void run(const char* name, F launch) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 3; ++i) launch();
  hipEventRecord(a);
  for (int i = 0; i < 20; ++i) launch();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  const double us = ms * 1e3 / 20;
  printf("%-44s %9.1f us  %7.0f GB/s\n", name, us, 2.0 * g_n4 * 16 / (us * 1e3));
  fflush(stdout);
  hipEventDestroy(a);
  hipEventDestroy(b);
}

#define STRIDE(U, NTL, NTS, BS, GRID)                                                                             \
  run("stride U=" #U " ntl=" #NTL " nts=" #NTS " bs=" #BS " grid=" #GRID, [] {                                   \
    k_copy_stride<U, NTL, NTS><<<GRID, BS>>>(g_n4, g_src, g_dst);                                                 \
  })
#define ONCE(U, NTL, NTS, BS, XCD)                                                                                \
  run("once   U=" #U " ntl=" #NTL " nts=" #NTS " bs=" #BS " xcd=" #XCD, [] {                                     \
    k_copy_once<U, NTL, NTS, XCD><<<(unsigned)(g_n4 / ((int64_t)(BS) * (U))), BS>>>(g_n4, g_src, g_dst);          \
  })

int main() {
  const int64_t bytes = 2ll << 30;
  void *a, *b;
  if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess) return 1;
  hipMemset(a, 1, bytes);
  hipMemset(b, 0, bytes);
  g_src = (const f4*)a;
  g_dst = (f4*)b;
  g_n4 = bytes / 16;
  // the library's k_copy: grid-stride, nontemporal, U = 4, 256 threads, grid capped at 8,192
  STRIDE(4, true, true, 256, 8192);
  STRIDE(4, false, false, 256, 8192);
  STRIDE(4, true, false, 256, 8192);
  STRIDE(4, false, true, 256, 8192);
  STRIDE(1, false, false, 256, 8192);
  STRIDE(2, false, false, 256, 8192);
  STRIDE(8, false, false, 256, 8192);
  STRIDE(4, false, false, 256, 2048);
  STRIDE(4, false, false, 256, 4096);
  STRIDE(4, false, false, 256, 16384);
  STRIDE(4, false, false, 512, 4096);
  STRIDE(4, false, false, 1024, 2048);
  ONCE(1, false, false, 256, false);
  ONCE(2, false, false, 256, false);
  ONCE(4, false, false, 256, false);
  ONCE(8, false, false, 256, false);
  ONCE(4, true, true, 256, false);
  ONCE(4, false, true, 256, false);
  ONCE(4, true, false, 256, false);
  ONCE(4, false, false, 512, false);
  ONCE(4, false, false, 1024, false);
  ONCE(4, false, false, 256, true);
  ONCE(8, false, false, 256, true);
  STRIDE(4, true, true, 256, 8192);  // the library form again (drift check)
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  return 0;
}

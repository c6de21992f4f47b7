// WaveletAttribution3D.visualize (lib/wam_3D.py:662-719) on the GPU.
//
// Per volume and level j (0 = approximation corner, 1..J = detail shells, coarsest first) the
// reference slices the |grad| cube, sums six of the seven orientation blocks
// (add + ada + add + daa + dad + dda: 'add' twice, 'aad' and 'ddd' never -- kept as is),
// upsamples the block by an integer factor with scipy.ndimage.zoom(order=1) and divides by its
// max; the last slot is the sum over levels divided by its max over the WHOLE batch.
// scipy's zoom (grid_mode=False) samples input coordinate o * (in - 1) / (out - 1) with linear
// spline weights (1 - t, t) per axis and accumulates value * w0 * w1 * w2 over the 8 corners in
// double (last axis fastest), cast to float32: reproduced term by term. Three passes: upsample +
// per-(volume, level) max; normalise + level sum + batch max; final division.
#include "kernels.hpp"

namespace {

struct Vis3Geom {
  int S, J;
  int start[WAM_MAX_LEVELS + 1], n[WAM_MAX_LEVELS + 1];  // per level j: block offset and edge length
};

__device__ __forceinline__ void atomic_max_f32(float* addr, float v) {
  unsigned int* a = reinterpret_cast<unsigned int*>(addr);
  unsigned int old = *a;
  while (true) {
    const float cur = __uint_as_float(old);
    if (!(v > cur)) return;
    const unsigned int prev = atomicCAS(a, old, __float_as_uint(v));
    if (prev == old) return;
    old = prev;
  }
}

__device__ __forceinline__ float wave_maxf(float m) {
#pragma unroll
  for (int s = 32; s > 0; s >>= 1) m = fmaxf(m, __shfl_xor(m, s, 64));
  return m;
}

// value of the level block at (a, b, c) (float32 sums in the reference's order)
__device__ __forceinline__ float block_at(const float* __restrict__ g, int S, int j, int s, int a, int b, int c) {
  const int64_t S2 = (int64_t)S * S;
  if (j == 0) return g[a * S2 + (int64_t)b * S + c];
  const float ada = g[a * S2 + (int64_t)(s + b) * S + c];
  const float add = g[a * S2 + (int64_t)(s + b) * S + s + c];
  const float daa = g[(s + a) * S2 + (int64_t)b * S + c];
  const float dad = g[(s + a) * S2 + (int64_t)b * S + s + c];
  const float dda = g[(s + a) * S2 + (int64_t)(s + b) * S + c];
  return ((((add + ada) + add) + daa) + dad) + dda;
}

// grid: x = voxel chunks (grid-stride), y = segment (volume, level)
__global__ void __launch_bounds__(256) k_vis3d_upsample(Vis3Geom g, const float* __restrict__ cube,
                                                        float* __restrict__ out, float* __restrict__ lmax) {
  const int S = g.S, L = g.J + 2;
  const int64_t vol = (int64_t)S * S * S;
  const int64_t q = blockIdx.y;
  const int j = (int)(q % (g.J + 1));
  const int64_t it = q / (g.J + 1);
  const int n = g.n[j], s = g.start[j];
  const int on = n * (S / n);  // zoom output edge (== S for dyadic cubes)
  const double zm = on > 1 ? (double)(n - 1) / (double)(on - 1) : 1.0;
  const float* gi = cube + it * vol;
  float* oi = out + (it * L + j) * vol;
  float m = -INFINITY;
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < vol; v += (int64_t)gridDim.x * blockDim.x) {
    const int o[3] = {(int)(v / ((int64_t)S * S)), (int)((v / S) % S), (int)(v % S)};
    int i0[3];
    double w[3][2];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      const double cc = (double)o[d] * zm;
      const double fl = floor(cc);
      i0[d] = (int)fl;
      const double tt = cc - fl;
      w[d][0] = 1.0 - tt;
      w[d][1] = tt;
    }
    double acc = 0.0;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const int za = min(i0[0] + a, n - 1), yb = min(i0[1] + b, n - 1), xc = min(i0[2] + c, n - 1);
          const double val = (double)block_at(gi, S, j, s, za, yb, xc);
          acc = __dadd_rn(acc, __dmul_rn(__dmul_rn(__dmul_rn(val, w[0][a]), w[1][b]), w[2][c]));
        }
    const float r = (float)acc;
    oi[v] = r;
    m = fmaxf(m, r);
  }
  m = wave_maxf(m);
  if ((threadIdx.x & 63) == 0) atomic_max_f32(&lmax[q], m);
}

__global__ void __launch_bounds__(256) k_vis3d_normalize(int64_t items, int S, int J, float* __restrict__ out,
                                                         const float* __restrict__ lmax, float* __restrict__ gmax) {
  const int L = J + 2;
  const int64_t vol = (int64_t)S * S * S;
  const int64_t total = items * vol;
  float m = -INFINITY;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t it = t / vol, v = t - it * vol;
    float sum = 0.f;
    for (int j = 0; j <= J; ++j) {
      float* p = out + (it * L + j) * vol + v;
      const float x = *p / lmax[it * (J + 1) + j];
      *p = x;
      sum = j == 0 ? x : sum + x;
    }
    out[(it * L + J + 1) * vol + v] = sum;
    m = fmaxf(m, sum);
  }
  m = wave_maxf(m);
  if ((threadIdx.x & 63) == 0) atomic_max_f32(gmax, m);
}

__global__ void __launch_bounds__(256) k_vis3d_final(int64_t items, int S, int J, float* __restrict__ out,
                                                     const float* __restrict__ gmax) {
  const int L = J + 2;
  const int64_t vol = (int64_t)S * S * S;
  const int64_t total = items * vol;
  const float gm = *gmax;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t it = t / vol, v = t - it * vol;
    float* p = out + (it * L + J + 1) * vol + v;
    *p = *p / gm;
  }
}

}  // namespace

extern "C" int wam_visualize3d(int64_t items, int size, int levels, const float* cube, float* out, float* scratch,
                               void* stream) {
  if (items < 0 || size < 1 || levels < 0 || levels >= WAM_MAX_LEVELS || !cube || !out || !scratch)
    return WAM_ERR_INVALID_ARG;
  if (items == 0) return WAM_OK;
  Vis3Geom g{};
  g.S = size;
  g.J = levels;
  // level_indices = [0] + [int(S / 2**j) for j in range(J + 1)][::-1]
  int idx[WAM_MAX_LEVELS + 2];
  idx[0] = 0;
  for (int j = 0; j <= levels; ++j) idx[j + 1] = (int)(size / (double)(1 << (levels - j)));
  for (int j = 0; j <= levels; ++j) {
    g.start[j] = idx[j];
    g.n[j] = j == 0 ? idx[1] : idx[j + 1] - idx[j];
    if (g.n[j] < 1 || (size / g.n[j]) * g.n[j] != size) return WAM_ERR_SHAPE;  // the reference's assignment fails
    if (j > 0 && g.n[j] != g.start[j]) return WAM_ERR_SHAPE;
  }
  if (items * (levels + 1) > 65535) return WAM_ERR_INVALID_ARG;
  hipStream_t st = (hipStream_t)stream;
  const int64_t vol = (int64_t)size * size * size;
  float* lmax = scratch;                      // items * (levels + 1)
  float* gmax = scratch + items * (levels + 1);
  WAM_HIP_CHECK(hipMemsetD32Async((hipDeviceptr_t)scratch, 0xFF800000u, items * (levels + 1) + 1, st));  // -inf
  {
    WamTimer tm(st, "k_vis3d_upsample", 4.0 * items * vol + 4.0 * items * (levels + 1) * vol);
    const dim3 grid(wam_grid(vol, 256, 512), (unsigned)(items * (levels + 1)));
    hipLaunchKernelGGL(k_vis3d_upsample, grid, dim3(256), 0, st, g, cube, out, lmax);
    WAM_LAUNCH_CHECK();
  }
  {
    WamTimer tm(st, "k_vis3d_normalize", 8.0 * items * (levels + 1) * vol + 4.0 * items * vol);
    hipLaunchKernelGGL(k_vis3d_normalize, dim3(wam_grid(items * vol, 256, 65536)), dim3(256), 0, st, items, size,
                       levels, out, lmax, gmax);
    WAM_LAUNCH_CHECK();
  }
  WamTimer tm(st, "k_vis3d_final", 8.0 * items * vol);
  hipLaunchKernelGGL(k_vis3d_final, dim3(wam_grid(items * vol, 256, 65536)), dim3(256), 0, st, items, size, levels,
                     out, gmax);
  WAM_LAUNCH_CHECK();
  return WAM_OK;
}

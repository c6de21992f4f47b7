// Generic per-axis filter-bank kernels (any ndim, any even filter length, every boundary mode).
// Used for 1D and 3D transforms and as the 2D path for filters longer than the fused kernels.
// The array is viewed as [outer, n, inner]; inner is the stride of the filtered axis, so for
// inner > 1 consecutive lanes read consecutive addresses (coalesced), and for inner == 1 they
// read with stride 2 (one coalesced window of 2*64 floats per wave per tap).
#include "kernels.hpp"

namespace {

__global__ void __launch_bounds__(256) k_analysis_axis(const float* __restrict__ in, float* __restrict__ lo,
                                                       float* __restrict__ hi, int64_t outer, int n, int m,
                                                       int64_t inner, int padl, int mode,
                                                       const float* __restrict__ flo,
                                                       const float* __restrict__ fhi, int L) {
  const int64_t total = outer * (int64_t)m * inner;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    int64_t r = t % inner;
    int64_t q = t / inner;
    int i = (int)(q % m);
    int64_t o = q / m;
    const float* src = in + o * (int64_t)n * inner + r;
    float a = 0.f, d = 0.f;
    int base = 2 * i - padl;
    for (int k = 0; k < L; ++k) {
      int j = wam_ext_index(base + k, n, mode);
      float v = j >= 0 ? src[(int64_t)j * inner] : 0.f;
      a = fmaf(flo[k], v, a);
      d = fmaf(fhi[k], v, d);
    }
    int64_t oi = (o * m + i) * inner + r;
    lo[oi] = a;
    hi[oi] = d;
  }
}

__global__ void __launch_bounds__(256) k_synthesis_axis(const float* __restrict__ a, const float* __restrict__ d,
                                                        float* __restrict__ out, int64_t outer, int m, int nout,
                                                        int64_t inner, int p, const float* __restrict__ rlo,
                                                        const float* __restrict__ rhi, int L, float sa, float sd) {
  const int64_t total = outer * (int64_t)nout * inner;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    int64_t r = t % inner;
    int64_t q = t / inner;
    int to = (int)(q % nout);
    int64_t o = q / nout;
    int tt = to + p;  // position in the uncropped conv_transpose output
    const float* pa = a + o * (int64_t)m * inner + r;
    const float* pd = d + o * (int64_t)m * inner + r;
    int imax = tt >> 1;
    if (imax > m - 1) imax = m - 1;
    int imin = (tt - L + 2) >> 1;  // ceil((tt - L + 1) / 2)
    if (imin < 0) imin = 0;
    float y = 0.f;
    for (int i = imax; i >= imin; --i) {
      int k = tt - 2 * i;
      float av = sa * pa[(int64_t)i * inner];
      float dv = sd * pd[(int64_t)i * inner];
      y = fmaf(rlo[k], av, y);
      y = fmaf(rhi[k], dv, y);
    }
    out[(o * nout + to) * inner + r] = y;
  }
}

}  // namespace

int launch_analysis_axis(const float* in, float* lo, float* hi, int64_t outer, int n, int m, int64_t inner, int padl,
                         int mode, const float* flo, const float* fhi, int L, hipStream_t st) {
  int64_t work = outer * (int64_t)m * inner;
  if (work == 0) return WAM_OK;
  WamTimer tm(st, "k_analysis_axis", 4.0 * (double)outer * inner * (n + 2.0 * m));
  hipLaunchKernelGGL(k_analysis_axis, dim3(wam_grid(work, 256)), dim3(256), 0, st, in, lo, hi, outer, n, m, inner,
                     padl, mode, flo, fhi, L);
  WAM_LAUNCH_CHECK();
  return WAM_OK;
}

int launch_synthesis_axis(const float* a, const float* d, float* out, int64_t outer, int m, int nout, int64_t inner,
                          int p, const float* rlo, const float* rhi, int L, float sa, float sd, hipStream_t st) {
  int64_t work = outer * (int64_t)nout * inner;
  if (work == 0) return WAM_OK;
  WamTimer tm(st, "k_synthesis_axis", 4.0 * (double)outer * inner * (2.0 * m + nout));
  hipLaunchKernelGGL(k_synthesis_axis, dim3(wam_grid(work, 256)), dim3(256), 0, st, a, d, out, outer, m, nout, inner,
                     p, rlo, rhi, L, sa, sd);
  WAM_LAUNCH_CHECK();
  return WAM_OK;
}

// Wavelet-domain insertion / deletion / mu-fidelity: the batched GPU form of
// the reference's evaluation helpers (src/evaluation_helpers.py:455-578) driven by Eval2DWAM
// (src/evaluators.py:553-801). Per image the reference loops over n_iter + 1 (or sample_size)
// masks and channels on the CPU: pywt.wavedec2 -> coeffs_to_array -> arr * mask ->
// array_to_coeffs -> waverec2 -> min-max normalise -> uint8 -> PIL -> ToTensor + Normalize. Here
// the analysis runs once per image (plan kernels), the masks multiply the coefficients in one
// gather pass that writes the band-major buffer the synthesis kernels read (all masks of all
// channels in one waverec launch), and the byte quantisation + ImageNet normalisation of every
// reconstruction is one fused pass. All kernels are HBM-bound elementwise / reduction passes.
#include "kernels.hpp"

namespace {

// ---- insertion / deletion masks from the importance ranking (generate_masks, :469-505):
// mask m keeps the pixels ranked < thr(m): thr(0) = 0, thr(m) = m * n_comp (m < n_iter),
// thr(n_iter) = every pixel (the reference overwrites the last mask with ones / zeros).
__global__ void __launch_bounds__(256) k_rank_masks(int64_t n_iter, int64_t n_comp, int64_t len,
                                                    const int32_t* __restrict__ rank, int deletion,
                                                    float* __restrict__ masks) {
  const int64_t total = (n_iter + 1) * len;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = t / len, p = t - m * len;
    int64_t thr = m >= n_iter ? len : m * n_comp;
    thr = thr < len ? thr : len;
    const bool keep = (int64_t)rank[p] < thr;
    masks[t] = (keep != (deletion != 0)) ? 1.f : 0.f;
  }
}

// ---- arr * masks[m] in pywt's coeffs_to_array layout: coefficient k of channel item i sits at
// array position pos[k]; out is band-major over items (m, i) -> m * items + i.
struct BandTable {
  int nbands;
  int64_t off[WAM_MAX_BANDS + 1];  // per-item element offsets
};

__global__ void __launch_bounds__(256) k_coeff_masks(int64_t items, int64_t n_masks, int64_t mask_len, BandTable bt,
                                                     const float* __restrict__ coeffs,
                                                     const int32_t* __restrict__ pos,
                                                     const float* __restrict__ masks, float* __restrict__ out) {
  const int64_t K = bt.off[bt.nbands];
  const int64_t out_items = n_masks * items;
  const int64_t total = out_items * K;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    // t walks the OUTPUT band-major buffer: band b, item it, element e
    int b = 0;
#pragma unroll 1
    while (b + 1 < bt.nbands && t >= out_items * bt.off[b + 1]) ++b;
    const int64_t bn = bt.off[b + 1] - bt.off[b];
    const int64_t r = t - out_items * bt.off[b];
    const int64_t it = r / bn, e = r - it * bn;
    const int64_t m = it / items, i = it - m * items;
    const float c = coeffs[items * bt.off[b] + i * bn + e];
    out[t] = c * masks[m * mask_len + pos[bt.off[b] + e]];
  }
}

// ---- normalize_data (:433-435) -> (x * 255).astype(uint8) -> ToTensor (/ 255) -> Normalize:
// one workgroup per image: min / max over all its channels, then the fused map.
__device__ __forceinline__ void block_minmax(float& mn, float& mx) {
  __shared__ float smn[16], smx[16];
  for (int s = 32; s > 0; s >>= 1) {
    mn = fminf(mn, __shfl_xor(mn, s, 64));
    mx = fmaxf(mx, __shfl_xor(mx, s, 64));
  }
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    smn[w] = mn;
    smx[w] = mx;
  }
  __syncthreads();
  mn = smn[0];
  mx = smx[0];
  for (int i = 1; i < nw; ++i) {
    mn = fminf(mn, smn[i]);
    mx = fmaxf(mx, smx[i]);
  }
}

struct ChanNorm {
  float mean[4], std[4];
};

__global__ void __launch_bounds__(1024) k_quantize_normalize(int channels, int64_t plane, const float* __restrict__ rec,
                                                             ChanNorm cn, float* __restrict__ out) {
  const int64_t n = (int64_t)channels * plane;
  const float* x = rec + blockIdx.x * n;
  float* o = out + blockIdx.x * n;
  float mn = INFINITY, mx = -INFINITY;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    mn = fminf(mn, x[i]);
    mx = fmaxf(mx, x[i]);
  }
  block_minmax(mn, mx);
  const float rng = mx - mn;  // numpy: (data - min) / (max - min), float32
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    const float v = __fdiv_rn(x[i] - mn, rng);
    const float s = __fmul_rn(v, 255.f);
    // astype(uint8): truncation, values in [0, 255]. A constant image (e.g. insertion step 0: all
    // coefficients masked, a zero reconstruction) gives 0 / 0 = NaN, which numpy's NaN -> uint8 cast
    // turns into 0 on x86 (cvttss2si's 0x80000000, low byte 0): pinned here explicitly rather than
    // left to the hardware's float -> int conversion of NaN
    const float q = (s != s) ? 0.f : (float)(unsigned char)(int)s;
    const int c = (int)(i / plane);
    o[i] = __fdiv_rn(__fdiv_rn(q, 255.f) - cn.mean[c], cn.std[c]);
  }
}

// ---- torchvision Resize((224, 224)) on the reference's PIL image of a reconstruction that is not
// 224 x 224 (src/evaluators.py:593-598): normalize_data -> uint8 -> PIL.Image -> Pillow's BILINEAR
// resample -> ToTensor + Normalize. Pillow's 8-bit resample (libImaging/Resample.c) is integer
// arithmetic: per output position a run of fixed-point weights (22 fractional bits, built on the
// host exactly as precompute_coeffs + normalize_coeffs_8bpc do), a horizontal pass into a uint8
// image of the source rows the vertical pass needs, then the vertical pass; every pass rounds with
// + 2^21 and clamps (ss >> 22) to [0, 255]. Bit-identical to Pillow (tests/test_gpu_eval.py).
constexpr int kPilBits = 22;

__device__ __forceinline__ int pil_clip8(int ss) {
  const int v = ss >> kPilBits;
  return v < 0 ? 0 : (v > 255 ? 255 : v);
}

// one workgroup per image: the min-max quantisation of k_quantize_normalize, written as bytes
__global__ void __launch_bounds__(1024) k_quantize_u8(int channels, int64_t plane, const float* __restrict__ rec,
                                                      uint8_t* __restrict__ u8) {
  const int64_t n = (int64_t)channels * plane;
  const float* x = rec + blockIdx.x * n;
  uint8_t* o = u8 + blockIdx.x * n;
  float mn = INFINITY, mx = -INFINITY;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    mn = fminf(mn, x[i]);
    mx = fmaxf(mx, x[i]);
  }
  block_minmax(mn, mx);
  const float rng = mx - mn;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    const float s = __fmul_rn(__fdiv_rn(x[i] - mn, rng), 255.f);
    o[i] = (s != s) ? (uint8_t)0 : (uint8_t)(int)s;  // NaN (constant image) -> 0, as numpy on x86
  }
}

// horizontal pass: planes of in_h x in_w bytes -> tmp planes of tmp_h x out_w (source rows
// y0 .. y0 + tmp_h - 1)
__global__ void __launch_bounds__(256) k_pil_resize_h(int64_t planes, int in_h, int in_w, int y0, int tmp_h, int out_w,
                                                      int ksize, const int32_t* __restrict__ bounds,
                                                      const int32_t* __restrict__ kk, const uint8_t* __restrict__ src,
                                                      uint8_t* __restrict__ tmp) {
  const int64_t total = planes * tmp_h * out_w;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int xx = (int)(t % out_w);
    const int64_t r = t / out_w;
    const int y = (int)(r % tmp_h);
    const int64_t pl = r / tmp_h;
    const uint8_t* row = src + (pl * in_h + y0 + y) * (int64_t)in_w;
    const int xmin = bounds[2 * xx], cnt = bounds[2 * xx + 1];
    const int32_t* k = kk + (int64_t)xx * ksize;
    int ss = 1 << (kPilBits - 1);
    for (int x = 0; x < cnt; ++x) ss += (int)row[xmin + x] * k[x];
    tmp[t] = (uint8_t)pil_clip8(ss);
  }
}

// vertical pass (or a copy when the height is unchanged) + ToTensor + Normalize: tmp planes of
// tmp_h x out_w -> out [images, channels, out_h, out_w] float32
__global__ void __launch_bounds__(256) k_pil_resize_v_norm(int64_t images, int channels, int tmp_h, int out_h, int out_w,
                                                           int vertical, int ksize, const int32_t* __restrict__ bounds,
                                                           const int32_t* __restrict__ kk,
                                                           const uint8_t* __restrict__ tmp, ChanNorm cn,
                                                           float* __restrict__ out) {
  const int64_t total = images * channels * (int64_t)out_h * out_w;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int x = (int)(t % out_w);
    const int64_t r = t / out_w;
    const int yy = (int)(r % out_h);
    const int64_t pl = r / out_h;
    const int c = (int)(pl % channels);
    const uint8_t* col = tmp + pl * (int64_t)tmp_h * out_w + x;
    int u;
    if (vertical) {
      const int ymin = bounds[2 * yy], cnt = bounds[2 * yy + 1];
      const int32_t* k = kk + (int64_t)yy * ksize;
      int ss = 1 << (kPilBits - 1);
      for (int y = 0; y < cnt; ++y) ss += (int)col[(int64_t)(ymin + y) * out_w] * k[y];
      u = pil_clip8(ss);
    } else {
      u = col[(int64_t)yy * out_w];
    }
    out[t] = __fdiv_rn(__fdiv_rn((float)u, 255.f) - cn.mean[c], cn.std[c]);
  }
}

// ---- scipy.ndimage.gaussian_filter (mode 'reflect' = half-sample symmetric, truncate 4): the
// two 1-D passes (axis 0, then axis 1) with scipy's symmetric-kernel accumulation order
// x0 w0 + (x[-r] + x[r]) w[r] + ... + (x[-1] + x[1]) w[1], every product and sum rounded (no fma).
constexpr int kMaxGaussR = 64;
struct GaussW {
  double w[kMaxGaussR + 1];  // w[j] = weight at offset +-j
};

template <int AXIS>
__global__ void __launch_bounds__(256) k_gauss_pass(int64_t items, int h, int w, int radius, GaussW gw,
                                                    const double* __restrict__ in, double* __restrict__ out) {
  const int64_t plane = (int64_t)h * w;
  const int64_t total = items * plane;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t it = t / plane;
    const int p = (int)(t - it * plane);
    const int r = p / w, c = p - r * w;
    const double* x = in + it * plane;
    auto at = [&](int d) -> double {
      if (AXIS == 0) return x[(int64_t)wam_ext_index(r + d, h, WAM_MODE_SYMMETRIC) * w + c];
      return x[(int64_t)r * w + wam_ext_index(c + d, w, WAM_MODE_SYMMETRIC)];
    };
    double acc = __dmul_rn(at(0), gw.w[0]);
    for (int j = radius; j >= 1; --j) acc = __dadd_rn(acc, __dmul_rn(__dadd_rn(at(-j), at(j)), gw.w[j]));
    out[t] = acc;
  }
}

// ---- nearest-neighbour upsampling of grid masks through a precomputed cell map (scipy zoom,
// order 0): out[m, p] = grid[m, cell[p]]
__global__ void __launch_bounds__(256) k_upsample_masks(int64_t n_masks, int64_t grid_len, const float* __restrict__ grid,
                                                        int64_t out_len, const int32_t* __restrict__ cell,
                                                        float* __restrict__ out) {
  const int64_t total = n_masks * out_len;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = t / out_len, p = t - m * out_len;
    out[t] = grid[m * grid_len + cell[p]];
  }
}

// ---- sum_importance (:361-393): per mask, sum over pixels of wam * upsampled subset mask (fp64)
__global__ void __launch_bounds__(256) k_masked_sums(int64_t len, const double* __restrict__ wam, int64_t grid_len,
                                                     const float* __restrict__ grid, const int32_t* __restrict__ cell,
                                                     double* __restrict__ out) {
  const float* g = grid + blockIdx.x * grid_len;
  double acc = 0.0;
  for (int64_t p = threadIdx.x; p < len; p += blockDim.x) acc += wam[p] * (double)g[cell[p]];
  __shared__ double part[256];
  part[threadIdx.x] = acc;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) part[threadIdx.x] += part[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[blockIdx.x] = part[0];
}

}  // namespace

extern "C" {

int wam_rank_masks(int64_t n_iter, int64_t n_comp, int64_t len, const int32_t* rank, int deletion, float* masks,
                   void* stream) {
  if (n_iter < 1 || n_comp < 0 || len < 1 || !rank || !masks) return WAM_ERR_INVALID_ARG;
  const int64_t work = (n_iter + 1) * len;
  WamTimer tm((hipStream_t)stream, "k_rank_masks", 4.0 * len + 4.0 * work);
  hipLaunchKernelGGL(k_rank_masks, dim3(wam_grid(work, 256)), dim3(256), 0, (hipStream_t)stream, n_iter, n_comp, len,
                     rank, deletion, masks);
  WAM_LAUNCH_CHECK();
  return WAM_OK;
}

int wam_coeff_masks(const wam_plan* plan, int64_t items, const float* coeffs, const int32_t* pos, int64_t n_masks,
                    int64_t mask_len, const float* masks, float* out, void* stream) {
  if (!plan || items < 0 || n_masks < 0 || mask_len < 1 || !coeffs || !pos || !masks || !out)
    return WAM_ERR_INVALID_ARG;
  BandTable bt{};
  bt.nbands = plan->nbands;
  for (int b = 0; b <= plan->nbands; ++b) bt.off[b] = plan->band_off[b];
  const int64_t K = bt.off[bt.nbands];
  const int64_t work = n_masks * items * K;
  if (work == 0) return WAM_OK;
  WamTimer tm((hipStream_t)stream, "k_coeff_masks", 4.0 * (items * K + n_masks * mask_len + work));
  hipLaunchKernelGGL(k_coeff_masks, dim3(wam_grid(work, 256)), dim3(256), 0, (hipStream_t)stream, items, n_masks,
                     mask_len, bt, coeffs, pos, masks, out);
  WAM_LAUNCH_CHECK();
  return WAM_OK;
}

int wam_quantize_normalize(int64_t images, int channels, int64_t plane, const float* rec, const float* mean,
                           const float* std, float* out, void* stream) {
  if (images < 0 || channels < 1 || channels > 4 || plane < 1 || !rec || !mean || !std || !out)
    return WAM_ERR_INVALID_ARG;
  if (images == 0) return WAM_OK;
  ChanNorm cn{};
  for (int c = 0; c < channels; ++c) {
    cn.mean[c] = mean[c];
    cn.std[c] = std[c];
  }
  WamTimer tm((hipStream_t)stream, "k_quantize_normalize", 8.0 * images * channels * plane);
  hipLaunchKernelGGL(k_quantize_normalize, dim3((unsigned)images), dim3(1024), 0, (hipStream_t)stream, channels, plane,
                     rec, cn, out);
  WAM_LAUNCH_CHECK();
  return WAM_OK;
}

int wam_quantize_resize_normalize(int64_t images, int channels, int in_h, int in_w, const float* rec, int out_h,
                                  int out_w, int ksize_h, const int32_t* bounds_h, const int32_t* kk_h, int ksize_v,
                                  const int32_t* bounds_v, const int32_t* kk_v, int y0, int tmp_h, const float* mean,
                                  const float* std, uint8_t* scratch, float* out, void* stream) {
  if (images < 0 || channels < 1 || channels > 4 || in_h < 1 || in_w < 1 || out_h < 1 || out_w < 1 || !rec ||
      !mean || !std || !scratch || !out)
    return WAM_ERR_INVALID_ARG;
  const bool horiz = bounds_h != nullptr, vert = bounds_v != nullptr;
  if ((horiz && (!kk_h || ksize_h < 1)) || (vert && (!kk_v || ksize_v < 1))) return WAM_ERR_INVALID_ARG;
  if (!horiz && out_w != in_w) return WAM_ERR_SHAPE;
  if (!vert && out_h != in_h) return WAM_ERR_SHAPE;
  if (horiz && (y0 < 0 || tmp_h < 1 || y0 + tmp_h > in_h)) return WAM_ERR_SHAPE;
  if (images == 0) return WAM_OK;
  ChanNorm cn{};
  for (int c = 0; c < channels; ++c) {
    cn.mean[c] = mean[c];
    cn.std[c] = std[c];
  }
  hipStream_t st = (hipStream_t)stream;
  const int64_t planes = images * channels;
  const int64_t in_px = planes * (int64_t)in_h * in_w;
  uint8_t* u8 = scratch;                 // planes x in_h x in_w
  uint8_t* tmp = scratch + in_px;        // planes x tmp_h x out_w (horizontal pass)
  {
    WamTimer tm(st, "k_quantize_u8", 5.0 * in_px);
    hipLaunchKernelGGL(k_quantize_u8, dim3((unsigned)images), dim3(1024), 0, st, channels, (int64_t)in_h * in_w, rec,
                       u8);
    WAM_LAUNCH_CHECK();
  }
  const uint8_t* vsrc = u8;
  int vh = in_h;
  if (horiz) {
    const int64_t work = planes * (int64_t)tmp_h * out_w;
    WamTimer tm(st, "k_pil_resize_h", (double)planes * tmp_h * in_w + (double)work);
    hipLaunchKernelGGL(k_pil_resize_h, dim3(wam_grid(work, 256)), dim3(256), 0, st, planes, in_h, in_w, y0, tmp_h,
                       out_w, ksize_h, bounds_h, kk_h, u8, tmp);
    WAM_LAUNCH_CHECK();
    vsrc = tmp;
    vh = tmp_h;
  }
  const int64_t work = planes * (int64_t)out_h * out_w;
  WamTimer tm(st, "k_pil_resize_v_norm", (double)planes * vh * out_w + 4.0 * work);
  hipLaunchKernelGGL(k_pil_resize_v_norm, dim3(wam_grid(work, 256)), dim3(256), 0, st, images, channels, vh, out_h,
                     out_w, (int)vert, ksize_v, bounds_v, kk_v, vsrc, cn, out);
  WAM_LAUNCH_CHECK();
  return WAM_OK;
}

int wam_gaussian_filter2d(int64_t items, int h, int w, const double* weights, int radius, const double* in,
                          double* tmp, double* out, void* stream) {
  if (items < 0 || h < 1 || w < 1 || radius < 0 || radius > kMaxGaussR || !weights || !in || !tmp || !out)
    return WAM_ERR_INVALID_ARG;
  const int64_t work = items * (int64_t)h * w;
  if (work == 0) return WAM_OK;
  GaussW gw{};
  for (int j = 0; j <= radius; ++j) gw.w[j] = weights[j];
  hipStream_t st = (hipStream_t)stream;
  {
    WamTimer tm(st, "k_gauss_pass", 16.0 * work);
    hipLaunchKernelGGL(k_gauss_pass<0>, dim3(wam_grid(work, 256)), dim3(256), 0, st, items, h, w, radius, gw, in, tmp);
    WAM_LAUNCH_CHECK();
  }
  WamTimer tm(st, "k_gauss_pass", 16.0 * work);
  hipLaunchKernelGGL(k_gauss_pass<1>, dim3(wam_grid(work, 256)), dim3(256), 0, st, items, h, w, radius, gw, tmp, out);
  WAM_LAUNCH_CHECK();
  return WAM_OK;
}

int wam_upsample_masks(int64_t n_masks, int64_t grid_len, const float* grid, int64_t out_len, const int32_t* cell,
                       float* out, void* stream) {
  if (n_masks < 0 || grid_len < 1 || out_len < 1 || !grid || !cell || !out) return WAM_ERR_INVALID_ARG;
  const int64_t work = n_masks * out_len;
  if (work == 0) return WAM_OK;
  WamTimer tm((hipStream_t)stream, "k_upsample_masks", 4.0 * (n_masks * grid_len + out_len + work));
  hipLaunchKernelGGL(k_upsample_masks, dim3(wam_grid(work, 256)), dim3(256), 0, (hipStream_t)stream, n_masks,
                     grid_len, grid, out_len, cell, out);
  WAM_LAUNCH_CHECK();
  return WAM_OK;
}

int wam_masked_sums(int64_t n_masks, int64_t len, const double* wam, int64_t grid_len, const float* grid,
                    const int32_t* cell, double* out, void* stream) {
  if (n_masks < 0 || len < 1 || grid_len < 1 || !wam || !grid || !cell || !out) return WAM_ERR_INVALID_ARG;
  if (n_masks == 0) return WAM_OK;
  WamTimer tm((hipStream_t)stream, "k_masked_sums", 8.0 * len + 4.0 * len + 4.0 * n_masks * grid_len);
  hipLaunchKernelGGL(k_masked_sums, dim3((unsigned)n_masks), dim3(256), 0, (hipStream_t)stream, len, wam, grid_len,
                     grid, cell, out);
  WAM_LAUNCH_CHECK();
  return WAM_OK;
}

}  // extern "C"

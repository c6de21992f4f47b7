// Fused elementwise steps of the explained model's input-gradient pass.
//
// WAM runs the model only for d loss / d input (lib/wam_2D.py:114-116). After BatchNorm folding
// (wam_amd/model_opt.py) a ResNet step is convolutions plus per-channel bias adds, ReLUs,
// residual adds and their backward masks -- and on MI355X those elementwise passes, each a full
// HBM round trip over an activation tensor, took about half of the c2 step (profiles/r01f_*: torch
// bias add, clamp, residual add, threshold_backward). The kernels below fold each chain into
// ONE pass:
//   k_bias_act      y = relu?(y + b[c])                        (conv bias + ReLU, in place)
//   k_add_bias_relu out = relu(a + ba[c] + s + bs[c])          (bottleneck tail + residual)
//   k_relu_mask     out = y > 0 ? g : 0                        (ReLU backward)
//   k_add_relu_mask out = y > 0 ? g1 + g2 : 0                  (gradient fan-in + ReLU backward)
// Arithmetic in fp32, storage fp32 or bf16 (round to nearest even on the store). Every kernel
// moves 16 bytes per access (8 bf16 / 4 fp32) with UNR accesses in flight per thread; the channel
// of an element is (i / inner) % C (inner = 1 for NHWC, H*W for NCHW).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.hpp"

namespace {

constexpr int kBlk = 256;
constexpr int kUnr = 4;

__device__ __forceinline__ float ld1(const float* p, int64_t i) { return p[i]; }
__device__ __forceinline__ float ld1(const uint16_t* p, int64_t i) { return __uint_as_float((uint32_t)p[i] << 16); }
__device__ __forceinline__ uint16_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40u);  // quiet NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
__device__ __forceinline__ void st1(float* p, int64_t i, float v) { p[i] = v; }
__device__ __forceinline__ void st1(uint16_t* p, int64_t i, float v) { p[i] = f2bf(v); }

// 16-byte vector of T as VEC floats
template <typename T>
struct Vec;
template <>
struct Vec<float> {
  static constexpr int N = 4;
  typedef float4 raw;
  __device__ static void unpack(const raw& r, float (&v)[4]) { v[0] = r.x, v[1] = r.y, v[2] = r.z, v[3] = r.w; }
  __device__ static raw pack(const float (&v)[4]) { return make_float4(v[0], v[1], v[2], v[3]); }
};
template <>
struct Vec<uint16_t> {
  static constexpr int N = 8;
  typedef uint4 raw;
  __device__ static void unpack(const raw& r, float (&v)[8]) {
    const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      v[2 * k] = __uint_as_float(w[k] << 16);
      v[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
    }
  }
  __device__ static raw pack(const float (&v)[8]) {
    uint32_t w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) w[k] = (uint32_t)f2bf(v[2 * k]) | ((uint32_t)f2bf(v[2 * k + 1]) << 16);
    return make_uint4(w[0], w[1], w[2], w[3]);
  }
};

// channel layout of a 16-byte vector starting at element i:
//   CH_VEC  inner == 1 and C % VEC == 0: channels c0 .. c0+VEC-1, c0 = i % C
//   CH_ONE  inner % VEC == 0: one channel (i / inner) % C for the whole vector
enum { CH_VEC = 0, CH_ONE = 1 };

template <typename T, int CH>
__device__ __forceinline__ void load_bias(const T* b, int64_t i, int64_t C, int64_t inner, float (&bv)[Vec<T>::N]) {
  constexpr int V = Vec<T>::N;
  if (b == nullptr) {
#pragma unroll
    for (int k = 0; k < V; ++k) bv[k] = 0.f;
    return;
  }
  if constexpr (CH == CH_VEC) {
    const int64_t c0 = i % C;
    Vec<T>::unpack(*reinterpret_cast<const typename Vec<T>::raw*>(b + c0), bv);
  } else {
    const float v = ld1(b, (i / inner) % C);
#pragma unroll
    for (int k = 0; k < V; ++k) bv[k] = v;
  }
}

template <typename T, int CH, bool RELU>
__global__ void __launch_bounds__(kBlk) k_bias_act(int64_t nvec, int64_t C, int64_t inner, T* __restrict__ y,
                                                     const T* __restrict__ b) {
  constexpr int V = Vec<T>::N;
  typedef typename Vec<T>::raw R;
  const int64_t base = (int64_t)blockIdx.x * (kBlk * kUnr) + threadIdx.x;
  R r[kUnr];
#pragma unroll
  for (int u = 0; u < kUnr; ++u) {
    const int64_t q = base + u * kBlk;
    if (q < nvec) r[u] = reinterpret_cast<const R*>(y)[q];
  }
#pragma unroll
  for (int u = 0; u < kUnr; ++u) {
    const int64_t q = base + u * kBlk;
    if (q >= nvec) continue;
    float v[V], bv[V];
    Vec<T>::unpack(r[u], v);
    load_bias<T, CH>(b, q * V, C, inner, bv);
#pragma unroll
    for (int k = 0; k < V; ++k) {
      v[k] += bv[k];
      if (RELU) v[k] = fmaxf(v[k], 0.f);
    }
    reinterpret_cast<R*>(y)[q] = Vec<T>::pack(v);
  }
}

template <typename T, int CH>
__global__ void __launch_bounds__(kBlk) k_add_bias_relu(int64_t nvec, int64_t C, int64_t inner, const T* a,
                                                          const T* __restrict__ ba, const T* s,
                                                          const T* __restrict__ bs, T* out) {
  constexpr int V = Vec<T>::N;
  typedef typename Vec<T>::raw R;
  const int64_t base = (int64_t)blockIdx.x * (kBlk * kUnr) + threadIdx.x;
  R ra[kUnr], rs[kUnr];
#pragma unroll
  for (int u = 0; u < kUnr; ++u) {
    const int64_t q = base + u * kBlk;
    if (q < nvec) {
      ra[u] = reinterpret_cast<const R*>(a)[q];
      rs[u] = reinterpret_cast<const R*>(s)[q];
    }
  }
#pragma unroll
  for (int u = 0; u < kUnr; ++u) {
    const int64_t q = base + u * kBlk;
    if (q >= nvec) continue;
    float va[V], vs[V], b1[V], b2[V];
    Vec<T>::unpack(ra[u], va);
    Vec<T>::unpack(rs[u], vs);
    load_bias<T, CH>(ba, q * V, C, inner, b1);
    load_bias<T, CH>(bs, q * V, C, inner, b2);
#pragma unroll
    for (int k = 0; k < V; ++k) va[k] = fmaxf((va[k] + b1[k]) + (vs[k] + b2[k]), 0.f);
    reinterpret_cast<R*>(out)[q] = Vec<T>::pack(va);
  }
}

// out = y > 0 ? (g1 [+ g2]) : 0
template <typename T, bool TWO>
__global__ void __launch_bounds__(kBlk) k_relu_mask(int64_t nvec, const T* g1, const T* g2, const T* __restrict__ y,
                                                      T* out) {
  constexpr int V = Vec<T>::N;
  typedef typename Vec<T>::raw R;
  const int64_t base = (int64_t)blockIdx.x * (kBlk * kUnr) + threadIdx.x;
  R rg[kUnr], rh[kUnr], ry[kUnr];
#pragma unroll
  for (int u = 0; u < kUnr; ++u) {
    const int64_t q = base + u * kBlk;
    if (q < nvec) {
      rg[u] = reinterpret_cast<const R*>(g1)[q];
      if (TWO) rh[u] = reinterpret_cast<const R*>(g2)[q];
      ry[u] = reinterpret_cast<const R*>(y)[q];
    }
  }
#pragma unroll
  for (int u = 0; u < kUnr; ++u) {
    const int64_t q = base + u * kBlk;
    if (q >= nvec) continue;
    float vg[V], vh[V], vy[V];
    Vec<T>::unpack(rg[u], vg);
    Vec<T>::unpack(ry[u], vy);
    if (TWO) Vec<T>::unpack(rh[u], vh);
#pragma unroll
    for (int k = 0; k < V; ++k) {
      const float gv = TWO ? vg[k] + vh[k] : vg[k];
      vg[k] = vy[k] > 0.f ? gv : 0.f;
    }
    reinterpret_cast<R*>(out)[q] = Vec<T>::pack(vg);
  }
}

// scalar fallbacks (unaligned pointers, ragged sizes, channel runs not a multiple of the vector)
template <typename T>
__global__ void __launch_bounds__(kBlk) k_ew_scalar(int op, int64_t n, int64_t C, int64_t inner, const T* a,
                                                      const T* ba, const T* s, const T* bs, T* out, int relu) {
  for (int64_t i = (int64_t)blockIdx.x * kBlk + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlk) {
    const int64_t c = (i / inner) % C;
    float v;
    if (op == 0) {  // bias_act: a = y, out = y
      v = ld1(a, i) + (ba ? ld1(ba, c) : 0.f);
      if (relu) v = fmaxf(v, 0.f);
    } else if (op == 1) {  // add_bias_relu
      v = fmaxf((ld1(a, i) + (ba ? ld1(ba, c) : 0.f)) + (ld1(s, i) + (bs ? ld1(bs, c) : 0.f)), 0.f);
    } else {  // relu mask: a = g1, s = g2 (or null), ba = y
      const float gv = s ? ld1(a, i) + ld1(s, i) : ld1(a, i);
      v = ld1(ba, i) > 0.f ? gv : 0.f;
    }
    st1(out, i, v);
  }
}

inline bool al16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

template <typename T>
int channel_layout(int64_t n, int64_t C, int64_t inner, std::initializer_list<const void*> ptrs,
                   std::initializer_list<const void*> biases) {
  constexpr int V = Vec<T>::N;
  if (n % V) return -1;
  for (const void* p : ptrs)
    if (p && !al16(p)) return -1;
  if (inner == 1 && C % V == 0) {
    for (const void* p : biases)
      if (p && !al16(p)) return -1;
    return CH_VEC;
  }
  if (inner % V == 0) return CH_ONE;
  return -1;
}

inline unsigned vec_grid(int64_t nvec) { return (unsigned)((nvec + kBlk * kUnr - 1) / (kBlk * kUnr)); }

template <typename T>
int bias_act(int64_t n, int64_t C, int64_t inner, void* y_, const void* b_, int relu, hipStream_t st) {
  T* y = (T*)y_;
  const T* b = (const T*)b_;
  const int lay = channel_layout<T>(n, C, inner, {y}, {b});
  const int64_t nv = n / Vec<T>::N;
  if (lay == CH_VEC && relu) hipLaunchKernelGGL((k_bias_act<T, CH_VEC, true>), vec_grid(nv), kBlk, 0, st, nv, C, inner, y, b);
  else if (lay == CH_VEC) hipLaunchKernelGGL((k_bias_act<T, CH_VEC, false>), vec_grid(nv), kBlk, 0, st, nv, C, inner, y, b);
  else if (lay == CH_ONE && relu) hipLaunchKernelGGL((k_bias_act<T, CH_ONE, true>), vec_grid(nv), kBlk, 0, st, nv, C, inner, y, b);
  else if (lay == CH_ONE) hipLaunchKernelGGL((k_bias_act<T, CH_ONE, false>), vec_grid(nv), kBlk, 0, st, nv, C, inner, y, b);
  else
    hipLaunchKernelGGL(k_ew_scalar<T>, wam_grid(n, kBlk), kBlk, 0, st, 0, n, C, inner, (const T*)y, b, (const T*)nullptr,
                       (const T*)nullptr, y, relu);
  WAM_LAUNCH_CHECK();
  return WAM_OK;
}

template <typename T>
int add_bias_relu(int64_t n, int64_t C, int64_t inner, const void* a_, const void* ba_, const void* s_,
                  const void* bs_, void* out_, hipStream_t st) {
  const T *a = (const T*)a_, *ba = (const T*)ba_, *s = (const T*)s_, *bs = (const T*)bs_;
  T* out = (T*)out_;
  const int lay = channel_layout<T>(n, C, inner, {a, s, out}, {ba, bs});
  const int64_t nv = n / Vec<T>::N;
  if (lay == CH_VEC)
    hipLaunchKernelGGL((k_add_bias_relu<T, CH_VEC>), vec_grid(nv), kBlk, 0, st, nv, C, inner, a, ba, s, bs, out);
  else if (lay == CH_ONE)
    hipLaunchKernelGGL((k_add_bias_relu<T, CH_ONE>), vec_grid(nv), kBlk, 0, st, nv, C, inner, a, ba, s, bs, out);
  else
    hipLaunchKernelGGL(k_ew_scalar<T>, wam_grid(n, kBlk), kBlk, 0, st, 1, n, C, inner, a, ba, s, bs, out, 1);
  WAM_LAUNCH_CHECK();
  return WAM_OK;
}

template <typename T>
int relu_mask(int64_t n, const void* g1_, const void* g2_, const void* y_, void* out_, hipStream_t st) {
  const T *g1 = (const T*)g1_, *g2 = (const T*)g2_, *y = (const T*)y_;
  T* out = (T*)out_;
  const bool vec = n % Vec<T>::N == 0 && al16(g1) && (!g2 || al16(g2)) && al16(y) && al16(out);
  const int64_t nv = n / Vec<T>::N;
  if (vec && g2) hipLaunchKernelGGL((k_relu_mask<T, true>), vec_grid(nv), kBlk, 0, st, nv, g1, g2, y, out);
  else if (vec) hipLaunchKernelGGL((k_relu_mask<T, false>), vec_grid(nv), kBlk, 0, st, nv, g1, g2, y, out);
  else
    hipLaunchKernelGGL(k_ew_scalar<T>, wam_grid(n, kBlk), kBlk, 0, st, 2, n, (int64_t)1, (int64_t)1, g1, y, g2,
                       (const T*)nullptr, out, 0);
  WAM_LAUNCH_CHECK();
  return WAM_OK;
}

}  // namespace

extern "C" {

int wam_ew_bias_act(int dtype, int64_t n, int64_t channels, int64_t inner, void* y, const void* bias, int relu,
                    void* stream) {
  if (n < 0 || channels < 1 || inner < 1 || (n > 0 && !y) || (dtype != WAM_DT_F32 && dtype != WAM_DT_BF16))
    return WAM_ERR_INVALID_ARG;
  if (n == 0) return WAM_OK;
  return dtype == WAM_DT_F32 ? bias_act<float>(n, channels, inner, y, bias, relu, (hipStream_t)stream)
                             : bias_act<uint16_t>(n, channels, inner, y, bias, relu, (hipStream_t)stream);
}

int wam_ew_add_bias_relu(int dtype, int64_t n, int64_t channels, int64_t inner, const void* a, const void* bias_a,
                         const void* s, const void* bias_s, void* out, void* stream) {
  if (n < 0 || channels < 1 || inner < 1 || (n > 0 && (!a || !s || !out)) ||
      (dtype != WAM_DT_F32 && dtype != WAM_DT_BF16))
    return WAM_ERR_INVALID_ARG;
  if (n == 0) return WAM_OK;
  return dtype == WAM_DT_F32
             ? add_bias_relu<float>(n, channels, inner, a, bias_a, s, bias_s, out, (hipStream_t)stream)
             : add_bias_relu<uint16_t>(n, channels, inner, a, bias_a, s, bias_s, out, (hipStream_t)stream);
}

int wam_ew_relu_mask(int dtype, int64_t n, const void* g1, const void* g2, const void* y, void* out, void* stream) {
  if (n < 0 || (n > 0 && (!g1 || !y || !out)) || (dtype != WAM_DT_F32 && dtype != WAM_DT_BF16))
    return WAM_ERR_INVALID_ARG;
  if (n == 0) return WAM_OK;
  return dtype == WAM_DT_F32 ? relu_mask<float>(n, g1, g2, y, out, (hipStream_t)stream)
                             : relu_mask<uint16_t>(n, g1, g2, y, out, (hipStream_t)stream);
}

}  // extern "C"

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
//   k_maxpool_fwd / k_maxpool_bwd  NHWC max pooling with a byte window index; the backward
//                   also applies the mask of the ReLU that fed the pool (stem relu -> maxpool)
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


// ---- max pooling over a channels_last (NHWC) activation, window index kept as one byte
// Forward: one thread per (n, oy, ox, 16-byte channel vector); max in window scan order with
// torch's rule (first maximum wins, NaN propagates, the index of an all -inf window is its first
// valid position). idx = window position kh * k + kw, bit 7 set when the maximum is > 0 -- the
// ReLU that produced the input is then folded into the backward (a ReLU output is 0 wherever the
// mask would cut the gradient, and a window whose maximum is 0 routes its gradient to a zero).
// Backward (gather, no atomics): one thread per input vector sums, in (oy, ox) order and in fp32,
// the gradients of the <= ceil(k/s)^2 windows whose recorded position is this pixel -- torch's
// max_pool2d backward order. The byte index replaces torch's int64 one: 8x less index traffic.
struct PoolGeom {
  int64_t n, h, w, c, ho, wo;
  int k, s, p;
  int cv, cv_sh, s_sh;  // channel vectors per pixel; log2 of cv / s when a power of two, else -1
};

// a / d through a shift when d is a power of two (floor division; callers clamp negatives to 0)
__device__ __forceinline__ int div_sh(int a, int sh, int d) { return sh >= 0 ? (a >> sh) : a / d; }

// KC: compile-time window size (3 for the ResNet stem; 0 = runtime g.k). With KC all k*k loads
// are issued at once from clamped addresses and masked afterwards, instead of a loop of dependent
// load rounds (the kernel is latency-bound otherwise).
template <typename T, int KC>
__global__ void __launch_bounds__(kBlk) k_maxpool_fwd(PoolGeom g, const T* __restrict__ x, T* __restrict__ y,
                                                        uint8_t* __restrict__ idx) {
  constexpr int V = Vec<T>::N;
  typedef typename Vec<T>::raw R;
  // grid (x: output column x channel vector, y: output row, z: image): no 64-bit divides, which
  // cost ~100 VALU ops each and made the first version issue-bound
  const int t = blockIdx.x * kBlk + threadIdx.x;
  const int ox = div_sh(t, g.cv_sh, g.cv);
  if (ox >= g.wo) return;
  const int64_t c0 = (int64_t)(t - ox * g.cv) * V;
  const int64_t oy = blockIdx.y, n = blockIdx.z;
  const int64_t y0 = oy * g.s - g.p, x0 = ox * g.s - g.p;
  const int ky0 = (int)max<int64_t>(0, -y0), ky1 = (int)min<int64_t>(g.k, g.h - y0);
  const int kx0 = (int)max<int64_t>(0, -x0), kx1 = (int)min<int64_t>(g.k, g.w - x0);
  float m[V];
  int id[V];
#pragma unroll
  for (int j = 0; j < V; ++j) m[j] = -INFINITY, id[j] = ky0 * g.k + kx0;
  if constexpr (KC > 0) {
    R raw[KC * KC];
#pragma unroll
    for (int ky = 0; ky < KC; ++ky) {
      const int64_t yy = min<int64_t>(max<int64_t>(y0 + ky, 0), g.h - 1);
#pragma unroll
      for (int kx = 0; kx < KC; ++kx) {
        const int64_t xx = min<int64_t>(max<int64_t>(x0 + kx, 0), g.w - 1);
        raw[ky * KC + kx] = *reinterpret_cast<const R*>(x + ((n * g.h + yy) * g.w + xx) * g.c + c0);
      }
    }
#pragma unroll
    for (int ky = 0; ky < KC; ++ky)
#pragma unroll
      for (int kx = 0; kx < KC; ++kx) {
        if (ky < ky0 || ky >= ky1 || kx < kx0 || kx >= kx1) continue;
        float v[V];
        Vec<T>::unpack(raw[ky * KC + kx], v);
#pragma unroll
        for (int j = 0; j < V; ++j)
          if (v[j] > m[j] || isnan(v[j])) m[j] = v[j], id[j] = ky * KC + kx;
      }
  } else {
    for (int ky = ky0; ky < ky1; ++ky) {
      const T* row = x + ((n * g.h + y0 + ky) * g.w) * g.c + c0;
      for (int kx = kx0; kx < kx1; ++kx) {
        float v[V];
        Vec<T>::unpack(*reinterpret_cast<const R*>(row + (x0 + kx) * g.c), v);
#pragma unroll
        for (int j = 0; j < V; ++j)
          if (v[j] > m[j] || isnan(v[j])) m[j] = v[j], id[j] = ky * g.k + kx;
      }
    }
  }
  const int64_t o = ((n * g.ho + oy) * g.wo + ox) * g.c + c0;
  *reinterpret_cast<R*>(y + o) = Vec<T>::pack(m);
  uint8_t b[V];
#pragma unroll
  for (int j = 0; j < V; ++j) b[j] = (uint8_t)(id[j] | (m[j] > 0.f ? 0x80 : 0));
  if constexpr (V == 8) {
    uint2 w;
    w.x = b[0] | (b[1] << 8) | (b[2] << 16) | ((uint32_t)b[3] << 24);
    w.y = b[4] | (b[5] << 8) | (b[6] << 16) | ((uint32_t)b[7] << 24);
    *reinterpret_cast<uint2*>(idx + o) = w;
  } else {
    *reinterpret_cast<uint32_t*>(idx + o) = b[0] | (b[1] << 8) | (b[2] << 16) | ((uint32_t)b[3] << 24);
  }
}

// W2: at most 2 windows per axis cover a pixel (ceil(k / s) <= 2, e.g. 3x3 stride 2): the four
// candidate (gradient, index) pairs are loaded at once from clamped addresses, then summed in
// the loop's (oy, ox) order.
template <typename T, bool RELU, bool W2>
__global__ void __launch_bounds__(kBlk) k_maxpool_bwd(PoolGeom g, const T* __restrict__ gy,
                                                        const uint8_t* __restrict__ idx, T* __restrict__ gx) {
  constexpr int V = Vec<T>::N;
  typedef typename Vec<T>::raw R;
  const int t = blockIdx.x * kBlk + threadIdx.x;
  const int ix = div_sh(t, g.cv_sh, g.cv);
  if (ix >= g.w) return;
  const int64_t c0 = (int64_t)(t - ix * g.cv) * V;
  const int iy = blockIdx.y;
  const int64_t n = blockIdx.z;
  // windows oy with oy*s - p <= iy <= oy*s - p + k - 1
  const int ho = (int)g.ho, wo = (int)g.wo;
  const int oy0 = max(0, div_sh(iy + g.p - g.k + g.s, g.s_sh, g.s)), oy1 = min(ho - 1, div_sh(iy + g.p, g.s_sh, g.s));
  const int ox0 = max(0, div_sh(ix + g.p - g.k + g.s, g.s_sh, g.s)), ox1 = min(wo - 1, div_sh(ix + g.p, g.s_sh, g.s));
  float acc[V];
#pragma unroll
  for (int j = 0; j < V; ++j) acc[j] = 0.f;
  auto unpack_idx = [&](const uint8_t* ip, uint8_t (&b)[V]) {
    if constexpr (V == 8) {
      const uint2 w = *reinterpret_cast<const uint2*>(ip);
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = (uint8_t)(w.x >> (8 * j)), b[4 + j] = (uint8_t)(w.y >> (8 * j));
    } else {
      const uint32_t w = *reinterpret_cast<const uint32_t*>(ip);
#pragma unroll
      for (int j = 0; j < V; ++j) b[j] = (uint8_t)(w >> (8 * j));
    }
  };
  auto add = [&](const float (&v)[V], const uint8_t (&b)[V], int pos) {
#pragma unroll
    for (int j = 0; j < V; ++j)
      if ((b[j] & 0x7f) == pos && (!RELU || (b[j] & 0x80))) acc[j] += v[j];
  };
  if constexpr (W2) {
    R rg[4];
    uint8_t rb[4][V];
    int wy[2], wx[2];
    bool ok[4];
    wy[0] = min(oy0, ho - 1), wy[1] = min(oy0 + 1, ho - 1);
    wx[0] = min(ox0, wo - 1), wx[1] = min(ox0 + 1, wo - 1);
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int64_t o = ((n * g.ho + wy[a]) * g.wo + wx[b]) * g.c + c0;
        rg[2 * a + b] = *reinterpret_cast<const R*>(gy + o);
        unpack_idx(idx + o, rb[2 * a + b]);
        ok[2 * a + b] = oy0 + a <= oy1 && ox0 + b <= ox1;
      }
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        if (!ok[2 * a + b]) continue;
        const int pos = (iy - ((oy0 + a) * g.s - g.p)) * g.k + (ix - ((ox0 + b) * g.s - g.p));
        float v[V];
        Vec<T>::unpack(rg[2 * a + b], v);
        add(v, rb[2 * a + b], pos);
      }
  } else {
    for (int oy = oy0; oy <= oy1; ++oy) {
      const int py = iy - (oy * g.s - g.p);
      for (int ox = ox0; ox <= ox1; ++ox) {
        const int pos = py * g.k + (ix - (ox * g.s - g.p));
        const int64_t o = ((n * g.ho + oy) * g.wo + ox) * g.c + c0;
        float v[V];
        Vec<T>::unpack(*reinterpret_cast<const R*>(gy + o), v);
        uint8_t b[V];
        unpack_idx(idx + o, b);
        add(v, b, pos);
      }
    }
  }
  *reinterpret_cast<R*>(gx + ((n * g.h + iy) * g.w + ix) * g.c + c0) = Vec<T>::pack(acc);
}

inline int log2_exact(int64_t d) {
  for (int b = 0; b < 31; ++b)
    if ((int64_t(1) << b) == d) return b;
  return -1;
}

// fill the launch-side fields; false when a grid dimension or a 32-bit index would overflow
inline bool pool_grid(PoolGeom& g, int V) {
  g.cv = (int)(g.c / V);
  g.cv_sh = (int)log2_exact(g.cv);
  g.s_sh = (int)log2_exact(g.s);
  const int64_t lim = 65535;
  return g.n <= lim && g.h <= lim && g.ho <= lim && g.w * g.cv < (int64_t(1) << 30) &&
         g.n * g.h * g.w * g.c < (int64_t(1) << 62);
}

template <typename T>
int maxpool(const PoolGeom& g, const void* x, void* y, void* idx, hipStream_t st) {
  constexpr int V = Vec<T>::N;
  if (g.c % V || !al16(x) || !al16(y) || ((uintptr_t)idx & (V - 1))) return WAM_ERR_UNSUPPORTED;
  PoolGeom gg = g;
  if (!pool_grid(gg, V)) return WAM_ERR_UNSUPPORTED;
  const dim3 grid((unsigned)((gg.wo * gg.cv + kBlk - 1) / kBlk), (unsigned)gg.ho, (unsigned)gg.n);
  if (gg.k == 3)
    hipLaunchKernelGGL((k_maxpool_fwd<T, 3>), grid, kBlk, 0, st, gg, (const T*)x, (T*)y, (uint8_t*)idx);
  else
    hipLaunchKernelGGL((k_maxpool_fwd<T, 0>), grid, kBlk, 0, st, gg, (const T*)x, (T*)y, (uint8_t*)idx);
  WAM_LAUNCH_CHECK();
  return WAM_OK;
}

template <typename T>
int maxpool_bwd(const PoolGeom& g, const void* gy, const void* idx, void* gx, int relu, hipStream_t st) {
  constexpr int V = Vec<T>::N;
  if (g.c % V || !al16(gy) || !al16(gx) || ((uintptr_t)idx & (V - 1))) return WAM_ERR_UNSUPPORTED;
  PoolGeom gg = g;
  if (!pool_grid(gg, V)) return WAM_ERR_UNSUPPORTED;
  const dim3 grid((unsigned)((gg.w * gg.cv + kBlk - 1) / kBlk), (unsigned)gg.h, (unsigned)gg.n);
  const bool w2 = (gg.k + gg.s - 1) / gg.s <= 2;
  const T* gyp = (const T*)gy;
  const uint8_t* ip = (const uint8_t*)idx;
  if (relu && w2) hipLaunchKernelGGL((k_maxpool_bwd<T, true, true>), grid, kBlk, 0, st, gg, gyp, ip, (T*)gx);
  else if (relu) hipLaunchKernelGGL((k_maxpool_bwd<T, true, false>), grid, kBlk, 0, st, gg, gyp, ip, (T*)gx);
  else if (w2) hipLaunchKernelGGL((k_maxpool_bwd<T, false, true>), grid, kBlk, 0, st, gg, gyp, ip, (T*)gx);
  else hipLaunchKernelGGL((k_maxpool_bwd<T, false, false>), grid, kBlk, 0, st, gg, gyp, ip, (T*)gx);
  WAM_LAUNCH_CHECK();
  return WAM_OK;
}

inline bool pool_geom(PoolGeom& g, int64_t n, int64_t h, int64_t w, int64_t c, int k, int s, int p) {
  if (n < 0 || h < 1 || w < 1 || c < 1 || k < 1 || k * k > 127 || s < 1 || p < 0 || 2 * p > k) return false;
  g.n = n, g.h = h, g.w = w, g.c = c, g.k = k, g.s = s, g.p = p;
  g.ho = (h + 2 * p - k) / s + 1;
  g.wo = (w + 2 * p - k) / s + 1;
  return g.ho >= 1 && g.wo >= 1;
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

int wam_ew_maxpool_nhwc(int dtype, int64_t n, int64_t h, int64_t w, int64_t c, int k, int stride, int pad,
                        const void* x, void* y, void* idx, void* stream) {
  PoolGeom g;
  if (!pool_geom(g, n, h, w, c, k, stride, pad) || (n > 0 && (!x || !y || !idx)) ||
      (dtype != WAM_DT_F32 && dtype != WAM_DT_BF16))
    return WAM_ERR_INVALID_ARG;
  if (n == 0) return WAM_OK;
  return dtype == WAM_DT_F32 ? maxpool<float>(g, x, y, idx, (hipStream_t)stream)
                             : maxpool<uint16_t>(g, x, y, idx, (hipStream_t)stream);
}

int wam_ew_maxpool_nhwc_backward(int dtype, int64_t n, int64_t h, int64_t w, int64_t c, int k, int stride, int pad,
                                 const void* gy, const void* idx, int relu, void* gx, void* stream) {
  PoolGeom g;
  if (!pool_geom(g, n, h, w, c, k, stride, pad) || (n > 0 && (!gy || !idx || !gx)) ||
      (dtype != WAM_DT_F32 && dtype != WAM_DT_BF16))
    return WAM_ERR_INVALID_ARG;
  if (n == 0) return WAM_OK;
  return dtype == WAM_DT_F32 ? maxpool_bwd<float>(g, gy, idx, gx, relu, (hipStream_t)stream)
                             : maxpool_bwd<uint16_t>(g, gy, idx, gx, relu, (hipStream_t)stream);
}

}  // extern "C"

// WAM-specific kernels around the transforms: SmoothGrad noise, per-subband channel-mean |.| with
// batch-global maxima, mosaic / cube accumulation (SmoothGrad mean, IG trapezoid, legacy 3D
// averaging), generic sample accumulators and the .scales reprojection.
// Reference: lib/wam_2D.py:200-264 (visualize_grad_wam), :268-341 (_reproject_wam),
// :379-415 (smooth_gradcam), :417-459 (intergrated_wam), :488-536 (reproject_wam);
// lib/wam_1D.py:294-343, :353-421; lib/wam_3D.py:127-166, :550-591, :614-643.
#include <math.h>

#include "kernels.hpp"
#include "rng.hpp"

namespace {

// numpy-compatible max: NaN propagates (fmaxf would drop it)
__device__ __forceinline__ float nan_max(float a, float b) { return (a != a || a > b) ? a : b; }

// ------------------------------------------------------------------------------ sigma
__device__ __forceinline__ float nan_min(float a, float b) { return (a != a || a < b) ? a : b; }

// One 1024-thread block per item; VEC4 streams 16-byte loads, 4 in flight per thread.
// max/min propagate NaN like torch.max / torch.min.
template <bool VEC4>
__global__ void __launch_bounds__(1024) k_item_sigma(const float* __restrict__ x, int64_t item_stride, int64_t len,
                                                     float spread, float* __restrict__ sigma) {
  const float* xi = x + blockIdx.x * item_stride;
  float mx = -INFINITY, mn = INFINITY;
  if constexpr (VEC4) {
    const float4* x4 = reinterpret_cast<const float4*>(xi);
    const int64_t n4 = len >> 2;
    int64_t e = threadIdx.x;
    for (; e + 3 * 1024 < n4; e += 4 * 1024) {
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = x4[e + u * 1024];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        mx = nan_max(nan_max(mx, v[u].x), nan_max(nan_max(v[u].y, v[u].z), v[u].w));
        mn = nan_min(nan_min(mn, v[u].x), nan_min(nan_min(v[u].y, v[u].z), v[u].w));
      }
    }
    for (; e < n4; e += 1024) {
      const float4 v = x4[e];
      mx = nan_max(nan_max(mx, v.x), nan_max(nan_max(v.y, v.z), v.w));
      mn = nan_min(nan_min(mn, v.x), nan_min(nan_min(v.y, v.z), v.w));
    }
  } else {
    for (int64_t e = threadIdx.x; e < len; e += 1024) {
      const float v = xi[e];
      mx = nan_max(mx, v);
      mn = nan_min(mn, v);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    mx = nan_max(mx, __shfl_xor(mx, o, 64));
    mn = nan_min(mn, __shfl_xor(mn, o, 64));
  }
  __shared__ float smx[16], smn[16];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) {
    smx[wv] = mx;
    smn[wv] = mn;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 16; ++w) {
      mx = nan_max(mx, smx[w]);
      mn = nan_min(mn, smn[w]);
    }
    // torch: spread * (max - min) in fp32 with the python scalar cast to fp32
    sigma[blockIdx.x] = spread * (mx - mn);
  }
}

// Full-chip form (wam_item_sigma_ws): each item is split into `chunks` ranges, one 256-thread
// workgroup per (item, range) -- thousands of workgroups where the one-block-per-item form had 16
// (c5) to 256 (c3) -- and the last workgroup of an item to arrive (arrival counter in the caller's
// workspace) combines the partial (max, min) pairs. max / min are exact, so the result is the
// single-block kernel's bit for bit, NaN propagation included.
constexpr int kSigT = 256;
template <bool VEC4>
__global__ void __launch_bounds__(kSigT) k_item_sigma_split(const float* __restrict__ x, int64_t item_stride,
                                                            int64_t len, int64_t chunk, int chunks, float spread,
                                                            float* __restrict__ sigma, float2* __restrict__ part,
                                                            unsigned int* __restrict__ cnt) {
  const int64_t wg = blockIdx.x, item = wg / chunks;
  const int64_t b = (wg - item * chunks) * chunk, e = min(len, b + chunk);
  const float* xi = x + item * item_stride;
  float mx = -INFINITY, mn = INFINITY;
  if constexpr (VEC4) {  // chunk and len multiples of 4
    const float4* x4 = reinterpret_cast<const float4*>(xi);
    const int64_t e4 = e >> 2;
    int64_t i = (b >> 2) + threadIdx.x;
    for (; i + 7 * kSigT < e4; i += 8 * kSigT) {  // 8 16-byte loads in flight per lane
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = x4[i + u * kSigT];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        mx = nan_max(nan_max(mx, v[u].x), nan_max(nan_max(v[u].y, v[u].z), v[u].w));
        mn = nan_min(nan_min(mn, v[u].x), nan_min(nan_min(v[u].y, v[u].z), v[u].w));
      }
    }
    for (; i < e4; i += kSigT) {
      const float4 v = x4[i];
      mx = nan_max(nan_max(mx, v.x), nan_max(nan_max(v.y, v.z), v.w));
      mn = nan_min(nan_min(mn, v.x), nan_min(nan_min(v.y, v.z), v.w));
    }
  } else {
    for (int64_t i = b + threadIdx.x; i < e; i += kSigT) {
      const float v = xi[i];
      mx = nan_max(mx, v);
      mn = nan_min(mn, v);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    mx = nan_max(mx, __shfl_xor(mx, o, 64));
    mn = nan_min(mn, __shfl_xor(mn, o, 64));
  }
  __shared__ float smx[kSigT / 64], smn[kSigT / 64];
  __shared__ unsigned int last;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) {
    smx[wv] = mx;
    smn[wv] = mn;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < kSigT / 64; ++w) {
      mx = nan_max(mx, smx[w]);
      mn = nan_min(mn, smn[w]);
    }
    if (chunks == 1) {
      sigma[item] = spread * (mx - mn);
      last = 0u;
    } else {
      // hand-off without fences (an agent-scope release writes back the whole L2 of this XCD --
      // every dirty line the previous kernels left -- and cost more than the reduction): the
      // partial goes out write-through (agent-scope store, sc1) and is drained before the arrival
      // is counted (MI355X_MICROARCH.md, inter-workgroup visibility, the sc1 form)
      __hip_atomic_store(reinterpret_cast<unsigned long long*>(part + wg),
                         (unsigned long long)__float_as_uint(mx) | ((unsigned long long)__float_as_uint(mn) << 32),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      last = __hip_atomic_fetch_add(cnt + item, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
             (unsigned)chunks - 1;
    }
  }
  __syncthreads();
  if (!last || wv != 0) return;
  // the last range of the item: its first wave reads the partials with agent-scope (sc1) loads, one
  // per lane, and reduces them across the wave
  const unsigned long long* pp = reinterpret_cast<const unsigned long long*>(part + item * chunks);
  float MX = -INFINITY, MN = INFINITY;
  for (int k = lane; k < chunks; k += 64) {
    const unsigned long long u = __hip_atomic_load(pp + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    MX = nan_max(MX, __uint_as_float((unsigned)u));
    MN = nan_min(MN, __uint_as_float((unsigned)(u >> 32)));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    MX = nan_max(MX, __shfl_xor(MX, o, 64));
    MN = nan_min(MN, __shfl_xor(MN, o, 64));
  }
  if (lane == 0) {
    // torch: spread * (max - min) in fp32 with the python scalar cast to fp32
    sigma[item] = spread * (MX - MN);
    // the counter is left zeroed for the next call (write-through, like the partials)
    __hip_atomic_store(cnt + item, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// ranges per item: about 2,048 workgroups over the call (every CU a few ranges, so the loads of
// one range overlap the next's), each range >= 8 K floats so that an item's arrivals on its counter
// (serialised at the memory side) stay few: c2 at 32 ranges of 4.7 K floats per image ran 21 us,
// 18 ranges of 8.4 K run at the copy rate (profiles/r05f_sigma_split.log)
void sigma_split(int64_t items, int64_t len, bool vec4, int64_t& chunk, int& chunks) {
  int64_t c = (2048 + items - 1) / items;
  const int64_t cap = len / 8192 > 1 ? len / 8192 : 1;
  if (c > cap) c = cap;
  if (c < 1) c = 1;
  chunk = (len + c - 1) / c;
  if (vec4) chunk = (chunk + 3) & ~int64_t(3);
  chunks = (int)((len + chunk - 1) / chunk);
}

// ------------------------------------------------------------------------------ Philox noise
// One thread per group of 4 consecutive elements of an item: one Philox call -> 4 normals.
// VEC4: item_stride % 4 == 0, so groups never straddle items and loads/stores are 16 B.
template <bool VEC4>
__global__ void __launch_bounds__(256) k_noise_add(int64_t n_samples, int64_t items, int64_t item_stride,
                                                   int64_t noised_len, const float* __restrict__ x,
                                                   const float* __restrict__ sigma,
                                                   const float* __restrict__ host_noise, uint32_t k0, uint32_t k1,
                                                   int64_t sample_base, int64_t item_base,
                                                   float* __restrict__ out) {
  const int64_t groups = (item_stride + 3) / 4;
  const int64_t total = n_samples * items * groups;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    int64_t g = t % groups;
    int64_t q = t / groups;
    int64_t i = q % items;
    int64_t s = q / items;
    float z[4] = {0.f, 0.f, 0.f, 0.f};
    if (!host_noise && 4 * g < noised_len) wam_normal4(g, item_base + i, sample_base + s, k0, k1, z);
    const float sg = host_noise ? 0.f : sigma[i];
    const float* xi = x + i * item_stride;
    float* oi = out + (s * items + i) * item_stride;
    const float* hn = host_noise ? host_noise + (s * items + i) * item_stride : nullptr;
    if (VEC4 && 4 * g + 4 <= noised_len) {
      float4 xv = *reinterpret_cast<const float4*>(xi + 4 * g);
      float4 o;
      if (hn) {
        float4 nv = *reinterpret_cast<const float4*>(hn + 4 * g);
        o = make_float4(xv.x + nv.x, xv.y + nv.y, xv.z + nv.z, xv.w + nv.w);
      } else {  // noisy = fma(sigma, z, x): the same rounding as the fused noisy analysis
        o = make_float4(fmaf(sg, z[0], xv.x), fmaf(sg, z[1], xv.y), fmaf(sg, z[2], xv.z), fmaf(sg, z[3], xv.w));
      }
      *reinterpret_cast<float4*>(oi + 4 * g) = o;
      continue;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      int64_t e = 4 * g + u;
      if (e >= item_stride) break;
      float v;
      if (e < noised_len) v = hn ? xi[e] + hn[e] : fmaf(sg, z[u], xi[e]);
      else v = 0.f;
      oi[e] = v;
    }
  }
}

// ------------------------------------------------------------------------------ subband maps
struct BandTable {
  int64_t off[WAM_MAX_BANDS + 1];   // per-item packed offsets
  int32_t tile0[WAM_MAX_BANDS + 1];  // first tile of each band (prefix over ceil(nb / TILE))
  int nbands;
};
constexpr int kMapTile = 8192;  // elements per block (32 per thread): one band-max atomic per 32 KB

// grid: x = tile (over all bands), y = item. One atomic max per block. Every thread issues all of
// its loads of a channel before using any (addresses clamped into the band, results of the clamped
// slots dropped at the store): a load guarded by `q < nb` made the compiler wait for each one in
// turn. VEC4 (host check: every band offset and length a multiple of 4): 16-byte loads / stores.
template <bool VEC4>
__global__ void __launch_bounds__(256) k_subband_maps(BandTable bt, int64_t items_total, int64_t group_items,
                                                      int channels, const float* __restrict__ g,
                                                      float* __restrict__ maps, float* __restrict__ band_max) {
  constexpr int PER = kMapTile / 256;  // elements per thread
  constexpr int V = VEC4 ? 4 : 1;
  constexpr int NL = PER / V;          // loads per thread and channel
  const int tile = blockIdx.x;
  int b = 0;
  while (b + 1 < bt.nbands && bt.tile0[b + 1] <= tile) ++b;
  const int64_t item = blockIdx.y;
  const int64_t nb = bt.off[b + 1] - bt.off[b];
  const int64_t q0 = (int64_t)(tile - bt.tile0[b]) * kMapTile;
  const float* base = g + items_total * channels * bt.off[b] + (item * channels) * nb;
  float* out = maps + item * bt.off[bt.nbands] + bt.off[b];
  float acc[PER];
  for (int c = 0; c < channels; ++c) {
    const float* bc = base + (int64_t)c * nb;
    float ld[PER];
#pragma unroll
    for (int u = 0; u < NL; ++u) {
      const int64_t q = q0 + ((int64_t)u * 256 + threadIdx.x) * V;
      const int64_t qc = q < nb ? q : nb - V;
      if constexpr (VEC4) {
        const float4 t = *reinterpret_cast<const float4*>(bc + qc);
        ld[4 * u] = t.x;
        ld[4 * u + 1] = t.y;
        ld[4 * u + 2] = t.z;
        ld[4 * u + 3] = t.w;
      } else {
        ld[u] = bc[qc];
      }
    }
#pragma unroll
    for (int k = 0; k < PER; ++k) acc[k] = c ? acc[k] + ld[k] : ld[k];  // ((g0 + g1) + g2): numpy's sum
  }
  const float inv_c = (float)channels;
  float m = 0.f;
#pragma unroll
  for (int u = 0; u < NL; ++u) {
    const int64_t q = q0 + ((int64_t)u * 256 + threadIdx.x) * V;
    float v[V];
#pragma unroll
    for (int k = 0; k < V; ++k) v[k] = fabsf(acc[V * u + k] / inv_c);  // numpy mean: sum then true_divide
    if (q < nb) {
      if constexpr (VEC4) *reinterpret_cast<float4*>(out + q) = make_float4(v[0], v[1], v[2], v[3]);
      else out[q] = v[0];
#pragma unroll
      for (int k = 0; k < V; ++k) m = nan_max(m, v[k]);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = nan_max(m, __shfl_xor(m, o, 64));
  __shared__ float sm[4];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) sm[wv] = m;
  __syncthreads();
  if (threadIdx.x == 0 && band_max) {  // band_max == NULL: maps only (3D cube, no normalisation)
    for (int w = 1; w < 4; ++w) m = nan_max(m, sm[w]);
    const int64_t grp = item / group_items;
    // non-negative floats order like their bit patterns; NaN (0x7fc00000) wins like numpy's max
    atomicMax(reinterpret_cast<unsigned int*>(band_max + grp * bt.nbands + b), __float_as_uint(m));
  }
}

// ------------------------------------------------------------------------------ frame accumulate
__global__ void __launch_bounds__(256) k_frame_accumulate(int64_t groups, int64_t group_items, int64_t frame_len,
                                                          const int32_t* __restrict__ src,
                                                          const int32_t* __restrict__ band,
                                                          const float* __restrict__ maps, int64_t maps_item_len,
                                                          const float* __restrict__ band_max, int n_bands,
                                                          int normalize, double* __restrict__ frame) {
  const int64_t total = group_items * frame_len;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t p = t % frame_len;
    const int64_t n = t / frame_len;
    const int32_t sidx = src[p];
    if (sidx < 0) continue;
    const int32_t b = band[p];
    double acc = frame[t];
    // samples in blocks of 8: the block's loads are issued together, the fp64 sum stays in
    // sample order (the reference accumulates sample by sample)
    const float* mp = maps + n * maps_item_len + sidx;
    const int64_t mstride = group_items * maps_item_len;
    int64_t s = 0;
    for (; s + 8 <= groups; s += 8) {
      float v[8], m[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        v[u] = mp[(s + u) * mstride];
        m[u] = normalize ? band_max[(s + u) * n_bands + b] : 1.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += (double)(normalize ? v[u] / m[u] : v[u]);
    }
    for (; s < groups; ++s) {
      float v = mp[s * mstride];
      if (normalize) v = v / band_max[s * n_bands + b];
      acc += (double)v;
    }
    frame[t] = acc;
  }
}

// the same accumulation in COEFFICIENT order (dst = frame pixel of coefficient k or -1; the mosaic
// is injective): the maps are read as contiguous rows (whole cache lines) and only the fp64 frame
// is addressed through the mosaic, so the partial lines at band-row edges fall on the 16-B/pixel
// frame instead of the per-sample map reads. Per pixel the sum order is unchanged (bit-identical).
__global__ void __launch_bounds__(256) k_frame_accumulate_coef(int64_t groups, int64_t group_items,
                                                               int64_t maps_item_len, int64_t frame_len,
                                                               const int32_t* __restrict__ dst,
                                                               const int32_t* __restrict__ cband,
                                                               const float* __restrict__ maps,
                                                               const float* __restrict__ band_max, int n_bands,
                                                               int normalize, int64_t items_per_thread,
                                                               double* __restrict__ frame) {
  // thread per (coefficient k, run of items_per_thread items): the mosaic tables (8 B per
  // coefficient, several MB at 512^2, beyond an XCD's L2) are read once per run of items instead of
  // once per item
  const int64_t mstride = group_items * maps_item_len;
  const int64_t runs = (group_items + items_per_thread - 1) / items_per_thread;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < runs * maps_item_len;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = t / maps_item_len;
    const int64_t k = t - r * maps_item_len;
    const int32_t d = dst[k];
    if (d < 0) continue;
    const int32_t b = cband[k];
    const int64_t n1 = min(group_items, (r + 1) * items_per_thread);
    for (int64_t n = r * items_per_thread; n < n1; ++n) {
      double* fp = frame + n * frame_len + d;
      double acc = *fp;
      const float* mp = maps + n * maps_item_len + k;
      int64_t s = 0;
      for (; s + 8 <= groups; s += 8) {
        float v[8], m[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          v[u] = mp[(s + u) * mstride];
          m[u] = normalize ? band_max[(s + u) * n_bands + b] : 1.f;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += (double)(normalize ? v[u] / m[u] : v[u]);
      }
      for (; s < groups; ++s) {
        float v = mp[s * mstride];
        if (normalize) v = v / band_max[s * n_bands + b];
        acc += (double)v;
      }
      *fp = acc;
    }
  }
}

__device__ __forceinline__ float nan_to_num(float v) {
  if (v != v) return 0.f;
  if (isinf(v)) return v > 0 ? 3.4028234663852886e+38f : -3.4028234663852886e+38f;
  return v;
}

__global__ void __launch_bounds__(256) k_frame_trapz(int64_t groups, int64_t k0, int64_t group_items, int64_t frame_len,
                                                     const int32_t* __restrict__ src, const int32_t* __restrict__ band,
                                                     const float* __restrict__ maps, int64_t maps_item_len,
                                                     const float* __restrict__ band_max, int n_bands, int normalize,
                                                     const float* __restrict__ weights, float* __restrict__ prev,
                                                     float* __restrict__ acc) {
  const int64_t total = group_items * frame_len;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t p = t % frame_len;
    const int64_t n = t / frame_len;
    const int32_t sidx = src[p];
    const int32_t b = sidx >= 0 ? band[p] : 0;  // pixels outside the mosaic load a valid dummy
    float a = acc[t];
    float pv = prev[t];
    // loads in blocks of 8 steps (issued together), the trapezoid / weighted sum in step order
    const float* mp = maps + n * maps_item_len + (sidx >= 0 ? sidx : 0);
    const int64_t mstride = group_items * maps_item_len;
    auto step = [&](int64_t s, float v, float m) {
      if (sidx < 0) v = 0.f;
      else if (normalize) v = v / m;
      v = nan_to_num(v);
      if (weights) {
        a = fmaf(weights[s], v, a);
      } else {
        if (k0 + s > 0) a = a + (pv + v) / 2.0f;
        pv = v;
      }
    };
    int64_t s = 0;
    for (; s + 8 <= groups; s += 8) {
      float v[8], m[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        v[u] = mp[(s + u) * mstride];
        m[u] = normalize ? band_max[(s + u) * n_bands + b] : 1.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) step(s + u, v[u], m[u]);
    }
    for (; s < groups; ++s) step(s, mp[s * mstride], normalize ? band_max[s * n_bands + b] : 1.f);
    acc[t] = a;
    prev[t] = pv;
  }
}

// k_frame_trapz in COEFFICIENT order (see k_frame_accumulate_coef): thread per (coefficient k,
// run of items), maps read as contiguous rows, the fp32 frame (acc, prev) addressed through the
// injective mosaic. Pixels outside the mosaic are never touched: the pixel-order kernel adds
// (0 + 0) / 2 or w * 0 to their zero-initialised sums, i.e. leaves them as they are. Per pixel the
// step order and arithmetic are those of k_frame_trapz (bit-identical).
__global__ void __launch_bounds__(256) k_frame_trapz_coef(int64_t groups, int64_t k0, int64_t group_items,
                                                          int64_t maps_item_len, int64_t frame_len,
                                                          const int32_t* __restrict__ dst,
                                                          const int32_t* __restrict__ cband,
                                                          const float* __restrict__ maps,
                                                          const float* __restrict__ band_max, int n_bands,
                                                          int normalize, const float* __restrict__ weights,
                                                          int64_t items_per_thread, float* __restrict__ prev,
                                                          float* __restrict__ acc) {
  const int64_t mstride = group_items * maps_item_len;
  const int64_t runs = (group_items + items_per_thread - 1) / items_per_thread;
  // XCD-aware block order: a thread's run of items and the neighbouring runs of the same
  // coefficients land on one XCD, whose L2 then holds the mosaic tables and the lines shared by
  // neighbouring blocks (c4 trapezoid PMC/algorithmic 1.19 without it, 1.07 with it)
  for (int64_t t = wam_xcd_block(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x; t < runs * maps_item_len;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = t / maps_item_len;
    const int64_t k = t - r * maps_item_len;
    const int32_t d = dst[k];
    if (d < 0) continue;
    const int32_t b = cband[k];
    const int64_t n1 = min(group_items, (r + 1) * items_per_thread);
    for (int64_t n = r * items_per_thread; n < n1; ++n) {
      const int64_t fi = n * frame_len + d;
      float a = acc[fi];
      float pv = prev[fi];
      const float* mp = maps + n * maps_item_len + k;
      auto step = [&](int64_t s, float v, float m) {
        if (normalize) v = v / m;
        v = nan_to_num(v);
        if (weights) {
          a = fmaf(weights[s], v, a);
        } else {
          if (k0 + s > 0) a = a + (pv + v) / 2.0f;
          pv = v;
        }
      };
      int64_t s = 0;
      for (; s + 8 <= groups; s += 8) {
        float v[8], m[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          v[u] = mp[(s + u) * mstride];
          m[u] = normalize ? band_max[(s + u) * n_bands + b] : 1.f;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) step(s + u, v[u], m[u]);
      }
      for (; s < groups; ++s) step(s, mp[s * mstride], normalize ? band_max[s * n_bands + b] : 1.f);
      acc[fi] = a;
      prev[fi] = pv;
    }
  }
}

// cube: value = |g| from item-major maps (channels = 1); see wam_cube_accumulate
__global__ void __launch_bounds__(256) k_cube_accumulate(int64_t groups, int64_t k0, int64_t group_items,
                                                         int64_t cube_len, const int32_t* __restrict__ src,
                                                         const float* __restrict__ maps, int64_t maps_item_len, int mode,
                                                         float n_total, const float* __restrict__ weights,
                                                         float* __restrict__ prev, float* __restrict__ acc) {
  const int64_t total = group_items * cube_len;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t p = t % cube_len;
    const int64_t n = t / cube_len;
    const int32_t sidx = src[p];
    float a = acc[t];
    float pv = prev ? prev[t] : 0.f;
    for (int64_t s = 0; s < groups; ++s) {
      float v = sidx >= 0 ? maps[(s * group_items + n) * maps_item_len + sidx] : 0.f;
      if (mode == 0) {
        a = (a + v) / n_total;
      } else if (mode == 1) {
        a = fmaf(weights[s], v, a);
      } else {
        v = nan_to_num(v);
        if (k0 + s > 0) a = a + (pv + v) / 2.0f;
        pv = v;
      }
    }
    acc[t] = a;
    if (prev) prev[t] = pv;
  }
}

// the same, four voxels per thread, all index / accumulator / gathered map loads of a thread issued
// before the first use -- the one-voxel form made every voxel a dependent index -> map load chain
// (c5: 178 us per launch, profiles/r06z_trace_window_c5.txt). Per voxel the sample order and the
// arithmetic are unchanged. STRIDED: voxels b + lane + 64 u (u < 4) of a 256-voxel wave block, so
// each load instruction covers 64 consecutive voxels (the gathers follow the mosaic's runs of
// consecutive coefficients); otherwise four consecutive voxels per thread with 16-byte index /
// accumulator accesses (cube_len % 4 == 0, 16-byte aligned).
template <bool STRIDED>
__global__ void __launch_bounds__(256) k_cube_accumulate4(int64_t groups, int64_t k0, int64_t group_items,
                                                          int64_t cube_len, const int32_t* __restrict__ src,
                                                          const float* __restrict__ maps, int64_t maps_item_len,
                                                          int mode, float n_total, const float* __restrict__ weights,
                                                          float* __restrict__ prev, float* __restrict__ acc) {
  const int64_t total4 = group_items * cube_len / 4;  // 4-voxel units (cube_len % 4 == 0)
  const int lane = threadIdx.x & 63;
  for (int64_t t4 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t4 < total4; t4 += (int64_t)gridDim.x * blockDim.x) {
    int64_t tv[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) tv[e] = STRIDED ? 4 * (t4 - lane) + lane + 64 * e : 4 * t4 + e;
    int sv[4];
    float a[4], pv[4] = {0.f, 0.f, 0.f, 0.f};
    if constexpr (STRIDED) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        sv[e] = src[tv[e] % cube_len];
        a[e] = acc[tv[e]];
        if (prev) pv[e] = prev[tv[e]];
      }
    } else {
      const int4 si = *reinterpret_cast<const int4*>(src + tv[0] % cube_len);
      sv[0] = si.x, sv[1] = si.y, sv[2] = si.z, sv[3] = si.w;
      const float4 a4 = *reinterpret_cast<const float4*>(acc + tv[0]);
      a[0] = a4.x, a[1] = a4.y, a[2] = a4.z, a[3] = a4.w;
      if (prev) {
        const float4 p4 = *reinterpret_cast<const float4*>(prev + tv[0]);
        pv[0] = p4.x, pv[1] = p4.y, pv[2] = p4.z, pv[3] = p4.w;
      }
    }
    int64_t nv[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) nv[e] = tv[e] / cube_len;
    for (int64_t s = 0; s < groups; s += 4) {  // up to 4 samples' gathers in flight per voxel
      float v[4][4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t su = s + u < groups ? s + u : s;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[u][e] = maps[(su * group_items + nv[e]) * maps_item_len + (sv[e] >= 0 ? sv[e] : 0)];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (s + u >= groups) break;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float x = sv[e] >= 0 ? v[u][e] : 0.f;
          if (mode == 0) {
            a[e] = (a[e] + x) / n_total;
          } else if (mode == 1) {
            a[e] = fmaf(weights[s + u], x, a[e]);
          } else {
            x = nan_to_num(x);
            if (k0 + s + u > 0) a[e] = a[e] + (pv[e] + x) / 2.0f;
            pv[e] = x;
          }
        }
      }
    }
    if constexpr (STRIDED) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        acc[tv[e]] = a[e];
        if (prev) prev[tv[e]] = pv[e];
      }
    } else {
      *reinterpret_cast<float4*>(acc + tv[0]) = make_float4(a[0], a[1], a[2], a[3]);
      if (prev) *reinterpret_cast<float4*>(prev + tv[0]) = make_float4(pv[0], pv[1], pv[2], pv[3]);
    }
  }
}

__global__ void __launch_bounds__(256) k_accumulate_f32(int64_t groups, int64_t len, const float* __restrict__ src,
                                                        float scale, float* __restrict__ acc) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < len; e += (int64_t)gridDim.x * blockDim.x) {
    float a = acc[e];
    for (int64_t s = 0; s < groups; ++s) a = a + src[s * len + e];
    if (scale != 0.f) a = a / scale;
    acc[e] = a;
  }
}

__global__ void __launch_bounds__(256) k_trapz_f32(int64_t groups, int64_t k0, int64_t len, const float* __restrict__ src,
                                                   const float* __restrict__ weights, float* __restrict__ prev32,
                                                   float* __restrict__ acc32, double* __restrict__ prev64,
                                                   double* __restrict__ acc64) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < len; e += (int64_t)gridDim.x * blockDim.x) {
    if (acc64) {
      double a = acc64[e], pv = prev64 ? prev64[e] : 0.0;
      for (int64_t s = 0; s < groups; ++s) {
        double v = (double)src[s * len + e];
        if (weights) {
          a = fma((double)weights[s], v, a);
        } else {
          if (k0 + s > 0) a = a + (pv + v) / 2.0;
          pv = v;
        }
      }
      acc64[e] = a;
      if (prev64) prev64[e] = pv;
    } else {
      float a = acc32[e], pv = prev32 ? prev32[e] : 0.f;
      for (int64_t s = 0; s < groups; ++s) {
        float v = src[s * len + e];
        if (weights) {
          a = fmaf(weights[s], v, a);
        } else {
          if (k0 + s > 0) a = a + (pv + v) / 2.0f;
          pv = v;
        }
      }
      acc32[e] = a;
      if (prev32) prev32[e] = pv;
    }
  }
}

// ------------------------------------------------------------------------------ .scales
// cv2.resize INTER_LINEAR (upsampling): src = (dst + 0.5) * (in / out) - 0.5, clamped to the edge.
// r = (double)in / out is computed on the host once per level (the same IEEE quotient the kernel formed
// per output before). One axis: source taps i0, i1 and the weight f of output coordinate o.
struct LinAxis {
  int i0, i1;
  double f;
};
__device__ __forceinline__ LinAxis lin_axis(int o, double r, int n_in) {
  double sv = ((double)o + 0.5) * r - 0.5;
  if (sv < 0) sv = 0;
  int i0 = (int)sv;
  if (i0 > n_in - 1) i0 = n_in - 1;
  const int i1 = i0 + (i0 < n_in - 1 ? 1 : 0);
  double f = sv - i0;
  if (f > 1) f = 1;
  return {i0, i1, f};
}
__device__ __forceinline__ double bilinear(const double* __restrict__ img, int ld, const LinAxis& y, const LinAxis& x) {
  const double fy = y.f, fx = x.f;
  double v00 = img[(int64_t)y.i0 * ld + x.i0], v01 = img[(int64_t)y.i0 * ld + x.i1];
  double v10 = img[(int64_t)y.i1 * ld + x.i0], v11 = img[(int64_t)y.i1 * ld + x.i1];
  return (1 - fy) * ((1 - fx) * v00 + fx * v01) + fy * ((1 - fx) * v10 + fx * v11);
}

// per level j (finest first): the quadrant split s = size / 2^(j+1), n = size / 2^j - s and the
// resize ratios s / size, n / size; the approximation (j = levels): e = size / 2^levels
struct ReprojGeom {
  int s[WAM_MAX_LEVELS + 1], n[WAM_MAX_LEVELS + 1];
  double rs[WAM_MAX_LEVELS + 1], rn[WAM_MAX_LEVELS + 1];
};

// grid: y = output plane (item, level) -- its index split once per workgroup, x = pixels with 32-bit
// row / column arithmetic (the flat 64-bit t -> (item, level, y, x) split cost three emulated 64-bit
// divisions per output: c4 1.41 ms per call)
__global__ void __launch_bounds__(256) k_reproject(int64_t items, int size, int levels, int approx, ReprojGeom g,
                                                   const double* __restrict__ avg, double* __restrict__ out) {
  const int nl = levels + (approx ? 1 : 0);
  const unsigned plane = (unsigned)size * (unsigned)size;
  for (int64_t q = blockIdx.y; q < items * nl; q += gridDim.y) {
    const int j = (int)(q % nl);
    const double* a = avg + (q / nl) * (int64_t)plane;
    double* o = out + q * (int64_t)plane;
    for (unsigned pix = blockIdx.x * 256u + threadIdx.x; pix < plane; pix += gridDim.x * 256u) {
      const int oy = (int)(pix / (unsigned)size), ox = (int)(pix - (unsigned)oy * (unsigned)size);
      double v;
      if (j < levels) {
        const int s = g.s[j], n = g.n[j];
        // the three quadrants share two row and two column interpolations
        const LinAxis ys = lin_axis(oy, g.rs[j], s), yn = lin_axis(oy, g.rn[j], n);
        const LinAxis xs = lin_axis(ox, g.rs[j], s), xn = lin_axis(ox, g.rn[j], n);
        // horizontal = avg[:s, s:e], vertical = avg[s:e, :s], diagonal = avg[s:e, s:e]
        v = bilinear(a + s, size, ys, xn) + bilinear(a + (int64_t)s * size, size, yn, xs) +
            bilinear(a + (int64_t)s * size + s, size, yn, xn);
      } else {
        const int e = g.n[levels];
        v = bilinear(a, size, lin_axis(oy, g.rn[levels], e), lin_axis(ox, g.rn[levels], e));
      }
      o[pix] = v;
    }
  }
}


// BaseWAM2D.disentangle_scales (lib/wam_2D.py:133-198): per image and level (finest first) the
// sum (V + D) + H of the batch-max-normalised |channel mean| maps, each upsampled to size x size
// by cv2 INTER_LINEAR on float32 data (half-pixel centres, edge clamp; torch's bilinear on the
// reference's float32 arrays), stored as float64; with approx the normalised approximation of the
// LAST image only (the reference's stale loop variable, :194-197).
struct ScalesGeom {
  int J;
  int nbands;
  int64_t item;                        // floats per item of the packed maps
  int64_t off[WAM_MAX_LEVELS][3];      // H, V, D offsets of level l (0 = finest)
  int band[WAM_MAX_LEVELS][3];
  int mh[WAM_MAX_LEVELS], mw[WAM_MAX_LEVELS];
  int64_t off_a;
};

__device__ __forceinline__ float bilinear_f32(const float* __restrict__ m, float band_mx, int ih, int iw, int oy,
                                              int ox, int out) {
  float sy = ((float)ih / (float)out) * ((float)oy + 0.5f) - 0.5f;
  float sx = ((float)iw / (float)out) * ((float)ox + 0.5f) - 0.5f;
  sy = sy < 0.f ? 0.f : sy;
  sx = sx < 0.f ? 0.f : sx;
  const int y0 = (int)sy, x0 = (int)sx;
  const float ly1 = fminf(sy - (float)y0, 1.f), lx1 = fminf(sx - (float)x0, 1.f);
  const float ly0 = 1.f - ly1, lx0 = 1.f - lx1;
  const int y1 = y0 + (y0 < ih - 1 ? 1 : 0), x1 = x0 + (x0 < iw - 1 ? 1 : 0);
  // the normalised map value first (numpy's a /= a.max()), then the interpolation
  const float v00 = m[(int64_t)y0 * iw + x0] / band_mx, v01 = m[(int64_t)y0 * iw + x1] / band_mx;
  const float v10 = m[(int64_t)y1 * iw + x0] / band_mx, v11 = m[(int64_t)y1 * iw + x1] / band_mx;
  return (v00 * lx0 + v01 * lx1) * ly0 + (v10 * lx0 + v11 * lx1) * ly1;
}

__global__ void __launch_bounds__(256) k_disentangle(int64_t items, int size, int approx, ScalesGeom g,
                                                     const float* __restrict__ maps, const float* __restrict__ bmax,
                                                     double* __restrict__ out) {
  const int nl = g.J + (approx ? 1 : 0);
  const int64_t plane = (int64_t)size * size;
  const int64_t total = items * nl * plane;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t pix = t % plane;
    const int64_t q = t / plane;
    const int j = (int)(q % nl);
    const int64_t it = q / nl;
    const int oy = (int)(pix / size), ox = (int)(pix % size);
    const float* m = maps + it * g.item;
    double v;
    if (j < g.J) {
      const int ih = g.mh[j], iw = g.mw[j];
      const float h = bilinear_f32(m + g.off[j][0], bmax[g.band[j][0]], ih, iw, oy, ox, size);
      const float vv = bilinear_f32(m + g.off[j][1], bmax[g.band[j][1]], ih, iw, oy, ox, size);
      const float d = bilinear_f32(m + g.off[j][2], bmax[g.band[j][2]], ih, iw, oy, ox, size);
      v = (double)((vv + d) + h);
    } else {
      v = it == items - 1 ? (double)bilinear_f32(m + g.off_a, bmax[0], g.mh[g.J - 1], g.mw[g.J - 1], oy, ox, size)
                          : 0.0;
    }
    out[t] = v;
  }
}


// Streaming copy: the measured HBM ceiling bench.py reports beside the 8 TB/s spec peak. One 16-B
// load and store per thread over a grid covering the buffer once (no grid-stride loop): the fastest
// of the forms swept by scripts/ubench_copy.hip on MI355X (6.17 TB/s for a 2 GiB copy against
// 5.28 TB/s for the round-5 grid-stride nontemporal form with 4 loads in flight per thread,
// profiles/r06e_ubench_copy.log); buffers past 2^31 blocks take the grid-stride loop.
typedef float wam_f4 __attribute__((ext_vector_type(4)));
__global__ void __launch_bounds__(256) k_copy(int64_t n4, const wam_f4* __restrict__ src, wam_f4* __restrict__ dst) {
  const int64_t step = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n4; t += step) wam_st(dst + t, src[t]);
}

}  // namespace

extern "C" {

int wam_item_sigma(int64_t items, int64_t item_stride, int64_t len, const float* x, float spread, float* sigma,
                   void* stream) {
  if (items < 0 || len < 1 || !x || !sigma) return WAM_ERR_INVALID_ARG;
  if (items == 0) return WAM_OK;
  const bool vec4 = item_stride % 4 == 0 && len % 4 == 0 && (uintptr_t)x % 16 == 0;
  WamTimer tm((hipStream_t)stream, "k_item_sigma", 4.0 * (double)items * len);
  if (vec4)
    hipLaunchKernelGGL(k_item_sigma<true>, dim3((unsigned)items), dim3(1024), 0, (hipStream_t)stream, x, item_stride,
                       len, spread, sigma);
  else
    hipLaunchKernelGGL(k_item_sigma<false>, dim3((unsigned)items), dim3(1024), 0, (hipStream_t)stream, x, item_stride,
                       len, spread, sigma);
  WAM_LAUNCH_CHECK();
  return WAM_OK;
}

int64_t wam_item_sigma_ws_bytes(int64_t items, int64_t len) {
  if (items < 1 || len < 1) return 0;
  int64_t chunk;
  int chunks;
  sigma_split(items, len, false, chunk, chunks);
  return items * (int64_t)chunks * (int64_t)sizeof(float2) + items * (int64_t)sizeof(unsigned int) + 16;
}

int wam_item_sigma_ws(int64_t items, int64_t item_stride, int64_t len, const float* x, float spread, float* sigma,
                      void* ws, int64_t ws_bytes, void* stream) {
  if (items < 0 || len < 1 || !x || !sigma) return WAM_ERR_INVALID_ARG;
  if (items == 0) return WAM_OK;
  if (!ws || ws_bytes < wam_item_sigma_ws_bytes(items, len) || ((uintptr_t)ws & 7)) return WAM_ERR_INVALID_ARG;
  const bool vec4 = item_stride % 4 == 0 && len % 4 == 0 && (uintptr_t)x % 16 == 0;
  int64_t chunk;
  int chunks;
  sigma_split(items, len, false, chunk, chunks);  // the split the workspace was sized for
  if (vec4) {
    chunk = (chunk + 3) & ~int64_t(3);
    chunks = (int)((len + chunk - 1) / chunk);  // <= the sized count
  }
  float2* part = reinterpret_cast<float2*>(ws);
  unsigned int* cnt = reinterpret_cast<unsigned int*>(part + items * chunks);
  WamTimer tm((hipStream_t)stream, "k_item_sigma", 4.0 * (double)items * len);
  const dim3 grid((unsigned)(items * chunks));
  if (vec4)
    hipLaunchKernelGGL(k_item_sigma_split<true>, grid, dim3(kSigT), 0, (hipStream_t)stream, x, item_stride, len, chunk,
                       chunks, spread, sigma, part, cnt);
  else
    hipLaunchKernelGGL(k_item_sigma_split<false>, grid, dim3(kSigT), 0, (hipStream_t)stream, x, item_stride, len,
                       chunk, chunks, spread, sigma, part, cnt);
  WAM_LAUNCH_CHECK();
  return WAM_OK;
}

int wam_noise_add_ex(int64_t n_samples, int64_t items, int64_t item_stride, int64_t noised_len, const float* x,
                     const float* sigma, const float* host_noise, uint64_t seed, int64_t sample_base,
                     int64_t item_base, float* out, void* stream) {
  if (item_base < 0 || n_samples < 0 || items < 0 || item_stride < 1 || noised_len < 0 || noised_len > item_stride || !x || !out)
    return WAM_ERR_INVALID_ARG;
  if (!host_noise && !sigma) return WAM_ERR_INVALID_ARG;
  int64_t work = n_samples * items * ((item_stride + 3) / 4);
  if (work == 0) return WAM_OK;
  WamTimer tm((hipStream_t)stream, item_stride % 4 == 0 ? "k_noise_add<v4>" : "k_noise_add",
              4.0 * (double)items * item_stride * (1 + n_samples * (host_noise ? 2 : 1)));
  if (item_stride % 4 == 0 && ((uintptr_t)x % 16 == 0) && ((uintptr_t)out % 16 == 0) &&
      (!host_noise || (uintptr_t)host_noise % 16 == 0))
    hipLaunchKernelGGL(k_noise_add<true>, dim3(wam_grid(work, 256)), dim3(256), 0, (hipStream_t)stream, n_samples,
                       items, item_stride, noised_len, x, sigma, host_noise, (uint32_t)seed, (uint32_t)(seed >> 32),
                       sample_base, item_base, out);
  else
    hipLaunchKernelGGL(k_noise_add<false>, dim3(wam_grid(work, 256)), dim3(256), 0, (hipStream_t)stream, n_samples,
                       items, item_stride, noised_len, x, sigma, host_noise, (uint32_t)seed, (uint32_t)(seed >> 32),
                       sample_base, item_base, out);
  WAM_LAUNCH_CHECK();
  return WAM_OK;
}

int wam_noise_add(int64_t n_samples, int64_t items, int64_t item_stride, int64_t noised_len, const float* x,
                  const float* sigma, const float* host_noise, uint64_t seed, int64_t sample_base, float* out,
                  void* stream) {
  return wam_noise_add_ex(n_samples, items, item_stride, noised_len, x, sigma, host_noise, seed, sample_base, 0, out,
                          stream);
}

int wam_subband_maps(const wam_plan* p, int64_t groups, int64_t group_items, int channels, const float* coeff_grads,
                     float* maps, float* band_max, void* stream) {
  if (!p || groups < 0 || group_items < 0 || channels < 1 || !coeff_grads || !maps) return WAM_ERR_INVALID_ARG;
  int64_t items = groups * group_items;
  if (items == 0) return WAM_OK;
  if (items > 65535) return WAM_ERR_UNSUPPORTED;
  BandTable bt;
  bt.nbands = p->nbands;
  int tiles = 0;
  for (int b = 0; b <= p->nbands; ++b) {
    bt.off[b] = p->band_off[b];
    bt.tile0[b] = tiles;
    if (b < p->nbands) tiles += (int)((p->band_off[b + 1] - p->band_off[b] + kMapTile - 1) / kMapTile);
  }
  WamTimer tm((hipStream_t)stream, "k_subband_maps", 4.0 * (double)items * (channels + 1) * p->band_off[p->nbands]);
  bool vec4 = ((uintptr_t)coeff_grads & 15) == 0 && ((uintptr_t)maps & 15) == 0;
  for (int b = 0; b <= p->nbands; ++b) vec4 = vec4 && (p->band_off[b] % 4 == 0);
  if (vec4)
    hipLaunchKernelGGL(k_subband_maps<true>, dim3((unsigned)tiles, (unsigned)items), dim3(256), 0,
                       (hipStream_t)stream, bt, items, group_items, channels, coeff_grads, maps, band_max);
  else
    hipLaunchKernelGGL(k_subband_maps<false>, dim3((unsigned)tiles, (unsigned)items), dim3(256), 0,
                       (hipStream_t)stream, bt, items, group_items, channels, coeff_grads, maps, band_max);
  WAM_LAUNCH_CHECK();
  return WAM_OK;
}

int wam_frame_accumulate(int64_t groups, int64_t group_items, int64_t frame_len, const int32_t* src,
                         const int32_t* band, const float* maps, int64_t maps_item_len, const float* band_max,
                         int n_bands, int normalize, double* frame, void* stream) {
  if (groups < 0 || group_items < 0 || frame_len < 0 || !src || !band || !maps || !frame) return WAM_ERR_INVALID_ARG;
  if (normalize && !band_max) return WAM_ERR_INVALID_ARG;
  int64_t work = group_items * frame_len;
  if (work == 0 || groups == 0) return WAM_OK;
  WamTimer tm((hipStream_t)stream, "k_frame_accumulate",
              4.0 * (double)groups * group_items * frame_len + 16.0 * group_items * frame_len + 8.0 * frame_len);
  hipLaunchKernelGGL(k_frame_accumulate, dim3(wam_grid(work, 256)), dim3(256), 0, (hipStream_t)stream, groups,
                     group_items, frame_len, src, band, maps, maps_item_len, band_max, n_bands, normalize, frame);
  WAM_LAUNCH_CHECK();
  return WAM_OK;
}

int wam_frame_accumulate_coef(int64_t groups, int64_t group_items, int64_t maps_item_len, int64_t frame_len,
                              const int32_t* dst, const int32_t* cband, const float* maps, const float* band_max,
                              int n_bands, int normalize, double* frame, void* stream) {
  if (groups < 0 || group_items < 0 || maps_item_len < 0 || frame_len < 0 || !dst || !cband || !maps || !frame)
    return WAM_ERR_INVALID_ARG;
  if (normalize && !band_max) return WAM_ERR_INVALID_ARG;
  const int64_t work = group_items * maps_item_len;
  if (work == 0 || groups == 0) return WAM_OK;
  WamTimer tm((hipStream_t)stream, "k_frame_accumulate_coef",
              4.0 * (double)groups * group_items * frame_len + 16.0 * group_items * frame_len + 8.0 * frame_len);
  // mosaic tables beyond ~2 MB (8 B per coefficient; 512^2 planes) would be re-read from HBM per
  // item: about a million threads then, each a run of items of one coefficient; small tables stay
  // in L2 and every (item, coefficient) gets its own thread
  int64_t ipt = maps_item_len * 8 > (int64_t(2) << 20) ? work / (int64_t(1) << 20) : 1;
  ipt = ipt < 1 ? 1 : (ipt > group_items ? group_items : ipt);
  const int64_t threads = (group_items + ipt - 1) / ipt * maps_item_len;
  hipLaunchKernelGGL(k_frame_accumulate_coef, dim3(wam_grid(threads, 256)), dim3(256), 0, (hipStream_t)stream, groups,
                     group_items, maps_item_len, frame_len, dst, cband, maps, band_max, n_bands, normalize, ipt,
                     frame);
  WAM_LAUNCH_CHECK();
  return WAM_OK;
}

int wam_frame_trapz_coef(int64_t groups, int64_t k0, int64_t group_items, int64_t maps_item_len, int64_t frame_len,
                         const int32_t* dst, const int32_t* cband, const float* maps, const float* band_max,
                         int n_bands, int normalize, const float* weights, float* prev, float* acc, void* stream) {
  if (groups < 0 || group_items < 0 || maps_item_len < 0 || frame_len < 0 || !dst || !cband || !maps || !prev || !acc)
    return WAM_ERR_INVALID_ARG;
  if (normalize && !band_max) return WAM_ERR_INVALID_ARG;
  const int64_t work = group_items * maps_item_len;
  if (work == 0 || groups == 0) return WAM_OK;
  WamTimer tm((hipStream_t)stream, "k_frame_trapz_coef",
              4.0 * (double)groups * group_items * frame_len + 16.0 * group_items * frame_len + 8.0 * frame_len);
  // runs of items per thread when the mosaic tables outgrow L2 (as in wam_frame_accumulate_coef),
  // sized for ~4 M threads: c4 (128 images x 293 K coefficients) runs 9 items per thread --
  // PMC/algorithmic 1.058 and 929 us per 21-step launch, against 1.066 / 1,007 us at ~1 M threads
  // and 1.133 / 1,066 us at one item per thread (profiles/r05o_trapz_runs_ab.log)
  int64_t ipt = maps_item_len * 8 > (int64_t(2) << 20) ? work / (int64_t(1) << 22) : 1;
  ipt = ipt < 1 ? 1 : (ipt > group_items ? group_items : ipt);
  const int64_t threads = (group_items + ipt - 1) / ipt * maps_item_len;
  hipLaunchKernelGGL(k_frame_trapz_coef, dim3(wam_grid(threads, 256)), dim3(256), 0, (hipStream_t)stream, groups, k0,
                     group_items, maps_item_len, frame_len, dst, cband, maps, band_max, n_bands, normalize, weights,
                     ipt, prev, acc);
  WAM_LAUNCH_CHECK();
  return WAM_OK;
}

int wam_frame_trapz(int64_t groups, int64_t k0, int64_t group_items, int64_t frame_len, const int32_t* src,
                    const int32_t* band, const float* maps, int64_t maps_item_len, const float* band_max, int n_bands,
                    int normalize, const float* weights, float* prev, float* acc, void* stream) {
  if (groups < 0 || group_items < 0 || frame_len < 0 || !src || !band || !maps || !prev || !acc)
    return WAM_ERR_INVALID_ARG;
  if (normalize && !band_max) return WAM_ERR_INVALID_ARG;
  int64_t work = group_items * frame_len;
  if (work == 0 || groups == 0) return WAM_OK;
  WamTimer tm((hipStream_t)stream, "k_frame_trapz",
              4.0 * (double)groups * group_items * frame_len + 16.0 * group_items * frame_len + 8.0 * frame_len);
  hipLaunchKernelGGL(k_frame_trapz, dim3(wam_grid(work, 256)), dim3(256), 0, (hipStream_t)stream, groups, k0,
                     group_items, frame_len, src, band, maps, maps_item_len, band_max, n_bands, normalize, weights,
                     prev, acc);
  WAM_LAUNCH_CHECK();
  return WAM_OK;
}

int wam_cube_accumulate(int64_t groups, int64_t k0, int64_t group_items, int64_t cube_len, const int32_t* src,
                        const float* maps, int64_t maps_item_len, int mode, float n_total, const float* weights,
                        float* prev, float* acc, void* stream) {
  if (groups < 0 || group_items < 0 || cube_len < 0 || !src || !maps || !acc || mode < 0 || mode > 2)
    return WAM_ERR_INVALID_ARG;
  if ((mode == 1 && !weights) || (mode == 2 && !prev)) return WAM_ERR_INVALID_ARG;
  int64_t work = group_items * cube_len;
  if (work == 0 || groups == 0) return WAM_OK;
  // algorithmic bytes: the gathered maps once per (sample, voxel), the accumulator (and trapezoid
  // state) read and written, the index map once
  WamTimer tm((hipStream_t)stream, "k_cube_accumulate",
              4.0 * (double)groups * work + (mode == 2 ? 16.0 : 8.0) * work + 4.0 * cube_len);
  const bool vec4 = cube_len % 4 == 0 && ((uintptr_t)src & 15) == 0 && ((uintptr_t)acc & 15) == 0 &&
                    ((uintptr_t)prev & 15) == 0;
  // strided (256-voxel wave blocks, work % 256 == 0): c5 154 -> 109 us per launch against the four
  // consecutive voxels per thread (profiles/r06zb_ab_cube_accumulate.log)
  if (vec4 && work % 256 == 0)
    hipLaunchKernelGGL(k_cube_accumulate4<true>, dim3(wam_grid(work / 4, 256)), dim3(256), 0, (hipStream_t)stream, groups,
                       k0, group_items, cube_len, src, maps, maps_item_len, mode, n_total, weights, prev, acc);
  else if (vec4)
    hipLaunchKernelGGL(k_cube_accumulate4<false>, dim3(wam_grid(work / 4, 256)), dim3(256), 0, (hipStream_t)stream,
                       groups, k0, group_items, cube_len, src, maps, maps_item_len, mode, n_total, weights, prev, acc);
  else
    hipLaunchKernelGGL(k_cube_accumulate, dim3(wam_grid(work, 256)), dim3(256), 0, (hipStream_t)stream, groups, k0,
                       group_items, cube_len, src, maps, maps_item_len, mode, n_total, weights, prev, acc);
  WAM_LAUNCH_CHECK();
  return WAM_OK;
}

int wam_accumulate_f32(int64_t groups, int64_t len, const float* src, float scale, float* acc, void* stream) {
  if (groups < 0 || len < 0 || !src || !acc) return WAM_ERR_INVALID_ARG;
  if (len == 0) return WAM_OK;
  WamTimer tm((hipStream_t)stream, "k_accumulate_f32", 4.0 * (double)groups * len + 8.0 * (double)len);
  hipLaunchKernelGGL(k_accumulate_f32, dim3(wam_grid(len, 256)), dim3(256), 0, (hipStream_t)stream, groups, len, src,
                     scale, acc);
  WAM_LAUNCH_CHECK();
  return WAM_OK;
}

int wam_trapz_f32(int64_t groups, int64_t k0, int64_t len, const float* src, const float* weights, float* prev_f32,
                  float* acc_f32, double* prev_f64, double* acc_f64, void* stream) {
  if (groups < 0 || len < 0 || !src) return WAM_ERR_INVALID_ARG;
  if (!acc_f64 && !acc_f32) return WAM_ERR_INVALID_ARG;
  if (!weights && !(acc_f64 ? (void*)prev_f64 : (void*)prev_f32)) return WAM_ERR_INVALID_ARG;
  if (len == 0 || groups == 0) return WAM_OK;
  WamTimer tm((hipStream_t)stream, "k_trapz_f32",
              4.0 * (double)groups * len + (acc_f64 ? 16.0 : 8.0) * (double)len * (weights ? 1.0 : 2.0));
  hipLaunchKernelGGL(k_trapz_f32, dim3(wam_grid(len, 256)), dim3(256), 0, (hipStream_t)stream, groups, k0, len, src,
                     weights, prev_f32, acc_f32, prev_f64, acc_f64);
  WAM_LAUNCH_CHECK();
  return WAM_OK;
}

int wam_reproject_scales(int64_t items, int size, int levels, int approx, const double* avg, double* out,
                         void* stream) {
  if (items < 0 || size < 1 || levels < 1 || !avg || !out) return WAM_ERR_INVALID_ARG;
  if (levels > WAM_MAX_LEVELS) return WAM_ERR_UNSUPPORTED;
  int64_t work = items * (levels + (approx ? 1 : 0)) * (int64_t)size * size;
  if (work == 0) return WAM_OK;
  ReprojGeom g{};
  for (int j = 0; j < levels; ++j) {  // the reference's int(size / 2**j) splits (lib/wam_2D.py:488-536)
    const int e = (int)(size / (double)(1 << j)), s = (int)(size / (double)(1 << (j + 1)));
    g.s[j] = s;
    g.n[j] = e - s;
    g.rs[j] = (double)s / size;
    g.rn[j] = (double)(e - s) / size;
  }
  g.n[levels] = (int)(size / (double)(1 << levels));
  g.rn[levels] = (double)g.n[levels] / size;
  // algorithmic bytes: every output written once, the averaged map read once
  WamTimer tm((hipStream_t)stream, "k_reproject", 8.0 * (double)work + 8.0 * (double)items * size * size);
  if ((int64_t)size * size >= (int64_t(1) << 32)) return WAM_ERR_UNSUPPORTED;  // 32-bit pixel index
  const int64_t planes = items * (levels + (approx ? 1 : 0));
  const dim3 grid(wam_grid((int64_t)size * size, 256, 4096), (unsigned)(planes < 65535 ? planes : 65535));
  hipLaunchKernelGGL(k_reproject, grid, dim3(256), 0, (hipStream_t)stream, items, size, levels, approx, g, avg, out);
  WAM_LAUNCH_CHECK();
  return WAM_OK;
}

int wam_disentangle_scales(const wam_plan* plan, int64_t items, const float* maps, const float* band_max, int approx,
                           int size, double* out, void* stream) {
  if (!plan || plan->ndim != 2 || items < 0 || size < 1 || !maps || !band_max || !out) return WAM_ERR_INVALID_ARG;
  ScalesGeom g{};
  g.J = plan->levels;
  g.nbands = plan->nbands;
  g.item = plan->band_off[plan->nbands];
  for (int l = 0; l < plan->levels; ++l) {
    g.mh[l] = (int)plan->lout[l][0];
    g.mw[l] = (int)plan->lout[l][1];
    for (int k = 0; k < 3; ++k) {
      g.band[l][k] = wam_band_of(plan, l, k);
      g.off[l][k] = plan->band_off[g.band[l][k]];
    }
  }
  g.off_a = plan->band_off[0];
  const int64_t work = items * (plan->levels + (approx ? 1 : 0)) * (int64_t)size * size;
  if (work == 0) return WAM_OK;
  WamTimer tm((hipStream_t)stream, "k_disentangle", 4.0 * items * g.item + 8.0 * work);
  hipLaunchKernelGGL(k_disentangle, dim3(wam_grid(work, 256)), dim3(256), 0, (hipStream_t)stream, items, size, approx,
                     g, maps, band_max, out);
  WAM_LAUNCH_CHECK();
  return WAM_OK;
}

int wam_copy(int64_t bytes, const void* src, void* dst, void* stream) {
  if (bytes < 0 || (bytes & 15) || !src || !dst || ((uintptr_t)src & 15) || ((uintptr_t)dst & 15))
    return WAM_ERR_INVALID_ARG;
  const int64_t n4 = bytes / 16;
  if (n4 == 0) return WAM_OK;
  WamTimer tm((hipStream_t)stream, "k_copy", 2.0 * bytes);
  hipLaunchKernelGGL(k_copy, dim3(wam_grid(n4, 256, int64_t(1) << 31)), dim3(256), 0, (hipStream_t)stream, n4,
                     (const wam_f4*)src, (wam_f4*)dst);
  WAM_LAUNCH_CHECK();
  return WAM_OK;
}

}  // extern "C"

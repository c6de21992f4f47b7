// Fused multi-level 1D transforms for gfx950 (config c3: db6 J=5 on 80,000-sample clips).
//
// The per-axis kernels make one HBM round trip per level; here one 256-thread workgroup owns a
// TILE of one signal and runs all J levels in LDS:
//   analysis  (wavedec / adjoint of waverec): the tile is a range of coarsest-level outputs; every
//             finer level computes its own share of outputs plus the halo the next level needs
//             (recomputed, never exchanged), starting from one window of the source signal loaded
//             with coalesced loads and the boundary extension applied on the load. Details of each
//             level's own range go to HBM; the approximation ladder stays in LDS.
//   synthesis (waverec, IG alpha fused on the load): the tile is a range of output samples; the
//             coefficient ranges every level needs (own share + filter support) are staged in LDS
//             and reconstructed coarse to fine; only the finest level writes to HBM.
// Tiles cover ~4096 source samples, so the recomputed halo ((L-2)(2^J - 1) samples) costs a few
// percent. Boundary modes: zero, reflect, symmetric, constant (periodic extensions are not local
// and stay on the per-axis kernels).
#include <algorithm>
#include <mutex>
#include <set>
#include <type_traits>

#include "kernels.hpp"
#include "rng.hpp"

namespace {

typedef float f2v __attribute__((ext_vector_type(2)));  // packed fp32 (v_pk_fma_f32)

// opt in to more than 64 KB of dynamic LDS, once per (kernel, device)
int lds_opt_in(const void* kern, int bytes) {
  static std::mutex mu;
  static std::set<std::pair<const void*, int>> done;
  if (bytes <= 64 * 1024) return WAM_OK;
  int dev = 0;
  WAM_HIP_CHECK(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(mu);
  if (done.count({kern, dev})) return WAM_OK;
  WAM_HIP_CHECK(hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
  done.insert({kern, dev});
  return WAM_OK;
}

constexpr int kT1 = 512;          // threads per workgroup (analysis)
constexpr int kT1S = 256;         // threads per workgroup (synthesis)
constexpr int kTile0 = 4096;      // synthesis: half the level-0 outputs of a tile
constexpr int kTileA = 4096;      // analysis: finest-level outputs per tile (source window ~2 x this)
constexpr int kAnaWgs = 2;        // analysis: persistent workgroups per CU
constexpr int kLds1Cap = 80 * 1024;  // two workgroups per CU

struct Dwt1Geom {
  int J;
  int mode;
  int n;                            // input length (level-0 input)
  int m[WAM_MAX_LEVELS];            // output length of level l (0 = finest)
  int64_t off_d[WAM_MAX_LEVELS];    // per-item offset of D of level l
  int64_t off_a;                    // per-item offset of A_J
  int64_t items;                    // items in the band-major coefficient buffer
  int tile_j;                       // coarsest-level outputs per tile (analysis)
  int tiles;                        // tiles per signal
  int syn_cap;                      // floats per LDS buffer of the synthesis
};

__host__ __device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// boundary extension for indices at most one signal length outside [0, n) (the tile halos);
// farther indices (tiny coarse levels) take the general rule
__host__ __device__ __forceinline__ int ext_near(int i, int n, int mode) {
  if (i >= 0 && i < n) return i;
  int r;
  switch (mode) {
    case WAM_MODE_ZERO: return -1;
    case WAM_MODE_CONSTANT: return i < 0 ? 0 : n - 1;
    case WAM_MODE_REFLECT: r = i < 0 ? -i : 2 * n - 2 - i; break;
    default: r = i < 0 ? -i - 1 : 2 * n - 1 - i; break;  // symmetric
  }
  return (r >= 0 && r < n) ? r : wam_ext_index(i, n, mode);
}

// SmoothGrad noise of source sample si of one signal (the wam_noise_add stream: one Philox call per
// group of 4 samples; here a call per sample -- the boundary tiles only)
__device__ __forceinline__ float noise_at(int64_t si, uint32_t img, uint32_t smp, uint32_t k0, uint32_t k1) {
  float z[4];
  wam_normal4(si >> 2, img, smp, k0, k1, z);
  const int q = (int)(si & 3);
  return q == 0 ? z[0] : q == 1 ? z[1] : q == 2 ? z[2] : z[3];
}

// NOISE: output item `item` (sample-major: s * images + i) is signal i noised for sample s
struct NoiseItem {
  int64_t src;   // clean signal index
  uint32_t img, smp;
  float sg;
};
__device__ __forceinline__ NoiseItem noise_item(const WamNoise& nz, int64_t item) {
  const int64_t s = item / nz.images, i = item - s * nz.images;
  return {i, (uint32_t)(nz.image_base + i), (uint32_t)(nz.sample_base + s), nz.sigma[i]};
}

// ranges (uniform): own [s, e) and computed [S, E) of every level for tile `tile`
__host__ __device__ __forceinline__ void ana_ranges(const Dwt1Geom& g, int tile, int p, int* S, int* E, int* s,
                                                    int* e) {
  const int J = g.J;
  for (int l = J - 1; l >= 0; --l) {
    const int T = g.tile_j << (J - 1 - l);
    const int m = g.m[l];
    s[l] = tile * T < m ? tile * T : m;
    e[l] = (tile + 1) * T < m ? (tile + 1) * T : m;
    int lo = 0x7fffffff, hi = -1;
    if (s[l] < e[l]) {
      lo = s[l];
      hi = e[l];
    }
    if (l < J - 1 && S[l + 1] < E[l + 1]) {
      // taps of level l+1 outputs [S, E): extended indices [a, b] = [2S - p, 2E - 1] of level l
      const int a = 2 * S[l + 1] - p, b = 2 * E[l + 1] - 1;
      int nlo = a > 0 ? a : 0, nhi = b < m - 1 ? b : m - 1;
      if (a < 0) nhi = std::max(nhi, std::min(-a, m - 1));                // single mirror / replicate at 0
      if (b > m - 1) nlo = std::min(nlo, std::max(0, 2 * (m - 1) - b - 1));  // ... and at m - 1
      if (a < -(m - 1) || b > 2 * (m - 1)) {                    // several reflections: everything
        nlo = 0;
        nhi = m - 1;
      }
      if (nlo <= nhi) {
        lo = std::min(lo, nlo);
        hi = std::max(hi, nhi + 1);
      }
    }
    S[l] = lo <= hi ? lo : 0;
    E[l] = lo <= hi ? hi : 0;
  }
}

// the J levels of one tile from its source window in smem[0, wlen) (extension applied on the
// load): level 0 from the window, levels 1..J-1 from two approximation buffers after it
template <int L>
__device__ __forceinline__ void ana_tile_levels(float* smem, const float* flo, const float* fhi, const Dwt1Geom& g,
                                                float* __restrict__ coeffs, int64_t item, const int* S,
                                                const int* E, const int* s, const int* e) {
  constexpr int p = L - 2;
  const int tid = threadIdx.x;
  const int J = g.J, mode = g.mode;
  const int wlen = 2 * (E[0] - S[0]) + L - 2;
  const int off_ll0 = (wlen + 63) & ~63;
  const int off_ll1 = off_ll0 + ((E[0] - S[0] + 63) & ~63);
  {
    const int ml = g.m[0];
    const bool last = J == 1;
    float* dout = coeffs + g.items * g.off_d[0] + item * (int64_t)ml;
    float* aout = coeffs + g.items * g.off_a + item * (int64_t)ml;
    const int s0 = s[0], e0 = e[0], S0 = S[0], E0 = E[0];
    for (int i = S0 + tid; i < E0; i += kT1) {
      const int w = 2 * (i - S0);
      float a = 0.f, d = 0.f;
#pragma unroll
      for (int k = 0; k < L; ++k) {
        const float v = smem[w + k];
        a = fmaf(flo[k], v, a);
        d = fmaf(fhi[k], v, d);
      }
      if (i >= s0 && i < e0) {
        dout[i] = d;
        if (last) aout[i] = a;
      }
      if (!last) smem[off_ll0 + i - S0] = a;
    }
    __syncthreads();
  }
  // levels 1..J-1 from the approximation buffers (ping-pong by level parity)
  for (int l = 1; l < J; ++l) {
    const int ml = g.m[l], nin = g.m[l - 1];
    const int in_off = (l & 1) ? off_ll0 : off_ll1, out_off = (l & 1) ? off_ll1 : off_ll0;
    const int base = S[l - 1];
    const bool last = l == J - 1;
    float* dout = coeffs + g.items * g.off_d[l] + item * (int64_t)ml;
    float* aout = coeffs + g.items * g.off_a + item * (int64_t)ml;
    const int sl = s[l], el = e[l], Sl = S[l], El = E[l];
    for (int i = Sl + tid; i < El; i += kT1) {
      const int t0 = 2 * i - p;
      float a = 0.f, d = 0.f;
      if (t0 >= 0 && t0 + L - 1 < nin) {
        const int w = in_off + t0 - base;
#pragma unroll
        for (int k = 0; k < L; ++k) {
          const float v = smem[w + k];
          a = fmaf(flo[k], v, a);
          d = fmaf(fhi[k], v, d);
        }
      } else {
#pragma unroll
        for (int k = 0; k < L; ++k) {
          const int mi = ext_near(t0 + k, nin, mode);
          const float v = mi >= 0 ? smem[in_off + mi - base] : 0.f;
          a = fmaf(flo[k], v, a);
          d = fmaf(fhi[k], v, d);
        }
      }
      if (i >= sl && i < el) {
        dout[i] = d;
        if (last) aout[i] = a;
      }
      if (!last) smem[out_off + i - Sl] = a;
    }
    __syncthreads();
  }
}

// tiles [t_lo, t_hi) are left to k_dwt1_ana_int; this kernel runs the others (nb per signal)
template <int L, bool NOISE>
__global__ void __launch_bounds__(kT1) k_dwt1_ana(const float* __restrict__ in, float* __restrict__ coeffs,
                                                 const float* __restrict__ filt, Dwt1Geom g, int t_lo, int t_hi,
                                                 WamNoise nz) {
  constexpr int p = L - 2;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x;
  const int nb = g.tiles - (t_hi - t_lo);
  const int64_t item = blockIdx.x / nb;
  const int kb = (int)(blockIdx.x % nb);
  const int tile = kb < t_lo ? kb : t_hi + (kb - t_lo);
  float flo[L], fhi[L];
#pragma unroll
  for (int k = 0; k < L; ++k) {
    flo[k] = filt[k];
    fhi[k] = filt[L + k];
  }
  __shared__ int S[WAM_MAX_LEVELS], E[WAM_MAX_LEVELS], s[WAM_MAX_LEVELS], e[WAM_MAX_LEVELS];
  if (tid == 0) ana_ranges(g, tile, p, S, E, s, e);
  __syncthreads();
  // window = extended indices [2 S0 - p, 2 E0 - 1) of the input
  const int w0 = 2 * S[0] - p;
  const int wlen = 2 * (E[0] - S[0]) + L - 2;
  NoiseItem ni{item, 0, 0, 0.f};
  if constexpr (NOISE) ni = noise_item(nz, item);
  const float* x = in + ni.src * (int64_t)g.n;
  for (int j = tid; j < wlen; j += kT1) {
    const int si = ext_near(w0 + j, g.n, g.mode);
    float v = si >= 0 ? x[si] : 0.f;
    if constexpr (NOISE)
      if (si >= 0) v = fmaf(ni.sg, noise_at(si, ni.img, ni.smp, nz.k0, nz.k1), v);  // wam_noise_add's rounding
    smem[j] = v;
  }
  __syncthreads();
  ana_tile_levels<L>(smem, flo, fhi, g, coeffs, item, S, E, s, e);
}

// the same boundary tiles, persistent: workgroups loop over (signal, boundary tile) units and fetch
// the next unit's window (extension applied) into registers while the current unit's levels run;
// used when every boundary window fits kPF floats per thread
constexpr int kPF = 20;  // window floats prefetched per thread (window <= kPF * kT1)

template <int L, bool NOISE>
__global__ void __launch_bounds__(kT1) k_dwt1_ana_p(const float* __restrict__ in, float* __restrict__ coeffs,
                                                   const float* __restrict__ filt, Dwt1Geom g, int t_lo, int t_hi,
                                                   int64_t units, WamNoise nz) {
  constexpr int p = L - 2;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x;
  const int nb = g.tiles - (t_hi - t_lo);
  float flo[L], fhi[L];
#pragma unroll
  for (int k = 0; k < L; ++k) {
    flo[k] = filt[k];
    fhi[k] = filt[L + k];
  }
  __shared__ int R[2][4][WAM_MAX_LEVELS];  // (S, E, s, e) of the current and the next unit
  auto ranges = [&](int64_t u, int slot) {
    const int kb = (int)(u % nb);
    ana_ranges(g, kb < t_lo ? kb : t_hi + (kb - t_lo), p, R[slot][0], R[slot][1], R[slot][2], R[slot][3]);
  };
  // NOISE: a thread takes runs of 4 consecutive window samples whose first source index is a
  // multiple of 4 (window offset shifted by w0 mod 4), so one Philox call (the group of wam_noise_add's
  // stream) serves the whole run away from the extension's turning points
  constexpr int kNG = kPF / 4 + 1;
  constexpr int kPFN = NOISE ? 4 * kNG : kPF;
  float pf[kPFN];
  uint32_t zmask = 0;  // window slots that are zeros (zero-mode extension, or outside the window):
                       // applied when stored, so the loads stay unconditional and all in flight together
  auto slot_j = [&](int r, int a) { return NOISE ? 4 * (tid + (r >> 2) * kT1) - a + (r & 3) : tid + r * kT1; };
  auto prefetch = [&](int64_t u, int slot) {
    const int64_t item = NOISE ? noise_item(nz, u / nb).src : u / nb;
    const int w0 = 2 * R[slot][0][0] - p;
    const int wlen = 2 * (R[slot][1][0] - R[slot][0][0]) + L - 2;
    const float* x = in + item * (int64_t)g.n;
    zmask = 0;
#pragma unroll
    for (int r = 0; r < kPFN; ++r) {
      const int j = slot_j(r, w0 & 3);
      const int si = (j >= 0 && j < wlen) ? ext_near(w0 + j, g.n, g.mode) : -1;
      zmask |= (si < 0 ? 1u : 0u) << r;
      pf[r] = x[si >= 0 ? si : 0];
    }
  };
  int64_t u = blockIdx.x;
  int cur = 0;
  if (u < units) {
    if (tid == 0) ranges(u, 0);
    __syncthreads();
    prefetch(u, 0);
  }
  for (; u < units; u += gridDim.x) {
    const int wlen = 2 * (R[cur][1][0] - R[cur][0][0]) + L - 2;
    if constexpr (NOISE) {
      const NoiseItem ni = noise_item(nz, u / nb);
      const int w0 = 2 * R[cur][0][0] - p;
#pragma unroll
      for (int q = 0; q < kNG; ++q) {
        const int jb = slot_j(4 * q, w0 & 3);
        if (jb >= wlen) continue;
        int si[4];
        int sf = -1, sl = -1;  // first / last source index of the run
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          si[k] = (zmask >> (4 * q + k)) & 1u ? -1 : ext_near(w0 + jb + k, g.n, g.mode);
          if (si[k] >= 0) {
            sf = sf < 0 ? si[k] : sf;
            sl = si[k];
          }
        }
        float za[4] = {0.f, 0.f, 0.f, 0.f}, zb[4] = {0.f, 0.f, 0.f, 0.f};
        if (sf >= 0) wam_normal4(sf >> 2, ni.img, ni.smp, nz.k0, nz.k1, za);
        if (sl >= 0 && (sl >> 2) != (sf >> 2)) wam_normal4(sl >> 2, ni.img, ni.smp, nz.k0, nz.k1, zb);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int j = jb + k;
          if (j < 0 || j >= wlen) continue;
          float v = 0.f;
          if (si[k] >= 0) {
            const int c = si[k] & 3;
            float z;
            if ((si[k] >> 2) == (sf >> 2))
              z = c == 0 ? za[0] : c == 1 ? za[1] : c == 2 ? za[2] : za[3];
            else if ((si[k] >> 2) == (sl >> 2))
              z = c == 0 ? zb[0] : c == 1 ? zb[1] : c == 2 ? zb[2] : zb[3];
            else  // a third group (a turning point inside the run)
              z = noise_at(si[k], ni.img, ni.smp, nz.k0, nz.k1);
            v = fmaf(ni.sg, z, pf[4 * q + k]);  // wam_noise_add's rounding
          }
          smem[j] = v;
        }
      }
    } else {
#pragma unroll
      for (int r = 0; r < kPF; ++r) {
        const int j = tid + r * kT1;
        if (j < wlen) smem[j] = (zmask >> r) & 1u ? 0.f : pf[r];
      }
    }
    const int64_t un = u + gridDim.x;
    if (tid == 0 && un < units) ranges(un, cur ^ 1);
    __syncthreads();
    if (un < units) prefetch(un, cur ^ 1);  // in flight while the levels run
    ana_tile_levels<L>(smem, flo, fhi, g, coeffs, u / nb, R[cur][0], R[cur][1], R[cur][2], R[cur][3]);
    cur ^= 1;
  }
}

// ------------------------------------------------------------------------------------------------
// Interior tiles (no boundary extension at any level): persistent workgroups over (signal, tile)
// units. Ranges are closed-form: coarsest computed range [S, E) = [t tj, (t + 1) tj), finer levels
// S_l = 2 S_(l+1) - p, E_l = 2 E_(l+1). The source window and every approximation level live in
// LDS de-interleaved (even / odd samples in separate arrays, the odd array offset by 16 banks), so
// output r reads E[r + m], O[r + m]: consecutive lanes hit consecutive banks and the taps keep the
// k = 0..L-1 fma order of the per-axis kernels (same sums). The next unit's window is fetched into
// registers before the current unit's levels run, hiding its HBM latency.

__host__ __device__ __forceinline__ int eo_cap(int n) { return (((n + 1) / 2 + 31) & ~31) + 16; }

// NOISE: the window is fetched as aligned groups of 4 samples (float4; the signal length is a
// multiple of 4, host check), each noised with ONE Philox call of wam_noise_add's stream (two
// groups per interleaved call pair); units run sample-fastest over XCD-swizzled workgroups, so
// the S samples of a (signal, tile) read its window from one L2.
constexpr int kPG = 6;  // noisy window: float4 groups per thread (window <= (kPG * kT1 - 1) * 4)

// fold != 0: the units cover ALL tiles; the boundary tiles (outside [t_lo, t_hi)) take the same
// closed-form ranges and fix the extension up where the signal ends: window slots whose source
// index falls outside [0, n) are loaded through the boundary rule (noise keyed by the source
// sample, as wam_noise_add noises the signal before it is extended), and after each level the
// computed entries outside [0, m_l) are replaced by their extension (mirrors of computed entries,
// host-checked) before the next level reads them; only own outputs inside [0, m_l) are stored.
template <int L, bool NOISE>
__global__ void __launch_bounds__(kT1) k_dwt1_ana_int(const float* __restrict__ in, float* __restrict__ coeffs,
                                                     const float* __restrict__ filt, Dwt1Geom g, int t_lo, int t_hi,
                                                     int64_t units, WamNoise nz, int64_t S, int fold) {
  constexpr int p = L - 2;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x;
  float flo[L], fhi[L];
#pragma unroll
  for (int k = 0; k < L; ++k) {
    flo[k] = filt[k];
    fhi[k] = filt[L + k];
  }
  const int J = g.J;
  const int tbase = fold ? 0 : t_lo;
  const int nti = fold ? g.tiles : t_hi - t_lo;
  const int tj = g.tile_j;
  const int n0 = (tj << (J - 1)) + p * ((1 << (J - 1)) - 1);  // level-0 computed outputs per tile
  const int wlen = 2 * n0 + p;
  const int cw = eo_cap(wlen);            // window: E at [0, cw), O at [cw, 2 cw)
  const int c0 = eo_cap(n0);              // level buffers (ping-pong): A at 2 cw, B after it
  float* winE = smem;
  float* winO = smem + cw;
  const int c1 = eo_cap((n0 - p) >> 1);
  float* bufA = smem + 2 * cw;            // even levels' outputs (level 0: n0 values)
  float* bufB = smem;                     // odd levels' outputs, in the window's space (dead after level 0)
  // unit -> output item and tile; NOISE: sample fastest, src = the clean signal
  auto unit_geom = [&](int64_t u, int64_t& item, int64_t& src, int& tile, int& S0) {
    if constexpr (NOISE) {
      const int64_t s = u % S, rest = u / S, i = rest / nti;
      tile = tbase + (int)(rest - i * nti);
      src = i;
      item = s * nz.images + i;
    } else {
      item = src = u / nti;
      tile = tbase + (int)(u - item * nti);
    }
    S0 = ((tile * tj) << (J - 1)) - p * ((1 << (J - 1)) - 1);
  };
  constexpr int NPF = NOISE ? 4 * kPG : kPF;
  float pf[NPF];
  auto prefetch = [&](int64_t u) {
    int64_t item, src;
    int tile, S0;
    unit_geom(u < units ? u : units - 1, item, src, tile, S0);
    if constexpr (NOISE) {
      // aligned groups [ga, gb) covering the window [w0, w0 + wlen); clamped to the last one
      const int w0 = 2 * S0 - p, ga = w0 >> 2, gb = (w0 + wlen + 3) >> 2;
      const float4* x4 = reinterpret_cast<const float4*>(in + src * (int64_t)g.n);
      const int g_last = (g.n >> 2) - 1;  // boundary tiles: groups past the signal are clamped
#pragma unroll
      for (int r = 0; r < kPG; ++r) {
        const int gi = ga + tid + r * kT1;
        const float4 t = x4[min(max(gi < gb ? gi : gb - 1, 0), g_last)];
        pf[4 * r] = t.x;
        pf[4 * r + 1] = t.y;
        pf[4 * r + 2] = t.z;
        pf[4 * r + 3] = t.w;
      }
    } else {
      const float* x = in + src * (int64_t)g.n;
      const int w0 = 2 * S0 - p;
#pragma unroll
      for (int r = 0; r < kPF; ++r) {
        const int j = tid + r * kT1;
        pf[r] = x[min(max(w0 + (j < wlen ? j : wlen - 1), 0), g.n - 1)];
      }
    }
  };
  int64_t u = NOISE ? wam_xcd_block(blockIdx.x, gridDim.x) : blockIdx.x;
  if (u < units) prefetch(u);
  for (; u < units; u += gridDim.x) {
    int64_t item, src;
    int tile, S0;
    unit_geom(u, item, src, tile, S0);
    const int w0 = 2 * S0 - p;
    const bool bnd = tile < t_lo || tile >= t_hi;  // (fold) a boundary tile: workgroup-uniform
    if constexpr (NOISE) {
      const NoiseItem ni = noise_item(nz, item);
      const int ga = w0 >> 2, gb = (w0 + wlen + 3) >> 2;
      // a group inside both the window and the signal lands whole: w0 is even (L is), so its
      // samples k = 0, 2 go to E[h], E[h + 1] and k = 1, 3 to O[h], O[h + 1] (h = (4 gi - w0) / 2);
      // the groups at the window's ends and past the signal take the per-sample checks
      auto commit = [&](int gi, const float* z, const float* x4) {
        const int j0 = 4 * gi - w0;
        if (gi >= 0 && j0 >= 0 && j0 + 4 <= wlen && 4 * gi + 4 <= g.n) {
          const int h = j0 >> 1;
          winE[h] = fmaf(ni.sg, z[0], x4[0]);  // wam_noise_add's rounding
          winO[h] = fmaf(ni.sg, z[1], x4[1]);
          winE[h + 1] = fmaf(ni.sg, z[2], x4[2]);
          winO[h + 1] = fmaf(ni.sg, z[3], x4[3]);
        } else {
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int j = j0 + k;
            // samples outside the signal (boundary tiles) come from the extension pass below
            if (gi < gb && j >= 0 && j < wlen && (unsigned)(4 * gi + k) < (unsigned)g.n)
              ((j & 1) ? winO : winE)[j >> 1] = fmaf(ni.sg, z[k], x4[k]);
          }
        }
      };
#pragma unroll
      for (int r = 0; r < kPG; r += 2) {
        const int gi0 = ga + tid + r * kT1, gi1 = gi0 + kT1;
        if (gi0 >= gb) continue;  // whole waves past the window skip the pair's Philox blocks
        float za[4], zb[4];
        wam_normal4_x2((uint32_t)gi0, (uint32_t)gi1, ni.img, ni.smp, nz.k0, nz.k1, za, zb);
        commit(gi0, za, pf + 4 * r);
        if (gi1 < gb) commit(gi1, zb, pf + 4 * (r + 1));
      }
      if (bnd) {
        const float* x = in + src * (int64_t)g.n;
        for (int j = tid; j < wlen; j += kT1) {
          const int gidx = w0 + j;
          if ((unsigned)gidx < (unsigned)g.n) continue;
          const int si = ext_near(gidx, g.n, g.mode);
          const float v = si >= 0 ? fmaf(ni.sg, noise_at(si, ni.img, ni.smp, nz.k0, nz.k1), x[si]) : 0.f;
          ((j & 1) ? winO : winE)[j >> 1] = v;
        }
      }
    } else {
#pragma unroll
      for (int r = 0; r < kPF; ++r) {
        const int j = tid + r * kT1;
        if (j < wlen && (unsigned)(w0 + j) < (unsigned)g.n) ((j & 1) ? winO : winE)[j >> 1] = pf[r];
      }
      if (bnd) {
        const float* x = in + src * (int64_t)g.n;
        for (int j = tid; j < wlen; j += kT1) {
          const int gidx = w0 + j;
          if ((unsigned)gidx < (unsigned)g.n) continue;
          const int si = ext_near(gidx, g.n, g.mode);
          ((j & 1) ? winO : winE)[j >> 1] = si >= 0 ? x[si] : 0.f;
        }
      }
    }
    __syncthreads();
    prefetch(u + gridDim.x);  // in flight while the levels run
    // level l: inputs (E, O) of length nin, outputs r in [0, nl), absolute index S_l + r
    const float* iE = winE;
    const float* iO = winO;
    int Sl = S0, nl = n0;
    for (int l = 0; l < J; ++l) {
      const bool last = l == J - 1;
      float* oE = (l & 1) ? bufB : bufA;
      float* oO = oE + ((l & 1) ? c1 : c0);
      const int ml = g.m[l];
      const int T = tj << (J - 1 - l);                       // own outputs per tile at this level
      const int own0 = tile * T;
      float* dout = coeffs + g.items * g.off_d[l] + item * (int64_t)ml;
      float* aout = coeffs + g.items * g.off_a + item * (int64_t)ml;
      // output pair (r, r + 1), r even: E/O[r .. r + H2] read once as float2, both outputs'
      // lo / hi sums as packed fp32 fma (per-output tap order unchanged)
      constexpr int H2 = L / 2, NP = H2 / 2 + 1;
      const bool dpair = ((reinterpret_cast<uintptr_t>(dout + Sl) | reinterpret_cast<uintptr_t>(aout + Sl)) & 7) == 0;
      // own outputs: i in [own0, oend) (the tile's range, the level's length and the computed range)
      const int oend = min(min(own0 + T, ml), Sl + nl);
      const unsigned ospan = (unsigned)max(oend - own0, 0);
      for (int r = 2 * tid; r < nl; r += 2 * kT1) {
        float e[2 * NP], o[2 * NP];
#pragma unroll
        for (int k = 0; k < NP; ++k) {
          const float2 te = *reinterpret_cast<const float2*>(iE + r + 2 * k);
          const float2 to = *reinterpret_cast<const float2*>(iO + r + 2 * k);
          e[2 * k] = te.x;
          e[2 * k + 1] = te.y;
          o[2 * k] = to.x;
          o[2 * k + 1] = to.y;
        }
        // packed as (lo, hi) tap pairs times a broadcast sample: each operand is one element of a
        // loaded pair (op_sel), no register moves to build straddling (E[r + m], E[r + m + 1]) pairs
        f2v P0 = {0.f, 0.f}, P1 = {0.f, 0.f};  // (a, d) of outputs r and r + 1
#pragma unroll
        for (int m2 = 0; m2 < H2; ++m2) {
          const f2v k0 = {flo[2 * m2], fhi[2 * m2]}, k1 = {flo[2 * m2 + 1], fhi[2 * m2 + 1]};
          P0 = __builtin_elementwise_fma(k0, (f2v)e[m2], P0);
          P1 = __builtin_elementwise_fma(k0, (f2v)e[m2 + 1], P1);
          P0 = __builtin_elementwise_fma(k1, (f2v)o[m2], P0);
          P1 = __builtin_elementwise_fma(k1, (f2v)o[m2 + 1], P1);
        }
        const f2v A = {P0.x, P1.x}, D = {P0.y, P1.y};
        const int i = Sl + r;
        const bool own_a = (unsigned)(i - own0) < ospan;
        const bool own_b = (unsigned)(i + 1 - own0) < ospan;
        if (own_a && own_b && dpair) {
          *reinterpret_cast<float2*>(dout + i) = make_float2(D.x, D.y);
          if (last) *reinterpret_cast<float2*>(aout + i) = make_float2(A.x, A.y);
        } else {
          if (own_a) {
            dout[i] = D.x;
            if (last) aout[i] = A.x;
          }
          if (own_b) {
            dout[i + 1] = D.y;
            if (last) aout[i + 1] = A.y;
          }
        }
        if (!last) {
          oE[r >> 1] = A.x;
          if (r + 1 < nl) oO[r >> 1] = A.y;
        }
      }
      __syncthreads();
      if (bnd && !last) {
        // entries outside [0, m_l) become the level's extension (their mirrors are computed
        // entries inside it, host-checked): the next level reads the extended approximation
        for (int r = tid; r < nl; r += kT1) {
          const int i = Sl + r;
          if ((unsigned)i < (unsigned)ml) continue;
          const int mi = ext_near(i, ml, g.mode);
          const int rm = mi - Sl;
          const float v = mi >= 0 ? ((rm & 1) ? oO : oE)[rm >> 1] : 0.f;
          ((r & 1) ? oO : oE)[r >> 1] = v;
        }
        __syncthreads();
      }
      iE = oE;
      iO = oO;
      Sl = (Sl + p) >> 1;
      nl = (nl - p) >> 1;
    }
  }
}

// ------------------------------------------------------------------------------------------------
// synthesis: tile of level-0 outputs [U0, U1); needed coefficient ranges per level
__device__ __forceinline__ void syn_ranges(const Dwt1Geom& g, int u0, int u1, int p, int L, int* I0, int* I1) {
  // (thread 0 only; the ranges are shared through LDS)
  // level l consumes coefficients [I0[l], I1[l]) to produce outputs [lo, hi) of its output length
  int lo = u0, hi = u1;
  for (int l = 0; l < g.J; ++l) {
    int a = (lo + p - L + 2) >> 1;  // ceil((lo + p - L + 1) / 2)
    int b = (hi - 1 + p) >> 1;
    a = max(a, 0);
    b = min(b, g.m[l] - 1);
    I0[l] = a;
    I1[l] = max(a, b + 1);
    lo = I0[l];
    hi = I1[l];
  }
}

template <int L>
__global__ void __launch_bounds__(kT1S) k_dwt1_syn(const float* __restrict__ coeffs, float* __restrict__ out,
                                                 const float* __restrict__ filt, Dwt1Geom g, int nout0, float sc,
                                                 int t_lo, int t_hi) {
  constexpr int p = L - 2;
  constexpr int H2 = L / 2;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x;
  // tiles [t_lo, t_hi) are left to k_dwt1_syn_int; this kernel runs the others (nb per signal)
  const int nb = g.tiles - (t_hi - t_lo);
  const int64_t item = blockIdx.x / nb;
  const int kb = (int)(blockIdx.x % nb);
  const int tile = kb < t_lo ? kb : t_hi + (kb - t_lo);
  float rlo[L], rhi[L];
#pragma unroll
  for (int k = 0; k < L; ++k) {
    rlo[k] = filt[k];
    rhi[k] = filt[L + k];
  }
  const int u0 = tile * (2 * kTile0), u1 = min(nout0, u0 + 2 * kTile0);
  __shared__ int I0[WAM_MAX_LEVELS], I1[WAM_MAX_LEVELS];
  if (tid == 0) syn_ranges(g, u0, u1, p, L, I0, I1);
  __syncthreads();
  const int J = g.J;
  // LDS: two approximation buffers and one detail buffer, each holding a level's coefficient
  // range [I0 - H2, I1 + H2) with zeros outside [0, m) so every output sums exactly H2 taps
  const int cap = g.syn_cap;
  const int off_a[2] = {0, cap};
  const int off_d = 2 * cap;
  auto stage = [&](int off, const float* src, int l) {  // src: the level's band for this item
    const int lo = I0[l] - H2, hi = I1[l] + H2, m = g.m[l];
    for (int i = lo + tid; i < hi; i += kT1S) smem[off + i - lo] = (i >= 0 && i < m) ? sc * src[i] : 0.f;
  };
  stage(off_a[(J - 1) & 1], coeffs + g.items * g.off_a + item * (int64_t)g.m[J - 1], J - 1);
  for (int l = J - 1; l >= 0; --l) {
    stage(off_d, coeffs + g.items * g.off_d[l] + item * (int64_t)g.m[l], l);
    __syncthreads();
    const int ain = off_a[l & 1];
    const int lo = I0[l] - H2;
    const int olo = l ? I0[l - 1] : u0, ohi = l ? I1[l - 1] : u1;
    const int aout = off_a[(l + 1) & 1];  // == off_a[(l - 1) & 1]
    float* o = out + item * (int64_t)nout0;
    for (int u = olo + tid; u < ohi; u += kT1S) {
      const int t = u + p;  // uncropped position
      const int ib = t >> 1;
      const int k0 = t - 2 * ib;
      float y = 0.f;
#pragma unroll
      for (int j = 0; j < H2; ++j) {  // i = ib - j, descending: the order of k_synthesis_axis
        const int idx = ib - j - lo;
        y = fmaf(rlo[k0 + 2 * j], smem[ain + idx], y);
        y = fmaf(rhi[k0 + 2 * j], smem[off_d + idx], y);
      }
      if (l) smem[aout + u - olo + H2] = y;  // staged layout of level l-1: index i at i - (I0 - H2)
      else o[u] = y;
    }
    __syncthreads();
    if (l) {  // zero the pads of the approximation just produced (only ever read outside [0, m))
      const int plo = I0[l - 1] - H2, phi = I1[l - 1] + H2;
      for (int i = plo + tid; i < phi; i += kT1S)
        if (i < I0[l - 1] || i >= I1[l - 1]) smem[aout + i - plo] = 0.f;
      __syncthreads();
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Interior synthesis tiles (no coefficient range clamped at any level): persistent workgroups over
// (signal, tile) units, shapes fixed at compile time by (L, J). An interior output tile
// [u0, u0 + 2 kTile0) needs coefficients [u0 >> (l+1), + n_l) of every level l (n_l below) and
// the same range of A_J-1: about 2 kTile0 floats, fetched into registers one unit ahead (slot
// counts per band known at compile time, one coalesced load per slot) and stored to LDS in one
// pass, so the next unit's HBM latency hides behind the current unit's J levels. A thread makes
// the output pair (2q, 2q + 1), which shares all 2 H2 coefficient reads; the taps keep the order
// of k_dwt1_syn / k_synthesis_axis (j ascending, lo then hi), so the sums are identical.
template <int L>
__host__ __device__ constexpr int syn_n(int l) {  // coefficients of level l for an interior tile
  int n = 2 * kTile0;
  for (int i = 0; i <= l; ++i) n = ((n - 1 + L - 2) >> 1) + 1;
  return n;
}

template <int L, int J>
struct SynShape {
  static constexpr int len(int s) { return syn_n<L>(s < J ? s : J - 1); }  // s = J: A_J-1
  static constexpr int cum(int s) { return s == 0 ? 0 : cum(s - 1) + ((len(s - 1) + 3) & ~3); }
  static constexpr int slots(int s) { return (len(s) + kT1 - 1) / kT1; }
  static constexpr int slot0(int s) { return s == 0 ? 0 : slot0(s - 1) + slots(s - 1); }
  static constexpr int stage = cum(J + 1);
  static constexpr int nslots = slot0(J + 1);
  static constexpr int abuf = (syn_n<L>(0) + 3) & ~3;  // largest reconstructed approximation
  static constexpr int lds_bytes = 4 * (stage + 2 * abuf);
};

// compile-time loop: f(std::integral_constant<int, I>) for I in [B, E)
template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

template <int L, int J>
__global__ void __launch_bounds__(kT1) k_dwt1_syn_int(const float* __restrict__ coeffs, float* __restrict__ out,
                                                     const float* __restrict__ filt, Dwt1Geom g, int nout0, float sc,
                                                     int t_lo, int t_hi, int64_t units) {
  using Sh = SynShape<L, J>;
  constexpr int H2 = L / 2;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x;
  float rlo[L], rhi[L];
#pragma unroll
  for (int k = 0; k < L; ++k) {
    rlo[k] = filt[k];
    rhi[k] = filt[L + k];
  }
  float* stage = smem;
  float* abuf0 = smem + Sh::stage;
  float* abuf1 = abuf0 + Sh::abuf;
  const int nti = t_hi - t_lo;
  float pf[Sh::nslots];
  auto prefetch = [&](int64_t u) {
    u = u < units ? u : units - 1;
    const int64_t item = u / nti;
    const int u0 = (t_lo + (int)(u - item * nti)) * (2 * kTile0);
    static_for<0, J + 1>([&](auto sv) {
      constexpr int s = decltype(sv)::value;
      constexpr int l = s < J ? s : J - 1;
      constexpr int LEN = Sh::len(s), NS = Sh::slots(s), S0 = Sh::slot0(s);
      const float* src = coeffs + g.items * (s < J ? g.off_d[l] : g.off_a) + item * (int64_t)g.m[l] + (u0 >> (l + 1));
      // the last tile's ranges run past the band: clamped (unconditional) loads here, zeros put in
      // when the unit is staged (k_dwt1_syn's rule)
      const int vlen = min(LEN, g.m[l] - (u0 >> (l + 1)));
#pragma unroll
      for (int k = 0; k < NS; ++k) {
        const int i = tid + k * kT1;
        pf[S0 + k] = src[i < vlen ? i : vlen - 1];
      }
    });
  };
  int64_t u = blockIdx.x;
  if (u < units) prefetch(u);
  for (; u < units; u += gridDim.x) {
    const int64_t item = u / nti;
    const int u0 = (t_lo + (int)(u - item * nti)) * (2 * kTile0);
    static_for<0, J + 1>([&](auto sv) {
      constexpr int s = decltype(sv)::value;
      constexpr int l = s < J ? s : J - 1;
      constexpr int LEN = Sh::len(s), NS = Sh::slots(s), S0 = Sh::slot0(s), C = Sh::cum(s);
      const int vlen = min(LEN, g.m[l] - (u0 >> (l + 1)));
#pragma unroll
      for (int k = 0; k < NS; ++k) {
        const int i = tid + k * kT1;
        if (i < LEN) stage[C + i] = i < vlen ? sc * pf[S0 + k] : 0.f;
      }
    });
    __syncthreads();
    prefetch(u + gridDim.x);  // in flight while the levels run
    float* o = out + item * (int64_t)nout0 + u0;
    const bool pairs_aligned = (reinterpret_cast<uintptr_t>(o) & 7) == 0;
    static_for<0, J>([&](auto iv) {
      constexpr int ll = J - 1 - decltype(iv)::value;  // coarse to fine
      // coefficient i of level ll sits at i - (u0 >> (ll + 1)); the pair q = outputs (2q, 2q + 1)
      // relative to the level's first output u0 >> ll reads coefficients q .. q + H2 - 1
      const float* ain = ll == J - 1 ? stage + Sh::cum(J) : ((ll & 1) ? abuf0 : abuf1);
      const float* din = stage + Sh::cum(ll);
      float* aout = (ll & 1) ? abuf1 : abuf0;
      constexpr int NOUT = ll ? syn_n<L>(ll > 0 ? ll - 1 : 0) : 2 * kTile0;
      // outputs past the approximation's band (or the signal) are zeros / not written
      const int vout = ll ? g.m[ll > 0 ? ll - 1 : 0] - (u0 >> ll) : nout0 - u0;
      for (int q = tid; q < (NOUT + 1) / 2; q += kT1) {
        // (ya, yb) as one packed chain: tap pairs (2j, 2j + 1) times the broadcast coefficient,
        // each output keeping the scalar chain's tap order (same sums)
        f2v y = {0.f, 0.f};
#pragma unroll
        for (int j = 0; j < H2; ++j) {
          const float av = ain[q + H2 - 1 - j], dv = din[q + H2 - 1 - j];
          y = __builtin_elementwise_fma(f2v{rlo[2 * j], rlo[2 * j + 1]}, (f2v)av, y);
          y = __builtin_elementwise_fma(f2v{rhi[2 * j], rhi[2 * j + 1]}, (f2v)dv, y);
        }
        const float ya = y.x, yb = y.y;
        if (ll) {
          aout[2 * q] = 2 * q < vout ? ya : 0.f;
          if (NOUT % 2 == 0 || 2 * q + 1 < NOUT) aout[2 * q + 1] = 2 * q + 1 < vout ? yb : 0.f;
        } else if (pairs_aligned && 2 * q + 1 < vout) {
          *reinterpret_cast<float2*>(o + 2 * q) = make_float2(ya, yb);
        } else {
          if (2 * q < vout) o[2 * q] = ya;
          if (2 * q + 1 < vout) o[2 * q + 1] = yb;
        }
      }
      __syncthreads();
    });
  }
}


// ------------------------------------------------------------------------------------------------
bool mode_ok(int mode) { return mode != WAM_MODE_PERIODIC; }

// the persistent synthesis' register footprint and LDS for (L, J)
bool syn_int_fits(int L, int J) {
#define WAM_SF(LL, JJ) \
  if (L == LL && J == JJ) return SynShape<LL, JJ>::nslots <= 40 && SynShape<LL, JJ>::lds_bytes <= kLds1Cap;
#define WAM_SFJ(LL) WAM_SF(LL, 1) WAM_SF(LL, 2) WAM_SF(LL, 3) WAM_SF(LL, 4) WAM_SF(LL, 5) WAM_SF(LL, 6) \
                    WAM_SF(LL, 7) WAM_SF(LL, 8)
  WAM_SFJ(2) WAM_SFJ(4) WAM_SFJ(6) WAM_SFJ(8) WAM_SFJ(10) WAM_SFJ(12) WAM_SFJ(14) WAM_SFJ(16) WAM_SFJ(18) WAM_SFJ(20)
#undef WAM_SFJ
#undef WAM_SF
  return false;
}

Dwt1Geom make_geom1(const wam_plan* p, int n, int mode, int64_t items) {
  Dwt1Geom g{};
  g.J = p->levels;
  g.mode = mode;
  g.n = n;
  for (int l = 0; l < p->levels; ++l) {
    g.m[l] = (int)p->lout[l][0];
    g.off_d[l] = p->band_off[wam_band_of(p, l, 0)];
  }
  g.off_a = p->band_off[0];
  g.items = items;
  g.tile_j = std::max(1, kTileA >> (p->levels - 1));
  int tiles = 1;
  for (int l = 0; l < p->levels; ++l) {
    const int T = g.tile_j << (p->levels - 1 - l);
    tiles = std::max(tiles, (g.m[l] + T - 1) / T);
  }
  g.tiles = tiles;
  return g;
}

// exact LDS of the analysis: the largest window + approximation buffers over all tiles (the
// first, an interior and the last tiles bound every case; ranges from the device's own rule)
int ana_lds_bytes(const wam_plan* p, const Dwt1Geom& g) {
  int best = 0;
  const int cand[4] = {0, 1, std::max(0, g.tiles - 2), g.tiles - 1};
  for (int c = 0; c < 4; ++c) {
    int S[WAM_MAX_LEVELS], E[WAM_MAX_LEVELS], s[WAM_MAX_LEVELS], e[WAM_MAX_LEVELS];
    ana_ranges(g, cand[c], p->L - 2, S, E, s, e);
    const int wlen = 2 * (E[0] - S[0]) + p->L - 2;
    const int need = ((wlen + 63) & ~63) + 2 * ((E[0] - S[0] + 63) & ~63);
    best = std::max(best, need);
  }
  return best * 4;
}

// interior tiles: every level's computed range and taps inside the signal, own range complete
bool tile_interior(const Dwt1Geom& g, int tile, int p) {
  int S = tile * g.tile_j, E = (tile + 1) * g.tile_j;
  for (int l = g.J - 1; l >= 0; --l) {
    const int T = g.tile_j << (g.J - 1 - l);
    const int nin = l ? g.m[l - 1] : g.n;
    if (S < 0 || E > g.m[l] || (tile + 1) * T > g.m[l]) return false;
    if (2 * S - p < 0 || 2 * E - 1 >= nin) return false;
    if (l) {
      S = 2 * S - p;
      E = 2 * E;
    }
  }
  return true;
}

// boundary tiles can run in the interior kernel (fold): at every level but the last, each
// computed entry outside [0, m_l) of a boundary tile's closed-form range mirrors to a zero or to a
// computed entry inside [0, m_l)
bool tiles_foldable(const Dwt1Geom& g, int p, int t_lo, int t_hi) {
  for (int t = 0; t < g.tiles; ++t) {
    if (t >= t_lo && t < t_hi) continue;
    for (int l = 0; l + 1 < g.J; ++l) {
      const int k = 1 << (g.J - 1 - l);
      const int Sl = ((t * g.tile_j) * k) - p * (k - 1);
      const int nl = g.tile_j * k + p * (k - 1);
      const int ml = g.m[l];
      for (int i = Sl; i < Sl + nl; ++i) {
        if (i >= 0 && i < ml) continue;
        const int mi = ext_near(i, ml, g.mode);
        if (mi >= 0 && (mi < Sl || mi >= Sl + nl)) return false;
      }
    }
  }
  return true;
}

void interior_range(const Dwt1Geom& g, int p, int& t_lo, int& t_hi) {
  t_lo = t_hi = 0;
  int t = 0;
  while (t < g.tiles && !tile_interior(g, t, p)) ++t;
  t_lo = t;
  while (t < g.tiles && tile_interior(g, t, p)) ++t;
  t_hi = t;
  if (t_hi <= t_lo) t_lo = t_hi = 0;
}

// window (E / O) + the even levels' buffer; the odd levels reuse the window's space: 51.5 KB at
// c3's 4,096-sample tiles, so three workgroups fit a CU (the noisy kernel's 57 VGPRs allow six
// waves per SIMD)
int ana_int_lds_bytes(const Dwt1Geom& g, int p) {
  const int n0 = (g.tile_j << (g.J - 1)) + p * ((1 << (g.J - 1)) - 1);
  return (2 * eo_cap(2 * n0 + p) + 2 * eo_cap(n0)) * 4;
}

int syn_lds_bytes(const wam_plan* p) {
  // level-0 coefficient range of a 2*kTile0 output tile: kTile0 + L/2 (+ the H2 zero pads)
  const int cap = ((kTile0 + 2 * p->L + 8) + 63) & ~63;
  return 3 * cap * 4;
}

}  // namespace

bool dwt1_tile_supported(const wam_plan* p, bool adjoint) {
  if (p->ndim != 1 || p->L > 20 || (p->L & 1)) return false;
  if (!mode_ok(adjoint ? WAM_MODE_ZERO : p->mode)) return false;
  if (p->lin[0][0] > (1 << 30)) return false;
  const Dwt1Geom g = make_geom1(p, (int)(adjoint ? p->rec_shape[0] : p->lin[0][0]), adjoint ? WAM_MODE_ZERO : p->mode, 1);
  return ana_lds_bytes(p, g) <= kLds1Cap && syn_lds_bytes(p) <= kLds1Cap;
}

int launch_dwt1_tile_analysis(const wam_plan* p, int64_t batch, const float* in, float* coeffs, bool adjoint,
                              hipStream_t st, const WamNoise* nz, int64_t n_samples) {
  if (!dwt1_tile_supported(p, adjoint)) return WAM_ERR_UNSUPPORTED;
  if (nz) {  // SmoothGrad noise fused on the load: single-channel signals, length a multiple of 4
    if (adjoint || nz->channels != 1 || batch != n_samples * nz->images || p->lin[0][0] % 4 ||
        ((uintptr_t)in & 15))
      return WAM_ERR_UNSUPPORTED;
  }
  const WamNoise none{nullptr, 1, 1, 0, 0, 0, 0};
  const WamNoise& NZ = nz ? *nz : none;
  const int64_t S = nz ? n_samples : 1;
  const int n = (int)(adjoint ? p->rec_shape[0] : p->lin[0][0]);
  const int mode = adjoint ? WAM_MODE_ZERO : p->mode;
  const Dwt1Geom g = make_geom1(p, n, mode, batch);
  const float* filt = p->d_filt + (adjoint ? WAM_F_ADJ_LO : WAM_F_ANA_LO) * p->L;
  const int64_t blocks = batch * g.tiles;
  if (blocks > 0x7fffffff) return WAM_ERR_UNSUPPORTED;
  const int lds = ana_lds_bytes(p, g);
  const int pp = p->L - 2;
  int t_lo, t_hi;
  interior_range(g, pp, t_lo, t_hi);
  const int n0 = (g.tile_j << (g.J - 1)) + pp * ((1 << (g.J - 1)) - 1);
  const int lds_i = ana_int_lds_bytes(g, pp);
  if (2 * n0 + pp > kPF * kT1 || lds_i > kLds1Cap) t_lo = t_hi = 0;  // window too long: all tiles generic
  // boundary tiles folded into the persistent launch (one launch, the interior kernel's level
  // loop for every tile) when their extension stays within the closed-form ranges
  const int fold = (t_hi > t_lo && tiles_foldable(g, pp, t_lo, t_hi)) ? 1 : 0;
  const int64_t units = batch * (int64_t)(fold ? g.tiles : t_hi - t_lo);
  const int64_t nb_blocks = fold ? 0 : batch * (int64_t)(g.tiles - (t_hi - t_lo));
  // algorithmic bytes: every input once (noisy: the clean signals once for all samples) and
  // every output once
  const double bytes = nz ? 4.0 * ((double)nz->images * n + (double)batch * p->band_off[p->nbands])
                          : 4.0 * (double)batch * ((double)n + (double)p->band_off[p->nbands]);
  if (units > 0) {
    int dev = 0;
    WAM_HIP_CHECK(hipGetDevice(&dev));
    int cus = 256;
    WAM_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    WamTimer tm(st, nz ? "k_dwt1_ana_int<noise>" : "k_dwt1_ana_int",
                fold ? bytes : bytes * (double)(t_hi - t_lo) / g.tiles);
    // persistent grid: exactly the resident workgroups (VGPRs and LDS decide: 2 per CU for the
    // clean kernel's 107 VGPRs, 3 for the noisy one's 57 at c3's 51.5 KB of LDS), so no workgroup
    // waits for a slot and the units split evenly
    switch (p->L) {
#define WAM_D1AIN(LL, NN)                                                                                         \
  {                                                                                                               \
    if (int rc = lds_opt_in((const void*)k_dwt1_ana_int<LL, NN>, lds_i)) return rc;                              \
    int wgs = kAnaWgs;                                                                                            \
    WAM_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&wgs, k_dwt1_ana_int<LL, NN>, kT1, lds_i));         \
    const int64_t grid = std::min<int64_t>(units, (int64_t)std::max(1, wgs) * cus);                              \
    hipLaunchKernelGGL((k_dwt1_ana_int<LL, NN>), dim3((unsigned)grid), dim3(kT1), lds_i, st, in, coeffs, filt, g, \
                       t_lo, t_hi, units, NZ, S, fold);                                                           \
  }
#define WAM_D1AI(LL)                                                                                            \
  case LL:                                                                                                      \
    if (nz) {                                                                                                   \
      WAM_D1AIN(LL, true)                                                                                       \
    } else {                                                                                                    \
      WAM_D1AIN(LL, false)                                                                                      \
    }                                                                                                           \
    break;
      WAM_D1AI(2) WAM_D1AI(4) WAM_D1AI(6) WAM_D1AI(8) WAM_D1AI(10) WAM_D1AI(12) WAM_D1AI(14) WAM_D1AI(16)
      WAM_D1AI(18) WAM_D1AI(20)
#undef WAM_D1AI
#undef WAM_D1AIN
      default: return WAM_ERR_UNSUPPORTED;
    }
    WAM_LAUNCH_CHECK();
  }
  // boundary tiles: persistent with window prefetch when every boundary window fits kPF * kT1
  int max_wlen = 0;
  for (int t = 0; t < g.tiles; ++t) {
    if (t >= t_lo && t < t_hi) continue;
    int S[WAM_MAX_LEVELS], E[WAM_MAX_LEVELS], s[WAM_MAX_LEVELS], e[WAM_MAX_LEVELS];
    ana_ranges(g, t, pp, S, E, s, e);
    max_wlen = std::max(max_wlen, 2 * (E[0] - S[0]) + pp);
  }
  if (nb_blocks > 0 && max_wlen <= kPF * kT1) {
    int dev = 0;
    WAM_HIP_CHECK(hipGetDevice(&dev));
    int cus = 256;
    WAM_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const int64_t grid = std::min<int64_t>(nb_blocks, (int64_t)kAnaWgs * cus);
    WamTimer tm(st, nz ? "k_dwt1_ana_p<noise>" : "k_dwt1_ana_p", bytes * (double)(g.tiles - (t_hi - t_lo)) / g.tiles);
    switch (p->L) {
#define WAM_D1APN(LL, NN)                                                                                      \
  if (int rc = lds_opt_in((const void*)k_dwt1_ana_p<LL, NN>, lds)) return rc;                                 \
  hipLaunchKernelGGL((k_dwt1_ana_p<LL, NN>), dim3((unsigned)grid), dim3(kT1), lds, st, in, coeffs, filt, g, t_lo, \
                     t_hi, nb_blocks, NZ);
#define WAM_D1AP(LL)                                                                                           \
  case LL:                                                                                                     \
    if (nz) {                                                                                                  \
      WAM_D1APN(LL, true)                                                                                      \
    } else {                                                                                                   \
      WAM_D1APN(LL, false)                                                                                     \
    }                                                                                                          \
    break;
      WAM_D1AP(2) WAM_D1AP(4) WAM_D1AP(6) WAM_D1AP(8) WAM_D1AP(10) WAM_D1AP(12) WAM_D1AP(14) WAM_D1AP(16)
      WAM_D1AP(18) WAM_D1AP(20)
#undef WAM_D1AP
#undef WAM_D1APN
      default: return WAM_ERR_UNSUPPORTED;
    }
    WAM_LAUNCH_CHECK();
  } else if (nb_blocks > 0) {
    WamTimer tm(st, nz ? "k_dwt1_ana<noise>" : "k_dwt1_ana", bytes * (double)(g.tiles - (t_hi - t_lo)) / g.tiles);
    switch (p->L) {
#define WAM_D1AN(LL, NN)                                                                                     \
  if (int rc = lds_opt_in((const void*)k_dwt1_ana<LL, NN>, lds)) return rc;                                 \
  hipLaunchKernelGGL((k_dwt1_ana<LL, NN>), dim3((unsigned)nb_blocks), dim3(kT1), lds, st, in, coeffs, filt, g, \
                     t_lo, t_hi, NZ);
#define WAM_D1A(LL)                                                                                          \
  case LL:                                                                                                   \
    if (nz) {                                                                                                \
      WAM_D1AN(LL, true)                                                                                     \
    } else {                                                                                                 \
      WAM_D1AN(LL, false)                                                                                    \
    }                                                                                                        \
    break;
      WAM_D1A(2) WAM_D1A(4) WAM_D1A(6) WAM_D1A(8) WAM_D1A(10) WAM_D1A(12) WAM_D1A(14) WAM_D1A(16) WAM_D1A(18)
      WAM_D1A(20)
#undef WAM_D1A
#undef WAM_D1AN
      default: return WAM_ERR_UNSUPPORTED;
    }
    WAM_LAUNCH_CHECK();
  }
  return WAM_OK;
}

int launch_dwt1_tile_synthesis(const wam_plan* p, int64_t batch, const float* coeffs, const float* alpha,
                               int n_alpha, float* out, hipStream_t st) {
  if (!dwt1_tile_supported(p, false)) return WAM_ERR_UNSUPPORTED;
  const int nout = (int)p->rec_shape[0];
  Dwt1Geom g = make_geom1(p, (int)p->lin[0][0], p->mode, batch);
  g.tiles = (nout + 2 * kTile0 - 1) / (2 * kTile0);
  g.syn_cap = syn_lds_bytes(p) / 12;
  const int64_t blocks = batch * g.tiles;
  if (blocks > 0x7fffffff) return WAM_ERR_UNSUPPORTED;
  const float* filt = p->d_filt + WAM_F_SYN_LO * p->L;
  const int lds = syn_lds_bytes(p);
  // every tile on the persistent kernel (J <= 8; coefficient ranges are only ever clamped at the
  // right end, which its zero rule covers), k_dwt1_syn otherwise
  int t_lo = 0, t_hi = 0;
  if (g.J <= 8 && syn_int_fits(p->L, g.J)) t_hi = g.tiles;
  const int64_t units = batch * (int64_t)(t_hi - t_lo);
  int cus = 256;
  if (units > 0) {
    int dev = 0;
    WAM_HIP_CHECK(hipGetDevice(&dev));
    WAM_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  }
  const double bytes_all = 4.0 * ((double)batch * p->band_off[p->nbands] + (double)batch * (double)nout);
  for (int ai = 0; ai < n_alpha && units > 0; ++ai) {
    const float sc = alpha ? alpha[ai] : 1.0f;
    float* o = out + (int64_t)ai * batch * nout;
    const int64_t grid = std::min<int64_t>(units, 2LL * cus);
    WamTimer tm(st, "k_dwt1_syn_int", bytes_all * (double)(t_hi - t_lo) / g.tiles);
    int rc = WAM_ERR_UNSUPPORTED;
#define WAM_D1SI(LL, JJ)                                                                                        \
  if (p->L == LL && g.J == JJ) {                                                                                \
    using Sh = SynShape<LL, JJ>;                                                                                \
    if (int e = lds_opt_in((const void*)k_dwt1_syn_int<LL, JJ>, Sh::lds_bytes)) return e;                        \
    hipLaunchKernelGGL((k_dwt1_syn_int<LL, JJ>), dim3((unsigned)grid), dim3(kT1), Sh::lds_bytes, st, coeffs, o, \
                       filt, g, nout, sc, t_lo, t_hi, units);                                                  \
    rc = WAM_OK;                                                                                                \
  }
#define WAM_D1SJ(LL) WAM_D1SI(LL, 1) WAM_D1SI(LL, 2) WAM_D1SI(LL, 3) WAM_D1SI(LL, 4) WAM_D1SI(LL, 5) \
                     WAM_D1SI(LL, 6) WAM_D1SI(LL, 7) WAM_D1SI(LL, 8)
    WAM_D1SJ(2) WAM_D1SJ(4) WAM_D1SJ(6) WAM_D1SJ(8) WAM_D1SJ(10) WAM_D1SJ(12) WAM_D1SJ(14) WAM_D1SJ(16)
    WAM_D1SJ(18) WAM_D1SJ(20)
#undef WAM_D1SJ
#undef WAM_D1SI
    if (rc) return rc;
    WAM_LAUNCH_CHECK();
  }
  const int64_t nb_blocks = batch * (int64_t)(g.tiles - (t_hi - t_lo));
  if (nb_blocks == 0) return WAM_OK;
  for (int ai = 0; ai < n_alpha; ++ai) {
    const float sc = alpha ? alpha[ai] : 1.0f;
    float* o = out + (int64_t)ai * batch * nout;
    WamTimer tm(st, "k_dwt1_syn", bytes_all * (double)(g.tiles - (t_hi - t_lo)) / g.tiles);
    switch (p->L) {
#define WAM_D1S(LL)                                                                                            \
  case LL:                                                                                                     \
    if (int rc = lds_opt_in((const void*)k_dwt1_syn<LL>, lds)) return rc;                                      \
    hipLaunchKernelGGL(k_dwt1_syn<LL>, dim3((unsigned)nb_blocks), dim3(kT1S), lds, st, coeffs, o, filt, g, nout, sc, \
                       t_lo, t_hi);                                                                            \
    break;
      WAM_D1S(2) WAM_D1S(4) WAM_D1S(6) WAM_D1S(8) WAM_D1S(10) WAM_D1S(12) WAM_D1S(14) WAM_D1S(16) WAM_D1S(18)
      WAM_D1S(20)
#undef WAM_D1S
      default: return WAM_ERR_UNSUPPORTED;
    }
    WAM_LAUNCH_CHECK();
  }
  return WAM_OK;
}

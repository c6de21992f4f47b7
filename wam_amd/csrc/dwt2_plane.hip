// Plane-resident multi-level 2D analysis for gfx950: ALL J levels of one plane in ONE workgroup,
// the LL pyramid never leaves LDS.
//
// Why: the per-level kernels (dwt2_rows.hip) write LL_1 to HBM and read it back for level 2, and
// every coarse level is its own small launch whose ramp-up dominates (a 224^2 db4 batch spends
// 45 us in levels 2-3 for 16% of the bytes). Here a 512-thread workgroup owns one plane (or one
// image of C planes for the WAM backward pass):
//   phase 1  level 1 (finest), row-resident: each of the 8 waves streams a chunk of whole source
//            rows with 16-B loads, 3 rows in flight (4-deep register ring of fetched rows), adds
//            the SmoothGrad noise at commit time (Philox, same stream as wam_noise_add) or
//            averages the C channel rows (WAM backward: mean over C commutes with the linear
//            adjoint), applies the boundary extension in LDS pad slots, filters horizontally from
//            LDS and vertically from a register ring of L rows. H/V/D go to HBM, LL_1 to LDS.
//   phase 2  levels 2..J from LDS: one thread per output column and row block, horizontal taps
//            through precomputed extended column indices, vertical register ring; LL ping-pongs
//            between two LDS buffers, the last level writes A_J.
// Two workgroups fit a CU for 224^2 inputs (LL_1 53 KB + 9 KB of wave rows), 16 waves per CU.
//
// Outputs: coefficient mode = band-major coefficients (as wam_wavedec); maps mode = the WAM
// epilogue (lib/wam_2D.py:227-256): |coefficient of the channel mean| packed item-major, and
// per-band maxima reduced wave -> LDS -> one global atomic max per workgroup and band.
//
// Workgroup order: an XCD-aware bijective swizzle makes consecutive logical workgroups share an
// XCD (L2); for noisy analysis the logical order is sample-fastest, so the S noise samples of one
// clean plane run back to back on one XCD and its rows are read from HBM about once.
#include <atomic>

#include "rowtools.hpp"

namespace {

using namespace wam_rows;

constexpr int kPW = 8;                 // waves per workgroup
constexpr int kPT = 64 * kPW;          // threads per workgroup
constexpr int kPlaneMaxW = 256;        // level-0 row width (one float4 per lane)
constexpr int kPlaneMaxMW = 128;       // level-1 output width (two columns per lane)
constexpr int kPlaneLdsCap = 160 * 1024 - 1024;
// noisy wave-chunk level 1 computes the halo rows of the boundaries where a pair of waves meets
// once (bidirectional chunks); at CPL = 2 lane l filters the ADJACENT columns
// 2l, 2l+1 (one run of L/2+1 LDS pairs feeds both, each band row stored as float2 pairs)

struct PlaneGeom {
  int J;
  int mode;
  int nh0, nw0;
  int mh[WAM_MAX_LEVELS], mw[WAM_MAX_LEVELS];
  int64_t off_a;                    // per-item offset of band 0 (A_J)
  int64_t off[WAM_MAX_LEVELS][3];   // per-item offsets of (H, V, D) of level l (0 = finest)
  int band[WAM_MAX_LEVELS][3];      // their band indices
  int nbands;
  int64_t items_total;              // band-major multiplier (coefficient mode)
  int64_t maps_item;                // packed floats per item (maps mode)
  int rowlds;                       // floats per wave-private row
  int llcap;                        // floats of LDS buffer A (LL_1, LL_3, ...)
  int sample_fast;                  // noisy analysis: logical order sample-fastest (1) or plane-fastest (0)
  int xcd_order;                    // workgroup ids through the XCD-aware swizzle (1) or as issued (0)
  int coop;                         // level 1 as the cooperative row stream (COOP kernels)
  int xend;                         // noisy wave chunks: float offset in buffer B of the END-boundary
                                    // exchange (-1: not allocated, halo rows computed by both waves)
};

template <bool MAPS>
struct BandOut {
  float* out;
  int64_t item;
  // columns idx, idx + 1 of one band row (pair: both inside the row) -- one 8-byte store (4-byte
  // aligned rows: unaligned access mode) instead of two
  __device__ __forceinline__ void put2(const PlaneGeom& g, int64_t off, int64_t numel, int64_t idx, float v0,
                                       float v1, bool pair, float& mx) const {
    typedef float f2s __attribute__((ext_vector_type(2)));
    if constexpr (MAPS) {
      put(g, off, numel, idx, v0, mx);
      if (pair) put(g, off, numel, idx + 1, v1, mx);
    } else if (pair) {
      const f2s v = {v0, v1};
      __builtin_memcpy(out + g.items_total * off + item * numel + idx, &v, 8);
    } else {
      out[g.items_total * off + item * numel + idx] = v0;
    }
  }
  __device__ __forceinline__ void put(const PlaneGeom& g, int64_t off, int64_t numel, int64_t idx, float v,
                                      float& mx) const {
    if constexpr (MAPS) {
      const float a = fabsf(v);
      out[item * g.maps_item + off + idx] = a;
      mx = nan_max(mx, a);
    } else {
      out[g.items_total * off + item * numel + idx] = v;
    }
  }
};

// compile-time loop: f(std::integral_constant<int, I>) for I in [B, E)
template <int B, int E, class F>
__device__ __forceinline__ void plane_static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    plane_static_for<B + 1, E>(f);
  }
}

__device__ __forceinline__ float wave_max(float m) {
#pragma unroll
  for (int s = 32; s > 0; s >>= 1) m = nan_max(m, __shfl_xor(m, s, 64));
  return m;
}

// Input formats of the COOP maps pass: fp32 planes, or the explained model's own bf16 input gradient
// in NHWC (channels_last) or NCHW order (widened on use: exact)
enum { kInF32 = 0, kInBf16Nhwc = 1, kInBf16Nchw = 2 };

// One source row of the COOP level 1 in registers (lane l: columns 4l .. 4l+3 of every channel).
// fp32: NCH planar rows, 16-byte loads. bf16 NHWC: the image row, channels interleaved, NCH * 8 bytes
// per lane; bf16 NCHW: NCH planar rows, 8 bytes per lane each.
// Loads stay in flight until v() is first used (clamped addresses, validity applied on use).
template <int NCH, int FMT>
struct CoopRow {
  RowRegs<4, 1> r[NCH];
  __device__ __forceinline__ void fetch(const float* src, int64_t in_plane, int row, int nw, int lane, bool valid) {
#pragma unroll
    for (int c = 0; c < NCH; ++c) r[c].fetch(src + c * in_plane + (int64_t)row * nw, nw, lane, valid);
  }
  __device__ __forceinline__ bool ok() const { return r[0].ok[0]; }
  __device__ __forceinline__ float v(int c, int k) const { return r[c].v[k]; }
};

template <int NCH>
struct CoopRow<NCH, kInBf16Nhwc> {
  uint2 raw[NCH];  // 4 * NCH bf16 values: pixel k, channel c at element k * NCH + c
  bool okv;
  __device__ __forceinline__ void fetch(const float* src, int64_t, int row, int nw, int lane, bool valid) {
    const int idx = lane * 4;
    okv = valid && idx < nw;
    const int ci = idx < nw ? idx : nw - 4;
    const uint2* p = reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(src) +
                                                    ((int64_t)row * nw + ci) * NCH);
#pragma unroll
    for (int k = 0; k < NCH; ++k) raw[k] = p[k];
  }
  __device__ __forceinline__ bool ok() const { return okv; }
  __device__ __forceinline__ float v(int c, int k) const {
    const int e = k * NCH + c;  // static after unrolling
    const uint32_t w = (e & 2) ? raw[e >> 2].y : raw[e >> 2].x;
    return __uint_as_float((e & 1) ? (w & 0xffff0000u) : (w << 16));
  }
};

template <int NCH>
struct CoopRow<NCH, kInBf16Nchw> {
  uint2 raw[NCH];  // channel c: pixels 4l .. 4l+3 of its plane's row
  bool okv;
  __device__ __forceinline__ void fetch(const float* src, int64_t in_plane, int row, int nw, int lane, bool valid) {
    const int idx = lane * 4;
    okv = valid && idx < nw;
    const int ci = idx < nw ? idx : nw - 4;
    const uint16_t* b = reinterpret_cast<const uint16_t*>(src) + (int64_t)row * nw + ci;
#pragma unroll
    for (int c = 0; c < NCH; ++c) raw[c] = *reinterpret_cast<const uint2*>(b + c * in_plane);
  }
  __device__ __forceinline__ bool ok() const { return okv; }
  __device__ __forceinline__ float v(int c, int k) const {
    const uint32_t w = (k & 2) ? raw[c].y : raw[c].x;
    return __uint_as_float((k & 1) ? (w & 0xffff0000u) : (w << 16));
  }
};

// MC: 0 = one input plane per item; C > 0 = item is an image of C planes, averaged on load
// CPL: level-1 output columns per lane (mw <= 64 * CPL): one wave covers a whole row
// COOP: level 1 as a cooperative row stream (see phase 1 below) instead of wave-private chunks
// IN (COOP maps only for the bf16 formats): kInF32, or bf16 images [items, nh, nw, MC] (kInBf16Nhwc)
// / [items, MC, nh, nw] (kInBf16Nchw)
template <int L, int CPL, bool NOISE, int MC, bool MAPS, bool COOP, int IN = kInF32, int PW = kPW>
__global__ void __launch_bounds__(64 * PW) __attribute__((amdgpu_waves_per_eu(PW > 8 ? 5 : 4, 8))) k_plane_ana(const float* __restrict__ in, float* __restrict__ out,
                                                   float* __restrict__ band_max, const float* __restrict__ filt,
                                                   PlaneGeom g, WamNoise nz, int64_t n_items, int64_t S,
                                                   int64_t group_items) {
  constexpr int p = L - 2;
  constexpr int NCH = MC > 0 ? MC : 1;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  __shared__ unsigned int wg_max[WAM_MAX_BANDS];

  // ---- logical workgroup: bijective XCD swizzle (consecutive logical ids share an XCD)
  const int64_t nwg = gridDim.x, bid = blockIdx.x;
  const int64_t q8 = nwg / 8, r8 = nwg % 8, xcd = bid % 8;
  const int64_t lwg = g.xcd_order ? (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8 : bid;
  if (lwg >= n_items) return;  // never taken (grid == n_items); keeps the barrier count uniform

  // the wave index is wave-uniform: readfirstlane puts it (and every row index, ring slot and
  // Philox counter word derived from it) in SGPRs, so row bookkeeping runs on the scalar unit
  const int tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nh = g.nh0, nw = g.nw0;
  const int64_t in_plane = (int64_t)nh * nw;

  int64_t item = lwg, src_plane = lwg, img = 0, smp = 0, ch = 0;
  float sg = 0.f;
  if constexpr (NOISE) {
    const int64_t nc = nz.images * nz.channels;
    int64_t s;
    if (g.sample_fast) {
      src_plane = lwg / S;                // sample-fastest: the S samples of a plane are adjacent
      s = lwg % S;
      item = s * nc + src_plane;          // output planes are (sample, image, channel)
    } else {
      s = lwg / nc;
      src_plane = lwg % nc;
    }
    smp = nz.sample_base + s;
    img = src_plane / nz.channels;
    ch = src_plane % nz.channels;
    sg = nz.sigma[img];
  }
  static_assert(IN == kInF32 || (COOP && MAPS && !NOISE), "bf16 input: COOP maps pass only");
  static_assert(PW == kPW || (!COOP && NOISE), "other workgroup sizes: noisy wave chunks only");
  const float* src = IN != kInF32 ? reinterpret_cast<const float*>(reinterpret_cast<const uint16_t*>(in) +
                                                                   src_plane * (int64_t)NCH * in_plane)
                                  : in + src_plane * (int64_t)NCH * in_plane;

  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 fh2[L];  // (lo, hi) tap pairs for packed fp32 FMAs
  float flo[L], fhi[L];
#pragma unroll
  for (int k = 0; k < L; ++k) {
    fh2[k] = f2{filt[k], filt[L + k]};
    // filter taps live in VGPRs: as 2L scalar registers they push the kernel past the SGPR budget
    // and the compiler spills uniform values to VGPR lanes (v_readlane + hazard nops per use)
    asm volatile("" : "+v"(fh2[k]));
    flo[k] = fh2[k].x;
    fhi[k] = fh2[k].y;
  }
  if constexpr (MAPS) {
    if (tid < g.nbands) wg_max[tid] = 0u;
    __syncthreads();
  }
  const BandOut<MAPS> bo{out, item};
  float* bufA = smem;
  float* bufB = smem + g.llcap;

  // SmoothGrad noise of two source rows sra, srb (< 0: zero rows, any value) of this plane,
  // generated together (two interleaved Philox chains). Element group g = (row's first element) / 4
  // + lane < 2^32 (host check), so wam_normal4_x2 reproduces wam_normal4's stream; lanes past the
  // row are never stored.
  auto noise2 = [&](float (&za)[4], float (&zb)[4], int sra, int srb) {
    if constexpr (NOISE) {
      const uint32_t rowg = (uint32_t)(ch * nh) * (uint32_t)nw / 4u + (uint32_t)lane;
      const uint32_t nw4 = (uint32_t)nw / 4u;
      wam_normal4_x2(rowg + (uint32_t)(sra >= 0 ? sra : 0) * nw4, rowg + (uint32_t)(srb >= 0 ? srb : 0) * nw4,
                     (uint32_t)(img + nz.image_base), (uint32_t)smp, nz.k0, nz.k1, za, zb);
      // both blocks used here: otherwise the compiler sinks row b's chain to its consume() one row
      // later and the two Philox chains no longer interleave
      asm volatile("" ::"v"(za[0]), "v"(za[1]), "v"(za[2]), "v"(za[3]), "v"(zb[0]), "v"(zb[1]), "v"(zb[2]),
                   "v"(zb[3]));
    }
  };

  // ================================================================ phase 1: level 1 (finest)
  if constexpr (COOP) {
    // Cooperative row stream. Extended rows e (ext row e = source row wam_ext_index(e)) are
    // produced in blocks of 16: wave w fetches rows 16b+2w, 16b+2w+1 (Philox noise / channel
    // mean applied on the commit to its padded LDS row), filters them horizontally and stores
    // (lo, hi) per output column into a ring of kRing ext rows; after a barrier the 512 threads
    // filter vertically: thread (column j, pair q) emits output rows 8b+2q, 8b+2q+1 from 10 ring
    // rows. Every source row is fetched and noised once (the wave-chunk form re-fetches L-2 halo
    // rows per wave, 29 % more at 224^2), and the row fetches of the next D-1 blocks stay in
    // flight in registers across both barriers (plain loads survive __syncthreads()).
    constexpr int RB = 8;                      // output rows per block
    constexpr int kRing = 2 * RB + L - 2;      // ext rows a block's vertical pass reads
    constexpr int D = NCH > 1 ? 1 : 2;         // blocks of row fetches in flight
    constexpr int PADL = 8;                    // left pad slots (>= p, 16-byte aligned row body)
    const int mh = g.mh[0], mw = g.mw[0];
    const int64_t bn = (int64_t)mh * mw;
    const bool lastlvl = g.J == 1;
    const int mode = g.mode;
    const bool zero_mode = mode == WAM_MODE_ZERO;
    float* wrow = bufB + wv * g.rowlds;
    float2* ring = reinterpret_cast<float2*>(bufB + PW * g.rowlds);
    const PadLane pl = pad_lane(lane, nw, p, mode, PADL);
    if (zero_mode && pl.dst >= 0) wrow[pl.dst] = 0.f;
    const int nb = (mh + RB - 1) / RB;
    float mx[4] = {0.f, 0.f, 0.f, 0.f};

    using CRow = CoopRow<NCH, IN>;
    auto fetch = [&](CRow& fr, int& sr_out, int e) {
      const int sr = row_src(e, nh, mode);
      const bool valid = sr >= 0;
      sr_out = sr;
      fr.fetch(src, in_plane, valid ? sr : 0, nw, lane, valid);
    };
    // horizontal pass of ext row e into its ring slot (nzr: its noise, from noise2)
    auto hrow = [&](CRow& fr, int sr, int e, const float (&nzr)[4]) {
      float4 o = fr.ok() ? make_float4(fr.v(0, 0), fr.v(0, 1), fr.v(0, 2), fr.v(0, 3)) : make_float4(0.f, 0.f, 0.f, 0.f);
      if constexpr (NCH > 1) {
#pragma unroll
        for (int c = 1; c < NCH; ++c) {
          o.x += fr.v(c, 0);
          o.y += fr.v(c, 1);
          o.z += fr.v(c, 2);
          o.w += fr.v(c, 3);
        }
        constexpr float inv = 1.0f / (float)NCH;
        o.x *= inv;
        o.y *= inv;
        o.z *= inv;
        o.w *= inv;
        if (!fr.ok()) o = make_float4(0.f, 0.f, 0.f, 0.f);
      }
      if constexpr (NOISE) {
        // zero rows (sr < 0, wave-uniform) stay zero: fma(0, z, 0) with a finite z
        const float sgr = sr >= 0 ? sg : 0.f;
        o.x = fmaf(sgr, nzr[0], o.x);
        o.y = fmaf(sgr, nzr[1], o.y);
        o.z = fmaf(sgr, nzr[2], o.z);
        o.w = fmaf(sgr, nzr[3], o.w);
      }
      if (lane * 4 < nw) *reinterpret_cast<float4*>(wrow + PADL + lane * 4) = o;
      wsync();
      if (!zero_mode) {
        refresh_pads(wrow, pl);
        wsync();
      }
      const int slot = (e + p) % kRing;
      // (lo, hi) of the CPL columns as packed FMAs, per accumulator in tap order 0..L-1 (the
      // wave-chunk form's order); the CPL chains interleaved to hide the packed-FMA hazard
      f2 acc[CPL];
#pragma unroll
      for (int c = 0; c < CPL; ++c) acc[c] = f2{0.f, 0.f};
#pragma unroll
      for (int m2 = 0; m2 < L / 2; ++m2) {
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
          const int j = min(lane + 64 * c, mw - 1);
          const float2 x = reinterpret_cast<const float2*>(wrow + PADL + 2 * j - p)[m2];
          acc[c] = __builtin_elementwise_fma(fh2[2 * m2], f2{x.x, x.x}, acc[c]);
          acc[c] = __builtin_elementwise_fma(fh2[2 * m2 + 1], f2{x.y, x.y}, acc[c]);
        }
      }
#pragma unroll
      for (int c = 0; c < CPL; ++c) {
        const int j = min(lane + 64 * c, mw - 1);
        if (lane + 64 * c < mw) ring[slot * mw + j] = make_float2(acc[c].x, acc[c].y);
      }
      wsync();
    };
    // vertical pass of block b: thread (j, q) -> output rows 8b + 2q, 8b + 2q + 1
    const int vj = tid & 127, vq = __builtin_amdgcn_readfirstlane(tid >> 7);  // wave-uniform
    const bool vcol = vj < mw;
    const int vjc = vcol ? vj : mw - 1;
    auto vblock = [&](int b) {
      const int i0 = RB * b + 2 * vq;
      const int base = (2 * i0) % kRing;  // slot of ext row 2 i0 - p
      // one pass over the L+2 ring rows feeds both output rows (row 1 starts two rows later);
      // per accumulator the fma order is tap 0..L-1, as in the wave-chunk form
      // packed FMAs: (a, h) += (flo, fhi) * lo and (v, d) += (flo, fhi) * hi
      f2 ah[2] = {f2{0.f, 0.f}, f2{0.f, 0.f}}, vd[2] = {f2{0.f, 0.f}, f2{0.f, 0.f}};
#pragma unroll
      for (int k = 0; k < L + 2; ++k) {
        int s = base + k;
        s = s >= kRing ? s - kRing : s;
        const float2 r = ring[s * mw + vjc];
        if (k < L) {
          ah[0] = __builtin_elementwise_fma(fh2[k], f2{r.x, r.x}, ah[0]);
          vd[0] = __builtin_elementwise_fma(fh2[k], f2{r.y, r.y}, vd[0]);
        }
        if (k >= 2) {
          ah[1] = __builtin_elementwise_fma(fh2[k - 2], f2{r.x, r.x}, ah[1]);
          vd[1] = __builtin_elementwise_fma(fh2[k - 2], f2{r.y, r.y}, vd[1]);
        }
      }
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        const float a = ah[h2].x, hh = ah[h2].y, v = vd[h2].x, d = vd[h2].y;
        const int i = i0 + h2;
        if (vcol && i < mh) {
          const int64_t idx = (int64_t)i * mw + vj;
          if (lastlvl) bo.put(g, g.off_a, bn, idx, a, mx[3]);
          else bufA[idx] = a;
          bo.put(g, g.off[0][0], bn, idx, hh, mx[0]);
          bo.put(g, g.off[0][1], bn, idx, v, mx[1]);
          bo.put(g, g.off[0][2], bn, idx, d, mx[2]);
        }
      }
    };

    // prologue: ext rows -p .. -1 (waves 0 .. p-1, one each) and the first D blocks in flight
    CRow fp;
    int spro;
    fetch(fp, spro, wv < p ? wv - p : -p);
    CRow F[D][2];
    int S[D][2];
#pragma unroll
    for (int u = 0; u < D; ++u) {
      fetch(F[u][0], S[u][0], 16 * u + 2 * wv);
      fetch(F[u][1], S[u][1], 16 * u + 2 * wv + 1);
    }
    if (wv < p) {
      float za[4] = {0.f, 0.f, 0.f, 0.f}, zb[4];
      noise2(za, zb, spro, spro);
      hrow(fp, spro, wv - p, za);
    }
    // the noise of block b + 1's rows is generated between the barrier and block b's vertical
    // pass: pure ALU work that overlaps the vertical pass's LDS reads (its rows are known: they
    // were fetched D - 1 blocks earlier)
    float Z[D][2][4];
#pragma unroll
    for (int u = 0; u < D; ++u)
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int k = 0; k < 4; ++k) Z[u][r][k] = 0.f;
    noise2(Z[0][0], Z[0][1], S[0][0], S[0][1]);
    for (int b0 = 0; b0 < nb; b0 += D) {
#pragma unroll
      for (int u = 0; u < D; ++u) {
        const int b = b0 + u;
        const int un = (u + 1) % D;  // static after unrolling
        if (b < nb) {  // workgroup-uniform
          hrow(F[u][0], S[u][0], 16 * b + 2 * wv, Z[u][0]);
          hrow(F[u][1], S[u][1], 16 * b + 2 * wv + 1, Z[u][1]);
        }
        // refill: block b + D (past the plane: clamped rows, never consumed)
        fetch(F[u][0], S[u][0], 16 * (b + D) + 2 * wv);
        fetch(F[u][1], S[u][1], 16 * (b + D) + 2 * wv + 1);
        if (b < nb) {
          __syncthreads();  // ring rows of block b complete
          if (b + 1 < nb) noise2(Z[un][0], Z[un][1], S[un][0], S[un][1]);
          vblock(b);
          __syncthreads();  // ring slots free for block b + 1
        }
      }
    }
    if constexpr (MAPS) {
#pragma unroll
      for (int b = 0; b < 4; ++b) mx[b] = wave_max(mx[b]);
      if (lane == 0) {
#pragma unroll
        for (int b = 0; b < 3; ++b) atomicMax(&wg_max[g.band[0][b]], __float_as_uint(mx[b]));
        if (lastlvl) atomicMax(&wg_max[0], __float_as_uint(mx[3]));
      }
    }
  } else {
    // Wave chunks: wave w owns output rows [i0, i1) and streams their 2R+L-2 ext rows. Lean
    // instruction stream (the kernel is VALU-issue bound, profiles/r01f_pmc.txt): the vertical
    // ring holds (lo, hi) pairs in ring slot t mod L and the loop is unrolled over lcm(L, NBL) rows so
    // every ring and fetch-buffer index is static (no register rotation); lo/hi and the (a, v) /
    // (h, d) output pairs are computed with packed fp32 FMAs in the scalar kernels' tap order.
    constexpr int NBL = (NCH > 1 || CPL > 1) ? 2 : 4;  // fetched rows in registers (NBL - 1 in flight)
    constexpr int GRPL = (L % NBL == 0) ? L : ((NBL % L == 0) ? NBL : L * NBL / 2);  // lcm(L, NBL)
    const int mh = g.mh[0], mw = g.mw[0];
    const int64_t bn = (int64_t)mh * mw;
    const bool lastlvl = g.J == 1;
    float* lds = bufB + wv * g.rowlds;
    const int mode = g.mode;
    const bool zero_mode = mode == WAM_MODE_ZERO;
    const PadLane pl = pad_lane(lane, nw, p, mode);
    if (zero_mode && pl.dst >= 0) lds[pl.dst] = 0.f;
    const int R = (mh + PW - 1) / PW;
    const int i0 = wv * R;
    const int i1 = min(mh, i0 + R);
    const int er0 = 2 * i0 - p;
    const int T = i1 > i0 ? 2 * (i1 - i0) + L - 2 : 0;
    // SHARE (noisy analysis): even waves stream their chunk bottom-up, odd waves top-down, so the
    // waves 2k and 2k + 1 both START at their common boundary b: each computes three of the L - 2
    // ext rows both need (2b-6 .. 2b-1 at L = 8) and takes the other three from its partner through
    // the LL_1 area of LDS (empty until the first emit), instead of both computing all six -- a
    // quarter of the halo rows (each row is fetched, noised and filtered once per wave that needs
    // it). Local step s runs 0 .. T-1 over the wave's ext rows in its own direction; ring slot s % L.
    constexpr bool SHARE = NOISE && MC == 0 && L >= 4 && NBL == 2;
    constexpr int HS = (L - 2) / 2;  // shared rows computed by each wave of a pair
    const bool up = SHARE && !(wv & 1);
    const int pw = wv ^ 1;  // partner
    // both waves of the pair have rows, and the LL_1 area (J > 1) holds the exchange
    const bool share = SHARE && T > 0 && pw * R < mh && g.llcap >= PW * HS * 2 * CPL * 64;
    // END boundaries (waves 2k-1 top-down | 2k bottom-up) meet at the end of both streams: each
    // computes the first HS of the L - 2 shared rows (its steps T-L+2 .. T-HS-1) and takes the rest
    // from its partner through buffer B (g.xend) after one workgroup barrier. Both waves need
    // >= L - 2 + 2*HS steps so that the START and END shared rows do not overlap.
    const int pe = (wv & 1) ? wv + 1 : wv - 1;
    const int pe_rows = (pe >= 0 && pe < PW) ? max(0, min(mh, (pe + 1) * R) - pe * R) : 0;
    const bool end_share = SHARE && g.xend >= 0 && T >= 2 * (L - 2) && 2 * pe_rows + L - 2 >= 2 * (L - 2);
    const int T_stop = end_share ? T - HS : T;  // the loop's last step + 1
    float mx[4] = {0.f, 0.f, 0.f, 0.f};
    // PAIRCOL: lane l owns columns 2l, 2l+1 (lanes past the row compute never-stored values from
    // the in-bounds tail of their LDS row); else columns l, l + 64
    constexpr bool PAIRCOL = CPL == 2 && !MAPS;
    auto colj = [&](int c) { return PAIRCOL ? 2 * lane + c : lane + 64 * c; };
    const float2* hsrc[CPL];
#pragma unroll
    for (int c = 0; c < CPL; ++c)
      hsrc[c] = reinterpret_cast<const float2*>(lds + kPadL + 2 * (PAIRCOL ? 2 * lane + c : min(colj(c), mw - 1)) - p);

    RowRegs<4, 1> f[NBL][NCH];
    int srow[NBL];
    auto fetch = [&](RowRegs<4, 1> (&fr)[NCH], int& sr_out, int t) {
      const int sr = row_src(up ? 2 * i1 - 1 - t : er0 + t, nh, mode);
      const bool valid = sr >= 0;
      const int rr = valid ? sr : 0;
      sr_out = sr;  // -1: zero row
#pragma unroll
      for (int c = 0; c < NCH; ++c) fr[c].fetch(src + c * in_plane + (int64_t)rr * nw, nw, lane, valid);
    };
    f2 rv[CPL][L];  // ring: (lo, hi) of ext row t in slot t % L
    // nzr: the row's noise from noise2 (rows are noised in pairs: ext rows t, t + 1 for even t)
    auto consume = [&](RowRegs<4, 1> (&fr)[NCH], int sr, int slot, const float (&nzr)[4]) {
      RowRegs<4, 1> m = fr[0];
      if constexpr (NCH > 1) {
#pragma unroll
        for (int c = 1; c < NCH; ++c)
#pragma unroll
          for (int u = 0; u < 4; ++u) m.v[u] += fr[c].v[u];
        constexpr float inv = 1.0f / (float)NCH;
#pragma unroll
        for (int u = 0; u < 4; ++u) m.v[u] *= inv;
      }
      if constexpr (NOISE) {
        // zero rows and the lanes past the row (their unguarded commit lands on the zero-mode pad
        // slots) stay zero: fma(0, z, 0)
        m.commit(lds, lane, nzr, (sr >= 0 && lane * 4 < nw) ? sg : 0.f);
      } else {
        m.commit(lds, lane, nullptr);
      }
      wsync();
      if (!zero_mode) {
        refresh_pads(lds, pl);
        wsync();
      }
      // the CPL columns' accumulation chains interleaved: back-to-back dependent packed FMAs
      // cost a hazard wait state each
      f2 acc[CPL];
#pragma unroll
      for (int c = 0; c < CPL; ++c) acc[c] = f2{0.f, 0.f};
      if constexpr (PAIRCOL) {
        // column 2l+1's taps start one pair after column 2l's: L/2 + 1 pairs feed both
        float2 xs[L / 2 + 1];
#pragma unroll
        for (int m2 = 0; m2 <= L / 2; ++m2) xs[m2] = hsrc[0][m2];
#pragma unroll
        for (int m2 = 0; m2 < L / 2; ++m2) {
#pragma unroll
          for (int c = 0; c < CPL; ++c) {
            const float2 x = xs[m2 + c];
            acc[c] = __builtin_elementwise_fma(fh2[2 * m2], f2{x.x, x.x}, acc[c]);
            acc[c] = __builtin_elementwise_fma(fh2[2 * m2 + 1], f2{x.y, x.y}, acc[c]);
          }
        }
      } else {
#pragma unroll
        for (int m2 = 0; m2 < L / 2; ++m2) {
#pragma unroll
          for (int c = 0; c < CPL; ++c) {
            const float2 x = hsrc[c][m2];
            acc[c] = __builtin_elementwise_fma(fh2[2 * m2], f2{x.x, x.x}, acc[c]);
            acc[c] = __builtin_elementwise_fma(fh2[2 * m2 + 1], f2{x.y, x.y}, acc[c]);
          }
        }
      }
#pragma unroll
      for (int c = 0; c < CPL; ++c) rv[c][slot] = acc[c];
      wsync();
    };
    // output row i from ring slots (s0 + k) % L, k = 0 .. L-1 (REV: bottom-up wave, tap k in slot
    // (s0 + L - 1 - k) % L); the fma chain is tap 0 .. L-1 either way
    auto emit_dir = [&](auto rev, int i, int s0) {
      f2 av[CPL], hd[CPL];
#pragma unroll
      for (int c = 0; c < CPL; ++c) av[c] = hd[c] = f2{0.f, 0.f};
#pragma unroll
      for (int k = 0; k < L; ++k) {
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
          const f2 r = rv[c][decltype(rev)::value ? (s0 + L - 1 - k) % L : (s0 + k) % L];
          av[c] = __builtin_elementwise_fma(f2{fh2[k].x, fh2[k].x}, r, av[c]);  // (a, v) = sum flo[k] * (lo, hi)
          hd[c] = __builtin_elementwise_fma(f2{fh2[k].y, fh2[k].y}, r, hd[c]);  // (h, d) = sum fhi[k] * (lo, hi)
        }
      }
      if constexpr (PAIRCOL) {
        const int j = 2 * lane;
        if (j < mw && i >= i0 && i < i1) {  // a partial last group: rows outside the chunk
          const bool pair = j + 1 < mw;
          const int64_t idx = (int64_t)i * mw + j;
          if (lastlvl) {
            bo.put2(g, g.off_a, bn, idx, av[0].x, av[1].x, pair, mx[3]);
          } else {
            bufA[idx] = av[0].x;
            if (pair) bufA[idx + 1] = av[1].x;
          }
          bo.put2(g, g.off[0][0], bn, idx, hd[0].x, hd[1].x, pair, mx[0]);
          bo.put2(g, g.off[0][1], bn, idx, av[0].y, av[1].y, pair, mx[1]);
          bo.put2(g, g.off[0][2], bn, idx, hd[0].y, hd[1].y, pair, mx[2]);
        }
      } else {
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
          const int j = lane + 64 * c;
          if (j < mw && i >= i0 && i < i1) {  // a partial last group: rows outside the chunk
            const int64_t idx = (int64_t)i * mw + j;
            if (lastlvl) bo.put(g, g.off_a, bn, idx, av[c].x, mx[3]);
            else bufA[idx] = av[c].x;
            bo.put(g, g.off[0][0], bn, idx, hd[c].x, mx[0]);
            bo.put(g, g.off[0][1], bn, idx, av[c].y, mx[1]);
            bo.put(g, g.off[0][2], bn, idx, hd[c].y, mx[2]);
          }
        }
      }
    };
    // after local step s = L-1 + 2m: output row i0 + m (top-down) or i1 - 1 - m (bottom-up)
    auto emit = [&](int m, int s0) {
      if (up) emit_dir(std::true_type{}, i1 - 1 - m, s0);
      else emit_dir(std::false_type{}, i0 + m, s0);
    };

    // Every fetch is unconditional (rows past the chunk are clamped to valid source rows and never
    // emitted): loads under divergent control flow would make the compiler drain vmcnt to 0 at the
    // join, serialising the row stream on memory latency.
    float za[4] = {0.f, 0.f, 0.f, 0.f}, zb[4] = {0.f, 0.f, 0.f, 0.f};
    if (T > 0) {
#pragma unroll
      for (int u = 0; u < NBL - 1; ++u) fetch(f[u], srow[u], u);
    }
    // prologue: ext rows 0 .. L-3 fill ring slots 0 .. L-3 (SHARE: rows HS .. L-3 come from the
    // partner between two workgroup barriers that every wave executes)
    auto prologue_step = [&](auto tc) {
      constexpr int t = decltype(tc)::value;
      fetch(f[(t + NBL - 1) % NBL], srow[(t + NBL - 1) % NBL], t + NBL - 1);
      if (!(t & 1)) noise2(za, zb, srow[t % NBL], srow[(t + 1) % NBL]);  // row t + 1 is fetched
      consume(f[t % NBL], srow[t % NBL], t, (t & 1) ? zb : za);
    };
    if constexpr (SHARE) {
      if (T > 0) {
        plane_static_for<0, HS - 1>([&](auto tc) { prologue_step(tc); });
        constexpr int t = HS - 1;  // last computed shared row
        if (share) {
          // no fetch of row HS: its slot takes row L-2, the first row after the exchange
          if (!(t & 1)) noise2(za, zb, srow[t % NBL], srow[t % NBL]);
          consume(f[t % NBL], srow[t % NBL], t, (t & 1) ? zb : za);
          fetch(f[(L - 2) % NBL], srow[(L - 2) % NBL], L - 2);
          float* xw = bufA + wv * (HS * 2 * CPL * 64);
#pragma unroll
          for (int s = 0; s < HS; ++s)
#pragma unroll
            for (int c = 0; c < CPL; ++c) {
              xw[((s * CPL + c) * 2) * 64 + lane] = rv[c][s].x;
              xw[((s * CPL + c) * 2 + 1) * 64 + lane] = rv[c][s].y;
            }
        } else {
          prologue_step(std::integral_constant<int, t>{});
        }
      }
      __syncthreads();  // the partners' shared rows are in LDS
      if (share) {
        // partner's step s is this wave's step L-3-s (the pair streams the rows in opposite orders)
        const float* xp = bufA + pw * (HS * 2 * CPL * 64);
#pragma unroll
        for (int s = 0; s < HS; ++s)
#pragma unroll
          for (int c = 0; c < CPL; ++c)
            rv[c][L - 3 - s] = f2{xp[((s * CPL + c) * 2) * 64 + lane], xp[((s * CPL + c) * 2 + 1) * 64 + lane]};
      }
      __syncthreads();  // every exchange read precedes the first LL_1 row written over the area
      if (T > 0 && !share) plane_static_for<HS, L - 2>([&](auto tc) { prologue_step(tc); });
    } else if (T > 0) {
      plane_static_for<0, L - 2>([&](auto tc) { prologue_step(tc); });
    }
    if (T > 0) {
      // steady state: GRPL ext rows per iteration; t = base + u with base = L-2 (mod GRPL), so
      // t % L and t % NBL are compile-time constants; a partial last group computes output rows
      // >= i1, which emit() drops
      for (int base = L - 2; base < T_stop; base += GRPL) {
#pragma unroll
        for (int u = 0; u < GRPL; ++u) {
          const int t = base + u;
          if constexpr (SHARE) {
            if (t >= T_stop) break;  // uniform: no garbage steps past the chunk
          }
          fetch(f[(L - 2 + u + NBL - 1) % NBL], srow[(L - 2 + u + NBL - 1) % NBL], t + NBL - 1);
          if (!(u & 1))  // t even (L - 2 and GRPL are even): rows t, t + 1 noised together
            noise2(za, zb, srow[(L - 2 + u) % NBL], srow[(L - 2 + u + 1) % NBL]);
          consume(f[(L - 2 + u) % NBL], srow[(L - 2 + u) % NBL], (L - 2 + u) % L, (u & 1) ? zb : za);
          // after odd u: output row (t - (L-1)) / 2 from ext rows t-L+1 .. t = slots (u-1+k) % L
          if (u & 1) emit((t - (L - 1)) / 2, (u - 1) % L);
        }
      }
    }
    if constexpr (SHARE) {
      // END exchange: this wave's rows of steps T-L+2 .. T-HS-1 out, its partner's (which are this
      // wave's steps T-1 .. T-HS, in the opposite order) in; then the last HS/2+... outputs. T % L
      // is even and fixes every ring slot: one static case per residue.
      constexpr int XR = HS * 2;  // floats per column of one direction (rows x (lo, hi))
      const int mw1 = g.mw[0];
      const int xb = (((wv & 1) ? (wv - 1) / 2 : (wv - 2) / 2) * 2) * XR * mw1;  // this boundary's block
      float* xme = bufB + g.xend + xb + (wv & 1) * XR * mw1;
      const float* xpe = bufB + g.xend + xb + (pe & 1) * XR * mw1;
      auto by_residue = [&](auto body) {
        plane_static_for<0, L / 2>([&](auto rc) {
          constexpr int R0 = 2 * decltype(rc)::value;
          if (T % L == R0) body(std::integral_constant<int, R0>{});
        });
      };
      if (end_share) {
        by_residue([&](auto rc) {
          constexpr int R0 = decltype(rc)::value;
#pragma unroll
          for (int k = 0; k < HS; ++k)
#pragma unroll
            for (int c = 0; c < CPL; ++c) {
              const int j = colj(c);
              if (j < mw1) {
                const f2 v = rv[c][(R0 + 2 * L - (L - 2) + k) % L];  // step T-(L-2)+k
                xme[(2 * k) * mw1 + j] = v.x;
                xme[(2 * k + 1) * mw1 + j] = v.y;
              }
            }
        });
      }
      __syncthreads();  // every END pair's rows are in buffer B
      if (end_share) {
        by_residue([&](auto rc) {
          constexpr int R0 = decltype(rc)::value;
          // received steps in stream order (T-HS .. T-1), each output emitted right after its last
          // step as in the loop -- a later step's row takes the ring slot an earlier output reads
#pragma unroll
          for (int k = HS - 1; k >= 0; --k) {  // partner's row k = this wave's step T-1-k
#pragma unroll
            for (int c = 0; c < CPL; ++c) {
              const int j = min(colj(c), mw1 - 1);  // lanes past the row: a duplicate, never stored
              rv[c][(R0 + 2 * L - 1 - k) % L] = f2{xpe[(2 * k) * mw1 + j], xpe[(2 * k + 1) * mw1 + j]};
            }
            if (k & 1) continue;  // step T-1-k is odd when k is even (T even)
            emit((T - 1 - k - (L - 1)) / 2, (R0 + 2 * L - 1 - k - (L - 1)) % L);
          }
        });
      }
    }
    if constexpr (MAPS) {
#pragma unroll
      for (int b = 0; b < 4; ++b) mx[b] = wave_max(mx[b]);
      if (lane == 0) {
#pragma unroll
        for (int b = 0; b < 3; ++b) atomicMax(&wg_max[g.band[0][b]], __float_as_uint(mx[b]));
        if (lastlvl) atomicMax(&wg_max[0], __float_as_uint(mx[3]));
      }
    }
  }

  // ================================================================ phase 2: levels 2..J in LDS
  const float* lsrc = bufA;
  float* ldst = bufB;
  for (int l = 1; l < g.J; ++l) {
    __syncthreads();  // LL_l complete in lsrc; the buffer ldst is free
    const int sh = g.mh[l - 1], sw = g.mw[l - 1], mh = g.mh[l], mw = g.mw[l];
    const int64_t bn = (int64_t)mh * mw;
    const bool lastlvl = l == g.J - 1;
    const int mode = g.mode;
    float mx[4] = {0.f, 0.f, 0.f, 0.f};
    // thread (rb, j): output column j, output rows [i0, i1) of row block rb; a block filters
    // 2R + L - 2 ext rows for R outputs, so blocks are kept >= L rows long where the level allows
    int nrb = 64 * PW / mw;  // mw <= kPT (geom_ok)
    if (nrb > max(1, mh / L)) nrb = max(1, mh / L);
    const int rb = tid / mw, j = tid - rb * mw;
    if (rb < nrb) {
      const int R2 = (mh + nrb - 1) / nrb;
      const int i0 = rb * R2;
      const int i1 = min(mh, i0 + R2);
      if (i0 < i1) {
        // ext column 2j - p + k of the level: a zero-mode tap outside the row gets a zero filter
        // pair and a clamped address (fma(0, x, acc) = acc: the sums of the skipped taps)
        int cofs[L];
        f2 fk[L];
#pragma unroll
        for (int k = 0; k < L; ++k) {
          const int c = wam_ext_index(2 * j - p + k, sw, mode);
          cofs[k] = c >= 0 ? c : 0;
          fk[k] = c >= 0 ? fh2[k] : f2{0.f, 0.f};
        }
        const int er0 = 2 * i0 - p;
        // (lo, hi) of ext row t of this block, packed FMAs in tap order (zero-mode rows outside
        // the level: (0, 0))
        auto hrow = [&](int t) {
          const int sr = row_src(er0 + t, sh, mode);
          f2 acc = f2{0.f, 0.f};
          if (sr >= 0) {
            const float* s = lsrc + sr * sw;
#pragma unroll
            for (int k = 0; k < L; ++k) {
              const float x = s[cofs[k]];
              acc = __builtin_elementwise_fma(fk[k], f2{x, x}, acc);
            }
          }
          return acc;
        };
        // ring: ext row t in slot t % L; output row i0 + ii reads ext rows 2ii .. 2ii + L - 1,
        // i.e. slots (2u + k) % L for ii = ib + u with ib a multiple of L / 2 (static indices)
        f2 r[L];
#pragma unroll
        for (int t = 0; t < L - 2; ++t) r[t] = hrow(t);
        for (int ib = 0; i0 + ib < i1; ib += L / 2) {
#pragma unroll
          for (int u = 0; u < L / 2; ++u) {
            const int ii = ib + u;
            const int i = i0 + ii;
            if (i < i1) {
              r[(2 * u + L - 2) % L] = hrow(2 * ii + L - 2);
              r[(2 * u + L - 1) % L] = hrow(2 * ii + L - 1);
              // (a, h) = sum (flo, fhi)[k] * lo_k, (v, d) = sum (flo, fhi)[k] * hi_k in tap order
              f2 ah = f2{0.f, 0.f}, vd = f2{0.f, 0.f};
#pragma unroll
              for (int k = 0; k < L; ++k) {
                const f2 q = r[(2 * u + k) % L];
                ah = __builtin_elementwise_fma(fh2[k], f2{q.x, q.x}, ah);
                vd = __builtin_elementwise_fma(fh2[k], f2{q.y, q.y}, vd);
              }
              const int64_t idx = (int64_t)i * mw + j;
              if (lastlvl) bo.put(g, g.off_a, bn, idx, ah.x, mx[3]);
              else ldst[idx] = ah.x;
              bo.put(g, g.off[l][0], bn, idx, ah.y, mx[0]);
              bo.put(g, g.off[l][1], bn, idx, vd.x, mx[1]);
              bo.put(g, g.off[l][2], bn, idx, vd.y, mx[2]);
            }
          }
        }
      }
    }
    if constexpr (MAPS) {
#pragma unroll
      for (int b = 0; b < 4; ++b) mx[b] = wave_max(mx[b]);
      if (lane == 0) {
#pragma unroll
        for (int b = 0; b < 3; ++b) atomicMax(&wg_max[g.band[l][b]], __float_as_uint(mx[b]));
        if (lastlvl) atomicMax(&wg_max[0], __float_as_uint(mx[3]));
      }
    }
    const float* t_ = lsrc;
    lsrc = ldst;
    ldst = const_cast<float*>(t_);
  }
  if constexpr (MAPS) {
    __syncthreads();
    if (tid < g.nbands) {
      const unsigned int m = wg_max[tid];
      if (m) atomicMax(reinterpret_cast<unsigned int*>(band_max) + (item / group_items) * g.nbands + tid, m);
    }
  }
}

// ================================================================================================
// Plane-resident multi-level synthesis (waverec2 with the IG alpha fused): one workgroup per
// (plane, alpha); the reconstructed approximations LL'_J-1 .. LL'_1 stay in LDS, every level is a
// streaming pass of the waves over coefficient rows (the per-lane vertical ring / LDS exchange
// scheme of k_dwt2_syn, same arithmetic order), coefficient rows are prefetched kSynPF rows ahead
// with clamped, unconditional loads; only level 0 writes to HBM.
constexpr int kMaxAlpha = 128;

struct SynGeom {
  int J;
  int mh[WAM_MAX_LEVELS], mw[WAM_MAX_LEVELS];  // coefficient dims of level l (0 = finest)
  int oh[WAM_MAX_LEVELS], ow[WAM_MAX_LEVELS];  // output dims of level l (l >= 1: LL'_l = lout[l-1])
  int64_t off_a;
  int64_t off[WAM_MAX_LEVELS][3];
  int64_t batch;     // items in the band-major coefficient buffer
  int lcap, scap;    // floats of LDS buffers L (odd levels' outputs) and S (even levels' outputs)
  int n_alpha;       // alphas in this launch
  int64_t out_base;  // output item offset of alpha 0 of this launch
};

struct SynAlphas {
  float v[kMaxAlpha];
};

// the waves of the workgroup split a level into strips x row chunks
template <int L>
__device__ __forceinline__ bool syn_work(int oh, int ow, int wv, int& strip, int& qbeg, int& qend) {
  constexpr int p = L - 2;
  constexpr int OUTQ = 65 - L / 2;
  const int qs = p >> 1;
  const int nstrips = ((ow + 1) / 2 + OUTQ - 1) / OUTQ;
  const int chunks = kPW / nstrips;
  strip = wv % nstrips;
  const int chunk = wv / nstrips;
  const int qlast = (p + oh - 1) >> 1;
  const int nq = qlast - qs + 1;
  const int RQ = (nq + chunks - 1) / chunks;
  qbeg = qs + chunk * RQ;
  qend = min(qbeg + RQ, qlast + 1);
  return chunk < chunks && qbeg < qend;
}

// OC: output format of level 0: 0 = fp32 planes [items, oh, ow]; C = 1 or 3: bf16 images in NHWC
// order [items / C, oh, ow, C] (item = image * C + channel; the explained model's own input dtype and
// layout, rounded as torch's fp32 -> bf16 cast rounds)
template <int L, int OC = 0>
__global__ void __launch_bounds__(kPT) __attribute__((amdgpu_waves_per_eu(4, 8)))
    k_plane_syn(const float* __restrict__ coeffs, void* __restrict__ out_v, const float* __restrict__ filt, SynGeom g,
                SynAlphas al, int64_t n_items) {
  float* out = static_cast<float*>(out_v);
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int64_t nwg = gridDim.x, bid = blockIdx.x;
  const int64_t q8 = nwg / 8, r8 = nwg % 8, xcd = bid % 8;
  const int64_t lwg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  if (lwg >= n_items) return;  // never taken (grid == n_items)
  const int tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  // alpha-fastest: the alphas of one plane share an XCD and its coefficient reads
  const int64_t item = lwg / g.n_alpha;
  const int ai = (int)(lwg % g.n_alpha);
  const float s = al.v[ai];
  float rlo[L], rhi[L];
#pragma unroll
  for (int k = 0; k < L; ++k) {
    rlo[k] = filt[k];
    rhi[k] = filt[L + k];
  }
  float* bufL = smem;
  float* bufS = smem + g.lcap;
  float4* xch = reinterpret_cast<float4*>(smem + g.lcap + g.scap) + wv * 64;
  for (int l = g.J - 1; l >= 0; --l) {
    if (l < g.J - 1) __syncthreads();  // LL'_{l+1} complete
    const int mh = g.mh[l], mw = g.mw[l], oh = g.oh[l], ow = g.ow[l];
    const int64_t bn = (int64_t)mh * mw;
    const float* pH = coeffs + g.batch * g.off[l][0] + item * bn;
    const float* pV = coeffs + g.batch * g.off[l][1] + item * bn;
    const float* pD = coeffs + g.batch * g.off[l][2] + item * bn;
    int strip, qbeg, qend;
    if (!syn_work<L>(oh, ow, wv, strip, qbeg, qend)) continue;
    const bool coarsest = l == g.J - 1;
    if (l == 0) {
      const int64_t oi = g.out_base + (int64_t)ai * g.batch + item;
      if constexpr (OC == 0) {
        float* dst = out + oi * ((int64_t)oh * ow);
        if (coarsest)
          syn_stream<L>(coeffs + g.batch * g.off_a + item * bn, s, pH, pV, pD, s, mh, mw, dst, oh, ow, strip, qbeg,
                        qend, xch, rlo, rhi, lane);
        else
          syn_stream<L>(bufL, 1.f, pH, pV, pD, s, mh, mw, dst, oh, ow, strip, qbeg, qend, xch, rlo, rhi, lane);
      } else {
        const SynOutBf16<OC> dst{static_cast<uint16_t*>(out_v) + (oi / OC) * ((int64_t)oh * ow * OC) + oi % OC};
        if (coarsest)
          syn_stream_to<L>(coeffs + g.batch * g.off_a + item * bn, s, pH, pV, pD, s, mh, mw, dst, oh, ow, strip,
                           qbeg, qend, xch, rlo, rhi, lane);
        else
          syn_stream_to<L>(bufL, 1.f, pH, pV, pD, s, mh, mw, dst, oh, ow, strip, qbeg, qend, xch, rlo, rhi, lane);
      }
    } else {
      float* dst = (l & 1) ? bufL : bufS;
      if (coarsest)
        syn_stream<L>(coeffs + g.batch * g.off_a + item * bn, s, pH, pV, pD, s, mh, mw, dst, oh, ow, strip, qbeg,
                      qend, xch, rlo, rhi, lane);
      else
        syn_stream<L>((l & 1) ? bufS : bufL, 1.f, pH, pV, pD, s, mh, mw, dst, oh, ow, strip, qbeg, qend, xch, rlo,
                      rhi, lane);
    }
  }
}

// ------------------------------------------------------------------------------------------------
// filters up to 8 taps (haar, db2-db4, sym2-sym4, coif1): longer filters keep the per-level kernels,
// whose register ring of L rows x 2 columns x lo/hi does not fit the 128-VGPR budget of 16 waves/CU
bool l_ok(int L) { return L == 2 || L == 4 || L == 6 || L == 8; }

// cooperative level 1 (COOP): wave rows with 8 left pad slots + a ring of 2*8+L-2 (lo, hi) rows;
// chosen when two workgroups still fit a CU (the ring replaces the wave-chunk halo re-fetch)
constexpr int kCoopPadL = 8;
constexpr int kTwoWgLds = 160 * 1024 / 2 - 4 * WAM_MAX_BANDS - 64;  // minus the static wg_max table

int coop_lds_floats(const wam_plan* p, int nw0, int& rowlds, int& llcap) {
  rowlds = (kCoopPadL + nw0 + p->pad + (nw0 & 1) + 1 + 3) & ~3;
  llcap = p->levels > 1 ? (int)((p->lout[0][0] * p->lout[0][1] + 63) & ~63) : 0;
  int64_t bcap = (int64_t)kPW * rowlds + 2 * (16 + p->L - 2) * p->lout[0][1];
  if (p->levels > 1) {
    const int64_t ll2 = p->lout[1][0] * p->lout[1][1];
    if (ll2 > bcap) bcap = ll2;
  }
  return (int)(llcap + bcap);
}

// The noisy analysis defaults to the wave-chunk form: it re-noises the L-2 halo rows of each
// wave's chunk but runs without the two workgroup barriers per 8 output rows, 8-10 % faster at the
// c2 shape (profiles/r02f_plane_ab.log); the clean analysis and the maps pass keep COOP.
bool coop_ok(const wam_plan* p, int nw0, bool noisy = false) {
  if (p->flags & WAM_PLAN_NO_COOP) return false;
  if (noisy && !(p->flags & WAM_PLAN_FORCE_COOP)) return false;
  if (p->lout[0][1] > 128 || p->pad > kCoopPadL) return false;
  int rowlds, llcap;
  return (int64_t)coop_lds_floats(p, nw0, rowlds, llcap) * 4 <= kTwoWgLds || (p->flags & WAM_PLAN_FORCE_COOP);
}

int lds_floats(const wam_plan* p, int nw0, int& rowlds, int& llcap, bool noisy = false, int* xend = nullptr,
               int pw = kPW) {
  if (coop_ok(p, nw0, noisy)) return coop_lds_floats(p, nw0, rowlds, llcap);
  rowlds = kPadL + 256 + 8;  // commit covers 256 samples; pads <= p + 2 <= 20 fit behind them
  if (rowlds < kPadL + nw0 + p->pad + 4) rowlds = kPadL + nw0 + p->pad + 4;
  rowlds = (rowlds + 3) & ~3;
  // buffer B (the wave rows, read and written with 16-byte ds ops) must start 16-byte aligned: a
  // misaligned b128/b64 LDS access is split by the hardware and made this kernel 3x slower
  llcap = p->levels > 1 ? (int)((p->lout[0][0] * p->lout[0][1] + 63) & ~63) : 0;
  int64_t bcap = (int64_t)pw * rowlds;
  int64_t ll2 = 0;
  if (p->levels > 1) {
    ll2 = p->lout[1][0] * p->lout[1][1];
    if (ll2 > bcap) bcap = ll2;
  }
  if (xend) *xend = -1;
  if (noisy) {
    // the END-boundary exchange behind the wave rows: (kPW/2 - 1) boundaries x 2 directions x
    // (L-2)/2 rows x (lo, hi) x mw floats, if two workgroups still fit a CU
    const int64_t xe = (int64_t)(pw / 2 - 1) * 2 * (p->L - 2) * p->lout[0][1];
    const int64_t b2 = std::max<int64_t>((int64_t)pw * rowlds + xe, ll2);
    if ((llcap + b2) * 4 + 4 * WAM_MAX_BANDS + 64 <= 160 * 1024 / 2) {
      if (xend) *xend = pw * rowlds;
      bcap = b2;
    }
  }
  return (int)(llcap + bcap);
}

bool geom_ok(const wam_plan* p, int nw0, int nh0) {
  if (p->ndim != 2 || !l_ok(p->L) || p->levels < 1 || p->levels > WAM_MAX_LEVELS) return false;
  if (nw0 % 4 || nw0 > kPlaneMaxW || nw0 < 4 || nh0 < 1) return false;
  if (p->lout[0][1] > kPlaneMaxMW) return false;
  for (int l = 1; l < p->levels; ++l)
    if (p->lout[l][1] > kPT) return false;
  int rowlds, llcap;
  return (int64_t)lds_floats(p, nw0, rowlds, llcap) * 4 <= kPlaneLdsCap;
}

PlaneGeom make_geom(const wam_plan* p, int nh0, int nw0, int mode, int64_t items_total, bool noisy = false,
                    int pw = kPW) {
  PlaneGeom g{};
  g.J = p->levels;
  g.mode = mode;
  g.nh0 = nh0;
  g.nw0 = nw0;
  for (int l = 0; l < p->levels; ++l) {
    g.mh[l] = (int)p->lout[l][0];
    g.mw[l] = (int)p->lout[l][1];
    for (int s = 0; s < 3; ++s) {
      g.band[l][s] = wam_band_of(p, l, s);
      g.off[l][s] = p->band_off[g.band[l][s]];
    }
  }
  g.off_a = p->band_off[0];
  g.nbands = p->nbands;
  g.items_total = items_total;
  g.maps_item = p->band_off[p->nbands];
  lds_floats(p, nw0, g.rowlds, g.llcap, noisy, &g.xend, pw);
  g.coop = coop_ok(p, nw0, noisy);
  // noisy analysis: sample-fastest through the XCD swizzle (the S samples of a plane read it from
  // one L2; plane-fastest and un-swizzled orders measured 684 / 681 vs 666 us,
  // profiles/r03e_plane_order_ab.log)
  g.sample_fast = 1;
  g.xcd_order = 1;
  return g;
}

template <int L, int CPL, bool NOISE, int MC, bool MAPS, bool COOP, int IN = kInF32, int PW = kPW>
int launch_plane_t(const PlaneGeom& g, int lds_bytes, int64_t n_items, const float* in, float* out, float* band_max,
                   const float* filt, const WamNoise& nz, int64_t S, int64_t group_items, const char* name,
                   double bytes, hipStream_t st) {
  auto kern = k_plane_ana<L, CPL, NOISE, MC, MAPS, COOP, IN, PW>;
  static std::atomic<uint64_t> attr_set{0};  // opt in to > 64 KB of dynamic LDS, once per device
  int dev = 0;
  WAM_HIP_CHECK(hipGetDevice(&dev));
  const uint64_t bit = 1ull << (dev & 63);
  if (!(attr_set.load(std::memory_order_relaxed) & bit)) {
    WAM_HIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      kPlaneLdsCap));
    attr_set.fetch_or(bit);
  }
  WamTimer tm(st, name, bytes);
  hipLaunchKernelGGL(kern, dim3((unsigned)n_items), dim3(64 * PW), lds_bytes, st, in, out, band_max, filt, g, nz, n_items,
                     S, group_items);
  WAM_LAUNCH_CHECK();
  return WAM_OK;
}

template <bool NOISE, int MC, bool MAPS>
int dispatch_plane(const wam_plan* p, const PlaneGeom& g, int lds_bytes, int64_t n_items, const float* in,
                   float* out, float* band_max, const float* filt, const WamNoise& nz, int64_t S,
                   int64_t group_items, const char* name, double bytes, hipStream_t st) {
  const bool two = g.mw[0] > 64;
#define WAM_PLANE_ARGS g, lds_bytes, n_items, in, out, band_max, filt, nz, S, group_items, name, bytes, st
#define WAM_PLANE_CASE(LL)                                                                                       \
  case LL:                                                                                                       \
    if (g.coop)                                                                                                  \
      return two ? launch_plane_t<LL, 2, NOISE, MC, MAPS, true>(WAM_PLANE_ARGS)                                  \
                 : launch_plane_t<LL, 1, NOISE, MC, MAPS, true>(WAM_PLANE_ARGS);                                 \
    return two ? launch_plane_t<LL, 2, NOISE, MC, MAPS, false>(WAM_PLANE_ARGS)                                   \
               : launch_plane_t<LL, 1, NOISE, MC, MAPS, false>(WAM_PLANE_ARGS);
  switch (p->L) {
    WAM_PLANE_CASE(2) WAM_PLANE_CASE(4) WAM_PLANE_CASE(6) WAM_PLANE_CASE(8)
    default: return WAM_ERR_UNSUPPORTED;
  }
#undef WAM_PLANE_CASE
#undef WAM_PLANE_ARGS
}

// the maps pass over bf16 input gradients (COOP level 1 only)
template <int MC, int IN>
int dispatch_maps_bf16(const wam_plan* p, const PlaneGeom& g, int lds_bytes, int64_t n_items, const float* in,
                       float* out, float* band_max, const float* filt, int64_t group_items, double bytes,
                       hipStream_t st) {
  if (!g.coop) return WAM_ERR_UNSUPPORTED;
  const WamNoise nz{nullptr, 1, 1, 0, 0, 0, 0};
  const bool two = g.mw[0] > 64;
  const char* name = IN == kInBf16Nhwc ? "k_plane_maps<bf16nhwc>" : "k_plane_maps<bf16>";
#define WAM_MAPS_CASE(LL)                                                                                          \
  case LL:                                                                                                         \
    return two ? launch_plane_t<LL, 2, false, MC, true, true, IN>(g, lds_bytes, n_items, in, out, band_max, filt,  \
                                                                   nz, 1, group_items, name, bytes, st)             \
               : launch_plane_t<LL, 1, false, MC, true, true, IN>(g, lds_bytes, n_items, in, out, band_max, filt,  \
                                                                   nz, 1, group_items, name, bytes, st);
  switch (p->L) {
    WAM_MAPS_CASE(2) WAM_MAPS_CASE(4) WAM_MAPS_CASE(6) WAM_MAPS_CASE(8)
    default: return WAM_ERR_UNSUPPORTED;
  }
#undef WAM_MAPS_CASE
}

}  // namespace

bool dwt2_plane_maps_coop(const wam_plan* p) {
  return dwt2_plane_supported(p, true) && coop_ok(p, (int)p->rec_shape[1]);
}

bool dwt2_plane_supported(const wam_plan* p, bool adjoint) {
  const int nh0 = (int)(adjoint ? p->rec_shape[0] : p->lin[0][0]);
  const int nw0 = (int)(adjoint ? p->rec_shape[1] : p->lin[0][1]);
  return geom_ok(p, nw0, nh0);
}

int launch_dwt2_plane_analysis(const wam_plan* p, int64_t items, const float* in, float* coeffs, bool adjoint,
                               const WamNoise* nz, int64_t n_samples, hipStream_t st) {
  if (((uintptr_t)in & 15) || !dwt2_plane_supported(p, adjoint)) return WAM_ERR_UNSUPPORTED;
  const int nh0 = (int)(adjoint ? p->rec_shape[0] : p->lin[0][0]);
  const int nw0 = (int)(adjoint ? p->rec_shape[1] : p->lin[0][1]);
  const int mode = adjoint ? WAM_MODE_ZERO : p->mode;
  const float* filt = p->d_filt + (adjoint ? WAM_F_ADJ_LO : WAM_F_ANA_LO) * p->L;
  const PlaneGeom g = make_geom(p, nh0, nw0, mode, items, nz != nullptr);
  int rowlds, llcap;
  const int lds_bytes = lds_floats(p, nw0, rowlds, llcap, nz != nullptr) * 4;
  const double in_planes = nz ? (double)nz->images * nz->channels : (double)items;
  const double bytes = 4.0 * (in_planes * nh0 * nw0 + (double)items * p->band_off[p->nbands]);
  if (nz) {
    if (items != n_samples * nz->images * nz->channels) return WAM_ERR_INVALID_ARG;
    // the fused noise counts element groups of an image in 32 bits (wam_normal4_x2)
    if ((int64_t)nz->channels * nh0 * nw0 >= (int64_t(1) << 34)) return WAM_ERR_UNSUPPORTED;
    return dispatch_plane<true, 0, false>(p, g, lds_bytes, items, in, coeffs, nullptr, filt, *nz, n_samples, 1,
                                          "k_plane_ana<noise>", bytes, st);
  }
  const WamNoise none{nullptr, 1, 1, 0, 0, 0, 0};
  return dispatch_plane<false, 0, false>(p, g, lds_bytes, items, in, coeffs, nullptr, filt, none, 1, 1,
                                         "k_plane_ana", bytes, st);
}

int launch_dwt2_plane_maps(const wam_plan* p, int64_t images, int channels, int64_t group_items, const void* grad_v,
                           int in_fmt, float* maps, float* band_max, hipStream_t st) {
  const float* grad = static_cast<const float*>(grad_v);
  if (((uintptr_t)grad & 15) || !dwt2_plane_supported(p, true)) return WAM_ERR_UNSUPPORTED;
  if (channels != 1 && channels != 3) return WAM_ERR_UNSUPPORTED;
  const int nh0 = (int)p->rec_shape[0], nw0 = (int)p->rec_shape[1];
  const float* filt = p->d_filt + WAM_F_ADJ_LO * p->L;
  PlaneGeom g = make_geom(p, nh0, nw0, WAM_MODE_ZERO, images);
  int rowlds, llcap;
  const int lds_bytes = lds_floats(p, nw0, rowlds, llcap) * 4;
  const WamNoise none{nullptr, 1, 1, 0, 0, 0, 0};
  const double bytes = (double)images * ((in_fmt ? 2.0 : 4.0) * channels * nh0 * nw0 +
                                          4.0 * (double)p->band_off[p->nbands]);
  if (in_fmt == kInBf16Nhwc && channels == 3)
    return dispatch_maps_bf16<3, kInBf16Nhwc>(p, g, lds_bytes, images, grad, maps, band_max, filt, group_items, bytes, st);
  if (in_fmt == kInBf16Nchw && channels == 3)
    return dispatch_maps_bf16<3, kInBf16Nchw>(p, g, lds_bytes, images, grad, maps, band_max, filt, group_items, bytes, st);
  if (in_fmt != kInF32)  // one channel: the two bf16 layouts coincide
    return dispatch_maps_bf16<1, kInBf16Nchw>(p, g, lds_bytes, images, grad, maps, band_max, filt, group_items, bytes, st);
  if (channels == 3)
    return dispatch_plane<false, 3, true>(p, g, lds_bytes, images, grad, maps, band_max, filt, none, 1, group_items,
                                          "k_plane_maps", bytes, st);
  return dispatch_plane<false, 1, true>(p, g, lds_bytes, images, grad, maps, band_max, filt, none, 1, group_items,
                                        "k_plane_maps", bytes, st);
}

// ------------------------------------------------------------------------------------------------ synthesis host
namespace {

int syn_lds_floats(const wam_plan* p, int& lcap, int& scap) {
  lcap = p->levels > 1 ? (int)((p->lout[0][0] * p->lout[0][1] + 63) & ~63) : 0;
  scap = p->levels > 2 ? (int)((p->lout[1][0] * p->lout[1][1] + 63) & ~63) : 0;
  return lcap + scap + kPW * 64 * 4;
}

bool syn_ok(const wam_plan* p) {
  if (p->ndim != 2 || !l_ok(p->L) || p->levels < 1 || p->levels > WAM_MAX_LEVELS) return false;
  if (p->rec_shape[0] * p->rec_shape[1] >= (int64_t(1) << 30)) return false;  // 32-bit byte offsets (at32)
  const int outq = 65 - p->L / 2;
  for (int l = 0; l < p->levels; ++l) {
    const int64_t ow = l ? p->lout[l - 1][1] : p->rec_shape[1];
    if (((ow + 1) / 2 + outq - 1) / outq > kPW) return false;
  }
  int lcap, scap;
  return (int64_t)syn_lds_floats(p, lcap, scap) * 4 <= kPlaneLdsCap;
}

template <int L, int OC>
int launch_syn_plane_t(const SynGeom& g, int lds_bytes, int64_t n_items, const float* coeffs, void* out,
                       const float* filt, const SynAlphas& al, double bytes, hipStream_t st) {
  auto kern = k_plane_syn<L, OC>;
  static std::atomic<uint64_t> attr_set{0};
  int dev = 0;
  WAM_HIP_CHECK(hipGetDevice(&dev));
  const uint64_t bit = 1ull << (dev & 63);
  if (!(attr_set.load(std::memory_order_relaxed) & bit)) {
    WAM_HIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      kPlaneLdsCap));
    attr_set.fetch_or(bit);
  }
  WamTimer tm(st, OC ? "k_plane_syn<bf16nhwc>" : "k_plane_syn", bytes);
  hipLaunchKernelGGL(kern, dim3((unsigned)n_items), dim3(kPT), lds_bytes, st, coeffs, out, filt, g, al, n_items);
  WAM_LAUNCH_CHECK();
  return WAM_OK;
}

template <int OC>
int syn_plane_l(int L, const SynGeom& g, int lds_bytes, int64_t n_items, const float* coeffs, void* out,
                const float* filt, const SynAlphas& al, double bytes, hipStream_t st) {
  switch (L) {
    case 2: return launch_syn_plane_t<2, OC>(g, lds_bytes, n_items, coeffs, out, filt, al, bytes, st);
    case 4: return launch_syn_plane_t<4, OC>(g, lds_bytes, n_items, coeffs, out, filt, al, bytes, st);
    case 6: return launch_syn_plane_t<6, OC>(g, lds_bytes, n_items, coeffs, out, filt, al, bytes, st);
    case 8: return launch_syn_plane_t<8, OC>(g, lds_bytes, n_items, coeffs, out, filt, al, bytes, st);
    default: return WAM_ERR_UNSUPPORTED;
  }
}

}  // namespace

bool dwt2_plane_syn_supported(const wam_plan* p) { return syn_ok(p); }

int launch_dwt2_plane_synthesis(const wam_plan* p, int64_t batch, const float* coeffs, const float* alpha,
                                int n_alpha, void* out, int out_channels, hipStream_t st) {
  if (!syn_ok(p)) return WAM_ERR_UNSUPPORTED;
  if (out_channels != 0 && (out_channels != 1 && out_channels != 3)) return WAM_ERR_UNSUPPORTED;
  if (out_channels && batch % out_channels) return WAM_ERR_INVALID_ARG;
  SynGeom g{};
  g.J = p->levels;
  for (int l = 0; l < p->levels; ++l) {
    g.mh[l] = (int)p->lout[l][0];
    g.mw[l] = (int)p->lout[l][1];
    g.oh[l] = (int)(l ? p->lout[l - 1][0] : p->rec_shape[0]);
    g.ow[l] = (int)(l ? p->lout[l - 1][1] : p->rec_shape[1]);
    for (int k = 0; k < 3; ++k) g.off[l][k] = p->band_off[wam_band_of(p, l, k)];
  }
  g.off_a = p->band_off[0];
  g.batch = batch;
  const int lds_bytes = syn_lds_floats(p, g.lcap, g.scap) * 4;
  const float* filt = p->d_filt + WAM_F_SYN_LO * p->L;
  const double out_item = (double)p->rec_shape[0] * p->rec_shape[1];
  for (int a0 = 0; a0 < n_alpha; a0 += kMaxAlpha) {
    const int na = n_alpha - a0 < kMaxAlpha ? n_alpha - a0 : kMaxAlpha;
    SynAlphas al{};
    for (int i = 0; i < na; ++i) al.v[i] = alpha ? alpha[a0 + i] : 1.0f;
    g.n_alpha = na;
    g.out_base = (int64_t)a0 * batch;
    // algorithmic bytes: the coefficients once, every reconstruction once (2 B per bf16 pixel)
    const double bytes = 4.0 * (double)batch * p->band_off[p->nbands] +
                         (out_channels ? 2.0 : 4.0) * (double)na * batch * out_item;
    const int64_t ni = batch * na;
    const int rc = out_channels == 3   ? syn_plane_l<3>(p->L, g, lds_bytes, ni, coeffs, out, filt, al, bytes, st)
                   : out_channels == 1 ? syn_plane_l<1>(p->L, g, lds_bytes, ni, coeffs, out, filt, al, bytes, st)
                                       : syn_plane_l<0>(p->L, g, lds_bytes, ni, coeffs, out, filt, al, bytes, st);
    if (rc) return rc;
  }
  return WAM_OK;
}

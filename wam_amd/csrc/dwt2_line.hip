// Line-streaming multi-level 2D analysis for gfx950: ONE wave per plane, all J levels streamed top
// to bottom in a single pass (the line-based wavelet transform), no workgroup barrier anywhere.
//
// Why: the plane-resident kernel (dwt2_plane.hip) pins LL_1 (53 KB at 224^2) in
// LDS and splits level 1 over 8 waves. That fixes it at 4 waves per SIMD, re-noises the L-2 halo
// rows of every wave's chunk (21 % of the rows at 224^2) and leaves 5-6 of its 8 waves idle in
// levels 2..J. Here a wave owns a whole plane:
//   level 1  the ext rows -p .. 2*mh-1 stream through a wave-private LDS row (16-byte fetches, one
//            row in flight, SmoothGrad noise added at the commit: Philox4x32-10, the stream of
//            wam_noise_add), horizontal pass from LDS, vertical pass from a static register ring of
//            the last L (lo, hi) rows. Every source row is fetched and noised once; only the
//            boundary ext rows (-p .. -1 and past the bottom) are re-fetched.
//   levels   each emitted LL row goes to a small LDS row buffer and is pushed into the next level at
//   2..J     once: horizontal pass into an LDS ring of 8 (lo, hi) rows indexed by SOURCE row, and a
//            level's output row i is emitted as soon as every source row its taps read (through the
//            boundary rule) has arrived. LL_l is never stored whole.
// Per wave: 32 ring VGPRs for level 1, ~7 KB of LDS at c2 (one row slot, one LL row, the level
// rings), so five waves per SIMD hold the 4,800 planes of a c2 call at once.
//
// Arithmetic order per output is the plane/row kernels' (taps 0..L-1 as one fma chain from +0,
// horizontal then vertical), so the results are bit-identical to k_plane_ana / k_dwt2_ana and, with
// the noise, to wam_noise_add followed by wam_wavedec (tests/test_gpu_dwt.py).
#include <atomic>

#include "rowtools.hpp"

namespace {

using namespace wam_rows;

constexpr int kLW = 4;         // waves (planes) per workgroup
constexpr int kLPad = 8;       // left pad slots of an LDS row (>= p for L <= 8; 16-byte aligned body)
constexpr int kRing = 8;       // (lo, hi) rows per ring of the levels >= 2 (>= L, power of two)
constexpr int kLineMaxJ = 3;
constexpr int kLQ = 2;         // LL_1 rows queued between pushes into level 2
#ifndef WAM_LINE_NX
#define WAM_LINE_NX 1
#endif
constexpr int NX = WAM_LINE_NX;  // Philox chains per noise call (1: per row, 2: row pairs interleaved)
// scheduling fences between the phases of a row (noise, commit + horizontal, vertical emit): left
// free, the machine scheduler interleaves neighbouring rows' phases and the live ranges overflow
// the 96-VGPR budget of five waves per SIMD
#ifndef WAM_LINE_NOSCHED
#define WAM_LINE_SCHED() __builtin_amdgcn_sched_barrier(0)
#else
#define WAM_LINE_SCHED()
#endif
#ifndef WAM_LINE_WAVES
#define WAM_LINE_WAVES 4
#endif
constexpr int kLineLdsCap = 160 * 1024 / 5 / kLW * kLW;  // bytes per workgroup that keep 5 waves per SIMD

struct LineGeom {
  int J;
  int mode;
  int nh0, nw0;
  int mh[kLineMaxJ], mw[kLineMaxJ];
  int64_t off_a;                   // per-item offset of A_J
  int64_t off[kLineMaxJ][3];       // per-item offsets of (H, V, D) of level l (0 = finest)
  int band[kLineMaxJ][3];
  int nbands;
  int64_t items_total;             // band-major multiplier (coefficient mode)
  int64_t maps_item;               // packed floats per item (maps mode)
  int wave_lds;                    // floats of LDS per wave
  int llbuf_off;                   // float offset of the LL_1 row queue in the wave's LDS
  int llbuf_stride;                // floats per queued LL row
  int ring_off[kLineMaxJ];         // float offsets of the rings of levels l >= 1
  int xcd_order;
  // boundary rule per level as tables (no mode switch in the kernels' loops): source row of ext row
  // e < 0 at ext_top[l][e + 8], of ext row e >= n at ext_bot[l][min(e - n, 31)] (-1: zero row)
  int ext_top[kLineMaxJ][8];
  int ext_bot[kLineMaxJ][32];
};

// source row of ext row e of level l (n rows)
__device__ __forceinline__ int line_src(const LineGeom& g, int l, int e, int n) {
  if (e < 0) return g.ext_top[l][e + 8];
  if (e >= n) return g.ext_bot[l][min(e - n, 31)];
  return e;
}

typedef float f2 __attribute__((ext_vector_type(2)));

// wam_normal4 for an element group g < 2^32 (the same stream: the counter word (g >> 32) ^ (item << 8)
// is item << 8). The key schedule is re-derived from an opaque copy of the seed at every call: left
// loop-invariant, the compiler keeps all 20 round keys in SGPRs for the whole kernel, and the filter
// taps (which this kernel keeps in SGPRs to save 16 VGPRs per lane) no longer fit.
__device__ __forceinline__ void line_normal4(uint32_t g, uint32_t item, uint32_t smp, uint32_t k0, uint32_t k1,
                                             float z[4]) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
  asm volatile("" : "+s"(k0), "+s"(k1));
  wam_u4 c = {g, item << 8, smp, item};
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)M0 * c.x, p1 = (uint64_t)M1 * c.z;
    c = {(uint32_t)__builtin_amdgcn_bitop3_b32((uint32_t)(p1 >> 32), c.y, k0, 0x96), (uint32_t)p1,
         (uint32_t)__builtin_amdgcn_bitop3_b32((uint32_t)(p0 >> 32), c.w, k1, 0x96), (uint32_t)p0};
    k0 += W0;
    k1 += W1;
  }
  wam_box_muller(c.x, c.y, z[0], z[1]);
  wam_box_muller(c.z, c.w, z[2], z[3]);
}

__device__ __forceinline__ float line_wave_max(float m) {
#pragma unroll
  for (int s = 32; s > 0; s >>= 1) m = nan_max(m, __shfl_xor(m, s, 64));
  return m;
}

// MC: 0 = one input plane per item; C > 0 = item is an image of C planes, averaged on the load
// CPL: level-1 output columns per lane (mw <= 64 * CPL); NBL: fetched rows held in registers
template <int L, int CPL, int J, bool NOISE, int MC, bool MAPS, int NBL>
__global__ void __launch_bounds__(64 * kLW) __attribute__((amdgpu_waves_per_eu(WAM_LINE_WAVES, 8))) k_plane_line(const float* __restrict__ in, float* __restrict__ out,
                                                         float* __restrict__ band_max,
                                                         const float* __restrict__ filt, LineGeom g, WamNoise nz,
                                                         int64_t n_items, int64_t S, int64_t group_items) {
  constexpr int p = L - 2;
  constexpr int NCH = MC > 0 ? MC : 1;
  extern __shared__ __attribute__((aligned(16))) float smem[];

  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t lwg = g.xcd_order ? wam_xcd_block(blockIdx.x, gridDim.x) : (int64_t)blockIdx.x;
  const int64_t lit = lwg * kLW + wv;
  if (lit >= n_items) return;  // no workgroup barrier in this kernel: a wave without a plane leaves

  const int nh = g.nh0, nw = g.nw0;
  const int64_t in_plane = (int64_t)nh * nw;
  int64_t item = lit, src_plane = lit, img = 0, smp = 0, ch = 0;
  float sg = 0.f;
  if constexpr (NOISE) {
    // sample-fastest: the S noise samples of one clean plane are consecutive waves (one L2)
    const int64_t nc = nz.images * nz.channels;
    src_plane = lit / S;
    const int64_t s = lit % S;
    item = s * nc + src_plane;  // output planes are (sample, image, channel)
    smp = nz.sample_base + s;
    img = src_plane / nz.channels;
    ch = src_plane % nz.channels;
    sg = nz.sigma[img];
  }
  const float* src = in + src_plane * (int64_t)NCH * in_plane;

  f2 fh2[L];  // (lo, hi) tap pairs for packed fp32 FMAs: uniform, SGPR operands
#pragma unroll
  for (int k = 0; k < L; ++k) fh2[k] = f2{filt[k], filt[L + k]};

  // output band bases of this item (uniform): one per level, (H, V, D) a 32-bit stride apart
  // (host check), A_J its own; stores take 32-bit element offsets from them
  float* pb[J];
  unsigned sstr[J];
#pragma unroll
  for (int l = 0; l < J; ++l) {
    const int64_t bn = (int64_t)g.mh[l] * g.mw[l];
    pb[l] = MAPS ? out + item * g.maps_item + g.off[l][0] : out + g.items_total * g.off[l][0] + item * bn;
    sstr[l] = (unsigned)(MAPS ? bn : g.items_total * bn);
  }
  float* const pa = MAPS ? out + item * g.maps_item + g.off_a
                         : out + g.items_total * g.off_a + item * ((int64_t)g.mh[J - 1] * g.mw[J - 1]);
  float mx[J][3], mxa = 0.f;  // MAPS: per-band maxima of |coefficient| (values >= 0)
#pragma unroll
  for (int l = 0; l < J; ++l) mx[l][0] = mx[l][1] = mx[l][2] = 0.f;
  auto put = [&](float* base, unsigned idx, float v, float& m) {
    if constexpr (MAPS) {
      const float a = fabsf(v);
      *at32(base, idx) = a;
      m = nan_max(m, a);
    } else {
      *at32(base, idx) = v;
    }
  };

  float* wl = smem + (int64_t)wv * g.wave_lds;  // level-1 row slot: body at wl[kLPad .. kLPad + nw)
  const int mode = g.mode;
  const bool zero_mode = mode == WAM_MODE_ZERO;

  // ================================================================ levels 2..J (streamed)
  // LL_1 rows emitted by level 1 wait in a queue of kLQ LDS rows and are pushed into level 2 in a
  // runtime loop at two points of the level-1 row group (one copy of the push code per point, not
  // per emitted row); a level-2 output row is written over the LL_1 row just consumed and pushed
  // into level 3 at once.
  PadLane plx[kLineMaxJ];  // pad lanes of the LL rows (level l reads rows of width mw[l - 1])
#pragma unroll
  for (int l = 1; l < J; ++l) plx[l] = pad_lane(lane, g.mw[l - 1], p, mode, kLPad);
  int io[kLineMaxJ];  // next output row of level l (uniform)
#pragma unroll
  for (int l = 0; l < J; ++l) io[l] = 0;

  // horizontal pass of LL_{l} row r (in xb) into ring slot r & 7 of level l
  auto hpass = [&](int l, int r, float* xb) {
    wsync();  // the row's lane writes precede (LDS ops of a wave retire in order)
    refresh_pads(xb, plx[l]);
    wsync();
    const int mwl = g.mw[l];
    const int jc = lane < mwl ? lane : mwl - 1;
    const float2* h = reinterpret_cast<const float2*>(xb + kLPad + 2 * jc - p);
    f2 acc = f2{0.f, 0.f};
#pragma unroll
    for (int m2 = 0; m2 < L / 2; ++m2) {
      const float2 x = h[m2];
      acc = __builtin_elementwise_fma(fh2[2 * m2], f2{x.x, x.x}, acc);
      acc = __builtin_elementwise_fma(fh2[2 * m2 + 1], f2{x.y, x.y}, acc);
    }
    float2* ring = reinterpret_cast<float2*>(wl + g.ring_off[l]);
    if (lane < mwl) ring[(r & (kRing - 1)) * mwl + lane] = make_float2(acc.x, acc.y);
    wsync();  // every lane's reads of xb precede the next writes to it
  };
  // largest source row (of nin) the taps of output row i of level lv read; -1: none
  auto need = [&](int lv, int i, int nin) {
    const int e0 = 2 * i - p;
    if (e0 >= 0 && e0 + L - 1 < nin) return e0 + L - 1;
    int m = -1;
#pragma unroll
    for (int k = 0; k < L; ++k) m = max(m, line_src(g, lv, e0 + k, nin));
    return m;
  };
  // vertical pass of output row i of level l from its ring: (a, h), (v, d); stores H, V, D
  auto vpass = [&](int l, int i, f2& ah, f2& vd) {
    const int mwl = g.mw[l], nin = g.mh[l - 1];
    const int jc = lane < mwl ? lane : mwl - 1;
    const float2* ring = reinterpret_cast<const float2*>(wl + g.ring_off[l]) + jc;
    ah = vd = f2{0.f, 0.f};
    const int e0 = 2 * i - p;
    if (e0 >= 0 && e0 + L - 1 < nin) {
#pragma unroll
      for (int k = 0; k < L; ++k) {
        const float2 q = ring[((e0 + k) & (kRing - 1)) * mwl];
        ah = __builtin_elementwise_fma(fh2[k], f2{q.x, q.x}, ah);
        vd = __builtin_elementwise_fma(fh2[k], f2{q.y, q.y}, vd);
      }
    } else {
      // boundary rows: source row through the extension rule; zero rows contribute fma(f, 0, acc)
      // = acc (acc is never -0), i.e. they are skipped
#pragma unroll
      for (int k = 0; k < L; ++k) {
        const int s = line_src(g, l, e0 + k, nin);
        if (s >= 0) {
          const float2 q = ring[(s & (kRing - 1)) * mwl];
          ah = __builtin_elementwise_fma(fh2[k], f2{q.x, q.x}, ah);
          vd = __builtin_elementwise_fma(fh2[k], f2{q.y, q.y}, vd);
        }
      }
    }
    if (lane < mwl) {
      const unsigned idx = (unsigned)(i * mwl + lane);
      put(pb[l], idx, ah.y, mx[l][0]);
      put(pb[l], idx + sstr[l], vd.x, mx[l][1]);
      put(pb[l], idx + 2 * sstr[l], vd.y, mx[l][2]);
    }
  };
  // level 3 (index 2): LL_2 row r in xb
  auto push2 = [&](int r, float* xb) {
    if constexpr (J > 2) {
      hpass(2, r, xb);
      while (io[2] < g.mh[2] && need(2, io[2], g.mh[1]) <= r) {
        f2 ah, vd;
        vpass(2, io[2], ah, vd);
        if (lane < g.mw[2]) put(pa, (unsigned)(io[2] * g.mw[2] + lane), ah.x, mxa);
        ++io[2];
      }
    }
  };
  // level 2 (index 1): LL_1 row r in xb
  auto push1 = [&](int r, float* xb) {
    if constexpr (J > 1) {
      hpass(1, r, xb);
      while (io[1] < g.mh[1] && need(1, io[1], g.mh[0]) <= r) {
        f2 ah, vd;
        vpass(1, io[1], ah, vd);
        if constexpr (J == 2) {
          if (lane < g.mw[1]) put(pa, (unsigned)(io[1] * g.mw[1] + lane), ah.x, mxa);
        } else {
          if (lane < g.mw[1]) xb[kLPad + lane] = ah.x;  // LL_2 row over the consumed LL_1 row
          push2(io[1], xb);
        }
        ++io[1];
      }
    }
  };
  float* const xq = wl + g.llbuf_off;  // queue of kLQ LL_1 rows, g.llbuf_stride floats apart
  int qn = 0, qrow = 0;                // queued rows, LL_1 row index of the first
  auto push_queue = [&]() {
    if constexpr (J > 1) {
      for (int q = 0; q < qn; ++q) push1(qrow + q, xq + q * g.llbuf_stride);
      qrow += qn;
      qn = 0;
    }
  };

  // ================================================================ level 1 (finest), streamed
  {
    const int mh = g.mh[0], mw = g.mw[0];
    const PadLane pl = pad_lane(lane, nw, p, mode, kLPad);
    if (zero_mode && pl.dst >= 0) wl[pl.dst] = 0.f;  // the zero-mode pads of the row slot, once
    const float2* hsrc[CPL];
#pragma unroll
    for (int c = 0; c < CPL; ++c)
      hsrc[c] = reinterpret_cast<const float2*>(wl + kLPad + 2 * min(lane + 64 * c, mw - 1) - p);
    const int T = 2 * mh + L - 2;  // ext rows -p .. 2 mh - 1
    constexpr int GRPL = (L % NBL == 0) ? L : ((NBL % L == 0) ? NBL : L * NBL / 2);  // lcm(L, NBL)

    RowRegs<4, 1> f[NBL][NCH];
    int srow[NBL];
    auto fetch = [&](RowRegs<4, 1> (&fr)[NCH], int& sr_out, int t) {
      const int sr = line_src(g, 0, t - p, nh);
      const bool valid = sr >= 0;
      sr_out = sr;  // -1: zero row
#pragma unroll
      for (int c = 0; c < NCH; ++c) fr[c].fetch(src + c * in_plane + (int64_t)(valid ? sr : 0) * nw, nw, lane, valid);
    };
    // SmoothGrad noise of source rows sra, srb (< 0: zero rows, any value) generated together: two
    // interleaved Philox chains; element group = (row's first element) / 4 + lane (< 2^32, host check)
    auto noise2 = [&](float (&za)[4], float (&zb)[4], int sra, int srb) {
      if constexpr (NOISE) {
        const uint32_t rowg = (uint32_t)(ch * nh) * (uint32_t)nw / 4u + (uint32_t)lane;
        const uint32_t nw4 = (uint32_t)nw / 4u;
        wam_normal4_x2(rowg + (uint32_t)(sra >= 0 ? sra : 0) * nw4, rowg + (uint32_t)(srb >= 0 ? srb : 0) * nw4,
                       (uint32_t)(img + nz.image_base), (uint32_t)smp, nz.k0, nz.k1, za, zb);
        asm volatile("" ::"v"(za[0]), "v"(za[1]), "v"(za[2]), "v"(za[3]), "v"(zb[0]), "v"(zb[1]), "v"(zb[2]),
                     "v"(zb[3]));
      }
    };
    // the noise of one source row (NX == 1: one Philox chain per row, fewer live registers)
    auto noise1 = [&](float (&z)[4], int sr) {
      WAM_LINE_SCHED();
      if constexpr (NOISE) {
        const uint32_t rowg = (uint32_t)(ch * nh) * (uint32_t)nw / 4u + (uint32_t)lane;
        line_normal4(rowg + (uint32_t)(sr >= 0 ? sr : 0) * ((uint32_t)nw / 4u), (uint32_t)(img + nz.image_base),
                     (uint32_t)smp, nz.k0, nz.k1, z);
      }
    };
    f2 rv[CPL][L];  // ring: (lo, hi) of ext row t in slot t % L
    auto consume = [&](RowRegs<4, 1> (&fr)[NCH], int sr, int slot, const float (&nzr)[4]) {
      WAM_LINE_SCHED();
      float4 o = fr[0].ok[0] ? make_float4(fr[0].v[0], fr[0].v[1], fr[0].v[2], fr[0].v[3])
                             : make_float4(0.f, 0.f, 0.f, 0.f);
      if constexpr (NCH > 1) {
#pragma unroll
        for (int c = 1; c < NCH; ++c) {
          o.x += fr[c].v[0];
          o.y += fr[c].v[1];
          o.z += fr[c].v[2];
          o.w += fr[c].v[3];
        }
        constexpr float inv = 1.0f / (float)NCH;
        o.x *= inv;
        o.y *= inv;
        o.z *= inv;
        o.w *= inv;
        if (!fr[0].ok[0]) o = make_float4(0.f, 0.f, 0.f, 0.f);
      }
      if constexpr (NOISE) {
        // noisy = fma(sigma, z, x): the rounding of wam_noise_add; zero rows stay zero
        const float sgr = sr >= 0 ? sg : 0.f;
        o.x = fmaf(sgr, nzr[0], o.x);
        o.y = fmaf(sgr, nzr[1], o.y);
        o.z = fmaf(sgr, nzr[2], o.z);
        o.w = fmaf(sgr, nzr[3], o.w);
      }
      if (lane * 4 < nw) *reinterpret_cast<float4*>(wl + kLPad + lane * 4) = o;
      wsync();
      if (!zero_mode) {
        refresh_pads(wl, pl);
        wsync();
      }
      f2 acc[CPL];
#pragma unroll
      for (int c = 0; c < CPL; ++c) acc[c] = f2{0.f, 0.f};
#pragma unroll
      for (int m2 = 0; m2 < L / 2; ++m2) {
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
          const float2 x = hsrc[c][m2];
          acc[c] = __builtin_elementwise_fma(fh2[2 * m2], f2{x.x, x.x}, acc[c]);
          acc[c] = __builtin_elementwise_fma(fh2[2 * m2 + 1], f2{x.y, x.y}, acc[c]);
        }
      }
#pragma unroll
      for (int c = 0; c < CPL; ++c) rv[c][slot] = acc[c];
      WAM_LINE_SCHED();
      wsync();
    };
    // output row i of level 1 from ring slots (s0 + k) % L, k = 0 .. L-1
    auto emit = [&](int i, int s0) {
      WAM_LINE_SCHED();
      if (i >= mh) return;  // the partial last group (uniform)
      f2 av[CPL], hd[CPL];
#pragma unroll
      for (int c = 0; c < CPL; ++c) av[c] = hd[c] = f2{0.f, 0.f};
#pragma unroll
      for (int k = 0; k < L; ++k) {
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
          const f2 r = rv[c][(s0 + k) % L];
          av[c] = __builtin_elementwise_fma(f2{fh2[k].x, fh2[k].x}, r, av[c]);  // (a, v)
          hd[c] = __builtin_elementwise_fma(f2{fh2[k].y, fh2[k].y}, r, hd[c]);  // (h, d)
        }
      }
      float* xb = xq + qn * g.llbuf_stride;
#pragma unroll
      for (int c = 0; c < CPL; ++c) {
        const int j = lane + 64 * c;
        if (j < mw) {
          const unsigned idx = (unsigned)(i * mw + j);
          put(pb[0], idx, hd[c].x, mx[0][0]);
          put(pb[0], idx + sstr[0], av[c].y, mx[0][1]);
          put(pb[0], idx + 2 * sstr[0], hd[c].y, mx[0][2]);
          if constexpr (J == 1) put(pa, idx, av[c].x, mxa);
          else xb[kLPad + j] = av[c].x;
        }
      }
      ++qn;
    };

    // Every fetch is unconditional (rows past the plane are clamped and never emitted): loads under
    // divergent control flow would make the compiler drain vmcnt at the join.
#pragma unroll
    for (int u = 0; u < NBL - 1; ++u) fetch(f[u], srow[u], u);
    float za[4] = {0.f, 0.f, 0.f, 0.f}, zb[4] = {0.f, 0.f, 0.f, 0.f};
    // prologue: ext rows 0 .. L-3 fill ring slots 0 .. L-3
#pragma unroll
    for (int t = 0; t < L - 2; ++t) {
      fetch(f[(t + NBL - 1) % NBL], srow[(t + NBL - 1) % NBL], t + NBL - 1);
      if constexpr (NX == 1) {
        noise1(za, srow[t % NBL]);
        consume(f[t % NBL], srow[t % NBL], t, za);
      } else {
        if (!(t & 1)) noise2(za, zb, srow[t % NBL], srow[(t + 1) % NBL]);
        consume(f[t % NBL], srow[t % NBL], t, (t & 1) ? zb : za);
      }
    }
    // steady state: GRPL ext rows per iteration (t % L and t % NBL compile-time)
    for (int base = L - 2; base < T; base += GRPL) {
#pragma unroll
      for (int u = 0; u < GRPL; ++u) {
        const int t = base + u;
        fetch(f[(L - 2 + u + NBL - 1) % NBL], srow[(L - 2 + u + NBL - 1) % NBL], t + NBL - 1);
        if constexpr (NX == 1) {
          noise1(za, srow[(L - 2 + u) % NBL]);
          consume(f[(L - 2 + u) % NBL], srow[(L - 2 + u) % NBL], (L - 2 + u) % L, za);
        } else {
          if (!(u & 1)) noise2(za, zb, srow[(L - 2 + u) % NBL], srow[(L - 2 + u + 1) % NBL]);
          consume(f[(L - 2 + u) % NBL], srow[(L - 2 + u) % NBL], (L - 2 + u) % L, (u & 1) ? zb : za);
        }
        if (u & 1) {
          emit((t - (L - 1)) / 2, (u - 1) % L);
          if (((u + 1) / 2) % kLQ == 0 || u == GRPL - 1) push_queue();  // static
        }
      }
    }
  }

  if constexpr (MAPS) {
    const int64_t grp = (item / group_items) * g.nbands;
    unsigned int* bm = reinterpret_cast<unsigned int*>(band_max) + grp;
#pragma unroll
    for (int l = 0; l < J; ++l)
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        const float m = line_wave_max(mx[l][s]);
        if (lane == 0 && m != 0.f) atomicMax(bm + g.band[l][s], __float_as_uint(m));
      }
    const float m = line_wave_max(mxa);
    if (lane == 0 && m != 0.f) atomicMax(bm, __float_as_uint(m));
  }
}

// ------------------------------------------------------------------------------------------------ host
bool l_ok(int L) { return L == 2 || L == 4 || L == 6 || L == 8; }

// Every output row of level l >= 2 must find the source rows its taps read (through the boundary
// rule) in the 8-slot ring when it is emitted: emission at the latest such row, in order.
bool rings_ok(const wam_plan* p, int mode) {
  const int L = p->L, pp = L - 2;
  for (int l = 1; l < p->levels; ++l) {
    const int nin = (int)p->lout[l - 1][0], mh = (int)p->lout[l][0];
    int last = -1;
    for (int i = 0; i < mh; ++i) {
      int mx = -1, mn = 1 << 30;
      for (int k = 0; k < L; ++k) {
        const int s = wam_ext_index(2 * i - pp + k, nin, mode);
        if (s < 0) continue;
        mx = s > mx ? s : mx;
        mn = s < mn ? s : mn;
      }
      const int at = mx > last ? mx : last;  // the row whose arrival emits output i
      last = at;
      if (mx >= 0 && mn <= at - kRing) return false;
    }
  }
  return true;
}

int line_lds_floats(const wam_plan* p, int nw0, LineGeom* g) {
  const int pp = p->L - 2;
  int rs = (kLPad + nw0 + pp + 2 + 3) & ~3;  // level-1 row: left pads, body, right pads (one spare)
  int mwmax = 0;
  for (int l = 0; l + 1 < p->levels; ++l) mwmax = (int)p->lout[l][1] > mwmax ? (int)p->lout[l][1] : mwmax;
  const int llb = p->levels > 1 ? (kLPad + mwmax + pp + 2 + 3) & ~3 : 0;
  int off = rs;
  if (g) {
    g->llbuf_off = off;
    g->llbuf_stride = llb;
  }
  off += kLQ * llb;
  for (int l = 1; l < p->levels; ++l) {
    if (g) g->ring_off[l] = off;
    off += (2 * kRing * (int)p->lout[l][1] + 3) & ~3;
  }
  return off;
}

bool line_geom_ok(const wam_plan* p, int nh0, int nw0, int mode) {
  if (p->ndim != 2 || !l_ok(p->L) || p->levels < 1 || p->levels > kLineMaxJ) return false;
  if (nw0 % 4 || nw0 < 4 || nw0 > 256 || nh0 < 1) return false;
  if (p->lout[0][1] > 128) return false;
  for (int l = 1; l < p->levels; ++l)
    if (p->lout[l][1] > 64) return false;
  // opt-in (WAM_PLAN_LINE) until it beats the plane kernel at the c2 shape
  if (!(p->flags & WAM_PLAN_LINE) || (p->flags & (WAM_PLAN_NO_COOP | WAM_PLAN_FORCE_COOP))) return false;
  if ((int64_t)line_lds_floats(p, nw0, nullptr) * 4 * kLW > kLineLdsCap) return false;
  return rings_ok(p, mode);
}

template <int L, int CPL, int J, bool NOISE, int MC, bool MAPS, int NBL>
int launch_line_t(const LineGeom& g, int64_t n_items, const float* in, float* out, float* band_max,
                  const float* filt, const WamNoise& nz, int64_t S, int64_t group_items, const char* name,
                  double bytes, hipStream_t st) {
  auto kern = k_plane_line<L, CPL, J, NOISE, MC, MAPS, NBL>;
  const int lds_bytes = g.wave_lds * 4 * kLW;
  const int64_t nwg = (n_items + kLW - 1) / kLW;
  WamTimer tm(st, name, bytes);
  hipLaunchKernelGGL(kern, dim3((unsigned)nwg), dim3(64 * kLW), lds_bytes, st, in, out, band_max, filt, g, nz,
                     n_items, S, group_items);
  WAM_LAUNCH_CHECK();
  return WAM_OK;
}

template <int L, bool NOISE, int MC, bool MAPS, int NBL>
int dispatch_line(const LineGeom& g, int64_t n_items, const float* in, float* out, float* band_max,
                  const float* filt, const WamNoise& nz, int64_t S, int64_t group_items, const char* name,
                  double bytes, hipStream_t st) {
#define WAM_LINE_ARGS g, n_items, in, out, band_max, filt, nz, S, group_items, name, bytes, st
  const bool two = g.mw[0] > 64;
  switch (g.J) {
    case 1:
      return two ? launch_line_t<L, 2, 1, NOISE, MC, MAPS, NBL>(WAM_LINE_ARGS)
                 : launch_line_t<L, 1, 1, NOISE, MC, MAPS, NBL>(WAM_LINE_ARGS);
    case 2:
      return two ? launch_line_t<L, 2, 2, NOISE, MC, MAPS, NBL>(WAM_LINE_ARGS)
                 : launch_line_t<L, 1, 2, NOISE, MC, MAPS, NBL>(WAM_LINE_ARGS);
    case 3:
      return two ? launch_line_t<L, 2, 3, NOISE, MC, MAPS, NBL>(WAM_LINE_ARGS)
                 : launch_line_t<L, 1, 3, NOISE, MC, MAPS, NBL>(WAM_LINE_ARGS);
    default:
      return WAM_ERR_UNSUPPORTED;
  }
#undef WAM_LINE_ARGS
}

LineGeom make_line_geom(const wam_plan* p, int nh0, int nw0, int mode, int64_t items_total) {
  LineGeom g{};
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
  g.wave_lds = line_lds_floats(p, nw0, &g);
  g.xcd_order = 1;
  // tables of the boundary rule: level 0 reads the nh0 input rows, level l the mh[l - 1] LL rows
  for (int l = 0; l < p->levels; ++l) {
    const int n = l ? g.mh[l - 1] : nh0;
    for (int k = 0; k < 8; ++k) g.ext_top[l][k] = wam_ext_index(k - 8, n, mode);
    for (int k = 0; k < 32; ++k) g.ext_bot[l][k] = wam_ext_index(n + k, n, mode);
  }
  return g;
}

}  // namespace

bool dwt2_line_supported(const wam_plan* p, bool adjoint) {
  const int nh0 = (int)(adjoint ? p->rec_shape[0] : p->lin[0][0]);
  const int nw0 = (int)(adjoint ? p->rec_shape[1] : p->lin[0][1]);
  return line_geom_ok(p, nh0, nw0, adjoint ? WAM_MODE_ZERO : p->mode);
}

// The SmoothGrad analysis (nz != nullptr): items = n_samples x images x channels output planes from
// images x channels clean planes. Only the noisy form is routed here: its input is L2-resident
// (the S samples of a plane are consecutive waves), so one row in flight per wave is enough; the
// clean analysis of distinct planes keeps the plane kernel's deeper fetch stream.
int launch_dwt2_line_analysis(const wam_plan* p, int64_t items, const float* in, float* coeffs, const WamNoise* nz,
                              int64_t n_samples, hipStream_t st) {
  if (!nz || ((uintptr_t)in & 15) || !dwt2_line_supported(p, false)) return WAM_ERR_UNSUPPORTED;
  const int nh0 = (int)p->lin[0][0], nw0 = (int)p->lin[0][1];
  if (items != n_samples * nz->images * nz->channels) return WAM_ERR_INVALID_ARG;
  if ((int64_t)nz->channels * nh0 * nw0 >= (int64_t(1) << 34)) return WAM_ERR_UNSUPPORTED;
  // (H, V, D) of a level are addressed by 32-bit byte offsets from the H band's base
  for (int l = 0; l < p->levels; ++l)
    if (3 * items * p->lout[l][0] * p->lout[l][1] >= (int64_t(1) << 30)) return WAM_ERR_UNSUPPORTED;
  const LineGeom g = make_line_geom(p, nh0, nw0, p->mode, items);
  const float* filt = p->d_filt + WAM_F_ANA_LO * p->L;
  const double in_planes = (double)nz->images * nz->channels;
  const double bytes = 4.0 * (in_planes * nh0 * nw0 + (double)items * p->band_off[p->nbands]);
  switch (p->L) {
    case 2: return dispatch_line<2, true, 0, false, 2>(g, items, in, coeffs, nullptr, filt, *nz, n_samples, 1, "k_plane_line<noise>", bytes, st);
    case 4: return dispatch_line<4, true, 0, false, 2>(g, items, in, coeffs, nullptr, filt, *nz, n_samples, 1, "k_plane_line<noise>", bytes, st);
    case 6: return dispatch_line<6, true, 0, false, 2>(g, items, in, coeffs, nullptr, filt, *nz, n_samples, 1, "k_plane_line<noise>", bytes, st);
    case 8: return dispatch_line<8, true, 0, false, 2>(g, items, in, coeffs, nullptr, filt, *nz, n_samples, 1, "k_plane_line<noise>", bytes, st);
    default: return WAM_ERR_UNSUPPORTED;
  }
}

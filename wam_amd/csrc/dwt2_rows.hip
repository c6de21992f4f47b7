// Row-resident fused 2D analysis kernels for gfx950 (rows up to 512 samples wide -- every 2D
// config of the WAM path: 224^2 ImageNet crops and their pyramids, 512^2 for IG).
//
// One wave = one plane (or, for the adjoint epilogue, one image = C planes) x one strip of
// 64*CPL output columns x one chunk of R output rows. The wave walks the extended input rows top
// to bottom. Each source row is fetched WHOLE with 16-byte loads (one float4 per lane covers 256
// samples) one row ahead of its use -- branch-free (clamped addresses + selects) so the compiler
// can keep the next row in flight with a counted vmcnt -- optionally gets its SmoothGrad noise
// generated at fetch time and added at commit time (Philox4x32-10, 4 normals per lane per float4,
// the same stream as wam_noise_add), and is committed to a wave-private LDS row that carries the
// boundary extension in explicit pad slots (refreshed per row from per-lane precomputed source
// columns; zero padding is written once). No halo is staged from HBM and no noisy copy of the input
// is ever written. Each lane filters its columns horizontally (ds_read_b64 pairs), pushes lo/hi
// into a register ring of the last L rows and, every second row, filters the ring vertically
// into LL / H / V / D.
//
// k_adj_maps is the backward pass fused with the WAM epilogue (lib/wam_2D.py:227-256): zero-mode
// analysis with reverse(rec) filters of all C channels of an image in one wave, then per
// coefficient the numpy channel mean ((g0 + g1) + g2) / C, |.|, a wave-level running max per band
// (one atomic max per wave and band: batch-global maxima per noise sample) and the item-major
// |mean| maps the mosaic kernels gather from. LL stays per channel for the next level; the
// per-channel detail gradients are only written when the caller asks for them (side attribute).
//
// Waves are independent (no workgroup barriers). LDS writes and reads of a wave-private row are
// ordered by the wave's in-order LDS queue; __builtin_amdgcn_wave_barrier() keeps the compiler
// from reordering them.
#include "rowtools.hpp"

namespace {

using namespace wam_rows;

template <int L>
constexpr bool kRolledPrologue = L >= 12;
// long filters also run their tap chains as packed (lo, hi) / (a, h) / (v, d) pairs (same sums)
template <int L>
constexpr bool kPackedTaps = L >= 12;

template <int L>
__device__ __forceinline__ void tap_pairs(const float (&flo)[L], const float (&fhi)[L], wam_f2 (&fp)[L]) {
#pragma unroll
  for (int k = 0; k < L; ++k) fp[k] = wam_f2{flo[k], fhi[k]};
}

// vertical filter of one column's ring: a = sum flo rl, h = sum fhi rl, v = sum flo rh, d = sum fhi rh
template <int L>
__device__ __forceinline__ void vfilter(const float (&flo)[L], const float (&fhi)[L], const wam_f2 (&fp)[L],
                                        const float (&rl)[L], const float (&rh)[L], float& a, float& h, float& v,
                                        float& d) {
  if constexpr (kPackedTaps<L>) {
    wam_f2 ah = {0.f, 0.f}, vd = {0.f, 0.f};
#pragma unroll
    for (int k = 0; k < L; ++k) {
      ah = __builtin_elementwise_fma(fp[k], wam_f2{rl[k], rl[k]}, ah);
      vd = __builtin_elementwise_fma(fp[k], wam_f2{rh[k], rh[k]}, vd);
    }
    a = ah.x;
    h = ah.y;
    v = vd.x;
    d = vd.y;
  } else {
    a = h = v = d = 0.f;
#pragma unroll
    for (int k = 0; k < L; ++k) {
      a = fmaf(flo[k], rl[k], a);
      h = fmaf(fhi[k], rl[k], h);
      v = fmaf(flo[k], rh[k], v);
      d = fmaf(fhi[k], rh[k], d);
    }
  }
}

template <int L>
__device__ __forceinline__ void hfilter_any(const float* lds, int j, int p, const float (&flo)[L],
                                            const float (&fhi)[L], const wam_f2 (&fp)[L], float& lo, float& hi) {
  if constexpr (kPackedTaps<L>) {
    const wam_f2 r = hfilter_pk<L>(lds, j, p, fp);
    lo = r.x;
    hi = r.y;
  } else {
    hfilter<L>(lds, j, p, flo, fhi, lo, hi);
  }
}

// ------------------------------------------------------------------------------------------------
template <int L, int CPL, int VEC, int MAXV, bool NOISE>
__global__ void __launch_bounds__(256) k_ana_rows(const float* __restrict__ in, int nh, int nw, int64_t in_plane,
                                                  float* __restrict__ oa, float* __restrict__ oh,
                                                  float* __restrict__ ov, float* __restrict__ od, int mh, int mw,
                                                  int64_t out_plane, int mode, const float* __restrict__ filt,
                                                  int nstrips, int nchunks, int R, int64_t total_waves, WamNoise nz) {
  constexpr int p = L - 2;
  __shared__ __attribute__((aligned(16))) float rows[kWaves][kRowLds];
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: SGPR bases
  const int64_t gw = wam_xcd_block(blockIdx.x, gridDim.x) * kWaves + wv;
  if (gw >= total_waves) return;
  // strip fastest: the strips of one (plane, row chunk) -- which fetch the same source rows --
  // are waves of one workgroup (one CU, one XCD L2) instead of landing on different XCDs
  const int strip = (int)(gw % nstrips);
  const int64_t t = gw / nstrips;
  const int chunk = (int)(t % nchunks);
  const int64_t plane = t / nchunks;

  float flo[L], fhi[L];
#pragma unroll
  for (int k = 0; k < L; ++k) {
    flo[k] = filt[k];
    fhi[k] = filt[L + k];
  }
  wam_f2 fp[L];
  tap_pairs<L>(flo, fhi, fp);
  // NOISE: planes are (sample, image, channel); the clean input x holds (image, channel)
  int64_t src_plane = plane, img = 0, smp = 0, ch = 0;
  float sg = 0.f;
  if constexpr (NOISE) {
    const int64_t per_sample = nz.images * nz.channels;
    src_plane = plane % per_sample;
    smp = nz.sample_base + plane / per_sample;
    img = src_plane / nz.channels;
    ch = src_plane % nz.channels;
    sg = nz.sigma[img];
  }
  const float* src = in + src_plane * in_plane;
  float* lds = rows[wv];
  const PadLane pl = pad_lane(lane, nw, p, mode);
  const bool zero_mode = mode == WAM_MODE_ZERO;
  if (zero_mode && pl.dst >= 0) lds[pl.dst] = 0.f;  // zero pads never change
  const int j0 = strip * 64 * CPL;
  const int i0 = chunk * R;
  const int i1 = min(mh, i0 + R);
  const int er0 = 2 * i0 - p;

  RowRegs<VEC, MAXV> f[2];
  constexpr int NZ = NOISE ? 4 * MAXV : 1;
  float nzv[2][NZ];
  auto fetch = [&](RowRegs<VEC, MAXV>& r, float (&nzr)[NZ], int er) {
    const int sr = row_src(er, nh, mode);
    const bool valid = sr >= 0;
    const int rr = valid ? sr : 0;
    r.fetch(src + (int64_t)rr * nw, nw, lane, valid);
    if constexpr (NOISE) make_noise<MAXV>(nzr, nw, lane, (ch * nh + rr) * (int64_t)nw, sg, img + nz.image_base, smp, nz.k0, nz.k1,
                                             valid);
  };
  auto process = [&](const RowRegs<VEC, MAXV>& r, const float (&nzr)[NZ], float (&lo)[CPL], float (&hi)[CPL]) {
    r.commit(lds, lane, NOISE ? nzr : nullptr, sg);
    wsync();
    if (!zero_mode) {
      refresh_pads(lds, pl);
      wsync();
    }
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      const int j = min(j0 + lane + 64 * c, mw - 1);  // clamp: the extra lanes compute a duplicate
      hfilter_any<L>(lds, j, p, flo, fhi, fp, lo[c], hi[c]);
    }
    wsync();
  };

  // Long filters (kRolledPrologue) fill the ring by (L - 2) / 2 warm-up passes of the row loop
  // itself (outputs not stored): unrolled, the prologue's L - 2 row passes are scheduled together
  // and hold ~4x the loop's registers at L = 16 (AGPR-resident LDS reads: 1 wave per SIMD instead
  // of 4). Short filters keep the unrolled prologue (the warm-up passes' vertical filters cost
  // 4-7 % at L = 8, profiles/r03i_kbench_c2_rows_rolled_ab.log).
  float rl[CPL][L], rh[CPL][L];
  fetch(f[0], nzv[0], er0);
  if constexpr (kRolledPrologue<L>) {
#pragma unroll
    for (int c = 0; c < CPL; ++c)
#pragma unroll
      for (int k = 0; k < L; ++k) rl[c][k] = rh[c][k] = 0.f;
  } else {
#pragma unroll
    for (int k = 0; k < L - 2; ++k) {
      fetch(f[(k + 1) & 1], nzv[(k + 1) & 1], er0 + k + 1);
      float lo[CPL], hi[CPL];
      process(f[k & 1], nzv[k & 1], lo, hi);
#pragma unroll
      for (int c = 0; c < CPL; ++c) {
        rl[c][k] = lo[c];
        rh[c][k] = hi[c];
      }
    }
  }
  // invariant: f[0] holds ext row er0 + 2*(i - i0) + L - 2
  for (int i = i0 - (kRolledPrologue<L> ? (L - 2) / 2 : 0); i < i1; ++i) {
    const int er = er0 + 2 * (i - i0) + L - 2;
    fetch(f[1], nzv[1], er + 1);
    float lo[CPL], hi[CPL];
    process(f[0], nzv[0], lo, hi);
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      rl[c][L - 2] = lo[c];
      rh[c][L - 2] = hi[c];
    }
    // on the last iteration the row after the chunk is never used: re-fetch the chunk's last ext
    // row (a cache hit) instead of the next chunk's first row (an HBM re-read: that chunk's wave
    // fetched it long before)
    fetch(f[0], nzv[0], min(er + 2, er0 + 2 * (i1 - i0) + L - 3));
    process(f[1], nzv[1], lo, hi);
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      rl[c][L - 1] = lo[c];
      rh[c][L - 1] = hi[c];
    }
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      const int j = j0 + lane + 64 * c;
      float a, h, v, d;
      vfilter<L>(flo, fhi, fp, rl[c], rh[c], a, h, v, d);
      if (j < mw && (!kRolledPrologue<L> || i >= i0)) {
        const int64_t o = plane * out_plane + (int64_t)i * mw + j;
        oa[o] = a;
        oh[o] = h;
        ov[o] = v;
        od[o] = d;
      }
#pragma unroll
      for (int k = 0; k < L - 2; ++k) {
        rl[c][k] = rl[c][k + 2];
        rh[c][k] = rh[c][k + 2];
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
struct MapsArgs {
  float* maps;          // item-major packed |mean_c| maps, item = image
  float* band_max;      // [groups, nbands]
  float* full;          // optional band-major per-channel grads (planes = full_items)
  int64_t maps_item;    // packed coefficients per item (plan coeff_numel)
  int64_t off_h, off_v, off_d, off_a;  // per-item offsets of this level's bands (off_a < 0: not last)
  int bh, bv, bd, ba;   // band indices
  int nbands;
  int64_t group_items;
  int64_t full_items;
};

// C: channels filtered separately (the per-channel form, numpy's mean-after-DWT order, needed when
// the caller wants the per-channel coefficient gradients); CIN > 1 (with C == 1): the CIN gradient
// planes of an image are averaged on the load and ONE plane is filtered (the mean commutes with the
// linear adjoint -- the k_plane_maps form, equal to fp32 rounding), and the next level's LL is one
// plane per image. CPL: output columns per lane (strip = 64 CPL columns).
// WIN (rows split into strips, 16-byte rows): a wave fetches only its strip's input window --
// columns [2 j0 - PW, 2 j0 - PW + WN) with PW = p rounded up to 4 -- instead of the whole row:
// every strip fetching whole rows read each row nstrips times from L2, and at c4's 28 alphas per
// launch enough of those re-reads missed L2 to make the level-0 kernel move 1.62x its bytes from
// HBM (profiles/r03l_bench_c4.log). Zero mode: window columns outside the row load as zeros.
template <int L, int CPL>
struct AdjWindow {
  static constexpr int PW = (L - 2 + 3) & ~3;
  static constexpr int WN = PW + 128 * CPL + 4;         // floats, multiple of 4
  static constexpr int MAXV = (WN + 255) / 256;         // float4 loads per lane
};

template <int L, int C, int CIN, int CPL, int VEC, int MAXV, bool WIN = false>
__global__ void __launch_bounds__(256) k_adj_maps(const float* __restrict__ in, int nh, int nw, int64_t in_plane,
                                                  float* __restrict__ ll_out, int mh, int mw,
                                                  const float* __restrict__ filt, int nstrips, int nchunks, int R,
                                                  int64_t total_waves, MapsArgs ma) {
  static_assert(CIN == 1 || C == 1, "channel mean on load filters one plane");
  constexpr int p = L - 2;
  __shared__ __attribute__((aligned(16))) float rows[kWaves][C][kRowLds];
  const int lane = threadIdx.x & 63;
  // wave-uniform wave index (SGPR bases) except in the windowed form: there the uniform form's
  // lower register count (165 vs 195 VGPRs: 3 instead of 2 waves per SIMD) let more strips of a
  // 28-alpha launch compete for L2 -- PMC/algorithmic 1.05 -> 1.13 and the c4 level-0 launch
  // 3,462 -> 3,633-3,894 us (profiles/r04x_ab_adj28.log) -- while levels 1-2 gain 15-17 %
  const int wv = WIN ? (int)(threadIdx.x >> 6) : __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t gw = wam_xcd_block(blockIdx.x, gridDim.x) * kWaves + wv;
  if (gw >= total_waves) return;
  // strip fastest: the strips of one (plane, row chunk) -- which fetch the same source rows --
  // are waves of one workgroup (one CU, one XCD L2) instead of landing on different XCDs
  const int strip = (int)(gw % nstrips);
  const int64_t t = gw / nstrips;
  const int chunk = (int)(t % nchunks);
  const int64_t img = t / nchunks;

  float flo[L], fhi[L];
#pragma unroll
  for (int k = 0; k < L; ++k) {
    flo[k] = filt[k];
    fhi[k] = filt[L + k];
  }
  wam_f2 fp[L];
  tap_pairs<L>(flo, fhi, fp);
  const float* src = in + img * (C * CIN) * in_plane;
  {
    const PadLane pl = pad_lane(lane, nw, p, WAM_MODE_ZERO);
    if (pl.dst >= 0) {
#pragma unroll
      for (int c = 0; c < C; ++c) rows[wv][c][pl.dst] = 0.f;
    }
  }
  int jcol[CPL];
  bool jv[CPL];
#pragma unroll
  for (int q = 0; q < CPL; ++q) {
    const int j = strip * 64 * CPL + lane + 64 * q;
    jv[q] = j < mw;
    jcol[q] = j;
  }
  const int i0 = chunk * R;
  const int i1 = min(mh, i0 + R);
  const int er0 = 2 * i0 - p;
  const int64_t out_plane = (int64_t)mh * mw;

  constexpr int NF = C * CIN;  // source rows fetched per extended row
  static_assert(!WIN || VEC == 4, "windowed rows are fetched as float4");
  constexpr int PW = AdjWindow<L, CPL>::PW;
  // window mode: the row buffer holds columns ws .. ws + WN - 1 (ws a multiple of 4); a global
  // output column j reads LDS column 2 (j - j0) + PW - p, i.e. hfilter with (j - j0, p - PW)
  const int j0w = strip * 64 * CPL;
  const int ws = 2 * j0w - PW;
  const int jofs = WIN ? j0w : 0;
  const int peff = WIN ? p - PW : p;
  RowRegs<VEC, MAXV> f[2][NF];
  auto fetch = [&](RowRegs<VEC, MAXV> (&r)[NF], int er) {
    const bool valid = er >= 0 && er < nh;  // zero padding
    const int rr = valid ? er : 0;
    if constexpr (WIN) {
#pragma unroll
      for (int c = 0; c < NF; ++c) {
        const float* row = src + c * in_plane + (int64_t)rr * nw;
#pragma unroll
        for (int q = 0; q < MAXV; ++q) {
          const int col = ws + (lane + 64 * q) * 4;
          r[c].ok[q] = valid && col >= 0 && col < nw;  // whole float4s: ws and nw are multiples of 4
          const int ci = min(max(col, 0), nw - 4);
          const float4 t = *reinterpret_cast<const float4*>(row + ci);
          r[c].v[4 * q] = t.x;
          r[c].v[4 * q + 1] = t.y;
          r[c].v[4 * q + 2] = t.z;
          r[c].v[4 * q + 3] = t.w;
        }
      }
    } else {
#pragma unroll
      for (int c = 0; c < NF; ++c) r[c].fetch(src + c * in_plane + (int64_t)rr * nw, nw, lane, valid);
    }
  };
  auto process = [&](RowRegs<VEC, MAXV> (&r)[NF], float (&lo)[C][CPL], float (&hi)[C][CPL]) {
    if constexpr (CIN > 1) {  // ((g0 + g1) + g2) * (1 / CIN), as k_plane_maps averages on its load
      constexpr float inv = 1.0f / (float)CIN;
#pragma unroll
      for (int i = 0; i < VEC * MAXV; ++i) {
        float sum = r[0].v[i];
#pragma unroll
        for (int c = 1; c < CIN; ++c) sum += r[c].v[i];
        r[0].v[i] = sum * inv;
      }
      r[0].commit(rows[wv][0], lane, nullptr);
    } else {
#pragma unroll
      for (int c = 0; c < C; ++c) r[c].commit(rows[wv][c], lane, nullptr);
    }
    wsync();
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int q = 0; q < CPL; ++q)
        hfilter_any<L>(rows[wv][c], (jv[q] ? jcol[q] : mw - 1) - jofs, peff, flo, fhi, fp, lo[c][q], hi[c][q]);
    wsync();
  };

  // long filters: ring filled by (L - 2) / 2 warm-up passes of the row loop (see k_ana_rows)
  float rl[C][CPL][L], rh[C][CPL][L];
  fetch(f[0], er0);
  if constexpr (kRolledPrologue<L>) {
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int q = 0; q < CPL; ++q)
#pragma unroll
        for (int k = 0; k < L; ++k) rl[c][q][k] = rh[c][q][k] = 0.f;
  } else {
#pragma unroll
    for (int k = 0; k < L - 2; ++k) {
      fetch(f[(k + 1) & 1], er0 + k + 1);
      float lo[C][CPL], hi[C][CPL];
      process(f[k & 1], lo, hi);
#pragma unroll
      for (int c = 0; c < C; ++c)
#pragma unroll
        for (int q = 0; q < CPL; ++q) {
          rl[c][q][k] = lo[c][q];
          rh[c][q][k] = hi[c][q];
        }
    }
  }
  float mx_h = 0.f, mx_v = 0.f, mx_d = 0.f, mx_a = 0.f;
  const bool last = ma.off_a >= 0;
  float* mrow = ma.maps + img * ma.maps_item;
  for (int i = i0 - (kRolledPrologue<L> ? (L - 2) / 2 : 0); i < i1; ++i) {
    const int er = er0 + 2 * (i - i0) + L - 2;
    const bool on = !kRolledPrologue<L> || i >= i0;
    fetch(f[1], er + 1);
    float lo[C][CPL], hi[C][CPL];
    process(f[0], lo, hi);
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int q = 0; q < CPL; ++q) {
        rl[c][q][L - 2] = lo[c][q];
        rh[c][q][L - 2] = hi[c][q];
      }
    fetch(f[0], min(er + 2, er0 + 2 * (i1 - i0) + L - 3));  // past the chunk: its last row (see k_ana_rows)
    process(f[1], lo, hi);
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int q = 0; q < CPL; ++q) {
        rl[c][q][L - 1] = lo[c][q];
        rh[c][q][L - 1] = hi[c][q];
      }
#pragma unroll
    for (int q = 0; q < CPL; ++q) {
      float sa = 0.f, sh = 0.f, sv = 0.f, sd = 0.f;
      const int64_t o = (int64_t)i * mw + jcol[q];
#pragma unroll
      for (int c = 0; c < C; ++c) {
        float a, h, v, d;
        vfilter<L>(flo, fhi, fp, rl[c][q], rh[c][q], a, h, v, d);
        if (jv[q] && on) {
          const int64_t plane = img * C + c;
          if (!last) ll_out[plane * out_plane + o] = a;
          if (ma.full) {  // band-major: band b starts at full_items * off_b
            ma.full[ma.full_items * ma.off_h + plane * out_plane + o] = h;
            ma.full[ma.full_items * ma.off_v + plane * out_plane + o] = v;
            ma.full[ma.full_items * ma.off_d + plane * out_plane + o] = d;
            if (last) ma.full[ma.full_items * ma.off_a + plane * out_plane + o] = a;
          }
        }
        // numpy float32 mean over the channel axis: sequential sum, then true_divide
        sa = c == 0 ? a : sa + a;
        sh = c == 0 ? h : sh + h;
        sv = c == 0 ? v : sv + v;
        sd = c == 0 ? d : sd + d;
#pragma unroll
        for (int k = 0; k < L - 2; ++k) {
          rl[c][q][k] = rl[c][q][k + 2];
          rh[c][q][k] = rh[c][q][k + 2];
        }
      }
      if (jv[q] && on) {
        const float mh_ = fabsf(sh / (float)C), mv_ = fabsf(sv / (float)C), md_ = fabsf(sd / (float)C);
        mrow[ma.off_h + o] = mh_;
        mrow[ma.off_v + o] = mv_;
        mrow[ma.off_d + o] = md_;
        mx_h = nan_max(mx_h, mh_);
        mx_v = nan_max(mx_v, mv_);
        mx_d = nan_max(mx_d, md_);
        if (last) {
          const float ma_ = fabsf(sa / (float)C);
          mrow[ma.off_a + o] = ma_;
          mx_a = nan_max(mx_a, ma_);
        }
      }
    }
  }
#pragma unroll
  for (int s = 32; s > 0; s >>= 1) {
    mx_h = nan_max(mx_h, __shfl_xor(mx_h, s, 64));
    mx_v = nan_max(mx_v, __shfl_xor(mx_v, s, 64));
    mx_d = nan_max(mx_d, __shfl_xor(mx_d, s, 64));
    mx_a = nan_max(mx_a, __shfl_xor(mx_a, s, 64));
  }
  if (lane == 0) {
    unsigned int* bm = reinterpret_cast<unsigned int*>(ma.band_max + (img / ma.group_items) * ma.nbands);
    atomicMax(bm + ma.bh, __float_as_uint(mx_h));
    atomicMax(bm + ma.bv, __float_as_uint(mx_v));
    atomicMax(bm + ma.bd, __float_as_uint(mx_d));
    if (last) atomicMax(bm + ma.ba, __float_as_uint(mx_a));
  }
}

// ------------------------------------------------------------------------------------------------
// waves per launch the row chunking aims for: fewer, longer chunks re-read fewer halo rows (L - 2 ext
// rows per chunk). 2,048 instead of 8,192: c4 wavedec same time, k_ana_rows PMC/algorithmic -11 %;
// c4 adjoint maps level 1 164 -> 102 us at 2 x 128 images (profiles/r05s_ab_row_chunk_target.log)
constexpr int64_t kTargetWaves = 2048;

void pick_chunks(int64_t base, int mh, int& nchunks, int& R) {
  int64_t want = (kTargetWaves + base - 1) / base;
  int maxchunks = (mh + 11) / 12;  // >= 12 output rows per chunk (L-2 halo rows per chunk)
  if (maxchunks < 1) maxchunks = 1;
  nchunks = (int)(want < 1 ? 1 : (want > maxchunks ? maxchunks : want));
  R = (mh + nchunks - 1) / nchunks;
  nchunks = (mh + R - 1) / R;
}

template <int L, int CPL, int VEC, int MAXV, bool NOISE>
int launch_ana_rows_t(int64_t batch, const float* in, int nh, int nw, int mh, int mw, int mode, const float* filt,
                      float* oa, float* oh, float* ov, float* od, const WamNoise* nz, hipStream_t st) {
  const int nstrips = (mw + 64 * CPL - 1) / (64 * CPL);
  int nchunks, R;
  pick_chunks(batch * nstrips, mh, nchunks, R);
  const int64_t waves = batch * nstrips * nchunks;
  WamNoise z = nz ? *nz : WamNoise{nullptr, 1, 1, 0, 0, 0, 0};
  double bytes = 4.0 * ((double)batch * 4.0 * mh * mw + (nz ? (double)z.images * z.channels : (double)batch) * nh * nw);
  WamTimer tm(st, NOISE ? "k_ana_rows<noise>" : "k_ana_rows", bytes);
  hipLaunchKernelGGL((k_ana_rows<L, CPL, VEC, MAXV, NOISE>), dim3((unsigned)((waves + kWaves - 1) / kWaves)),
                     dim3(256), 0, st, in, nh, nw, (int64_t)nh * nw, oa, oh, ov, od, mh, mw, (int64_t)mh * mw, mode,
                     filt, nstrips, nchunks, R, waves, z);
  WAM_LAUNCH_CHECK();
  return WAM_OK;
}

template <int L, int CPL>
int dispatch_ana_cpl(int64_t batch, const float* in, int nh, int nw, int mh, int mw, int mode, const float* filt,
                     float* oa, float* oh, float* ov, float* od, const WamNoise* nz, hipStream_t st) {
  const bool vec4 = (nw % 4 == 0) && ((uintptr_t)in % 16 == 0);
  if (nz) {
    if (!vec4) return WAM_ERR_UNSUPPORTED;
    return nw <= 256 ? launch_ana_rows_t<L, CPL, 4, 1, true>(batch, in, nh, nw, mh, mw, mode, filt, oa, oh, ov, od, nz, st)
                     : launch_ana_rows_t<L, CPL, 4, 2, true>(batch, in, nh, nw, mh, mw, mode, filt, oa, oh, ov, od, nz, st);
  }
  if (vec4)
    return nw <= 256
               ? launch_ana_rows_t<L, CPL, 4, 1, false>(batch, in, nh, nw, mh, mw, mode, filt, oa, oh, ov, od, nullptr, st)
               : launch_ana_rows_t<L, CPL, 4, 2, false>(batch, in, nh, nw, mh, mw, mode, filt, oa, oh, ov, od, nullptr,
                                                        st);
  return nw <= 128
             ? launch_ana_rows_t<L, CPL, 1, 2, false>(batch, in, nh, nw, mh, mw, mode, filt, oa, oh, ov, od, nullptr, st)
             : launch_ana_rows_t<L, CPL, 1, 8, false>(batch, in, nh, nw, mh, mw, mode, filt, oa, oh, ov, od, nullptr, st);
}

template <int L>
int dispatch_ana(int64_t batch, const float* in, int nh, int nw, int mh, int mw, int mode, const float* filt,
                 float* oa, float* oh, float* ov, float* od, const WamNoise* nz, hipStream_t st) {
  // long filters: one column per lane (4 waves per SIMD at L = 16; two columns measured 157 vs
  // 116 us at c4 level 1, profiles/r03i_kbench_c4_rows_rolled_ab.log)
  if (mw > 64 && L < 12) return dispatch_ana_cpl<L, 2>(batch, in, nh, nw, mh, mw, mode, filt, oa, oh, ov, od, nz, st);
  return dispatch_ana_cpl<L, 1>(batch, in, nh, nw, mh, mw, mode, filt, oa, oh, ov, od, nz, st);
}

template <int L, int C, int CIN, int CPL, int VEC, int MAXV, bool WIN = false>
int launch_adj_t(int64_t images, const float* in, int nh, int nw, int mh, int mw, const float* filt, float* ll_out,
                 const MapsArgs& ma, hipStream_t st) {
  const int nstrips = (mw + 64 * CPL - 1) / (64 * CPL);
  int nchunks, R;
  pick_chunks(images * nstrips, mh, nchunks, R);
  const int64_t waves = images * nstrips * nchunks;
  const bool last = ma.off_a >= 0;
  double bytes = 4.0 * (double)images * ((double)C * CIN * nh * nw + 4.0 * mh * mw + (last ? 0.0 : (double)C * mh * mw) +
                                         (ma.full ? (double)C * 4 * mh * mw : 0.0));
  WamTimer tm(st, "k_adj_maps", bytes);
  hipLaunchKernelGGL((k_adj_maps<L, C, CIN, CPL, VEC, MAXV, WIN>), dim3((unsigned)((waves + kWaves - 1) / kWaves)),
                     dim3(256), 0, st, in, nh, nw, (int64_t)nh * nw, ll_out, mh, mw, filt, nstrips, nchunks, R, waves,
                     ma);
  WAM_LAUNCH_CHECK();
  return WAM_OK;
}

template <int L, int C, int CIN, int CPL>
int dispatch_adj_c(int64_t images, const float* in, int nh, int nw, int mh, int mw, const float* filt, float* ll_out,
                   const MapsArgs& ma, hipStream_t st) {
  const bool vec4 = (nw % 4 == 0) && ((uintptr_t)in % 16 == 0);
  // several strips per row: each wave fetches its strip's window only (AdjWindow)
  constexpr int WMAXV = AdjWindow<L, CPL>::MAXV;
  if (vec4 && nw > 256 && mw > 64 * CPL && WMAXV <= 2)
    return launch_adj_t<L, C, CIN, CPL, 4, WMAXV, true>(images, in, nh, nw, mh, mw, filt, ll_out, ma, st);
  if (vec4)
    return nw <= 256 ? launch_adj_t<L, C, CIN, CPL, 4, 1>(images, in, nh, nw, mh, mw, filt, ll_out, ma, st)
                     : launch_adj_t<L, C, CIN, CPL, 4, 2>(images, in, nh, nw, mh, mw, filt, ll_out, ma, st);
  return nw <= 128 ? launch_adj_t<L, C, CIN, CPL, 1, 2>(images, in, nh, nw, mh, mw, filt, ll_out, ma, st)
                   : launch_adj_t<L, C, CIN, CPL, 1, 8>(images, in, nh, nw, mh, mw, filt, ll_out, ma, st);
}

// mean_first: the channel mean on the load (one plane filtered; LL out one plane per image)
template <int L>
int dispatch_adj(int channels, bool mean_first, int64_t images, const float* in, int nh, int nw, int mh, int mw,
                 const float* filt, float* ll_out, const MapsArgs& ma, hipStream_t st) {
  // up to three output columns per lane: fewer strips; filters past 12 taps keep two (their
  // (lo, hi) rings of 2 x L registers per column)
  const int cpl = mw <= 64 ? 1 : (mw <= 128 ? 2 : (L > 12 ? 2 : 3));
  if (channels == 3 && mean_first) {
    if (cpl == 1) return dispatch_adj_c<L, 1, 3, 1>(images, in, nh, nw, mh, mw, filt, ll_out, ma, st);
    if (cpl == 2) return dispatch_adj_c<L, 1, 3, 2>(images, in, nh, nw, mh, mw, filt, ll_out, ma, st);
    return dispatch_adj_c<L, 1, 3, 3>(images, in, nh, nw, mh, mw, filt, ll_out, ma, st);
  }
  if (channels == 3) return dispatch_adj_c<L, 3, 1, 1>(images, in, nh, nw, mh, mw, filt, ll_out, ma, st);
  if (channels == 1) {
    if (cpl == 1) return dispatch_adj_c<L, 1, 1, 1>(images, in, nh, nw, mh, mw, filt, ll_out, ma, st);
    if (cpl == 2) return dispatch_adj_c<L, 1, 1, 2>(images, in, nh, nw, mh, mw, filt, ll_out, ma, st);
    return dispatch_adj_c<L, 1, 1, 3>(images, in, nh, nw, mh, mw, filt, ll_out, ma, st);
  }
  return WAM_ERR_UNSUPPORTED;
}

bool l_supported(int L) { return L == 2 || L == 4 || L == 6 || L == 8 || L == 12 || L == 16 || L == 20; }

}  // namespace

bool dwt2_rows_supported(const wam_plan* p, int level, bool adjoint) {
  if (p->ndim != 2 || !l_supported(p->L)) return false;
  const int64_t nw = (adjoint && level == 0) ? p->rec_shape[1] : p->lin[level][1];
  return nw <= kMaxRow && nw >= 4;
}

int launch_dwt2_analysis_rows(const wam_plan* p, int64_t batch, const float* in, const int64_t* in_dims,
                              const int64_t* out_dims, int mode, int fset, float* out_a, float* const* sub,
                              const WamNoise* nz, hipStream_t st) {
  const float* filt = p->d_filt + fset * p->L;
  const int nh = (int)in_dims[0], nw = (int)in_dims[1], mh = (int)out_dims[0], mw = (int)out_dims[1];
  float *oa = out_a, *oh = sub[0], *ov = sub[1], *od = sub[2];
  switch (p->L) {
    case 2: return dispatch_ana<2>(batch, in, nh, nw, mh, mw, mode, filt, oa, oh, ov, od, nz, st);
    case 4: return dispatch_ana<4>(batch, in, nh, nw, mh, mw, mode, filt, oa, oh, ov, od, nz, st);
    case 6: return dispatch_ana<6>(batch, in, nh, nw, mh, mw, mode, filt, oa, oh, ov, od, nz, st);
    case 8: return dispatch_ana<8>(batch, in, nh, nw, mh, mw, mode, filt, oa, oh, ov, od, nz, st);
    case 12: return dispatch_ana<12>(batch, in, nh, nw, mh, mw, mode, filt, oa, oh, ov, od, nz, st);
    case 16: return dispatch_ana<16>(batch, in, nh, nw, mh, mw, mode, filt, oa, oh, ov, od, nz, st);
    case 20: return dispatch_ana<20>(batch, in, nh, nw, mh, mw, mode, filt, oa, oh, ov, od, nz, st);
    default: return WAM_ERR_UNSUPPORTED;
  }
}

int launch_dwt2_adjoint_maps_level(const wam_plan* p, int level, int64_t images, int channels, bool mean_first,
                                   int64_t group_items, const float* in, const int64_t* in_dims, float* ll_out,
                                   float* maps, float* band_max, float* full_grads, int64_t full_items, hipStream_t st) {
  if (mean_first && full_grads) return WAM_ERR_INVALID_ARG;  // per-channel grads need the per-channel form
  const float* filt = p->d_filt + WAM_F_ADJ_LO * p->L;
  const int nh = (int)in_dims[0], nw = (int)in_dims[1];
  const int mh = (int)p->lout[level][0], mw = (int)p->lout[level][1];
  MapsArgs ma;
  ma.maps = maps;
  ma.band_max = band_max;
  ma.full = full_grads;
  ma.maps_item = p->band_off[p->nbands];
  ma.bh = wam_band_of(p, level, 0);
  ma.bv = wam_band_of(p, level, 1);
  ma.bd = wam_band_of(p, level, 2);
  ma.ba = 0;
  ma.off_h = p->band_off[ma.bh];
  ma.off_v = p->band_off[ma.bv];
  ma.off_d = p->band_off[ma.bd];
  ma.off_a = (level == p->levels - 1) ? p->band_off[0] : -1;
  ma.nbands = p->nbands;
  ma.group_items = group_items;
  ma.full_items = full_items;
  switch (p->L) {
    case 2: return dispatch_adj<2>(channels, mean_first, images, in, nh, nw, mh, mw, filt, ll_out, ma, st);
    case 4: return dispatch_adj<4>(channels, mean_first, images, in, nh, nw, mh, mw, filt, ll_out, ma, st);
    case 6: return dispatch_adj<6>(channels, mean_first, images, in, nh, nw, mh, mw, filt, ll_out, ma, st);
    case 8: return dispatch_adj<8>(channels, mean_first, images, in, nh, nw, mh, mw, filt, ll_out, ma, st);
    case 12: return dispatch_adj<12>(channels, mean_first, images, in, nh, nw, mh, mw, filt, ll_out, ma, st);
    case 16: return dispatch_adj<16>(channels, mean_first, images, in, nh, nw, mh, mw, filt, ll_out, ma, st);
    case 20: return dispatch_adj<20>(channels, mean_first, images, in, nh, nw, mh, mw, filt, ll_out, ma, st);
    default: return WAM_ERR_UNSUPPORTED;
  }
}

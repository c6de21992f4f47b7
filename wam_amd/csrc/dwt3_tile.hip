// Fused 3D analysis / synthesis LEVELS for filters up to 8 taps (db1-db4, sym2-sym4, coif1; every
// boundary mode): one launch per level instead of the three per-axis passes (and their two
// intermediate volumes in HBM) of dwt_axis.hip -- the wavedec3 / waverec3 / adjoint the reference
// reaches through ptwt with non-Haar wavelets (lib/wam_3D.py:194,206,222,620; Haar with sizes
// divisible by 2^J, J <= 2, has the all-levels block kernels of dwt3_haar.hip).
//
// Analysis: a 512-thread workgroup owns a TD x TH x TW tile of every subband of the level. It loads
// the tile's input footprint ((2T + L - 2) samples per axis; the boundary extension of each axis
// resolved once into a small LDS index table, zero where the mode extends by zeros) into LDS, filters
// it along W (lo, hi), H and D there and writes the 8 subbands.
// Synthesis: a workgroup owns a TD x TH x TW tile of the level's output. With ptwt's padding
// (p = L - 2) output t of an axis takes, for j = 0 .. L/2 - 1, tap 2j + (t & 1) against coefficient
// t / 2 + (L - 2) / 2 - j -- a polyphase form with compile-time taps in registers; the 8 subbands'
// coefficient footprints (T/2 + L/2 - 1 per axis, zero outside the band: a zero tap leaves the fmaf
// chain unchanged, as the per-axis kernel's skipped taps do) are loaded once, then synthesised along
// W, H and D in LDS, two outputs (both parities) per thread and pass.
// Arithmetic follows the per-axis kernels exactly (axis order W, H, D; every output an fmaf chain
// from 0 in the same tap order; the IG scales applied at the W pass as `s * value`), so results are
// bit-identical to the generic path (tests/test_gpu_dwt.py). Longer filters keep the per-axis kernels:
// their footprints leave too little of a tile in LDS to beat them (measured: sym8 2.4-8x slower in a
// cubic-tile form, profiles/r06k_kbench_3d.log).
#include "kernels.hpp"

namespace {

constexpr int kT3T = 512;  // threads per workgroup

// analysis tiles (outputs per axis D, H, W): <= 48 KB of static LDS, two workgroups per CU
template <int L> struct AnaTile { static constexpr int D = 4, H = 8, W = L <= 4 ? 16 : 8; };
// synthesis tiles: outputs per axis
constexpr int kSD = 8, kSH = 8, kSW = 16;

struct Tile3Geom {
  int nd, nh, nw;        // level input dims (analysis) / output dims (synthesis)
  int md, mh, mw;        // subband dims
  int pad;               // p->pad = L - 2
  int mode;
  int td, th, tw;        // tiles per axis
  int64_t items;
};

struct Tile3Bands {
  float* b[8];           // subband pointers by key = (D hi) 4 | (H hi) 2 | (W hi) 1 (analysis outputs)
  const float* c[8];     // the same for synthesis inputs
  float s[8];            // synthesis scales (IG alpha on the approximation / details; 1 otherwise)
};

// ------------------------------------------------------------------------------------- analysis
template <int L>
__global__ void __launch_bounds__(kT3T) k_dwt3_ana_tile(const float* __restrict__ in, Tile3Bands bands,
                                                        const float* __restrict__ filt, Tile3Geom g) {
  constexpr int TD = AnaTile<L>::D, TH = AnaTile<L>::H, TW = AnaTile<L>::W;
  constexpr int FD = 2 * TD + L - 2, FH = 2 * TH + L - 2, FW = 2 * TW + L - 2;  // footprint
  __shared__ float xs[FD * FH * FW];         // input footprint; reused for the H-pass output
  __shared__ float ws[FD * FH * TW * 2];     // W-pass output [fd][fh][j][lo/hi]
  __shared__ int ext[FD + FH + FW];          // source index per footprint position and axis (-1: zero)
  const int tid = threadIdx.x;
  int64_t t = blockIdx.x;
  const int bw = (int)(t % g.tw);
  t /= g.tw;
  const int bh = (int)(t % g.th);
  t /= g.th;
  const int bd = (int)(t % g.td);
  const int64_t item = t / g.td;
  const int d0 = bd * TD, h0 = bh * TH, w0 = bw * TW;  // first output index per axis
  const float* src = in + item * ((int64_t)g.nd * g.nh * g.nw);
  float flo[L], fhi[L];
#pragma unroll
  for (int k = 0; k < L; ++k) {
    flo[k] = filt[k];
    fhi[k] = filt[L + k];
  }
  if (tid < FD) ext[tid] = wam_ext_index(2 * d0 - g.pad + tid, g.nd, g.mode);
  else if (tid < FD + FH) ext[tid] = wam_ext_index(2 * h0 - g.pad + tid - FD, g.nh, g.mode);
  else if (tid < FD + FH + FW) ext[tid] = wam_ext_index(2 * w0 - g.pad + tid - FD - FH, g.nw, g.mode);
  __syncthreads();
  // 1. footprint
  for (int e = tid; e < FD * FH * FW; e += kT3T) {
    const int fw = e % FW, fh = (e / FW) % FH, fd = e / (FW * FH);
    const int sd = ext[fd], sh = ext[FD + fh], sw = ext[FD + FH + fw];
    xs[e] = (sd >= 0 && sh >= 0 && sw >= 0) ? src[((int64_t)sd * g.nh + sh) * g.nw + sw] : 0.f;
  }
  __syncthreads();
  // 2. W pass: (fd, fh, j) -> lo, hi
  for (int e = tid; e < FD * FH * TW; e += kT3T) {
    const int j = e % TW, r = e / TW;  // r = fd * FH + fh
    const float* x = xs + r * FW + 2 * j;
    float a = 0.f, d = 0.f;
#pragma unroll
    for (int k = 0; k < L; ++k) {
      a = fmaf(flo[k], x[k], a);
      d = fmaf(fhi[k], x[k], d);
    }
    ws[2 * e] = a;
    ws[2 * e + 1] = d;
  }
  __syncthreads();
  // 3. H pass: (fd, i, j, wbit) -> lo (H), hi (H), into xs as [fd][i][j][wbit][hbit]
  for (int e = tid; e < FD * TH * TW * 2; e += kT3T) {
    const int wb = e & 1, j = (e >> 1) % TW, i = ((e >> 1) / TW) % TH, fd = (e >> 1) / (TW * TH);
    const float* x = ws + ((fd * FH + 2 * i) * TW + j) * 2 + wb;
    float a = 0.f, d = 0.f;
#pragma unroll
    for (int k = 0; k < L; ++k) {
      const float v = x[k * TW * 2];
      a = fmaf(flo[k], v, a);
      d = fmaf(fhi[k], v, d);
    }
    xs[2 * e] = a;
    xs[2 * e + 1] = d;
  }
  __syncthreads();
  // 4. D pass: (i_d, i_h, j, wbit, hbit) -> the 8 subbands (j fastest: row runs of each band)
  const int64_t bn = (int64_t)g.md * g.mh * g.mw;
  for (int e = tid; e < TD * TH * TW * 4; e += kT3T) {
    const int j = e % TW, wb = (e / TW) & 1, hb = (e / (2 * TW)) & 1, i = (e / (4 * TW)) % TH, q = e / (4 * TW * TH);
    const int od = d0 + q, oh = h0 + i, ow = w0 + j;
    const float* x = xs + (((2 * q) * TH + i) * TW + j) * 4 + wb * 2 + hb;  // [fd][i][j][wb][hb]
    float a = 0.f, d = 0.f;
#pragma unroll
    for (int k = 0; k < L; ++k) {
      const float v = x[k * TH * TW * 4];
      a = fmaf(flo[k], v, a);
      d = fmaf(fhi[k], v, d);
    }
    if (od < g.md && oh < g.mh && ow < g.mw) {
      const int64_t o = item * bn + ((int64_t)od * g.mh + oh) * g.mw + ow;
      const int key = (hb << 1) | wb;
      bands.b[key][o] = a;
      bands.b[4 | key][o] = d;
    }
  }
}

// ------------------------------------------------------------------------------------ synthesis
// one axis of the polyphase synthesis: outputs 2u, 2u + 1 from the L/2 coefficient pairs
// (a[u + H2 - 1 - j], d[...]) at stride st, j = 0 .. H2 - 1 (the per-axis kernel's descending
// coefficient order), taps 2j (even output) and 2j + 1 (odd output)
template <int L>
__device__ __forceinline__ void syn_pair(const float* a, const float* d, int st, float sa, float sd,
                                         const float (&rlo)[L], const float (&rhi)[L], float& y0, float& y1) {
  constexpr int H2 = L / 2;
  y0 = 0.f;
  y1 = 0.f;
#pragma unroll
  for (int j = 0; j < H2; ++j) {
    const float av = sa * a[(H2 - 1 - j) * st], dv = sd * d[(H2 - 1 - j) * st];
    y0 = fmaf(rlo[2 * j], av, y0);
    y0 = fmaf(rhi[2 * j], dv, y0);
    y1 = fmaf(rlo[2 * j + 1], av, y1);
    y1 = fmaf(rhi[2 * j + 1], dv, y1);
  }
}

template <int L>
__global__ void __launch_bounds__(kT3T) k_dwt3_syn_tile(Tile3Bands bands, float* __restrict__ out,
                                                        const float* __restrict__ filt, Tile3Geom g) {
  constexpr int H2 = L / 2;
  constexpr int CD = kSD / 2 + H2 - 1, CH = kSH / 2 + H2 - 1, CW = kSW / 2 + H2 - 1;  // footprints
  __shared__ float cs[8 * CD * CH * CW];   // [key][cd][ch][cw]; later the H pass [dbit][cd][y][x]
  __shared__ float ws[4 * CD * CH * kSW];  // W pass [(dbit, hbit)][cd][ch][x]
  const int tid = threadIdx.x;
  int64_t t = blockIdx.x;
  const int bw = (int)(t % g.tw);
  t /= g.tw;
  const int bh = (int)(t % g.th);
  t /= g.th;
  const int bd = (int)(t % g.td);
  const int64_t item = t / g.td;
  const int d0 = bd * kSD, h0 = bh * kSH, w0 = bw * kSW;
  // footprint of an axis starts at coefficient t0 / 2 (p = L - 2, t0 even)
  const int cd0 = d0 / 2, ch0 = h0 / 2, cw0 = w0 / 2;
  float rlo[L], rhi[L];
#pragma unroll
  for (int k = 0; k < L; ++k) {
    rlo[k] = filt[k];
    rhi[k] = filt[L + k];
  }
  const int64_t bn = (int64_t)g.md * g.mh * g.mw;
  // 1. coefficient footprints (outside the band: zero)
  for (int e = tid; e < 8 * CD * CH * CW; e += kT3T) {
    const int cw = e % CW, ch = (e / CW) % CH, cd = (e / (CW * CH)) % CD, key = e / (CW * CH * CD);
    const int id = cd0 + cd, ih = ch0 + ch, iw = cw0 + cw;
    const bool ok = id < g.md && ih < g.mh && iw < g.mw;
    cs[e] = ok ? bands.c[key][item * bn + ((int64_t)id * g.mh + ih) * g.mw + iw] : 0.f;
  }
  __syncthreads();
  // 2. W pass: ((dbit, hbit), cd, ch, u) -> outputs x = 2u, 2u + 1
  for (int e = tid; e < 4 * CD * CH * (kSW / 2); e += kT3T) {
    const int u = e % (kSW / 2), r = e / (kSW / 2);  // r = (dh * CD + cd) * CH + ch
    const int dh = r / (CD * CH), rr = r % (CD * CH);
    const int ka = dh << 1, kd = ka | 1;
    const float* pa = cs + (ka * CD * CH + rr) * CW + u;
    const float* pd = cs + (kd * CD * CH + rr) * CW + u;
    float y0, y1;
    syn_pair<L>(pa, pd, 1, bands.s[ka], bands.s[kd], rlo, rhi, y0, y1);
    ws[r * kSW + 2 * u] = y0;
    ws[r * kSW + 2 * u + 1] = y1;
  }
  __syncthreads();
  // 3. H pass: (dbit, cd, v, x) -> outputs y = 2v, 2v + 1, into cs as [dbit][cd][y][x]
  for (int e = tid; e < 2 * CD * (kSH / 2) * kSW; e += kT3T) {
    const int x = e % kSW, v = (e / kSW) % (kSH / 2), cd = (e / (kSW * (kSH / 2))) % CD, db = e / (kSW * (kSH / 2) * CD);
    const float* pa = ws + (((db * 2 + 0) * CD + cd) * CH + v) * kSW + x;
    const float* pd = ws + (((db * 2 + 1) * CD + cd) * CH + v) * kSW + x;
    float y0, y1;
    syn_pair<L>(pa, pd, kSW, 1.0f, 1.0f, rlo, rhi, y0, y1);
    float* o = cs + ((db * CD + cd) * kSH + 2 * v) * kSW + x;
    o[0] = y0;
    o[kSW] = y1;
  }
  __syncthreads();
  // 4. D pass: (z pair, y, x) -> the output tile
  const int64_t ob = (int64_t)g.nd * g.nh * g.nw;
  for (int e = tid; e < (kSD / 2) * kSH * kSW; e += kT3T) {
    const int x = e % kSW, yy = (e / kSW) % kSH, zp = e / (kSW * kSH);
    const float* pa = cs + ((0 * CD + zp) * kSH + yy) * kSW + x;
    const float* pd = cs + ((1 * CD + zp) * kSH + yy) * kSW + x;
    float y0, y1;
    syn_pair<L>(pa, pd, kSH * kSW, 1.0f, 1.0f, rlo, rhi, y0, y1);
    const int oh = h0 + yy, ow = w0 + x;
    if (oh < g.nh && ow < g.nw) {
      const int od = d0 + 2 * zp;
      float* o = out + item * ob + ((int64_t)od * g.nh + oh) * g.nw + ow;
      if (od < g.nd) o[0] = y0;
      if (od + 1 < g.nd) o[(int64_t)g.nh * g.nw] = y1;
    }
  }
}

template <int L>
int launch_ana3(const Tile3Geom& g0, const float* in, const Tile3Bands& b, const float* filt, hipStream_t st) {
  Tile3Geom g = g0;
  g.td = (g.md + AnaTile<L>::D - 1) / AnaTile<L>::D;
  g.th = (g.mh + AnaTile<L>::H - 1) / AnaTile<L>::H;
  g.tw = (g.mw + AnaTile<L>::W - 1) / AnaTile<L>::W;
  const int64_t blocks = g.items * g.td * g.th * g.tw;
  if (blocks == 0) return WAM_OK;
  if (blocks > 0x7fffffff) return WAM_ERR_UNSUPPORTED;
  WamTimer tm(st, "k_dwt3_ana_tile",
              4.0 * (double)g.items * ((double)g.nd * g.nh * g.nw + 8.0 * g.md * g.mh * g.mw));
  hipLaunchKernelGGL(k_dwt3_ana_tile<L>, dim3((unsigned)blocks), dim3(kT3T), 0, st, in, b, filt, g);
  WAM_LAUNCH_CHECK();
  return WAM_OK;
}

template <int L>
int launch_syn3(const Tile3Geom& g0, const Tile3Bands& b, float* out, const float* filt, hipStream_t st) {
  Tile3Geom g = g0;
  g.td = (g.nd + kSD - 1) / kSD;
  g.th = (g.nh + kSH - 1) / kSH;
  g.tw = (g.nw + kSW - 1) / kSW;
  const int64_t blocks = g.items * g.td * g.th * g.tw;
  if (blocks == 0) return WAM_OK;
  if (blocks > 0x7fffffff) return WAM_ERR_UNSUPPORTED;
  WamTimer tm(st, "k_dwt3_syn_tile",
              4.0 * (double)g.items * (8.0 * g.md * g.mh * g.mw + (double)g.nd * g.nh * g.nw));
  hipLaunchKernelGGL(k_dwt3_syn_tile<L>, dim3((unsigned)blocks), dim3(kT3T), 0, st, b, out, filt, g);
  WAM_LAUNCH_CHECK();
  return WAM_OK;
}

bool tile3_ok(const wam_plan* p) {
  return p->ndim == 3 && p->L >= 2 && p->L <= 8 && !(p->L & 1) && p->pad == p->L - 2 &&
         !(p->flags & WAM_PLAN_GENERIC);
}

}  // namespace

bool dwt3_tile_supported(const wam_plan* p) { return tile3_ok(p); }

int launch_dwt3_analysis_tile(const wam_plan* p, int64_t batch, const float* in, const int64_t* in_dims,
                              const int64_t* out_dims, int mode, int fset, float* out_a, float* const* sub,
                              hipStream_t st) {
  if (!tile3_ok(p)) return WAM_ERR_UNSUPPORTED;
  for (int a = 0; a < 3; ++a)
    if (in_dims[a] >= (int64_t(1) << 30) || out_dims[a] >= (int64_t(1) << 30)) return WAM_ERR_UNSUPPORTED;
  Tile3Geom g{};
  g.nd = (int)in_dims[0], g.nh = (int)in_dims[1], g.nw = (int)in_dims[2];
  g.md = (int)out_dims[0], g.mh = (int)out_dims[1], g.mw = (int)out_dims[2];
  g.pad = p->pad;
  g.mode = mode;
  g.items = batch;
  Tile3Bands b{};
  b.b[0] = out_a;
  for (int key = 1; key < 8; ++key) b.b[key] = sub[key - 1];  // 3D: sub index = key - 1
  const float* filt = p->d_filt + fset * p->L;  // fset, fset + 1: lo then hi, adjacent
  switch (p->L) {
    case 2: return launch_ana3<2>(g, in, b, filt, st);
    case 4: return launch_ana3<4>(g, in, b, filt, st);
    case 6: return launch_ana3<6>(g, in, b, filt, st);
    case 8: return launch_ana3<8>(g, in, b, filt, st);
    default: return WAM_ERR_UNSUPPORTED;
  }
}

int launch_dwt3_synthesis_tile(const wam_plan* p, int64_t batch, int level, const float* a_in, float a_scale,
                               const float* const* sub, float d_scale, float* out, hipStream_t st) {
  if (!tile3_ok(p)) return WAM_ERR_UNSUPPORTED;
  Tile3Geom g{};
  g.md = (int)p->lout[level][0], g.mh = (int)p->lout[level][1], g.mw = (int)p->lout[level][2];
  int64_t n[3];
  for (int a = 0; a < 3; ++a) {
    n[a] = 2 * p->lout[level][a] - 2 + p->L - 2 * p->pad - p->extra[level][a];
    if (n[a] >= (int64_t(1) << 30)) return WAM_ERR_UNSUPPORTED;
  }
  g.nd = (int)n[0], g.nh = (int)n[1], g.nw = (int)n[2];
  g.pad = p->pad;
  g.items = batch;
  Tile3Bands b{};
  b.c[0] = a_in;
  b.s[0] = a_scale;
  for (int key = 1; key < 8; ++key) {
    b.c[key] = sub[key - 1];
    b.s[key] = d_scale;
  }
  const float* filt = p->d_filt + WAM_F_SYN_LO * p->L;  // synthesis lo, then hi
  switch (p->L) {
    case 2: return launch_syn3<2>(g, b, out, filt, st);
    case 4: return launch_syn3<4>(g, b, out, filt, st);
    case 6: return launch_syn3<6>(g, b, out, filt, st);
    case 8: return launch_syn3<8>(g, b, out, filt, st);
    default: return WAM_ERR_UNSUPPORTED;
  }
}

// Fused 3D analysis / synthesis LEVELS for any even filter length (db-N, sym-N, coif-N; every
// boundary mode): one launch per level instead of the three per-axis passes (and their two
// intermediate volumes in HBM) of dwt_axis.hip -- the wavedec3 / waverec3 the reference calls with
// non-Haar wavelets (lib/wam_3D.py:194,206,222,620; Haar J <= 2 has the all-levels block kernels of
// dwt3_haar.hip).
//
// Analysis: a 512-thread workgroup owns a T x T x T tile of every subband of the level. It loads the
// tile's input footprint ((2T + L - 2)^3 samples, the boundary extension applied per axis on the
// load, zero where the mode extends by zeros) into LDS once, then filters it along W (lo, hi), H and
// D in LDS and writes the 8 subbands. Synthesis: a workgroup owns a T x T x T tile of the level's
// output; it loads the 8 subbands' coefficient footprints (T/2 + L/2 per axis), synthesises along W,
// H and D in LDS and writes the tile. Arithmetic follows the per-axis kernels exactly (axis order W,
// H, D; every output an fmaf chain from 0 in the same tap order; the IG scales applied at the W
// pass as `s * value`), so results are bit-identical to the generic path.
//
// Tiles: T = 8 for L <= 6, 6 at L = 8 (footprint 20^3 = 32 KB of LDS), 4 for L <= 16 (22^3 at
// L = 16): at most 58 KB of static LDS, two 512-thread workgroups per CU; longer filters keep the
// per-axis kernels.
#include "kernels.hpp"

namespace {

constexpr int kT3T = 512;  // threads per workgroup

template <int L>
constexpr int tile3() { return L <= 6 ? 8 : (L == 8 ? 6 : 4); }

struct Tile3Geom {
  int nd, nh, nw;        // level input dims (analysis) / output dims (synthesis)
  int md, mh, mw;        // subband dims
  int pad;               // p->pad (analysis: left extension; synthesis: crop)
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
  constexpr int T = tile3<L>();
  constexpr int F = 2 * T + L - 2;  // footprint per axis
  __shared__ float xs[F * F * F];          // input footprint; reused for the H-pass output
  __shared__ float ws[F * F * T * 2];      // W-pass output [fd][fh][j][lo/hi]
  const int tid = threadIdx.x;
  int64_t t = blockIdx.x;
  const int bw = (int)(t % g.tw);
  t /= g.tw;
  const int bh = (int)(t % g.th);
  t /= g.th;
  const int bd = (int)(t % g.td);
  const int64_t item = t / g.td;
  const int d0 = bd * T, h0 = bh * T, w0 = bw * T;  // first output index per axis
  const float* src = in + item * ((int64_t)g.nd * g.nh * g.nw);
  float flo[L], fhi[L];
#pragma unroll
  for (int k = 0; k < L; ++k) {
    flo[k] = filt[k];
    fhi[k] = filt[L + k];
  }
  // 1. footprint (extension per axis on the load)
  for (int e = tid; e < F * F * F; e += kT3T) {
    const int fw = e % F, fh = (e / F) % F, fd = e / (F * F);
    const int sd = wam_ext_index(2 * d0 - g.pad + fd, g.nd, g.mode);
    const int sh = wam_ext_index(2 * h0 - g.pad + fh, g.nh, g.mode);
    const int sw = wam_ext_index(2 * w0 - g.pad + fw, g.nw, g.mode);
    xs[e] = (sd >= 0 && sh >= 0 && sw >= 0) ? src[((int64_t)sd * g.nh + sh) * g.nw + sw] : 0.f;
  }
  __syncthreads();
  // 2. W pass: (fd, fh, j) -> lo, hi
  for (int e = tid; e < F * F * T; e += kT3T) {
    const int j = e % T, r = e / T;  // r = fd * F + fh
    const float* x = xs + r * F + 2 * j;
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
  for (int e = tid; e < F * T * T * 2; e += kT3T) {
    const int wb = e & 1, j = (e >> 1) % T, i = ((e >> 1) / T) % T, fd = (e >> 1) / (T * T);
    const float* x = ws + ((fd * F + 2 * i) * T + j) * 2 + wb;
    float a = 0.f, d = 0.f;
#pragma unroll
    for (int k = 0; k < L; ++k) {
      const float v = x[k * T * 2];
      a = fmaf(flo[k], v, a);
      d = fmaf(fhi[k], v, d);
    }
    xs[2 * e] = a;
    xs[2 * e + 1] = d;
  }
  __syncthreads();
  // 4. D pass: (i_d, i_h, j, wbit, hbit) -> the 8 subbands
  const int64_t bn = (int64_t)g.md * g.mh * g.mw;
  for (int e = tid; e < T * T * T * 4; e += kT3T) {
    const int hb = e & 1, wb = (e >> 1) & 1, j = (e >> 2) % T, i = ((e >> 2) / T) % T, q = (e >> 2) / (T * T);
    const int od = d0 + q, oh = h0 + i, ow = w0 + j;
    const float* x = xs + (((2 * q) * T + i) * T + j) * 4 + wb * 2 + hb;  // [fd][i][j][wb][hb]
    float a = 0.f, d = 0.f;
#pragma unroll
    for (int k = 0; k < L; ++k) {
      const float v = x[k * T * T * 4];
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
// output t of one axis (uncropped position tt = t + pad) takes coefficients i in
// [ceil((tt - L + 1) / 2), floor(tt / 2)] within [0, m), in descending order (the per-axis kernel's)
template <int L>
__global__ void __launch_bounds__(kT3T) k_dwt3_syn_tile(Tile3Bands bands, float* __restrict__ out,
                                                        const float* __restrict__ filt, Tile3Geom g) {
  constexpr int T = tile3<L>();
  constexpr int C = T / 2 + L / 2;  // coefficient footprint per axis
  __shared__ float cs[8 * C * C * C];   // the 8 subbands' footprints [key][cd][ch][cw]
  __shared__ float ws[4 * C * C * T];   // W pass [dh key][cd][ch][x]; later the H pass [d key][cd][y][x]
  const int tid = threadIdx.x;
  int64_t t = blockIdx.x;
  const int bw = (int)(t % g.tw);
  t /= g.tw;
  const int bh = (int)(t % g.th);
  t /= g.th;
  const int bd = (int)(t % g.td);
  const int64_t item = t / g.td;
  const int d0 = bd * T, h0 = bh * T, w0 = bw * T;
  // first coefficient of the footprint per axis: ceil((t0 + pad - L + 1) / 2)
  auto c0 = [&](int t0) { const int v = t0 + g.pad - L + 2; return v >= 0 ? v / 2 : -((1 - v) / 2); };
  const int cd0 = c0(d0), ch0 = c0(h0), cw0 = c0(w0);
  // taps are picked by a data-dependent index (k = tt - 2 i): LDS, not a register array (scratch)
  __shared__ float fs[2 * L];
  if (tid < 2 * L) fs[tid] = filt[tid];
  const float* rlo = fs;
  const float* rhi = fs + L;
  const int64_t bn = (int64_t)g.md * g.mh * g.mw;
  // 1. coefficient footprints (outside [0, m): never read by a tap, zero-filled)
  for (int e = tid; e < 8 * C * C * C; e += kT3T) {
    const int cw = e % C, ch = (e / C) % C, cd = (e / (C * C)) % C, key = e / (C * C * C);
    const int id = cd0 + cd, ih = ch0 + ch, iw = cw0 + cw;
    const bool ok = id >= 0 && id < g.md && ih >= 0 && ih < g.mh && iw >= 0 && iw < g.mw;
    cs[e] = ok ? bands.c[key][item * bn + ((int64_t)id * g.mh + ih) * g.mw + iw] : 0.f;
  }
  __syncthreads();
  // taps of output position t0 + o along an axis: coefficient i (footprint index i - c0) with
  // k = tt - 2 i, i from min(floor(tt / 2), m - 1) down to max(ceil((tt - L + 1) / 2), 0)
  // 2. W pass: for each (D, H) key pair, footprint (cd, ch) and output x -> ws[dh][cd][ch][x]
  for (int e = tid; e < 4 * C * C * T; e += kT3T) {
    const int x = e % T, ch = (e / T) % C, cd = (e / (T * C)) % C, dh = e / (T * C * C);
    const int tt = w0 + x + g.pad;
    int imax = tt >> 1;
    if (imax > g.mw - 1) imax = g.mw - 1;
    int imin = (tt - L + 2) >> 1;
    if (imin < 0) imin = 0;
    const int ka = dh << 1, kd = ka | 1;  // keys (D, H, W lo) and (D, H, W hi)
    const float* pa = cs + ((ka * C + cd) * C + ch) * C - cw0;
    const float* pd = cs + ((kd * C + cd) * C + ch) * C - cw0;
    const float sa = bands.s[ka], sd = bands.s[kd];
    float y = 0.f;
    for (int i = imax; i >= imin; --i) {
      const int k = tt - 2 * i;
      y = fmaf(rlo[k], sa * pa[i], y);
      y = fmaf(rhi[k], sd * pd[i], y);
    }
    ws[e] = y;
  }
  __syncthreads();
  // 3. H pass: for each D key, footprint cd, output (y, x) -> cs[d][cd][y][x] (the footprints are dead)
  for (int e = tid; e < 2 * C * T * T; e += kT3T) {
    const int x = e % T, yy = (e / T) % T, cd = (e / (T * T)) % C, db = e / (T * T * C);
    const int tt = h0 + yy + g.pad;
    int imax = tt >> 1;
    if (imax > g.mh - 1) imax = g.mh - 1;
    int imin = (tt - L + 2) >> 1;
    if (imin < 0) imin = 0;
    const float* pa = ws + (((db * 2 + 0) * C + cd) * C) * T + x;  // dh = db * 2 + hbit
    const float* pd = ws + (((db * 2 + 1) * C + cd) * C) * T + x;
    float y = 0.f;
    for (int i = imax; i >= imin; --i) {
      const int k = tt - 2 * i;
      y = fmaf(rlo[k], 1.0f * pa[(i - ch0) * T], y);
      y = fmaf(rhi[k], 1.0f * pd[(i - ch0) * T], y);
    }
    cs[e] = y;
  }
  __syncthreads();
  // 4. D pass -> the output tile
  const int64_t ob = (int64_t)g.nd * g.nh * g.nw;
  for (int e = tid; e < T * T * T; e += kT3T) {
    const int x = e % T, yy = (e / T) % T, z = e / (T * T);
    const int od = d0 + z, oh = h0 + yy, ow = w0 + x;
    const int tt = od + g.pad;
    int imax = tt >> 1;
    if (imax > g.md - 1) imax = g.md - 1;
    int imin = (tt - L + 2) >> 1;
    if (imin < 0) imin = 0;
    const float* pa = cs + (0 * C * T * T) + yy * T + x;
    const float* pd = cs + (1 * C * T * T) + yy * T + x;
    float y = 0.f;
    for (int i = imax; i >= imin; --i) {
      const int k = tt - 2 * i;
      y = fmaf(rlo[k], 1.0f * pa[(i - cd0) * T * T], y);
      y = fmaf(rhi[k], 1.0f * pd[(i - cd0) * T * T], y);
    }
    if (od < g.nd && oh < g.nh && ow < g.nw) out[item * ob + ((int64_t)od * g.nh + oh) * g.nw + ow] = y;
  }
}

template <int L>
int launch_ana3(const Tile3Geom& g0, const float* in, const Tile3Bands& b, const float* filt, hipStream_t st) {
  constexpr int T = tile3<L>();
  Tile3Geom g = g0;
  g.td = (g.md + T - 1) / T;
  g.th = (g.mh + T - 1) / T;
  g.tw = (g.mw + T - 1) / T;
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
  constexpr int T = tile3<L>();
  Tile3Geom g = g0;
  g.td = (g.nd + T - 1) / T;
  g.th = (g.nh + T - 1) / T;
  g.tw = (g.nw + T - 1) / T;
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
  return p->ndim == 3 && p->L >= 2 && p->L <= 16 && !(p->L & 1) && !(p->flags & WAM_PLAN_GENERIC);
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
    case 10: return launch_ana3<10>(g, in, b, filt, st);
    case 12: return launch_ana3<12>(g, in, b, filt, st);
    case 14: return launch_ana3<14>(g, in, b, filt, st);
    case 16: return launch_ana3<16>(g, in, b, filt, st);
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
    case 10: return launch_syn3<10>(g, b, out, filt, st);
    case 12: return launch_syn3<12>(g, b, out, filt, st);
    case 14: return launch_syn3<14>(g, b, out, filt, st);
    case 16: return launch_syn3<16>(g, b, out, filt, st);
    default: return WAM_ERR_UNSUPPORTED;
  }
}

// Fused 2D filter-bank kernels for gfx950: one level of analysis (both axes) and one level of
// synthesis (both axes) per launch, "column-strip" layout.
//
// Analysis (k_dwt2_ana): one wave owns 64 output columns (one per lane) and a chunk of R output
// rows of one plane. It walks the extended input rows top to bottom: each row segment
// (128 + L - 2 extended columns, boundary-mapped) is staged through a wave-private LDS row with
// coalesced dword loads, every lane filters its window horizontally (lo/hi along W, LDS reads as
// conflict-free ds_read_b64 pairs) and pushes the two results into a register ring of the last
// L rows; after every second row the ring is filtered vertically into LL / H / V / D. No vertical
// halo is re-read inside a chunk and nothing but the four outputs goes back to HBM. The same
// kernel is the adjoint (zero padding, reverse(rec) filters) used for the backward pass.
//
// Synthesis (k_dwt2_syn): one wave owns 64 coefficient columns and a chunk of coefficient rows and
// runs the streaming level synthesis shared with the plane-resident kernel (wam_rows::syn_stream:
// L/2-row register rings, polyphase vertical pass, LDS float4 exchange, horizontal pass; rows
// fetched 4 ahead, output pairs stored as float2); a strip produces 130 - L output columns. The IG
// path scaling alpha is applied on load.
//
// Waves are independent (no workgroup barriers): 4 waves per 256-thread block, LDS only for the
// wave-private rows, ordered by the wave's own in-order LDS queue (wave-scope fences).
#include "rowtools.hpp"

namespace {

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int L>
__global__ void __launch_bounds__(256) k_dwt2_ana(const float* __restrict__ in, int nh, int nw, int64_t in_plane,
                                                  float* __restrict__ oa, float* __restrict__ oh,
                                                  float* __restrict__ ov, float* __restrict__ od, int mh, int mw,
                                                  int64_t out_plane, int p, int mode,
                                                  const float* __restrict__ filt, int nstrips, int nchunks, int R,
                                                  int64_t total_waves) {
  constexpr int SEGW = 128 + L - 2;
  __shared__ __attribute__((aligned(16))) float seg[4][SEGW + 2];
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: SGPR bases
  const int64_t gw = wam_xcd_block(blockIdx.x, gridDim.x) * 4 + wv;
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
  const float* src = in + plane * in_plane;
  const int j0 = strip * 64;
  const int j = j0 + lane;
  const int i0 = chunk * R;
  const int i1 = min(mh, i0 + R);
  const int cbase = 2 * j0 - p;
  int sc[3];
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    int c = lane + 64 * q;
    sc[q] = (c < SEGW) ? wam_ext_index(cbase + c, nw, mode) : -2;
  }
  float* myseg = seg[wv];

  auto row_filter = [&](int er, float& lo, float& hi) {
    int sr = wam_ext_index(er, nh, mode);
    const float* row = src + (int64_t)(sr < 0 ? 0 : sr) * nw;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      if (sc[q] >= -1) {
        float v = (sr >= 0 && sc[q] >= 0) ? row[sc[q]] : 0.f;
        myseg[lane + 64 * q] = v;
      }
    }
    wave_sync();
    const float2* s2 = reinterpret_cast<const float2*>(myseg + 2 * lane);
    float a = 0.f, d = 0.f;
#pragma unroll
    for (int k = 0; k < L; k += 2) {
      float2 v = s2[k >> 1];
      a = fmaf(flo[k], v.x, a);
      d = fmaf(fhi[k], v.x, d);
      a = fmaf(flo[k + 1], v.y, a);
      d = fmaf(fhi[k + 1], v.y, d);
    }
    wave_sync();
    lo = a;
    hi = d;
  };

  float rl[L], rh[L];
#pragma unroll
  for (int k = 0; k < L - 2; ++k) row_filter(2 * i0 - p + k, rl[k], rh[k]);
  for (int i = i0; i < i1; ++i) {
    row_filter(2 * i - p + L - 2, rl[L - 2], rh[L - 2]);
    row_filter(2 * i - p + L - 1, rl[L - 1], rh[L - 1]);
    float a = 0.f, h = 0.f, v = 0.f, d = 0.f;
#pragma unroll
    for (int k = 0; k < L; ++k) {
      a = fmaf(flo[k], rl[k], a);
      h = fmaf(fhi[k], rl[k], h);
      v = fmaf(flo[k], rh[k], v);
      d = fmaf(fhi[k], rh[k], d);
    }
    if (j < mw) {
      int64_t o = plane * out_plane + (int64_t)i * mw + j;
      oa[o] = a;
      oh[o] = h;
      ov[o] = v;
      od[o] = d;
    }
#pragma unroll
    for (int k = 0; k < L - 2; ++k) {
      rl[k] = rl[k + 2];
      rh[k] = rh[k + 2];
    }
  }
}

template <int L>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(L <= 16 ? 4 : 3, 8))) k_dwt2_syn(const float* __restrict__ Hh, const float* __restrict__ Vv,
                                                  const float* __restrict__ Dd, int mh, int mw, SynBatch sb,
                                                  int nh, int nw, const float* __restrict__ filt, int nstrips,
                                                  int nchunks, int RQ, int64_t total_waves) {
  __shared__ __attribute__((aligned(16))) float4 xch[4][64];
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: SGPR bases
  const int64_t gw = wam_xcd_block(blockIdx.x, gridDim.x) * 4 + wv;
  if (gw >= total_waves) return;
  // strip fastest, then alpha: the strips of one (plane, row chunk) -- which fetch the same source
  // rows -- and the alphas of it -- which fetch the same detail rows -- are waves of one or two
  // neighbouring workgroups (one XCD L2, close in time), so the details come from HBM once per
  // launch rather than once per alpha
  const int strip = (int)(gw % nstrips);
  int64_t t = gw / nstrips;
  const int ai = __builtin_amdgcn_readfirstlane((int)(t % sb.na));  // wave-uniform: kernarg index
  t /= sb.na;
  const int chunk = (int)(t % nchunks);
  const int64_t plane = t / nchunks;
  const float* __restrict__ A = sb.a[ai];
  float* __restrict__ out = sb.out[ai];
  const float sa = sb.sa[ai], sd = sb.sd[ai];
  float rlo[L], rhi[L];
#pragma unroll
  for (int k = 0; k < L; ++k) {
    rlo[k] = filt[k];
    rhi[k] = filt[L + k];
  }
  constexpr int qs = (L - 2) >> 1;
  const int qlast = (L - 2 + nh - 1) >> 1;
  const int qbeg = qs + chunk * RQ;
  const int qend = min(qbeg + RQ, qlast + 1);
  const int64_t in_plane = (int64_t)mh * mw;
  // long filters prefetch 3 rows ahead: at 2 the L = 14 / 16 kernels kept 4-5 VGPRs in scratch (128
  // VGPRs, ROCm 7.2), at 3 they need 110 / 122 and none (c4 level 0 at 8 alphas 1,491 -> 1,394 us,
  // profiles/r06h_kc4_*.log); 4 would cost the L = 16 kernel 3 waves per SIMD
  wam_rows::syn_stream<L, (L >= 12 ? 3 : 4)>(A + plane * in_plane, sa, Hh + plane * in_plane, Vv + plane * in_plane, Dd + plane * in_plane,
                          sd, mh, mw, out + plane * (int64_t)nh * nw, nh, nw, strip, qbeg, qend, xch[wv], rlo, rhi,
                          lane, (nw & 1) == 0);
}

constexpr int kTargetWaves = 16384;

template <int L>
int launch_ana_L(int64_t batch, const float* in, int nh, int nw, int mh, int mw, int mode, const float* filt, float* oa,
                 float* oh, float* ov, float* od, int p, hipStream_t st) {
  int nstrips = (mw + 63) / 64;
  int64_t base = batch * nstrips;
  int64_t want = (kTargetWaves + base - 1) / base;
  int maxchunks = (mh + 7) / 8;
  int nchunks = (int)(want < 1 ? 1 : (want > maxchunks ? maxchunks : want));
  if (nchunks < 1) nchunks = 1;
  int R = (mh + nchunks - 1) / nchunks;
  nchunks = (mh + R - 1) / R;
  int64_t waves = base * nchunks;
  int64_t blocks = (waves + 3) / 4;
  WamTimer tm(st, "k_dwt2_ana", 4.0 * (double)batch * ((double)nh * nw + 4.0 * mh * mw));
  hipLaunchKernelGGL(k_dwt2_ana<L>, dim3((unsigned)blocks), dim3(256), 0, st, in, nh, nw, (int64_t)nh * nw, oa, oh, ov,
                     od, mh, mw, (int64_t)mh * mw, p, mode, filt, nstrips, nchunks, R, waves);
  WAM_LAUNCH_CHECK();
  return WAM_OK;
}

template <int L>
int launch_syn_L(int64_t batch, const float* H, const float* V, const float* D, int mh, int mw, const SynBatch& sb,
                 int nh, int nw, int p, const float* filt, hipStream_t st) {
  constexpr int OUTQ = 65 - L / 2;
  int qcols = (nw + 1) / 2;
  int nstrips = (qcols + OUTQ - 1) / OUTQ;
  int nq = (nh + 1) / 2;
  int64_t base = batch * nstrips * sb.na;
  int64_t want = (kTargetWaves + base - 1) / base;
  int maxchunks = (nq + 3) / 4;
  int nchunks = (int)(want < 1 ? 1 : (want > maxchunks ? maxchunks : want));
  if (nchunks < 1) nchunks = 1;
  int RQ = (nq + nchunks - 1) / nchunks;
  nchunks = (nq + RQ - 1) / RQ;
  int64_t waves = base * nchunks;
  int64_t blocks = (waves + 3) / 4;
  // algorithmic bytes: per alpha its LL in and its output, the three detail bands once
  WamTimer tm(st, "k_dwt2_syn", 4.0 * (double)batch * (sb.na * ((double)mh * mw + (double)nh * nw) + 3.0 * mh * mw));
  hipLaunchKernelGGL(k_dwt2_syn<L>, dim3((unsigned)blocks), dim3(256), 0, st, H, V, D, mh, mw, sb, nh, nw, filt,
                     nstrips, nchunks, RQ, waves);
  WAM_LAUNCH_CHECK();
  return WAM_OK;
}

}  // namespace

bool dwt2_fused_supported(const wam_plan* p) {
  // the streaming synthesis addresses a plane with 32-bit byte offsets (rowtools.hpp at32): a plane
  // of 2^30 floats or more would wrap, so such plans take the per-axis kernels
  return p->ndim == 2 && p->L <= 20 && !(p->L & 1) && (p->shape[0] < (1 << 30)) && (p->shape[1] < (1 << 30)) &&
         p->shape[0] * p->shape[1] < (int64_t(1) << 30) && p->rec_shape[0] * p->rec_shape[1] < (int64_t(1) << 30);
}

int launch_dwt2_analysis_fused(const wam_plan* p, int64_t batch, const float* in, const int64_t* in_dims,
                               const int64_t* out_dims, int mode, int fset, float* out_a, float* const* sub,
                               hipStream_t st) {
  const float* filt = p->d_filt + fset * p->L;  // fset, fset+1 are adjacent (lo then hi)
  int nh = (int)in_dims[0], nw = (int)in_dims[1], mh = (int)out_dims[0], mw = (int)out_dims[1];
  // sub order (ptwt): 0 = H ('da': hi along rows), 1 = V ('ad'), 2 = D
  float *oa = out_a, *oh = sub[0], *ov = sub[1], *od = sub[2];
#define WAM_ANA_CASE(LL) \
  case LL: return launch_ana_L<LL>(batch, in, nh, nw, mh, mw, mode, filt, oa, oh, ov, od, p->pad, st);
  switch (p->L) {
    WAM_ANA_CASE(2) WAM_ANA_CASE(4) WAM_ANA_CASE(6) WAM_ANA_CASE(8) WAM_ANA_CASE(10)
    WAM_ANA_CASE(12) WAM_ANA_CASE(14) WAM_ANA_CASE(16) WAM_ANA_CASE(18) WAM_ANA_CASE(20)
    default: return WAM_ERR_UNSUPPORTED;
  }
#undef WAM_ANA_CASE
}

int launch_dwt2_synthesis_fused(const wam_plan* p, int64_t batch, int level, const SynBatch& sb,
                                const float* const* sub, hipStream_t st) {
  if (sb.na < 1 || sb.na > kSynMaxAlpha) return WAM_ERR_INVALID_ARG;
  const float* filt = p->d_filt + WAM_F_SYN_LO * p->L;
  int mh = (int)p->lout[level][0], mw = (int)p->lout[level][1];
  int nh = (int)(2 * mh - 2 + p->L - 2 * p->pad - p->extra[level][0]);
  int nw = (int)(2 * mw - 2 + p->L - 2 * p->pad - p->extra[level][1]);
#define WAM_SYN_CASE(LL) \
  case LL: return launch_syn_L<LL>(batch, sub[0], sub[1], sub[2], mh, mw, sb, nh, nw, p->pad, filt, st);
  switch (p->L) {
    WAM_SYN_CASE(2) WAM_SYN_CASE(4) WAM_SYN_CASE(6) WAM_SYN_CASE(8) WAM_SYN_CASE(10)
    WAM_SYN_CASE(12) WAM_SYN_CASE(14) WAM_SYN_CASE(16) WAM_SYN_CASE(18) WAM_SYN_CASE(20)
    default: return WAM_ERR_UNSUPPORTED;
  }
#undef WAM_SYN_CASE
}

// Plans, size bookkeeping and the multi-level transform drivers of libwam_hip.so.
//
// Semantics (restated from ptwt, the reference's wavelet dependency):
//   analysis per axis: p = (2L-3)//2, pad (p, p + n%2), m = (n + 2p + n%2 - L)//2 + 1
//   synthesis per axis: conv_transpose stride 2 (length 2m-2+L), crop p at both ends, plus one
//   more at the end when the next finer coefficient is one shorter (ptwt
//   _adjust_padding_at_reconstruction)
//   adjoint of synthesis = zero-padded analysis with reverse(rec) filters.
// 2D transforms run on the fused LDS kernels in dwt2_fused.hip; 1D / 3D (and 2D with filters
// longer than the fused kernels support) run on the generic per-axis kernels in dwt_axis.hip.
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "common.hpp"
#include "kernels.hpp"

extern "C" {

int wam_version(void) { return 2; }

const char* wam_strerror(int status) {
  switch (status) {
    case WAM_OK: return "success";
    case WAM_ERR_INVALID_ARG: return "wam: invalid argument";
    case WAM_ERR_SHAPE: return "wam: shape error (coefficient sizes do not match the plan)";
    case WAM_ERR_UNSUPPORTED: return "wam: unsupported configuration";
    case WAM_ERR_NO_MEMORY: return "wam: out of memory";
    default: break;
  }
  if (status >= WAM_ERR_HIP_BASE) return hipGetErrorString((hipError_t)(status - WAM_ERR_HIP_BASE));
  return "wam: unknown error";
}

int wam_plan_create(wam_plan** out, int ndim, const int64_t* shape, int levels, const double* dec_lo,
                    const double* dec_hi, const double* rec_lo, const double* rec_hi, int L, int mode) {
  return wam_plan_create_ex(out, ndim, shape, levels, dec_lo, dec_hi, rec_lo, rec_hi, L, mode, 0);
}

// geometry of a plan (sizes per level, crop flags, band layout, fp32 filters): host arithmetic only
static int plan_geometry(wam_plan* p, int ndim, const int64_t* shape, int levels, const double* dec_lo,
                         const double* dec_hi, const double* rec_lo, const double* rec_hi, int L, int mode,
                         int flags) {
  if (!shape || !dec_lo || !dec_hi || !rec_lo || !rec_hi) return WAM_ERR_INVALID_ARG;
  if (ndim < 1 || ndim > WAM_MAX_NDIM || levels < 1 || levels > WAM_MAX_LEVELS) return WAM_ERR_INVALID_ARG;
  if (L < 2 || L > WAM_MAX_FILT || (L & 1)) return WAM_ERR_UNSUPPORTED;
  if (mode < WAM_MODE_ZERO || mode > WAM_MODE_PERIODIC) return WAM_ERR_INVALID_ARG;
  p->ndim = ndim;
  p->levels = levels;
  p->L = L;
  p->mode = mode;
  p->flags = flags;
  p->pad = (2 * L - 3) / 2;
  p->device = -1;
  // each axis below 2^31 and the whole item below 2^40 elements: every per-item size and offset
  // (and batch x offset products of sane batches) stays far from int64 overflow
  int64_t vol = 1;
  for (int a = 0; a < ndim; ++a) {
    if (shape[a] < 1 || shape[a] >= (int64_t(1) << 31)) return WAM_ERR_SHAPE;
    p->shape[a] = shape[a];
    if (shape[a] > ((int64_t(1) << 40) - 1) / vol) return WAM_ERR_SHAPE;  // vol * shape[a] >= 2^40
    vol *= shape[a];
  }
  // analysis sizes per level
  for (int a = 0; a < ndim; ++a) {
    int64_t n = shape[a];
    for (int l = 0; l < levels; ++l) {
      p->lin[l][a] = n;
      int64_t m = (n + 2 * p->pad + (n % 2) - L) / 2 + 1;
      if (m < 1) return WAM_ERR_SHAPE;
      p->lout[l][a] = m;
      n = m;
    }
  }
  // synthesis crop flags: level l (0 finest) reconstructs 2m-2+L-2p samples; when a finer level
  // exists its detail length decides whether one more sample is cropped at the end.
  for (int l = levels - 1; l >= 0; --l) {
    for (int a = 0; a < ndim; ++a) {
      int64_t pred = 2 * p->lout[l][a] - 2 + L - 2 * p->pad;
      int e = 0;
      if (l > 0) {
        int64_t next = p->lout[l - 1][a];
        if (next == pred - 1) e = 1;
        else if (next != pred) return WAM_ERR_SHAPE;
      } else {
        p->rec_shape[a] = pred;
      }
      p->extra[l][a] = e;
    }
  }
  // bands
  int per = (1 << ndim) - 1;
  p->nbands = 1 + levels * per;
  int64_t off = 0;
  for (int b = 0; b < p->nbands; ++b) {
    int lvl = (b == 0) ? levels - 1 : levels - 1 - (b - 1) / per;
    for (int a = 0; a < ndim; ++a) p->band_dims[b][a] = p->lout[lvl][a];
    p->band_off[b] = off;
    off += wam_prod(p->band_dims[b], ndim);
  }
  p->band_off[p->nbands] = off;
  // filters (fp32, as ptwt casts the pywt float64 tables to the data dtype)
  for (int k = 0; k < L; ++k) {
    p->h_filt[WAM_F_ANA_LO][k] = (float)dec_lo[L - 1 - k];
    p->h_filt[WAM_F_ANA_HI][k] = (float)dec_hi[L - 1 - k];
    p->h_filt[WAM_F_SYN_LO][k] = (float)rec_lo[k];
    p->h_filt[WAM_F_SYN_HI][k] = (float)rec_hi[k];
    p->h_filt[WAM_F_ADJ_LO][k] = (float)rec_lo[k];
    p->h_filt[WAM_F_ADJ_HI][k] = (float)rec_hi[k];
  }
  return WAM_OK;
}

int wam_plan_create_ex(wam_plan** out, int ndim, const int64_t* shape, int levels, const double* dec_lo,
                       const double* dec_hi, const double* rec_lo, const double* rec_hi, int L, int mode,
                       int flags) {
  if (!out) return WAM_ERR_INVALID_ARG;
  wam_plan* p = (wam_plan*)calloc(1, sizeof(wam_plan));
  if (!p) return WAM_ERR_NO_MEMORY;
  int rc = plan_geometry(p, ndim, shape, levels, dec_lo, dec_hi, rec_lo, rec_hi, L, mode, flags);
  if (rc) {
    free(p);
    return rc;
  }
  hipError_t e = hipGetDevice(&p->device);
  if (e != hipSuccess) { free(p); return WAM_ERR_HIP_BASE + (int)e; }
  e = hipMalloc((void**)&p->d_filt, sizeof(float) * WAM_F_COUNT * L);
  if (e != hipSuccess) { free(p); return WAM_ERR_HIP_BASE + (int)e; }
  std::vector<float> packed(WAM_F_COUNT * L);
  for (int f = 0; f < WAM_F_COUNT; ++f)
    for (int k = 0; k < L; ++k) packed[f * L + k] = p->h_filt[f][k];
  e = hipMemcpy(p->d_filt, packed.data(), sizeof(float) * packed.size(), hipMemcpyHostToDevice);
  if (e != hipSuccess) { (void)hipFree(p->d_filt); free(p); return WAM_ERR_HIP_BASE + (int)e; }
  *out = p;
  return WAM_OK;
}

int wam_plan_create_host(wam_plan** out, int ndim, const int64_t* shape, int levels, const double* dec_lo,
                         const double* dec_hi, const double* rec_lo, const double* rec_hi, int L, int mode,
                         int flags) {
  if (!out) return WAM_ERR_INVALID_ARG;
  wam_plan* p = (wam_plan*)calloc(1, sizeof(wam_plan));
  if (!p) return WAM_ERR_NO_MEMORY;
  int rc = plan_geometry(p, ndim, shape, levels, dec_lo, dec_hi, rec_lo, rec_hi, L, mode, flags);
  if (rc) {
    free(p);
    return rc;
  }
  *out = p;
  return WAM_OK;
}

void wam_plan_destroy(wam_plan* p) {
  if (!p) return;
  if (p->d_filt) (void)hipFree(p->d_filt);
  free(p);
}

int wam_plan_num_bands(const wam_plan* p) { return p ? p->nbands : -WAM_ERR_INVALID_ARG; }

int wam_plan_band_shape(const wam_plan* p, int band, int64_t* dims) {
  if (!p || !dims || band < 0 || band >= p->nbands) return WAM_ERR_INVALID_ARG;
  for (int a = 0; a < p->ndim; ++a) dims[a] = p->band_dims[band][a];
  return WAM_OK;
}

int64_t wam_plan_band_offset(const wam_plan* p, int band) {
  if (!p || band < 0 || band > p->nbands) return -1;
  return p->band_off[band];
}

int64_t wam_plan_coeff_numel(const wam_plan* p) { return p ? p->band_off[p->nbands] : -1; }

int wam_plan_rec_shape(const wam_plan* p, int64_t* dims) {
  if (!p || !dims) return WAM_ERR_INVALID_ARG;
  for (int a = 0; a < p->ndim; ++a) dims[a] = p->rec_shape[a];
  return WAM_OK;
}

}  // extern "C"

// ------------------------------------------------------------------------------------------------
// Generic separable drivers (per-axis kernels). Axis passes go from the last axis to the first;
// intermediate results live in the workspace.
// ------------------------------------------------------------------------------------------------
namespace {

// Size (elements) of the largest intermediate set of one generic analysis level.
int64_t generic_level_tmp(const wam_plan* p, const int64_t* in_dims, const int64_t* out_dims, int64_t batch) {
  int nd = p->ndim;
  int64_t best = 0;
  int64_t dims[WAM_MAX_NDIM];
  for (int a = 0; a < nd; ++a) dims[a] = in_dims[a];
  int parts = 1;
  for (int ax = nd - 1; ax >= 1; --ax) {  // the last pass (ax 0) writes the final outputs
    dims[ax] = out_dims[ax];
    parts *= 2;
    best += parts * batch * wam_prod(dims, nd);
  }
  return best;
}

int64_t generic_syn_tmp(const wam_plan* p, int64_t batch) {
  int nd = p->ndim;
  int64_t best = 0;
  for (int l = p->levels - 1; l >= 0; --l) {
    int64_t dims[WAM_MAX_NDIM];
    for (int a = 0; a < nd; ++a) dims[a] = p->lout[l][a];
    int parts = 1 << nd;
    int64_t tot = 0;
    for (int ax = nd - 1; ax >= 1; --ax) {
      dims[ax] = 2 * p->lout[l][ax] - 2 + p->L - 2 * p->pad - p->extra[l][ax];
      parts /= 2;
      tot += parts * batch * wam_prod(dims, nd);
    }
    if (tot > best) best = tot;
  }
  return best;
}

int sub_of_key(int nd, int key) {
  if (nd == 2) return key == 2 ? 0 : (key == 1 ? 1 : 2);  // (H='da', V='ad', D='dd')
  return key - 1;
}

}  // namespace

// 2D plans whose waverec runs the per-level row synthesis (k_dwt2_syn) rather than the
// plane-resident kernel: their IG alphas are synthesised kSynWsAlpha per level launch
static bool syn_rows_alpha_batched(const wam_plan* p) {
  return p->ndim == 2 && !(p->flags & WAM_PLAN_GENERIC) && dwt2_fused_supported(p) &&
         ((p->flags & (WAM_PLAN_NO_ROWS | WAM_PLAN_NO_PLANE)) || !dwt2_plane_syn_supported(p));
}

// floats per synthesis LL slot (the largest intermediate approximation of the batch), rounded up
// to 4 floats: slots stay 16-byte aligned, so the float2 output stores of the row synthesis
// (rowtools.hpp syn_stream, vec2 on even level widths) land on 8-byte aligned addresses whatever
// the batch and level sizes (an odd count, e.g. db3 at 226^2 with an odd batch, misaligned them)
static int64_t syn_ll_stride(const wam_plan* p, int64_t batch) {
  int64_t rec_ll = 0;
  for (int l = p->levels - 1; l >= 1; --l) {
    const int64_t v = batch * wam_prod(p->lout[l - 1], p->ndim);
    if (v > rec_ll) rec_ll = v;
  }
  return (rec_ll + 3) & ~(int64_t)3;
}

extern "C" int64_t wam_plan_workspace_bytes(const wam_plan* p, int64_t batch) {
  if (!p || batch < 0) return -1;
  int nd = p->ndim;
  // LL ping-pong for analysis / adjoint (level 0 output) and A ping-pong for synthesis
  int64_t ll = batch * wam_prod(p->lout[0], nd);
  const int64_t rec_ll = syn_ll_stride(p, batch);
  int64_t tmp_a = 0;
  int64_t rec0[WAM_MAX_NDIM];
  for (int a = 0; a < nd; ++a) rec0[a] = p->rec_shape[a];
  for (int l = 0; l < p->levels; ++l) {
    int64_t v = generic_level_tmp(p, l == 0 ? rec0 : p->lin[l], p->lout[l], batch);
    int64_t v2 = generic_level_tmp(p, p->lin[l], p->lout[l], batch);
    if (v > tmp_a) tmp_a = v;
    if (v2 > tmp_a) tmp_a = v2;
  }
  int64_t tmp_s = generic_syn_tmp(p, batch);
  int64_t a_side = 2 * ll + tmp_a;
  int64_t s_side = 2 * rec_ll + tmp_s;
  // row-synthesis 2D plans: the LL ping-pong of kSynWsAlpha alphas per level launch
  if (syn_rows_alpha_batched(p) && 2 * kSynWsAlpha * rec_ll > s_side) s_side = 2 * kSynWsAlpha * rec_ll;
  int64_t elems = a_side > s_side ? a_side : s_side;
  return (elems + 64) * (int64_t)sizeof(float);
}

namespace {

// One analysis level over arbitrary ndim via per-axis passes. `in` has dims in_dims; outputs:
// approx -> out_a, details -> bands (pointers per sub index).
int generic_analysis_level(const wam_plan* p, int64_t batch, const float* in, const int64_t* in_dims,
                           const int64_t* out_dims, int mode, int fset, float* out_a, float* const* out_sub,
                           float* tmp, hipStream_t st) {
  int nd = p->ndim;
  const float* flo = p->d_filt + (fset + 0) * p->L;
  const float* fhi = p->d_filt + (fset + 1) * p->L;
  // parts: (key, pointer, dims)
  struct Part { int key; const float* ptr; };
  Part cur[8], nxt[8];
  int ncur = 1;
  cur[0] = {0, in};
  int64_t dims[WAM_MAX_NDIM];
  for (int a = 0; a < nd; ++a) dims[a] = in_dims[a];
  float* tcur = tmp;
  for (int ax = nd - 1; ax >= 0; --ax) {
    int64_t outer = batch;
    for (int a = 0; a < ax; ++a) outer *= dims[a];
    int64_t inner = 1;
    for (int a = ax + 1; a < nd; ++a) inner *= dims[a];
    int n = (int)dims[ax];
    int m = (int)out_dims[ax];
    int64_t odims[WAM_MAX_NDIM];
    for (int a = 0; a < nd; ++a) odims[a] = dims[a];
    odims[ax] = m;
    int64_t part_elems = batch * wam_prod(odims, nd);
    int bit = 1 << (nd - 1 - ax);
    for (int i = 0; i < ncur; ++i) {
      float* lo;
      float* hi;
      int klo = cur[i].key, khi = cur[i].key | bit;
      if (ax == 0) {
        lo = (klo == 0) ? out_a : out_sub[sub_of_key(nd, klo)];
        hi = out_sub[sub_of_key(nd, khi)];
      } else {
        lo = tcur;
        hi = tcur + part_elems;
        tcur += 2 * part_elems;
      }
      int rc = launch_analysis_axis(cur[i].ptr, lo, hi, outer, n, m, inner, p->pad, mode, flo, fhi, p->L, st);
      if (rc) return rc;
      nxt[2 * i] = {klo, lo};
      nxt[2 * i + 1] = {khi, hi};
    }
    ncur *= 2;
    for (int i = 0; i < ncur; ++i) cur[i] = nxt[i];
    for (int a = 0; a < nd; ++a) dims[a] = odims[a];
  }
  return WAM_OK;
}

// One synthesis level (c_pos order handled by the caller). a_in: approximation (band or previous
// output), sub[k]: detail bands; out: cropped result.
int generic_synthesis_level(const wam_plan* p, int64_t batch, int level, const float* a_in, float a_scale,
                            const float* const* sub, float d_scale, float* out, float* tmp, hipStream_t st) {
  int nd = p->ndim;
  const float* rlo = p->d_filt + WAM_F_SYN_LO * p->L;
  const float* rhi = p->d_filt + WAM_F_SYN_HI * p->L;
  struct Part { int key; const float* ptr; float scale; };
  Part cur[8];
  int ncur = 1 << nd;
  for (int key = 0; key < ncur; ++key) {
    if (key == 0) cur[key] = {0, a_in, a_scale};
    else cur[key] = {key, sub[sub_of_key(nd, key)], d_scale};
  }
  int64_t dims[WAM_MAX_NDIM];
  for (int a = 0; a < nd; ++a) dims[a] = p->lout[level][a];
  float* tcur = tmp;
  for (int ax = nd - 1; ax >= 0; --ax) {
    int64_t outer = batch;
    for (int a = 0; a < ax; ++a) outer *= dims[a];
    int64_t inner = 1;
    for (int a = ax + 1; a < nd; ++a) inner *= dims[a];
    int m = (int)dims[ax];
    int nout = (int)(2 * dims[ax] - 2 + p->L - 2 * p->pad - p->extra[level][ax]);
    int64_t odims[WAM_MAX_NDIM];
    for (int a = 0; a < nd; ++a) odims[a] = dims[a];
    odims[ax] = nout;
    int64_t part_elems = batch * wam_prod(odims, nd);
    int bit = 1 << (nd - 1 - ax);
    Part nxt[8];
    int nn = 0;
    for (int i = 0; i < ncur; ++i) {
      if (cur[i].key & bit) continue;
      const Part* pa = &cur[i];
      const Part* pd = nullptr;
      for (int j = 0; j < ncur; ++j)
        if (cur[j].key == (cur[i].key | bit)) pd = &cur[j];
      float* dst = (ax == 0) ? out : tcur;
      if (ax != 0) tcur += part_elems;
      int rc = launch_synthesis_axis(pa->ptr, pd->ptr, dst, outer, m, nout, inner, p->pad, rlo, rhi, p->L,
                                     pa->scale, pd->scale, st);
      if (rc) return rc;
      nxt[nn++] = {cur[i].key, dst, 1.0f};
    }
    ncur = nn;
    for (int i = 0; i < ncur; ++i) cur[i] = nxt[i];
    for (int a = 0; a < nd; ++a) dims[a] = odims[a];
  }
  return WAM_OK;
}

void band_ptrs(const wam_plan* p, int64_t batch, float* coeffs, int level, float** sub) {
  int per = (1 << p->ndim) - 1;
  for (int k = 0; k < per; ++k) sub[k] = coeffs + batch * p->band_off[wam_band_of(p, level, k)];
}

bool use_rows(const wam_plan* p, int level, bool adjoint) {
  return p->ndim == 2 && !(p->flags & (WAM_PLAN_GENERIC | WAM_PLAN_NO_ROWS)) && dwt2_rows_supported(p, level, adjoint);
}

bool use_plane(const wam_plan* p, bool adjoint) {
  return p->ndim == 2 && !(p->flags & (WAM_PLAN_GENERIC | WAM_PLAN_NO_ROWS | WAM_PLAN_NO_PLANE)) &&
         dwt2_plane_supported(p, adjoint);
}

bool use_colstrip(const wam_plan* p) {
  return p->ndim == 2 && !(p->flags & WAM_PLAN_GENERIC) && dwt2_fused_supported(p);
}

// noise (level 0 only): fused SmoothGrad noise on the load; `batch` then counts the virtual
// (sample, image, channel) planes and x holds the clean (image, channel) planes.
int analysis_driver(const wam_plan* p, int64_t batch, const float* x, float* coeffs, void* ws, hipStream_t st,
                    bool adjoint, const WamNoise* noise = nullptr, int64_t n_samples = 1) {
  if (use_plane(p, adjoint)) {  // all levels in one launch, LL pyramid in LDS
    int rc = launch_dwt2_plane_analysis(p, batch, x, coeffs, adjoint, noise, n_samples, st);
    if (rc != WAM_ERR_UNSUPPORTED) return rc;
  }
  if (p->ndim == 1 && !(p->flags & WAM_PLAN_GENERIC)) {  // all levels per signal tile
    int rc = launch_dwt1_tile_analysis(p, batch, x, coeffs, adjoint, st, noise, n_samples);
    if (rc != WAM_ERR_UNSUPPORTED) return rc;
  }
  if (p->ndim == 3 && !(p->flags & WAM_PLAN_GENERIC)) {  // Haar: all levels per block
    int rc = noise ? launch_dwt3_haar_analysis_noisy(p, batch, x, coeffs, noise, n_samples, st)
                   : launch_dwt3_haar_analysis(p, batch, x, coeffs, adjoint, st);
    if (rc != WAM_ERR_UNSUPPORTED) return rc;
  }
  int nd = p->ndim;
  float* w = (float*)ws;
  int64_t ll = batch * wam_prod(p->lout[0], nd);
  float* llbuf[2] = {w, w + ll};
  float* tmp = w + 2 * ll;
  const float* cur = x;
  int mode = adjoint ? WAM_MODE_ZERO : p->mode;
  int fset = adjoint ? WAM_F_ADJ_LO : WAM_F_ANA_LO;
  for (int l = 0; l < p->levels; ++l) {
    int64_t in_dims[WAM_MAX_NDIM];
    for (int a = 0; a < nd; ++a) in_dims[a] = (adjoint && l == 0) ? p->rec_shape[a] : p->lin[l][a];
    float* sub[7];
    band_ptrs(p, batch, coeffs, l, sub);
    float* out_a = (l == p->levels - 1) ? coeffs : llbuf[l & 1];
    const WamNoise* nz = (l == 0) ? noise : nullptr;
    int rc;
    if (use_rows(p, l, adjoint)) {
      rc = launch_dwt2_analysis_rows(p, batch, cur, in_dims, p->lout[l], mode, fset, out_a, sub, nz, st);
    } else if (nz) {
      rc = WAM_ERR_UNSUPPORTED;
    } else if (use_colstrip(p)) {
      rc = launch_dwt2_analysis_fused(p, batch, cur, in_dims, p->lout[l], mode, fset, out_a, sub, st);
    } else {
      rc = WAM_ERR_UNSUPPORTED;
      if (p->ndim == 3 && dwt3_tile_supported(p))  // all three axes of the level in one pass
        rc = launch_dwt3_analysis_tile(p, batch, cur, in_dims, p->lout[l], mode, fset, out_a, sub, st);
      if (rc == WAM_ERR_UNSUPPORTED)
        rc = generic_analysis_level(p, batch, cur, in_dims, p->lout[l], mode, fset, out_a, sub, tmp, st);
    }
    if (rc) return rc;
    cur = out_a;
  }
  return WAM_OK;
}

}  // namespace

extern "C" {

int wam_wavedec(const wam_plan* p, int64_t batch, const float* x, float* coeffs, void* ws, void* stream) {
  if (!p || !p->d_filt || !x || !coeffs || !ws || batch < 0) return WAM_ERR_INVALID_ARG;
  if (batch == 0) return WAM_OK;
  return analysis_driver(p, batch, x, coeffs, ws, (hipStream_t)stream, false);
}

int wam_waverec_adjoint(const wam_plan* p, int64_t batch, const float* grad, float* coeff_grads, void* ws,
                        void* stream) {
  if (!p || !p->d_filt || !grad || !coeff_grads || !ws || batch < 0) return WAM_ERR_INVALID_ARG;
  if (batch == 0) return WAM_OK;
  return analysis_driver(p, batch, grad, coeff_grads, ws, (hipStream_t)stream, true);
}

int wam_plan_caps(const wam_plan* p) {
  if (!p) return 0;
  int caps = 0;
  bool rows_all = true;
  for (int l = 0; l < p->levels; ++l) rows_all = rows_all && use_rows(p, l, true);
  if (rows_all || use_plane(p, true)) caps |= WAM_CAP_ADJOINT_MAPS;
  if (use_plane(p, false) || (use_rows(p, 0, false) && p->lin[0][1] % 4 == 0)) caps |= WAM_CAP_NOISY_WAVEDEC;
  if (p->ndim == 1 && !(p->flags & WAM_PLAN_GENERIC) && dwt1_tile_supported(p, false) && p->lin[0][0] % 4 == 0)
    caps |= WAM_CAP_NOISY_WAVEDEC;  // single-channel signals (channels != 1: WAM_ERR_UNSUPPORTED)
  if (p->ndim == 3 && !(p->flags & WAM_PLAN_GENERIC) && dwt3_haar_supported(p) && p->lin[0][2] % 4 == 0)
    caps |= WAM_CAP_NOISY_WAVEDEC;  // single-channel volumes (channels != 1: WAM_ERR_UNSUPPORTED)
  // the bf16 NHWC model hand-off: plane-resident synthesis and the COOP maps pass of the plane kernel
  if (p->ndim == 2 && !(p->flags & (WAM_PLAN_GENERIC | WAM_PLAN_NO_ROWS | WAM_PLAN_NO_PLANE)) &&
      dwt2_plane_syn_supported(p) && use_plane(p, true) && dwt2_plane_maps_coop(p))
    caps |= WAM_CAP_BF16_NHWC;
  return caps;
}

int wam_wavedec_noisy_ex(const wam_plan* p, int64_t n_samples, int64_t images, int channels, const float* x,
                         const float* sigma, uint64_t seed, int64_t sample_base, int64_t image_base, float* coeffs,
                         void* ws, void* stream) {
  if (!p || !p->d_filt || !x || !sigma || !coeffs || !ws || n_samples < 0 || images < 0 || channels < 1 || image_base < 0)
    return WAM_ERR_INVALID_ARG;
  if (!(wam_plan_caps(p) & WAM_CAP_NOISY_WAVEDEC)) return WAM_ERR_UNSUPPORTED;
  const int64_t batch = n_samples * images * channels;
  if (batch == 0) return WAM_OK;
  WamNoise nz{sigma, images, channels, (uint32_t)seed, (uint32_t)(seed >> 32), sample_base, image_base};
  return analysis_driver(p, batch, x, coeffs, ws, (hipStream_t)stream, false, &nz, n_samples);
}

int wam_wavedec_noisy(const wam_plan* p, int64_t n_samples, int64_t images, int channels, const float* x,
                      const float* sigma, uint64_t seed, int64_t sample_base, float* coeffs, void* ws, void* stream) {
  return wam_wavedec_noisy_ex(p, n_samples, images, channels, x, sigma, seed, sample_base, 0, coeffs, ws, stream);
}

int wam_waverec_adjoint_maps(const wam_plan* p, int64_t groups, int64_t group_items, int channels, const float* grad,
                             float* maps, float* band_max, float* coeff_grads, void* ws, void* stream) {
  if (!p || !p->d_filt || !grad || !maps || !band_max || !ws || groups < 0 || group_items < 0 || channels < 1)
    return WAM_ERR_INVALID_ARG;
  if (!(wam_plan_caps(p) & WAM_CAP_ADJOINT_MAPS) || (channels != 1 && channels != 3)) return WAM_ERR_UNSUPPORTED;
  const int64_t images = groups * group_items;
  if (images == 0) return WAM_OK;
  hipStream_t st = (hipStream_t)stream;
  const int64_t planes = images * channels;
  if (use_plane(p, true)) {
    // maps from the channel-mean gradient (one pass); per-channel grads only when asked for
    int rc = launch_dwt2_plane_maps(p, images, channels, group_items, grad, 0, maps, band_max, st);
    if (rc != WAM_ERR_UNSUPPORTED) {
      if (rc || !coeff_grads) return rc;
      return analysis_driver(p, planes, grad, coeff_grads, ws, st, true);
    }
  }
  // per level (rows kernels): maps from the channel mean taken on the level-0 load (the plane
  // kernels' form: one plane filtered per image at every level); the per-channel coefficient
  // gradients, when asked for, by a separate adjoint afterwards
  float* w = (float*)ws;
  int64_t ll = images * wam_prod(p->lout[0], 2);
  float* llbuf[2] = {w, w + ll};
  const float* cur = grad;
  for (int l = 0; l < p->levels; ++l) {
    int64_t in_dims[2];
    for (int a = 0; a < 2; ++a) in_dims[a] = (l == 0) ? p->rec_shape[a] : p->lin[l][a];
    float* ll_out = (l == p->levels - 1) ? nullptr : llbuf[l & 1];
    const bool mean_first = l == 0 && channels > 1;
    int rc = launch_dwt2_adjoint_maps_level(p, l, images, l == 0 ? channels : 1, mean_first, group_items, cur, in_dims,
                                            ll_out, maps, band_max, nullptr, images, st);
    if (rc) return rc;
    cur = ll_out;
  }
  if (coeff_grads) return analysis_driver(p, planes, grad, coeff_grads, ws, st, true);
  return WAM_OK;
}

int wam_waverec_bf16_nhwc(const wam_plan* p, int64_t batch, const float* coeffs, const float* alpha, int n_alpha,
                          int channels, void* out, void* stream) {
  if (!p || !p->d_filt || !coeffs || !out || batch < 0 || n_alpha < 1 || channels < 1) return WAM_ERR_INVALID_ARG;
  if (!alpha && n_alpha != 1) return WAM_ERR_INVALID_ARG;
  if (!(wam_plan_caps(p) & WAM_CAP_BF16_NHWC) || (channels != 1 && channels != 3)) return WAM_ERR_UNSUPPORTED;
  if (batch % channels) return WAM_ERR_INVALID_ARG;
  if (batch == 0) return WAM_OK;
  return launch_dwt2_plane_synthesis(p, batch, coeffs, alpha, n_alpha, out, channels, (hipStream_t)stream);
}

int wam_waverec_adjoint_maps_bf16(const wam_plan* p, int64_t groups, int64_t group_items, int channels, int nhwc,
                                  const void* grad, float* maps, float* band_max, void* stream) {
  if (!p || !p->d_filt || !grad || !maps || !band_max || groups < 0 || group_items < 0 || channels < 1)
    return WAM_ERR_INVALID_ARG;
  if (!(wam_plan_caps(p) & WAM_CAP_BF16_NHWC) || (channels != 1 && channels != 3)) return WAM_ERR_UNSUPPORTED;
  const int64_t images = groups * group_items;
  if (images == 0) return WAM_OK;
  return launch_dwt2_plane_maps(p, images, channels, group_items, grad, nhwc ? 1 : 2, maps, band_max,
                                (hipStream_t)stream);
}

int wam_waverec_adjoint_maps_bf16_nhwc(const wam_plan* p, int64_t groups, int64_t group_items, int channels,
                                       const void* grad, float* maps, float* band_max, void* stream) {
  return wam_waverec_adjoint_maps_bf16(p, groups, group_items, channels, 1, grad, maps, band_max, stream);
}

int wam_waverec(const wam_plan* p, int64_t batch, const float* coeffs, const float* alpha, int n_alpha, float* out,
                void* ws, void* stream) {
  if (!p || !p->d_filt || !coeffs || !out || !ws || batch < 0 || n_alpha < 1) return WAM_ERR_INVALID_ARG;
  if (!alpha && n_alpha != 1) return WAM_ERR_INVALID_ARG;
  if (batch == 0) return WAM_OK;
  hipStream_t st = (hipStream_t)stream;
  if (p->ndim == 2 && !(p->flags & (WAM_PLAN_GENERIC | WAM_PLAN_NO_ROWS | WAM_PLAN_NO_PLANE)) &&
      dwt2_plane_syn_supported(p)) {  // all levels and all alphas in one launch
    int rc = launch_dwt2_plane_synthesis(p, batch, coeffs, alpha, n_alpha, out, 0, st);
    if (rc != WAM_ERR_UNSUPPORTED) return rc;
  }
  if (p->ndim == 1 && !(p->flags & WAM_PLAN_GENERIC)) {
    int rc = launch_dwt1_tile_synthesis(p, batch, coeffs, alpha, n_alpha, out, st);
    if (rc != WAM_ERR_UNSUPPORTED) return rc;
  }
  if (p->ndim == 3 && !(p->flags & WAM_PLAN_GENERIC)) {
    int rc = launch_dwt3_haar_synthesis(p, batch, coeffs, alpha, n_alpha, out, st);
    if (rc != WAM_ERR_UNSUPPORTED) return rc;
  }
  int nd = p->ndim;
  int64_t out_item = wam_prod(p->rec_shape, nd);
  const int64_t rec_ll = syn_ll_stride(p, batch);
  float* w = (float*)ws;
  if (nd == 2 && !(p->flags & WAM_PLAN_GENERIC) && dwt2_fused_supported(p)) {
    // alphas in groups: one launch per level per group, each level's detail bands read once per
    // group; the group's intermediate LL planes ping-pong between two workspace sets
    const int64_t ws_elems = wam_plan_workspace_bytes(p, batch) / (int64_t)sizeof(float) - 64;
    int64_t g = rec_ll > 0 ? ws_elems / (2 * rec_ll) : kSynWsAlpha;
    const int G = (int)(g < 1 ? 1 : (g > kSynWsAlpha ? kSynWsAlpha : g));
    for (int a0 = 0; a0 < n_alpha; a0 += G) {
      SynBatch sb{};
      sb.na = n_alpha - a0 < G ? n_alpha - a0 : G;
      for (int c = 0; c < p->levels; ++c) {
        const int l = p->levels - 1 - c;
        float* sub[7];
        band_ptrs(p, batch, (float*)coeffs, l, sub);
        for (int i = 0; i < sb.na; ++i) {
          const float s = alpha ? alpha[a0 + i] : 1.0f;
          sb.a[i] = c == 0 ? coeffs : w + (int64_t)(((c - 1) & 1) * G + i) * rec_ll;  // band 0 = A_J
          sb.sa[i] = c == 0 ? s : 1.0f;
          sb.sd[i] = s;
          sb.out[i] = l == 0 ? out + (int64_t)(a0 + i) * batch * out_item : w + (int64_t)((c & 1) * G + i) * rec_ll;
        }
        int rc = launch_dwt2_synthesis_fused(p, batch, l, sb, sub, st);
        if (rc) return rc;
      }
    }
    return WAM_OK;
  }
  float* abuf[2] = {w, w + rec_ll};
  float* tmp = w + 2 * rec_ll;
  for (int ai = 0; ai < n_alpha; ++ai) {
    float s = alpha ? alpha[ai] : 1.0f;
    const float* a_cur = coeffs;  // band 0 = A_J
    float a_scale = s;
    for (int c = 0; c < p->levels; ++c) {
      int l = p->levels - 1 - c;
      float* sub[7];
      band_ptrs(p, batch, (float*)coeffs, l, sub);
      float* dst = (l == 0) ? out + (int64_t)ai * batch * out_item : abuf[c & 1];
      int rc = WAM_ERR_UNSUPPORTED;
      if (nd == 3 && dwt3_tile_supported(p))  // all three axes of the level in one pass
        rc = launch_dwt3_synthesis_tile(p, batch, l, a_cur, a_scale, sub, s, dst, st);
      if (rc == WAM_ERR_UNSUPPORTED) rc = generic_synthesis_level(p, batch, l, a_cur, a_scale, sub, s, dst, tmp, st);
      if (rc) return rc;
      a_cur = dst;
      a_scale = 1.0f;
    }
  }
  return WAM_OK;
}

}  // extern "C"

// ------------------------------------------------------------------------------------------------
// Live per-launch timing (see timing.hpp)
// ------------------------------------------------------------------------------------------------
#include <atomic>
#include <mutex>

namespace {
struct TimingRec {
  const char* name;
  hipEvent_t s, e;
  double bytes;
};
std::atomic<int> g_timing{0};
std::mutex g_timing_mu;
std::vector<TimingRec> g_timing_recs;
}  // namespace

WamTimer::WamTimer(hipStream_t st_, const char* name_, double bytes_) : st(st_), name(name_), bytes(bytes_) {
  if (!g_timing.load(std::memory_order_relaxed)) return;
  if (hipEventCreate(&s) != hipSuccess || hipEventCreate(&e) != hipSuccess) {
    s = e = nullptr;
    return;
  }
  (void)hipEventRecord(s, st);
}

WamTimer::~WamTimer() {
  if (!s) return;
  (void)hipEventRecord(e, st);
  std::lock_guard<std::mutex> lk(g_timing_mu);
  g_timing_recs.push_back({name, s, e, bytes});
}

extern "C" {

int wam_timing_enable(int on) {
  g_timing.store(on ? 1 : 0);
  return WAM_OK;
}

int wam_timing_drain(int max_records, char* names, float* ms, double* bytes) {
  if (max_records < 0 || (max_records > 0 && (!names || !ms || !bytes))) return -WAM_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(g_timing_mu);
  int n = 0;
  for (auto& r : g_timing_recs) {
    if (n < max_records) {
      float t = 0.f;
      if (hipEventSynchronize(r.e) == hipSuccess) (void)hipEventElapsedTime(&t, r.s, r.e);
      strncpy(names + 64 * n, r.name, 63);
      names[64 * n + 63] = 0;
      ms[n] = t;
      bytes[n] = r.bytes;
      ++n;
    }
    (void)hipEventDestroy(r.s);
    (void)hipEventDestroy(r.e);
  }
  g_timing_recs.clear();
  return n;
}

}  // extern "C"

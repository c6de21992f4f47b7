// Shared device/host helpers for libwam_hip.so (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/wam_hip.h"

#define WAM_MAX_NDIM 3
#define WAM_MAX_LEVELS 16
#define WAM_MAX_BANDS (1 + WAM_MAX_LEVELS * 7)
#define WAM_MAX_FILT 128

#define WAM_HIP_CHECK(expr)                                           \
  do {                                                                \
    hipError_t _e = (expr);                                           \
    if (_e != hipSuccess) return WAM_ERR_HIP_BASE + (int)_e;          \
  } while (0)

#define WAM_LAUNCH_CHECK() WAM_HIP_CHECK(hipGetLastError())

// Boundary extension: map an extended-signal position to a source index (-1 = zero padding).
// reflect / symmetric handle any number of reflections (pywt semantics; ptwt's torch 'reflect'
// pad is the single-reflection special case).
__host__ __device__ __forceinline__ int wam_ext_index(int i, int n, int mode) {
  if (i >= 0 && i < n) return i;
  switch (mode) {
    case WAM_MODE_ZERO:
      return -1;
    case WAM_MODE_CONSTANT:
      return i < 0 ? 0 : n - 1;
    case WAM_MODE_PERIODIC: {
      int r = i % n;
      return r < 0 ? r + n : r;
    }
    case WAM_MODE_REFLECT: {
      if (n == 1) return 0;
      int per = 2 * n - 2;
      int r = i % per;
      if (r < 0) r += per;
      return r >= n ? per - r : r;
    }
    default: {  // symmetric
      int per = 2 * n;
      int r = i % per;
      if (r < 0) r += per;
      return r >= n ? per - 1 - r : r;
    }
  }
}

// Filter set as stored on the device by the plan (fp32):
//   [0] analysis lo  = flip(dec_lo)      [1] analysis hi  = flip(dec_hi)
//   [2] synthesis lo = rec_lo            [3] synthesis hi = rec_hi
//   [4] adjoint lo   = flip(reverse(rec_lo)) = rec_lo   [5] adjoint hi = rec_hi
// so "correlate with f[k]" is the common form of analysis and adjoint.
enum { WAM_F_ANA_LO = 0, WAM_F_ANA_HI = 1, WAM_F_SYN_LO = 2, WAM_F_SYN_HI = 3, WAM_F_ADJ_LO = 4,
       WAM_F_ADJ_HI = 5, WAM_F_COUNT = 6 };

struct wam_plan {
  int ndim;
  int levels;
  int L;
  int mode;
  int pad;                               // p = (2L-3)//2
  int64_t shape[WAM_MAX_NDIM];           // input spatial dims
  // per level j = 0..levels-1 (finest first): input dims and coefficient dims
  int64_t lin[WAM_MAX_LEVELS][WAM_MAX_NDIM];
  int64_t lout[WAM_MAX_LEVELS][WAM_MAX_NDIM];
  // synthesis: per level (coarsest first, c_pos) crop-one-more-at-end flags per axis
  int extra[WAM_MAX_LEVELS][WAM_MAX_NDIM];
  int64_t rec_shape[WAM_MAX_NDIM];
  int nbands;
  int64_t band_dims[WAM_MAX_BANDS][WAM_MAX_NDIM];
  int64_t band_off[WAM_MAX_BANDS + 1];   // per-item element offsets (band_off[nbands] = total)
  float* d_filt;                         // WAM_F_COUNT * L floats on the device
  float h_filt[WAM_F_COUNT][WAM_MAX_FILT];
  int device;
  int flags;                             // WAM_PLAN_GENERIC: force the per-axis kernels
};

static inline int64_t wam_prod(const int64_t* d, int n) {
  int64_t p = 1;
  for (int i = 0; i < n; ++i) p *= d[i];
  return p;
}

static inline unsigned wam_grid(int64_t work, int block, int64_t cap = 262144) {
  int64_t g = (work + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

// band index helpers for a level l (0 = finest) in ptwt order [A_J, details_J, ..., details_1]
static inline int wam_band_of(const wam_plan* p, int level, int sub /* 0..2^ndim-2 */) {
  int per = (1 << p->ndim) - 1;
  return 1 + (p->levels - 1 - level) * per + sub;
}

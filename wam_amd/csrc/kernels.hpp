// Internal launch interfaces shared between the translation units of libwam_hip.so.
#pragma once
#include "common.hpp"

// Logical workgroup id under which consecutive ids run on one XCD. Workgroup b is observed to land
// on XCD b % 8 (round robin; not a contract, so only locality depends on it): the bijection maps
// each XCD's physical blocks onto one contiguous logical range, so neighbouring work items (the row
// chunks and column strips of a plane, which re-read each other's halo rows) share an L2.
__device__ __forceinline__ int64_t wam_xcd_block(int64_t bid, int64_t nwg) {
  const int64_t q8 = nwg / 8, r8 = nwg % 8, xcd = bid % 8;
  return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
}

// Streaming stores (global_store ... nt): same bytes, same values, no write-allocation in the caches.
// Used where they won in the bench's own pipeline: the 3D Haar synthesis, whose output is the model's
// input and read by no WAM kernel (c5 in-bench, profiles/r06y_*: k_haar3_syn 103 -> 87 us per launch,
// WAM 4.88 -> 4.65 ms per step), and k_copy (the copy ceiling 6.18 -> 6.32 TB/s,
// r06w_ab_copy_nt.log). Back-to-back microbenchmarks flatter them -- there plain stores pay the
// previous launch's write-back (c5 maps 110 -> 83 us in kbench, 111 -> 100-118 in the pipeline,
// r06t_* / r06x_*) -- and elsewhere they measured the same or slower: c4's finest synthesis level
// (r06y_*), the plane / row / 1D / mel kernels (noisy plane analysis 606-641 -> 644-667 us; the bf16
// NHWC synthesis's 2-byte stores 496 -> 1,070 us; r06u_*, r06v_*). WAM_NT_STORES=0 builds the plain
// stores for A/B runs.
#ifndef WAM_NT_STORES
#define WAM_NT_STORES 1
#endif
typedef float wam_f2v __attribute__((ext_vector_type(2)));  // 8-byte aligned pair
typedef float wam_f4v __attribute__((ext_vector_type(4)));
template <class T>
__device__ __forceinline__ void wam_st(T* p, T v) {
#if WAM_NT_STORES
  __builtin_nontemporal_store(v, p);
#else
  *p = v;
#endif
}
__device__ __forceinline__ void wam_st4(float* p, float a, float b, float c, float d) {  // 16-byte aligned
  wam_st(reinterpret_cast<wam_f4v*>(p), wam_f4v{a, b, c, d});
}

// generic per-axis kernels (dwt_axis.hip)
int launch_analysis_axis(const float* in, float* lo, float* hi, int64_t outer, int n, int m, int64_t inner,
                         int padl, int mode, const float* flo, const float* fhi, int L, hipStream_t st);
int launch_synthesis_axis(const float* a, const float* d, float* out, int64_t outer, int m, int nout,
                          int64_t inner, int p, const float* rlo, const float* rhi, int L, float sa, float sd,
                          hipStream_t st);

// fused 2D kernels (dwt2_fused.hip)
bool dwt2_fused_supported(const wam_plan* p);
int launch_dwt2_analysis_fused(const wam_plan* p, int64_t batch, const float* in, const int64_t* in_dims,
                               const int64_t* out_dims, int mode, int fset, float* out_a, float* const* sub,
                               hipStream_t st);
// One synthesis level for up to kSynMaxAlpha IG alphas in one launch: alpha i reads its LL from
// a[i] (scaled by sa[i]) and the shared detail bands (scaled by sd[i]) and writes out[i].
constexpr int kSynMaxAlpha = 32;
// alphas whose intermediate LL planes the plan workspace holds at once (2D row-synthesis plans)
#ifndef WAM_SYN_WS_ALPHA
#define WAM_SYN_WS_ALPHA 8
#endif
constexpr int kSynWsAlpha = WAM_SYN_WS_ALPHA;
static_assert(kSynWsAlpha >= 1 && kSynWsAlpha <= kSynMaxAlpha, "alpha group");
struct SynBatch {
  const float* a[kSynMaxAlpha];
  float* out[kSynMaxAlpha];
  float sa[kSynMaxAlpha];
  float sd[kSynMaxAlpha];
  int na;
};
int launch_dwt2_synthesis_fused(const wam_plan* p, int64_t batch, int level, const SynBatch& sb,
                                const float* const* sub, hipStream_t st);

#include "timing.hpp"

// row-resident fused 2D kernels (dwt2_rows.hip): whole source rows staged in wave-private LDS
bool dwt2_rows_supported(const wam_plan* p, int level, bool adjoint);
int launch_dwt2_analysis_rows(const wam_plan* p, int64_t batch, const float* in, const int64_t* in_dims,
                              const int64_t* out_dims, int mode, int fset, float* out_a, float* const* sub,
                              const struct WamNoise* noise, hipStream_t st);
// mean_first: the C gradient planes of an image averaged on the load, one plane filtered (level 0
// of the maps-only pass; LL out is then one plane per image and later levels take channels = 1)
int launch_dwt2_adjoint_maps_level(const wam_plan* p, int level, int64_t images, int channels, bool mean_first,
                                   int64_t group_items, const float* in, const int64_t* in_dims, float* ll_out,
                                   float* maps, float* band_max, float* full_grads, int64_t full_items, hipStream_t st);

// fused SmoothGrad noise on the analysis load (Philox4x32-10, same stream as wam_noise_add)
struct WamNoise {
  const float* sigma;     // per image
  int64_t images;         // N (x holds N*C planes)
  int channels;           // C
  uint32_t k0, k1;        // seed
  int64_t sample_base;
  int64_t image_base;     // global index of image 0 (Philox counter word; batch-sharded ranks)
};

// plane-resident multi-level 2D analysis (dwt2_plane.hip): all levels of a plane in one workgroup
bool dwt2_plane_supported(const wam_plan* p, bool adjoint);
bool dwt2_plane_maps_coop(const wam_plan* p);  // the maps pass runs the COOP level 1 (bf16 input possible)
int launch_dwt2_plane_analysis(const wam_plan* p, int64_t items, const float* in, float* coeffs, bool adjoint,
                               const WamNoise* nz, int64_t n_samples, hipStream_t st);
// grad (in_fmt): 0 = fp32 planes [images, channels, nh, nw]; 1 = bf16 images [images, nh, nw, channels];
// 2 = bf16 planes [images, channels, nh, nw]
int launch_dwt2_plane_maps(const wam_plan* p, int64_t images, int channels, int64_t group_items, const void* grad,
                           int in_fmt, float* maps, float* band_max, hipStream_t st);
bool dwt2_plane_syn_supported(const wam_plan* p);
// out_channels 0: fp32 planes; 1 or 3: bf16 NHWC images (planes = images x out_channels)
int launch_dwt2_plane_synthesis(const wam_plan* p, int64_t batch, const float* coeffs, const float* alpha,
                                int n_alpha, void* out, int out_channels, hipStream_t st);

// fused 3D levels, any even filter up to 16 taps (dwt3_tile.hip): one launch per level
bool dwt3_tile_supported(const wam_plan* p);
int launch_dwt3_analysis_tile(const wam_plan* p, int64_t batch, const float* in, const int64_t* in_dims,
                              const int64_t* out_dims, int mode, int fset, float* out_a, float* const* sub,
                              hipStream_t st);
int launch_dwt3_synthesis_tile(const wam_plan* p, int64_t batch, int level, const float* a_in, float a_scale,
                               const float* const* sub, float d_scale, float* out, hipStream_t st);

// fused multi-level 1D tiles (dwt1_tile.hip)
bool dwt1_tile_supported(const wam_plan* p, bool adjoint);

int launch_dwt1_tile_synthesis(const wam_plan* p, int64_t batch, const float* coeffs, const float* alpha,
                               int n_alpha, float* out, hipStream_t st);

// fused 3D Haar blocks (dwt3_haar.hip): J <= 2, dims divisible by 2^J
bool dwt3_haar_supported(const wam_plan* p);
int launch_dwt3_haar_analysis(const wam_plan* p, int64_t batch, const float* in, float* coeffs, bool adjoint,
                              hipStream_t st);
// 1D tiles (dwt1_tile.hip); nz: SmoothGrad noise fused on the load (single-channel signals whose
// length is a multiple of 4; batch = n_samples x images, sample-major)
int launch_dwt1_tile_analysis(const wam_plan* p, int64_t batch, const float* in, float* coeffs, bool adjoint,
                              hipStream_t st, const WamNoise* nz = nullptr, int64_t n_samples = 1);
// noise fused on the load (single-channel volumes; wam_wavedec_noisy for 3D Haar plans)
int launch_dwt3_haar_analysis_noisy(const wam_plan* p, int64_t batch, const float* in, float* coeffs,
                                    const WamNoise* nz, int64_t n_samples, hipStream_t st);
int launch_dwt3_haar_synthesis(const wam_plan* p, int64_t batch, const float* coeffs, const float* alpha, int n_alpha,
                               float* out, hipStream_t st);

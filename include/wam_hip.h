/*
 * wam_hip.h -- C-ABI of libwam_hip.so, the MI355X (gfx950) kernels behind the WAM attribution path.
 *
 * The reference (michalpiasecki0/wam) is pure Python: its hot path calls the third-party ptwt
 * package (not vendored; ptwt>=0.1.0, de-facto 1.0.1) for every wavelet transform and numpy for
 * the per-subband post-processing. The entry points below replace exactly those calls; the
 * Python classes in wam_amd/ keep the reference's class / method signatures and bind these
 * symbols with ctypes (see INTEGRATION.md for the binding a maintainer would add).
 *
 * Conventions
 *   - plain pointers + sizes only; every device buffer is allocated by the caller (torch);
 *   - every compute entry point is asynchronous on the given hipStream_t (passed as void*);
 *   - return value: 0 = success, otherwise a code for wam_strerror(); nothing throws;
 *   - plans are immutable after creation and may be shared by concurrent streams;
 *   - coefficient buffers are BAND-MAJOR: band b occupies [batch, band dims...] contiguously at
 *     element offset batch * wam_plan_band_offset(plan, b). Band order is ptwt's:
 *       1D: [A_J, D_J, ..., D_1]
 *       2D: [A_J, (H_J, V_J, D_J), ..., (H_1, V_1, D_1)]   H = hi along rows, lo along columns
 *       3D: [A_J, (aad, ada, add, daa, dad, dda, ddd)_J, ..., (...)_1]  letters = axes (-3,-2,-1)
 */
#ifndef WAM_HIP_H
#define WAM_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* boundary modes (ptwt names; 'constant' is ptwt's alias of torch 'replicate') */
enum wam_mode { WAM_MODE_ZERO = 0, WAM_MODE_REFLECT = 1, WAM_MODE_SYMMETRIC = 2,
                WAM_MODE_CONSTANT = 3, WAM_MODE_PERIODIC = 4 };

/* error codes (HIP runtime errors are returned as WAM_ERR_HIP_BASE + hipError_t) */
enum wam_status { WAM_OK = 0, WAM_ERR_INVALID_ARG = 1, WAM_ERR_SHAPE = 2, WAM_ERR_UNSUPPORTED = 3,
                  WAM_ERR_NO_MEMORY = 4, WAM_ERR_HIP_BASE = 1000 };

typedef struct wam_plan wam_plan;

const char* wam_strerror(int status);
/* library / ABI version; bumped on any signature change */
int wam_version(void);

/* ------------------------------------------------------------------------------------------------
 * Plans: one per (ndim, spatial shape, levels, filter bank, mode). Replaces ptwt's per-call
 * filter construction (_get_filter_tensors / _construct_{2,3}d_filt) and size bookkeeping
 * (_get_pad, _adjust_padding_at_reconstruction).
 * filters are pywt's float64 tables, cast to fp32 on the device (as ptwt casts to x.dtype).
 * ---------------------------------------------------------------------------------------------- */
int wam_plan_create(wam_plan** plan, int ndim, const int64_t* shape, int levels,
                    const double* dec_lo, const double* dec_hi,
                    const double* rec_lo, const double* rec_hi, int filt_len, int mode);
/* flags: WAM_PLAN_GENERIC forces the per-axis kernels, WAM_PLAN_NO_ROWS skips the row-resident
 * and plane-resident 2D kernels, WAM_PLAN_NO_PLANE skips only the plane-resident (all levels in
 * one workgroup) kernels; WAM_PLAN_NO_COOP / WAM_PLAN_FORCE_COOP pick the plane kernels' level-1
 * form (wave chunks / cooperative row stream) instead of the size-based choice (all used by tests to
 * cross-check the fused 2D kernels); 0 selects the fastest path. Bit 32 (a line-streaming analysis
 * that never beat the plane kernel) is retired and ignored.
 * wam_plan_create == wam_plan_create_ex(..., 0). */
enum wam_plan_flags { WAM_PLAN_GENERIC = 1, WAM_PLAN_NO_ROWS = 2, WAM_PLAN_NO_PLANE = 4, WAM_PLAN_NO_COOP = 8,
                      WAM_PLAN_FORCE_COOP = 16 };
int wam_plan_create_ex(wam_plan** plan, int ndim, const int64_t* shape, int levels,
                       const double* dec_lo, const double* dec_hi,
                       const double* rec_lo, const double* rec_hi, int filt_len, int mode, int flags);
/* a host-only plan: the same geometry, band layout, caps and workspace queries, no device (no
 * filters uploaded). Every compute entry point refuses it with WAM_ERR_INVALID_ARG. Used by the
 * sanitizer build of the host code (tests/native/). */
int wam_plan_create_host(wam_plan** plan, int ndim, const int64_t* shape, int levels,
                         const double* dec_lo, const double* dec_hi,
                         const double* rec_lo, const double* rec_hi, int filt_len, int mode, int flags);
void wam_plan_destroy(wam_plan* plan);
int wam_plan_num_bands(const wam_plan* plan);
/* dims of band b (ndim values) */
int wam_plan_band_shape(const wam_plan* plan, int band, int64_t* dims);
/* element offset of band b for ONE item (multiply by batch for a batched buffer) */
int64_t wam_plan_band_offset(const wam_plan* plan, int band);
/* coefficients per item (sum over bands) */
int64_t wam_plan_coeff_numel(const wam_plan* plan);
/* spatial dims produced by wam_waverec (ptwt: odd n reconstructs to n+1) */
int wam_plan_rec_shape(const wam_plan* plan, int64_t* dims);
/* bytes of scratch the transforms need for `batch` items (caller allocates). For 2D plans on the
 * per-level row synthesis it covers the intermediate approximations of 8 IG alphas, which
 * wam_waverec synthesises per level launch. */
int64_t wam_plan_workspace_bytes(const wam_plan* plan, int64_t batch);

/* ------------------------------------------------------------------------------------------------
 * Transforms
 * ---------------------------------------------------------------------------------------------- */
/* ptwt.wavedec / wavedec2 / wavedec3 (lib/wam_2D.py:96,430; lib/wam_1D.py:109,370;
 * lib/wam_3D.py:194,620). x: [batch, shape...]; coeffs: band-major, batch items. */
int wam_wavedec(const wam_plan* plan, int64_t batch, const float* x, float* coeffs,
                void* workspace, void* stream);

/* ptwt.waverec / waverec2 / waverec3 (lib/wam_2D.py:113; lib/wam_1D.py:117; lib/wam_3D.py:206,222)
 * with the Integrated-Gradients path scaling fused into the coefficient load
 * (lib/wam_2D.py:461-476 alter()): out[a, b] = waverec(fp32(alpha[a]) * coeffs[b]) for
 * a < n_alpha; alpha is a HOST array (alpha == NULL: n_alpha must be 1, no scaling).
 * out: [n_alpha, batch, rec_shape...]. */
int wam_waverec(const wam_plan* plan, int64_t batch, const float* coeffs, const float* alpha,
                int n_alpha, float* out, void* workspace, void* stream);

/* Adjoint of wam_waverec w.r.t. its coefficients = the backward pass of waverec in the
 * reference's loss.backward() (lib/wam_2D.py:116): zero-padded analysis with reverse(rec)
 * filters. grad: [batch, rec_shape...]; coeff_grads: band-major. */
int wam_waverec_adjoint(const wam_plan* plan, int64_t batch, const float* grad, float* coeff_grads,
                        void* workspace, void* stream);

/* ------------------------------------------------------------------------------------------------
 * Fused WAM passes (2D, rows <= 512 samples, filter length in {2,4,6,8,12,16,20})
 * ---------------------------------------------------------------------------------------------- */
enum wam_caps { WAM_CAP_NOISY_WAVEDEC = 1, WAM_CAP_ADJOINT_MAPS = 2, WAM_CAP_BF16_NHWC = 4 };
/* which fused entry points below this plan supports (bit set of wam_caps) */
int wam_plan_caps(const wam_plan* plan);

/* SmoothGrad sample generation fused into the first analysis level (lib/wam_2D.py:390-406):
 * coeffs of x_i + sigma_i * N(0,1) for n_samples x images x channels planes, with the same
 * Philox stream as wam_noise_add (counter (sample_base + s, image, element / 4)), without
 * materialising the noisy input. x: [images, channels, H, W]; coeffs band-major over the
 * (sample, image, channel) planes. WAM_ERR_UNSUPPORTED unless WAM_CAP_NOISY_WAVEDEC. Also 3D Haar
 * plans (J <= 2, dims divisible by 2^J, W % 4 == 0; lib/wam_3D.py:565-582) for channels == 1:
 * x [images, 1, D, H, W], coeffs over the (sample, image) volumes. */
int wam_wavedec_noisy(const wam_plan* plan, int64_t n_samples, int64_t images, int channels,
                      const float* x, const float* sigma, uint64_t seed, int64_t sample_base,
                      float* coeffs, void* workspace, void* stream);
/* the same with the Philox image counter offset by image_base: x holds images [image_base,
 * image_base + images) of a batch sharded over ranks, so every image keeps the noise it gets
 * unsharded (wam_wavedec_noisy == image_base 0) */
int wam_wavedec_noisy_ex(const wam_plan* plan, int64_t n_samples, int64_t images, int channels,
                         const float* x, const float* sigma, uint64_t seed, int64_t sample_base,
                         int64_t image_base, float* coeffs, void* workspace, void* stream);

/* Backward pass of waverec fused with the WAM epilogue (lib/wam_2D.py:116 loss.backward() through
 * ptwt.waverec2, then :227-256 channel mean, |.|, batch-global max): for every image
 * (groups x group_items, channels planes each) the item-major |mean_c| maps (as
 * wam_subband_maps) and band_max[group, band] (caller zero-fills). coeff_grads != NULL also
 * receives the per-channel coefficient gradients (band-major), e.g. for side attributes.
 * WAM_ERR_UNSUPPORTED unless WAM_CAP_ADJOINT_MAPS and channels in {1, 3}. */
int wam_waverec_adjoint_maps(const wam_plan* plan, int64_t groups, int64_t group_items, int channels,
                             const float* grad, float* maps, float* band_max, float* coeff_grads,
                             void* workspace, void* stream);

/* The model hand-off in the explained model's own dtype and layout (lib/wam_2D.py:113-116 with a
 * bf16 channels-last model): wam_waverec_bf16_nhwc is wam_waverec whose reconstruction is written
 * as bf16 images in NHWC order, out [n_alpha * batch / channels, H, W, channels] (plane b = image
 * b / channels, channel b % channels), each value rounded to nearest even exactly as torch's
 * float -> bfloat16 cast; wam_waverec_adjoint_maps_bf16_nhwc is wam_waverec_adjoint_maps over
 * a bf16 NHWC input gradient grad [groups * group_items, H, W, channels] (values widened exactly;
 * no coefficient gradients). Both need WAM_CAP_BF16_NHWC and channels in {1, 3}; no workspace. */
int wam_waverec_bf16_nhwc(const wam_plan* plan, int64_t batch, const float* coeffs, const float* alpha,
                          int n_alpha, int channels, void* out, void* stream);
int wam_waverec_adjoint_maps_bf16_nhwc(const wam_plan* plan, int64_t groups, int64_t group_items, int channels,
                                       const void* grad, float* maps, float* band_max, void* stream);
/* the same for a bf16 gradient in either layout: nhwc != 0 as above, nhwc == 0 planar NCHW
 * [groups * group_items, channels, H, W] (what a model whose first layer's backward ends in a
 * planar op, e.g. a pixel shuffle, hands back) */
int wam_waverec_adjoint_maps_bf16(const wam_plan* plan, int64_t groups, int64_t group_items, int channels, int nhwc,
                                  const void* grad, float* maps, float* band_max, void* stream);

/* ------------------------------------------------------------------------------------------------
 * Live per-launch timing (profiling aid used by bench.py). While enabled every kernel launch is
 * bracketed by hipEventRecord on its stream and logged with its kernel name and ALGORITHMIC
 * bytes; wam_timing_drain synchronises on the recorded events, copies up to max_records
 * (names: 64 chars each) and clears the log. Returns the number of records copied.
 * ---------------------------------------------------------------------------------------------- */
int wam_timing_enable(int on);
/* dst = src (bytes % 16 == 0, 16-B aligned): a streaming copy kernel, the measured HBM ceiling */
int wam_copy(int64_t bytes, const void* src, void* dst, void* stream);
int wam_timing_drain(int max_records, char* names, float* ms, double* bytes);

/* ------------------------------------------------------------------------------------------------
 * SmoothGrad noise (lib/wam_2D.py:390-403, lib/wam_1D.py:311-322, lib/wam_3D.py:565-579)
 * ---------------------------------------------------------------------------------------------- */
/* sigma[i] = fp32(spread) * (max(x_i[0:len]) - min(x_i[0:len])), x_i = x + i*item_stride */
int wam_item_sigma(int64_t items, int64_t item_stride, int64_t len, const float* x, float spread,
                   float* sigma, void* stream);
/* the same sigma as a full-chip split reduction (items x ranges workgroups; the last range of an
 * item to finish combines the partials). ws: wam_item_sigma_ws_bytes(items, len) bytes, 8-byte
 * aligned, zero-filled before its first use with these (items, len); the call leaves it reusable
 * for the same (items, len). */
int64_t wam_item_sigma_ws_bytes(int64_t items, int64_t len);
int wam_item_sigma_ws(int64_t items, int64_t item_stride, int64_t len, const float* x, float spread,
                      float* sigma, void* ws, int64_t ws_bytes, void* stream);

/* out[s, i, e] = x[i, e] + noise  for e < noised_len,  0 for noised_len <= e < item_stride
 * noise = host_noise[s, i, e] if host_noise != NULL (parity mode: the numpy legacy stream), else
 *         sigma[i] * N(0,1) from Philox4x32-10 keyed by (seed), counter (sample_base + s, i, e/4).
 * s ranges over [0, n_samples). */
int wam_noise_add(int64_t n_samples, int64_t items, int64_t item_stride, int64_t noised_len,
                  const float* x, const float* sigma, const float* host_noise, uint64_t seed,
                  int64_t sample_base, float* out, void* stream);
/* the same with the Philox item counter offset by item_base (items of a batch-sharded rank) */
int wam_noise_add_ex(int64_t n_samples, int64_t items, int64_t item_stride, int64_t noised_len,
                     const float* x, const float* sigma, const float* host_noise, uint64_t seed,
                     int64_t sample_base, int64_t item_base, float* out, void* stream);

/* ------------------------------------------------------------------------------------------------
 * Per-subband reduction and accumulation (lib/wam_2D.py:200-264 visualize_grad_wam,
 * :268-341 _reproject_wam, :388-415 SmoothGrad mean, :441-459 IG trapezoid;
 * lib/wam_3D.py:127-166 refactor, :585-587 legacy averaging)
 * ---------------------------------------------------------------------------------------------- */
/* maps[item, band-packed] = | mean over `channels` of coeff_grads |   (numpy float32 mean:
 * ((g0 + g1) + g2 ...) / C);  band_max[group, band] = max over the group's items of maps
 * (atomic; caller zero-fills; NULL: maps only). items = groups * group_items; coeff_grads hold
 * items*channels signals. maps layout: item-major, bands packed with wam_plan_band_offset. */
int wam_subband_maps(const wam_plan* plan, int64_t groups, int64_t group_items, int channels,
                     const float* coeff_grads, float* maps, float* band_max, void* stream);

/* SmoothGrad mosaic accumulation. For each group s in [0, groups) in order and item n:
 *   frame[n, p] += fp64( maps[(s*group_items+n), src[p]] / band_max[s, band[p]] )  (normalize)
 *   frame[n, p] += fp64( maps[...] )                                              (!normalize)
 * src[p] = -1 leaves frame[n, p] unchanged (the reference's zero canvas). frame: [group_items,
 * frame_len] float64. src/band: the mosaic gather map built on the host from the reference's
 * slice-assignment rules (frame geometry lives in the Python layer). */
int wam_frame_accumulate(int64_t groups, int64_t group_items, int64_t frame_len, const int32_t* src,
                         const int32_t* band, const float* maps, int64_t maps_item_len,
                         const float* band_max, int n_bands, int normalize, double* frame,
                         void* stream);

/* wam_frame_accumulate in coefficient order (same sums, bit-identical): dst[k] = the frame pixel
 * of packed coefficient k or -1, cband[k] its band (the inverse of the injective src/band mosaic
 * map, built by the caller: wam_amd/plan.py frame_accumulate). The maps are read as contiguous
 * rows, only the fp64 frame goes through the mosaic. */
int wam_frame_accumulate_coef(int64_t groups, int64_t group_items, int64_t maps_item_len, int64_t frame_len,
                              const int32_t* dst, const int32_t* cband, const float* maps,
                              const float* band_max, int n_bands, int normalize, double* frame, void* stream);

/* Integrated-Gradients mosaic + trapezoid (np.trapz(np.nan_to_num(G), axis=1), dx = 1, fp32).
 * For step k = k0 + s, s in [0, groups):  G = nan_to_num(fp32 mosaic value (normalised));
 *   sequential (weights == NULL): if k > 0: acc += (prev + G) / 2;  prev = G
 *   weighted   (weights != NULL): acc += weights[s] * G     (used when steps are sharded)
 * prev / acc: [group_items, frame_len] fp32. */
int wam_frame_trapz(int64_t groups, int64_t k0, int64_t group_items, int64_t frame_len,
                    const int32_t* src, const int32_t* band, const float* maps, int64_t maps_item_len,
                    const float* band_max, int n_bands, int normalize, const float* weights,
                    float* prev, float* acc, void* stream);

/* wam_frame_trapz in coefficient order (dst / cband as for wam_frame_accumulate_coef): the maps
 * are read as contiguous rows, prev / acc go through the mosaic. Pixels outside the mosaic are not
 * touched -- their G is 0, so with prev == 0 there (zero-initialised, as wam_amd/wam_2D.py passes
 * them) the result is bit-identical to wam_frame_trapz. */
int wam_frame_trapz_coef(int64_t groups, int64_t k0, int64_t group_items, int64_t maps_item_len, int64_t frame_len,
                         const int32_t* dst, const int32_t* cband, const float* maps, const float* band_max,
                         int n_bands, int normalize, const float* weights, float* prev, float* acc, void* stream);

/* 3D cube (lib/wam_3D.py:127-166 refactor; :585-587 legacy averaging; :638 IG trapezoid):
 * value = maps[item, src[p]] with maps = |coeff grads| from wam_subband_maps(channels = 1)
 * (no channel mean, no normalisation). For s in [0, groups) in order:
 * mode 0 (legacy smooth, sequential): acc = (acc + value) / n_total                    (fp32)
 * mode 1 (weighted):                   acc += weights[s] * value
 * mode 2 (IG sequential trapz):        G = nan_to_num(value); if k0+s > 0: acc += (prev+G)/2;
 *                                      prev = G
 * acc / prev: [group_items, cube_len] fp32. */
int wam_cube_accumulate(int64_t groups, int64_t k0, int64_t group_items, int64_t cube_len,
                        const int32_t* src, const float* maps, int64_t maps_item_len, int mode,
                        float n_total, const float* weights, float* prev, float* acc, void* stream);

/* Sum reduction in sample order: acc[e] (+)= src[s*len + e] for s < groups (fp32, sequential);
 * scale != 0: afterwards acc[e] = acc[e] / scale (numpy mean's true_divide). */
int wam_accumulate_f32(int64_t groups, int64_t len, const float* src, float scale, float* acc,
                       void* stream);

/* IG trapezoid over a generic fp32 stream (1D melspec / coefficient gradients):
 * G_s = src[s*len + e]; sequential (weights == NULL) or weighted trapz as in wam_frame_trapz;
 * acc_f64 != NULL accumulates in fp64 (the reference's float64 path_melspecs), else acc_f32. */
int wam_trapz_f32(int64_t groups, int64_t k0, int64_t len, const float* src, const float* weights,
                  float* prev_f32, float* acc_f32, double* prev_f64, double* acc_f64, void* stream);

/* .scales side output (lib/wam_2D.py:488-536 reproject_wam): for each item and level j,
 * out[item, j] = sum over the H, V, D quadrants of bilinear (cv2 INTER_LINEAR, half-pixel)
 * upsampling to size x size; with approx, out[item, J] = upsampled approximation corner. */
int wam_reproject_scales(int64_t items, int size, int levels, int approx, const double* avg,
                         double* out, void* stream);

/* BaseWAM2D.scales (lib/wam_2D.py:133-198 disentangle_scales): maps = item-major |channel mean|
 * coefficient-gradient maps of `items` images (wam_subband_maps / wam_waverec_adjoint_maps with one
 * group), band_max = their per-band maxima over the batch. out[item, j] (j < levels, finest
 * first) = (V + D) + H, each band / band_max upsampled to size x size (cv2 INTER_LINEAR on float32,
 * half-pixel centres) in float32, stored as float64; with approx, out[items-1, levels] = the
 * upsampled normalised approximation and out[i < items-1, levels] = 0 (the reference writes only
 * its stale loop index, :194-197). out: [items, levels (+1), size, size] float64. */
int wam_disentangle_scales(const wam_plan* plan, int64_t items, const float* maps, const float* band_max,
                           int approx, int size, double* out, void* stream);

/* ------------------------------------------------------------------------------------------------
 * Wavelet-domain insertion / deletion / mu-fidelity (src/evaluation_helpers.py:
 * 361-594 called by Eval2DWAM, src/evaluators.py:553-801). The reference's per-mask CPU loop
 * pywt.wavedec2 -> coeffs_to_array -> arr * mask -> waverec2 -> uint8 -> ToTensor/Normalize
 * becomes: wam_wavedec (mode symmetric) once per image, wam_coeff_masks, wam_waverec of all masks
 * in one launch, wam_quantize_normalize.
 * ---------------------------------------------------------------------------------------------- */
/* generate_masks (:455-505) from a ranking: rank[p] = position of pixel p in the descending
 * importance order; masks [n_iter + 1, len] float32: mask m = 1 where rank < thr(m), thr(0) = 0,
 * thr(m) = m * n_comp, thr(n_iter) = len (deletion != 0: the complement). */
int wam_rank_masks(int64_t n_iter, int64_t n_comp, int64_t len, const int32_t* rank, int deletion,
                   float* masks, void* stream);
/* arr * masks[m] in pywt.coeffs_to_array's layout: coefficient k (band-major item offset) of each
 * of `items` planes sits at array position pos[k] (< mask_len). out: band-major coefficients of
 * n_masks * items planes, plane (m, i) = m * items + i. */
int wam_coeff_masks(const wam_plan* plan, int64_t items, const float* coeffs, const int32_t* pos,
                    int64_t n_masks, int64_t mask_len, const float* masks, float* out, void* stream);
/* per image (channels x plane floats): normalize_data (min-max, float32), (v * 255) -> uint8
 * (truncation), / 255, (- mean[c]) / std[c] (torchvision ToTensor + Normalize); mean / std are
 * HOST arrays of `channels` (<= 4) values. */
int wam_quantize_normalize(int64_t images, int channels, int64_t plane, const float* rec, const float* mean,
                           const float* std, float* out, void* stream);
/* The same quantisation followed by torchvision Resize((out_h, out_w)) on the PIL image (Pillow's
 * 8-bit BILINEAR resample) and ToTensor + Normalize, for reconstructions that are not 224 x 224:
 * Eval2DWAM's default transform (src/evaluators.py:593-598) on e.g. 256^2 inputs. Replaces the
 * reference's per-image PIL path (src/evaluators.py:631-633). rec [images, channels, in_h, in_w]
 * float32 -> out [images, channels, out_h, out_w] float32. The resample tables are Pillow's
 * (precompute_coeffs + normalize_coeffs_8bpc, wam_amd/evaluation.py pil_bilinear_coeffs): per
 * output column xx bounds_h[2 xx] = first source column, bounds_h[2 xx + 1] = count, kk_h[xx *
 * ksize_h + k] = 22-bit fixed-point weights (device int32); likewise vertically with the bounds
 * relative to source row y0. bounds_h == NULL: the width is unchanged (no horizontal pass; y0 /
 * tmp_h ignored, bounds_v absolute); bounds_v == NULL: the height is unchanged. tmp_h = source
 * rows the vertical pass reads (y0 .. y0 + tmp_h - 1). scratch: images * channels * (in_h * in_w +
 * tmp_h * out_w) bytes. Bit-identical to PIL.Image.resize((out_w, out_h), BILINEAR). */
int wam_quantize_resize_normalize(int64_t images, int channels, int in_h, int in_w, const float* rec, int out_h,
                                  int out_w, int ksize_h, const int32_t* bounds_h, const int32_t* kk_h, int ksize_v,
                                  const int32_t* bounds_v, const int32_t* kk_v, int y0, int tmp_h, const float* mean,
                                  const float* std, uint8_t* scratch, float* out, void* stream);
/* scipy.ndimage.gaussian_filter of items h x w float64 maps, mode 'reflect' (half-sample
 * symmetric): weights[0..radius] = the symmetric 1-D kernel (host), axis 0 then axis 1, scipy's
 * accumulation order; tmp: items * h * w doubles of scratch. */
int wam_gaussian_filter2d(int64_t items, int h, int w, const double* weights, int radius, const double* in,
                          double* tmp, double* out, void* stream);
/* out[m, p] = grid[m, cell[p]]  (nearest-neighbour zoom through a precomputed cell map) */
int wam_upsample_masks(int64_t n_masks, int64_t grid_len, const float* grid, int64_t out_len,
                       const int32_t* cell, float* out, void* stream);
/* sum_importance (:361-393): out[m] = sum_p wam[p] * grid[m, cell[p]] (float64) */
int wam_masked_sums(int64_t n_masks, int64_t len, const double* wam, int64_t grid_len, const float* grid,
                    const int32_t* cell, double* out, void* stream);

/* WaveletAttribution3D.visualize (lib/wam_3D.py:662-719): cube [items, S, S, S]
 * float32 (the |grad| cube of smooth / IG) -> out [items, levels + 2, S, S, S] float32: per level
 * the block (approximation corner, or add + ada + add + daa + dad + dda of the detail shell, as
 * the reference sums them) upsampled by scipy.ndimage.zoom order 1 and divided by its max; slot
 * levels + 1 = the level sum divided by its max over the batch. scratch: items * (levels + 1) + 1
 * floats. WAM_ERR_SHAPE when S is not divisible as the reference's assignment needs. */
int wam_visualize3d(int64_t items, int size, int levels, const float* cube, float* out, float* scratch,
                    void* stream);

/* ------------------------------------------------------------------------------------------------
 * 1D mel front-end (replaces lib/wam_1D.py:194-219, BaseWAM1D.compute_melspec: torchaudio
 * MelSpectrogram(sample_rate, n_fft, n_mels) with its defaults -- periodic Hann, hop n_fft / 2,
 * center + reflect padding, power 2, HTK mel without normalisation -- followed by AmplitudeToDB()
 * when to_db, and the gradient torch autograd takes through it).
 * wave [items, samples] float32 (samples > n_fft / 2); out / grad_out [items, F, n_mels] with
 * F = samples / (n_fft / 2) + 1 (the reference's [N, 1, F, n_mels] stack); n_fft a power of two
 * in [64, 2048], n_mels <= 256 (WAM_ERR_UNSUPPORTED otherwise).
 * tables (float, device): window[n_fft] | twiddle[2 n_fft] (cos, sin of -2 pi m / n_fft) |
 *   band_w[nnz] | bin_w[nnz];
 * index (int32, device): band_ptr[n_mels + 1] | band_bin[nnz] | bin_ptr[n_fft / 2 + 2] |
 *   bin_band[nnz] -- the filterbank's nonzeros by band (bins ascending) and by bin (bands
 *   ascending); wam_amd/melspec.py (MelTables) builds them from torchaudio's filterbank formula.
 * grad_wave is written (not accumulated). */
int wam_melspec(int64_t items, int64_t samples, int n_fft, int n_mels, int nnz, int to_db, const float* wave,
                const float* tables, const int32_t* index, float* out, void* stream);
int wam_melspec_adjoint(int64_t items, int64_t samples, int n_fft, int n_mels, int nnz, int to_db,
                        const float* wave, const float* grad_out, const float* tables, const int32_t* index,
                        float* grad_wave, void* stream);

/* ------------------------------------------------------------------------------------------------
 * Explained-model input-gradient pass (lib/wam_2D.py:114-116: model forward, diag-mean loss,
 * backward). Not a ptwt replacement: fused elementwise steps of a BN-folded ReLU network, each one
 * HBM pass instead of the 2-4 torch kernels it replaces (wam_amd/model_fuse.py drives them).
 * dtype: WAM_DT_F32 or WAM_DT_BF16 (storage; arithmetic is fp32). Tensors are contiguous with n
 * elements; the channel of element i is (i / inner) % channels (inner = 1: NHWC, H*W: NCHW).
 * Bias vectors (length channels, same dtype) may be NULL (= 0). out may alias an input.
 * ---------------------------------------------------------------------------------------------- */
enum wam_dtype { WAM_DT_F32 = 0, WAM_DT_BF16 = 1 };

/* y = relu ? max(y + bias[c], 0) : y + bias[c]      (in place; conv bias + ReLU) */
int wam_ew_bias_act(int dtype, int64_t n, int64_t channels, int64_t inner, void* y, const void* bias,
                    int relu, void* stream);
/* out = max((a + bias_a[c]) + (s + bias_s[c]), 0)   (residual tail of a bottleneck block) */
int wam_ew_add_bias_relu(int dtype, int64_t n, int64_t channels, int64_t inner, const void* a,
                         const void* bias_a, const void* s, const void* bias_s, void* out, void* stream);
/* out = y > 0 ? g1 (+ g2 if g2 != NULL) : 0          (ReLU backward, optionally fused fan-in) */
int wam_ew_relu_mask(int dtype, int64_t n, const void* g1, const void* g2, const void* y, void* out,
                     void* stream);
/* NHWC max pooling (k x k window, stride, zero-area padding pad <= k/2, floor output size):
 * y [n, ho, wo, c], idx [n, ho, wo, c] uint8 = window position kh*k+kw | 0x80 if the max is > 0.
 * Replaces torch max_pool2d_with_indices after the stem ReLU (torchvision ResNet maxpool);
 * WAM_ERR_UNSUPPORTED when c is not a multiple of the 16-byte vector or pointers are unaligned. */
int wam_ew_maxpool_nhwc(int dtype, int64_t n, int64_t h, int64_t w, int64_t c, int k, int stride, int pad,
                        const void* x, void* y, void* idx, void* stream);
/* gx [n, h, w, c] = sum of gy over the windows whose idx points at the pixel (fp32 sums in window
 * order); relu != 0 also drops windows whose max was not > 0 (mask of the ReLU feeding the pool). */
int wam_ew_maxpool_nhwc_backward(int dtype, int64_t n, int64_t h, int64_t w, int64_t c, int k, int stride,
                                 int pad, const void* gy, const void* idx, int relu, void* gx, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* WAM_HIP_H */

/*
 * wgsr.h -- C ABI of the MI355X-native WildGS Gaussian-splatting hot path.
 *
 * This is the drop-in boundary for the two native extensions WildGS-SLAM
 * loads on its mapping path:
 *
 *   diff_gaussian_rasterization._C  (empty submodule in the reference,
 *       .gitmodules:7-9; bound by the Python layer that
 *       thirdparty/gaussian_splatting/gaussian_renderer/__init__.py:15-18,
 *       58-74 and 130-141 imports)
 *   simple_knn._C.distCUDA2          (.gitmodules:10-12; called at
 *       thirdparty/gaussian_splatting/scene/gaussian_model.py:18,201-207)
 *
 * Each entry point below names the upstream `_C` function it replaces.  All
 * pointers are DEVICE pointers (HIP, gfx950) unless stated, all arrays are
 * contiguous fp32 (int32 where noted), and every launch goes on `stream`
 * (a hipStream_t; NULL = the null stream).  Scratch memory is obtained through
 * caller-supplied allocation callbacks -- the C analogue of upstream's
 * `std::function<char*(size_t)>` resize functors -- so the caller's allocator
 * (e.g. the torch caching allocator) owns every byte and the library keeps no
 * global device state.
 *
 * Return value: 0 on success, a WGSR_E* code otherwise; wgsr_last_error()
 * returns a thread-local message for the last failure.
 */
#ifndef WGSR_H
#define WGSR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define WGSR_OK 0
#define WGSR_EINVAL 1   /* argument misuse (upstream: AT_ERROR / Exception) */
#define WGSR_EHIP 2     /* HIP runtime / launch failure                     */
#define WGSR_EALLOC 3   /* an allocation callback returned NULL             */

/* Returns a device pointer to at least `bytes` bytes, 256-byte aligned, that
 * stays valid until the caller releases it.  `bytes` may be 0.  Within one
 * library call a callback may be called twice for the same buffer (the
 * forward's binning buffer: a predicted size before its host wait, then the
 * exact size) only when the predicted size was too small: the library then
 * uses the pointer of the second call and has written nothing through the
 * first, which the callback may release or grow.  A large-enough prediction
 * is used as it is (no second call). */
typedef void* (*wgsr_alloc_fn)(void* ctx, size_t bytes);

/* The rasterisation inputs shared by forward and backward: the tensors and
 * scalars of upstream's rasterize_gaussians / rasterize_gaussians_backward
 * argument lists (GaussianRasterizationSettings + per-Gaussian tensors). */
typedef struct wgsr_raster_args {
  int P;                        /* number of Gaussians                        */
  int D;                        /* active SH degree (sh_degree)               */
  int M;                        /* stored SH coefficients per Gaussian        */
  int W, H;                     /* image_width, image_height                  */
  const float* bg;              /* [3]                                        */
  const float* means3D;         /* [P,3]                                      */
  const float* colors;          /* [P,3] colors_precomp, or NULL             */
  const float* opacities;       /* [P,1]                                      */
  const float* scales;          /* [P,3] or NULL (then cov3D_precomp)         */
  const float* rotations;       /* [P,4] (w,x,y,z) or NULL                    */
  const float* cov3D_precomp;   /* [P,6] or NULL                              */
  const float* shs;             /* [P,M,3] or NULL (then colors)              */
  const float* viewmatrix;      /* [4,4] world_view_transform (row-vector)    */
  const float* projmatrix;      /* [4,4] full_proj_transform                  */
  const float* projmatrix_raw;  /* [4,4] projection_matrix                    */
  const float* campos;          /* [3]  camera_center                         */
  float scale_modifier;
  float tan_fovx, tan_fovy;
  int prefiltered;              /* upstream: trap if a prefiltered point is culled */
  int debug;                    /* synchronise + check after every kernel     */
} wgsr_raster_args;

/* Replaces _C.rasterize_gaussians (forward).
 * Outputs (caller-allocated, fully written): out_color [3,H,W],
 * out_depth [1,H,W], out_opacity [1,H,W] (= 1 - T), radii [P] int32,
 * n_touched [P] int32.  Three state buffers are requested through the
 * callbacks (geometry ~ P, binning ~ num_rendered, image ~ H*W); the caller
 * must keep them for wgsr_rasterize_backward.  *num_rendered receives the
 * number of (Gaussian, tile) pairs.  One device->host read (num_rendered)
 * synchronises `stream`, as upstream does. */
int wgsr_rasterize_forward(const wgsr_raster_args* args,
                           wgsr_alloc_fn geom_alloc, wgsr_alloc_fn binning_alloc,
                           wgsr_alloc_fn image_alloc, void* alloc_ctx,
                           float* out_color, float* out_depth, float* out_opacity,
                           int32_t* radii, int32_t* n_touched, int64_t* num_rendered,
                           void* stream);

/* Capacity mode of wgsr_rasterize_forward (no upstream counterpart): the
 * same outputs with NO host synchronisation, so that a whole mapping
 * iteration can be captured in a HIP graph (wgsr/online.py).  The state
 * buffers are sized for `cap` (Gaussian, tile) rectangle pairs (upstream's
 * num_rendered bounds the exact and bin pairs); pass cap as num_rendered to
 * wgsr_rasterize_backward.  counts (device, 5 uint32): N_rect, N_exact,
 * N_bin (saturating), overflow (N_rect > cap), min(N_bin, cap).  After an
 * overflow the images are undefined and the backward writes zero gradients;
 * callers skip their optimizer step on counts[3] (wgsr_adam_step_dev).
 * Needs the default sort-bin configuration (WGSR_EINVAL otherwise) and
 * prefiltered = 0. */
int wgsr_rasterize_forward_cap(const wgsr_raster_args* args, int64_t cap,
                               wgsr_alloc_fn geom_alloc, wgsr_alloc_fn binning_alloc,
                               wgsr_alloc_fn image_alloc, void* alloc_ctx,
                               float* out_color, float* out_depth, float* out_opacity,
                               int32_t* radii, int32_t* n_touched, uint32_t* counts,
                               void* stream);
/* Bytes of the binning buffer wgsr_rasterize_forward_cap requests for `cap`. */
size_t wgsr_binning_bytes_cap(const wgsr_raster_args* args, int64_t cap);

/* Consistency check of a forward's tile lists (test and debug aid, no
 * upstream counterpart): for every tile, its [start, end) lies inside the
 * list region the forward sized from num_rendered (the capacity in capacity
 * mode) and matches its list length, every listed Gaussian id is < P, and no
 * pixel's last contributor lies beyond its tile's list.  Adds the number of
 * bad tiles, bad ids and bad pixels to bad[0..2] (device uint32 words, not
 * zeroed here).  Stream-ordered with no host wait, so it can sit inside a
 * captured graph between the forward and the backward. */
int wgsr_check_tile_lists(const wgsr_raster_args* args, int64_t num_rendered, const void* binning,
                          const void* image, uint32_t* bad, void* stream);

/* Replaces _C.rasterize_gaussians_backward.
 * Inputs: the forward's radii, state buffers and num_rendered; upstream
 * gradients dL_dcolor [3,H,W] and dL_ddepth [1,H,W].
 * Outputs (caller-allocated, fully written, zeros for culled Gaussians):
 * dL_dmeans2D [P,3] (w.r.t. NDC xy; z = 0), dL_dcolors [P,3],
 * dL_dopacity [P,1], dL_dmeans3D [P,3], dL_dcov3D [P,6], dL_dsh [P,M,3]
 * (NULL when M == 0), dL_dscales [P,3], dL_drotations [P,4],
 * dL_dtau [P,6] (per-Gaussian pose gradient, rho then theta).
 * A scratch buffer of ~48 bytes per rendered pair is requested through
 * `scratch_alloc`.  The binning buffer's per-pair flag bytes and the image
 * buffer's backward launch order are written (the same values on every
 * backward of one forward). */
int wgsr_rasterize_backward(const wgsr_raster_args* args, const int32_t* radii,
                            const void* geom_buffer, void* binning_buffer,
                            void* image_buffer, int64_t num_rendered,
                            const float* dL_dcolor, const float* dL_ddepth,
                            wgsr_alloc_fn scratch_alloc, void* alloc_ctx,
                            float* dL_dmeans2D, float* dL_dcolors, float* dL_dopacity,
                            float* dL_dmeans3D, float* dL_dcov3D, float* dL_dsh,
                            float* dL_dscales, float* dL_drotations, float* dL_dtau,
                            void* stream);

/* ---- view-sharded data-parallel backward ----------------
 * No upstream counterpart (the reference is single-GPU; its mapper renders
 * one keyframe view per step, src/mapper.py:1089-1170).  Splits
 * wgsr_rasterize_backward at the per-Gaussian screen-space partial sums so
 * ranks exchange 48 bytes per Gaussian per view instead of all-reducing the
 * 59-float parameter gradients (wgsr/dp.py). */
#define WGSR_VIEW_RECORD_FLOATS 12  /* g[10] (as k_gauss_bwd), radius, SH clamp bits */
#define WGSR_VIEW_CAMERA_FLOATS 64  /* view[16] proj[16] proj_raw[16] campos[3] tanx tany W H, pad */

/* Packs args' camera (viewmatrix, projmatrix, projmatrix_raw, campos,
 * tan_fovx/y, W, H) into one device row of WGSR_VIEW_CAMERA_FLOATS floats. */
int wgsr_pack_view_camera(const wgsr_raster_args* args, float* camera_row, void* stream);

/* First half of wgsr_rasterize_backward for one view: render backward, then
 * per Gaussian i < P_pad one record of WGSR_VIEW_RECORD_FLOATS floats in
 * records [P_pad, 12]: dL/dmean2D (NDC x, y), dL/dconic (3), dL/dopacity,
 * dL/dcolor (3), dL/ddepth, radius (float), SH clamp bits (float).  Rows of
 * culled Gaussians and rows >= P are zero (radius 0 = not visible). */
int wgsr_rasterize_backward_records(const wgsr_raster_args* args, const int32_t* radii,
                                    const void* geom_buffer, void* binning_buffer,
                                    void* image_buffer, int64_t num_rendered,
                                    const float* dL_dcolor, const float* dL_ddepth,
                                    wgsr_alloc_fn scratch_alloc, void* alloc_ctx, int P_pad,
                                    float* records, void* stream);

/* Number of pose-gradient partial rows wgsr_gauss_backward_views writes. */
int wgsr_gauss_backward_views_blocks(int lo, int hi);

/* Second half, for Gaussians [lo, hi) over n_views views: view v's camera is
 * row v of `cameras` [n_views, 64] and its records for the shard start at
 * records + v * record_view_stride (floats; row i - lo).  Writes rows
 * [lo, hi) of dL_dmeans3D [P,3], dL_dsh [P,M,3], dL_dopacity [P,1],
 * dL_dscales [P,3], dL_drotations [P,4] = the SUM over the views of what
 * wgsr_rasterize_backward returns per view.  tau_partials (or NULL):
 * [wgsr_gauss_backward_views_blocks(lo, hi)][n_views][6] per-block sums of
 * the pose gradient (rho, theta) per view.  stats (or NULL): [hi - lo][3] =
 * sum over views of ||dL/dmean2D[:2]||, number of views with radius > 0,
 * max radius (the reference's add_densification_stats inputs).  params uses
 * P, D, M, means3D, scales, rotations, shs, scale_modifier; cov3D_precomp is
 * not supported. */
int wgsr_gauss_backward_views(const wgsr_raster_args* params, int lo, int hi, int n_views,
                              const float* cameras, const float* records,
                              int64_t record_view_stride, float* dL_dmeans3D, float* dL_dsh,
                              float* dL_dopacity, float* dL_dscales, float* dL_drotations,
                              float* tau_partials, float* stats, void* stream);

/* ---- sparse view-sharded exchange (csrc/dp_sparse.hip, wgsr/dp.py) ----
 * Most visible Gaussians get no gradient from a view (their pixels saturate
 * before them), so ranks move only rows with a non-zero record / gradient.
 * No reference counterpart: this replaces the dense exchange behind
 * ViewShardedBackward, which stands in for the reference's per-view
 * optimiser.step() accumulation (mapper.py:1089-1219). */

/* Floats per packed gradient row: index, dL/dmeans3D (3), dL/dsh (3M),
 * dL/dopacity, dL/dscales (3), dL/drotations (4). */
int wgsr_sparse_grad_row_floats(int M);

/* 32-bit mask words per owner segment of S rows: ceil(S / 32). */
int64_t wgsr_sparse_mask_words(int64_t S);

/* records [P_pad, 12] of one view -> per owner o (segment [o S, (o+1) S)),
 * the rows with a non-zero partial sum compacted to packed + o S * 12, field
 * 10 replaced by the row's index inside the segment (uint32 bits).
 * counts[P_pad / S] (zeroed by the caller) receive the rows per owner; with
 * nzmask (zeroed, [P_pad / S][wgsr_sparse_mask_words(S)], may be null) bit j
 * of owner o's words is set for each packed row j.  Row order inside a
 * segment is unspecified. */
int wgsr_sparse_pack_records(const float* records, int64_t P_pad, int64_t S, uint32_t* counts,
                             float* packed, uint32_t* nzmask, void* stream);

/* uint32 words of one rank's block in the exchange's small all-gather:
 * WGSR_VIEW_CAMERA_FLOATS (the camera row's float bits) + world (rows sent to
 * each owner) + world x wgsr_sparse_mask_words(S) (non-zero row masks). */
int64_t wgsr_sparse_summary_block_words(int world, int64_t S);

/* blocks [world][wgsr_sparse_summary_block_words] (every rank's block,
 * gathered) -> summary [world * world + world]: count[v][o] (rows view v sends
 * owner o) then owner o's union row count (rows some view gives gradient);
 * offsets [world + 1]: exclusive prefix over v of count[v][rank] (where view
 * v's rows land in this rank's all_to_all output) and the total; cams
 * [world][WGSR_VIEW_CAMERA_FLOATS]. */
int wgsr_sparse_exchange_summary(const uint32_t* blocks, int world, int rank, int64_t S, uint32_t* summary,
                                 uint32_t* offsets, float* cams, void* stream);

/* Owner side: received [offsets[n_views]][12], view v's packed rows at
 * [offsets[v], offsets[v + 1]), scattered into records [n_views][S][12]
 * (zeroed by the caller) and mask[S] (zeroed) set for every received row.
 * keep_radius: keep the radius field already in `records`
 * (wgsr_sparse_fill_radius), else 1. */
int wgsr_sparse_unpack_records(const float* received, const uint32_t* offsets, int n_views, int64_t S,
                               int keep_radius, float* records, uint8_t* mask, void* stream);

/* records[j].radius = radii[j] for j < n (rows of WGSR_VIEW_RECORD_FLOATS). */
int wgsr_sparse_fill_radius(const float* radii, int64_t n, float* records, void* stream);

/* Gradient rows [lo, hi) whose mask[i - lo] is set -> packed rows of
 * wgsr_sparse_grad_row_floats(M) floats; *count (zeroed) = rows written. */
int wgsr_sparse_pack_grads(int64_t lo, int64_t hi, int M, const uint8_t* mask, const float* dL_dmeans3D,
                           const float* dL_dsh, const float* dL_dopacity, const float* dL_dscales,
                           const float* dL_drotations, uint32_t* count, float* packed, void* stream);

/* gathered: owner r's packed rows at gathered + r * block_stride floats,
 * counts[r] (<= cap) rows, indices into shard r (rows r S + index).  Scatters
 * every owner's rows except `rank`'s into the [P, ...] gradient tensors
 * (zeroed by the caller), or with clear != 0 writes zeros at those rows
 * (undoes an earlier call's scatter, so the tensors need no full re-zeroing). */
int wgsr_sparse_unpack_grads(const float* gathered, int64_t block_stride, const uint32_t* counts, int world,
                             int rank, int64_t cap, int64_t S, int64_t P, int M, float* dL_dmeans3D,
                             float* dL_dsh, float* dL_dopacity, float* dL_dscales, float* dL_drotations,
                             int clear, void* stream);

/* ---- the mapping iteration around the path ----
 * src/mapper.py:1083-1219 per iteration, as fused launches (csrc/mapping.hip;
 * driven by wgsr/mapping.py).  Partial sums are one float (or float pair) per
 * workgroup of wgsr_map_blocks(n) workgroups; callers reduce them in order. */
int wgsr_map_blocks(int64_t n);

/* GaussianModel.get_opacity / get_scaling / get_rotation (gaussian_model.py:
 * sigmoid, exp, F.normalize(eps 1e-12)) of the raw [P,1] / [P,3] / [P,4]
 * parameters, plus iso_partials[wgsr_map_blocks(P)] = per-block sums of
 * sum_k |exp(s_k) - mean_k exp(s_k)| (mapper.py:1167-1169). */
int wgsr_gaussian_activate(int P, const float* opacity_raw, const float* scaling_raw,
                           const float* rotation_raw, float* opacity, float* scales,
                           float* rotations, float* iso_partials, void* stream);

/* Chain rule of wgsr_gaussian_activate back to the raw parameters; adds the
 * gradient of iso_weight * sum |exp(s) - mean_row exp(s)| (iso_weight = 10 /
 * (3 P) for the reference's 10 * isotropic_loss.mean()). */
int wgsr_gaussian_activate_backward(int P, const float* opacity_raw, const float* scaling_raw,
                                    const float* rotation_raw, const float* dL_dopacity,
                                    const float* dL_dscales, const float* dL_drotations,
                                    float iso_weight, float* dL_dopacity_raw,
                                    float* dL_dscaling_raw, float* dL_drotation_raw, void* stream);
/* ... and, in the same pass, wgsr_densification_stats' update of
 * max_radii2D / grad_accum / denom (one launch instead of two).  skip
 * (nullable device word): when non-zero the statistics are left unchanged --
 * pass the capacity-mode forward's overflow word (counts[3]), whose iteration
 * produced no gradient. */
int wgsr_gaussian_activate_backward_stats(int P, const float* opacity_raw, const float* scaling_raw,
                                          const float* rotation_raw, const float* dL_dopacity,
                                          const float* dL_dscales, const float* dL_drotations, float iso_weight,
                                          float* dL_dopacity_raw, float* dL_dscaling_raw, float* dL_drotation_raw,
                                          const int32_t* radii, const float* dL_dmeans2D, float* max_radii2D,
                                          float* grad_accum, float* denom, const uint32_t* skip, void* stream);

/* get_loss_mapping_rgbd (slam_utils.py:107-143) without its SSIM term:
 * image_ab = exp(exposure_a) image + exposure_b ([3,H,W], written for the
 * SSIM kernels); partials[wgsr_map_blocks(H*W)][2] = per-block sums of the
 * boundary-masked rgb L1 (mask: sum_c gt > rgb_threshold) and of the masked
 * depth L1 (gt_depth > 0.01).  exposure_a/b: device scalars. */
int wgsr_mapping_loss_forward(int H, int W, const float* image, const float* gt_image,
                              const float* depth, const float* gt_depth, const float* exposure_a,
                              const float* exposure_b, float rgb_threshold, float* image_ab,
                              float* partials, void* stream);

/* Backward of w_rgb * sum(rgb L1) + w_depth * sum(depth L1) + the SSIM term
 * whose gradient w.r.t. image_ab is ssim_grad ([3,H,W], already scaled; NULL =
 * none): dL_dimage [3,H,W], dL_ddepth [1,H,W] and partials[blocks][2] = per-
 * block sums of dL/dexposure_a and dL/dexposure_b. */
int wgsr_mapping_loss_backward(int H, int W, const float* image, const float* image_ab,
                               const float* gt_image, const float* depth, const float* gt_depth,
                               const float* exposure_a, float rgb_threshold, float w_rgb,
                               float w_depth, const float* ssim_grad, float* dL_dimage,
                               float* dL_ddepth, float* partials, void* stream);

/* ---- The uncertainty-aware mapping loss ---------
 * get_loss_mapping_uncertainty (src/utils/slam_utils.py:146-258) with
 * compute_mapping_loss_components (src/utils/dyn_uncertainty/mapping_utils.py:
 * 206-323): the reference's default mapping loss (uncertainty_params.activate).
 * csrc/uncertainty.hip; driven by wgsr/mapping.py.  Images are [3,H,W] /
 * [1,H,W]; the uncertainty map (the MLP output) is [h,w] (h, w > 2).
 * median_depth: device scalar = ref_depth.median(); the depth threshold is
 * min(10 median, 50).  Partials: per block of wgsr_uncer_blocks(n). */
typedef struct wgsr_uncer_params {
  int H, W;               /* image */
  int h, w;               /* uncertainty map */
  float rgb_threshold;    /* Training.rgb_boundary_threshold */
  float data_rate;        /* 1 + compute_bias_factor(train_frac, 0.8) */
  float ssim_weight;      /* 100 + 900 compute_bias_factor(ssim_frac, 0.8) */
  float opacity_th;       /* uncertainty_params.opacity_th_for_uncer_loss */
  float uncer_depth_mult; /* uncertainty_params.uncer_depth_mult */
  int initialization;     /* 1: no exposure correction */
  int pre_exposed;        /* 1: fuse the mapper's own exposure step: map_opt_online passes
                             exp(a) x + b into the loss (mapper.py:1127-1129), which applies
                             it again (slam_utils.py:179-181).  `image` is the raw render,
                             image_ab = exp(a) (exp(a) x + b) + b, and the image and
                             exposure gradients chain through both applications. */
} wgsr_uncer_params;
int wgsr_uncer_blocks(int64_t n);
/* image_ab = exp(a) image + b (applied twice when pre_exposed); partials[blocks(H*W)][3] = sums of
 * w * masked rgb L1 (over channels), of w, and of the re-weighted depth L1
 * (w where ref_depth < depth + 1), w = the uncertainty weight map. */
int wgsr_uncer_loss_forward(const wgsr_uncer_params* prm, const float* image, const float* gt_image,
                            const float* depth, const float* ref_depth, const float* exposure_a,
                            const float* exposure_b, const float* uncertainty, const float* median_depth,
                            float* image_ab, float* partials, void* stream);
/* The feature-resolution inputs of the uncertainty loss: bilinear downsamples
 * of the opacity image and of clip(opacity ssim_weight (1-l)(1-s)(1-c), 5)
 * (l, c, s: wgsr_ssim_components of (gt, image_ab), full resolution) and the
 * bicubic clipped depth L1, zeroed where the bicubic ref depth > threshold. */
int wgsr_uncer_small_maps(const wgsr_uncer_params* prm, const float* opacity, const float* depth,
                          const float* ref_depth, const float* median_depth, const float* luminance,
                          const float* contrast, const float* structure, float* small_ssim_loss,
                          float* small_depth_loss, float* small_opacity, void* stream);
/* uncertainty_loss (5x5 reflect median of the SSIM loss; zero where the small
 * opacity < opacity_th): loss_map [h,w] (optional), partials[blocks(h*w)],
 * dL_duncertainty = grad_scale * d(loss)/d(uncertainty) (optional; grad_scale
 * = ssim_mult / (h w) for the reference's ssim_mult * mean). */
int wgsr_uncer_loss_small(const wgsr_uncer_params* prm, const float* uncertainty, const float* small_ssim_loss,
                          const float* small_depth_loss, const float* small_opacity, float grad_scale,
                          float* loss_map, float* partials, float* dL_duncertainty, void* stream);
/* The loss epilogue in one launch: fixed-order sums of partials
 * ([blocks(H*W)][3] from wgsr_uncer_loss_forward) and small_partials
 * (wgsr_uncer_loss_small), *loss = alpha rgb + (1 - alpha) depth + ssim_mult
 * mean(uncertainty loss) + extra_weight sum(extra_partials[n_extra]) (e.g. the
 * isotropic term), sums[3] = the three full-resolution sums, ssim_scale[3] =
 * the SSIM backward's per-plane dL/dS (ssim_mean: device scalar from
 * wgsr_ssim_forward; ignored unless ssim_loss). */
int wgsr_uncer_loss_combine(const wgsr_uncer_params* prm, const float* partials, const float* small_partials,
                            const float* ssim_mean, const float* extra_partials, int n_extra, float extra_weight,
                            float alpha, float lambda_dssim, float ssim_mult, int ssim_loss, float* loss,
                            float* sums, float* ssim_scale, void* stream);
/* wgsr_uncer_loss_combine taking the SSIM forward's tile partials
 * (wgsr_ssim_forward_partials of the 3 planes) instead of its mean: the
 * partials are reduced in this launch, in k_ssim_reduce's order (the same
 * mean, bit for bit), and the mean written to ssim_mean (may be NULL). */
int wgsr_uncer_loss_combine_ssim(const wgsr_uncer_params* prm, const float* partials, const float* small_partials,
                                 const float* ssim_partials, float* ssim_mean, const float* extra_partials,
                                 int n_extra, float extra_weight, float alpha, float lambda_dssim, float ssim_mult,
                                 float* loss, float* sums, float* ssim_scale, void* stream);
/* dL_dimage / dL_ddepth of loss_grad x (w_rgb sum(w rgb L1) + w_depth
 * sum(re-weighted depth L1)) + the SSIM term (ssim_grad: its gradient w.r.t.
 * image_ab, already scaled; NULL = none); loss_grad: device scalar (NULL = 1);
 * partials[blocks(H*W)][2] = dL/dexposure_a, _b.  exposure_b is read only
 * when pre_exposed (NULL otherwise allowed). */
int wgsr_uncer_loss_backward(const wgsr_uncer_params* prm, const float* image, const float* image_ab,
                             const float* gt_image, const float* depth, const float* ref_depth,
                             const float* exposure_a, const float* exposure_b, const float* uncertainty, const float* median_depth,
                             float w_rgb, float w_depth, const float* loss_grad, const float* ssim_grad,
                             float* dL_dimage, float* dL_ddepth, float* partials, void* stream);

/* ---- The mapper's pose-refinement loss (tracking) --
 * csrc/tracking.hip; driven by wgsr/tracking.py.
 * wgsr_tracking_loss: get_loss_tracking(..., monocular=True) (src/utils/
 * slam_utils.py:47-82) forward AND backward in one pass: partials[blocks(H*W)]
 * [3] = per-block sums of the opacity-weighted L1 (divide by 3HW for the
 * loss), of dL/dexposure_a and of dL/dexposure_b; dL_dimage [3,H,W] and
 * dL_dopacity [1,H,W] (optional) for dL/dloss = 1.  grad_mask ([1,H,W], the
 * keyframe's Camera.grad_mask) and uncertainty ([H,W], already resized) are
 * optional (NULL: ones / no weights). */
int wgsr_track_blocks(int64_t n);
int wgsr_tracking_loss(int H, int W, const float* image, const float* gt_image, const float* opacity,
                       const float* grad_mask, const float* uncertainty, const float* exposure_a,
                       const float* exposure_b, float rgb_threshold, float* dL_dimage, float* dL_dopacity,
                       float* partials, void* stream);
/* One pose-refinement update (mapper.py:884-906 after loss.backward()): Adam
 * (torch semantics; bias corrections of `step`) over cam_rot_delta (grad =
 * dtau[3:6]), cam_trans_delta (dtau[0:3]), exposure_a / exposure_b (sums of
 * columns 1 / 2 of wgsr_tracking_loss's partials), then update_pose
 * (pose_utils.py:81-98: w2c <- SE3_exp([trans, rot]) w2c, deltas back to 0,
 * *converged = |tau| < threshold) and the next iteration's rasteriser camera
 * (viewmatrix, projmatrix, campos).  state: wgsr_pose_state_floats() floats,
 * layout in csrc/tracking.hip (R, T, exposures, Adam moments, camera).
 * camera_only = 1 only writes the camera fields from the stored (R, T). */
int wgsr_pose_state_floats(void);
int wgsr_pose_step(float* state, const float* dtau, const float* loss_partials, int n_partials,
                   const float* projection_matrix, float lr_rot, float lr_trans, float lr_exposure, float beta1,
                   float beta2, float eps, int step, float converged_threshold, int* converged, int camera_only,
                   void* stream);
/* Camera.compute_grad_mask (src/utils/camera_utils.py:157-180): grad_mask
 * [H,W] of the [3,H,W] image (edge_threshold: Training.edge_threshold).
 * Needs (H/32)(W/32) <= 8192. */
int wgsr_grad_mask(int H, int W, const float* image, float edge_threshold, float* grad_mask, void* stream);

/* ---- The uncertainty MLP ------------------------
 * uncertainty_model.MLPNetwork with its defaults (src/utils/dyn_uncertainty/
 * uncertainty_model.py:5-68): C -> 64 -> 64 -> 1, ReLU, dropout p after each
 * hidden layer, softplus.  csrc/mlp.hip; driven by wgsr/mlp.py.  X [N][C]
 * (C a multiple of 64), weights row-major as torch.nn.Linear keeps them.
 * Forward keeps h1d/h2d ([N][64], post-dropout) and o_pre ([N]) for the
 * backward; dropout masks are a counter hash of (seed, layer, row, column).
 * Backward: grad (wgsr_mlp_grad_floats(C) floats) = dW1 [64][C] | db1 [64] |
 * dW2 [64][64] | db2 [64] | dW3 [64] | db3 [1] for dL_du [N]; scratch:
 * wgsr_mlp_scratch_bytes(N, C). */
size_t wgsr_mlp_scratch_bytes(int N, int C);
int wgsr_mlp_grad_floats(int C);
int wgsr_mlp_forward(int N, int C, const float* X, const float* W1, const float* b1, const float* W2,
                     const float* b2, const float* W3, const float* b3, float dropout_p, uint32_t seed,
                     float* h1d, float* h2d, float* o_pre, float* u, void* stream);
/* wgsr_mlp_forward with the dropout seed read from device memory (a
 * graph-replayed mapping iteration draws a new seed per step). */
int wgsr_mlp_forward_dev_seed(int N, int C, const float* X, const float* W1, const float* b1, const float* W2,
                              const float* b2, const float* W3, const float* b3, float dropout_p,
                              const uint32_t* seed, float* h1d, float* h2d, float* o_pre, float* u, void* stream);
/* keys[i] = 31-bit hash of (seed, i), i < n (seed_dev, when not NULL, holds
 * the seed): sorting the keys gives the DINO term's random sample order. */
int wgsr_random_keys(int64_t n, uint32_t seed, const uint32_t* seed_dev, int32_t* keys, void* stream);
/* perm[0..n) = the stable ascending order of wgsr_random_keys(n, seed) (the
 * DINO term's sample draw) in two launches; keys: n words of scratch.
 * n <= wgsr_random_perm_max(). */
int64_t wgsr_random_perm_max(void);
int wgsr_random_perm(int64_t n, uint32_t seed, const uint32_t* seed_dev, uint32_t* keys, int32_t* perm,
                     void* stream);
/* perm[0..k) = the first k entries of wgsr_random_perm's permutation (the
 * DINO term keeps only n / reg_stride^4 of the draw), in one launch and
 * without a sort of all n; n <= wgsr_random_perm_prefix_max_n(),
 * k <= min(n, wgsr_random_perm_prefix_max_k()). */
int64_t wgsr_random_perm_prefix_max_n(void);
int64_t wgsr_random_perm_prefix_max_k(void);
int wgsr_random_perm_prefix(int64_t n, int64_t k, uint32_t seed, const uint32_t* seed_dev, int32_t* perm,
                            void* stream);
/* Two uncertainty-MLP forwards in one launch (the mapping iteration's
 * keyframe features and the DINO term's sample): rows [0, N1) are X1's with
 * the dropout seed *seed1, rows [N1, N1 + N2) X2's with *seed2 -- each
 * segment's dropout draw is the one its own wgsr_mlp_forward_dev_seed would
 * make; h1d / h2d / o_pre / u hold N1 + N2 rows.  The backward sums both
 * segments' parameter gradients (upstream du1 x du_scale1 and du2 x
 * du_scale2) into grad (added to it with accumulate != 0); scratch:
 * wgsr_mlp_scratch_bytes(N1 + N2, C). */
int wgsr_mlp_forward_seg2(int N1, int N2, int C, const float* X1, const float* X2, const float* W1, const float* b1,
                          const float* W2, const float* b2, const float* W3, const float* b3, float dropout_p,
                          const uint32_t* seed1, const uint32_t* seed2, float* h1d, float* h2d, float* o_pre,
                          float* u, void* stream);
int wgsr_mlp_backward_seg2(int N1, int N2, int C, const float* X1, const float* X2, const float* W2, const float* W3,
                           float dropout_p, const float* h1d, const float* h2d, const float* o_pre, const float* du1,
                           const float* du2, float du_scale1, float du_scale2, int accumulate, float* scratch,
                           float* grad, void* stream);
/* wgsr_mlp_backward with dL_du scaled by du_scale, and with accumulate != 0
 * the gradient ADDED to grad (a second backward into the same parameters,
 * as autograd accumulates). */
int wgsr_mlp_backward_acc(int N, int C, const float* X, const float* W2, const float* W3, float dropout_p,
                          const float* h1d, const float* h2d, const float* o_pre, const float* dL_du, float du_scale,
                          int accumulate, float* scratch, float* grad, void* stream);
int wgsr_mlp_backward(int N, int C, const float* X, const float* W2, const float* W3, float dropout_p,
                      const float* h1d, const float* h2d, const float* o_pre, const float* dL_du,
                      float* scratch, float* grad, void* stream);

/* DINO feature-similarity regulariser: compute_dino_regularization_loss
 * (src/utils/dyn_uncertainty/mapping_utils.py:332-389, replaces its
 * normalize / N x N matmul / topk / gathers on the mapper's uncertainty
 * branch, mapper.py:986-997, 1122-1140).  u [N] uncertainty samples, feat
 * [N, C] features (row-major).  Writes loss[0] = mean_i var_i over the
 * min(top_k, N) most similar samples with cosine similarity > thresh, and
 * grad_u [N] = d loss / d u (zeroed by the call; float atomics, so the
 * order of its adds is not fixed).  Scratch: fn [N, C], sim [N, N], row_var
 * [N].  N <= 16384, thresh > 0.  loss may be NULL: the gradient only (one
 * launch fewer). */
int wgsr_dino_reg(const float* u, const float* feat, int N, int C, int top_k, float thresh, float eps,
                  float* fn_scratch, float* sim_scratch, float* row_var, float* grad_u, float* loss, void* stream);

/* One view's densification bookkeeping (mapper.py:1177-1183,
 * gaussian_model.py:745-749) for Gaussians with radii > 0:
 * max_radii2D = max(max_radii2D, radii); grad_accum += ||dL_dmeans2D[:2]||;
 * denom += 1. */
int wgsr_densification_stats(int P, const int32_t* radii, const float* dL_dmeans2D,
                             float* max_radii2D, float* grad_accum, float* denom, void* stream);

/* Replaces _C.mark_visible: present[i] = (view-space z of point i > 0.2). */
int wgsr_mark_visible(int P, const float* means3D, const float* viewmatrix,
                      const float* projmatrix, uint8_t* present, void* stream);

/* Replaces simple_knn._C.distCUDA2: out[i] = mean of the squared distances
 * to the 3 nearest other points of `points` [P,3] (exact). */
int wgsr_dist_cuda2(int P, const float* points, float* out,
                    wgsr_alloc_fn scratch_alloc, void* alloc_ctx, void* stream);

/* ---- what follows the rasteriser each iteration ---- */

/* One Adam parameter tensor (contiguous fp32, `numel` elements).  The host
 * supplies torch.optim.Adam's per-step scalars: step_size = lr / (1 -
 * beta1^step), bias_correction2_sqrt = sqrt(1 - beta2^step). */
typedef struct wgsr_adam_tensor {
  float* param;
  const float* grad;
  float* exp_avg;
  float* exp_avg_sq;
  int64_t numel;
  float step_size;
  float bias_correction2_sqrt;
  /* Optional two-rate split (0 = off): element e with e % split_period >=
   * split_len steps with step_size_tail instead of step_size.  Lets one
   * [P,16,3] SH storage carry the reference's f_dc (first 3 floats of each
   * 48, lr 2.5e-3) and f_rest (lr / 20) parameter groups in one tensor. */
  int64_t split_period;
  int64_t split_len;
  float step_size_tail;
} wgsr_adam_tensor;
#define WGSR_ADAM_MAX_TENSORS 16

/* Replaces optimizer.step() of the reference's torch.optim.Adam(param_groups,
 * lr=0.0, eps=1e-15) (gaussian_model.py:309; no weight decay, no amsgrad)
 * for up to WGSR_ADAM_MAX_TENSORS tensors in one launch, element arithmetic
 * in torch's order: exp_avg.lerp_(grad, 1-beta1);
 * exp_avg_sq.mul_(beta2).addcmul_(grad, grad, 1-beta2);
 * param.addcdiv_(exp_avg, sqrt(exp_avg_sq)/bias_correction2_sqrt + eps,
 * -step_size).  beta1/beta2/eps are the Python (double) hyper-parameters:
 * 1-beta is formed in double and rounded once, as torch does. */
int wgsr_adam_step(const wgsr_adam_tensor* tensors, int n, double beta1, double beta2, double eps,
                   void* stream);

/* wgsr_adam_step with the per-step scalars in DEVICE memory, for a step
 * replayed from a HIP graph: tensor i uses scalars[3 i + 0..2] = step_size,
 * bias_correction2_sqrt, step_size_tail (its own fields are ignored);
 * skip (or NULL): no update at all when *skip != 0 (a capacity-mode forward
 * that overflowed); weight_decay: torch.optim.Adam's L2 term, the gradient
 * used is grad + weight_decay * param (0: none). */
int wgsr_adam_step_dev(const wgsr_adam_tensor* tensors, int n, double beta1, double beta2, double eps,
                       double weight_decay, const float* scalars, const uint32_t* skip, void* stream);
/* Two optimisers sharing beta1 / beta2 in one launch (the Gaussians' and the
 * uncertainty MLP's in the mapping iteration): tensors [0, n1) step with
 * eps1 / weight_decay1 / scalars1, tensors [n1, n) with eps2 /
 * weight_decay2 / scalars2 (3 floats per tensor, from tensor n1 on). */
int wgsr_adam_step_dev2(const wgsr_adam_tensor* tensors, int n1, int n, double beta1, double beta2, double eps1,
                        double weight_decay1, const float* scalars1, double eps2, double weight_decay2,
                        const float* scalars2, const uint32_t* skip, void* stream);

/* ---- The graph-replayed mapping iteration (wgsr/online_graph.py) -------
 * No reference counterpart: device-side steps that let one captured graph
 * serve every keyframe (mapper.py:1083-1219 per iteration). */
typedef struct wgsr_gather_job {
  const void* src;            /* rows of src_stride_words 32-bit words       */
  void* dst;                  /* nrows contiguous rows of row_words words    */
  int64_t row_words;
  int64_t src_stride_words;   /* >= row_words                                */
  int32_t idx_offset;         /* row r of dst = src row idx[idx_offset + r]  */
  int32_t nrows;
} wgsr_gather_job;
#define WGSR_GATHER_MAX_JOBS 8
/* Every job's rows in one launch (the chosen keyframe's image, depth,
 * features, camera, median depth and exposure, its neighbours' features). */
int wgsr_gather_rows(const wgsr_gather_job* jobs, int n, const int64_t* idx, void* stream);
/* The keyframe exposure optimiser's step (torch.optim.Adam arithmetic, as
 * wgsr_adam_step) on row idx[0] of bank [K][3][2] = (a, b), exp_avg,
 * exp_avg_sq, with grad = the sum of nparts (a, b) rows (the loss
 * backward's per-block partials, added in a fixed order; nparts = 1: the
 * gradient itself) and scalars = (step_size, sqrt(1 - beta2^n)); skipped
 * when *skip_a or *skip_b is non-zero.  With sticky and counts (the
 * capacity-mode forward's, or NULL): sticky[0] += counts[3], sticky[1] =
 * max(sticky[1], counts[0]).  slot_skips (nullable, one word per bank row):
 * slot_skips[idx[0]] += 1 when the step was meant to run (*skip_b == 0) but
 * *skip_a held it back, so the host can roll back that row's step count. */
int wgsr_exposure_step(float* bank, const int64_t* idx, const float* grad, int nparts, const float* scalars,
                       const uint32_t* skip_a, const uint32_t* skip_b, double beta1, double beta2, double eps,
                       int64_t* sticky, const uint32_t* counts, int64_t* slot_skips, void* stream);

/* One row-major tensor for row compaction: rows of `row_bytes` (a multiple
 * of 4) from `src` [P rows]; `dst` receives the kept rows in order. */
typedef struct wgsr_row_tensor {
  const void* src;
  void* dst;
  int64_t row_bytes;
} wgsr_row_tensor;
#define WGSR_COMPACT_MAX_TENSORS 32

/* Replaces prune_points / _prune_optimizer's `t[keep]` (gaussian_model.py:
 * 526-564) over up to WGSR_COMPACT_MAX_TENSORS per-Gaussian tensors at once:
 * dst_i = src_i[keep] for every tensor (keep: [P] bytes, 0/1).  Each dst must
 * hold sum(keep) rows. */
int wgsr_compact_rows(const uint8_t* keep, int64_t P, const wgsr_row_tensor* tensors, int n,
                      wgsr_alloc_fn scratch_alloc, void* alloc_ctx, void* stream);

/* ---- densification on the device (csrc/densify.hip, wgsr/store.py) -------
 * The GaussianModel state lives in a capacity-preallocated SoA of two banks;
 * one bank = the five parameter tensors (xyz [C,3], features [C,M,3],
 * opacity [C,1], scaling [C,3], rotation [C,4]; raw, as GaussianModel's
 * _xyz ... _rotation), their Adam moments in that order, and per-row
 * keyframe ids / observation counts (optional).  Rows are addressed by
 * index; a densify reads one bank and writes the other. */
typedef struct wgsr_gaussian_bank {
  float* xyz;
  float* features;
  float* opacity;
  float* scaling;
  float* rotation;
  float* exp_avg[5];
  float* exp_avg_sq[5];
  int32_t* kf_id;
  int32_t* n_obs;
} wgsr_gaussian_bank;

/* Workgroups of the select / emit kernels over P rows; block_counts holds
 * 4 x (wgsr_densify_blocks(P) + 1) uint32. */
int64_t wgsr_densify_blocks(int64_t P);

/* Replaces the selection of GaussianModel.densify_and_prune(max_grad,
 * min_opacity, extent, max_screen_size) (gaussian_model.py:646-743):
 * grad_threshold = max_grad (> 0), dense_threshold = percent_dense * extent,
 * world_threshold = 0.1 * extent, use_screen_size = bool(max_screen_size).
 * Per row a flag byte (kept original, kept clone, kept split pair, split
 * selected) and, after the built-in scan, block_counts = exclusive per-block
 * offsets of the four regions with the totals (kept originals Ko, kept
 * clones Kc, kept split rows per copy Ks, selected split rows Ns) at
 * [4 * wgsr_densify_blocks(P)].  New row count: Ko + Kc + 2 Ks.
 * With prune_mask (bytes, 1 = prune) instead: prune_points(mask)
 * (gaussian_model.py:548-564) -- only kept originals. */
int wgsr_densify_select(int64_t P, const float* accum, const float* denom, const float* opacity,
                        const float* scaling, const uint8_t* prune_mask, float grad_threshold,
                        float dense_threshold, float min_opacity, float world_threshold, int use_screen_size,
                        float max_screen_size, uint8_t* flags, uint32_t* block_counts, void* stream);

/* Writes the densified / pruned table into bank dst (capacity >= the new row
 * count): kept originals with their moments, then kept clones, kept split
 * copies A and B (zero moments): split xyz = R(q) (z * exp(s)) + xyz with z
 * [2 Ns, 3] standard-normal samples (copy A rows first, by selection rank),
 * split scaling = log(exp(s) / 1.6). */
int wgsr_densify_emit(int64_t P, int M, const uint8_t* flags, const uint32_t* block_counts, const float* z,
                      const wgsr_gaussian_bank* src, const wgsr_gaussian_bank* dst, void* stream);

/* reset_opacity (visible = null, value = inverse_sigmoid(0.01)) and
 * reset_opacity_nonvisible (value = inverse_sigmoid(0.4); visible rows get
 * sigmoid(raw): the reference writes get_opacity[filter] into the raw
 * tensor) (gaussian_model.py:389-402); the opacity moments -> 0. */
int wgsr_reset_opacity(int64_t P, float* opacity_raw, const uint8_t* visible, float value, float* exp_avg,
                       float* exp_avg_sq, void* stream);

/* ---- map deformation (csrc/deform.hip, wgsr/store.py) ---------------------
 * One keyframe's pose / depth update of Mapper._update_mapping_points
 * (src/mapper.py:431-558; caller: _update_keyframes_from_frontend,
 * mapper.py:365-429).  Host-computed, fp32, row-major:
 *   T       = inv(inv(w2c_old) @ w2c_new)                (mapper.py:449 / 530)
 *   q       = rotation_matrix_to_quaternion(T) (w,x,y,z)  (general_utils.py:138-162)
 *   w2c_old, c2w_old = inv(w2c_old), K (the mapper's 3x3 intrinsics), depth /
 *   depth_old ([H,W] device maps) -- the depth-rescale branch (method 1) only. */
typedef struct wgsr_deform_frame {
  int32_t kf_id;
  int32_t method;       /* 0 = "rigid", 1 = depth rescale (method=None)      */
  float T[16];
  float q[4];
  float w2c_old[16];
  float c2w_old[16];
  float K[9];
  int32_t H, W;
  const float* depth;
  const float* depth_old;
} wgsr_deform_frame;

/* Applies every frame of `frames` (DEVICE array of nframes) to the rows of
 * `bank` anchored to its keyframe (lut: DEVICE [lut_size] int32, kf_id ->
 * frame index or -1): xyz, rotation (and scaling for method 1) as the
 * reference does, and -- when any frame has rows -- every row's rotation
 * normalised and the xyz / rotation (and, with a method-1 frame that has rows,
 * scaling) Adam moments zeroed (replace_tensor_to_optimizer,
 * gaussian_model.py:495-508).  flags: DEVICE scratch of 2 uint32. */
int wgsr_deform_points(int64_t P, const wgsr_gaussian_bank* bank, const wgsr_deform_frame* frames, int nframes,
                       const int32_t* lut, int lut_size, uint32_t* flags, void* stream);

/* ---- SSIM for the mapping loss -------------------
 * Images are `planes` contiguous H x W fp32 planes (any leading dims
 * flattened; zero padding at the borders, as F.conv2d(padding=ws//2)).
 * window_size in {3,5,7,9,11}; Gaussian window, sigma 1.5.
 *
 * wgsr_ssim_forward replaces loss_utils.ssim(img1, img2, window_size)
 * (thirdparty/gaussian_splatting/utils/loss_utils.py:61-101): *mean = mean
 * SSIM over all pixels (size_average=True), plane_mean[p] (optional) = per
 * plane mean.  dmap (optional, 3 x planes x H x W floats) receives the
 * per-pixel derivatives the backward needs (dS/dmu1, dS/dE[x^2], dS/dE[xy]).
 * Scratch: wgsr_ssim_scratch_bytes(planes, H, W) through scratch_alloc. */
size_t wgsr_ssim_scratch_bytes(int64_t planes, int H, int W);
int wgsr_ssim_forward(const float* img1, const float* img2, int64_t planes, int H, int W, int window_size,
                      float* dmap, float* plane_mean, float* mean, wgsr_alloc_fn scratch_alloc, void* alloc_ctx,
                      void* stream);
/* The SSIM forward without its reduction launch: per-tile partial sums
 * (wgsr_ssim_tiles(H, W) per plane, plane-major) into `partials`, for a
 * consumer that reduces them itself (wgsr_uncer_loss_combine_ssim). */
int wgsr_ssim_forward_partials(const float* img1, const float* img2, int64_t planes, int H, int W, int window_size,
                               float* dmap, float* partials, void* stream);
int wgsr_ssim_tiles(int H, int W);
/* dL/dimg1 of the forward above given plane_scale[p] = dL/dS for every pixel
 * of plane p (device array; e.g. dL/dmean / (planes*H*W)).  img2 gets no
 * gradient (the reference passes the ground-truth image there). */
int wgsr_ssim_backward(const float* img1, const float* img2, int64_t planes, int H, int W, int window_size,
                       const float* dmap, const float* plane_scale, float* grad_img1, void* stream);
/* compute_ssim_components(img1, img2, window_size) (src/utils/dyn_uncertainty/
 * mapping_utils.py:99-204) for `images` images of `channels` planes each:
 * channel means of the clipped luminance, contrast and structure maps
 * (each images x H x W).  Forward only (the reference detaches them). */
int wgsr_ssim_components(const float* img1, const float* img2, int64_t images, int channels, int H, int W,
                         int window_size, float* luminance, float* contrast, float* structure, void* stream);

/* ---- PLY vertex records ------------------------
 * GaussianModel.save_ply / load_ply (gaussian_model.py:338-493) keep the
 * Gaussians as P fixed-size records of `ncol` float32 properties.  A column
 * set names one contiguous device tensor [P, cols] and, for each of its
 * columns, the record column it maps to.  pack writes records (record
 * columns no set maps -- the reference's zero normals -- become 0); unpack
 * reads them.  Both run on the device (LDS transpose, coalesced on both
 * sides); the host moves only the record block between file and HBM. */
#define WGSR_PLY_MAX_TENSORS 8
#define WGSR_PLY_MAX_COLS 128
typedef struct wgsr_ply_column_set {
  float* data;              /* [P, cols] contiguous fp32 (device) */
  int cols;
  const int* record_col;    /* host array [cols] */
} wgsr_ply_column_set;
int wgsr_ply_pack(const wgsr_ply_column_set* sets, int ntens, int64_t P, int ncol, float* records, void* stream);
int wgsr_ply_unpack(const float* records, int64_t P, int ncol, const wgsr_ply_column_set* sets, int ntens,
                    void* stream);

/* Byte sizes of the forward state buffers (for callers that pre-allocate). */
size_t wgsr_geometry_bytes(int P);
size_t wgsr_binning_bytes(int64_t num_rendered, int W, int H);
size_t wgsr_image_bytes(int W, int H);

/* Optional per-stage timing: HIP events recorded on the caller's stream
 * around each stage (preprocess, depth_sort, offsets_scan, duplicate,
 * tile_sort, ranges, render_fwd, render_bwd, gauss_bwd, dist_cuda2).
 * wgsr_profile_read synchronises on the recorded events and returns the
 * accumulated milliseconds and launch counts per stage (returns the number
 * of stages).  Not thread-safe; meant for benchmarks. */
#define WGSR_NUM_STAGES 10
/* on = 0: off; 1: every stage; (mask << 1) for mask != 0: only the stages
 * whose bit is set (bit i = stage i), e.g. (1 << 7) << 1 times render_bwd
 * alone -- each timed stage adds two event records to the stream. */
void wgsr_profile_enable(int on);
int wgsr_profile_read(double* ms, int64_t* counts, int n, int reset);
const char* wgsr_profile_stage_name(int i);

const char* wgsr_last_error(void);
const char* wgsr_version(void);

/* Byte offset, inside the geometry buffer of this thread's last
 * wgsr_rasterize_forward call, of its depth order: P uint32 Gaussian ids by
 * ascending view-space depth (ties in index order, culled Gaussians last) --
 * the order upstream's (tile | depth) key sort gives every tile list.  Only
 * WGSR_DEPTH_SORT=global (three passes over the visible key range) or =full
 * (four 8-bit passes over the whole keys), or sort bins off, produce one;
 * where it lands varies.  -1 when the last forward had none: by default the
 * entries of every sort bin are ordered by depth after the bin sort. */
int64_t wgsr_depth_order_offset(void);

#ifdef __cplusplus
}
#endif
#endif /* WGSR_H */

/*
 * omnigs_raster.h — C ABI of the MI355X (gfx950) omnidirectional Gaussian-splat rasterizer.
 *
 * These entry points replace, one for one, the raw-pointer rasterizer interface of OmniGS
 * (raikuma/OmniGS-fork @ 2025-03-04, cuda_rasterizer/rasterizer.h:28-156):
 *
 *   omr_rasterizer_mark_visible  <- CudaRasterizer::Rasterizer::markVisible        (rasterizer.h:32-37)
 *   omr_rasterizer_forward       <- CudaRasterizer::Rasterizer::forward            (rasterizer.h:39-62)
 *   omr_rasterizer_backward      <- CudaRasterizer::Rasterizer::backward           (rasterizer.h:64-93)
 *   omr_lonlat_mark_visible      <- CudaRasterizer::LonlatRasterizer::markVisible  (rasterizer.h:98-100)
 *   omr_lonlat_forward           <- CudaRasterizer::LonlatRasterizer::forward      (rasterizer.h:102-121)
 *   omr_lonlat_backward          <- CudaRasterizer::LonlatRasterizer::backward     (rasterizer.h:124-154)
 *
 * and sit under the LibTorch boundary of include/rasterize_points.h (RasterizeGaussiansCUDA /
 * RasterizeGaussiansBackwardCUDA / markVisible, reference include/rasterize_points.h:29-80), which
 * omnigs-fork_amd/csrc/rasterize_points.cpp implements on top of them.
 *
 * Conventions (same as the reference unless stated):
 *   - all pointers are device pointers on the current HIP device, fp32 unless typed otherwise;
 *     means3D [P,3], shs [P,M,3], colors_precomp [P,3], opacities [P], scales [P,3], rotations [P,4]
 *     (r,x,y,z; not renormalised), cov3D_precomp [P,6], viewmatrix / projmatrix 16 floats column-major
 *     (Tcw^T, (P Tcw)^T as tensors), cam_pos [3], background [3];
 *   - NULL for shs / colors_precomp / scales / rotations / cov3D_precomp means "absent" (the reference tests
 *     data_ptr() != nullptr of empty tensors);
 *   - out_color is [3,H,W]; radii [P] int32 (NULL: internal buffer, as the reference);
 *   - scratch memory comes from three allocation callbacks (geometry, binning, image) replacing the
 *     reference's std::function<char*(size_t)>; the returned memory must stay valid and be passed back
 *     unchanged to the backward call together with R = *num_rendered; its layout is private;
 *   - `stream` is a hipStream_t (NULL = legacy default stream). The forward does not wait for the GPU before it
 *     has queued all its kernels: the binning buffer is sized from a capacity hint (the last num_rendered of the
 *     view shape + 12.5 %) instead of the reference's mid-forward cudaMemcpy (rasterizer_impl.cu:628); the call
 *     then waits for num_rendered to return it (and re-runs the binning at the exact size if the hint was short);
 *   - ADDED vs the reference: the backward writes EVERY element of its gradient outputs (zeros where the
 *     reference leaves its zero-initialised tensors untouched), so they need not be zeroed by the caller.
 *     dL_dconic ([P,4], slots 0,1,3) and, for lonlat, dpx_dt / dpy_dt ([P,3]) are optional (NULL = skip), and
 *     so is dL_dsh (its SH backward still feeds dL_dmean3D; a view-parallel host rebuilds the summed SH gradient
 *     from the colour gradients instead, omr_sh_grad_from_colors_packed);
 *   - the forward keeps, in the geometry buffer, what the backward would otherwise recompute from the inputs it
 *     is passed again: with 16-coefficient SH rows, each visible Gaussian's dRGB/ddir (from the forward's SH
 *     rows and camera position). The backward must therefore be given the forward's inputs, as the reference's
 *     autograd callers do (its gradients are those of that forward). CONTRACT: the SH array, means3D and campos
 *     must not be modified in place between a forward and its backward. The backward recognises other arrays or
 *     another campos by a key of their addresses and the campos bits, and then recomputes dRGB/ddir from the SH
 *     it is given as the reference does (backward.cu:56-112). The key does not cover the contents: an in-place
 *     edit at the same addresses yields the gradients of the forward's SH/means;
 *   - errors: calls return OMR_OK (0) or an OMR_ERR_* code; omr_last_error() gives the message of the last
 *     failing call on this thread. The reference throws std::runtime_error / traps instead.
 */
#ifndef OMNIGS_RASTER_H
#define OMNIGS_RASTER_H

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OMR_ABI_VERSION 1

enum omr_status {
    OMR_OK = 0,
    OMR_ERR_INVALID_ARGUMENT = 1, /* bad sizes / missing required pointer */
    OMR_ERR_CAMERA_TYPE = 2,      /* "[CudaRasterizer]Invalid camera_type" (rasterize_points.cu:160) */
    OMR_ERR_ALLOCATION = 3,       /* an allocation callback returned NULL */
    OMR_ERR_HIP = 4,              /* a HIP runtime / launch error */
    OMR_ERR_PREFILTERED = 5,      /* prefiltered set but a point was culled (auxiliary.h:183-187 traps) */
};

enum omr_camera_type { OMR_CAMERA_PINHOLE = 1, OMR_CAMERA_LONLAT = 3 };

/* replaces std::function<char*(size_t)> (rasterizer.h:43-45); must return device memory of >= bytes */
typedef void* (*omr_alloc_fn)(void* ctx, size_t bytes);

int omr_abi_version(void);
const char* omr_last_error(void);

/* --- pinhole (camera_type = 1) ------------------------------------------------------------------- */
int omr_rasterizer_mark_visible(int P, const float* means3D, const float* viewmatrix, const float* projmatrix,
                                bool* present, void* stream);

int omr_rasterizer_forward(omr_alloc_fn geometry_alloc, void* geometry_ctx, omr_alloc_fn binning_alloc,
                           void* binning_ctx, omr_alloc_fn image_alloc, void* image_ctx, int P, int D, int M,
                           const float* background, int width, int height, const float* means3D, const float* shs,
                           const float* colors_precomp, const float* opacities, const float* scales,
                           float scale_modifier, const float* rotations, const float* cov3D_precomp,
                           const float* viewmatrix, const float* projmatrix, const float* cam_pos, float tan_fovx,
                           float tan_fovy, bool prefiltered, float* out_color, int* radii, bool render_depth,
                           void* stream, int* num_rendered);

int omr_rasterizer_backward(int P, int D, int M, int R, const float* background, int width, int height,
                            const float* means3D, const float* shs, const float* colors_precomp, const float* scales,
                            float scale_modifier, const float* rotations, const float* cov3D_precomp,
                            const float* viewmatrix, const float* projmatrix, const float* campos, float tan_fovx,
                            float tan_fovy, const int* radii, char* geom_buffer, char* binning_buffer,
                            char* image_buffer, const float* dL_dpix, float* dL_dmean2D, float* dL_dconic,
                            float* dL_dopacity, float* dL_dcolor, float* dL_dmean3D, float* dL_dcov3D, float* dL_dsh,
                            float* dL_dscale, float* dL_drot, void* stream);

/* --- equirectangular / lonlat (camera_type = 3) -------------------------------------------------- */
int omr_lonlat_mark_visible(int P, bool* present, void* stream);

int omr_lonlat_forward(omr_alloc_fn geometry_alloc, void* geometry_ctx, omr_alloc_fn binning_alloc, void* binning_ctx,
                       omr_alloc_fn image_alloc, void* image_ctx, int P, int D, int M, const float* background,
                       int width, int height, const float* means3D, const float* shs, const float* colors_precomp,
                       const float* opacities, const float* scales, float scale_modifier, const float* rotations,
                       const float* cov3D_precomp, const float* viewmatrix, const float* cam_pos, bool prefiltered,
                       float* out_color, int* radii, void* stream, int* num_rendered);

int omr_lonlat_backward(int P, int D, int M, int R, const float* background, int width, int height,
                        const float* means3D, const float* shs, const float* colors_precomp, const float* scales,
                        float scale_modifier, const float* rotations, const float* cov3D_precomp,
                        const float* viewmatrix, const float* campos, const int* radii, char* geom_buffer,
                        char* binning_buffer, char* image_buffer, const float* dL_dpix, float* dL_dmean2D,
                        float* dL_dconic, float* dL_dopacity, float* dL_dcolor, float* dL_dmean3D, float* dL_dcov3D,
                        float* dL_dsh, float* dL_dscale, float* dL_drot, float* dpx_dt, float* dpy_dt, void* stream);

/* Status of a forward's device-side binning (emit, tile sort), which may still be running when omr_*_forward
 * returns. A decoupled look-back of the tile sort that gave up makes that view render background only; the next
 * omr_*_backward on the same buffers returns OMR_ERR_HIP for it, and a forward-only caller (evaluation, inference)
 * checks it here: synchronises `stream`, returns OMR_OK or OMR_ERR_HIP (message in omr_last_error). Extension. */
int omr_forward_status(char* geom_buffer, int P, void* stream);

/* --- view-parallel data parallelism (extension, not in the reference; omnigs-fork_amd/parallel.py) -- */
/* The next omr_*_backward call on this thread records `event` (a hipEvent_t) on its stream as soon as dL_dcolor is
 * final — after the per-Gaussian row sums, before the per-Gaussian backward (gaussian_bwd) — and forgets it. A
 * view-parallel host starts the all-gather of the colour gradients on another stream waiting on that event, so the
 * collective overlaps the rest of the backward. NULL clears a pending event. */
void omr_backward_colors_event(void* event);
/* The next omr_*_backward call on this thread runs the per-Gaussian backward (gaussian_bwd) as n launches over the
 * Gaussian ranges [omr_backward_chunk_begin(P, n, k), omr_backward_chunk_begin(P, n, k + 1)) and records events[k]
 * (hipEvent_t) on its stream after range k, then forgets them: a view-parallel host all-reduces each range's xyz /
 * opacity / scale / rotation gradients as soon as they are final. n = 0 or events = NULL clears. */
void omr_backward_chunk_events(int n, void* const* events);
/* First Gaussian of range k of n (a multiple of 256; 0 for k <= 0, P for k >= n). */
int omr_backward_chunk_begin(int P, int n, int k);
/* dL_dsh [P,M,3] = sum over nviews views of the SH gradient the backward computes for each, rebuilt from each
 * view's dL_dcolors ([nviews][P][3], RasterizeGaussiansBackwardCUDA's second output) and camera position
 * (campos [nviews][3]) with the backward's own SH arithmetic. Lets view-parallel ranks exchange 12 B per
 * Gaussian and view instead of all-reducing the 192-B SH gradient (M = 16). */
int omr_sh_grad_from_colors(int P, int D, int M, int nviews, const float* means3D, const float* shs,
                            const float* campos, const float* dL_dcolors, float* dL_dsh, void* stream);
/* The same with both inputs in one array packed[nviews][P + 1][3]: rows 0..P-1 of view v are its dL_dcolors, row P
 * its camera position, so ranks exchange one all-gather of P + 1 rows instead of two collectives. */
int omr_sh_grad_from_colors_packed(int P, int D, int M, int nviews, const float* means3D, const float* shs,
                                   const float* packed, float* dL_dsh, void* stream);

/* --- training loss (extension; reference include/loss_utils.h:31-129, gaussian_trainer.cpp:88-90) --- */
/* loss = (1 - lambda) * mean|img - gt| + lambda * (1 - ssim(img, gt)) over [C,H,W] float images (11x11 Gaussian
 * window, sigma 1.5, zero padding, C1 = 0.01^2, C2 = 0.03^2), forward and backward in one pass:
 * dL_dimg [C,H,W] = dloss/dimg, out3 (device, 3 floats) = {loss, l1, ssim}. scratch: device floats, at least
 * omr_l1_ssim_scratch_floats(C, H, W). */
size_t omr_l1_ssim_scratch_floats(int C, int H, int W);
int omr_l1_ssim_loss(const float* img, const float* gt, int C, int H, int W, float lambda_dssim, float* dL_dimg,
                     float* out3, float* scratch, void* stream);

/* --- training step after the backward (extension) ------------------------------- */
/* Adam over the six GaussianModel parameter groups in ONE launch, replacing torch::optim::Adam::step (LibTorch
 * 2.0.1 adam.cpp; groups, learning rates and eps 1e-15 from gaussian_model.cpp:485-518, stepped at
 * gaussian_mapper.cpp:486). Group order k: 0 xyz [P,3], 1 features_dc [P,1,3], 2 features_rest [P,Mr,3],
 * 3 opacity [P,1] (logit), 4 scaling [P,3] (log), 5 rotation [P,4] (raw). params / exp_avg / exp_avg_sq are
 * updated in place and must be 16-byte aligned. step[k] is the step count AFTER this step's increment (>= 1).
 * A group with params[k] or grads[k] NULL is skipped (adam.cpp skips parameters whose gradient is undefined).
 * grad_kind:
 *   OMR_ADAM_RAW_GRADS     grads[k] has params[k]'s layout (the gradients autograd would leave in .grad);
 *   OMR_ADAM_RASTER_GRADS  grads are the rasterizer backward's outputs w.r.t. the ACTIVATED tensors the renderer
 *                          feeds it (gaussian_renderer.cpp:167-290): grads[0] dL_dmeans3D, grads[1] = grads[2] =
 *                          dL_dsh [P,Mr+1,3], grads[3] dL_dopacity (of sigmoid(opacity)), grads[4] dL_dscales (of
 *                          exp(scaling)), grads[5] dL_drotations (of normalize(rotation)); the activation
 *                          backward (cat / sigmoid / exp / normalize) is applied in registers. */
#define OMR_ADAM_RAW_GRADS 0
#define OMR_ADAM_RASTER_GRADS 1
int omr_adam_step(int P, int Mr, float* const params[6], float* const exp_avg[6], float* const exp_avg_sq[6],
                  const float* const grads[6], int grad_kind, const float lr[6], const int64_t step[6], float beta1,
                  float beta2, float eps, void* stream);
/* The renderer's activations of the six raw groups in one launch (gaussian_model.cpp:54-77 as
 * gaussian_renderer.cpp:175-200 applies them): shs = cat(features_dc, features_rest) [P,Mr+1,3] (skipped when shs is
 * NULL), opacity = sigmoid(params[3]) [P], scales = exp(params[4]) [P,3], rotations = normalize(params[5]) [P,4]
 * (x / max(||x||_2, 1e-12)); xyz (params[0]) is used as is. params[5], rotations and shs 16-byte aligned. */
int omr_activate(int P, int Mr, const float* const params[6], float* shs, float* opacity, float* scales,
                 float* rotations, void* stream);
/* omr_adam_step with OMR_ADAM_RASTER_GRADS that also writes omr_activate's four outputs from the UPDATED parameters
 * (bitwise what omr_activate would give after the step), so a training loop needs no separate activation launch
 * before its next forward. Any output may be NULL (not written); the others must be 16-byte aligned and their
 * groups must step (an output of a skipped group would be stale: OMR_ERR_INVALID_ARGUMENT). With radii != NULL the
 * same launch also does omr_densification_stats(P, radii, viewspace_grad, viewspace_stride, xyz_gradient_accum,
 * denom, max_radii2D) (the same arithmetic; the statistics and Adam touch disjoint arrays). */
int omr_adam_step_activate(int P, int Mr, float* const params[6], float* const exp_avg[6],
                           float* const exp_avg_sq[6], const float* const grads[6], const float lr[6],
                           const int64_t step[6], float beta1, float beta2, float eps, float* shs, float* opacity,
                           float* scales, float* rotations, const int* radii, const float* viewspace_grad,
                           int viewspace_stride, float* xyz_gradient_accum, float* denom, float* max_radii2D,
                           void* stream);
/* addDensificationStats (gaussian_model.cpp:839-853) + the max_radii2D update (gaussian_mapper.cpp:427-432) for
 * visibility_filter = radii > 0: accum[i] += |viewspace_grad[i][0:2]|, denom[i] += 1, max_radii2D[i] =
 * max(max_radii2D[i], radii[i]). viewspace_grad is dL_dmeans2D with row stride viewspace_stride (3). */
int omr_densification_stats(int P, const int* radii, const float* viewspace_grad, int viewspace_stride,
                            float* xyz_gradient_accum, float* denom, float* max_radii2D, void* stream);
/* densifyAndPrune (gaussian_model.cpp:812-837 with densifyAndClone / densifyAndSplit / prunePoints :619-810) in
 * two calls. omr_densify_plan classifies every Gaussian into `plan` (device, omr_densify_plan_bytes(P)) and
 * synchronises the stream (the reference reads counts to the host too, :768) to return counts = {P_new, clones
 * kept, split-selected S, splits kept}. The caller allocates the P_new-row outputs and 2*S*3 standard normal
 * samples (batch-major: copy 1 of every selected split, then copy 2; the reference draws them with at::normal,
 * :751) and calls omr_densify_apply, which writes the final arrays in the reference's order. exp_avg / exp_avg_sq
 * arrays may be NULL (no optimizer state) or hold NULL entries; exist_in / exist_out (int32 exist_since_iter)
 * may be NULL. xyz_gradient_accum, denom and max_radii2D of the result are zeros (the caller's memset). */
size_t omr_densify_plan_bytes(int P);
int omr_densify_plan(int P, const float* xyz_gradient_accum, const float* denom, const float* scaling,
                     const float* opacity, float max_grad, float min_opacity, float extent, float percent_dense,
                     int max_screen_size, int prune_by_extent, void* plan, int64_t counts[4], void* stream);
int omr_densify_apply(int P, int Mr, const void* plan, const float* const params_in[6],
                      const float* const exp_avg_in[6], const float* const exp_avg_sq_in[6], const int32_t* exist_in,
                      const float* normals, float* const params_out[6], float* const exp_avg_out[6],
                      float* const exp_avg_sq_out[6], int32_t* exist_out, void* stream);
/* resetOpacity (gaussian_model.cpp:564-572): opacity = inverse_sigmoid(min(sigmoid(opacity), ceiling)) and the
 * opacity group's Adam moments zeroed (either may be NULL). The reference passes
 * ones_like(sigmoid(opacity) * 0.01) as the bound, i.e. ceiling = 1 (value unchanged up to rounding; only the
 * moments reset); 0.01 gives the 3DGS behaviour. */
int omr_reset_opacity(int P, float* opacity, float* exp_avg, float* exp_avg_sq, float ceiling, void* stream);

/* --- formats (extension) ------------------------------------------------------------ */
/* distCUDA2 (third_party/simple-knn/spatial.cu:15-25, simple_knn.cu:185-220): mean_dists[i] = mean of the squared
 * distances from points[i] ([P,3]) to its 3 nearest other points (exact; FLT_MAX stands in for missing neighbours
 * when P < 4, as in the reference). scratch: device bytes, at least omr_dist2_scratch_bytes(P). */
size_t omr_dist2_scratch_bytes(int P);
int omr_dist2(int P, const float* points, float* mean_dists, void* scratch, void* stream);
/* GaussianModel::loadPly / savePly (gaussian_model.cpp:860-1070) — the 62-property binary PLY. Reading takes two
 * calls so the caller can allocate: omr_ply_open parses the header (requires x y z f_dc_0..2 f_rest_0..(3Mr-1)
 * opacity scale_0..2 rot_0..3 in the vertex element, Mr = (max_sh_degree + 1)^2 - 1; any order, extra properties,
 * ascii / big-endian / non-float types accepted) and returns the vertex count; omr_ply_read fills the six device
 * parameter arrays (xyz [P,3], features_dc [P,1,3], features_rest [P,Mr,3], opacity [P,1], scaling [P,3],
 * rotation [P,4]) and synchronises the stream; omr_ply_close frees the handle. omr_ply_save writes the file
 * savePly writes (header as tinyply.h:664-703, zero normals, channel-major SH). Both use a temporary device buffer
 * of P records (hipMalloc) and move it in one copy. */
typedef struct omr_ply omr_ply;
int omr_ply_open(const char* path, int max_sh_degree, omr_ply** out, int64_t* num_points);
int omr_ply_read(omr_ply* ply, float* const params[6], void* stream);
void omr_ply_close(omr_ply* ply);
int omr_ply_save(const char* path, int P, int Mr, const float* const params[6], void* stream);

/* --- scratch sizes (bytes the allocation callbacks are asked for) -------------------------------- */
/* geometry: the size for a view that takes the row binning (at most 1024 tiles a side) with colours from 16-coefficient
   SH rows (the forward then stores dRGB/ddir, 36 B per Gaussian); wider views are asked for about 56 B per Gaussian
   less (no row-binning arrays) and other colour sources 36 B less, so this is an upper bound for any forward */
size_t omr_geometry_bytes(int P);
size_t omr_image_bytes(int width, int height);
size_t omr_binning_bytes(int num_rendered, int width, int height);

/* --- stage timing (HIP events recorded on the launch stream; for bench.py / tools) --------------- */
/* stages: 0 preprocess, 1 depth_sort, 2 scan, 3 emit, 4 tile_sort, 5 tile_ranges, 6 render_forward,
 *         7 render_backward, 8 gaussian_backward, 9 row_sums                                       */
#define OMR_NUM_STAGES 10
void omr_profile_enable(int on);
/* restrict recording to the stages whose bit (1 << stage) is set (default: all); each recorded stage costs a
 * few microseconds of GPU idle at its boundaries, so a timed run records only the kernel it reports */
void omr_profile_set_mask(uint32_t mask);
void omr_profile_reset(void);
/* waits for the recorded events; fills total milliseconds and launch counts per stage since the last reset;
 * returns the number of stages written (<= n) */
int omr_profile_read(double* total_ms, uint64_t* counts, int n);
const char* omr_profile_stage_name(int stage);

/* --- host-side runtime counters (process-wide, since load or the last reset; for bench.py / tools) ----- */
/* 0 forwards, 1 backwards, 2 first_call_syncs (forwards that waited for num_rendered before sizing the binning
 * buffer), 3 back_half_reruns (capacity hint too small), 4 count_wait_ns (host time waiting for num_rendered),
 * 5 backward_wait_ns (host time waiting for the forward's error word), 6 alloc_calls, 7 alloc_bytes (allocation
 * callbacks), 8 lookback_errors (decoupled look-backs that gave up; the call returned OMR_ERR_HIP) */
#define OMR_NUM_RUNTIME_STATS 9
int omr_runtime_stats(uint64_t* out, int n);
const char* omr_runtime_stat_name(int i);
void omr_runtime_stats_reset(void);

/* --- introspection for tests / tools (read from the private scratch layout) ---------------------- */
/* copies the sorted per-instance Gaussian indices (R entries) and tile ranges ([T] uint2) to device dst */
int omr_debug_point_list(char* binning_buffer, int R, int width, int height, uint32_t* dst, void* stream);
/* The point list's raw entries [R]: Gaussian index in the low 28 bits, the instance's band mask (the 16x4 bands of its
 * tile the alpha >= 1/255 ellipse can reach) in the top 4. Diagnostic (tests/test_gpu_parity.py checks the masks). */
int omr_debug_point_list_raw(char* binning_buffer, int R, int width, int height, uint32_t* dst, void* stream);
int omr_debug_ranges(char* image_buffer, int width, int height, uint32_t* dst, void* stream);
/* per-pixel final transmittance [N] f32 and contributor count [N] u32 */
int omr_debug_image_state(char* image_buffer, int width, int height, float* final_T, uint32_t* n_contrib, void* stream);
/* the forward's per-tile count of (instance, 16x4 band) evaluations [T] (the backward's schedule key) */
int omr_debug_tile_cost(char* image_buffer, int width, int height, uint32_t* dst, void* stream);
/* the forward's count words: [0] num_rendered, [1] prefiltered flag, [2] huge-Gaussian count, [3] look-back error,
 * [4] row slots M of the row binning (bin.hip; 0 on sort.hip's path), [5] the stored-dRGB/ddir key (sh_jac: a key of
 * the forward's SH array, means and campos, 0 if not stored), [6] the same key (omr_debug_set_sh_jac restores [5]
 * from it); dst: 8 device words */
int omr_debug_counters(char* geom_buffer, int P, uint32_t* dst, void* stream);
/* clears (0) or restores (1) the key by which the backward uses the forward's stored dRGB/ddir (GeomState::sh_jac)
 * instead of reading the SH rows: lets a test run both backward paths on one forward */
int omr_debug_set_sh_jac(char* geom_buffer, int P, int enabled, void* stream);
/* the forward's depth sort: 0 = by size and camera type (views of at most 12288 Gaussians: the sort by counting;
 * else pinhole: the sort that sets culled Gaussians aside first; lonlat: the plain 4 x 8-bit radix sort), 1 = always
 * the plain sort, 2 = always the culled-aside sort, 3 = the sort by counting up to 2^18 Gaussians (the same
 * permutation every way); process-wide, for tests and A/B runs (the environment's OMR_DEPTH_SORT=bytes / visible /
 * count sets the start value). Returns the previous mode, or -1 for a mode outside 0..3 (omr_last_error says why) */
int omr_debug_depth_sort_mode(int mode);
/* the forward's binning: 0 = by view (the emit + radix tile sort up to 1024 tiles and past 1024 tiles a side, the row
 * binning between), 1 = the row binning wherever the grid allows it, 2 = always the emit + tile sort (the same point
 * list and ranges); process-wide, for tests and A/B runs (OMR_BINNING=rows / sort sets the start value). A forward and
 * its backward must run under the same mode. Returns the previous mode, or -1 outside 0..2 */
int omr_debug_binning_mode(int mode);
/* omr_l1_ssim_loss's kernel: 0 = by image size (the streaming kernel once its strips fill the chip, else the tiled
 * one), 1 = always tiled, 2 = always streaming (both give bitwise the same dL_dimg); process-wide, for tests and A/B
 * runs. Returns the previous mode, or -1 for a mode outside 0..2 */
int omr_debug_ssim_mode(int mode);
/* the render backward's mapping: 0 = by view (two waves per (tile, segment) unit, two 16x4 bands each, when every
 * unit is resident at once — small views; else one wave of four bands), 2 / 4 = always that one (rows equal up to the
 * order of the float additions; A/B runs and tests). Process-wide; the environment's OMR_BWD_BANDS=2|4 sets the start
 * value. Returns the previous mode, or -1 for another value */
int omr_debug_bwd_bands(int mode);
/* omr_adam_step / omr_adam_step_activate: 1 = f_dc and f_rest stepped as one walk over dL_dsh's rows (the default),
 * 0 = two gathering groups, the activated SH array then written by a separate copy launch (same results; A/B runs).
 * Process-wide; the environment's OMR_ADAM_SH_ROWS=0 sets the start value. Returns the previous value, or -1 for a
 * value outside 0..1 */
int omr_debug_adam_sh_rows(int enabled);
/* per-Gaussian pixel centre [P,2], conic+opacity [P,4], rgb [P,3], depth [P], tiles_touched [P] */
/* one wave64 through the render backward's gradient reduction: in [64][9] -> out [9] (column sums) */
int omr_debug_wave_sum9(const float* in, float* out, void* stream); /* wave_sum9_rows */
int omr_debug_wave_sum9_lds(const float* in, float* out, void* stream); /* wave_sum9_lds (render backward, unpaired) */
int omr_debug_wave_sum9x2(const float* in, float* out, void* stream); /* wave_sum9x2_stored: [2][64][9] -> [2][9] (render backward) */
int omr_debug_wave_scans(const uint32_t* in, uint32_t* out, void* stream); /* DPP wave scans: [2][64] -> [3][64] (incl. sum, incl. max, wave max) */
int omr_debug_geometry(char* geom_buffer, int P, float* means2D, float* conic_opacity, float* rgb, float* depths,
                       uint32_t* tiles_touched, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* OMNIGS_RASTER_H */

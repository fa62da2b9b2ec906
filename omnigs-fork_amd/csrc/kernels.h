// kernels.h — launch-side declarations shared by the orchestration (capi.hip) and the kernel files.
#pragma once

#include <string>

#include <hip/hip_ext.h>

#include "raster_common.h"

namespace omr {

// a run of u32 words the preprocess kernel zeroes before anything reads them (replaces memset launches)
struct ZeroSpan {
    uint32_t* p = nullptr;
    size_t n = 0;
};
constexpr int PRE_ZERO_SPANS = 5;

struct PreprocessArgs {
    ZeroSpan zero[PRE_ZERO_SPANS];
    int P, D, M;
    int W, H;
    uint32_t gx, gy;
    const float* means3D;
    const float* scales;
    float scale_modifier;
    const float* rotations;
    const float* opacities;
    const float* shs;
    const float* cov3D_precomp;
    const float* colors_precomp;
    const float* viewmatrix;
    const float* projmatrix;
    const float* campos;
    float tan_fovx, tan_fovy, focal_x, focal_y;
    int prefiltered;
    int* radii;
    GeomState g;
    int* error_flag;  // set to 1 if prefiltered and a point is culled (auxiliary.h:183-187 traps instead)
};

void launch_preprocess(int camera_type, const PreprocessArgs& a, hipStream_t s);
void launch_mark_visible(int camera_type, int P, const float* means3D, const float* viewmatrix, const float* projmatrix,
                         bool* present, hipStream_t s);

// sort.hip
// scan block-sum scratch for n items (words)
size_t scan_partials_size(size_t n);
size_t radix_hist_size(size_t n);
// words of the `hist` and `scan_partials` scratch radix_sort_pairs needs for n items over `passes` passes
size_t radix_scratch_words(size_t n, int passes);
size_t radix_partials_words(size_t n);
// the forward's scans of tiles_touched (sort.hip): row_first = exclusive scan in index order (gradient row
// numbering), *count_out = its total (num_rendered); huge_list / *huge_count (zeroed by the caller) = the Gaussians
// with more than ROW_SUM_HUGE tiles; status: scan2_status_words(n) words, zeroed before the launch (one look-back
// kernel); err (device word, zeroed by the caller; NULL = a private word) is OR-ed with 1 if a look-back gave up
// (sort.hip: LB_SPIN_MAX). rects == NULL (sort path): offsets = inclusive scan in depth order (gather by order).
// rects != NULL (row path): drect = rects in depth order, row_offsets = inclusive scan of their rows in depth order,
// count_out[4] = its total M, desc_r = each BIN_CHUNK-slot chunk's first and last owner rank. nvis (device word, may
// be NULL): depth ranks from *nvis on are culled (depth_sort_nvis); their depth-order words are neither gathered nor,
// on the row path, written.
size_t scan2_status_words(size_t n);
void launch_forward_scans(const uint32_t* tiles_touched, const uint2* rects, const uint32_t* order, uint32_t* offsets,
                          uint32_t* row_first, uint32_t* row_offsets, uint2* drect, uint2* desc_r, uint32_t* huge_list,
                          uint32_t* huge_count, uint32_t* status, uint32_t* count_out, uint32_t* err, size_t n,
                          hipStream_t s, const uint32_t* nvis = nullptr);
// stable LSD radix sort of (key, value) over bits [0, 8*passes); returns which buffer holds the result (0: a, 1: b).
// n = capacity; count (device, may be NULL) = live element count <= n. canon != NULL: the last pass writes the
// values to the canonical point list of the binning buffer at canon (raster_common.h) instead of val_a / val_b.
// scratch_zeroed: the caller has zeroed radix_zero_span(hist, n, passes) (else the sort clears it itself).
// err (device word; NULL = a private word in the scratch) is OR-ed with 1 if a decoupled look-back gave up.
// K = uint32_t, or uint16_t for keys below 2^16 (the tile sort of views with at most 65536 tiles: 2 B less per key
// and pass read and written).
template <typename K>
int radix_sort_pairs(K* key_a, K* key_b, uint32_t* val_a, uint32_t* val_b, uint32_t* hist, uint32_t* scan_partials,
                     size_t n, const uint32_t* count, char* canon, int first_pass, int passes, hipStream_t s,
                     bool scratch_zeroed = false, uint32_t* err = nullptr);
// the words of `hist` a sort of n items over `passes` passes needs zeroed before it starts (possibly none)
ZeroSpan radix_zero_span(uint32_t* hist, size_t n, int passes);
// The depth sort (sort.hip, DepthPass): stable sort of the n Gaussians' depth keys (float bits of positive depths;
// culled = 0xFFFFFFFF) in four 8-bit-wide passes, of which the first also moves the culled Gaussians behind the
// visible ones and the other three sort the visible keys alone; the permutation of the visible Gaussians, ties in
// index order, then the culled ones in index order, lands in `order` (key_a / val_a: the keys and 0..n-1 on entry;
// key_b / val_b: scratch). hist: depth_sort_scratch_words(n) words, of which depth_sort_zero_span(hist, n) zeroed
// before the call; scan_partials: depth_sort_partials_words(n) words.
size_t depth_sort_scratch_words(size_t n);
size_t depth_sort_partials_words(size_t n);
ZeroSpan depth_sort_zero_span(uint32_t* hist, size_t n);
void depth_sort(uint32_t* key_a, uint32_t* key_b, uint32_t* val_a, uint32_t* val_b, uint32_t* order, uint32_t* hist,
                uint32_t* scan_partials, size_t n, hipStream_t s, uint32_t* err);
// the device word holding the visible count once depth_sort has run (pass 0 sets it: the culled bucket's start)
const uint32_t* depth_sort_nvis(const uint32_t* hist, size_t n);
// The depth sort of small views (sort.hip): the same permutation as depth_sort / the plain radix sort (visible keys in
// order, ties by index, then the culled ones by index) by counting, O(n^2) compares in one launch; keys: the n keys.
// the default up to this many keys (capi.hip: depth_sort_kind): 18.8 us at 10 k keys on 157 CUs against the radix
// sort's 29 us; past ~15 k keys every CU is busy and the time grows with n^2 (profiles/r06m_ab_A.txt)
constexpr size_t DEPTH_COUNT_SORT_MAX = 12288;
constexpr size_t DEPTH_COUNT_SORT_FORCED_MAX = 1u << 18;  // forced (tests, A/Bs) up to this many
void depth_count_sort(const uint32_t* keys, uint32_t* order, size_t n, hipStream_t s);
// one-launch exclusive scan of n u32 (in may equal out) of in[i] & mask; n_dev (device word, may be NULL) = live
// length <= n; status: scan_status_words(n) words zeroed before the launch; err: the look-back error word (NULL: a
// private one)
size_t scan_status_words(size_t n);
void launch_exclusive_scan(const uint32_t* in, uint32_t* out, size_t n, const uint32_t* n_dev, uint32_t* status,
                           uint32_t* err, hipStream_t s, uint32_t mask = 0xFFFFFFFFu);

// duplicateWithKeys; L_cap = capacity, *count (device) = num_rendered; block_owner: emit_index_size(L_cap) words
#ifndef OMR_EMIT_THREADS
#define OMR_EMIT_THREADS 256
#endif
constexpr int EMIT_THREADS = OMR_EMIT_THREADS;
#ifndef OMR_EMIT_PER
#define OMR_EMIT_PER 4
#endif
constexpr int EMIT_PER = OMR_EMIT_PER;                // consecutive instance slots per emit thread (1, 2 or 4)
constexpr int EMIT_SLOTS = EMIT_THREADS * EMIT_PER;   // slots per emit block (block_owner granularity)
size_t emit_index_size(size_t L_cap);
// Words the host reads back (capi.hip: HostRead): src[0..n) into pinned fine-grained memory at dst, then seq into
// seq_dst once they are acknowledged, with system-scope vector stores. Written by the first wave of a kernel that runs
// anyway (emit_index or the row binning's first kernel, backward_schedule), or by host_words_kernel; dst == NULL: nothing to write.
struct HostWords {
    uint32_t* dst = nullptr;
    const uint32_t* src = nullptr;
    int n = 0;
    uint32_t* seq_dst = nullptr;
    uint32_t seq = 0;
};
#if defined(__HIPCC__)
__device__ __forceinline__ void write_host_words(const HostWords& h, uint32_t lane)  // all 64 lanes of one wave
{
    if (lane < (uint32_t)h.n) __hip_atomic_store(h.dst + lane, h.src[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __builtin_amdgcn_s_waitcnt(0);  // the data stores are acknowledged before the sequence number is written
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) __hip_atomic_store(h.seq_dst, h.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
#endif
void launch_host_words(const HostWords& h, hipStream_t s);

// bin.hip: tile binning by rows, then columns (the point list, its band masks and the tile ranges) for views of at most
// BIN_MAX_GRID tiles a side; sort.hip's emit + tile sort + ranges otherwise
constexpr uint32_t BIN_MAX_GRID = 1024;
constexpr size_t BIN_SORT_MAX_TILES = 1024;  // views of at most this many tiles take the emit + tile sort (capi.hip)
struct BinArgs {
    HostWords hw;               // the forward's count words, written by the first kernel
    int P;
    uint32_t gx, gy;
    size_t cap;                 // binning capacity (instances)
    const uint32_t* counters;   // GeomState::counters: [0] L, [3] error word, [4] M (row slots)
    uint32_t* err;              // look-back error word (counters + 3)
    const uint32_t* order;      // depth order
    const uint32_t* row_offsets;  // inclusive scan of the rect rows in depth order
    const uint2* drect;         // rect words in depth order (launch_forward_scans)
    const float4* splat;        // render records (rect in slot 3)
    const float4* bin_rec;      // [P][2] band-mask constants, x0 | width << 16 (preprocess)
    uint32_t *ent_gid, *ent_w, *ent_ex;  // row entries [cap]: Gaussian, rect width | x0 << 16, first instance slot
    uint32_t* hist_r;           // [2][gy][live row chunks] entry counts, width sums; scanned in place
    size_t chunks_r;            // row chunks of the capacity (grid size; the live count is div_up(M, chunk))
    const uint2* desc_r;        // owners of each row chunk: first, last (depth ranks; launch_forward_scans)
    uint32_t* hist_b;           // [tile][chunk] counts (row-major chunk blocks), scanned in place; chunks_b * gx words
    size_t chunks_b;
    uint32_t cb_shift;          // columns-pass chunk = 1 << cb_shift slots (bin_cols_shift; set by launch_row_binning)
    uint4* desc_b;              // [chunks_b][2] column chunks: {y, chunk of the row, row chunks, row's first chunk},
                                // {first slot, end slot, first owner entry, owners}
    uint32_t* words;            // [0] live M, [1] column chunks, [2] live hist_r length, [3] live hist_b length
    uint32_t* zero;             // look-back words of the two scans (bin_zero_words)
    size_t nzero;
    uint2* ranges;              // [T] tile ranges
    char* binning;              // the binning buffer (canonical point list, row_valid at L-only offsets)
};
size_t bin_chunks_r(size_t cap);
uint32_t bin_cols_shift(size_t cap);
size_t bin_chunks_b(size_t cap, uint32_t gy);
inline size_t bin_zero_words(size_t cap, uint32_t gx, uint32_t gy)
{
    return scan_status_words(2 * (size_t)gy * bin_chunks_r(cap)) + scan_status_words(bin_chunks_b(cap, gy) * gx);
}
void launch_row_binning(const BinArgs& a, hipStream_t s);


// tile_keys: uint16_t[L_cap] when keys16 (at most 65536 tiles), else uint32_t[L_cap]
void launch_emit_instances(const HostWords& hw, int P, size_t L_cap, const uint32_t* count, const GeomState& g,
                           uint32_t gx, uint32_t* block_owner, void* tile_keys, bool keys16, uint32_t* gauss_vals,
                           char* binning, hipStream_t s);
void launch_tile_ranges(size_t L_cap, const uint32_t* count, const void* sorted_tiles, bool keys16, uint2* ranges,
                        hipStream_t s);
// render schedule: within each of 8 contiguous shares of the tiles (one per XCD), tiles by descending cost
// (cost[t] if cost != NULL, else the instance count ranges[t].y - ranges[t].x)
void launch_tile_order(const uint2* ranges, const uint32_t* cost, uint32_t T, uint32_t* order, hipStream_t s);

// render_fwd.hip
struct RenderFwdArgs {
    int W, H;
    uint32_t gx, gy;
    const uint2* ranges;
    const uint32_t* tile_order;  // [T] schedule (launch_tile_order), or NULL: tiles in index order
    char* binning;               // binning buffer: point list at binning + canonical_list_offset(L); checkpoints, segment work
    const uint32_t* count;       // device count words (GeomState::counters; raster_common.h binning_count)
    size_t capacity;             // instances the binning buffer was sized for (count > capacity: render nothing)
    const float4* splat;  // [P][SPLAT_F4] render records
    const float* bg;
    uint32_t* tile_cost;  // [T] zeroed; receives the (instance, band) pairs each tile evaluated
    uint32_t* max_contrib;  // [T][FWD_GROUPS] each wave's largest last contributor (backward schedule)
    float* final_T;
    float* final_C;         // [3][N] colour before the background term (backward segment starts)
    uint32_t* n_contrib;
    float* out_color;
};
void launch_render_forward(const RenderFwdArgs& a, bool depth_mode, hipStream_t s);
// whether the forward of a T-tile view wants the longest-first tile order: not at two or fewer waves per SIMD (config
// A), where every wave starts at once and dispatch order does not change the makespan
bool render_forward_needs_order(uint32_t T);

// render_bwd.hip
struct RenderBwdArgs {
    int W, H;
    uint32_t gx, gy;
    const uint2* ranges;
    const uint2* units;          // {tile, chunk} depth segments, longest first per XCD share (launch_backward_schedule)
    const uint32_t* unit_count;  // device word: number of units
    const float4* ckpt;          // the forward's checkpoints (raster_common.h: ckpt_offset)
    const float* final_C;        // [3][N]
    const uint32_t* point_list;
    const float4* splat;  // [P][SPLAT_F4] render records
    const uint32_t* row_first;  // [P] first gradient row of each Gaussian (index-order scan, launch_forward_scans)
    const float* bg;
    const float* final_T;
    const uint32_t* n_contrib;
    const float* dL_dpix;
    float* inst_grad;
    uint8_t* row_valid;  // [L] zeroed; 1 where inst_grad holds a row
};
// grid: an upper bound on the unit count (seg_count(R, T)); waves past the device count exit at once
// ev_start / ev_stop (optional): timing events carried by the dispatch packet itself (hipExtLaunchKernelGGL), so
// profiling the stage inserts no marker packets around it (each costs a system-scope release: GPU idle, capi.hip)
void launch_render_backward(const RenderBwdArgs& a, size_t max_units, hipStream_t s, hipEvent_t ev_start = nullptr,
                            hipEvent_t ev_stop = nullptr);
// the render backward's mapping: 0 by view (two waves per unit when every unit is resident at once, else one), 2 or 4
// forces two / one wave(s) per unit; process-wide (omr_debug_bwd_bands, OMR_BWD_BANDS), returns the previous mode
int bwd_bands_mode(int mode);
// the backward's work list: every (tile, depth segment) below the tile's last contributor (max over the forward's
// max_contrib words), costed by its positions, sorted longest first within each of the 8 XCD shares of the unit list
// (the shares xcd_remap gives each XCD), or, sorted = false, in tile order; writes units, *unit_count
void launch_backward_schedule(const HostWords& hw, const uint2* ranges, const uint32_t* max_contrib, uint32_t T, uint2* units_tmp,
                              uint32_t* cost_tmp, uint2* units, uint32_t* unit_count, bool sorted, hipStream_t s);
// whether the backward of a view with at most max_units units wants them longest first: not when the kernel that
// launch_render_backward picks holds every unit's workgroup at once (configs A, B)
bool render_backward_needs_order(size_t max_units);
#ifdef OMR_STAMPS
int omr_debug_stamps_bwd(uint64_t* dst, size_t bytes);  // diagnostic builds only (tile_wave.h)
#endif

// gaussian_bwd.hip
struct GaussBwdArgs {
    int P, D, M, W, H;
    int g_begin, g_end;  // the Gaussians of this launch, [g_begin, g_end) (g_begin a multiple of 256)
    const float* means3D;
    const int* radii;
    const float* shs;
    const float* scales;
    const float* rotations;
    float scale_modifier;
    const float* cov3D_precomp;
    const float* viewmatrix;
    const float* projmatrix;
    const float* campos;
    float tan_fovx, tan_fovy, focal_x, focal_y;
    const uint8_t* clamped;
    const float* sh_jac;       // [P][9] the forward's dRGB/ddir (GeomState::sh_jac), used when *jac_flag says it is there
    const uint32_t* jac_flag;  // GeomState::counters + 5 (sh_jac_key of the forward's inputs, 0: none)
    const float* row_sums;  // [P][GRAD_ROW] each Gaussian's instance rows summed (launch_row_sums)
    const float4* conic_op;  // [P] conic + opacity (GeomState) for the raw-moment rows
    float* dL_dmean2D;   // [P,3]
    float* dL_dconic;    // [P,4] optional (may be null)
    float* dL_dopacity;  // [P]
    float* dL_dcolor;    // [P,3]
    float* dL_dmean3D;   // [P,3]
    float* dL_dcov3D;    // [P,6]
    float* dL_dsh;       // [P,M,3]
    float* dL_dscale;    // [P,3]
    float* dL_drot;      // [P,4]
    float* dpx_dt;       // [P,3] optional (lonlat only; may be null)
    float* dpy_dt;       // [P,3] optional
};
void launch_gaussian_backward(int camera_type, const GaussBwdArgs& a, hipStream_t s, hipEvent_t ev_start = nullptr,
                              hipEvent_t ev_stop = nullptr);
// Per-Gaussian sums of the render backward's instance rows: Gaussian i owns rows [row_first[i], row_first[i] +
// tiles_touched[i]) of inst_grad (index-order numbering, launch_forward_scans); only rows marked in row_valid are read.
// Gaussians in huge_list (*huge_count of them) are summed by whole workgroups. Also writes dL_dcolor [P][3] (the
// colour part of the sums; zeros for culled Gaussians), which gaussian_bwd then leaves alone. One launch covers the
// Gaussians [g_begin, g_end); huge = it also sums the huge_list ones (the first launch of a split backward).
void launch_row_sums(int g_begin, int g_end, bool huge, const uint32_t* row_first, const uint32_t* tiles_touched,
                     const uint32_t* huge_list, const uint32_t* huge_count, const float* inst_grad,
                     const uint8_t* row_valid, uint32_t R, float* row_sums, float* dL_dcolor, hipStream_t s);
// view-parallel DP: dL_dsh[P,M,3] = sum over views of dL/dsh rebuilt from dL_dcolors [nviews][P][3] + campos [nviews][3]
// view v's colour gradient at dL_dcolors + v * dc_stride, its camera position at campos + v * cp_stride (floats)
void launch_sh_grad_from_colors(int P, int D, int M, int nviews, const float* means3D, const float* shs,
                                const float* campos, size_t cp_stride, const float* dL_dcolors, size_t dc_stride,
                                float* dL_dsh, hipStream_t s);

// ssim.hip: fused L1 + SSIM loss (loss_utils.h:31-129), forward and backward
struct SsimWindow {
    float w[11];
};
SsimWindow ssim_window();
size_t l1_ssim_scratch_floats(int C, int H, int W);
void launch_l1_ssim(const float* img, const float* gt, int C, int H, int W, float lambda, float* dimg, float* out3,
                    float* scratch, hipStream_t s);
// 0: kernel by image size, 1: tiled, 2: streaming; returns the previous mode (omr_debug_ssim_mode)
int ssim_debug_mode(int mode);

// optim.hip: Adam over the GaussianModel groups, densification stats, densifyAndPrune, resetOpacity
constexpr int ADAM_MAX_GROUPS = 6;
enum AdamKind : int { ADAM_PLAIN = 0, ADAM_SH_DC = 1, ADAM_SH_REST = 2, ADAM_OPACITY = 3, ADAM_SCALING = 4,
                      ADAM_ROTATION = 5, ADAM_SH_ROWS = 6 };
// ADAM_SH_ROWS: f_rest (p / m / v, 16-B chunks) and f_dc (p2 / m2 / v2) as ONE group, each block stepping a range of
// f_rest plus the f_dc of the Gaussians whose rows start there, so the block's dL_dsh positions are one contiguous
// span, read once (and the activated SH copy, act, written as that span); f_rest's constants are neg_step_size /
// bc2_sqrt, f_dc's the *2 ones. n = f_rest floats (3 Mr P, Mr > 0).
struct AdamGroup {
    float* p;               // raw parameter (16-B aligned)
    float* m;               // exp_avg
    float* v;               // exp_avg_sq
    const float* g;         // gradient: same layout as p (ADAM_PLAIN / OPACITY / SCALING / ROTATION) or dL_dsh
    uint32_t n;             // floats in p
    int kind;               // AdamKind
    float neg_step_size;    // -(lr / (1 - beta1^step))
    float bc2_sqrt;         // sqrt(1 - beta2^step)
    float* act;             // NULL, or the activation of the updated parameter (the next forward's input): sigmoid
                            // (OPACITY), exp (SCALING), normalize (ROTATION), cat(f_dc, f_rest) (SH_ROWS)
    float *p2, *m2, *v2;    // ADAM_SH_ROWS: f_dc and its state
    float neg_step_size2, bc2_sqrt2;
};
// addDensificationStats + the max_radii2D update as extra blocks of the Adam launch (omr_adam_step_activate)
struct DensifyStatsArgs {
    int P = 0;                        // 0: none
    const int* radii = nullptr;
    const float* vgrad = nullptr;     // dL_dmeans2D, row stride vstride
    int vstride = 0;
    float *accum = nullptr, *denom = nullptr, *max_radii = nullptr;
};
struct AdamArgs {
    AdamGroup group[ADAM_MAX_GROUPS];
    uint32_t block0[ADAM_MAX_GROUPS];  // first block of each group (filled by launch_adam)
    uint32_t stats_block0;             // blocks from here on: the densification statistics (filled by launch_adam)
    DensifyStatsArgs stats;
    int ngroups;
    int M;                             // SH coefficients per Gaussian in dL_dsh (f_dc + f_rest)
    float beta1, beta2, omb1, omb2, eps;
};
void launch_adam(AdamArgs a, hipStream_t s);
// the renderer's activations of the raw parameters in one launch (optim.hip: activate_kernel)
struct ActivateArgs {
    int P, Mr;
    const float *f_dc, *f_rest, *opacity, *scaling, *rotation;  // [P,1,3], [P,Mr,3], [P], [P,3], [P,4] (16-B aligned)
    float *shs, *opacity_out, *scales_out, *rotations_out;      // [P,Mr+1,3] (NULL: no SH copy), [P], [P,3], [P,4]
};
void launch_activate(const ActivateArgs& a, hipStream_t s);
void launch_densification_stats(int P, const int* radii, const float* vgrad, int vstride, float* accum, float* denom,
                                float* max_radii, hipStream_t s);
struct DensifyParams {
    float max_grad, min_opacity, extent, percent_dense;
    int max_screen_size, prune_by_extent;
};
struct DensifyIO {
    const float* p_in[6];   // xyz, f_dc, f_rest, opacity, scaling, rotation (raw)
    const float* m_in[6];   // exp_avg per group (null: no state)
    const float* v_in[6];
    float* p_out[6];
    float* m_out[6];        // null: skip
    float* v_out[6];
    const int32_t* exist_in;
    int32_t* exist_out;     // null: skip
    const float* normals;   // [2 S, 3] standard normal samples of the split copies (batch-major)
    int Mr;                 // f_rest coefficients per Gaussian
};
size_t densify_plan_bytes(int P);
void launch_densify_plan(int P, const float* accum, const float* denom, const float* scaling, const float* opacity,
                         float max_grad, float min_opacity, float extent, float percent_dense, int max_screen_size,
                         int prune_by_extent, char* plan, hipStream_t s);
const uint4* densify_plan_totals(int P, const char* plan);
void launch_densify_apply(int P, const char* plan, const DensifyIO& io, hipStream_t s);
void launch_reset_opacity(int P, float* opacity, float* m, float* v, float ceiling, hipStream_t s);

// knn.hip: distCUDA2 (simple_knn.cu:185-220)
size_t knn_scratch_bytes(int P);
void launch_knn(int P, const float* pts, float* dists, char* scratch, hipStream_t s);

// formats.hip: Gaussian PLY files (gaussian_model.cpp:860-1070)
struct PlyFile;
PlyFile* ply_open(const char* path, int max_sh_degree, std::string& err);
int64_t ply_num_points(const PlyFile* f);
int ply_rest_coeffs(const PlyFile* f);
void ply_close(PlyFile* f);
bool ply_read(PlyFile* f, float* const params[6], hipStream_t s, std::string& err);
bool ply_save(const char* path, int P, int Mr, const float* const params[6], hipStream_t s, std::string& err);

}  // namespace omr

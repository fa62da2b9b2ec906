// raster_common.h — constants, device helpers and the private scratch layouts of the gfx950 rasterizer.
//
// The three scratch buffers (geometry / binning / image) play the role of the reference's GeometryState,
// BinningState and ImageState (cuda_rasterizer/rasterizer_impl.h:37-102). Their layout is private to this
// library: forward writes them, backward re-carves them from the same byte buffers (the host only stores the
// buffers and hands them back, gaussian_rasterizer.cpp:85-98). Every array starts on a 256-B boundary.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "omni_math.h"

namespace omr {

constexpr int BLOCK_X = 16;  // cuda_rasterizer/config.h:26 — part of the key semantics, kept
constexpr int BLOCK_Y = 16;  // config.h:27
constexpr int BLOCK_SIZE = BLOCK_X * BLOCK_Y;
constexpr int NUM_CHANNELS = 3;  // config.h:25
constexpr int CAM_PINHOLE = 1;
constexpr int CAM_LONLAT = 3;

// radix sort geometry (sort.hip)
constexpr int SORT_THREADS = 256;
#ifndef OMR_SORT_ITEMS
#define OMR_SORT_ITEMS 16
#endif
constexpr int SORT_ITEMS = OMR_SORT_ITEMS;  // items per thread per block tile of the multi-launch passes
constexpr int SORT_TILE = SORT_THREADS * SORT_ITEMS;
constexpr int RADIX_BITS = 8;
constexpr int RADIX = 1 << RADIX_BITS;
constexpr int DEPTH_SORT_PASSES = 4;  // the depth sort's 32-bit keys (float bits of the depth)
// scan geometry
#ifndef OMR_SCAN_THREADS
#define OMR_SCAN_THREADS 1024
#endif
constexpr int SCAN_THREADS = OMR_SCAN_THREADS;
constexpr int SCAN_TILE = 4096;
constexpr int SCAN_ITEMS = SCAN_TILE / SCAN_THREADS;
constexpr uint32_t SCAN_GRID_MAX = 512;  // blocks of the persistent look-back scan (two 16-wave blocks per CU, 256 CUs)
// row binning (bin.hip): slots per chunk of both passes, and the rect word's row-count field (rows <= BIN_MAX_GRID)
constexpr uint32_t BIN_CHUNK = 2048;
constexpr int RECT_ROWS_BITS = 11;

// per-instance gradient row written by the render backward (render_bwd.hip) and reduced per Gaussian
// (gaussian_bwd.hip). The row holds the instance's raw pixel-weight moments S_u dx, S_u dy, S_u dx^2, S_u dx dy,
// S_u dy^2, S_u, then dcolor.rgb: every factor of backward.cu:805-840 that is the same for all of a Gaussian's
// instances (conic, opacity, W/2, H/2) is applied once to the Gaussian's sums by gaussian_bwd (raw_row_to_grads),
// not once per instance. Row sums of Gaussians without instances are neither written (row_sum_kernel) nor read
// (gaussian_bwd_kernel).
constexpr int GRAD_ROW = 9;
// a Gaussian touching more tiles than this gets a whole workgroup for its row sums (gaussian_bwd.hip); the
// forward's scan lists these Gaussians (sort.hip: scan2_downsweep_kernel)
constexpr uint32_t ROW_SUM_HUGE = 256;

constexpr size_t ALIGN = 256;
__host__ __device__ inline size_t align_up(size_t x) { return (x + ALIGN - 1) & ~(ALIGN - 1); }
inline uint32_t div_up(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }

struct Carver {
    char* base;
    size_t off = 0;
    explicit Carver(char* b) : base(b) {}
    template <typename T> T* take(size_t count)
    {
        off = align_up(off);
        T* p = base ? reinterpret_cast<T*>(base + off) : nullptr;
        off += count * sizeof(T);
        return p;
    }
    size_t size() const { return align_up(off) + ALIGN; }
};

// ---- per-Gaussian render record ----------------------------------------------------------------------------
// The render kernels gather one record per (tile, Gaussian) instance in depth order, i.e. at random Gaussian
// indices. Keeping everything an instance needs in ONE 64-B aligned record makes that one random 64-B line
// instead of five (means2D, conic_opacity, rgb, radii, emit offset in separate arrays: measured 2.8 GB of
// traffic per render backward at config C against 0.45 GB of algorithmic bytes).
//   [0] pos   = {x, y, depth, -}           means2D (forward.cu:699), depth (:697 / :334)
//   [1] conic = {a, b, c, opacity}         conic_opacity (forward.cu:701)
//   [2] rgb   = {r, g, b, w}               colour (SH or colors_precomp); w = rect width in tiles (u32 bits)
//   [3] rect  = {x0, y0, x1, y1}           getRect (u32 bits), read by emit
constexpr int SPLAT_F4 = 4;

// ---- point list entries -------------------------------------------------------------------------------------
// The sorted point list holds, per (tile, Gaussian) instance, the Gaussian index in the low PL_GID_BITS bits and
// the instance's band mask in the top four: bit b set iff the Gaussian's alpha >= 1/255 ellipse can reach pixel rows
// 4b..4b+3 of the tile (band_mask, computed once per instance by emit). Both render kernels read the mask with the
// index and gather the Gaussian's record only when it is non-zero. Limits P to 2^28 (checked by the forward). The
// binning buffer is private scratch (rasterizer_impl.h:37-102); omr_debug_point_list returns the indices alone.
constexpr uint32_t PL_GID_BITS = 28;
constexpr uint32_t PL_GID_MASK = (1u << PL_GID_BITS) - 1u;
constexpr int PL_BANDS = 4;

// ---- geometry state: P Gaussians --------------------------------------------------------------------------
struct GeomState {
    float4* splat;            // [P][SPLAT_F4] render records (above)
    uint8_t* clamped;         // bit c set if channel c was clamped (forward.cu:79-81)
    uint32_t* tiles_touched;  // rect area (forward.cu:702)
    uint32_t* key_a;          // depth sort ping-pong keys (float bits of depth; culled -> 0xFFFFFFFF)
    uint32_t* key_b;
    uint32_t* val_a;          // depth sort ping-pong values (Gaussian index)
    uint32_t* val_b;
    uint32_t* hist;           // radix histograms [RADIX][blocks]
    uint32_t* scan_partials;  // scan block sums
    uint32_t* scan2_status;   // look-back words of the forward scans (launch_forward_scans), zeroed by preprocess
    uint32_t* offsets;        // inclusive scan of tiles_touched in depth order
    uint32_t* counters;       // [0] num_rendered, [1] prefiltered-cull flag, [2] huge_list count, [3] look-back error,
                              // [4] M = row slots of the row binning (sum of rect heights), [5] sh_jac_key of the
                              // inputs when preprocess stored sh_jac (else 0), [6] the same key, kept for
                              // omr_debug_set_sh_jac (which clears and restores [5])
    uint32_t* order;          // [P] depth order: the visible Gaussians by depth key (ties by index), then the culled (depth_sort)
    uint32_t* row_first;      // first gradient row of each Gaussian (index-order exclusive scan, launch_forward_scans)
    float* row_sums;          // backward: [P][GRAD_ROW] each Gaussian's instance rows summed (launch_row_sums)
    float4* conic_op;         // [P] conic + opacity (= splat record slot 1), contiguous for gaussian_bwd's coalesced
                              // read (raw-moment rows, GRAD_ROW above)
    uint32_t* huge_list;      // Gaussians with more than ROW_SUM_HUGE tiles, any order; count in counters[2]
    uint2* rect;              // rect word: rows | y0 << 11 | width << 21, x0 (0 if culled), for the row binning (bin.hip)
    uint2* drect;             // the rect words in depth order (launch_forward_scans, row path)
    uint32_t* row_offsets;    // inclusive scan of the rect rows in depth order (launch_forward_scans, row path)
    uint2* desc_r;            // [P / 2 + 2] first / last owner rank of each row-binning chunk (launch_forward_scans)
    float4* bin_rec;          // [P][2] {x, y, k, dd}, {1/a, t, dyR, Dt} (band_row_consts): the constants the binning's
                              // columns pass turns into each (Gaussian, row)'s reachable columns per band
    int* internal_radii;      // used when the caller passes radii == NULL (rasterizer_impl.cu:284-287)
    float* sh_jac;            // [P][9] dRGB/ddir per channel (gx[3], gy[3], gz[3]; sh_eval.h: sh_dir_grad) of the
                              // visible Gaussians, stored by preprocess for gaussian_bwd when it stages 16-coefficient rows

    // The carve's tail is optional: the row binning's arrays (rect .. bin_rec, ~56 B per Gaussian) only for views that
    // take it (capi.hip: row_binning), then sh_jac only when preprocess stores it (sh_jac_stored). Every other array
    // keeps its offset, so a reader that needs neither carves with the defaults, which leave the tail's pointers NULL.
    static size_t carve(char* base, size_t P, GeomState* s, bool rows = false, bool jac = false);
};

// ---- image state: N pixels, T tiles ------------------------------------------------------------------------
struct ImageState {
    float* final_T;     // accum_alpha in the reference (rasterizer_impl.cu:222)
    uint32_t* n_contrib;
    uint2* ranges;      // [T] (the reference allocates N, uses T)
    uint32_t* tile_order;  // [T] render schedule: tiles by descending cost within each XCD's share (launch_tile_order)
    uint32_t* tile_cost;   // [T] (instance, band) pairs the forward evaluated per tile (bench.py's VALU secondary)
    uint32_t* max_contrib;  // [T][FWD_GROUPS] each forward wave's largest last contributor (backward schedule)
    float* final_C;         // [3][N] blended colour before the background term (backward segment starts)
    static size_t carve(char* base, size_t N, size_t T, ImageState* s);
};

// ---- binning state: L instances ----------------------------------------------------------------------------
// The forward sizes this buffer BEFORE it knows L (capacity `cap` >= L from a hint, see capi.hip) so that it never
// waits for the host; the backward only learns R = L. So the two arrays the backward reads sit at offsets that
// depend on L alone: inst_grad at 0, the sorted point list right after R rows of it (canonical_list_offset), then
// row_valid (row_valid_offset). In the forward, the region [0, align(36 cap) + align(4 cap) + cap) is reserved for
// them; the final tile-sort pass writes the point list to base + canonical_list_offset(L) and render_fwd zeroes row_valid
// at base + row_valid_offset(L), with L read on the device.
__host__ __device__ inline size_t canonical_list_offset(size_t L)
{
    return (L * GRAD_ROW * sizeof(float) + ALIGN - 1) & ~(ALIGN - 1);
}
// the backward's row_valid bytes [L], right after the point list; render_fwd zeroes them (render_fwd.hip)
__host__ __device__ inline size_t row_valid_offset(size_t L)
{
    return canonical_list_offset(L) + ((L * sizeof(uint32_t) + ALIGN - 1) & ~(ALIGN - 1));
}
// Depth segments of the render backward: a tile's instance list is cut at the global positions that are multiples
// of CKPT (one backward wave per (tile, segment), render_bwd.hip). The forward checkpoints every pixel's state at
// each boundary it crosses (T and the colour accumulated in front, 16 B per pixel per boundary), so a segment's wave
// can start there instead of at the tile's last contributor. Segment (tile t, chunk c) has the unique id t + c
// (a later tile's chunks never precede an earlier tile's), so per-segment arrays take T + L / CKPT + 1 entries.
// The checkpoints are addressed through a buffer descriptor with 32-bit offsets: ckpt_bytes(L) < 2^31, i.e.
// L < 2^28 instances per view (checked by the forward).
#ifndef OMR_BWD_CK
#define OMR_BWD_CK 1024
#endif
constexpr uint32_t CKPT = OMR_BWD_CK;
// forward waves per tile (render_fwd.hip: launch_render_forward picks 1, 2 or 4 bands per wave, i.e. four, two or
// one wave(s) per tile, by the view's tile count); max_contrib keeps FWD_GROUPS slots per tile either way
constexpr int FWD_GROUPS = 4;
// views with at least this many tiles render one wave per tile: enough waves to fill the chip without splitting, and
// each tile's instances staged once (config E, 32 k tiles: render_fwd 0.476 -> 0.449 ms; config C, 8 k tiles: 0.272
// with two waves per tile vs 0.295 with one, profiles/r03z_ab_fwd_bands.txt)
constexpr uint32_t FWD_ONE_WAVE_TILES = 16384;
// views of at most this many tiles render four waves per tile (one band each): config A, 512 tiles (round 6)
constexpr uint32_t FWD_FOUR_WAVE_TILES = 1024;
// OMR_SH_JAC (default 1): preprocess stores each visible Gaussian's dRGB/ddir (GeomState::sh_jac) for gaussian_bwd
// when it stages 16-coefficient SH rows (0: never; gaussian_bwd then reads the SH rows)
#ifndef OMR_SH_JAC
#define OMR_SH_JAC 1
#endif
// whether a forward with these inputs stores sh_jac: preprocess's sh16 condition (colours from 16-coefficient rows on
// a 16-B aligned array), evaluated on the host to size the geometry buffer and in the kernel to write it
__host__ __device__ inline bool sh_jac_stored(const float* colors_precomp, int M, const float* shs)
{
    return OMR_SH_JAC && colors_precomp == nullptr && shs != nullptr && M == 16 &&
           (reinterpret_cast<uintptr_t>(shs) & 15u) == 0;
}
// GeomState::counters[5] after a forward that stored sh_jac: a key of the inputs sh_jac was computed from (the SH
// array, the means and the camera position; sh_eval.h: sh_dir_grad). gaussian_bwd takes sh_jac only if its own
// inputs give the same key, so a backward called with other SH, means or campos than its forward recomputes
// dRGB/ddir from its own SH rows, as the reference does (backward.cu:56-112). Never 0 (0 = not stored).
__host__ __device__ inline uint32_t sh_jac_key(const float* shs, const float* means3D, uint32_t cx, uint32_t cy,
                                               uint32_t cz)
{
    const uint64_t words[4] = {(uint64_t)reinterpret_cast<uintptr_t>(shs),
                               (uint64_t)reinterpret_cast<uintptr_t>(means3D), (uint64_t)cx | ((uint64_t)cy << 32),
                               (uint64_t)cz};
    uint64_t h = 0x4A41430B9E3779B9ull;
    for (int i = 0; i < 4; ++i) {
        h ^= words[i];
        h *= 0xFF51AFD7ED558CCDull;
        h ^= h >> 33;
    }
    return (uint32_t)h | 1u;
}
__host__ __device__ inline size_t ckpt_count(size_t L) { return L / CKPT + 1; }
__host__ __device__ inline size_t seg_count(size_t L, uint32_t T) { return (size_t)T + L / CKPT + 1; }
// the L-indexed region of the binning buffer, after row_valid: checkpoints [ckpt_count][256 pixels] float4
// {T, C_r, C_g, C_b} (pixel = band * 64 + lane), then the backward's schedule (units uint2 {tile, chunk}
// [seg_count], its unsorted form + costs, the unit count)
__host__ __device__ inline size_t ckpt_offset(size_t L) { return row_valid_offset(L) + align_up(L); }
__host__ __device__ inline size_t ckpt_bytes(size_t L) { return ckpt_count(L) * BLOCK_X * BLOCK_Y * 16; }
__host__ __device__ inline size_t units_offset(size_t L, uint32_t T) { return ckpt_offset(L) + align_up(ckpt_bytes(L)); }
__host__ __device__ inline size_t units_tmp_offset(size_t L, uint32_t T) { return units_offset(L, T) + align_up(seg_count(L, T) * 8); }
__host__ __device__ inline size_t unit_words_offset(size_t L, uint32_t T)
{
    return units_tmp_offset(L, T) + align_up(seg_count(L, T) * 12);
}
__host__ __device__ inline size_t l_region_end(size_t L, uint32_t T) { return unit_words_offset(L, T) + ALIGN; }

// The forward's device count word: counters[0] = num_rendered, counters[3] = look-back error word (GeomState).
// The binning kernels (sort.hip: live_count) and the forward render see 0 instances when the count exceeds the
// capacity the binning buffer was sized for or when a decoupled look-back gave up.
__device__ __forceinline__ size_t binning_count(const uint32_t* counters, size_t capacity)
{
    const uint32_t L = counters[0];
    return (L <= capacity && counters[3] == 0u) ? (size_t)L : 0u;
}

struct BinningState {
    float* inst_grad;      // [L][GRAD_ROW] backward scratch, indexed by gradient row slot (offset 0)
    uint32_t* point_list;  // sorted Gaussian indices at base + canonical_list_offset(L) (host-known only when L is)
    uint32_t* key_a;       // tile id ping-pong
    uint32_t* key_b;
    uint32_t* val_a;       // Gaussian index ping-pong
    uint32_t* val_b;
    uint32_t* hist;        // radix histograms
    uint32_t* scan_partials;
    uint32_t* block_owner;  // emit index: owner rank of every EMIT_SLOTS-th slot
    // the row binning (bin.hip; views of at most BIN_MAX_GRID tiles a side): row entries reuse key_a / key_b / val_a
    uint32_t* bin_hist_r;   // [2][gy][bin_chunks_r]
    uint32_t* bin_hist_b;   // [bin_chunks_b][gx]
    uint4* bin_desc_b;      // [bin_chunks_b][2]
    uint32_t* bin_words;    // [4]
    uint32_t* bin_zero;     // bin_zero_words look-back words
    uint8_t* row_valid;     // backward: 1 where inst_grad holds a row (at row_valid_offset(L); zeroed by render_fwd)
    uint32_t* point_keys;  // sorted tile ids (points at key_a or key_b)
    // carve for capacity cap; point_list is set for L = cap (exact sizing: backward, debug, omr_binning_bytes)
    static size_t carve(char* base, size_t cap, uint32_t gx, uint32_t gy, BinningState* s);
};

// number of 8-bit passes needed for tile ids < T (rasterizer_impl.cu:651: sort end bit = 32 + getHigherMsb(T))
inline uint32_t getHigherMsb(uint32_t n)  // rasterizer_impl.cu:47-62
{
    uint32_t msb = sizeof(n) * 4;
    uint32_t step = msb;
    while (step > 1) {
        step /= 2;
        if (n >> msb) msb += step;
        else msb -= step;
    }
    if (n >> msb) msb++;
    return msb;
}
inline int tile_sort_passes(uint32_t T) { return (int)div_up(getHigherMsb(T), RADIX_BITS); }

// ---- device helpers ----------------------------------------------------------------------------------------
#if defined(__HIPCC__)

__device__ __forceinline__ float3 transformPoint4x3(const float3& p, const float* m)  // auxiliary.h:85-93
{
    return {m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12], m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13],
            m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14]};
}
__device__ __forceinline__ float4 transformPoint4x4(const float3& p, const float* m)  // auxiliary.h:95-104
{
    return {m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12], m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13],
            m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14], m[3] * p.x + m[7] * p.y + m[11] * p.z + m[15]};
}
__device__ __forceinline__ float3 transformVec4x3Transpose(const float3& p, const float* m)  // auxiliary.h:116-124
{
    return {m[0] * p.x + m[1] * p.y + m[2] * p.z, m[4] * p.x + m[5] * p.y + m[6] * p.z,
            m[8] * p.x + m[9] * p.y + m[10] * p.z};
}
__device__ __forceinline__ float ndc2Pix(float v, int S)  // auxiliary.h:51-54 (double arithmetic)
{
    return (float)((((double)v + 1.0) * S - 1.0) * 0.5);
}
// auxiliary.h:56-66; returns rect in tiles, clamped to the grid
__device__ __forceinline__ void getRect(float2 p, int max_radius, uint32_t gx, uint32_t gy, uint32_t& x0, uint32_t& y0,
                                        uint32_t& x1, uint32_t& y1)
{
    const float r = (float)max_radius;
    x0 = min(gx, (uint32_t)max(0, (int)((p.x - r) / (float)BLOCK_X)));
    y0 = min(gy, (uint32_t)max(0, (int)((p.y - r) / (float)BLOCK_Y)));
    // ((p.x + r) + 16) - 1: the reference's macro arithmetic, evaluated left to right in float
    x1 = min(gx, (uint32_t)max(0, (int)((p.x + r + (float)BLOCK_X - 1.0f) / (float)BLOCK_X)));
    y1 = min(gy, (uint32_t)max(0, (int)((p.y + r + (float)BLOCK_Y - 1.0f) / (float)BLOCK_Y)));
}

// The per-Gaussian part of band_mask: threshold t and the completed-square terms. A Gaussian with 255 o < 1 gets
// t = -inf (no band), a degenerate conic a = k = dd = 0 and t = +inf (every band), so band_mask_of needs no branch.
struct BandConsts {
    float t, k, dd, a;
};
__device__ __forceinline__ BandConsts band_consts(float4 co)
{
    if (!(co.w * 255.0f >= 1.0f)) return {-__builtin_inff(), 0.f, 0.f, 0.f};  // even G = 1 gives alpha < 1/255
    const float a = co.x, b = co.y, c = co.z;
    if (!(a * c - b * b > 0.0f) || !(a > 0.0f)) return {__builtin_inff(), 0.f, 0.f, 0.f};  // degenerate: every band
    const float t = 2.0f * __logf(255.0f * co.w) * 1.002f + 0.02f;
    // completed square: q = a (dx - k dy)^2 + (det / a) dy^2 with k = -b / a (no cancellation between large terms)
    const float ra = __builtin_amdgcn_rcpf(a);
    return {t, -b * ra, (a * c - b * b) * ra, a};
}
template <int NB>
__device__ __forceinline__ uint32_t band_mask_of(const BandConsts& bc, float2 xy, uint32_t tx, uint32_t ty,
                                                 uint32_t band0)
{
    const float x0 = (float)(tx * BLOCK_X);
    const float lo = xy.x - (x0 + (float)(BLOCK_X - 1)), hi = xy.x - x0;  // dx over the tile's columns
    const float dy0 = xy.y - (float)(ty * BLOCK_Y + 4 * band0);
    uint32_t m = 0;
#pragma unroll
    for (int bb = 0; bb < NB; ++bb) {
        bool hit = false;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float dy = dy0 - (float)(4 * bb + r);
            const float kdy = bc.k * dy;
            const float e = __builtin_amdgcn_fmed3f(kdy, lo, hi) - kdy;  // the strip's column nearest the row minimum
            const float q = __builtin_fmaf(bc.a * e, e, bc.dd * dy * dy);
            hit = hit || q <= bc.t;
        }
        if (hit) m |= 1u << bb;
    }
    return m;
}
// The same question answered per band instead of per pixel row (emit's staged-owner path; a superset of
// band_mask_of, so result-identical): the rows a tile's column strip dx in [lo, hi] can reach form the interval
// [Y1, Y2] of dy = y - pixel row, the extent in dy of {q <= t} within the strip. Its top is on the column clamp(k Dt,
// lo, hi) (Dt = sqrt(t / dd): the ellipse's highest point, where dq/ddx = 0, lies at dx = k dy), where q = t has the
// roots dy = (a k l +- sqrt(A t - a dd l^2)) / A, A = a k^2 + dd; likewise the bottom on clamp(-k Dt, lo, hi). A band is
// kept if its rows' span [dy0 - 4b - 3, dy0 - 4b] meets [Y1, Y2], widened by 0.02 px + 2e-6 |Y| against rounding.
// About 30 VALU and two v_sqrt per instance instead of 16 rows x ~10 VALU.
struct BandSpan {
    float kDt, ak, adt, At, invA;  // per Gaussian; At = -inf: no band, At = +inf: every band
};
__device__ __forceinline__ BandSpan band_span_consts(const BandConsts& bc)
{
    if (bc.t == -__builtin_inff()) return {0.f, 0.f, 0.f, -__builtin_inff(), 1.f};
    if (bc.t == __builtin_inff()) return {0.f, 0.f, 0.f, __builtin_inff(), 1.f};
    const float A = __builtin_fmaf(bc.a * bc.k, bc.k, bc.dd);
    const float Dt = sqrtf(bc.t / bc.dd);
    return {bc.k * Dt, bc.a * bc.k, bc.a * bc.dd, A * bc.t, 1.0f / A};
}
template <int NB>
__device__ __forceinline__ uint32_t band_mask_span(const BandSpan& sp, float2 xy, uint32_t tx, uint32_t ty)
{
    const float x0 = (float)(tx * BLOCK_X);
    const float lo = xy.x - (x0 + (float)(BLOCK_X - 1)), hi = xy.x - x0;
    const float lt = __builtin_amdgcn_fmed3f(sp.kDt, lo, hi), lb = __builtin_amdgcn_fmed3f(-sp.kDt, lo, hi);
    const float dt = __builtin_fmaf(-sp.adt, lt * lt, sp.At), db = __builtin_fmaf(-sp.adt, lb * lb, sp.At);
    if (!(dt >= 0.0f)) return 0u;  // the strip misses the ellipse (or no band at all)
    // v_sqrt_f32 (1 ulp; the 0.02 px widening covers it)
    float y2 = (sp.ak * lt + __builtin_amdgcn_sqrtf(dt)) * sp.invA;
    float y1 = (sp.ak * lb - __builtin_amdgcn_sqrtf(fmaxf(db, 0.0f))) * sp.invA;
    y2 += 0.02f + 2e-6f * fabsf(y2);
    y1 -= 0.02f + 2e-6f * fabsf(y1);
    const float dy0 = xy.y - (float)(ty * BLOCK_Y);
    uint32_t m = 0;
#pragma unroll
    for (int b = 0; b < NB; ++b)
        if (dy0 - (float)(4 * b + 3) <= y2 && dy0 - (float)(4 * b) >= y1) m |= 1u << b;
    return m;
}

// The same question posed per (Gaussian, tile row) for the row binning's columns pass (bin.hip): for each band b of
// tile row ty, the tile columns x whose strip [16x, 16x + 15] meets the ellipse {q <= t} inside the band's slab of
// pixel rows, as an interval. Restricted to the slab dy in S = [dy0 - 4b - 3, dy0 - 4b] ∩ [-Dt, Dt] (Dt = sqrt(t /
// dd)), the ellipse a (dx - k dy)^2 + dd dy^2 <= t spans dx from the minimum over S of k dy - sqrt((t - dd dy^2) /
// a) to the maximum of k dy + sqrt(...): the right edge is concave with its top at dyR = k sqrt(a t / (dd A)), A =
// a k^2 + dd, so its maximum over S is at dyR clamped to S; the left edge is the mirror image (-dyR). "The ellipse
// meets strip x slab" is band_mask_span's question answered per slab instead of per strip, so it is likewise a
// superset of band_mask_of's per-row test; the extent is widened by 0.02 px + 2e-6 |X| against rounding, so a
// render kernel never skips a pixel it would blend (tests/test_gpu_parity.py checks the masks against every pixel).
// Per-Gaussian constants (preprocess -> bin_rec): {x, y, k, dd}, {1/a, t, dyR, Dt}; t = -inf: no band, +inf: every.
__device__ __forceinline__ void band_row_consts(const BandConsts& bc, float2 xy, float4& r0, float4& r1)
{
    if (!(bc.t > -__builtin_inff() && bc.t < __builtin_inff())) {
        r0 = make_float4(xy.x, xy.y, 0.f, 0.f);
        r1 = make_float4(0.f, bc.t, 0.f, 0.f);
        return;
    }
    const float A = __builtin_fmaf(bc.a * bc.k, bc.k, bc.dd);
    r0 = make_float4(xy.x, xy.y, bc.k, bc.dd);
    r1 = make_float4(1.0f / bc.a, bc.t, bc.k * sqrtf(bc.a * bc.t / (bc.dd * A)), sqrtf(bc.t / bc.dd));
}
// per band b: the reachable tile columns of tile row ty as xa | count << 16 (count 0: none), clipped to [x_lo, x_hi)
__device__ __forceinline__ uint4 band_row_intervals(float4 r0, float4 r1, uint32_t ty, uint32_t x_lo, uint32_t x_hi)
{
    const float mx = r0.x, my = r0.y, k = r0.z, dd = r0.w, inv_a = r1.x, t = r1.y, dyR = r1.z, Dt = r1.w;
    uint32_t out[4];
    const uint32_t full = x_lo | ((x_hi - x_lo) << 16);
    const float dy0 = my - (float)(ty * BLOCK_Y);
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const float s_hi = fminf(dy0 - (float)(4 * b), Dt), s_lo = fmaxf(dy0 - (float)(4 * b + 3), -Dt);
        const float da = __builtin_amdgcn_fmed3f(dyR, s_lo, s_hi), db = __builtin_amdgcn_fmed3f(-dyR, s_lo, s_hi);
        const float ra = __builtin_amdgcn_sqrtf(fmaxf(t - dd * da * da, 0.0f) * inv_a);
        const float rb = __builtin_amdgcn_sqrtf(fmaxf(t - dd * db * db, 0.0f) * inv_a);
        float xmax = k * da + ra, xmin = k * db - rb;
        xmax += 0.02f + 2e-6f * fabsf(xmax);
        xmin -= 0.02f + 2e-6f * fabsf(xmin);
        // strip x reaches [xmin, xmax] in dx = mx - px:  16 x + 15 >= mx - xmax  and  16 x <= mx - xmin
        const float fa = ceilf((mx - xmax - 15.0f) * (1.0f / BLOCK_X)), fb = floorf((mx - xmin) * (1.0f / BLOCK_X));
        const int xa = (int)fmaxf(fa, (float)x_lo), xb = (int)fminf(fb, (float)x_hi - 1.0f);
        out[b] = (s_lo <= s_hi && xa <= xb) ? (uint32_t)xa | ((uint32_t)(xb - xa + 1) << 16) : 0u;
    }
    if (t == __builtin_inff()) out[0] = out[1] = out[2] = out[3] = full;  // degenerate conic: every band
    if (t == -__builtin_inff()) out[0] = out[1] = out[2] = out[3] = 0u;   // 255 o < 1: no band
    return make_uint4(out[0], out[1], out[2], out[3]);
}
// the band mask of tile column x from band_row_intervals' words
__device__ __forceinline__ uint32_t band_mask_of_intervals(uint4 iv, uint32_t x)
{
    auto in = [&](uint32_t w) { return (x - (w & 0xFFFFu)) < (w >> 16) ? 1u : 0u; };
    return in(iv.x) | (in(iv.y) << 1) | (in(iv.z) << 2) | (in(iv.w) << 3);
}

// Which of the bands band0 .. band0 + NB - 1 of tile (tx, ty) (band b = pixel rows 4b..4b+3 of the tile, 16
// columns: the pixels of one wave's lanes, tile_wave.h) contain a pixel where alpha = min(0.99, o * exp(power))
// >= 1/255 can hold. With d = mean - pixel, that is q(d) = a dx^2 + 2 b dx dy + c dy^2 <= t = 2 ln(255 o). Along
// one pixel row (fixed dy) the minimum of q over the 16 columns is at dx* = -b dy / a clamped to the columns'
// range, so a band is reached iff one of its 4 rows reaches t: exact up to the continuous column range, and 17 %
// fewer (instance, band) pairs than the ellipse's bounding box at config C. t is widened (x 1.002 + 0.02) so that
// float rounding can never make the test drop a pixel the render kernels' own alpha test would blend: skipping an
// unreachable band is result-identical.
template <int NB>
__device__ __forceinline__ uint32_t band_mask(float2 xy, float4 co, uint32_t tx, uint32_t ty, uint32_t band0)
{
    return band_mask_of<NB>(band_consts(co), xy, tx, ty, band0);
}

__device__ __forceinline__ uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }

// Wave64 inclusive scans on DPP (gfx9 row_shr / row_bcast): four row_shr levels scan each 16-lane row, then
// row_bcast:15 carries rows 0 / 2 into rows 1 / 3 and row_bcast:31 carries row 1 into rows 2 and 3. Six VALU ops with
// no LDS round trip, where the __shfl_up ladder issues six dependent ds_bpermute. All 64 lanes must be active.
// dpp_ctrl: row_shr:n = 0x110 + n, row_bcast:15 = 0x142, row_bcast:31 = 0x143.
template <int CTRL, int ROW_MASK, bool BOUND_ZERO>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t x)
{
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROW_MASK, 0xf, BOUND_ZERO);
}
__device__ __forceinline__ uint32_t wave_incl_sum_u32(uint32_t x)
{
    x += dpp_u32<0x111, 0xf, true>(x);  // lanes without a source read 0 (bound_ctrl)
    x += dpp_u32<0x112, 0xf, true>(x);
    x += dpp_u32<0x114, 0xf, true>(x);
    x += dpp_u32<0x118, 0xf, true>(x);
    x += dpp_u32<0x142, 0xa, false>(x);  // rows 1, 3 += lane 15 / 47; rows 0, 2 add the old value 0
    x += dpp_u32<0x143, 0xc, false>(x);  // rows 2, 3 += lane 31
    return x;
}
// the same for max (values >= 0: the zero fill is the identity)
__device__ __forceinline__ uint32_t wave_incl_max_u32(uint32_t x)
{
    x = max(x, dpp_u32<0x111, 0xf, true>(x));
    x = max(x, dpp_u32<0x112, 0xf, true>(x));
    x = max(x, dpp_u32<0x114, 0xf, true>(x));
    x = max(x, dpp_u32<0x118, 0xf, true>(x));
    x = max(x, dpp_u32<0x142, 0xa, false>(x));
    x = max(x, dpp_u32<0x143, 0xc, false>(x));
    return x;
}
// number of set bits of `mask` below this lane
__device__ __forceinline__ uint32_t mask_rank(uint64_t mask)
{
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// The lanes of this wave whose BITS-bit digit equals this lane's (and that are valid): one ballot per bit, each
// folded in as peers &= ~(m ^ s) with s = the bit sign-extended (0 or ~0) — 6 VALU per bit on two 32-bit halves,
// against 11 for the `bit ? m : ~m` select the compiler builds through 64-bit masks (the ranks of the binning
// scatters and the radix downsweeps, sort.hip / bin.hip).
template <int BITS>
__device__ __forceinline__ uint64_t wave_match_digit(uint32_t d, bool valid)
{
    const uint64_t v = __ballot(valid);
    uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
#pragma unroll
    for (int b = 0; b < BITS; ++b) {
        const uint32_t sx = (uint32_t)((int32_t)(d << (31 - b)) >> 31);  // v_bfe_i32
        const uint64_t m = __ballot(sx != 0u);
        lo &= ~((uint32_t)m ^ sx);
        hi &= ~((uint32_t)(m >> 32) ^ sx);
    }
    return ((uint64_t)hi << 32) | lo;
}

// The peer masks of R rounds of digits (the lanes of this wave whose digit equals this lane's, as wave_match_digit
// returns them) by LDS ORs: each lane ORs its bit into its digit's 64-bit word of a wave-private table of NB words,
// reads the word back — every lane's OR of that instruction is in it, and OR commutes, so the order in which the LDS
// performs the atomics does not matter — and zeroes it for the next round. A wave's LDS operations complete in issue
// order, so the R rounds' 3R operations go out back to back with one wait, instead of one ballot per digit bit per
// round. An invalid lane ORs nothing in (its digit must still be < NB); its own mask is garbage and must not be used.
template <int R, uint32_t NB>
__device__ __forceinline__ void wave_peer_masks(const uint32_t (&d)[R], const bool (&valid)[R], uint64_t (&pm)[R],
                                                uint64_t* s_peer)
{
    const uint32_t lane = threadIdx.x & 63u;
    for (uint32_t i = lane; i < NB / 2; i += 64) reinterpret_cast<uint4*>(s_peer)[i] = make_uint4(0u, 0u, 0u, 0u);
    __builtin_amdgcn_wave_barrier();
    const uint64_t bit = 1ull << lane;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        __hip_atomic_fetch_or(&s_peer[d[r]], valid[r] ? bit : 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        __builtin_amdgcn_wave_barrier();
        pm[r] = s_peer[d[r]];
        __builtin_amdgcn_wave_barrier();
        s_peer[d[r]] = 0ull;  // lands after every lane's read of this round
        __builtin_amdgcn_wave_barrier();
    }
}

#endif  // __HIPCC__

}  // namespace omr

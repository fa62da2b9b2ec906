// tile_wave.h — shared pieces of the one-wave-per-tile render kernels (render_fwd.hip, render_bwd.hip).
//
// Layout: one wave64 owns one 16x16 tile. Lane l owns pixel column l % 16 and, in each of the four 16x4 bands
// b = 0..3 of the tile, the pixel row 4b + l / 16: four pixels per lane, one per band. An instance's band mask
// (band_mask, raster_common.h) is therefore wave-uniform, and a band the instance cannot reach is skipped with a
// scalar branch. Per instance, the per-lane work is amortised over up to four pixels and, in the backward, the
// wave reduction of the gradient row over up to 256 pixels happens once.
#pragma once

#include "raster_common.h"

namespace omr {

typedef float f2v __attribute__((ext_vector_type(2)));  // a VGPR pair for v_pk_* f32 ops
typedef uint32_t v4u __attribute__((ext_vector_type(4)));  // 16-B payload of raw buffer stores
constexpr int TW_BANDS = 4;       // 16x4 bands per 16x16 tile = pixels per lane
constexpr int TW_BATCH = 64;      // instances staged per batch (one per lane)
constexpr float LOG2E = 1.4426950408889634f;

// Gaussian falloff in base 2: p2 = log2(e) * power, power = -1/2 (a dx^2 + c dy^2) - b dx dy
// (forward.cu:434 / backward.cu:774). The staging lane folds -1/2 and log2(e) into q = {qa, qb, qc} once per
// instance, so each (pixel, instance) pair costs three VALU ops (dy, two FMAs) before v_exp_f32. Forward and backward
// evaluate exactly this expression, so they take identical contribute / skip decisions.
struct Quad {
    float qa, qb, qc;
};
__device__ __forceinline__ Quad quad_of_conic(float4 co)
{
    return {-0.5f * LOG2E * co.x, -LOG2E * co.y, -0.5f * LOG2E * co.z};
}
// The opacity rides in the exponent: o 2^p = 2^(p + log2 o), so the staging lane adds lo = log2(o) to the constant
// term and v_exp_f32 returns o G directly — one multiply less per (pixel, instance) in both render kernels.
// A lane's pixels share one column (dx), so p2 = p + lo is taken as a quadratic in dy whose dx-terms are formed once
// per instance: p2 = A + dy (B + qc dy), A = qa dx^2 + lo, B = qb dx — two FMAs per pixel after the per-instance
// setup. Explicit FMAs: render_fwd.o and render_bwd.o are built with different contraction flags and must take the
// same contribute / skip decisions.
struct ColQuad {
    float A, B, C;
};
__device__ __forceinline__ ColQuad column_quad(const Quad& q, float dx, float lo)
{
    return {__builtin_fmaf(q.qa * dx, dx, lo), q.qb * dx, q.qc};
}
__device__ __forceinline__ float falloff_p2(const ColQuad& k, float dy)
{
    return __builtin_fmaf(dy, __builtin_fmaf(k.C, dy, k.B), k.A);
}

// The reference's tests power > 0 and alpha = min(0.99, o 2^p) < 1/255 (forward.cu:434-437, backward.cu:774-779)
// on p2 = p + log2 o: p <= 0  <=>  p2 <= lo, and o 2^p >= 1/255  <=>  p2 >= -log2(255). Both render kernels test
// P2_FLOOR <= p2 <= lo BEFORE v_exp_f32 and feed v_exp -inf for a pixel that does not contribute, so o G, alpha and
// every product built from them are exactly 0 there without per-result selects. v_log_f32 is within an ulp and p2
// rounds at |p2| <= 8, so the boundary moves by ~1e-6 relative in alpha (the same class as v_exp_f32 vs expf; the
// parity allowance's power window carries 1e-5 for the exp implementations).
constexpr float P2_FLOOR = -7.99435343685885793769f;  // -log2(255)
// lo of a staged instance; clamped to >= P2_FLOOR: instances with 255 o < 1 are never staged (band_mask is 0 for
// them), and the clamp keeps the in-band test below exact for every staged one
__device__ __forceinline__ float p2_log2o(float opacity)
{
    return fmaxf(__builtin_amdgcn_logf(opacity), P2_FLOOR);
}
// P2_FLOOR <= p2 <= lo as ONE vector compare: v_med3 returns one of its inputs, and p2 itself exactly when it lies in
// [P2_FLOOR, lo]; a NaN p2 compares unequal. Two v_cmp and an s_and otherwise — the scalar unit is the render
// forward's tighter issue port.
__device__ __forceinline__ bool p2_in_band(float p2, float lo)
{
    return __builtin_amdgcn_fmed3f(p2, P2_FLOOR, lo) == p2;
}

// The per-Gaussian factors of backward.cu:805-840 applied to a Gaussian's summed raw moments g[0..5] = S_u dx,
// S_u dy, S_u dx^2, S_u dx dy, S_u dy^2, S_u (raster_common.h: GRAD_ROW), where u = o G dL/dalpha (the render backward's
// v_exp_f32 returns o G, see column_quad) = dL/dG G, the weight of the mean and conic terms: dG/ddelx = -G (a dx +
// b dy), ... With the staged quadratic form q = (-a/2, -b, -c/2) log2(e):  -(a S_ux + b S_uy) = (2 / log2 e) (qa S_ux +
// qb/2 S_uy), so dL/dmean2D.x = W/2 (2 / log2 e) (qa S_ux + qb/2 S_uy), likewise y with (qc, qb/2) and H/2;
// dL/dconic = -1/2 x the second moments (the reference's half-weight dconic.y slot); dL/dopacity = sum G dL/dalpha =
// S_u / o (o >= 1/255 for every Gaussian with a row: band_mask stages none below). In place.
__device__ __forceinline__ void raw_row_to_grads(float (&g)[9], float4 co, int W, int H)
{
    const Quad q = quad_of_conic(co);
    const float kx = (float)W / LOG2E, ky = (float)H / LOG2E;
    const float sux = g[0], suy = g[1], hb = 0.5f * q.qb;
    g[0] = kx * __builtin_fmaf(q.qa, sux, hb * suy);
    g[1] = ky * __builtin_fmaf(q.qc, suy, hb * sux);
    g[2] = -0.5f * g[2];
    g[3] = -0.5f * g[3];
    g[4] = -0.5f * g[4];
    g[5] = g[5] != 0.0f ? g[5] / co.w : g[5];  // a Gaussian without rows keeps +0 (any opacity, 0 included)
}

// one lane's view of a tile: pixel coordinates of its band pixels; band b of the tile = rows 4b..4b+3
struct TileLane {
    uint32_t tx, ty, lane;
    uint32_t px, py0;  // band b pixel = (px, py0 + 4b)
    __device__ __forceinline__ TileLane(uint32_t tile, uint32_t gx)
    {
        tx = tile % gx;
        ty = tile / gx;
        lane = threadIdx.x & 63u;
        px = tx * BLOCK_X + (lane & (BLOCK_X - 1));
        py0 = ty * BLOCK_Y + (lane / BLOCK_X);
    }
    __device__ __forceinline__ uint32_t py(int b) const { return py0 + 4u * (uint32_t)b; }
};

// bijective XCD-aware remap: blocks that share an XCD (orig % 8 equal) get consecutive logical ids, so
// neighbouring tiles (which share most of their Gaussians) hit the same L2 (MI355X: 8 XCDs, block b -> XCD b % 8)
__device__ __forceinline__ uint32_t xcd_remap(uint32_t orig, uint32_t nwg)
{
    const uint32_t q = nwg / 8, r = nwg % 8, xcd = orig % 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

// Max over the full wave, on every lane: DPP inside each 16-lane row (quad_perm xor1 / xor2, row_ror 4 / 8), then
// v_permlane16_swap / v_permlane32_swap across rows (see wave_ops.h: cross_row_sum) — no LDS round trip per level,
// unlike the ds_bpermute shuffles of __shfl_xor. All 64 lanes must be active.
template <int CTRL>
__device__ __forceinline__ uint32_t max_dpp(uint32_t v)
{
    return max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xf, 0xf, true));
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v)
{
    v = max_dpp<0xb1>(v);   // quad_perm [1,0,3,2]
    v = max_dpp<0x4e>(v);   // quad_perm [2,3,0,1]
    v = max_dpp<0x124>(v);  // row_ror:4
    v = max_dpp<0x128>(v);  // row_ror:8
    uint32_t a = v, b = v;
    asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
    v = max(a, b);
    a = v;
    b = v;
    asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b));
    return max(a, b);
}

__device__ __forceinline__ uint32_t uniform(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// ---- diagnostic wave timeline (build with -DOMR_STAMPS only; profiles/wave_timeline.py) ---------------------
// per wave: [0] s_memrealtime at start (100 MHz), [1] at end, [2] HW_ID | XCC_ID << 32, [3] unit index
#ifdef OMR_STAMPS
constexpr int STAMP_CAP = 1 << 17;
#define OMR_STAMP_DECL(name) __device__ uint64_t name[STAMP_CAP][4];
#define OMR_STAMP_BEGIN const uint64_t stamp_t0_ = __builtin_amdgcn_s_memrealtime();
#define OMR_STAMP_END(arr, unit)                                                                          \
    do {                                                                                                 \
        const uint64_t t1_ = __builtin_amdgcn_s_memrealtime();                                            \
        if ((threadIdx.x & 63) == 0 && (unit) < (uint32_t)STAMP_CAP) {                                    \
            arr[unit][0] = stamp_t0_;                                                                     \
            arr[unit][1] = t1_;                                                                           \
            arr[unit][2] = (uint64_t)__builtin_amdgcn_s_getreg(63492) |                                   \
                           ((uint64_t)__builtin_amdgcn_s_getreg(63508) << 32);                            \
            arr[unit][3] = (unit);                                                                        \
        }                                                                                                \
    } while (0)
#else
#define OMR_STAMP_DECL(name)
#define OMR_STAMP_BEGIN
#define OMR_STAMP_END(arr, unit) \
    do {                         \
    } while (0)
#endif

// Several independent waves share one workgroup (TW_WAVES tiles per block): gfx950 caps resident workgroups per
// CU, so one-wave workgroups would cap occupancy at a few waves per SIMD. The waves never synchronise with each
// other; each orders its own LDS staging with wave_sync().
#ifndef OMR_TW_WAVES
#define OMR_TW_WAVES 1
#endif
constexpr int TW_WAVES = OMR_TW_WAVES;
__device__ __forceinline__ void wave_sync()
{
    // LDS operations of one wave complete in issue order; this keeps the compiler from moving LDS accesses
    // across the staging boundary
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

}  // namespace omr

// render_bwd.hip — per-tile back-to-front gradient replay, gfx950.
//
// Follows cuda_rasterizer/backward.cu:671-843 (renderCUDA backward). Per pixel, the tile's instances are replayed
// back to front from the last contributor; for each contributing instance the reference accumulates, with nine
// float atomics into per-Gaussian arrays, dL/dmean2D.xy, dL/dconic.{x,y,w}, dL/dopacity and dL/dcolour.
//
// Structure (MI355X): ONE wave64 per (16x16 tile, depth segment) unit, four pixels per lane (one per 16x4 band,
// tile_wave.h), as in render_fwd.hip. A tile's instance list is cut at global positions that are multiples of
// CKPT (raster_common.h); the forward stored every pixel's T and accumulated colour at each boundary it crossed,
// so the wave of a segment starts at its upper boundary from that state (or from the final state for a pixel whose
// last contributor lies in front of it) and replays only its own positions. Units are ordered longest first by
// the forward's per-segment work (sort.hip: backward_schedule_kernel): long tiles no longer form the launch's tail. For each instance the wave accumulates, per lane and over the bands the instance reaches,
// nine moments of the pixel weights u = o G * dL/dalpha (v_exp_f32 returns o G: tile_wave.h, column_quad) and the
// colour weights alpha * T:
//     S_u, S_u dx, S_u dy, S_u dx^2, S_u dx dy, S_u dy^2, S_aT dpix_{r,g,b}
// (a lane's four pixels share one column, so only S_u, S_u dy, S_u dy^2 are summed per band; the x-moments are
// their dx-multiples)
// The per-Gaussian constants of the reference's expressions (conic, opacity, 0.5 W, 0.5 H, -1/2) are linear
// factors that every instance of the Gaussian shares, so they are applied neither per pixel nor per instance but
// once to the Gaussian's summed rows (raster_common.h: GRAD_ROW); the nine values of an instance are
// summed over the wave: eight transposed through LDS, the ninth by v_permlane{16,32}_swap + DPP (wave_ops.h).
// Contributing instances are summed in pairs: the first one's eight values wait in LDS rows 0-7
// until the second's fill rows 8-15, then one pass sums both (wave_sum9x2_stored).
// Lanes 0..8 store the instance's 36-B gradient row, indexed by its row slot (Gaussian-index-major: row_first), with
// plain stores, and lane 0 marks the slot in row_valid (zeroed before the launch); an instance no pixel takes a contribution from writes
// nothing — at dense configs most instances lie behind every pixel's last contributor. gaussian_bwd.hip sums each
// Gaussian's marked rows in a fixed order. No atomics: gradients are bitwise reproducible.
//
// The per-pixel recurrence keeps two numbers instead of the reference's seven (T, accum_rec[3], last_alpha,
// last_color[3]): T and s = bg . dL/dpix * T_final + sum over the contributors j behind the current instance of
// (c_j . dL/dpix) alpha_j T_j. Since T_i (1 - alpha_i) accum_rec_i = sum_j c_j alpha_j T_j (unroll
// backward.cu:790-797), the reference's
//     dL/dalpha_i = T_i (c_i - accum_rec_i) . dL/dpix - T_final / (1 - alpha_i) bg . dL/dpix
// equals T_i c_i . dL/dpix - s / (1 - alpha_i): the same quantity, rounded differently.
// T_i is recovered with v_rcp_f32 (T_{i+1} / (1 - alpha_i)), as the reference divides (backward.cu:782).
// Instances at or behind every band's last contributor are skipped; batches in front of every pixel's last
// contributor run an instance loop without the per-lane position test (min_last below).
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "kernels.h"
#include "tile_wave.h"
#include "wave_ops.h"

namespace omr {

namespace {


OMR_STAMP_DECL(g_stamps_bwd)

// diagnostic (A/B only): OMR_BWD_DIAG_EXTRA independent extra VALU per evaluated band, to price one VALU op there
// diagnostic (A/B only, wrong gradients): OMR_BWD_DIAG_NOMARK drops the row_valid marks, to price their stores
#ifndef OMR_BWD_DIAG_NOMARK
#define OMR_BWD_DIAG_NOMARK 0
#endif
#ifndef OMR_BWD_DIAG_EXTRA
#define OMR_BWD_DIAG_EXTRA 0
#endif

#ifdef OMR_BWD_COUNT
// diagnostic: staged instances, (instance, band) evaluations, evaluations with a contributing pixel, instances
// with any contribution, contributing (pixel, instance) pairs
__device__ unsigned long long g_bwd_counts[5];
#define BWD_COUNT(k, v) cnt_[k] += (v)
#else
#define BWD_COUNT(k, v)
#endif

#ifndef OMR_BWD_MINW
#define OMR_BWD_MINW 1
#endif
// Positions staged per batch (<= TW_BATCH). The staging arrays take 48 B per position: with 64 the workgroup's LDS is
// 7424 B, which caps residency at 21-22 waves per CU, below the 24 (6 per SIMD) its 78 VGPRs allow; with 40 it is
// 6272 B. Views with more units than resident wave slots (launch_render_backward) take OMR_BWD_BATCH (interleaved A/B,
// profiles/r04n_ab_*.txt: render_bwd C 0.3935 -> 0.3880 ms, E 0.8003 -> 0.7853 ms with 40); views whose units all fit
// at once keep 64, where the extra batches' round trips cost more than residency gains (B 0.0756 vs 0.0770 ms).
#ifndef OMR_BWD_BATCH
#define OMR_BWD_BATCH 40
#endif
template <int BWD_BATCH>
__global__ __launch_bounds__(64 * TW_WAVES, OMR_BWD_MINW) void render_bwd_kernel(RenderBwdArgs a)
{
    static_assert(BWD_BATCH <= TW_BATCH, "one position per lane");
    OMR_STAMP_BEGIN
    __shared__ float4 s_geo_all[TW_WAVES][BWD_BATCH];   // x, y, position in range (u32 bits), band mask (u32 bits)
    __shared__ float4 s_quad_all[TW_WAVES][BWD_BATCH];  // qa, qb, qc, log2(opacity) (tile_wave.h: column_quad)
    __shared__ float4 s_rgb_all[TW_WAVES][BWD_BATCH];   // colour, gradient row slot (u32 bits)
    // rows 0-7: the held instance's eight values, rows 8-15: its partner's (wave_sum9x2_stored)
    __shared__ __attribute__((aligned(16))) float s_red_all[TW_WAVES][16 * WS_LDS_STRIDE];

    static_assert(TW_WAVES == 1, "one (tile, segment) unit per workgroup");
    const uint32_t wv = 0;
    const uint32_t nunits = *a.unit_count;
    if (blockIdx.x >= nunits) return;  // the grid is an upper bound on the unit count
    const uint2 unit = a.units[xcd_remap(blockIdx.x, nunits)];
    const uint32_t tile = unit.x, chunk = unit.y;
    float4* s_geo = s_geo_all[wv];
    float4* s_quad = s_quad_all[wv];
    float4* s_rgb = s_rgb_all[wv];
    const TileLane tl(tile, a.gx);
    const uint32_t lane = tl.lane;
    const float pxf = (float)tl.px;
    const size_t plane = (size_t)a.H * a.W;

    float T[TW_BANDS], s[TW_BANDS];
    f2v dp01[TW_BANDS];  // dL/dpix r, g: one register pair, the packed FMA's operand
    float dp2[TW_BANDS];
    uint32_t last[TW_BANDS];
    uint32_t band_end[TW_BANDS];  // wave-uniform: max last contributor of the band
    // wave-uniform: below this position every pixel of the tile that has a last contributor is in front of it. A pixel
    // without one has no in-band instance in the tile's list at all (the forward blends every in-band instance until
    // saturation, with the same arithmetic), so it imposes nothing; a pixel outside the image (T = 0, dL/dpix = 0)
    // imposes 0 so that it never marks a row
    uint32_t min_last = ~0u;
    // the four bands' per-pixel loads are issued together (addresses clamped to pixel 0 outside the image, the
    // values masked after), so the prologue waits for one round trip per group instead of one per band
    bool inside[TW_BANDS];
    uint32_t pix[TW_BANDS];
#pragma unroll
    for (int b = 0; b < TW_BANDS; ++b) {
        const uint32_t py = tl.py(b);
        inside[b] = tl.px < (uint32_t)a.W && py < (uint32_t)a.H;
        pix[b] = inside[b] ? a.W * py + tl.px : 0u;
    }
    uint32_t max_c = 0;
#pragma unroll
    for (int b = 0; b < TW_BANDS; ++b) last[b] = a.n_contrib[pix[b]];
    // the range and the per-pixel state depend on none of the last contributors: requested with them, one memory
    // round trip for the prologue's independent loads instead of three (n_contrib, then ranges, then the pixels)
    const uint2 range = a.ranges[tile];
    const float bg0 = a.bg[0], bg1 = a.bg[1], bg2 = a.bg[2];
    float Tf[TW_BANDS], d0[TW_BANDS], d1[TW_BANDS], d2[TW_BANDS];
#pragma unroll
    for (int b = 0; b < TW_BANDS; ++b) {
        Tf[b] = a.final_T[pix[b]];
        d0[b] = a.dL_dpix[pix[b]];
        d1[b] = a.dL_dpix[plane + pix[b]];
        d2[b] = a.dL_dpix[2 * plane + pix[b]];
    }
#pragma unroll
    for (int b = 0; b < TW_BANDS; ++b) {
        last[b] = inside[b] ? last[b] : 0u;
        band_end[b] = uniform(wave_max_u32(last[b]));
        min_last = min(min_last, ~uniform(wave_max_u32(~(inside[b] ? (last[b] ? last[b] : ~0u) : 0u))));
        max_c = max(max_c, band_end[b]);
    }
    const uint32_t n = range.y - range.x;
    max_c = min(max_c, n);
    // this unit's depth segment of the list, local positions [seg_lo, seg_hi) (raster_common.h: CKPT)
    const uint32_t seg_lo = max(range.x, chunk * CKPT) - range.x;
    const uint32_t seg_hi = min(range.x + max_c, (chunk + 1) * CKPT) - range.x;
    const bool resume = seg_hi < max_c;  // a boundary inside the list: some pixels blend behind it
    float4 ck[TW_BANDS];
    float fc0[TW_BANDS], fc1[TW_BANDS], fc2[TW_BANDS];
    if (resume) {  // wave-uniform; the checkpoint row (chunk + 1) exists: its boundary lies inside this tile's list
#pragma unroll
        for (int b = 0; b < TW_BANDS; ++b) {
            ck[b] = a.ckpt[(size_t)(chunk + 1) * BLOCK_SIZE + b * 64 + lane];
            fc0[b] = a.final_C[pix[b]];
            fc1[b] = a.final_C[plane + pix[b]];
            fc2[b] = a.final_C[2 * plane + pix[b]];
        }
    }
#pragma unroll
    for (int b = 0; b < TW_BANDS; ++b) {
        const float e0 = inside[b] ? d0[b] : 0.f, e1 = inside[b] ? d1[b] : 0.f, e2 = inside[b] ? d2[b] : 0.f;
        dp01[b] = f2v{e0, e1};
        dp2[b] = e2;
        T[b] = inside[b] ? Tf[b] : 0.f;
        s[b] = T[b] * (bg0 * e0 + bg1 * e1 + bg2 * e2);
        if (resume && last[b] > seg_hi) {
            // the pixel still blends behind the boundary: start from the forward's state there, T in front of the
            // boundary and s = bg . dL/dpix T_final + dL/dpix . (C_final - C in front of the boundary)
            T[b] = ck[b].x;
            s[b] += e0 * (fc0[b] - ck[b].y) + e1 * (fc1[b] - ck[b].z) + e2 * (fc2[b] - ck[b].w);
        }
    }

    // instances behind every pixel's last contributor get no row (row_valid stays 0 for them)

#ifdef OMR_BWD_COUNT
    uint32_t cnt_[5] = {0, 0, 0, 0, 0};
#endif
    float pv8 = 0.f;        // the held instance's 9th value (its first eight wait in rows 0-7 of s_red)
    uint32_t pslot = ~0u;   // its gradient row slot (wave-uniform: an SGPR); ~0: nothing held

    // positions seg_hi-1 .. seg_lo, BWD_BATCH per batch, back to front: batch entry `lane` <-> position hi-1-lane
    for (int hi = (int)seg_hi; hi > (int)seg_lo; hi -= BWD_BATCH) {
        const int cnt = min(hi - (int)seg_lo, BWD_BATCH);
        uint32_t m = 0;
        float4 p, co, c;
        uint32_t pos = 0, slot = 0;
        if ((int)lane < cnt) {
            pos = (uint32_t)(hi - 1 - (int)lane);
            const uint32_t v = a.point_list[range.x + pos];  // Gaussian index | band mask (emit)
            m = v >> PL_GID_BITS;
#pragma unroll
            for (int b = 0; b < TW_BANDS; ++b)
                if (pos >= band_end[b]) m &= ~(1u << b);
            if (m) {  // record and row base are gathered only for an instance some band still needs
                const uint32_t gid = v & PL_GID_MASK;
                const float4* rec = a.splat + (size_t)gid * SPLAT_F4;  // one 64-B line
                const uint32_t first = a.row_first[gid];
                p = rec[0];
                co = rec[1];
                c = rec[2];
                const float4 rect = rec[3];
                // gradient row of (Gaussian, tile): its rows follow its rect row-major (duplicateWithKeys order)
                slot = first + (tl.ty - __builtin_bit_cast(uint32_t, rect.y)) * __builtin_bit_cast(uint32_t, c.w) +
                       (tl.tx - __builtin_bit_cast(uint32_t, rect.x));
            }
        }
        const uint64_t useful = __ballot(m != 0);
        if (m != 0) {
            const uint32_t r = mask_rank(useful);
            const Quad q = quad_of_conic(co);
            s_geo[r] = make_float4(p.x, p.y, __builtin_bit_cast(float, pos), __builtin_bit_cast(float, m));
            s_quad[r] = make_float4(q.qa, q.qb, q.qc, p2_log2o(co.w));
            s_rgb[r] = make_float4(c.x, c.y, c.z, __builtin_bit_cast(float, slot));
        }
        wave_sync();  // orders this wave's LDS stores before its reads below
        const uint32_t nuse = (uint32_t)__popcll(useful);
        BWD_COUNT(0, nuse);
        // the instance loop, instantiated with and without the per-lane position test: a batch whose positions all
        // lie below every band's smallest last contributor (band_min) needs none (one VALU per evaluated band less)
        auto instances = [&](auto pos_test) {
            for (uint32_t j = 0; j < nuse; ++j) {
                const float4 g = s_geo[j];
                const float4 qo = s_quad[j];
                const float4 f = s_rgb[j];
                const uint32_t mb = uniform(__builtin_bit_cast(uint32_t, g.w));
                const uint32_t ipos = __builtin_bit_cast(uint32_t, g.z);
                const Quad q = {qo.x, qo.y, qo.z};
                const float dx = g.x - pxf;
                const float lo = qo.w;
                const ColQuad kq = column_quad(q, dx, lo);
                const float dy0 = g.y - (float)tl.py0;
                // dx is the same for all four of the lane's pixels (one column), so the x-moments are dx-multiples of
                // the band sums: S_u dx = dx S_u, S_u dx^2 = dx^2 S_u, S_u dx dy = dx S_u dy (applied after the bands)
                f2v s_uy = {0.f, 0.f};  // S_u, S_u dy
                f2v sc01 = {0.f, 0.f};  // S_aT dpix_r, S_aT dpix_g
                float suyy = 0.f, sc2 = 0.f;
                uint32_t any = 0;  // bands with a contributing pixel (set in wave-uniform branches: an SGPR)
    #pragma unroll
                for (int b = 0; b < TW_BANDS; ++b) {
                    if (!(mb & (1u << b))) continue;  // scalar branch
                    const float dp0b = dp01[b].x, dp1b = dp01[b].y, dp2b = dp2[b];
                    const uint32_t lastb = last[b];
                    const float dy = dy0 - (float)(4 * b);
                    const float p2 = falloff_p2(kq, dy);
                    // backward.cu:770-781: skip positions at/after the pixel's last contributor, power > 0, alpha < 1/255
                    const bool contrib = (decltype(pos_test)::value ? ipos < lastb : true) && p2_in_band(p2, lo);
                    BWD_COUNT(1, 1);
                    if (!__ballot(contrib)) continue;
                    BWD_COUNT(2, 1);
                    BWD_COUNT(4, (uint32_t)__popcll(__ballot(contrib)));
                    any |= 1u << b;
                    // a lane that does not contribute gets oG = alpha = 0: inv = 1, T and s unchanged, u = wc = 0
                    const float oG = __builtin_amdgcn_exp2f(contrib ? p2 : -__builtin_inff());  // o G (column_quad)
                    const float alpha = fminf(0.99f, oG);
                    const float inv = __builtin_amdgcn_rcpf(1.0f - alpha);
                    T[b] *= inv;
                    const float Ti = T[b];
                    const float cdot = __builtin_fmaf(f.x, dp0b, __builtin_fmaf(f.y, dp1b, f.z * dp2b));
                    const float dL_dalpha = __builtin_fmaf(Ti, cdot, -s[b] * inv);
                    const float wc = alpha * Ti;  // dchannel/dcolour (backward.cu:800)
                    s[b] = __builtin_fmaf(cdot, wc, s[b]);
                    const float u = oG * dL_dalpha;  // dL/dG G; dL/dopacity gets u / o (raw_row_to_grads)
                    const float uy = u * dy;
                    s_uy += f2v{u, uy};
                    suyy = __builtin_fmaf(uy, dy, suyy);
                    sc01 = __builtin_elementwise_fma(f2v{wc, wc}, dp01[b], sc01);
                    sc2 = __builtin_fmaf(wc, dp2b, sc2);
#if OMR_BWD_DIAG_EXTRA
#pragma unroll
                    for (int e = 0; e < OMR_BWD_DIAG_EXTRA; ++e) asm volatile("v_mov_b32 %0, %0" : "+v"(sc2));  // 1 VALU each
#endif
                }
                const uint32_t slot_j = __builtin_bit_cast(uint32_t, f.w);
                if (!any) continue;  // no pixel took a contribution: no row
                BWD_COUNT(3, 1);
                const float su = s_uy.x, suy = s_uy.y;
                const float sux = su * dx, suxx = sux * dx, suxy = suy * dx;
                float v[8];
                // the raw moments: their per-Gaussian factors are applied once to the Gaussian's sums (raw_row_to_grads)
                v[0] = sux;
                v[1] = suy;
                v[2] = suxx;
                v[3] = suxy;
                v[4] = suyy;
                v[5] = su;                                         // dL/dopacity
                v[6] = sc01.x;                                     // dL/dcolour
                v[7] = sc01.y;
                float t8;
                float* s_red = s_red_all[wv];
                const uint32_t slot_u = uniform(slot_j);
                const bool held = pslot != ~0u;  // scalar
                const uint32_t base = held ? 8u * WS_LDS_STRIDE : 0u;
    #pragma unroll
                for (int k = 0; k < 8; ++k) s_red[base + k * WS_LDS_STRIDE + lane] = v[k];
                if (!held) {
                    pv8 = sc2;
                    pslot = slot_u;
                    continue;
                }
                {
                    const float tv = wave_sum9x2_stored(pv8, sc2, lane, s_red, &t8);
                    // lane 4k holds value k (k < 8 the held row's, k >= 8 this one's); lanes 1 and 33 the 9th values
                    const bool lead = (lane & 3) == 0;
                    const uint32_t dslot = (lane < 32) ? pslot : slot_u;
                    if (lead || (lane & 31) == 1)
                        a.inst_grad[(size_t)dslot * GRAD_ROW + (lead ? ((lane >> 2) & 7u) : 8u)] = lead ? tv : t8;
                    if (!OMR_BWD_DIAG_NOMARK && (lane & 31) == 0) a.row_valid[dslot] = 1;
                    pslot = ~0u;
                }
            }
        };
        if ((uint32_t)(hi - 1) < min_last) instances(std::false_type{});
        else instances(std::true_type{});
        wave_sync();  // the next batch overwrites the staging arrays
    }
    if (pslot != ~0u) {  // the unit's last contributing instance had no partner: sum its rows 0-7 alone
        float v[8], t8;
        const float* r8 = s_red_all[wv];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = r8[k * WS_LDS_STRIDE + lane];
        const float tv = wave_sum9_lds(v, pv8, lane, s_red_all[wv], &t8);
        const bool lead = (lane & 7) == 0;
        if (lead || lane == 1) a.inst_grad[(size_t)pslot * GRAD_ROW + (lead ? (lane >> 3) : 8u)] = lead ? tv : t8;
        if (!OMR_BWD_DIAG_NOMARK && lane == 0) a.row_valid[pslot] = 1;
    }
    OMR_STAMP_END(g_stamps_bwd, blockIdx.x);
#ifdef OMR_BWD_COUNT
    if (lane == 0)
        for (int k = 0; k < 5; ++k) atomicAdd(&g_bwd_counts[k], (unsigned long long)cnt_[k]);
#endif
}

// ---- small views: two waves per unit, two bands per wave ----------------------------
// Each (tile, segment) unit is one 128-thread workgroup: wave h owns bands 2h and 2h + 1 (rows 8h .. 8h + 7), so a
// lane carries two pixels' state instead of four. Wave 0 stages each batch for both; each wave walks the staged
// instances its bands reach and reduces its own nine moments per contributing instance (paired as in
// render_bwd_kernel when PAIR, else one wave_sum9_lds each) into an LDS row per (half, staged instance); after the
// batch the two half-tile rows are added (a half that took no contribution adds nothing) and stored as the
// instance's 36-B row. The same rows as render_bwd_kernel up to the order of the float additions (both fixed:
// deterministic).
// It issues 27 % more VALU than one wave per unit (instances reaching both halves are set up and reduced twice) and
// its two waves meet at three barriers per batch: at config C it is 45 % slower. But on
// views whose units all fit on the chip at once as one-wave workgroups (A, B) the kernel's time is the chains of its
// few waves per SIMD, and twice the waves cover them: A render_bwd 25.6 -> 21.6 us, B 75.8 -> 71.6 us
// (profiles/r06h_ab_{A,B}.txt). launch_render_backward takes it there.
template <int BWD_BATCH, bool PAIR>
__global__ __launch_bounds__(128) void render_bwd2_kernel(RenderBwdArgs a)
{
    constexpr int NB = 2;  // bands per wave
    __shared__ float4 s_geo[BWD_BATCH];   // x, y, position in range (u32 bits), band mask (u32 bits)
    __shared__ float4 s_quad[BWD_BATCH];  // qa, qb, qc, log2(opacity)
    __shared__ float4 s_rgb[BWD_BATCH];   // colour, gradient row slot (u32 bits)
    __shared__ __attribute__((aligned(16))) float s_red_all[2][(PAIR ? 16 : 8) * WS_LDS_STRIDE];
    __shared__ float s_R[2][BWD_BATCH][GRAD_ROW];  // each half's reduced nine values per staged instance
    __shared__ uint32_t s_F[2][BWD_BATCH];         // 1: that half reduced the instance
    __shared__ uint32_t s_bend[4], s_maxc[2], s_nuse;

    const uint32_t nunits = *a.unit_count;
    if (blockIdx.x >= nunits) return;  // block-uniform
    const uint2 unit = a.units[xcd_remap(blockIdx.x, nunits)];
    const uint32_t tile = unit.x, chunk = unit.y;
    const uint32_t h = uniform(threadIdx.x >> 6);
    float* s_red = s_red_all[h];
    const TileLane tl(tile, a.gx);
    const uint32_t lane = tl.lane;
    const float pxf = (float)tl.px;
    const size_t plane = (size_t)a.H * a.W;

    float T[NB], s[NB];
    f2v dp01[NB];
    float dp2[NB];
    uint32_t last[NB], band_end[NB];
    uint32_t min_last = ~0u;
    bool inside[NB];
    uint32_t pix[NB];
#pragma unroll
    for (int bb = 0; bb < NB; ++bb) {
        const uint32_t py = tl.py(2 * (int)h + bb);
        inside[bb] = tl.px < (uint32_t)a.W && py < (uint32_t)a.H;
        pix[bb] = inside[bb] ? a.W * py + tl.px : 0u;
    }
#pragma unroll
    for (int bb = 0; bb < NB; ++bb) last[bb] = a.n_contrib[pix[bb]];
    const uint2 range = a.ranges[tile];
    const float bg0 = a.bg[0], bg1 = a.bg[1], bg2 = a.bg[2];
    float Tf[NB], d0[NB], d1[NB], d2[NB];
#pragma unroll
    for (int bb = 0; bb < NB; ++bb) {
        Tf[bb] = a.final_T[pix[bb]];
        d0[bb] = a.dL_dpix[pix[bb]];
        d1[bb] = a.dL_dpix[plane + pix[bb]];
        d2[bb] = a.dL_dpix[2 * plane + pix[bb]];
    }
    uint32_t max_c = 0;
#pragma unroll
    for (int bb = 0; bb < NB; ++bb) {
        last[bb] = inside[bb] ? last[bb] : 0u;
        band_end[bb] = uniform(wave_max_u32(last[bb]));
        min_last = min(min_last, ~uniform(wave_max_u32(~(inside[bb] ? (last[bb] ? last[bb] : ~0u) : 0u))));
        max_c = max(max_c, band_end[bb]);
    }
    if (lane == 0) {
        s_bend[2 * h] = band_end[0];
        s_bend[2 * h + 1] = band_end[1];
        s_maxc[h] = max_c;
    }
    for (uint32_t j = threadIdx.x; j < 2u * BWD_BATCH; j += 128u) (&s_F[0][0])[j] = 0u;
    __syncthreads();
    const uint32_t bend_all[4] = {s_bend[0], s_bend[1], s_bend[2], s_bend[3]};
    const uint32_t n = range.y - range.x;
    max_c = min(max(s_maxc[0], s_maxc[1]), n);
    const uint32_t seg_lo = max(range.x, chunk * CKPT) - range.x;
    const uint32_t seg_hi = min(range.x + max_c, (chunk + 1) * CKPT) - range.x;
    const bool resume = seg_hi < max_c;
    float4 ck[NB];
    float fc0[NB], fc1[NB], fc2[NB];
    if (resume) {
#pragma unroll
        for (int bb = 0; bb < NB; ++bb) {
            ck[bb] = a.ckpt[(size_t)(chunk + 1) * BLOCK_SIZE + (2 * h + bb) * 64 + lane];
            fc0[bb] = a.final_C[pix[bb]];
            fc1[bb] = a.final_C[plane + pix[bb]];
            fc2[bb] = a.final_C[2 * plane + pix[bb]];
        }
    }
#pragma unroll
    for (int bb = 0; bb < NB; ++bb) {
        const float e0 = inside[bb] ? d0[bb] : 0.f, e1 = inside[bb] ? d1[bb] : 0.f, e2 = inside[bb] ? d2[bb] : 0.f;
        dp01[bb] = f2v{e0, e1};
        dp2[bb] = e2;
        T[bb] = inside[bb] ? Tf[bb] : 0.f;
        s[bb] = T[bb] * (bg0 * e0 + bg1 * e1 + bg2 * e2);
        if (resume && last[bb] > seg_hi) {
            T[bb] = ck[bb].x;
            s[bb] += e0 * (fc0[bb] - ck[bb].y) + e1 * (fc1[bb] - ck[bb].z) + e2 * (fc2[bb] - ck[bb].w);
        }
    }

    float pv8 = 0.f;       // PAIR: the held instance's 9th value
    uint32_t pj = ~0u;     // PAIR: its staged index (an SGPR); ~0: nothing held
    for (int hi = (int)seg_hi; hi > (int)seg_lo; hi -= BWD_BATCH) {
        const int cnt = min(hi - (int)seg_lo, BWD_BATCH);
        if (h == 0) {  // wave 0 stages the batch for both halves
            uint32_t m = 0;
            float4 p, co, c;
            uint32_t pos = 0, slot = 0;
            if ((int)lane < cnt) {
                pos = (uint32_t)(hi - 1 - (int)lane);
                const uint32_t v = a.point_list[range.x + pos];
                m = v >> PL_GID_BITS;
#pragma unroll
                for (int b = 0; b < 4; ++b)
                    if (pos >= bend_all[b]) m &= ~(1u << b);
                if (m) {
                    const uint32_t gid = v & PL_GID_MASK;
                    const float4* rec = a.splat + (size_t)gid * SPLAT_F4;
                    const uint32_t first = a.row_first[gid];
                    p = rec[0];
                    co = rec[1];
                    c = rec[2];
                    const float4 rect = rec[3];
                    slot = first + (tl.ty - __builtin_bit_cast(uint32_t, rect.y)) * __builtin_bit_cast(uint32_t, c.w) +
                           (tl.tx - __builtin_bit_cast(uint32_t, rect.x));
                }
            }
            const uint64_t useful = __ballot(m != 0);
            if (m != 0) {
                const uint32_t r = mask_rank(useful);
                const Quad q = quad_of_conic(co);
                s_geo[r] = make_float4(p.x, p.y, __builtin_bit_cast(float, pos), __builtin_bit_cast(float, m));
                s_quad[r] = make_float4(q.qa, q.qb, q.qc, p2_log2o(co.w));
                s_rgb[r] = make_float4(c.x, c.y, c.z, __builtin_bit_cast(float, slot));
            }
            if (lane == 0) s_nuse = (uint32_t)__popcll(useful);
        }
        __syncthreads();
        const uint32_t nuse = uniform(s_nuse);
        auto reduce_store = [&](const float (&v)[8], float v8, uint32_t j) {  // one instance, unpaired
            float t8;
            const float tv = wave_sum9_lds(v, v8, lane, s_red, &t8);
            if ((lane & 7) == 0) s_R[h][j][lane >> 3] = tv;
            if (lane == 1) s_R[h][j][8] = t8;
            if (lane == 0) s_F[h][j] = 1u;
            wave_sync();  // the image is rewritten by the next instance
        };
        auto instances = [&](auto pos_test) {
            for (uint32_t j = 0; j < nuse; ++j) {
                const float4 g = s_geo[j];
                const uint32_t mb = (uniform(__builtin_bit_cast(uint32_t, g.w)) >> (2 * h)) & 3u;
                if (!mb) continue;  // scalar: this half's bands are not reached
                const float4 qo = s_quad[j];
                const float4 f = s_rgb[j];
                const uint32_t ipos = __builtin_bit_cast(uint32_t, g.z);
                const Quad q = {qo.x, qo.y, qo.z};
                const float dx = g.x - pxf;
                const float lo = qo.w;
                const ColQuad kq = column_quad(q, dx, lo);
                const float dy0 = g.y - (float)tl.py0;
                f2v s_uy = {0.f, 0.f};
                f2v sc01 = {0.f, 0.f};
                float suyy = 0.f, sc2 = 0.f;
                uint32_t any = 0;
#pragma unroll
                for (int bb = 0; bb < NB; ++bb) {
                    if (!(mb & (1u << bb))) continue;
                    const float dp0b = dp01[bb].x, dp1b = dp01[bb].y, dp2b = dp2[bb];
                    const uint32_t lastb = last[bb];
                    const float dy = dy0 - (float)(4 * (2 * (int)h + bb));
                    const float p2 = falloff_p2(kq, dy);
                    const bool contrib = (decltype(pos_test)::value ? ipos < lastb : true) && p2_in_band(p2, lo);
                    if (!__ballot(contrib)) continue;
                    any |= 1u << bb;
                    const float oG = __builtin_amdgcn_exp2f(contrib ? p2 : -__builtin_inff());
                    const float alpha = fminf(0.99f, oG);
                    const float inv = __builtin_amdgcn_rcpf(1.0f - alpha);
                    T[bb] *= inv;
                    const float Ti = T[bb];
                    const float cdot = __builtin_fmaf(f.x, dp0b, __builtin_fmaf(f.y, dp1b, f.z * dp2b));
                    const float dL_dalpha = __builtin_fmaf(Ti, cdot, -s[bb] * inv);
                    const float wc = alpha * Ti;
                    s[bb] = __builtin_fmaf(cdot, wc, s[bb]);
                    const float u = oG * dL_dalpha;
                    const float uy = u * dy;
                    s_uy += f2v{u, uy};
                    suyy = __builtin_fmaf(uy, dy, suyy);
                    sc01 = __builtin_elementwise_fma(f2v{wc, wc}, dp01[bb], sc01);
                    sc2 = __builtin_fmaf(wc, dp2b, sc2);
                }
                if (!any) continue;
                const float su = s_uy.x, suy = s_uy.y;
                const float sux = su * dx, suxx = sux * dx, suxy = suy * dx;
                float v[8] = {sux, suy, suxx, suxy, suyy, su, sc01.x, sc01.y};
                if constexpr (PAIR) {
                    const bool held = pj != ~0u;  // scalar
                    const uint32_t base = held ? 8u * WS_LDS_STRIDE : 0u;
#pragma unroll
                    for (int k = 0; k < 8; ++k) s_red[base + k * WS_LDS_STRIDE + lane] = v[k];
                    if (!held) {
                        pv8 = sc2;
                        pj = j;
                        continue;
                    }
                    float t8;
                    const float tv = wave_sum9x2_stored(pv8, sc2, lane, s_red, &t8);
                    const bool lead = (lane & 3) == 0;
                    const uint32_t dj = (lane < 32) ? pj : j;
                    if (lead) s_R[h][dj][(lane >> 2) & 7u] = tv;
                    if ((lane & 31) == 1) s_R[h][dj][8] = t8;
                    if ((lane & 31) == 0) s_F[h][dj] = 1u;
                    pj = ~0u;
                    wave_sync();  // the image is rewritten by the next pair
                } else {
                    reduce_store(v, sc2, j);
                }
            }
        };
        if ((uint32_t)(hi - 1) < min_last) instances(std::false_type{});
        else instances(std::true_type{});
        if constexpr (PAIR) {
            if (pj != ~0u) {  // the batch's last contributing instance of this half had no partner
                float v[8];
                wave_sync();
#pragma unroll
                for (int k = 0; k < 8; ++k) v[k] = s_red[k * WS_LDS_STRIDE + lane];
                reduce_store(v, pv8, pj);
                pj = ~0u;
            }
        }
        __syncthreads();  // both halves' rows of the batch are in s_R
        for (uint32_t e = threadIdx.x; e < nuse * (uint32_t)GRAD_ROW; e += 128u) {
            const uint32_t j = e / GRAD_ROW, k = e - j * GRAD_ROW;
            const uint32_t f0 = s_F[0][j], f1 = s_F[1][j];
            if (f0 | f1) {
                const float v = (f0 ? s_R[0][j][k] : 0.f) + (f1 ? s_R[1][j][k] : 0.f);
                const uint32_t slot = __builtin_bit_cast(uint32_t, s_rgb[j].w);
                a.inst_grad[(size_t)slot * GRAD_ROW + k] = v;
                if (k == 0) a.row_valid[slot] = 1;
            }
        }
        __syncthreads();  // the combine's reads are done before the flags are cleared and the next batch is staged
        for (uint32_t j = threadIdx.x; j < nuse; j += 128u) s_F[0][j] = s_F[1][j] = 0u;
    }
}

}  // namespace

#ifdef OMR_STAMPS
int omr_debug_stamps_bwd(uint64_t* dst, size_t bytes)
{
    return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_stamps_bwd), bytes);
}
#endif

#ifdef OMR_BWD_COUNT
extern "C" int omr_debug_bwd_counts(uint64_t* dst, int reset)
{
    int rc = (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_bwd_counts), 5 * sizeof(uint64_t));
    if (reset) {
        const uint64_t z[5] = {0, 0, 0, 0, 0};
        rc |= (int)hipMemcpyToSymbol(HIP_SYMBOL(g_bwd_counts), z, sizeof(z));
    }
    return rc;
}
#endif

int bwd_bands_mode(int mode)
{
    static std::atomic<int> m{[] {
        const char* v = std::getenv("OMR_BWD_BANDS");
        const int b = v ? std::atoi(v) : 0;
        return (b == 2 || b == 4) ? b : 0;
    }()};
    return mode < 0 ? m.load() : m.exchange(mode);
}

// workgroups of `kernel` (block size `threads`) the device holds at once, asked of the runtime; `fallback` per CU
// when it cannot say
template <class K>
static size_t device_resident(K kernel, int threads, int fallback)
{
    int dev = 0, cus = 0, per_cu = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, threads, 0) != hipSuccess || per_cu <= 0)
        per_cu = fallback;
    return (size_t)cus * (size_t)per_cu;
}
struct BwdResident {
    size_t one_wave = 0, two_band = 0;  // render_bwd_kernel<OMR_BWD_BATCH> (one wave), render_bwd2_kernel (128 threads)
};
static const BwdResident& bwd_resident()  // once per device and host thread
{
    static thread_local int cached_dev = -1;
    static thread_local BwdResident r;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    if (dev != cached_dev) {
        r.one_wave = device_resident(render_bwd_kernel<OMR_BWD_BATCH>, 64 * TW_WAVES, 24);
        r.two_band = device_resident(render_bwd2_kernel<TW_BATCH, true>, 128, 0);  // 0 (unknown): units stay sorted
        cached_dev = dev;
    }
    return r;
}
// the two-band kernel runs when every unit fits the resident one-wave workgroups (or OMR_BWD_BANDS=2 forces it)
static bool bwd_two_band(size_t max_units)
{
    const int bands = bwd_bands_mode(-1);
    return bands == 2 || (bands == 0 && max_units <= bwd_resident().one_wave);
}

bool render_backward_needs_order(size_t max_units)
{
    // OMR_BWD_SCHED_SORT=1 / 0 (A/B runs): units longest first always / never
    static const int forced = [] { const char* v = std::getenv("OMR_BWD_SCHED_SORT"); return v ? std::atoi(v) : -1; }();
    if (forced == 0 || forced == 1) return forced == 1;
    return !(bwd_two_band(max_units) && max_units <= bwd_resident().two_band);
}

void launch_render_backward(const RenderBwdArgs& a, size_t max_units, hipStream_t s, hipEvent_t ev_start,
                            hipEvent_t ev_stop)
{
    if (max_units == 0) return;
    // max_units (tiles + L / CKPT + 1) bounds the unit count; it is compared with the one-wave workgroups of the
    // batch-BWD_BATCH kernel the device holds at once (24 per CU on MI355X's 256 CUs: 6144), asked of the runtime once
    // per device
    const size_t RESIDENT = bwd_resident().one_wave;
    auto launch = [&](auto kernel) {
        if (ev_start || ev_stop)
            hipExtLaunchKernelGGL(kernel, dim3((uint32_t)max_units), dim3(64 * TW_WAVES), 0, s, ev_start, ev_stop, 0, a);
        else
            kernel<<<(uint32_t)max_units, 64 * TW_WAVES, 0, s>>>(a);
    };
    // views whose units all fit at once as one-wave workgroups (A, B): two waves per unit, 64-position batches;
    // larger views (C, D, E): one wave per unit and 40-position batches. OMR_BWD_BANDS=4 / 2 (omr_debug_bwd_bands)
    // forces one kernel for A/B runs and tests: 4 = the one-wave kernel with its own batch rule (64 below RESIDENT)
    if (bwd_two_band(max_units)) {
        if (ev_start || ev_stop)
            hipExtLaunchKernelGGL(render_bwd2_kernel<TW_BATCH, true>, dim3((uint32_t)max_units), dim3(128), 0, s, ev_start,
                                  ev_stop, 0, a);
        else
            render_bwd2_kernel<TW_BATCH, true><<<(uint32_t)max_units, 128, 0, s>>>(a);
        return;
    }
    if (max_units > RESIDENT) launch(render_bwd_kernel<OMR_BWD_BATCH>);
    else launch(render_bwd_kernel<TW_BATCH>);
}

}  // namespace omr

// render_fwd.hip — per-tile front-to-back alpha blending, gfx950.
//
// Follows cuda_rasterizer/forward.cu:346-467 (renderCUDA) and :472-590 (renderDepthCUDA): per pixel, walk the
// tile's depth-sorted instances front to back; skip power > 0 and alpha < 1/255; stop (without blending) once
// T * (1 - alpha) < 1e-4; C += feature * alpha * T; record the last contributor; out = C + T * bg.
//
// Structure (MI355X): ONE wave64 per 16x16 tile, four pixels per lane (one per 16x4 band, tile_wave.h).
//  * Batches of 64 instances: each lane reads one point list entry (Gaussian index + the bands its alpha >= 1/255
//    ellipse can reach, computed by emit) and, if it reaches one of the wave's live bands, gathers the Gaussian's
//    64-B render record (raster_common.h) and stages it in LDS at its ballot rank — a compacted, order-preserving
//    list of the batch's useful instances.
//  * The wave then walks that list; for each instance the band mask is wave-uniform (readfirstlane), so
//    unreachable bands cost one scalar branch and reachable ones ~20 VALU per lane.
//  * A band whose 64 pixels are all saturated leaves the active set; the tile exits when none is left.
//  * No workgroup barriers (the block is one wave); XCD-aware tile order (tile_wave.h).
// Results are those of the reference up to the exp implementation (v_exp_f32 on log2(e)-scaled powers).
// HBM per tile instance: 4 (point_list) + 48 of the Gaussian's 64-B record (one random line);
// per pixel: 12 (colour) + 4 (final_T) + 4 (n_contrib) = 20 B written.
#include <algorithm>
#include <cstdlib>

#include "kernels.h"
#include "tile_wave.h"

namespace omr {

namespace {

// bands per wave (NB): 4 = one wave per tile; 2 splits a tile over 2 independent waves (shorter work units for load
// balance and occupancy on views of few tiles; each wave stages the tile's instances itself)
#ifndef OMR_FWD_MINW
#define OMR_FWD_MINW 8
#endif
// OMR_FWD_BATCH: positions staged per batch (<= TW_BATCH; A/B knob)
#ifndef OMR_FWD_BATCH
#define OMR_FWD_BATCH TW_BATCH
#endif
constexpr uint32_t FWD_BATCH = OMR_FWD_BATCH;
static_assert(FWD_BATCH <= (uint32_t)TW_BATCH, "one position per lane");

OMR_STAMP_DECL(g_stamps_fwd)

// diagnostic (A/B only): OMR_FWD_DIAG_EXTRA extra VALU issue slots per evaluated band, to price one VALU op there
#ifndef OMR_FWD_DIAG_EXTRA
#define OMR_FWD_DIAG_EXTRA 0
#endif

template <bool DEPTH, int FWD_BANDS>
__global__ __launch_bounds__(64 * TW_WAVES, OMR_FWD_MINW) void render_fwd_kernel(RenderFwdArgs a)
{
    constexpr uint32_t NG = 4 / FWD_BANDS;  // waves per tile
    __shared__ float4 s_geo_all[TW_WAVES][FWD_BATCH];  // x, y, position in range (u32 bits), band mask (u32 bits)
    __shared__ float4 s_quad_all[TW_WAVES][FWD_BATCH]; // qa, qb, qc, log2(opacity) (tile_wave.h: column_quad)
    __shared__ float4 s_rgb_all[TW_WAVES][FWD_BATCH];  // feature (colour, or depth for DEPTH)

    OMR_STAMP_BEGIN
    const uint32_t wv = threadIdx.x >> 6;
    const uint32_t unit = xcd_remap(blockIdx.x, gridDim.x) * TW_WAVES + wv;
    if (unit >= a.gx * a.gy * NG) return;  // wave-uniform; the block's waves never synchronise
    float4* s_geo = s_geo_all[wv];
    float4* s_quad = s_quad_all[wv];
    float4* s_rgb = s_rgb_all[wv];
    const uint32_t tile = a.tile_order ? a.tile_order[unit / NG] : unit / NG;  // NULL: every workgroup resident at once
    const uint32_t grp = unit % NG;
    const uint32_t band0 = grp * FWD_BANDS;  // this wave's bands: band0 .. band0 + FWD_BANDS - 1
    const TileLane tl(tile, a.gx);
    const uint32_t lane = tl.lane;
    const float pxf = (float)tl.px;
    // read before any store: the compiler cannot prove the stores below miss a.bg and would reload it after each
    const float bg0 = a.bg[0], bg1 = a.bg[1], bg2 = a.bg[2];

    // T carries the pixel's "done" state in its sign: a saturated (or out-of-image) pixel holds -T, so the per-band
    // test is one compare and no bool array lives in VGPRs; |T| is the transmittance
    float T[FWD_BANDS], C0[FWD_BANDS], C1[FWD_BANDS], C2[FWD_BANDS];
    uint32_t last[FWD_BANDS];
    uint32_t active = 0;  // local bands with at least one unsaturated in-image pixel (wave-uniform)
    uint64_t done[FWD_BANDS];  // per band, the lanes whose pixel is done (saturated or outside the image): SGPR masks
    uint32_t work = 0;    // (instance, band) pairs staged for evaluation (omr_debug_tile_cost, bench.py's VALU secondary)
#pragma unroll
    for (int b = 0; b < FWD_BANDS; ++b) {
        const bool inside = tl.px < (uint32_t)a.W && tl.py(band0 + b) < (uint32_t)a.H;
        T[b] = inside ? 1.0f : -1.0f;
        C0[b] = C1[b] = C2[b] = 0.f;
        last[b] = 0;
        done[b] = __ballot(!inside);
        if (~done[b]) active |= 1u << b;
    }

    // a count past the capacity or a failed look-back: the binning kernels did nothing and the ranges stay empty
    const size_t L = binning_count(a.count, a.capacity);
    const uint32_t* point_list = reinterpret_cast<const uint32_t*>(a.binning + canonical_list_offset(L));
    const uint2 range = L ? a.ranges[tile] : make_uint2(0u, 0u);
    const uint32_t n = range.y - range.x;
    // The backward's depth segments (raster_common.h: CKPT): batches never straddle a boundary, and the batch that
    // starts at one stores this wave's pixel states there (T, colour so far). Those stores are straight-line buffer
    // stores issued AFTER the batch's gathers and after the next batch's point-list prefetch (a batch at no boundary
    // stores at an out-of-range offset, which the descriptor's range check drops): vector-memory counters retire in
    // issue order, so no wait for a gather ever includes a checkpoint store.
    const size_t ck_bytes = L ? ckpt_count(L) * BLOCK_SIZE * sizeof(float4) : 0;
    const __amdgpu_buffer_rsrc_t ck_rsrc = __builtin_amdgcn_make_buffer_rsrc(
        a.binning + ckpt_offset(L), (short)0, (int)(uint32_t)ck_bytes, 0x00020000);
    auto batch_end = [&](uint32_t s0) {  // [s0, end): at most FWD_BATCH positions, never past a boundary or n
        const uint32_t nb = (range.x + s0) / CKPT * CKPT + CKPT - range.x;
        return min(min(s0 + FWD_BATCH, n), nb);
    };
    // checkpoint stores of the batch that starts at `start` (OOB offset = dropped); issued as the last vector-memory
    // operations of each batch, and twice after the prologue's prefetch too, so that the loop head sees the same
    // issue pattern from both edges and waits only for the prefetched entry (vmcnt(2)), never for the stores
    auto store_ckpt = [&](uint32_t s0) {
        const uint32_t g0 = range.x + s0;
        const bool at_boundary = s0 > 0 && g0 % CKPT == 0;
        const uint32_t base = at_boundary ? (uint32_t)(((size_t)(g0 / CKPT) * BLOCK_SIZE + band0 * 64 + lane) * 16)
                                          : 0x80000000u;
#pragma unroll
        for (int b = 0; b < FWD_BANDS; ++b)
            __builtin_amdgcn_raw_buffer_store_b128(
                __builtin_bit_cast(v4u, make_float4(fabsf(T[b]), C0[b], C1[b], C2[b])), ck_rsrc,
                base + (uint32_t)(b * 64 * 16), 0, 0);  // distinct offsets even when dropped: no store is merged away
    };
    // point-list entries are loaded one batch ahead, unconditionally (index clamped into the list; lanes past the
    // batch ignore theirs), so no exec-masked write to the prefetch register forces an early wait
    const uint32_t last_idx = L ? (uint32_t)L - 1u : 0u;
    uint32_t start = 0, end = n ? batch_end(0) : 0;
    uint32_t v_next = 0;
    if (n) {
        v_next = point_list[min(range.x + lane, last_idx)];
        store_ckpt(0);  // at_boundary is false for s0 = 0: two dropped stores
    }
    for (; start < n && active;) {
        const uint32_t k = start + lane;
        float4 pos, co, c;
        const uint32_t v = v_next;  // Gaussian index | band mask (emit)
        const uint32_t m = k < end ? (v >> (PL_GID_BITS + band0)) & ((1u << FWD_BANDS) - 1u) & active : 0u;
        if (m) {  // the record is gathered only for an instance that reaches one of this wave's live bands
            const float4* rec = a.splat + (size_t)(v & PL_GID_MASK) * SPLAT_F4;  // one 64-B record
            pos = rec[0];
            co = rec[1];
            c = DEPTH ? make_float4(pos.z, pos.z, pos.z, 0.f) : rec[2];
        }
        const uint32_t next_start = end, next_end = end < n ? batch_end(end) : end;
        v_next = point_list[min(range.x + next_start + lane, last_idx)];
        // the state at a boundary = after every instance in front of it (this batch has not blended yet)
        store_ckpt(start);
        const uint64_t useful = __ballot(m != 0);
        // counted per batch from the staging masks (two scalar ops per instance less in the blend loop); a band that
        // saturates inside the batch is still counted for the batch's later instances
#pragma unroll
        for (int b = 0; b < FWD_BANDS; ++b) work += (uint32_t)__popcll(__ballot((m >> b) & 1u));
        if (m != 0) {
            const uint32_t r = mask_rank(useful);
            const Quad q = quad_of_conic(co);
            s_geo[r] = make_float4(pos.x, pos.y, __builtin_bit_cast(float, k), __builtin_bit_cast(float, m));
            s_quad[r] = make_float4(q.qa, q.qb, q.qc, p2_log2o(co.w));
            s_rgb[r] = c;
        }
        wave_sync();  // orders this wave's LDS stores before its reads below
        const uint32_t cnt = (uint32_t)__popcll(useful);
        for (uint32_t j = 0; j < cnt; ++j) {
            const float4 g = s_geo[j], qo = s_quad[j], f = s_rgb[j];
            const uint32_t mb = uniform(__builtin_bit_cast(uint32_t, g.w)) & active;
            const uint32_t contributor = __builtin_bit_cast(uint32_t, g.z) + 1u;
            const Quad q = {qo.x, qo.y, qo.z};
            const float lo = qo.w;
            const float dx = g.x - pxf;
            const ColQuad kq = column_quad(q, dx, lo);
            // dy as the backward forms it (render_bwd.hip): from the tile's first pixel row, then minus 4 x the band,
            // so both kernels round dy — and take every contribute / skip decision — identically
            const float dy0 = g.y - (float)tl.py0;
            uint64_t sat_any = 0;  // lanes that saturated at this instance (a wave mask: SALU only)
            // one band of the wave (the reference's per-pixel loop body, forward.cu:428-455)
            auto band = [&](const int b) {
                const float dy = dy0 - (float)(4 * (band0 + b));
                const float p2 = falloff_p2(kq, dy);
                // a done pixel (T < 0) may evaluate: its test_T is negative, so sat holds, wgt = 0, T keeps -|T| and
                // `last` stays (wgt > 0 below) — the same results with one scalar AND less per band
                const bool ok = p2_in_band(p2, lo);  // power <= 0, alpha >= 1/255 (tile_wave.h)
                // a lane that is not ok gets alpha = 0: test_T = T, wgt = 0; v_exp_f32 returns o G (column_quad)
                const float alpha = fminf(0.99f, __builtin_amdgcn_exp2f(ok ? p2 : -__builtin_inff()));
                const float aT = alpha * T[b];
                const float test_T = T[b] * (1.0f - alpha);
                // a live T is >= 1e-4 (T only takes values that passed this test) and a lane that is not ok has
                // test_T = T, so `sat` holds for newly saturated and already done (negative) pixels alike
                const bool sat = test_T < 0.0001f;
                // the done lanes are exactly the sat ones from here on: a mask OR on the scalar unit tracks them
                // (a ballot of a plain compare stays in SGPRs), no per-band compare of T's sign
                const uint64_t satm = __ballot(sat);
                sat_any |= satm & ~done[b];  // newly saturated lanes
                done[b] |= satm;
                const float wgt = sat ? 0.0f : aT;
                C0[b] = __builtin_fmaf(f.x, wgt, C0[b]);
                C1[b] = __builtin_fmaf(f.y, wgt, C1[b]);
                C2[b] = __builtin_fmaf(f.z, wgt, C2[b]);
                T[b] = sat ? -fabsf(T[b]) : test_T;  // done: keeps the last live T, negated
                // blended iff ok and not sat (alpha >= 1/255, T >= 1e-4: wgt > 0); a done lane is sat. Both are compare
                // masks already, so this is a scalar and-not, not a third vector compare
                last[b] = (ok && !sat) ? contributor : last[b];
#if OMR_FWD_DIAG_EXTRA
#pragma unroll
                for (int e = 0; e < OMR_FWD_DIAG_EXTRA; ++e) asm volatile("v_mov_b32 %0, %0" : "+v"(C2[b]));
#endif
            };
#pragma unroll
            for (int b = 0; b < FWD_BANDS; ++b) {
                if (!(mb & (1u << b))) continue;  // scalar branch
                band(b);
            }
            if (sat_any) {  // some pixel saturated: drop bands with no live pixel left
#pragma unroll
                for (int b = 0; b < FWD_BANDS; ++b)
                    if (!~done[b]) active &= ~(1u << b);
                if (!active) break;
            }
        }
        wave_sync();  // the next batch overwrites the staging arrays
        start = next_start;
        end = next_end;
    }

    const size_t plane = (size_t)a.H * a.W;
    uint32_t maxc = 0;
#pragma unroll
    for (int b = 0; b < FWD_BANDS; ++b) {
        const uint32_t py = tl.py(band0 + b);
        maxc = max(maxc, last[b]);
        if (tl.px < (uint32_t)a.W && py < (uint32_t)a.H) {
            const uint32_t pix = a.W * py + tl.px;
            const float Tf = fabsf(T[b]);
            a.final_T[pix] = Tf;
            a.n_contrib[pix] = last[b];
            a.final_C[pix] = C0[b];
            a.final_C[plane + pix] = C1[b];
            a.final_C[2 * plane + pix] = C2[b];
            a.out_color[pix] = C0[b] + Tf * bg0;
            a.out_color[plane + pix] = C1[b] + Tf * bg1;
            a.out_color[2 * plane + pix] = C2[b] + Tf * bg2;
        }
    }
    maxc = wave_max_u32(maxc);
    if (lane == 0) a.max_contrib[(size_t)tile * FWD_GROUPS + grp] = maxc;
    // the slots no wave of this tile writes (NG < FWD_GROUPS) are cleared by its first wave
    if (grp == 0 && lane >= NG && lane < (uint32_t)FWD_GROUPS) a.max_contrib[(size_t)tile * FWD_GROUPS + lane] = 0u;
    if (lane == 0 && work) atomicAdd(&a.tile_cost[tile], work);
    // The backward's row_valid map is zeroed here, one slice per wave with 16-B stores after the wave's image stores, in
    // the shadow of the VALU-bound blend, rather than by the binning's latency-bound scatter loop (one byte store per
    // instance there: config E tile sort 1.090 -> 1.044 ms, C and A unchanged, profiles/r04p_ab_*.txt)
    if (L) {  // raster_common.h: row_valid_offset, align_up(L) bytes
        uint4* rv = reinterpret_cast<uint4*>(a.binning + row_valid_offset(L));
        const uint32_t n16 = (uint32_t)(align_up(L) / sizeof(uint4)), nw = a.gx * a.gy * NG;
        const uint32_t per = (n16 + nw - 1u) / nw, span = (per + 63u) & ~63u;
        const uint32_t b0 = unit * span, b1 = min(b0 + span, n16);
        for (uint32_t i = b0 + lane; i < b1; i += 64u) rv[i] = make_uint4(0u, 0u, 0u, 0u);
    }
    OMR_STAMP_END(g_stamps_fwd, unit);
}

}  // namespace

// bands per wave by view: one (four waves per tile) up to FWD_FOUR_WAVE_TILES tiles, where two bands would give at
// most two waves per SIMD (config A: render_fwd 12.4 -> 10.9 us; at B, 2048 tiles, one band is slower: 40.4 vs
// 38.5 us; profiles/r06j_ab_{A,B}.txt), two below FWD_ONE_WAVE_TILES, four from there; OMR_FWD_BANDS=1|2|4 forces
static int forward_bands(uint32_t T)
{
    static const int forced = [] { const char* v = std::getenv("OMR_FWD_BANDS"); return v ? std::atoi(v) : 0; }();
    if (forced == 1 || (forced == 0 && T <= FWD_FOUR_WAVE_TILES)) return 1;
    if (forced == 4 || (forced != 2 && T >= FWD_ONE_WAVE_TILES)) return 4;
    return 2;
}

bool render_forward_needs_order(uint32_t T)
{
    // OMR_FWD_TILE_ORDER=1 / 0 (A/B runs): the longest-first order always / never
    static const int forced = [] { const char* v = std::getenv("OMR_FWD_TILE_ORDER"); return v ? std::atoi(v) : -1; }();
    if (forced == 0 || forced == 1) return forced == 1;
    // at most two waves per SIMD (config A, 512 tiles x 4 waves): all start at once and none shares its SIMD with
    // more than one other, so the order changes nothing and its launch is saved (A 896 -> 962 MP/s with the backward
    // schedule's sort also skipped). At B (4 waves per SIMD) the order still spreads the heavy tiles over the SIMDs:
    // render_fwd 36.9 vs 42.8 us without it (profiles/r06p_ab_{A,B}.txt)
    static thread_local int cached_dev = -1;
    static thread_local size_t simds = 0;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    if (dev != cached_dev) {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 0;
        simds = 4 * (size_t)std::max(cus, 0);  // 0 (unknown): the order is kept
        cached_dev = dev;
    }
    return (size_t)T * (size_t)(4 / forward_bands(T)) > 2 * simds;
}

void launch_render_forward(const RenderFwdArgs& a, bool depth_mode, hipStream_t s)
{
    const uint32_t T = a.gx * a.gy;
    if (T == 0) return;
    const int bands = forward_bands(T);
    if (bands == 1) {
        const uint32_t blocks = div_up(T * 4, TW_WAVES);
        if (depth_mode) render_fwd_kernel<true, 1><<<blocks, 64 * TW_WAVES, 0, s>>>(a);
        else render_fwd_kernel<false, 1><<<blocks, 64 * TW_WAVES, 0, s>>>(a);
        return;
    }
    if (bands == 4) {
        const uint32_t blocks = div_up(T, TW_WAVES);
        if (depth_mode) render_fwd_kernel<true, 4><<<blocks, 64 * TW_WAVES, 0, s>>>(a);
        else render_fwd_kernel<false, 4><<<blocks, 64 * TW_WAVES, 0, s>>>(a);
    } else {
        const uint32_t blocks = div_up(T * 2, TW_WAVES);
        if (depth_mode) render_fwd_kernel<true, 2><<<blocks, 64 * TW_WAVES, 0, s>>>(a);
        else render_fwd_kernel<false, 2><<<blocks, 64 * TW_WAVES, 0, s>>>(a);
    }
}

#ifdef OMR_STAMPS
extern "C" int omr_debug_stamps(int which, uint64_t* dst, int n)
{
    const size_t bytes = (size_t)std::min(n, STAMP_CAP) * 4 * sizeof(uint64_t);
    return which == 0 ? (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_stamps_fwd), bytes)
                      : (int)omr_debug_stamps_bwd(dst, bytes);
}
#endif

}  // namespace omr

// render_bwd.hip — per-tile back-to-front gradient replay, gfx950.
//
// Follows cuda_rasterizer/backward.cu:671-843 (renderCUDA backward) for the per-pixel arithmetic: T is
// recovered by division, accum_rec / last_alpha / last_color carry the colour behind each instance, and the
// background term uses T_final.
//
// What is different, and why (MI355X):
//  * The reference issues 9 float atomicAdds per contributing (pixel, Gaussian) pair into per-Gaussian
//    arrays. On MI355X float atomics run at ~1.3 TB/s chip-wide and ~17x slower still when the 64 lanes of
//    an instruction hit 64 different rows (MI355X_MICROARCH.md, Global float atomics) — that would bound the
//    kernel. Here each wave64 sums its 64 pixels' 9 gradient values in registers: a transposed butterfly
//    inside each 16-lane DPP row (8 values in 22 DPP-fused VALU ops: each step halves the values a lane
//    holds), then v_permlane16_swap / v_permlane32_swap across rows (gfx950). The 4 waves' partials are
//    combined in LDS and ONE 36-B row per (tile, Gaussian) instance is stored with plain stores, indexed by
//    the instance's emission slot; gaussian_bwd.hip sums each Gaussian's rows in a fixed order. No atomics:
//    gradients are bitwise reproducible run to run.
//  * Per pair the math is predicated (no divergent branches), T is recovered with v_rcp_f32 instead of an
//    IEEE division sequence, and each wave walks only the instances whose alpha >= 1/255 ellipse reaches
//    its 16x4 band (band_mask) and that lie in front of some pixel's last contributor: every staged batch
//    is compacted into one ordered list per wave (band_lists.h). Built with FMA contraction.
//  * Instances behind the last contributor of every pixel in the tile are skipped (their rows zero-filled).
//  * XCD-aware tile order, as in the forward.
#include "band_lists.h"
#include "kernels.h"
#include "wave_ops.h"

namespace omr {

namespace {

constexpr int BATCH = 128;
constexpr int WAVES = BLOCK_SIZE / 64;

__device__ __forceinline__ uint32_t xcd_remap(uint32_t orig, uint32_t nwg)
{
    const uint32_t q = nwg / 8, r = nwg % 8, xcd = orig % 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

__device__ __forceinline__ uint32_t block_max(uint32_t v, uint32_t* s_tmp)
{
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o, 64));
    if ((threadIdx.x & 63) == 0) s_tmp[threadIdx.x >> 6] = v;
    __syncthreads();
    uint32_t m = s_tmp[0];
#pragma unroll
    for (int k = 1; k < WAVES; ++k) m = max(m, s_tmp[k]);
    __syncthreads();
    return m;
}


__global__ __launch_bounds__(BLOCK_SIZE) void render_bwd_kernel(RenderBwdArgs a)
{
    __shared__ float2 s_xy[BATCH];
    __shared__ float4 s_co[BATCH];
    __shared__ float4 s_rgb[BATCH];
    __shared__ uint32_t s_slot[BATCH];
    __shared__ uint32_t s_mask[BATCH];
    __shared__ float s_part[WAVES][BATCH][GRAD_ROW];
    __shared__ BandLists<BATCH> s_lists;
    __shared__ uint32_t s_tmp[WAVES];
    __shared__ uint32_t s_wave_max_c[WAVES];

    const uint32_t tile = xcd_remap(blockIdx.x, gridDim.x);
    const uint32_t tx = tile % a.gx, ty = tile / a.gx;
    const uint32_t t = threadIdx.x;
    const uint32_t lane = t & 63, w = t >> 6;
    const uint32_t px = tx * BLOCK_X + (t & (BLOCK_X - 1));
    const uint32_t py = ty * BLOCK_Y + (t / BLOCK_X);
    const bool inside = px < (uint32_t)a.W && py < (uint32_t)a.H;
    const uint32_t pix_id = a.W * py + px;
    const float pxf = (float)px, pyf = (float)py;
    const size_t plane = (size_t)a.H * a.W;

    const uint2 range = a.ranges[tile];
    const uint32_t n = range.y - range.x;
    const float T_final = inside ? a.final_T[pix_id] : 0.f;
    const uint32_t last_contributor = inside ? a.n_contrib[pix_id] : 0u;
    float dpix0 = 0.f, dpix1 = 0.f, dpix2 = 0.f;
    if (inside) {
        dpix0 = a.dL_dpix[pix_id];
        dpix1 = a.dL_dpix[plane + pix_id];
        dpix2 = a.dL_dpix[2 * plane + pix_id];
    }
    const float bg_dot = a.bg[0] * dpix0 + a.bg[1] * dpix1 + a.bg[2] * dpix2;
    const float ddelx_dx = (float)(0.5 * a.W);
    const float ddely_dy = (float)(0.5 * a.H);
    // lane (l < 9) of a wave writes value slot slot_of_lane of the wave partial
    const uint32_t slot_of_lane = transposed_slot_of_lane(lane);

    // positions >= wave_max_c are behind the last contributor of every pixel of the wave
    uint32_t wave_max_c = last_contributor;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) wave_max_c = max(wave_max_c, (uint32_t)__shfl_xor((int)wave_max_c, o, 64));
    if (lane == 0) s_wave_max_c[w] = wave_max_c;
    // instances at positions >= max_c are behind every pixel's last contributor
    const uint32_t max_c = min(n, block_max(last_contributor, s_tmp));  // (its barriers publish s_wave_max_c)

    for (uint32_t k = max_c + t; k < n; k += BLOCK_SIZE) {
        const float4* rec = a.splat + (size_t)a.point_list[range.x + k] * SPLAT_F4;
        float* row = a.inst_grad + (size_t)splat_slot(rec[0], rec[2], tx, ty) * GRAD_ROW;
#pragma unroll
        for (int c = 0; c < GRAD_ROW; ++c) row[c] = 0.f;
    }

    float T = T_final;
    float acc0 = 0.f, acc1 = 0.f, acc2 = 0.f;  // accum_rec
    float last_alpha = 0.f;
    float lc0 = 0.f, lc1 = 0.f, lc2 = 0.f;  // last_color

    // walk positions max_c-1 .. 0 in batches of BATCH, back to front
    for (int hi = (int)max_c; hi > 0; hi -= BATCH) {
        const int lo = max(0, hi - BATCH);
        const int cnt = hi - lo;
        // batch entry j <-> position hi-1-j
        uint32_t m = 0;
        if ((int)t < cnt) {
            const uint32_t pos = (uint32_t)(hi - 1 - (int)t);
            const float4* rec = a.splat + (size_t)a.point_list[range.x + pos] * SPLAT_F4;  // one 64-B line
            const float4 p = rec[0];
            const float4 co = rec[1];
            const float4 c = rec[2];
            const float2 xy = {p.x, p.y};
            s_xy[t] = xy;
            s_co[t] = co;
            s_rgb[t] = c;
            s_slot[t] = splat_slot(p, c, tx, ty);
            m = band_mask(xy, co, tx, ty);
#pragma unroll
            for (int b = 0; b < WAVES; ++b)
                if (pos >= s_wave_max_c[b]) m &= ~(1u << b);
            s_mask[t] = m;
        }
        s_lists.build(m, t);
        const uint32_t lcnt = s_lists.count(w);
        const uint8_t* list = s_lists.idx[w];
        for (uint32_t k4 = 0; k4 < lcnt; k4 += 4) {
            const uint32_t packed = *reinterpret_cast<const uint32_t*>(list + k4);
#pragma unroll
            for (uint32_t u = 0; u < 4; ++u) {
                if (k4 + u >= lcnt) break;
                const uint32_t j = (packed >> (8 * u)) & 0xffu;
                const uint32_t pos = (uint32_t)(hi - 1) - j;
                float* part = s_part[w][j];
                const float2 xy = s_xy[j];
                const float4 co = s_co[j];
                const float dx = xy.x - pxf, dy = xy.y - pyf;
                const float power = -0.5f * (co.x * dx * dx + co.z * dy * dy) - co.y * dx * dy;
                const float G = __expf(power);
                const float alpha = fminf(0.99f, co.w * G);
                // reference: skip if contributor >= last_contributor, power > 0 or alpha < 1/255
                const bool contrib = pos < last_contributor && power <= 0.0f && alpha >= 1.0f / 255.0f;
                if (__ballot(contrib) == 0ull) {
                    if (lane < GRAD_ROW) part[lane] = 0.f;
                    continue;
                }
                const float4 c = s_rgb[j];
                const float inv = __builtin_amdgcn_rcpf(1.f - alpha);
                const float Tn = T * inv;
                const float dchannel_dcolor = alpha * Tn;
                const float n0 = last_alpha * lc0 + (1.f - last_alpha) * acc0;
                const float n1 = last_alpha * lc1 + (1.f - last_alpha) * acc1;
                const float n2 = last_alpha * lc2 + (1.f - last_alpha) * acc2;
                float dL_dalpha = ((c.x - n0) * dpix0 + (c.y - n1) * dpix1 + (c.z - n2) * dpix2) * Tn;
                dL_dalpha += (-T_final * inv) * bg_dot;
                const float dL_dG = co.w * dL_dalpha;
                const float gdx = G * dx;
                const float gdy = G * dy;
                float v[8];
                v[0] = dL_dG * (-gdx * co.x - gdy * co.y) * ddelx_dx;
                v[1] = dL_dG * (-gdy * co.z - gdx * co.y) * ddely_dy;
                v[2] = -0.5f * gdx * dx * dL_dG;
                v[3] = -0.5f * gdx * dy * dL_dG;
                v[4] = -0.5f * gdy * dy * dL_dG;
                v[5] = G * dL_dalpha;
                v[6] = dchannel_dcolor * dpix0;
                v[7] = dchannel_dcolor * dpix1;
                float v8 = dchannel_dcolor * dpix2;
#pragma unroll
                for (int q = 0; q < 8; ++q) v[q] = contrib ? v[q] : 0.f;
                v8 = contrib ? v8 : 0.f;
                T = contrib ? Tn : T;
                acc0 = contrib ? n0 : acc0;
                acc1 = contrib ? n1 : acc1;
                acc2 = contrib ? n2 : acc2;
                lc0 = contrib ? c.x : lc0;
                lc1 = contrib ? c.y : lc1;
                lc2 = contrib ? c.z : lc2;
                last_alpha = contrib ? alpha : last_alpha;
                float t8;
                const float tv = wave_sum8_transposed(v, v8, lane, &t8);
                if (lane < GRAD_ROW) part[slot_of_lane] = lane < 8 ? tv : t8;
            }
        }
        __syncthreads();
        // one row per instance: the sum of the partials of the waves whose list held it
        if ((int)t < cnt) {
            const uint32_t mt = s_mask[t];
            float* row = a.inst_grad + (size_t)s_slot[t] * GRAD_ROW;
#pragma unroll
            for (int c = 0; c < GRAD_ROW; ++c) {
                float v = 0.f;
#pragma unroll
                for (int q = 0; q < WAVES; ++q) v += (mt >> q) & 1u ? s_part[q][t][c] : 0.f;
                row[c] = v;
            }
        }
        __syncthreads();
    }
}

}  // namespace

void launch_render_backward(const RenderBwdArgs& a, hipStream_t s)
{
    const uint32_t T = a.gx * a.gy;
    if (T == 0) return;
    render_bwd_kernel<<<T, BLOCK_SIZE, 0, s>>>(a);
}

}  // namespace omr

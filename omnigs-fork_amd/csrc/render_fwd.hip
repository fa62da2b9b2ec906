// render_fwd.hip — per-tile front-to-back alpha blending, gfx950.
//
// Follows cuda_rasterizer/forward.cu:346-467 (renderCUDA) and :472-590 (renderDepthCUDA): one 16x16 tile per
// 256-thread workgroup (four wave64s, each 16 px x 4 rows), one pixel per thread, instances of the tile's
// sorted range fetched 256 at a time into LDS, block-vote early exit when every pixel saturated.
//
// Differences from the reference kernel (results identical up to the exp() implementation):
//  * the colour of each instance is staged in LDS with its centre and conic (the reference re-reads
//    features[] from global memory inside the per-pixel loop, forward.cu:447-448);
//  * blockIdx is remapped so that consecutive tiles (which share most of their Gaussians) run on the same
//    XCD and hit the same L2 (MI355X: 8 XCDs, blocks b and b+8 share one);
//  * exp uses the hardware v_exp_f32 path (__expf);
//  * each staged instance carries a 4-bit mask of the 16x4 wave bands its alpha >= 1/255 ellipse reaches
//    (band_mask, raster_common.h); the batch is compacted into one ordered list per band (band_lists.h) and
//    each wave walks only its own list, four instances per step with predicated (branch-free) blending.
// HBM per tile instance: 4 (point_list) + 40 of the Gaussian's 64-B render record (xy, conic/opacity, rgb:
// one random line, raster_common.h) gathered;
// per pixel: 12 (colour) + 4 (final_T) + 4 (n_contrib) = 20 B written.
#include "band_lists.h"
#include "kernels.h"

namespace omr {

namespace {

// bijective XCD-aware remap: blocks that share an XCD (orig % 8 equal) get consecutive logical ids
__device__ __forceinline__ uint32_t xcd_remap(uint32_t orig, uint32_t nwg)
{
    const uint32_t q = nwg / 8, r = nwg % 8, xcd = orig % 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

template <bool DEPTH>
__global__ __launch_bounds__(BLOCK_SIZE) void render_fwd_kernel(RenderFwdArgs a)
{
    __shared__ float2 s_xy[BLOCK_SIZE];
    __shared__ float4 s_co[BLOCK_SIZE];
    __shared__ float4 s_rgb[BLOCK_SIZE];
    __shared__ BandLists<BLOCK_SIZE> s_lists;

    const uint32_t tile = xcd_remap(blockIdx.x, gridDim.x);
    const uint32_t tx = tile % a.gx, ty = tile / a.gx;
    const uint32_t t = threadIdx.x;
    const uint32_t w = t >> 6;
    const uint32_t px = tx * BLOCK_X + (t & (BLOCK_X - 1));
    const uint32_t py = ty * BLOCK_Y + (t / BLOCK_X);
    const bool inside = px < (uint32_t)a.W && py < (uint32_t)a.H;
    const uint32_t pix_id = a.W * py + px;
    const float pxf = (float)px, pyf = (float)py;

    const uint2 range = a.ranges[tile];
    const int n = (int)(range.y - range.x);
    bool done = !inside;
    float T = 1.0f;
    float C0 = 0.f, C1 = 0.f, C2 = 0.f;
    uint32_t last_contributor = 0;

    for (int start = 0; start < n; start += BLOCK_SIZE) {
        if (__syncthreads_count(done) == BLOCK_SIZE) break;
        const int k = start + (int)t;
        uint32_t m = 0;
        if (k < n) {
            const uint32_t gid = a.point_list[range.x + k];
            const float4* rec = a.splat + (size_t)gid * SPLAT_F4;  // one 64-B record per instance
            const float4 pos = rec[0];
            const float4 co = rec[1];
            const float2 xy = {pos.x, pos.y};
            s_xy[t] = xy;
            s_co[t] = co;
            m = band_mask(xy, co, tx, ty);
            if (DEPTH) {
                s_rgb[t] = make_float4(pos.z, pos.z, pos.z, 0.f);
            } else {
                s_rgb[t] = rec[2];
            }
        }
        s_lists.build(m, t);
        // this wave's instances, in front-to-back order, 4 per step; the math is predicated (no per-lane
        // branches): a lane that is done, or an entry past the end of the list, changes nothing
        const uint32_t cnt = s_lists.count(w);
        const uint8_t* list = s_lists.idx[w];
        for (uint32_t k4 = 0; k4 < cnt; k4 += 4) {
            if (__ballot(!done) == 0ull) break;  // every pixel of the wave saturated
            const uint32_t packed = *reinterpret_cast<const uint32_t*>(list + k4);
#pragma unroll
            for (uint32_t u = 0; u < 4; ++u) {
                const uint32_t j = (packed >> (8 * u)) & 0xffu;
                const float2 xy = s_xy[j];
                const float4 co = s_co[j];
                const float4 c = s_rgb[j];
                const float dx = xy.x - pxf, dy = xy.y - pyf;
                const float power = -0.5f * (co.x * dx * dx + co.z * dy * dy) - co.y * dx * dy;
                const float alpha = fminf(0.99f, co.w * __expf(power));
                // forward.cu:424-452: skip power > 0 and alpha < 1/255; stop (without blending) when
                // T * (1 - alpha) < 1e-4
                bool ok = !done && k4 + u < cnt && power <= 0.0f && alpha >= 1.0f / 255.0f;
                const float test_T = T * (1.0f - alpha);
                const bool sat = ok && test_T < 0.0001f;
                done = done || sat;
                ok = ok && !sat;
                // selects, not multiplies by 0: entries past the end of the list may hold stale LDS words
                const float wgt = alpha * T;
                C0 = ok ? C0 + c.x * wgt : C0;
                C1 = ok ? C1 + c.y * wgt : C1;
                C2 = ok ? C2 + c.z * wgt : C2;
                T = ok ? test_T : T;
                last_contributor = ok ? (uint32_t)(start + (int)j + 1) : last_contributor;
            }
        }
    }
    if (inside) {
        a.final_T[pix_id] = T;
        a.n_contrib[pix_id] = last_contributor;
        const size_t plane = (size_t)a.H * a.W;
        a.out_color[pix_id] = C0 + T * a.bg[0];
        a.out_color[plane + pix_id] = C1 + T * a.bg[1];
        a.out_color[2 * plane + pix_id] = C2 + T * a.bg[2];
    }
}

}  // namespace

void launch_render_forward(const RenderFwdArgs& a, bool depth_mode, hipStream_t s)
{
    const uint32_t T = a.gx * a.gy;
    if (T == 0) return;
    if (depth_mode) render_fwd_kernel<true><<<T, BLOCK_SIZE, 0, s>>>(a);
    else render_fwd_kernel<false><<<T, BLOCK_SIZE, 0, s>>>(a);
}

}  // namespace omr

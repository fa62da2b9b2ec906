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
//    (band_mask, raster_common.h); a wave skips instances outside its band with one uniform branch.
// HBM per tile instance: 4 (point_list) + 8 (xy) + 16 (conic/opacity) + 16 (rgb) = 44 B gathered;
// per pixel: 12 (colour) + 4 (final_T) + 4 (n_contrib) = 20 B written.
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
    __shared__ uint32_t s_mask[BLOCK_SIZE];

    const uint32_t tile = xcd_remap(blockIdx.x, gridDim.x);
    const uint32_t tx = tile % a.gx, ty = tile / a.gx;
    const uint32_t t = threadIdx.x;
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
    const uint32_t wave_bit = 1u << (t >> 6);

    for (int start = 0; start < n; start += BLOCK_SIZE) {
        if (__syncthreads_count(done) == BLOCK_SIZE) break;
        const int k = start + (int)t;
        if (k < n) {
            const uint32_t gid = a.point_list[range.x + k];
            const float2 xy = a.means2D[gid];
            const float4 co = a.conic_opacity[gid];
            s_xy[t] = xy;
            s_co[t] = co;
            s_mask[t] = band_mask(xy, co, tx, ty);
            if (DEPTH) {
                const float d = a.depths[gid];
                s_rgb[t] = make_float4(d, d, d, 0.f);
            } else {
                s_rgb[t] = a.rgb[gid];
            }
        }
        __syncthreads();
        const int cnt = min(BLOCK_SIZE, n - start);
        for (int j = 0; !done && j < cnt; ++j) {
            if (!(s_mask[j] & wave_bit)) continue;  // wave-uniform: no pixel of this wave can be reached
            const float2 xy = s_xy[j];
            const float4 co = s_co[j];
            const float dx = xy.x - pxf, dy = xy.y - pyf;
            const float power = -0.5f * (co.x * dx * dx + co.z * dy * dy) - co.y * dx * dy;
            if (power > 0.0f) continue;
            const float alpha = fminf(0.99f, co.w * __expf(power));
            if (alpha < 1.0f / 255.0f) continue;
            const float test_T = T * (1.0f - alpha);
            if (test_T < 0.0001f) {
                done = true;
                continue;
            }
            const float4 c = s_rgb[j];
            const float w = alpha * T;
            C0 += c.x * w;
            C1 += c.y * w;
            C2 += c.z * w;
            T = test_T;
            last_contributor = (uint32_t)(start + j + 1);  // the reference's running contributor count
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

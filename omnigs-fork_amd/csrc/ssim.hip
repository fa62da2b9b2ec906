// ssim.hip — the training loss of OmniGS, (1 - lambda) * L1 + lambda * (1 - SSIM), forward AND backward in one
// pass over the image, gfx950.
//
// Reference: include/loss_utils.h:31-129 (l1_loss, gaussian, create_window, _ssim, ssim) as used by
// gaussian_trainer.cpp:88-90 / gaussian_mapper.cpp:403-412: SSIM with an 11x11 Gaussian window (sigma 1.5,
// normalised 1-D window, outer product), zero padding 5, per channel (depthwise conv2d over [C,H,W]), C1 = 0.01^2,
// C2 = 0.03^2, mean over all C*H*W entries; L1 = mean |img - gt|. The reference runs five 11x11 depthwise
// convolutions forward and autograd's transposed convolutions backward.
//
// Here dL/dS = -lambda / (C H W) is a constant, so the gradient does not wait for the loss value and one kernel
// does both. Per 16x16 output tile and channel (256 threads): the 36x36 input halo of img and gt is staged in LDS;
// the five moments E[x], E[y], E[x^2], E[y^2], E[xy] are filtered separably (11 + 11 taps instead of 121) on the
// 26x26 region whose SSIM values feed the tile's gradient; SSIM and its partials
//     A = dS/dmu1, B = dS/dE[x^2], C = dS/dE[xy]   (sigma terms folded in)
// are formed there (zero where the output pixel is outside the image), filtered back separably, and
//     dL/dx = dL/dS (G * A + 2 x G * B + y G * C) + (1 - lambda) sign(x - y) / (C H W).
// Per-block partial sums of S and |x - y| go to scratch; loss_finish_kernel adds them in a fixed order, so the loss
// is deterministic. HBM: reads img and gt once (plus halo), writes dL/dimg once: 12 B per pixel-channel.
//
// Both kernels (tiled, streaming) sum every filter's taps in the same order with fused multiply-adds and form SSIM
// and its partials with the same helper (ssim_partials), so their dL/dimg is bitwise identical
// (tests/test_gpu_losses.py). The streaming kernel runs the x | y and x^2 | y^2 taps as packed FMAs.
#include <algorithm>
#include <atomic>
#include <cmath>

#include "kernels.h"
#include "tile_wave.h"

namespace omr {

namespace {

constexpr int SS_TILE = 16;
constexpr int SS_HALO = 5;
constexpr int SS_WIN = 2 * SS_HALO + 1;
constexpr int SS_R1 = SS_TILE + 2 * SS_HALO;  // 26: SSIM values feeding the tile's gradient
constexpr int SS_R2 = SS_R1 + 2 * SS_HALO;    // 36: input region
constexpr float SS_C1 = 0.01f * 0.01f;
constexpr float SS_C2 = 0.03f * 0.03f;

// 0: by image size, 1: tiled, 2: streaming (omr_debug_ssim_mode: tests run both kernels on the same images)
std::atomic<int> g_ssim_mode{0};

// SSIM at one position from its five local moments E[x], E[y], E[x^2], E[y^2], E[xy], and its partials times dL/dS
//   A = dS/dmu1, B = dS/dE[x^2], C = dS/dE[xy] (zero outside the image: the zero padding's positions have no SSIM)
// One reciprocal (v_rcp_f32, 1 ulp) for the three quotients: den = a2 b2 >= C1 C2 > 0; 1 / b2 = a2 / den.
struct SsimPart {
    float S, A, B, C;
};
__device__ __forceinline__ SsimPart ssim_partials(float mu1, float mu2, float exx, float eyy, float exy, float dS,
                                                  bool in)
{
    const float mu1_sq = mu1 * mu1, mu2_sq = mu2 * mu2, mu1_mu2 = mu1 * mu2;
    const float s11 = exx - mu1_sq, s22 = eyy - mu2_sq, s12 = exy - mu1_mu2;
    const float a1 = 2.f * mu1_mu2 + SS_C1, b1 = 2.f * s12 + SS_C2;
    const float a2 = mu1_sq + mu2_sq + SS_C1, b2 = s11 + s22 + SS_C2;
    const float inv = __builtin_amdgcn_rcpf(a2 * b2);
    SsimPart p;
    p.S = (a1 * b1) * inv;
    p.A = in ? dS * ((2.f * mu2 * (b1 - a1)) * inv - p.S * (2.f * mu1 * (b2 - a2)) * inv) : 0.f;
    p.B = in ? dS * (-p.S * (a2 * inv)) : 0.f;
    p.C = in ? dS * (2.f * a1 * inv) : 0.f;
    return p;
}
// dL/dimg at one pixel from its back-filtered partials: dL/dS (G*A + 2 x G*B + y G*C) + (1 - lambda) sign(x - y) / n
__device__ __forceinline__ float ssim_pixel_grad(float fa, float fb, float fc, float x, float y, float l1_scale)
{
    const float d = x - y;
    const float sgn = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);  // torch.abs backward: sign(0) = 0
    return fa + 2.f * x * fb + y * fc + l1_scale * sgn;
}

__global__ __launch_bounds__(256) void l1_ssim_kernel(const float* img, const float* gt, int H, int W, SsimWindow win,
                                                      float l1_scale, float dS_scale, float* dimg, float* partials)
{
    __shared__ float s_x[SS_R2][SS_R2 + 1];
    __shared__ float s_y[SS_R2][SS_R2 + 1];
    __shared__ float s_h[5][SS_R2][SS_R1];  // horizontal pass of x, y, xx, yy, xy; later of A, B, C
    __shared__ float s_m[5][SS_R1][SS_R1];  // moments; later A, B, C
    __shared__ float s_red[2][4];
    const int t = threadIdx.x;
    const int ch = blockIdx.z;
    const int ox = blockIdx.x * SS_TILE, oy = blockIdx.y * SS_TILE;
    const size_t plane = (size_t)H * W;
    const float* X = img + ch * plane;
    const float* Y = gt + ch * plane;
    float w[SS_WIN];
#pragma unroll
    for (int k = 0; k < SS_WIN; ++k) w[k] = win.w[k];

    // 1. input halo, zero outside the image (the reference's padding)
    for (int i = t; i < SS_R2 * SS_R2; i += 256) {
        const int r = i / SS_R2, c = i - r * SS_R2;
        const int gy = oy - 2 * SS_HALO + r, gx = ox - 2 * SS_HALO + c;
        const bool in = gy >= 0 && gy < H && gx >= 0 && gx < W;
        s_x[r][c] = in ? X[(size_t)gy * W + gx] : 0.f;
        s_y[r][c] = in ? Y[(size_t)gy * W + gx] : 0.f;
    }
    __syncthreads();
    // 2. horizontal 11-tap pass of the five products, rows 0..35, columns 0..25 of the 26-wide region
    for (int i = t; i < SS_R2 * SS_R1; i += 256) {
        const int r = i / SS_R1, c = i - r * SS_R1;
        float hx = 0.f, hy = 0.f, hxx = 0.f, hyy = 0.f, hxy = 0.f;
#pragma unroll
        for (int k = 0; k < SS_WIN; ++k) {
            const float x = s_x[r][c + k], y = s_y[r][c + k];
            hx = __builtin_fmaf(w[k], x, hx);
            hy = __builtin_fmaf(w[k], y, hy);
            hxx = __builtin_fmaf(w[k], x * x, hxx);
            hyy = __builtin_fmaf(w[k], y * y, hyy);
            hxy = __builtin_fmaf(w[k], x * y, hxy);
        }
        s_h[0][r][c] = hx;
        s_h[1][r][c] = hy;
        s_h[2][r][c] = hxx;
        s_h[3][r][c] = hyy;
        s_h[4][r][c] = hxy;
    }
    __syncthreads();
    // 3. vertical pass -> moments on 26x26
    for (int i = t; i < SS_R1 * SS_R1; i += 256) {
        const int r = i / SS_R1, c = i - r * SS_R1;
#pragma unroll
        for (int q = 0; q < 5; ++q) {
            float m = 0.f;
#pragma unroll
            for (int k = 0; k < SS_WIN; ++k) m = __builtin_fmaf(w[k], s_h[q][r + k][c], m);
            s_m[q][r][c] = m;
        }
    }
    __syncthreads();
    // 4. SSIM and its partials (times dL/dS) on 26x26; the central 16x16 inside the image feed the loss sum
    float ssim_sum = 0.f;
    for (int i = t; i < SS_R1 * SS_R1; i += 256) {
        const int r = i / SS_R1, c = i - r * SS_R1;
        const int gy = oy - SS_HALO + r, gx = ox - SS_HALO + c;
        const bool in = gy >= 0 && gy < H && gx >= 0 && gx < W;
        const SsimPart p = ssim_partials(s_m[0][r][c], s_m[1][r][c], s_m[2][r][c], s_m[3][r][c], s_m[4][r][c],
                                         dS_scale, in);
        if (in && r >= SS_HALO && r < SS_HALO + SS_TILE && c >= SS_HALO && c < SS_HALO + SS_TILE) ssim_sum += p.S;
        // s_m[0..2] are read only by this thread at this position: overwrite in place
        s_m[0][r][c] = p.A;
        s_m[1][r][c] = p.B;
        s_m[2][r][c] = p.C;
    }
    __syncthreads();
    // 5. horizontal pass of A, B, C: rows 0..25, columns 0..15
    for (int i = t; i < SS_R1 * SS_TILE; i += 256) {
        const int r = i / SS_TILE, c = i - r * SS_TILE;
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            float h = 0.f;
#pragma unroll
            for (int k = 0; k < SS_WIN; ++k) h = __builtin_fmaf(w[k], s_m[q][r][c + k], h);
            s_h[q][r][c] = h;
        }
    }
    __syncthreads();
    // 6. vertical pass + combine: one output pixel per thread
    const int r = t / SS_TILE, c = t % SS_TILE;
    const int gy = oy + r, gx = ox + c;
    float fa = 0.f, fb = 0.f, fc = 0.f;
#pragma unroll
    for (int k = 0; k < SS_WIN; ++k) {
        fa = __builtin_fmaf(w[k], s_h[0][r + k][c], fa);
        fb = __builtin_fmaf(w[k], s_h[1][r + k][c], fb);
        fc = __builtin_fmaf(w[k], s_h[2][r + k][c], fc);
    }
    float l1_sum = 0.f;
    if (gy < H && gx < W) {
        const float x = s_x[r + 2 * SS_HALO][c + 2 * SS_HALO], y = s_y[r + 2 * SS_HALO][c + 2 * SS_HALO];
        dimg[ch * plane + (size_t)gy * W + gx] = ssim_pixel_grad(fa, fb, fc, x, y, l1_scale);
        l1_sum = fabsf(x - y);
    }
    // 7. block partial sums (fixed order: wave shuffle tree, then the 4 waves in order)
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        ssim_sum += __shfl_xor(ssim_sum, o, 64);
        l1_sum += __shfl_xor(l1_sum, o, 64);
    }
    if ((t & 63) == 0) {
        s_red[0][t >> 6] = ssim_sum;
        s_red[1][t >> 6] = l1_sum;
    }
    __syncthreads();
    if (t == 0) {
        const size_t b = ((size_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
        partials[2 * b] = (s_red[0][0] + s_red[0][1]) + (s_red[0][2] + s_red[0][3]);
        partials[2 * b + 1] = (s_red[1][0] + s_red[1][1]) + (s_red[1][2] + s_red[1][3]);
    }
}

// ---- streaming variant (default) ------------------------------------------------------------------------------
// One wave per strip of 54 output columns x `rows` output rows and channel, walking the input rows top to
// bottom. Each lane owns one column of the 64 product / partial columns (x0-5 .. x0+58) and keeps, in registers,
// rings of the last 11 rows of its column's horizontally filtered products (5 values) and of its output column's
// horizontally back-filtered partials (3 values), so every vertical 11-tap pass is register-only and every value is
// computed once per strip instead of once per 16x16 tile (36x26 / 26x26 halo regions there). Per input row i:
// horizontal products of row i; moments, SSIM and partials of row i - 5; the back-filtered gradient of output row
// i - 10.
//  * Input rows are requested 11 rows ahead into registers (3 words per lane per row: x and y of the lane's column,
//    and one of the 20 words of the strip's last 10 columns), one ring slot per unrolled row, so a row's loads have
//    eleven rows of filtering to land in; the only other vector-memory operation is the gradient store.
//  * LDS keeps the last 11 input rows (x, y): the output row's own x and y (row i - 10) come from there, not from a
//    second global load whose wait would also wait for every prefetch issued before it.
//  * x^2, y^2, xy are formed once per input column (not once per tap); the x | y and x^2 | y^2 taps, the vertical
//    moment pairs and the A | B back-filter pairs are v_pk_fma_f32 — the kernel is VALU-bound once the loads are
//    hidden (VALU per row: ~450 issue slots as separate multiply + add, ~190 fused and packed).
constexpr int ST_OUT = 54;  // output columns per strip: lanes 0..53
constexpr int ST_IN = 74;   // input columns x0-10 .. x0+63
// Strip height: the tallest that still gives every resident wave slot of the device one strip (stream_rows below):
// each strip re-walks 2 x 10 halo rows, so fewer, taller strips do less work, while a second round of strips would
// leave most of the chip idle behind the first. 3x1024x2048 on MI355X: 40 rows, 2964 strips for 3072 slots
// (48 rows: 0.136 ms, 40: 0.127, 32: 0.146; profiles/r05m_ssim_ab.txt).
constexpr int ST_ROWS_MIN = 16;   // the strip height used to size the partial sums (the shortest stream_rows gives)
constexpr int ST_ROWS_AUTO = 48;  // the tiled / streaming decision counts strips of this height
constexpr int ST_EXTRA = ST_IN - 64;  // input columns past the wave's 64 lanes

struct StreamCtx {
    const float* X;
    const float* Y;
    int H, W, x0, y0, i1, lane, rows;
    float l1_scale, dS_scale;
    float* dimg;
};

// this lane's three words of input row i: x and y of input column `lane`, and x (lanes 0..9) or y (lanes 10..19) of
// input column 64 + lane % 10; zero outside the image and past the strip's last input row (never requested)
struct RowWords {
    float x, y, e;
};
__device__ __forceinline__ RowWords ssim_fetch_row(const StreamCtx& c, int i)
{
    RowWords r{0.f, 0.f, 0.f};
    if (i > c.i1 || i < 0 || i >= c.H) return r;  // wave-uniform
    const size_t row = (size_t)i * c.W;
    const int gx = c.x0 - 2 * SS_HALO + c.lane;
    if (gx >= 0 && gx < c.W) {
        r.x = c.X[row + gx];
        r.y = c.Y[row + gx];
    }
    const bool ex = c.lane < ST_EXTRA;
    const int ge = c.x0 - 2 * SS_HALO + 64 + (ex ? c.lane : c.lane - ST_EXTRA);  // >= 54 > 0
    if (c.lane < 2 * ST_EXTRA && ge < c.W) r.e = (ex ? c.X : c.Y)[row + ge];
    return r;
}

template <int S>
__device__ __forceinline__ void ssim_stream_row(const StreamCtx& c, const float* w, int i, float2 (*s_xy)[ST_IN],
                                                float4* s_sq, float4* s_p, f2v (&hm)[SS_WIN], f2v (&hs)[SS_WIN],
                                                float (&hc)[SS_WIN], f2v (&dab)[SS_WIN], float (&dc)[SS_WIN],
                                                RowWords (&pre)[SS_WIN], float& ssim_sum, float& l1_sum)
{
    if (i > c.i1) return;  // wave-uniform
    const int lane = c.lane;
    float2* row = s_xy[S];  // ring slot of input row i (rows base .. base + 10 of this 11-row step)
    wave_sync();  // the previous row's LDS reads before this row's writes (other lanes read what a lane overwrites)
    // A. input row i to LDS; row i + 11 requested into the registers it came from
    {
        const RowWords r = pre[S];
        row[lane] = make_float2(r.x, r.y);
        if (lane < ST_EXTRA) row[64 + lane].x = r.e;
        else if (lane < 2 * ST_EXTRA) row[64 + lane - ST_EXTRA].y = r.e;
        s_sq[lane] = make_float4(r.x * r.x, r.y * r.y, r.x * r.y, 0.f);
        pre[S] = ssim_fetch_row(c, i + SS_WIN);
    }
    wave_sync();
    if (lane < ST_EXTRA) {  // the last 10 columns' products: their x and y came from two lanes
        const float2 v = row[64 + lane];
        s_sq[64 + lane] = make_float4(v.x * v.x, v.y * v.y, v.x * v.y, 0.f);
    }
    wave_sync();
    // B. horizontal 11-tap pass of x | y, x^2 | y^2, xy at product column x0 - 5 + lane
    {
        f2v m = {0.f, 0.f}, q = {0.f, 0.f};
        float xy = 0.f;
#pragma unroll
        for (int k = 0; k < SS_WIN; ++k) {
            const f2v wk = {w[k], w[k]};
            const float2 v = row[lane + k];
            const float4 p = s_sq[lane + k];
            m = __builtin_elementwise_fma(wk, f2v{v.x, v.y}, m);
            q = __builtin_elementwise_fma(wk, f2v{p.x, p.y}, q);
            xy = __builtin_fmaf(w[k], p.z, xy);
        }
        hm[S] = m;
        hs[S] = q;
        hc[S] = xy;
    }
    // C. moments, SSIM and partials of row m = i - 5 (the ring holds input rows i-10 .. i)
    if (i >= c.y0) {
        const int mr = i - SS_HALO, pc = c.x0 - SS_HALO + lane;
        f2v mu = {0.f, 0.f}, ex2 = {0.f, 0.f};
        float exy = 0.f;
#pragma unroll
        for (int k = 0; k < SS_WIN; ++k) {
            const int j = (S + 1 + k) % SS_WIN;
            const f2v wk = {w[k], w[k]};
            mu = __builtin_elementwise_fma(wk, hm[j], mu);
            ex2 = __builtin_elementwise_fma(wk, hs[j], ex2);
            exy = __builtin_fmaf(w[k], hc[j], exy);
        }
        const bool in = mr >= 0 && mr < c.H && pc >= 0 && pc < c.W;
        const SsimPart p = ssim_partials(mu.x, mu.y, ex2.x, ex2.y, exy, c.dS_scale, in);
        if (in && mr >= c.y0 && mr < c.y0 + c.rows && lane >= SS_HALO && lane < SS_HALO + ST_OUT)
            ssim_sum += p.S;  // the strip's own output rows and columns
        s_p[lane] = make_float4(p.A, p.B, p.C, 0.f);
        wave_sync();  // the next row's syncs separate these reads from the next write
        if (lane < ST_OUT) {
            f2v ab = {0.f, 0.f};
            float cc = 0.f;
#pragma unroll
            for (int k = 0; k < SS_WIN; ++k) {
                const float4 v = s_p[lane + k];
                ab = __builtin_elementwise_fma(f2v{w[k], w[k]}, f2v{v.x, v.y}, ab);
                cc = __builtin_fmaf(w[k], v.z, cc);
            }
            dab[S] = ab;
            dc[S] = cc;
        }
    }
    // D. output row o = i - 10 (the partial ring holds moment rows o-5 .. o+5; the input ring holds row o)
    if (i >= c.y0 + 2 * SS_HALO && lane < ST_OUT) {
        const int o = i - 2 * SS_HALO, col = c.x0 + lane;
        f2v ab = {0.f, 0.f};
        float cc = 0.f;
#pragma unroll
        for (int k = 0; k < SS_WIN; ++k) {
            const int j = (S + 1 + k) % SS_WIN;
            ab = __builtin_elementwise_fma(f2v{w[k], w[k]}, dab[j], ab);
            cc = __builtin_fmaf(w[k], dc[j], cc);
        }
        if (o < c.H && col < c.W) {
            const float2 v = s_xy[(S + 1) % SS_WIN][lane + 2 * SS_HALO];
            c.dimg[(size_t)o * c.W + col] = ssim_pixel_grad(ab.x, ab.y, cc, v.x, v.y, c.l1_scale);
            l1_sum += fabsf(v.x - v.y);
        }
    }
}

__global__ __launch_bounds__(64) void l1_ssim_stream_kernel(const float* img, const float* gt, int H, int W,
                                                            SsimWindow win, float l1_scale, float dS_scale,
                                                            float* dimg, float* partials, int rows)
{
    __shared__ float2 s_xy[SS_WIN][ST_IN];
    __shared__ float4 s_sq[ST_IN];
    __shared__ float4 s_p[64];
    const int ch = blockIdx.z;
    const size_t plane = (size_t)H * W;
    StreamCtx c;
    c.X = img + ch * plane;
    c.Y = gt + ch * plane;
    c.H = H, c.W = W;
    c.rows = rows;
    c.x0 = blockIdx.x * ST_OUT, c.y0 = blockIdx.y * rows;
    c.i1 = min(c.y0 + rows, H) - 1 + 2 * SS_HALO;  // input row of the chunk's last output row
    c.lane = threadIdx.x;
    c.l1_scale = l1_scale, c.dS_scale = dS_scale;
    c.dimg = dimg + ch * plane;
    float w[SS_WIN];
#pragma unroll
    for (int k = 0; k < SS_WIN; ++k) w[k] = win.w[k];
    f2v hm[SS_WIN], hs[SS_WIN], dab[SS_WIN];
    float hc[SS_WIN], dc[SS_WIN];
    RowWords pre[SS_WIN];
    const int first = c.y0 - 2 * SS_HALO;
#pragma unroll
    for (int k = 0; k < SS_WIN; ++k) {
        hm[k] = hs[k] = dab[k] = f2v{0.f, 0.f};
        hc[k] = dc[k] = 0.f;
        pre[k] = ssim_fetch_row(c, first + k);
    }
    float ssim_sum = 0.f, l1_sum = 0.f;
    for (int base = first; base <= c.i1; base += SS_WIN) {
        ssim_stream_row<0>(c, w, base + 0, s_xy, s_sq, s_p, hm, hs, hc, dab, dc, pre, ssim_sum, l1_sum);
        ssim_stream_row<1>(c, w, base + 1, s_xy, s_sq, s_p, hm, hs, hc, dab, dc, pre, ssim_sum, l1_sum);
        ssim_stream_row<2>(c, w, base + 2, s_xy, s_sq, s_p, hm, hs, hc, dab, dc, pre, ssim_sum, l1_sum);
        ssim_stream_row<3>(c, w, base + 3, s_xy, s_sq, s_p, hm, hs, hc, dab, dc, pre, ssim_sum, l1_sum);
        ssim_stream_row<4>(c, w, base + 4, s_xy, s_sq, s_p, hm, hs, hc, dab, dc, pre, ssim_sum, l1_sum);
        ssim_stream_row<5>(c, w, base + 5, s_xy, s_sq, s_p, hm, hs, hc, dab, dc, pre, ssim_sum, l1_sum);
        ssim_stream_row<6>(c, w, base + 6, s_xy, s_sq, s_p, hm, hs, hc, dab, dc, pre, ssim_sum, l1_sum);
        ssim_stream_row<7>(c, w, base + 7, s_xy, s_sq, s_p, hm, hs, hc, dab, dc, pre, ssim_sum, l1_sum);
        ssim_stream_row<8>(c, w, base + 8, s_xy, s_sq, s_p, hm, hs, hc, dab, dc, pre, ssim_sum, l1_sum);
        ssim_stream_row<9>(c, w, base + 9, s_xy, s_sq, s_p, hm, hs, hc, dab, dc, pre, ssim_sum, l1_sum);
        ssim_stream_row<10>(c, w, base + 10, s_xy, s_sq, s_p, hm, hs, hc, dab, dc, pre, ssim_sum, l1_sum);
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        ssim_sum += __shfl_xor(ssim_sum, o, 64);
        l1_sum += __shfl_xor(l1_sum, o, 64);
    }
    if (threadIdx.x == 0) {
        const size_t b = ((size_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
        partials[2 * b] = ssim_sum;
        partials[2 * b + 1] = l1_sum;
    }
}

// loss = (1 - lambda) * sum|x - y| / n + lambda * (1 - sum S / n); out = {loss, l1, ssim}
__global__ __launch_bounds__(1024) void loss_finish_kernel(const float* partials, uint32_t nblocks, float inv_n,
                                                           float lambda, float* out)
{
    __shared__ double s_s[16], s_l[16];
    double ss = 0.0, sl = 0.0;
    for (uint32_t b = threadIdx.x; b < nblocks; b += 1024) {
        ss += partials[2 * b];
        sl += partials[2 * b + 1];
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        ss += __shfl_xor(ss, o, 64);
        sl += __shfl_xor(sl, o, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        s_s[threadIdx.x >> 6] = ss;
        s_l[threadIdx.x >> 6] = sl;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double a = 0.0, l = 0.0;
        for (int k = 0; k < 16; ++k) {
            a += s_s[k];
            l += s_l[k];
        }
        const float ssim = (float)(a * inv_n), l1 = (float)(l * inv_n);
        out[0] = (1.f - lambda) * l1 + lambda * (1.f - ssim);
        out[1] = l1;
        out[2] = ssim;
    }
}

}  // namespace

// loss_utils.h:54-67 gaussian(11, 1.5): float exp, then normalised by the float sum (torch's float sum is a
// pairwise tree; for 11 terms any order differs by at most an ulp)
SsimWindow ssim_window()
{
    SsimWindow w;
    float sum = 0.f;
    for (int x = 0; x < SS_WIN; ++x) {
        const int temp = x - SS_WIN / 2;
        w.w[x] = std::exp(-(float)(temp * temp) / (2.0f * 1.5f * 1.5f));
        sum += w.w[x];
    }
    for (int x = 0; x < SS_WIN; ++x) w.w[x] /= sum;
    return w;
}

// the streaming kernel's strip height for a [C,H,W] image (see ST_ROWS_MIN): one strip per resident wave slot
static int stream_rows(int C, int H, int W)
{
    static thread_local int cached_dev = -1;
    static thread_local long slots = 0;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    if (dev != cached_dev) {
        int cus = 0, per_cu = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 256;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, l1_ssim_stream_kernel, 64, 0) != hipSuccess ||
            per_cu <= 0)
            per_cu = 12;
        slots = (long)cus * per_cu;
        cached_dev = dev;
    }
    const long per_column = slots / ((long)div_up(W, ST_OUT) * C);  // strips each strip column may have
    if (per_column <= 1) return std::max(H, 1);
    return std::max(ST_ROWS_MIN, (int)div_up((uint32_t)H, (uint32_t)per_column));
}

size_t l1_ssim_scratch_floats(int C, int H, int W)
{
    return 2 * std::max((size_t)div_up(W, SS_TILE) * div_up(H, SS_TILE), (size_t)div_up(W, ST_OUT) * div_up(H, ST_ROWS_MIN)) *
           (size_t)C;
}

void launch_l1_ssim(const float* img, const float* gt, int C, int H, int W, float lambda, float* dimg, float* out3,
                    float* scratch, hipStream_t s)
{
    const double n = (double)C * H * W;
    // the streaming kernel walks its strip's rows in sequence: it needs enough strips to fill the chip
    // (>= ~2 waves per SIMD); smaller images take the tiled kernel (same dL/dimg bits)
    const int mode = g_ssim_mode.load(std::memory_order_relaxed);
    const bool stream = mode ? mode == 2 : (size_t)div_up(W, ST_OUT) * div_up(H, ST_ROWS_AUTO) * C >= 2048;
    dim3 grid;
    if (stream) {
        const int rows = stream_rows(C, H, W);
        grid = dim3(div_up(W, ST_OUT), div_up(H, rows), C);
        l1_ssim_stream_kernel<<<grid, 64, 0, s>>>(img, gt, H, W, ssim_window(), (float)((1.0 - lambda) / n),
                                                  (float)(-(double)lambda / n), dimg, scratch, rows);
    } else {
        grid = dim3(div_up(W, SS_TILE), div_up(H, SS_TILE), C);
        l1_ssim_kernel<<<grid, 256, 0, s>>>(img, gt, H, W, ssim_window(), (float)((1.0 - lambda) / n),
                                            (float)(-(double)lambda / n), dimg, scratch);
    }
    loss_finish_kernel<<<1, 1024, 0, s>>>(scratch, grid.x * grid.y * grid.z, (float)(1.0 / n), lambda, out3);
}

int ssim_debug_mode(int mode) { return g_ssim_mode.exchange(mode); }

}  // namespace omr

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
#include <algorithm>
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
            hx += w[k] * x;
            hy += w[k] * y;
            hxx += w[k] * (x * x);
            hyy += w[k] * (y * y);
            hxy += w[k] * (x * y);
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
            for (int k = 0; k < SS_WIN; ++k) m += w[k] * s_h[q][r + k][c];
            s_m[q][r][c] = m;
        }
    }
    __syncthreads();
    // 4. SSIM and its partials (times dL/dS) on 26x26; the central 16x16 inside the image feed the loss sum
    float ssim_sum = 0.f;
    for (int i = t; i < SS_R1 * SS_R1; i += 256) {
        const int r = i / SS_R1, c = i - r * SS_R1;
        const int gy = oy - SS_HALO + r, gx = ox - SS_HALO + c;
        const float mu1 = s_m[0][r][c], mu2 = s_m[1][r][c];
        const float mu1_sq = mu1 * mu1, mu2_sq = mu2 * mu2, mu1_mu2 = mu1 * mu2;
        const float s11 = s_m[2][r][c] - mu1_sq, s22 = s_m[3][r][c] - mu2_sq, s12 = s_m[4][r][c] - mu1_mu2;
        const float a1 = 2.f * mu1_mu2 + SS_C1, b1 = 2.f * s12 + SS_C2;
        const float a2 = mu1_sq + mu2_sq + SS_C1, b2 = s11 + s22 + SS_C2;
        const float den = a2 * b2;
        const float S = (a1 * b1) / den;
        const bool in = gy >= 0 && gy < H && gx >= 0 && gx < W;
        float A = 0.f, B = 0.f, C = 0.f;
        if (in) {
            const float inv = 1.f / den;
            A = dS_scale * ((2.f * mu2 * (b1 - a1)) * inv - S * (2.f * mu1 * (b2 - a2)) * inv);
            B = dS_scale * (-S / b2);
            C = dS_scale * (2.f * a1 * inv);
            if (r >= SS_HALO && r < SS_HALO + SS_TILE && c >= SS_HALO && c < SS_HALO + SS_TILE) ssim_sum += S;
        }
        // s_m[0..2] are read only by this thread at this position: overwrite in place
        s_m[0][r][c] = A;
        s_m[1][r][c] = B;
        s_m[2][r][c] = C;
    }
    __syncthreads();
    // 5. horizontal pass of A, B, C: rows 0..25, columns 0..15
    for (int i = t; i < SS_R1 * SS_TILE; i += 256) {
        const int r = i / SS_TILE, c = i - r * SS_TILE;
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            float h = 0.f;
#pragma unroll
            for (int k = 0; k < SS_WIN; ++k) h += w[k] * s_m[q][r][c + k];
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
        fa += w[k] * s_h[0][r + k][c];
        fb += w[k] * s_h[1][r + k][c];
        fc += w[k] * s_h[2][r + k][c];
    }
    float l1_sum = 0.f;
    if (gy < H && gx < W) {
        const float x = s_x[r + 2 * SS_HALO][c + 2 * SS_HALO], y = s_y[r + 2 * SS_HALO][c + 2 * SS_HALO];
        const float d = x - y;
        const float sgn = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);  // torch.abs backward: sign(0) = 0
        dimg[ch * plane + (size_t)gy * W + gx] = fa + 2.f * x * fb + y * fc + l1_scale * sgn;
        l1_sum = fabsf(d);
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
// One wave per strip of 54 output columns x OMR_SSIM_ROWS output rows and channel, walking the input rows top to
// bottom. Each lane owns one column of the 64 product / partial columns (x0-5 .. x0+58) and keeps, in registers,
// rings of the last 11 rows of its column's horizontally filtered products (5 values) and of its output column's
// horizontally back-filtered partials (3 values), so every vertical 11-tap pass is register-only and every value is
// computed once per strip instead of once per 16x16 tile (36x26 / 26x26 halo regions there). LDS holds one input
// row (x, y) and one row of partials. Per input row i: horizontal products of row i; moments, SSIM and partials
// of row i - 5; the back-filtered gradient of output row i - 10. The taps are summed in the same order as the tiled
// kernel above, so dL/dimg is bitwise the same; the loss sums differ only in their (fixed) blocking.
#ifndef OMR_SSIM_ROWS
#define OMR_SSIM_ROWS 48
#endif
constexpr int ST_OUT = 54;  // output columns per strip: lanes 0..53
constexpr int ST_IN = 74;   // input columns x0-10 .. x0+63
constexpr int ST_ROWS = OMR_SSIM_ROWS;

struct StreamCtx {
    const float* X;
    const float* Y;
    int H, W, x0, y0, i1, lane;
    float l1_scale, dS_scale;
    float* dimg;
};

// this lane's input columns (lane and 64 + lane) of row i, zero outside the image
__device__ __forceinline__ void ssim_load_row(const StreamCtx& c, int i, float2 (&pre)[2])
{
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int k = c.lane + 64 * h;
        const int gx = c.x0 - 2 * SS_HALO + k;
        const bool in = k < ST_IN && i >= 0 && i < c.H && gx >= 0 && gx < c.W;
        pre[h] = in ? make_float2(c.X[(size_t)i * c.W + gx], c.Y[(size_t)i * c.W + gx]) : make_float2(0.f, 0.f);
    }
}

template <int S>
__device__ __forceinline__ void ssim_stream_row(const StreamCtx& c, const float* w, int i, float2 (*s_in)[ST_IN],
                                                float4* s_p, float (&hb)[SS_WIN][5], float (&hd)[SS_WIN][3],
                                                float2 (&pre)[2], float& ssim_sum, float& l1_sum)
{
    if (i > c.i1) return;  // wave-uniform
    const int lane = c.lane;
    // A. input row i to LDS (a one-row register prefetch measured no faster); horizontal products at product
    //    column x0 - 5 + lane
    float2* buf = s_in[i & 1];
    ssim_load_row(c, i, pre);
    buf[lane] = pre[0];
    if (lane < ST_IN - 64) buf[64 + lane] = pre[1];
    wave_sync();
    {
        float hx = 0.f, hy = 0.f, hxx = 0.f, hyy = 0.f, hxy = 0.f;
#pragma unroll
        for (int k = 0; k < SS_WIN; ++k) {
            const float2 v = buf[lane + k];
            hx += w[k] * v.x;
            hy += w[k] * v.y;
            hxx += w[k] * (v.x * v.x);
            hyy += w[k] * (v.y * v.y);
            hxy += w[k] * (v.x * v.y);
        }
        hb[S][0] = hx, hb[S][1] = hy, hb[S][2] = hxx, hb[S][3] = hyy, hb[S][4] = hxy;
    }
    // B. moments, SSIM and partials of row m = i - 5 (the ring holds input rows i-10 .. i)
    if (i >= c.y0) {
        const int m = i - SS_HALO, pc = c.x0 - SS_HALO + lane;
        float mo[5];
#pragma unroll
        for (int q = 0; q < 5; ++q) {
            float acc = 0.f;
#pragma unroll
            for (int k = 0; k < SS_WIN; ++k) acc += w[k] * hb[(S + 1 + k) % SS_WIN][q];
            mo[q] = acc;
        }
        const float mu1 = mo[0], mu2 = mo[1];
        const float mu1_sq = mu1 * mu1, mu2_sq = mu2 * mu2, mu1_mu2 = mu1 * mu2;
        const float s11 = mo[2] - mu1_sq, s22 = mo[3] - mu2_sq, s12 = mo[4] - mu1_mu2;
        const float a1 = 2.f * mu1_mu2 + SS_C1, b1 = 2.f * s12 + SS_C2;
        const float a2 = mu1_sq + mu2_sq + SS_C1, b2 = s11 + s22 + SS_C2;
        const float den = a2 * b2;
        const float Sv = (a1 * b1) / den;
        const bool in = m >= 0 && m < c.H && pc >= 0 && pc < c.W;
        float A = 0.f, B = 0.f, C = 0.f;
        if (in) {
            const float inv = 1.f / den;
            A = c.dS_scale * ((2.f * mu2 * (b1 - a1)) * inv - Sv * (2.f * mu1 * (b2 - a2)) * inv);
            B = c.dS_scale * (-Sv / b2);
            C = c.dS_scale * (2.f * a1 * inv);
            if (m >= c.y0 && m < c.y0 + ST_ROWS && lane >= SS_HALO && lane < SS_HALO + ST_OUT) ssim_sum += Sv;
        }
        s_p[lane] = make_float4(A, B, C, 0.f);
        wave_sync();  // the next row's input sync separates these reads from the next write
        if (lane < ST_OUT) {
            float fa = 0.f, fb = 0.f, fc = 0.f;
#pragma unroll
            for (int k = 0; k < SS_WIN; ++k) {
                const float4 v = s_p[lane + k];
                fa += w[k] * v.x;
                fb += w[k] * v.y;
                fc += w[k] * v.z;
            }
            hd[S][0] = fa, hd[S][1] = fb, hd[S][2] = fc;
        }
    }
    // D. output row o = i - 10 (the partial ring holds moment rows o-5 .. o+5)
    if (i >= c.y0 + 2 * SS_HALO && lane < ST_OUT) {
        const int o = i - 2 * SS_HALO, col = c.x0 + lane;
        float fa = 0.f, fb = 0.f, fc = 0.f;
#pragma unroll
        for (int k = 0; k < SS_WIN; ++k) {
            fa += w[k] * hd[(S + 1 + k) % SS_WIN][0];
            fb += w[k] * hd[(S + 1 + k) % SS_WIN][1];
            fc += w[k] * hd[(S + 1 + k) % SS_WIN][2];
        }
        if (o < c.H && col < c.W) {
            const size_t at = (size_t)o * c.W + col;
            const float x = c.X[at], y = c.Y[at];
            const float d = x - y;
            const float sgn = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
            c.dimg[at] = fa + 2.f * x * fb + y * fc + c.l1_scale * sgn;
            l1_sum += fabsf(d);
        }
    }
}

__global__ __launch_bounds__(64) void l1_ssim_stream_kernel(const float* img, const float* gt, int H, int W,
                                                            SsimWindow win, float l1_scale, float dS_scale,
                                                            float* dimg, float* partials)
{
    __shared__ float2 s_in[2][ST_IN];
    __shared__ float4 s_p[64 + SS_WIN];
    const int ch = blockIdx.z;
    const size_t plane = (size_t)H * W;
    StreamCtx c;
    c.X = img + ch * plane;
    c.Y = gt + ch * plane;
    c.H = H, c.W = W;
    c.x0 = blockIdx.x * ST_OUT, c.y0 = blockIdx.y * ST_ROWS;
    c.i1 = min(c.y0 + ST_ROWS, H) - 1 + 2 * SS_HALO;  // input row of the chunk's last output row
    c.lane = threadIdx.x;
    c.l1_scale = l1_scale, c.dS_scale = dS_scale;
    c.dimg = dimg + ch * plane;
    float w[SS_WIN];
#pragma unroll
    for (int k = 0; k < SS_WIN; ++k) w[k] = win.w[k];
    if (threadIdx.x < SS_WIN) s_p[64 + threadIdx.x] = make_float4(0.f, 0.f, 0.f, 0.f);  // lanes 54..63 read up to 63
    float hb[SS_WIN][5], hd[SS_WIN][3];
#pragma unroll
    for (int k = 0; k < SS_WIN; ++k) {
#pragma unroll
        for (int q = 0; q < 5; ++q) hb[k][q] = 0.f;
#pragma unroll
        for (int q = 0; q < 3; ++q) hd[k][q] = 0.f;
    }
    float ssim_sum = 0.f, l1_sum = 0.f;
    float2 pre[2];
    for (int base = c.y0 - 2 * SS_HALO; base <= c.i1; base += SS_WIN) {
        ssim_stream_row<0>(c, w, base + 0, s_in, s_p, hb, hd, pre, ssim_sum, l1_sum);
        ssim_stream_row<1>(c, w, base + 1, s_in, s_p, hb, hd, pre, ssim_sum, l1_sum);
        ssim_stream_row<2>(c, w, base + 2, s_in, s_p, hb, hd, pre, ssim_sum, l1_sum);
        ssim_stream_row<3>(c, w, base + 3, s_in, s_p, hb, hd, pre, ssim_sum, l1_sum);
        ssim_stream_row<4>(c, w, base + 4, s_in, s_p, hb, hd, pre, ssim_sum, l1_sum);
        ssim_stream_row<5>(c, w, base + 5, s_in, s_p, hb, hd, pre, ssim_sum, l1_sum);
        ssim_stream_row<6>(c, w, base + 6, s_in, s_p, hb, hd, pre, ssim_sum, l1_sum);
        ssim_stream_row<7>(c, w, base + 7, s_in, s_p, hb, hd, pre, ssim_sum, l1_sum);
        ssim_stream_row<8>(c, w, base + 8, s_in, s_p, hb, hd, pre, ssim_sum, l1_sum);
        ssim_stream_row<9>(c, w, base + 9, s_in, s_p, hb, hd, pre, ssim_sum, l1_sum);
        ssim_stream_row<10>(c, w, base + 10, s_in, s_p, hb, hd, pre, ssim_sum, l1_sum);
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

size_t l1_ssim_scratch_floats(int C, int H, int W)
{
    return 2 * std::max((size_t)div_up(W, SS_TILE) * div_up(H, SS_TILE), (size_t)div_up(W, ST_OUT) * div_up(H, ST_ROWS)) *
           (size_t)C;
}

void launch_l1_ssim(const float* img, const float* gt, int C, int H, int W, float lambda, float* dimg, float* out3,
                    float* scratch, hipStream_t s)
{
    const double n = (double)C * H * W;
    // the streaming kernel walks its strip's rows in sequence: it needs enough strips to fill the chip
    // (>= ~2 waves per SIMD); smaller images take the tiled kernel (same dL/dimg bits)
    const bool stream = (size_t)div_up(W, ST_OUT) * div_up(H, ST_ROWS) * C >= 2048;
    dim3 grid;
    if (stream) {
        grid = dim3(div_up(W, ST_OUT), div_up(H, ST_ROWS), C);
        l1_ssim_stream_kernel<<<grid, 64, 0, s>>>(img, gt, H, W, ssim_window(), (float)((1.0 - lambda) / n),
                                                  (float)(-(double)lambda / n), dimg, scratch);
    } else {
        grid = dim3(div_up(W, SS_TILE), div_up(H, SS_TILE), C);
        l1_ssim_kernel<<<grid, 256, 0, s>>>(img, gt, H, W, ssim_window(), (float)((1.0 - lambda) / n),
                                            (float)(-(double)lambda / n), dimg, scratch);
    }
    loss_finish_kernel<<<1, 1024, 0, s>>>(scratch, grid.x * grid.y * grid.z, (float)(1.0 / n), lambda, out3);
}

}  // namespace omr

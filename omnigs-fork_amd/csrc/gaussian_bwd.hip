// gaussian_bwd.hip — fused per-Gaussian backward, gfx950.
//
// One thread per Gaussian does, in registers, what the reference spreads over three kernels and two
// zero-filled scratch tensors:
//   * sums the Gaussian's per-instance gradient rows written by render_bwd.hip (fixed order -> deterministic),
//     giving dL/dmean2D, dL/dconic, dL/dopacity, dL/dcolor (the reference's atomicAdd targets,
//     backward.cu:805-840);
//   * computeCov2DLonLatCUDA / computeCov2DCUDA (backward.cu:297-485 / :156-292): dL/dcov3D and the
//     covariance part of dL/dmean3D; dpx_dt / dpy_dt stay in registers (the reference round-trips them
//     through two [P,3] HBM tensors);
//   * preprocessLonLatCUDA / preprocessCUDA backward (backward.cu:613-669 / :557-608): projection part of
//     dL/dmean3D, SH backward (:30-151), cov3D -> scale/rotation backward (:489-552).
// Every output element is written exactly once (zeros for culled Gaussians and unused SH slots), so the
// caller needs no zero-initialised gradient tensors (the reference zero-fills ~324 B/Gaussian first,
// rasterize_points.cu:200-208).
#include "kernels.h"
#include "sh_eval.h"
#include "tile_wave.h"
#include "wave_ops.h"
#include "wave_rows.h"

namespace omr {

namespace {

constexpr float INV_PI = 0.318309886183790671537767526745028724f;

struct F3 {
    float x, y, z;
};

// dL/dconic -> dL/dcov2D -> dL/dcov3D and dL/dT (backward.cu:387-443). T0 = T[0][*], T1 = T[1][*] (glm).
__device__ __forceinline__ void cov2d_backward(const float T0[3], const float T1[3], const float c3[6], F3 dL_dconic,
                                               float dcov[6], float dT0[3], float dT1[3])
{
    const float V[3][3] = {{c3[0], c3[1], c3[2]}, {c3[1], c3[3], c3[4]}, {c3[2], c3[4], c3[5]}};
    // cov2D = T^T Vrk T (same evaluation as the forward)
    float B0[3], B1[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        B0[j] = T0[0] * V[j][0] + T0[1] * V[j][1] + T0[2] * V[j][2];
        B1[j] = T1[0] * V[j][0] + T1[1] * V[j][1] + T1[2] * V[j][2];
    }
    const float a = B0[0] * T0[0] + B0[1] * T0[1] + B0[2] * T0[2] + 0.3f;
    const float b = B1[0] * T0[0] + B1[1] * T0[1] + B1[2] * T0[2];
    const float c = B1[0] * T1[0] + B1[1] * T1[1] + B1[2] * T1[2] + 0.3f;
    const float denom = a * c - b * b;
    const float denom2inv = 1.0f / ((denom * denom) + 0.0000001f);
    // denom2inv == 0: every gradient term is 0 (backward.cu's branch, as selects: a branch here kept part of dcov
    // in scratch memory)
    const bool ok = denom2inv != 0.f;
    const float dL_da = ok ? denom2inv * (-c * c * dL_dconic.x + 2 * b * c * dL_dconic.y + (denom - a * c) * dL_dconic.z) : 0.f;
    const float dL_dc = ok ? denom2inv * (-a * a * dL_dconic.z + 2 * a * b * dL_dconic.y + (denom - a * c) * dL_dconic.x) : 0.f;
    const float dL_db = ok ? denom2inv * 2 * (b * c * dL_dconic.x - (denom + 2 * b * b) * dL_dconic.y + a * b * dL_dconic.z) : 0.f;
    dcov[0] = ok ? (T0[0] * T0[0] * dL_da + T0[0] * T1[0] * dL_db + T1[0] * T1[0] * dL_dc) : 0.f;
    dcov[3] = ok ? (T0[1] * T0[1] * dL_da + T0[1] * T1[1] * dL_db + T1[1] * T1[1] * dL_dc) : 0.f;
    dcov[5] = ok ? (T0[2] * T0[2] * dL_da + T0[2] * T1[2] * dL_db + T1[2] * T1[2] * dL_dc) : 0.f;
    dcov[1] = ok ? 2 * T0[0] * T0[1] * dL_da + (T0[0] * T1[1] + T0[1] * T1[0]) * dL_db + 2 * T1[0] * T1[1] * dL_dc : 0.f;
    dcov[2] = ok ? 2 * T0[0] * T0[2] * dL_da + (T0[0] * T1[2] + T0[2] * T1[0]) * dL_db + 2 * T1[0] * T1[2] * dL_dc : 0.f;
    dcov[4] = ok ? 2 * T0[2] * T0[1] * dL_da + (T0[1] * T1[2] + T0[2] * T1[1]) * dL_db + 2 * T1[1] * T1[2] * dL_dc : 0.f;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float v0 = T0[0] * V[k][0] + T0[1] * V[k][1] + T0[2] * V[k][2];
        const float v1 = T1[0] * V[k][0] + T1[1] * V[k][1] + T1[2] * V[k][2];
        dT0[k] = 2 * v0 * dL_da + v1 * dL_db;
        dT1[k] = 2 * v1 * dL_dc + v0 * dL_db;
    }
}

// backward.cu:489-552
__device__ __forceinline__ void cov3d_backward(float sx, float sy, float sz, float mod, float4 q, const float d[6],
                                               float dscale[3], float drot[4])
{
    const float r = q.x, x = q.y, y = q.z, z = q.w;
    const float R[3][3] = {{1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y)},
                           {2.f * (x * y + r * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x)},
                           {2.f * (x * z - r * y), 2.f * (y * z + r * x), 1.f - 2.f * (x * x + y * y)}};
    const float s[3] = {mod * sx, mod * sy, mod * sz};
    float M[3][3];  // M = S * R: M[j][i] = s_i * R[j][i]
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int i = 0; i < 3; ++i) M[j][i] = s[i] * R[j][i];
    const float dS[3][3] = {{d[0], 0.5f * d[1], 0.5f * d[2]}, {0.5f * d[1], d[3], 0.5f * d[4]}, {0.5f * d[2], 0.5f * d[4], d[5]}};
    float dM[3][3];  // dL_dM = (2 M) * dL_dSigma
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int i = 0; i < 3; ++i) dM[j][i] = 2.f * M[0][i] * dS[j][0] + 2.f * M[1][i] * dS[j][1] + 2.f * M[2][i] * dS[j][2];
    // dL_dMt[j][i] = dM[i][j]; dscale_c = dot(Rt[c], dL_dMt[c]) = sum_k R[k][c] * dM[k][c]
#pragma unroll
    for (int cidx = 0; cidx < 3; ++cidx) dscale[cidx] = R[0][cidx] * dM[0][cidx] + R[1][cidx] * dM[1][cidx] + R[2][cidx] * dM[2][cidx];
    float Mt[3][3];  // dL_dMt scaled: Mt[j][i] = dM[i][j] * s_j
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int i = 0; i < 3; ++i) Mt[j][i] = dM[i][j] * s[j];
    drot[0] = 2 * z * (Mt[0][1] - Mt[1][0]) + 2 * y * (Mt[2][0] - Mt[0][2]) + 2 * x * (Mt[1][2] - Mt[2][1]);
    drot[1] = 2 * y * (Mt[1][0] + Mt[0][1]) + 2 * z * (Mt[2][0] + Mt[0][2]) + 2 * r * (Mt[1][2] - Mt[2][1]) - 4 * x * (Mt[2][2] + Mt[1][1]);
    drot[2] = 2 * x * (Mt[1][0] + Mt[0][1]) + 2 * r * (Mt[2][0] - Mt[0][2]) + 2 * z * (Mt[1][2] + Mt[2][1]) - 4 * y * (Mt[2][2] + Mt[0][0]);
    drot[3] = 2 * r * (Mt[0][1] - Mt[1][0]) + 2 * x * (Mt[2][0] + Mt[0][2]) + 2 * y * (Mt[1][2] + Mt[2][1]) - 4 * z * (Mt[1][1] + Mt[0][0]);
}

// forward.cu:194-228 (recomputed instead of stored: saves 48 B/Gaussian of HBM round trip)
__device__ __forceinline__ void cov3d_forward(float sx, float sy, float sz, float mod, float4 q, float c[6])
{
    const float s[3] = {mod * sx, mod * sy, mod * sz};
    const float r = q.x, x = q.y, y = q.z, z = q.w;
    const float R[3][3] = {{1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y)},
                           {2.f * (x * y + r * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x)},
                           {2.f * (x * z - r * y), 2.f * (y * z + r * x), 1.f - 2.f * (x * x + y * y)}};
    float M[3][3];
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int i = 0; i < 3; ++i) M[j][i] = s[i] * R[j][i];
    auto sig = [&](int j, int i) { return M[i][0] * M[j][0] + M[i][1] * M[j][1] + M[i][2] * M[j][2]; };
    c[0] = sig(0, 0);
    c[1] = sig(0, 1);
    c[2] = sig(0, 2);
    c[3] = sig(1, 1);
    c[4] = sig(1, 2);
    c[5] = sig(2, 2);
}

// backward.cu:30-151; writes dL_dsh for all M coefficients (zeros beyond (deg+1)^2), returns dL/dmean part.
// MC == 16: the SH row is read as 12 float4 from row4 and the dL_dsh row written as 12 float4 to out4 (both the
// lane's row of the wave's LDS staging image, or both global rows; the row is read before it is overwritten);
// otherwise both are read/written in global memory at idx.
// A visible Gaussian's per-Gaussian inputs, loaded together with its row sums (the MC == 16 kernel): read where
// gaussian_bwd_point uses them, the loads issued only after its first stores (which may alias them, as far as the
// compiler knows), a second memory round trip on every wave's chain
struct GIn {
    F3 mean;
    float s[3];
    float4 q;
    float jac[9];
    uint8_t clamp;
};

// jac != NULL: the forward's dRGB/ddir of this Gaussian (GeomState::sh_jac: gx, gy, gz per channel), and the SH row is
// not read at all.
template <int MC>
__device__ __forceinline__ F3 sh_backward(int idx, int deg, int M, F3 pos, const float* campos, const float* shs,
                                          const float4* row4, uint8_t clamp_bits, F3 dRGB, float* dL_dsh,
                                          float4* out4, const float* jac = nullptr, const GIn* gin = nullptr,
                                          bool gin_jac = false)
{
    const int Mr = MC > 0 ? MC : M;
    const float dox = pos.x - campos[0], doy = pos.y - campos[1], doz = pos.z - campos[2];
    const float len = sqrtf(dox * dox + doy * doy + doz * doz);
    const float x = dox / len, y = doy / len, z = doz / len;
    if (clamp_bits & 1) dRGB.x = 0.f;
    if (clamp_bits & 2) dRGB.y = 0.f;
    if (clamp_bits & 4) dRGB.z = 0.f;
    float coef[16];
    sh_basis(deg, x, y, z, coef);
    float gx[3], gy[3], gz[3];  // dRGB/dx etc per channel
    if (gin_jac) {  // the same nine values, already in registers (GIn)
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) gx[ch] = gin->jac[ch], gy[ch] = gin->jac[3 + ch], gz[ch] = gin->jac[6 + ch];
    } else if (jac) {
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) gx[ch] = jac[ch], gy[ch] = jac[3 + ch], gz[ch] = jac[6 + ch];
    } else if constexpr (MC == 16) {
        const int nf4 = (3 * (deg + 1) * (deg + 1) + 3) >> 2;
        float shv[48];
#pragma unroll
        for (int q = 0; q < 12; ++q) {
            const float4 v = q < nf4 ? row4[q] : make_float4(0.f, 0.f, 0.f, 0.f);
            shv[4 * q] = v.x;
            shv[4 * q + 1] = v.y;
            shv[4 * q + 2] = v.z;
            shv[4 * q + 3] = v.w;
        }
        sh_dir_grad(deg, x, y, z, [&](int k, int ch) { return shv[3 * k + ch]; }, gx, gy, gz);
    } else {
        const float* sh_row = shs + (size_t)idx * Mr * 3;
        sh_dir_grad(deg, x, y, z, [&](int k, int ch) { return sh_row[3 * k + ch]; }, gx, gy, gz);
    }
    const float d[3] = {dRGB.x, dRGB.y, dRGB.z};
    if constexpr (MC == 16) {
        // 16 coefficients x 3 channels = 48 floats = 12 float4
#pragma unroll
        for (int q = 0; q < 12; ++q) {
            float v[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int f = 4 * q + e;
                v[e] = (f / 3) < (deg + 1) * (deg + 1) ? coef[f / 3] * d[f % 3] : 0.f;
            }
            out4[q] = make_float4(v[0], v[1], v[2], v[3]);
        }
    } else if (dL_dsh) {  // NULL: the caller skips the SH gradient (omr_backward's skip_dsh), any M
        float* out = dL_dsh + (size_t)idx * Mr * 3;
        const int nk = (deg + 1) * (deg + 1);
        for (int k = 0; k < Mr; ++k)
#pragma unroll
            for (int ch = 0; ch < 3; ++ch) out[3 * k + ch] = (k < nk && k < 16) ? coef[k] * d[ch] : 0.f;
    }
    const F3 dL_ddir = {gx[0] * d[0] + gx[1] * d[1] + gx[2] * d[2], gy[0] * d[0] + gy[1] * d[1] + gy[2] * d[2],
                        gz[0] * d[0] + gz[1] * d[1] + gz[2] * d[2]};
    // dnormvdv (auxiliary.h:134-144)
    const float sum2 = dox * dox + doy * doy + doz * doz;
    const float invsum32 = 1.0f / sqrtf(sum2 * sum2 * sum2);
    F3 r;
    r.x = ((+sum2 - dox * dox) * dL_ddir.x - doy * dox * dL_ddir.y - doz * dox * dL_ddir.z) * invsum32;
    r.y = (-dox * doy * dL_ddir.x + (sum2 - doy * doy) * dL_ddir.y - doz * doy * dL_ddir.z) * invsum32;
    r.z = (-dox * doz * dL_ddir.x - doy * doz * dL_ddir.y + (sum2 - doz * doz) * dL_ddir.z) * invsum32;
    return r;
}

// ---- per-Gaussian sums of the instance rows (the reference's atomicAdd targets, backward.cu:805-840) ---------
// Gaussian i owns the contiguous rows [row_first[i], row_first[i] + tiles_touched[i]) of inst_grad: the backward
// numbers the rows in Gaussian INDEX order (launch_forward_scans), so the 64 Gaussians of a wave own one contiguous
// span of rows (507 rows on average at config C, 24 % of them marked valid by render_bwd). Chunks of 128 rows (half
// the LDS of 256-row chunks, more waves per CU): 0.070 ms vs 0.073 (256) and 0.091 (64) at config C.
// The wave streams its span through LDS in chunks of RS_ROWS rows: every lane loads RS_Q rows of the chunk, rows
// q*64 + lane (coalesced), marked ones only, then
//  * a Gaussian with at most RS_LONG rows adds its rows of the chunk itself, in row order, from LDS;
//  * a longer one is summed by the whole wave: each lane adds the chunk rows it holds, then one wave reduction
//    (wave_ops.h) per (long Gaussian, chunk), in chunk order.
// The row_valid bytes of the next window are requested with the rows of the current one: one HBM round trip per
// window for the whole wave. Gaussians with more than ROW_SUM_HUGE rows (polar Gaussians reach every tile of the
// image; 0.1 % of them at config C, 13 % of the rows) would make their wave the kernel's tail: the wave skips them
// (and the chunks only they own), and RS_HUGE_BLOCKS extra workgroups at the start of the grid take them from the
// forward's huge_list, one wave per Gaussian. The order of every sum is fixed: the result is deterministic.
#ifndef OMR_RS_ROWS
#define OMR_RS_ROWS 128
#endif
constexpr int RS_ROWS = OMR_RS_ROWS;  // rows per staged chunk (a multiple of 64)
constexpr int RS_Q = RS_ROWS / 64;    // rows per lane per chunk
#ifndef OMR_RS_LONG
#define OMR_RS_LONG 32
#endif
constexpr uint32_t RS_LONG = OMR_RS_LONG;

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) { return ~wave_max_u32(~v); }  // DPP (tile_wave.h)

__device__ __forceinline__ void add_marked_row(float* acc, const float* __restrict__ inst_grad, uint32_t row, bool ok)
{
    if (ok) {
        const float* p = inst_grad + (size_t)row * GRAD_ROW;
#pragma unroll
        for (int c = 0; c < GRAD_ROW; ++c) acc[c] += p[c];
    }
}

struct RowSumArgs {
    int g_begin, g_end;     // the Gaussians [g_begin, g_end) of this launch (g_begin a multiple of 256)
    uint32_t huge_blocks;   // RS_HUGE_BLOCKS workgroups for the huge Gaussians at the start of the grid, or 0
    uint32_t R;
    const uint32_t* row_first;
    const uint32_t* tiles_touched;
    const uint32_t* huge_list;
    const uint32_t* huge_count;
    const float* inst_grad;
    const uint8_t* row_valid;
    float* row_sums;
    float* dL_dcolor;  // [P][3] = row_sums[:, 6:9], written here so that it is final before gaussian_bwd runs
};

// The huge Gaussians, one per wave of the first RS_HUGE_BLOCKS workgroups of the grid. A pass covers 64 x
// RS_HUGE_GROUPS 16-row mark groups (4096 rows: one 16-B mark load per group, all in flight at once), then loads the
// lane's marked rows four at a time; each lane adds its rows in row order, then one wave reduction in a fixed order. (One workgroup per Gaussian with byte marks took 345 us at config E: its many huge Gaussians, mostly a few
// hundred rows each, paid two barriers and a 256-thread reduction apiece.)
#ifndef OMR_RS_HUGE_BLOCKS
#define OMR_RS_HUGE_BLOCKS 512
#endif
constexpr uint32_t RS_HUGE_BLOCKS = OMR_RS_HUGE_BLOCKS;
constexpr int RS_HUGE_GROUPS = 4;
__device__ __forceinline__ void huge_row_sums(const RowSumArgs& a, uint32_t hb)
{
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t count = *a.huge_count;
    for (uint32_t t = hb * 4u + (threadIdx.x >> 6); t < count; t += RS_HUGE_BLOCKS * 4u) {
        const uint32_t idx = a.huge_list[t];
        const uint32_t s = a.row_first[idx];
        uint32_t n = a.tiles_touched[idx];
        if (s >= a.R || n > a.R - s) n = 0;  // never true for a consistent forward
        const uint32_t e = s + n;
        float acc[GRAD_ROW];
#pragma unroll
        for (int c = 0; c < GRAD_ROW; ++c) acc[c] = 0.f;
        // row_valid is 256-B aligned and its region holds R bytes rounded up to 256: a 16-row group starting
        // below e <= R is readable whole
        for (uint32_t g0 = s & ~15u; g0 < e; g0 += 64u * 16u * RS_HUGE_GROUPS) {
            uint4 f[RS_HUGE_GROUPS];
#pragma unroll
            for (int q = 0; q < RS_HUGE_GROUPS; ++q) {
                const uint32_t r = g0 + ((uint32_t)q * 64u + lane) * 16u;
                f[q] = r < e ? *reinterpret_cast<const uint4*>(a.row_valid + r) : make_uint4(0u, 0u, 0u, 0u);
            }
            uint64_t mk = 0;  // bit 16 q + j: row g0 + (64 q + lane) * 16 + j is marked and Gaussian idx's
#pragma unroll
            for (int q = 0; q < RS_HUGE_GROUPS; ++q) {
                const uint32_t w[4] = {f[q].x, f[q].y, f[q].z, f[q].w};
                const uint32_t r = g0 + ((uint32_t)q * 64u + lane) * 16u;
#pragma unroll
                for (uint32_t j = 0; j < 16; ++j)
                    if (((w[j >> 2] >> (8u * (j & 3u))) & 0xFFu) != 0u && r + j >= s && r + j < e)
                        mk |= 1ull << (16 * q + j);
            }
            while (mk) {  // four marked rows in flight, added in row order
                uint32_t rr[4];
                bool ok[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    ok[u] = mk != 0;
                    const uint32_t b = ok[u] ? (uint32_t)__builtin_ctzll(mk) : 0u;
                    rr[u] = g0 + ((b >> 4) * 64u + lane) * 16u + (b & 15u);
                    mk &= mk - 1;
                }
                float x[4][GRAD_ROW];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
#pragma unroll
                    for (int c = 0; c < GRAD_ROW; ++c) x[u][c] = 0.f;
                    add_marked_row(x[u], a.inst_grad, rr[u], ok[u]);
                }
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (ok[u])
#pragma unroll
                        for (int c = 0; c < GRAD_ROW; ++c) acc[c] += x[u][c];
            }
        }
        float t8;
        const float tv = wave_sum9_rows(acc, acc[8], lane, &t8);  // lane l: total of value (l >> 3) & 7
        if ((lane & 7) == 0) {
            const uint32_t c = lane >> 3;
            a.row_sums[(size_t)idx * GRAD_ROW + c] = tv;
            if (c >= 6) a.dL_dcolor[(size_t)idx * 3 + (c - 6)] = tv;
        }
        if (lane == 1) {
            a.row_sums[(size_t)idx * GRAD_ROW + 8] = t8;
            a.dL_dcolor[(size_t)idx * 3 + 2] = t8;
        }
    }
}

#ifndef OMR_RS_WIN
#define OMR_RS_WIN 512
#endif
constexpr uint32_t RS_WIN = OMR_RS_WIN;  // rows whose marks a wave compacts at once (8 per lane, one load; 1024
                                         // rows, 16 per lane: C 0.060 vs 0.056 ms, E 0.40 vs 0.37 ms, round 2)
constexpr uint32_t RS_RPL = RS_WIN / 64;
static_assert(RS_RPL == 8, "8-B mark loads");

__device__ __forceinline__ uint32_t wave_exclusive_scan_u32(uint32_t x, uint32_t lane, uint32_t* total)
{
    (void)lane;
    const uint32_t inc = wave_incl_sum_u32(x);
    *total = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
    return inc - x;
}

// six waves per SIMD (80 VGPRs, 36 B of spills) instead of five: the row sums are latency-bound (E 0.211 -> 0.205 ms,
// C unchanged: profiles/r03z_ab_row_sums_waves.txt)
#ifndef OMR_RS_MINW
#define OMR_RS_MINW 6
#endif
__global__ __launch_bounds__(256, OMR_RS_MINW) void row_sum_kernel(RowSumArgs a)
{
    __shared__ float s_rows_all[4][RS_ROWS * GRAD_ROW];  // row-major, 9 floats per row (odd stride: no conflicts)
    __shared__ uint32_t s_list_all[4][RS_WIN];
    if (blockIdx.x < a.huge_blocks) {  // dispatched first: the huge Gaussians overlap the rest of the grid
        huge_row_sums(a, blockIdx.x);
        return;
    }
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const int g0 = a.g_begin + (int)((blockIdx.x - a.huge_blocks) * 256u + wv * 64u);
    if (g0 >= a.g_end) return;  // wave-uniform
    float* s_rows = s_rows_all[wv];
    const int idx = g0 + (int)lane;
    uint32_t n = 0, s = 0, n_all = 0;
    bool huge = false;
    if (idx < a.g_end) {
        n = n_all = a.tiles_touched[idx];
        s = a.row_first[idx];
        huge = n > ROW_SUM_HUGE;  // summed by the workgroups at the end of the grid
        if (huge || (n != 0 && (s >= a.R || n > a.R - s))) n = 0;  // the latter: never for a consistent forward
    }
    const uint32_t e = s + n;
    const uint32_t lo = __builtin_amdgcn_readfirstlane(wave_min_u32(n ? s : 0xFFFFFFFFu));
    const uint32_t hi = __builtin_amdgcn_readfirstlane(wave_max_u32(n ? e : 0u));
    float acc[GRAD_ROW];
#pragma unroll
    for (int c = 0; c < GRAD_ROW; ++c) acc[c] = 0.f;

    // Sparse rows (config C: 24 % of the rows are marked, config E: 4 %): the wave compacts the marked rows of
    // each 512-row window of its span into an LDS list (one 8-B load of marks per lane, a wave scan), then
    // streams the list in chunks of RS_ROWS marked rows: one HBM round trip per 128 marked rows instead of one
    // per 128 rows. Each Gaussian's marked rows are a contiguous run of the sorted list; the sums keep row order.
    uint32_t* s_list = s_list_all[wv];
    const uint64_t huges = __ballot(huge && idx < a.g_end && s < a.R);
    // the marks of window W, 8 rows per lane (row_valid is 256-B aligned and padded to a multiple of 256 B). W is
    // 0xFFFFFFF8 past the last window: the first test keeps W + 8 lane from wrapping into [0, hi).
#define RS_MARKS(W)                                                                                                    \
    ((W) < hi && (W) + RS_RPL * lane < hi                                                                             \
         ? *reinterpret_cast<const uint2*>(a.row_valid + (size_t)((W) + RS_RPL * lane))                               \
         : make_uint2(0u, 0u))
    uint32_t w0 = lo & ~(RS_RPL - 1u);  // lo > hi when the wave owns no rows
    uint2 f_cur = RS_MARKS(w0);
    while (w0 < hi) {
        // the next window starts at the first row of the wave's own Gaussians past this one: the spans of huge
        // Gaussians between them (summed by huge_row_sums; tens of thousands of rows at config E) are skipped. Its
        // marks are requested now, with this window's rows.
        const uint32_t nx = w0 + RS_WIN;
        const uint32_t w1 =
            __builtin_amdgcn_readfirstlane(wave_min_u32(n != 0 && e > nx ? max(s, nx) : 0xFFFFFFFFu)) & ~(RS_RPL - 1u);
        const uint2 f_next = RS_MARKS(w1);
        const uint32_t r0 = w0 + RS_RPL * lane;
        uint32_t m = 0;  // bit j: row r0 + j is marked, inside [lo, hi) and not a huge Gaussian's
        if (r0 < hi) {
            const uint32_t fw[2] = {f_cur.x, f_cur.y};
#pragma unroll
            for (uint32_t j = 0; j < RS_RPL; ++j) {
                const uint32_t r = r0 + j;
                const uint32_t byte = (fw[j >> 2] >> (8u * (j & 3u))) & 0xFFu;
                if (byte != 0 && r >= lo && r < hi) m |= 1u << j;
            }
            for (uint64_t hb = huges; hb; hb &= hb - 1) {  // rare: a huge Gaussian's rows inside the span
                const int jl = __builtin_ctzll(hb);
                const uint32_t hs = __builtin_amdgcn_readlane(s, jl), he = hs + __builtin_amdgcn_readlane(n_all, jl);
#pragma unroll
                for (uint32_t j = 0; j < RS_RPL; ++j)
                    if (r0 + j >= hs && r0 + j < he) m &= ~(1u << j);
            }
        }
        uint32_t total;
        const uint32_t k0 = wave_exclusive_scan_u32((uint32_t)__popc(m), lane, &total);
        uint32_t k = k0;
        for (uint32_t mm = m; mm; mm &= mm - 1) s_list[k++] = r0 + (uint32_t)__builtin_ctz(mm);
        // this lane's Gaussian's marked rows in the window: list positions [PA, PB), the marked rows before s and
        // before e, counted from the scan (the lane holding window row d has k0 before its rows and m over them)
        const uint32_t ds = s > w0 ? min(s - w0, RS_WIN) : 0u, de = e > w0 ? min(e - w0, RS_WIN) : 0u;
        const uint32_t la = min(ds / RS_RPL, 63u), lb = min(de / RS_RPL, 63u);
        const uint32_t ba = ds - la * RS_RPL, bb = de - lb * RS_RPL;  // 0 .. 8
        const uint32_t ka = (uint32_t)__shfl((int)k0, (int)la, 64), ma = (uint32_t)__shfl((int)m, (int)la, 64);
        const uint32_t kb = (uint32_t)__shfl((int)k0, (int)lb, 64), mb = (uint32_t)__shfl((int)m, (int)lb, 64);
        const uint32_t PA = n != 0 ? ka + (uint32_t)__popc(ma & ((1u << ba) - 1u)) : 0u;
        const uint32_t PB = n != 0 ? kb + (uint32_t)__popc(mb & ((1u << bb) - 1u)) : 0u;
        wave_sync();
        for (uint32_t c0 = 0; c0 < total; c0 += RS_ROWS) {
            const uint32_t c1 = min(total, c0 + RS_ROWS);
            float x[RS_Q][GRAD_ROW];
#pragma unroll
            for (int q = 0; q < RS_Q; ++q) {
                const uint32_t p = c0 + (uint32_t)q * 64u + lane;
#pragma unroll
                for (int c = 0; c < GRAD_ROW; ++c) x[q][c] = 0.f;
                add_marked_row(x[q], a.inst_grad, p < c1 ? s_list[p] : 0u, p < c1);
            }
#pragma unroll
            for (int q = 0; q < RS_Q; ++q)
#pragma unroll
                for (int c = 0; c < GRAD_ROW; ++c) s_rows[(q * 64 + lane) * GRAD_ROW + c] = x[q][c];
            // this lane's Gaussian's marked rows in the chunk: list positions [pa, pb)
            const uint32_t pa = min(max(PA, c0), c1), pb = min(max(PB, c0), c1);
            wave_sync();
            const bool is_long = pb - pa > RS_LONG;
            if (!is_long)
                for (uint32_t j = pa - c0; j < pb - c0; ++j)
#pragma unroll
                    for (int c = 0; c < GRAD_ROW; ++c) acc[c] += s_rows[j * GRAD_ROW + c];
            // long runs: the whole wave, one Gaussian at a time
            uint64_t longs = __ballot(is_long);
            while (longs) {
                const int jl = __builtin_ctzll(longs);
                longs &= longs - 1;
                const uint32_t sj = __builtin_amdgcn_readlane(pa, jl) - c0, ej = __builtin_amdgcn_readlane(pb, jl) - c0;
                float v[GRAD_ROW];
#pragma unroll
                for (int c = 0; c < GRAD_ROW; ++c) v[c] = 0.f;
#pragma unroll
                for (int q = 0; q < RS_Q; ++q) {
                    const uint32_t pos = (uint32_t)q * 64u + lane;
                    if (pos >= sj && pos < ej)
#pragma unroll
                        for (int c = 0; c < GRAD_ROW; ++c) v[c] += x[q][c];
                }
                float t8;
                const float tv = wave_sum9_rows(v, v[8], lane, &t8);  // lane l: total of value (l >> 3) & 7
#pragma unroll
                for (int c = 0; c < 8; ++c) {
                    const float tc = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, tv), 8 * c));
                    if ((int)lane == jl) acc[c] += tc;
                }
                if ((int)lane == jl) acc[8] += t8;
            }
            wave_sync();  // the next chunk overwrites the staging rows
        }
        wave_sync();  // the next window overwrites the list
        w0 = w1;
        f_cur = f_next;
    }
#undef RS_MARKS
    if (idx < a.g_end && !huge) {
        // a Gaussian without instances (culled: radii 0) has no sums to keep; gaussian_bwd does not read them
        if (n_all != 0) {
            float* out = a.row_sums + (size_t)idx * GRAD_ROW;
#pragma unroll
            for (int c = 0; c < GRAD_ROW; ++c) out[c] = acc[c];
        }
        // dL/dcolour (backward.cu:805-808 sums) is final here: the view-parallel exchange can gather it while
        // gaussian_bwd still runs (parallel.py); zeros for a culled Gaussian, which has no rows
#pragma unroll
        for (int c = 0; c < 3; ++c) a.dL_dcolor[(size_t)idx * 3 + c] = acc[6 + c];
    }
}

#ifndef OMR_GBWD_MINW
#define OMR_GBWD_MINW 1
#endif


// A Gaussian's small outputs (every [P][k] gradient but dL_dsh and dL_dcolor), held in registers until its wave
// stores them as contiguous spans through LDS (wave_small_store; the MC == 16 kernel), or written lane by lane (so ==
// nullptr).
struct SmallOut {
    float m2[2], op, con[3], cov[6], px[3], py[3], m3[3], sc[3], rot[4];
};

// Everything after the row sums for one visible Gaussian idx (radii > 0). dsh4: where the MC == 16 dL_dsh row goes.
template <int CAM, int MC>
__device__ __forceinline__ void gaussian_bwd_point(const GaussBwdArgs& a, int idx, float (&g)[GRAD_ROW],
                                                   const float4* sh4, float4* dsh4, const float* jac = nullptr,
                                                   SmallOut* so = nullptr, const GIn* gin = nullptr)
{
    const int Mr = MC > 0 ? MC : a.M;
    // 1. this Gaussian's summed instance rows
    if (so) {
        so->m2[0] = g[0];
        so->m2[1] = g[1];
        so->op = g[5];
        so->con[0] = g[2];
        so->con[1] = g[3];
        so->con[2] = g[4];
    } else {
        a.dL_dmean2D[3 * idx + 0] = g[0];
        a.dL_dmean2D[3 * idx + 1] = g[1];
        a.dL_dmean2D[3 * idx + 2] = 0.f;
        a.dL_dopacity[idx] = g[5];  // dL_dcolor = g[6..8] was written by row_sum_kernel
        if (a.dL_dconic) {
            a.dL_dconic[4 * idx + 0] = g[2];
            a.dL_dconic[4 * idx + 1] = g[3];
            a.dL_dconic[4 * idx + 2] = 0.f;
            a.dL_dconic[4 * idx + 3] = g[4];
        }
    }

    // 2. covariance backward
    const F3 mean = gin ? gin->mean : F3{a.means3D[3 * idx], a.means3D[3 * idx + 1], a.means3D[3 * idx + 2]};
    const float* v = a.viewmatrix;
    float c3[6];
    float4 q = make_float4(0.f, 0.f, 0.f, 0.f);
    float sc[3] = {0.f, 0.f, 0.f};
    if (a.scales) {
        if (gin) {
            q = gin->q;
#pragma unroll
            for (int k = 0; k < 3; ++k) sc[k] = gin->s[k];
        } else {
            if ((reinterpret_cast<uintptr_t>(a.rotations) & 15u) == 0) q = reinterpret_cast<const float4*>(a.rotations)[idx];
            else q = make_float4(a.rotations[4 * idx], a.rotations[4 * idx + 1], a.rotations[4 * idx + 2], a.rotations[4 * idx + 3]);
#pragma unroll
            for (int k = 0; k < 3; ++k) sc[k] = a.scales[3 * idx + k];
        }
    }
    if (a.cov3D_precomp) {
#pragma unroll
        for (int k = 0; k < 6; ++k) c3[k] = a.cov3D_precomp[6 * idx + k];
    } else {
        cov3d_forward(sc[0], sc[1], sc[2], a.scale_modifier, q, c3);
    }
    const float tx = v[0] * mean.x + v[4] * mean.y + v[8] * mean.z + v[12];
    const float ty = v[1] * mean.x + v[5] * mean.y + v[9] * mean.z + v[13];
    const float tz = v[2] * mean.x + v[6] * mean.y + v[10] * mean.z + v[14];
    const float W[3][3] = {{v[0], v[4], v[8]}, {v[1], v[5], v[9]}, {v[2], v[6], v[10]}};
    const F3 dL_dconic = {g[2], g[3], g[4]};
    float dcov[6], dT0[3], dT1[3];
    F3 dmean;           // dL/dmean3D accumulator
    F3 dpx = {0, 0, 0}, dpy = {0, 0, 0};
    if constexpr (CAM == CAM_LONLAT) {
        const float txtx = tx * tx, tyty = ty * ty, tztz = tz * tz, txtytz = tx * ty * tz;
        const float trxztrxz = txtx + tztz;
        const float trxztrxz_inv = 1.0f / (trxztrxz + 0.0000001f);
        const float trxztrxztrxztrxz_inv = trxztrxz_inv * trxztrxz_inv;
        const float trxz = sqrtf(trxztrxz);
        const float trxz_inv = 1.0f / (trxz + 0.0000001f);
        const float trtr = trxztrxz + tyty;
        const float trtr_inv = 1.0f / (trtr + 0.0000001f);
        const float trtrtrtr_inv = trtr_inv * trtr_inv;
        const float trxz_trtrtrtr_inv = trxz_inv * trtrtrtr_inv;
        const float trxztrxztrxz_trtrtrtr_inv = trxztrxz_inv * trxz_trtrtrtr_inv;
        const float tyty_minus_trxztrxz = tyty - trxztrxz;
        const float W_div_2pi = (float)a.W * 0.5f * INV_PI;
        const float H_div_pi = (float)a.H * INV_PI;
        const float dpx_dtx = W_div_2pi * tz * trxztrxz_inv;
        const float dpx_dtz = -W_div_2pi * tx * trxztrxz_inv;
        const float dpy_dtx = -H_div_pi * tx * ty * trxz_inv * trtr_inv;
        const float dpy_dty = H_div_pi * trxz * trtr_inv;
        const float dpy_dtz = -H_div_pi * tz * ty * trxz_inv * trtr_inv;
        dpx = {dpx_dtx, 0.f, dpx_dtz};
        dpy = {dpy_dtx, dpy_dty, dpy_dtz};
        const float J0[3] = {dpx_dtx, 0.f, dpx_dtz}, J1[3] = {dpy_dtx, dpy_dty, dpy_dtz};
        float T0[3], T1[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            T0[i] = W[0][i] * J0[0] + W[1][i] * J0[1] + W[2][i] * J0[2];
            T1[i] = W[0][i] * J1[0] + W[1][i] * J1[1] + W[2][i] * J1[2];
        }
        cov2d_backward(T0, T1, c3, dL_dconic, dcov, dT0, dT1);
        const float dL_dJ00 = W[0][0] * dT0[0] + W[0][1] * dT0[1] + W[0][2] * dT0[2];
        const float dL_dJ02 = W[2][0] * dT0[0] + W[2][1] * dT0[1] + W[2][2] * dT0[2];
        const float dL_dJ10 = W[0][0] * dT1[0] + W[0][1] * dT1[1] + W[0][2] * dT1[2];
        const float dL_dJ11 = W[1][0] * dT1[0] + W[1][1] * dT1[1] + W[1][2] * dT1[2];
        const float dL_dJ12 = W[2][0] * dT1[0] + W[2][1] * dT1[1] + W[2][2] * dT1[2];
        // second derivatives of the lonlat projection (backward.cu:455-475; supp.pdf App. A)
        const float temp1 = H_div_pi * tyty_minus_trxztrxz * trxz_trtrtrtr_inv;
        const float temp2 = H_div_pi * txtytz * (trtr + 2.0f * trxztrxz) * trxztrxztrxz_trtrtrtr_inv;
        const float temp3 = W_div_2pi * (txtx - tztz) * trxztrxztrxztrxz_inv;
        const float temp4 = W_div_2pi * 2.0f * tx * tz * trxztrxztrxztrxz_inv;
        const float temp5 = H_div_pi * ty * trxztrxztrxz_trtrtrtr_inv;
        const float dL_dtx = -dL_dJ00 * temp4 + dL_dJ02 * temp3 + dL_dJ10 * temp5 * (2.0f * txtx * trxztrxz - tztz * trtr) +
                             dL_dJ11 * tx * temp1 + dL_dJ12 * temp2;
        const float dL_dty = dL_dJ10 * tx * temp1 - dL_dJ11 * H_div_pi * 2.0f * trxz * ty * trtrtrtr_inv + dL_dJ12 * tz * temp1;
        const float dL_dtz = dL_dJ00 * temp3 + dL_dJ02 * temp4 + dL_dJ10 * temp2 + dL_dJ11 * tz * temp1 +
                             dL_dJ12 * temp5 * (2.0f * tztz * trxztrxz - txtx * trtr);
        const float3 m = transformVec4x3Transpose({dL_dtx, dL_dty, dL_dtz}, v);
        dmean = {m.x, m.y, m.z};
        // projection part (backward.cu:643-660)
        const float dL_dpx = g[0] * (2.0f / (float)a.W);
        const float dL_dpy = g[1] * (2.0f / (float)a.H);
        const float3 mp = transformVec4x3Transpose({dL_dpx * dpx.x + dL_dpy * dpy.x, dL_dpx * dpx.y + dL_dpy * dpy.y,
                                                    dL_dpx * dpx.z + dL_dpy * dpy.z}, v);
        dmean.x += mp.x;
        dmean.y += mp.y;
        dmean.z += mp.z;
    } else {
        const float h_x = a.focal_x, h_y = a.focal_y;
        const float limx = 1.3f * a.tan_fovx, limy = 1.3f * a.tan_fovy;
        const float txtz = tx / tz, tytz = ty / tz;
        const float txc = fminf(limx, fmaxf(-limx, txtz)) * tz;
        const float tyc = fminf(limy, fmaxf(-limy, tytz)) * tz;
        const float x_grad_mul = txtz < -limx || txtz > limx ? 0.f : 1.f;
        const float y_grad_mul = tytz < -limy || tytz > limy ? 0.f : 1.f;
        const float J0[3] = {h_x / tz, 0.f, -(h_x * txc) / (tz * tz)}, J1[3] = {0.f, h_y / tz, -(h_y * tyc) / (tz * tz)};
        float T0[3], T1[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            T0[i] = W[0][i] * J0[0] + W[1][i] * J0[1] + W[2][i] * J0[2];
            T1[i] = W[0][i] * J1[0] + W[1][i] * J1[1] + W[2][i] * J1[2];
        }
        cov2d_backward(T0, T1, c3, dL_dconic, dcov, dT0, dT1);
        const float dL_dJ00 = W[0][0] * dT0[0] + W[0][1] * dT0[1] + W[0][2] * dT0[2];
        const float dL_dJ02 = W[2][0] * dT0[0] + W[2][1] * dT0[1] + W[2][2] * dT0[2];
        const float dL_dJ11 = W[1][0] * dT1[0] + W[1][1] * dT1[1] + W[1][2] * dT1[2];
        const float dL_dJ12 = W[2][0] * dT1[0] + W[2][1] * dT1[1] + W[2][2] * dT1[2];
        const float itz = 1.f / tz, tz2 = itz * itz, tz3 = tz2 * itz;
        const float dL_dtx = x_grad_mul * -h_x * tz2 * dL_dJ02;
        const float dL_dty = y_grad_mul * -h_y * tz2 * dL_dJ12;
        const float dL_dtz = -h_x * tz2 * dL_dJ00 - h_y * tz2 * dL_dJ11 + (2 * h_x * txc) * tz3 * dL_dJ02 + (2 * h_y * tyc) * tz3 * dL_dJ12;
        const float3 m = transformVec4x3Transpose({dL_dtx, dL_dty, dL_dtz}, v);
        dmean = {m.x, m.y, m.z};
        // projection part (backward.cu:583-599)
        const float* proj = a.projmatrix;
        const float4 m_hom = transformPoint4x4({mean.x, mean.y, mean.z}, proj);
        const float m_w = 1.0f / (m_hom.w + 0.0000001f);
        const float mul1 = (proj[0] * mean.x + proj[4] * mean.y + proj[8] * mean.z + proj[12]) * m_w * m_w;
        const float mul2 = (proj[1] * mean.x + proj[5] * mean.y + proj[9] * mean.z + proj[13]) * m_w * m_w;
        dmean.x += (proj[0] * m_w - proj[3] * mul1) * g[0] + (proj[1] * m_w - proj[3] * mul2) * g[1];
        dmean.y += (proj[4] * m_w - proj[7] * mul1) * g[0] + (proj[5] * m_w - proj[7] * mul2) * g[1];
        dmean.z += (proj[8] * m_w - proj[11] * mul1) * g[0] + (proj[9] * m_w - proj[11] * mul2) * g[1];
    }
    if (so) {
#pragma unroll
        for (int k = 0; k < 6; ++k) so->cov[k] = dcov[k];
        so->px[0] = dpx.x; so->px[1] = dpx.y; so->px[2] = dpx.z;
        so->py[0] = dpy.x; so->py[1] = dpy.y; so->py[2] = dpy.z;
    } else {
#pragma unroll
        for (int k = 0; k < 6; ++k) a.dL_dcov3D[6 * idx + k] = dcov[k];
        if (a.dpx_dt) {
            a.dpx_dt[3 * idx + 0] = dpx.x; a.dpx_dt[3 * idx + 1] = dpx.y; a.dpx_dt[3 * idx + 2] = dpx.z;
            a.dpy_dt[3 * idx + 0] = dpy.x; a.dpy_dt[3 * idx + 1] = dpy.y; a.dpy_dt[3 * idx + 2] = dpy.z;
        }
    }

    // 3. SH backward
    if (a.shs) {
        const F3 dm = sh_backward<MC>(idx, a.D, a.M, mean, a.campos, a.shs, sh4, gin ? gin->clamp : a.clamped[idx],
                                      F3{g[6], g[7], g[8]}, a.dL_dsh, dsh4, gin ? nullptr : jac, gin, gin && jac);
        dmean.x += dm.x;
        dmean.y += dm.y;
        dmean.z += dm.z;
    } else if (a.dL_dsh) {
        if constexpr (MC == 16) {
#pragma unroll
            for (int q = 0; q < 12; ++q) dsh4[q] = make_float4(0.f, 0.f, 0.f, 0.f);
        } else {
            for (int c = 0; c < Mr * 3; ++c) a.dL_dsh[(size_t)idx * Mr * 3 + c] = 0.f;
        }
    }
    // 4. scale / rotation backward
    float ds[3] = {0.f, 0.f, 0.f}, dr[4] = {0.f, 0.f, 0.f, 0.f};
    if (a.scales) cov3d_backward(sc[0], sc[1], sc[2], a.scale_modifier, q, dcov, ds, dr);
    if (so) {
        so->m3[0] = dmean.x; so->m3[1] = dmean.y; so->m3[2] = dmean.z;
#pragma unroll
        for (int k = 0; k < 3; ++k) so->sc[k] = ds[k];
#pragma unroll
        for (int k = 0; k < 4; ++k) so->rot[k] = dr[k];
    } else {
        a.dL_dmean3D[3 * idx + 0] = dmean.x;
        a.dL_dmean3D[3 * idx + 1] = dmean.y;
        a.dL_dmean3D[3 * idx + 2] = dmean.z;
#pragma unroll
        for (int k = 0; k < 3; ++k) a.dL_dscale[3 * idx + k] = ds[k];
#pragma unroll
        for (int k = 0; k < 4; ++k) a.dL_drot[4 * idx + k] = dr[k];
    }
}

// backward.cu:805-840 targets etc. of a culled Gaussian (radii == 0): every output zero (the caller allocates the
// gradient tensors without zero-filling them)
template <int MC>
__device__ __forceinline__ void gaussian_bwd_culled(const GaussBwdArgs& a, int idx, float4* dsh4, SmallOut* so = nullptr)
{
    const int Mr = MC > 0 ? MC : a.M;
    if (so) {
        // the caller zeroed *so
        if (a.dL_dsh && MC == 16)
#pragma unroll
            for (int q = 0; q < 12; ++q) dsh4[q] = make_float4(0.f, 0.f, 0.f, 0.f);
        return;
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        a.dL_dmean2D[3 * idx + c] = 0.f;  // dL_dcolor: zeros from row_sum_kernel
        a.dL_dmean3D[3 * idx + c] = 0.f;
        a.dL_dscale[3 * idx + c] = 0.f;
    }
    a.dL_dopacity[idx] = 0.f;
#pragma unroll
    for (int c = 0; c < 6; ++c) a.dL_dcov3D[6 * idx + c] = 0.f;
#pragma unroll
    for (int c = 0; c < 4; ++c) a.dL_drot[4 * idx + c] = 0.f;
    if (a.dL_dconic)
#pragma unroll
        for (int c = 0; c < 4; ++c) a.dL_dconic[4 * idx + c] = 0.f;
    if (a.dL_dsh) {
        if constexpr (MC == 16) {
#pragma unroll
            for (int q = 0; q < 12; ++q) dsh4[q] = make_float4(0.f, 0.f, 0.f, 0.f);
        } else {
            for (int c = 0; c < Mr * 3; ++c) a.dL_dsh[(size_t)idx * Mr * 3 + c] = 0.f;
        }
    }
    if (a.dpx_dt)
#pragma unroll
        for (int c = 0; c < 3; ++c) a.dpx_dt[3 * idx + c] = a.dpy_dt[3 * idx + c] = 0.f;
}

// The wave's small outputs as contiguous spans: each lane parks its values in the LDS image ([array][lane][k]), then
// every [P][k] array gets its 64 k floats from wave_first on as 16-B stores (1 KiB per instruction) where the span is
// 16-B aligned, else as dword stores (256 B per instruction), instead of k dword stores per lane 4k bytes apart.
// n: the wave's valid Gaussians (a tail wave stores only theirs).
__device__ __forceinline__ void wave_small_store(const GaussBwdArgs& a, const SmallOut& so, int wave_first, int n,
                                                 float* img, uint32_t lane)
{
    constexpr int O_M2 = 0, O_OP = O_M2 + 64 * 3, O_CON = O_OP + 64, O_COV = O_CON + 64 * 4, O_PX = O_COV + 64 * 6,
                  O_PY = O_PX + 64 * 3, O_M3 = O_PY + 64 * 3, O_SC = O_M3 + 64 * 3, O_ROT = O_SC + 64 * 3;
    float* m2 = img + O_M2 + lane * 3;
    m2[0] = so.m2[0]; m2[1] = so.m2[1]; m2[2] = 0.f;
    img[O_OP + lane] = so.op;
    float* con = img + O_CON + lane * 4;
    con[0] = so.con[0]; con[1] = so.con[1]; con[2] = 0.f; con[3] = so.con[2];
#pragma unroll
    for (int k = 0; k < 6; ++k) img[O_COV + lane * 6 + k] = so.cov[k];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        img[O_PX + lane * 3 + k] = so.px[k];
        img[O_PY + lane * 3 + k] = so.py[k];
        img[O_M3 + lane * 3 + k] = so.m3[k];
        img[O_SC + lane * 3 + k] = so.sc[k];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) img[O_ROT + lane * 4 + k] = so.rot[k];
    wave_sync();
    auto span = [&](float* dst, int off, int K) {
        if (!dst) return;
        dst += (size_t)wave_first * K;
        const int nf = n * K;
        if (((reinterpret_cast<uintptr_t>(dst) & 15u) == 0) && (nf & 3) == 0) {  // wave-uniform
            float4* d4 = reinterpret_cast<float4*>(dst);
            const float4* s4 = reinterpret_cast<const float4*>(img + off);
            for (int j = (int)lane; j < nf / 4; j += 64) d4[j] = s4[j];
        } else {
            for (int j = (int)lane; j < nf; j += 64) dst[j] = img[off + j];
        }
    };
    span(a.dL_dmean2D, O_M2, 3);
    span(a.dL_dopacity, O_OP, 1);
    span(a.dL_dconic, O_CON, 4);
    span(a.dL_dcov3D, O_COV, 6);
    span(a.dpx_dt, O_PX, 3);
    span(a.dpy_dt, O_PY, 3);
    span(a.dL_dmean3D, O_M3, 3);
    span(a.dL_dscale, O_SC, 3);
    span(a.dL_drot, O_ROT, 4);
}

// One wave per 64 consecutive Gaussians. For MC == 16 (launch_gaussian_backward checks the 16-B alignment) the
// wave reads its 64 SH rows and writes its 64 dL_dsh rows as contiguous 12-KiB spans through LDS (wave_rows.h):
// each lane reads its SH row from the image where it needs it and overwrites the same row with its dL_dsh row
// (only that lane touches it), so one image serves both directions. SH rows of culled Gaussians are not read;
// their dL_dsh rows are written as zeros.
template <int CAM, int MC>
__global__ __launch_bounds__(256, OMR_GBWD_MINW) void gaussian_bwd_kernel(GaussBwdArgs a)
{
    constexpr int SH_F4 = 12;
    constexpr bool STAGED = MC == 16;
    __shared__ float4 s_stage[4][STAGED ? stage_f4<SH_F4>() : 1];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const int wave_first = a.g_begin + (int)(blockIdx.x * 256u + wv * 64u);
    if (wave_first >= a.g_end) return;  // wave-uniform
    const int idx = wave_first + (int)lane;
    float g[GRAD_ROW];
    float4 co = make_float4(0.f, 0.f, 0.f, 0.f);  // conic + opacity of the render record (raw-moment rows)
    const bool valid = idx < a.g_end;
    const bool vis = valid && a.radii[idx] > 0;
    // the forward stored dRGB/ddir (sh_jac) when it staged these rows: the SH rows are then not needed here, unless
    // this backward was handed other SH, means or campos than that forward (raster_common.h: sh_jac_key)
    const bool jac = STAGED && a.shs && a.sh_jac && a.campos &&
                     *a.jac_flag == sh_jac_key(a.shs, a.means3D, __float_as_uint(a.campos[0]),
                                               __float_as_uint(a.campos[1]), __float_as_uint(a.campos[2]));  // uniform
    // sums and conic are read for visible Gaussians only (radii > 0 implies instances, preprocess.hip, so
    // row_sum_kernel wrote the row): at config E pinhole 88 % of the Gaussians are culled. The MC == 16 kernel reads
    // every other per-Gaussian input with them (GIn)
    GIn gin;
    if (vis) {
#pragma unroll
        for (int c = 0; c < GRAD_ROW; ++c) g[c] = a.row_sums[(size_t)idx * GRAD_ROW + c];
        co = a.conic_op[idx];
        if constexpr (STAGED) {
            gin.mean = F3{a.means3D[3 * idx], a.means3D[3 * idx + 1], a.means3D[3 * idx + 2]};
            if (a.scales) {
#pragma unroll
                for (int k = 0; k < 3; ++k) gin.s[k] = a.scales[3 * idx + k];
                if ((reinterpret_cast<uintptr_t>(a.rotations) & 15u) == 0) gin.q = reinterpret_cast<const float4*>(a.rotations)[idx];
                else gin.q = make_float4(a.rotations[4 * idx], a.rotations[4 * idx + 1], a.rotations[4 * idx + 2], a.rotations[4 * idx + 3]);
            }
            if (a.shs) gin.clamp = a.clamped[idx];
            if (jac)
#pragma unroll
                for (int k = 0; k < 9; ++k) gin.jac[k] = a.sh_jac[(size_t)idx * 9 + k];
        }
    }
    float4* stage = s_stage[wv];
    // MC == 16 only (the MC == 0 path reads and writes the rows itself, and skips the write for dL_dsh == NULL)
    float4* dsh4 = STAGED ? stage + lane * stage_stride<SH_F4>() : nullptr;
    const float4* sh4 = dsh4;
    if constexpr (STAGED) {
        if (a.shs && !jac) {
            const int nf4 = (3 * (a.D + 1) * (a.D + 1) + 3) >> 2;
            wave_rows_load<SH_F4>(reinterpret_cast<const float4*>(a.shs) + (size_t)wave_first * SH_F4, __ballot(vis), nf4,
                                  stage, lane);
            wave_sync();
        }
    }
    // pinhole views store the small outputs as spans (wave_small_store): their waves are mostly culled Gaussians, whose
    // zeros are most of the bytes (E pinhole gaussian_bwd 0.445 -> 0.396 ms); at lonlat views, whose Gaussians are
    // nearly all visible, the LDS round trip at the end of the chain costs more than the coalescing gains (C 0.081 ->
    // 0.089, E 0.376 -> 0.386 ms), so they keep the lane stores (profiles/r05ai_ab.txt)
    constexpr bool SPANS = STAGED && CAM == CAM_PINHOLE;
    SmallOut so;
    if constexpr (SPANS) {  // a culled Gaussian's values; a visible one overwrites them all
        so.m2[0] = so.m2[1] = so.op = 0.f;
#pragma unroll
        for (int k = 0; k < 3; ++k) so.con[k] = so.px[k] = so.py[k] = so.m3[k] = so.sc[k] = 0.f;
#pragma unroll
        for (int k = 0; k < 6; ++k) so.cov[k] = 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k) so.rot[k] = 0.f;
    }
    SmallOut* sop = SPANS ? &so : nullptr;
    if (vis) {
        raw_row_to_grads(g, co, a.W, a.H);
        gaussian_bwd_point<CAM, MC>(a, idx, g, sh4, dsh4, jac ? a.sh_jac + (size_t)idx * 9 : nullptr, sop,
                                    STAGED ? &gin : nullptr);
    }
    else if (valid) gaussian_bwd_culled<MC>(a, idx, dsh4, sop);
    if constexpr (STAGED) {
        if (a.dL_dsh) {
            wave_sync();
            wave_rows_store<SH_F4>(reinterpret_cast<float4*>(a.dL_dsh) + (size_t)wave_first * SH_F4, __ballot(valid),
                                   stage, lane);
        }
        if constexpr (SPANS) {
            wave_sync();  // the image's dL_dsh rows are read: it now stages the small outputs
            wave_small_store(a, so, wave_first, min(64, a.g_end - wave_first), reinterpret_cast<float*>(stage), lane);
        }
    }
}

// View-parallel data parallelism (parallel.py): the sum over n views of dL/dsh, rebuilt from each view's colour
// gradient. Per view v, backward.cu:30-151 gives dL/dsh_k = basis_k(dir_v) * dRGB_v, dRGB_v = dL/dcolour_v masked
// by the forward's clamp bits; the basis and the clamp bits are functions of (mean, SH row, campos_v), which every
// rank holds. So ranks exchange dL/dcolour (12 B per Gaussian and view) and campos instead of all-reducing the
// 192-B SH gradient, and each rebuilds the sum with the per-view backward's own arithmetic (sh_eval.h), summing the
// views in index order. A view whose colour gradient is zero (culled there) adds nothing and is skipped.
template <int MC>
__global__ __launch_bounds__(256) void sh_grad_from_colors_kernel(int P, int D, int M, int nviews,
                                                                  const float* means3D, const float* shs,
                                                                  const float* campos, size_t cp_stride,
                                                                  const float* dL_dcolors, size_t dc_stride,
                                                                  float* dL_dsh)
{
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= P) return;
    const int Mr = MC > 0 ? MC : M;
    const int nk = min(16, min(Mr, (D + 1) * (D + 1)));
    const float* row = shs + (size_t)idx * Mr * 3;
    float shv[48];
#pragma unroll
    for (int f = 0; f < 48; ++f) shv[f] = 0.f;
    if constexpr (MC == 16) {
        const int nf4 = (3 * nk + 3) >> 2;
#pragma unroll
        for (int q = 0; q < 12; ++q) {
            if (q < nf4) {
                const float4 v = reinterpret_cast<const float4*>(row)[q];
                shv[4 * q] = v.x;
                shv[4 * q + 1] = v.y;
                shv[4 * q + 2] = v.z;
                shv[4 * q + 3] = v.w;
            }
        }
    } else {
        for (int f = 0; f < 3 * nk; ++f) shv[f] = row[f];
    }
    float acc[48];
#pragma unroll
    for (int f = 0; f < 48; ++f) acc[f] = 0.f;
    const float px = means3D[3 * idx], py = means3D[3 * idx + 1], pz = means3D[3 * idx + 2];
    for (int v = 0; v < nviews; ++v) {
        const float* dc = dL_dcolors + (size_t)v * dc_stride + (size_t)idx * 3;
        float d[3] = {dc[0], dc[1], dc[2]};
        if (d[0] == 0.f && d[1] == 0.f && d[2] == 0.f) continue;
        float x, y, z;
        sh_direction(px, py, pz, campos + (size_t)v * cp_stride, x, y, z);
        float rgb[3];
        uint8_t clamp_bits;
        sh_to_rgb(D, x, y, z, shv, rgb, clamp_bits);
#pragma unroll
        for (int c = 0; c < 3; ++c)
            if (clamp_bits & (1u << c)) d[c] = 0.f;
        float coef[16];
        sh_basis(D, x, y, z, coef);
#pragma unroll
        for (int f = 0; f < 48; ++f) acc[f] += coef[f / 3] * d[f % 3];
    }
    float* out = dL_dsh + (size_t)idx * Mr * 3;
    if constexpr (MC == 16) {
        float4* o4 = reinterpret_cast<float4*>(out);
#pragma unroll
        for (int q = 0; q < 12; ++q) {
            float w[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) w[e] = (4 * q + e) / 3 < nk ? acc[4 * q + e] : 0.f;
            o4[q] = make_float4(w[0], w[1], w[2], w[3]);
        }
    } else {
        for (int f = 0; f < Mr * 3; ++f) out[f] = f / 3 < nk ? acc[f < 48 ? f : 0] : 0.f;
    }
}

}  // namespace

void launch_sh_grad_from_colors(int P, int D, int M, int nviews, const float* means3D, const float* shs,
                                const float* campos, size_t cp_stride, const float* dL_dcolors, size_t dc_stride,
                                float* dL_dsh, hipStream_t s)
{
    if (P <= 0) return;
    const bool m16 = M == 16 && (reinterpret_cast<uintptr_t>(shs) % 16) == 0 &&
                     (reinterpret_cast<uintptr_t>(dL_dsh) % 16) == 0;
    const dim3 grid(div_up(P, 256));
    if (m16)
        sh_grad_from_colors_kernel<16><<<grid, 256, 0, s>>>(P, D, M, nviews, means3D, shs, campos, cp_stride, dL_dcolors,
                                                            dc_stride, dL_dsh);
    else
        sh_grad_from_colors_kernel<0><<<grid, 256, 0, s>>>(P, D, M, nviews, means3D, shs, campos, cp_stride, dL_dcolors,
                                                           dc_stride, dL_dsh);
}

void launch_row_sums(int g_begin, int g_end, bool huge, const uint32_t* row_first, const uint32_t* tiles_touched,
                     const uint32_t* huge_list, const uint32_t* huge_count, const float* inst_grad,
                     const uint8_t* row_valid, uint32_t R, float* row_sums, float* dL_dcolor, hipStream_t s)
{
    if (g_end <= g_begin && !huge) return;
    RowSumArgs a;
    a.g_begin = g_begin;
    a.g_end = g_end;
    a.huge_blocks = huge ? RS_HUGE_BLOCKS : 0u;
    a.R = R;
    const uint32_t main_blocks = g_end > g_begin ? div_up(g_end - g_begin, 256) : 0u;  // after the huge workgroups
    a.row_first = row_first;
    a.tiles_touched = tiles_touched;
    a.huge_list = huge_list;
    a.huge_count = huge_count;
    a.inst_grad = inst_grad;
    a.row_valid = row_valid;
    a.row_sums = row_sums;
    a.dL_dcolor = dL_dcolor;
    row_sum_kernel<<<main_blocks + a.huge_blocks, 256, 0, s>>>(a);
}

void launch_gaussian_backward(int camera_type, const GaussBwdArgs& a, hipStream_t s, hipEvent_t ev_start,
                              hipEvent_t ev_stop)
{
    if (a.g_end <= a.g_begin) return;
    const dim3 grid(div_up(a.g_end - a.g_begin, 256));
    const bool m16 = a.M == 16 && (reinterpret_cast<uintptr_t>(a.dL_dsh) % 16) == 0 &&
                     (reinterpret_cast<uintptr_t>(a.shs) % 16) == 0;
    auto k = camera_type == CAM_LONLAT ? (m16 ? gaussian_bwd_kernel<CAM_LONLAT, 16> : gaussian_bwd_kernel<CAM_LONLAT, 0>)
                                       : (m16 ? gaussian_bwd_kernel<CAM_PINHOLE, 16> : gaussian_bwd_kernel<CAM_PINHOLE, 0>);
    if (ev_start || ev_stop) hipExtLaunchKernelGGL(k, grid, dim3(256), 0, s, ev_start, ev_stop, 0, a);
    else k<<<grid, 256, 0, s>>>(a);
}

}  // namespace omr

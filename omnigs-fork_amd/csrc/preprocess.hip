// preprocess.hip — per-Gaussian forward preprocess for the lonlat (camera_type 3) and pinhole (camera_type 1)
// projections, gfx950.
//
// Follows cuda_rasterizer/forward.cu:593-703 (preprocessLonlatCUDA) and :231-340 (preprocessCUDA):
// cull, project, 3D covariance from scale+rotation, 2D covariance through the projection Jacobian, conic,
// radius, tile rect, SH -> RGB. Compiled with -ffp-contract=off and evaluated in the reference's expression
// order (glm column-major products, left-to-right sums), so radii, pixel centres, conics, tile rects and the
// depth sort keys are bit-identical to the CPU oracle.
//
// MI355X notes: one wave64 per 64 Gaussians; the stores are SoA so every output array is written with
// contiguous lanes; the depth sort's first-pass keys/values are written here directly (no extra pass).
// HBM per Gaussian (D=3): reads 12 (xyz) + 12 (scale) + 16 (rot) + 4 (opacity) + 192 (SH) = 236 B,
// writes 8 + 16 + 16 + 4 + 1 + 4 + 4 (radius) + 8 (sort key/value) = 61 B.
#include "kernels.h"
#include "sh_eval.h"
#include "wave_rows.h"

namespace omr {

#pragma clang fp contract(off)

namespace {

constexpr float INV_PI = 0.318309886183790671537767526745028724f;  // M_1_PIf32
constexpr float TWO_INV_PI = 0.636619772367581343075535053490057448f;  // M_2_PIf32

// forward.cu:194-228. Sigma = (S R)^T (S R) written out entry by entry in glm's evaluation order.
__device__ __forceinline__ void cov3d_from_scale_rot(float sx, float sy, float sz, float mod, float4 q, float* c)
{
    const float s0 = mod * sx, s1 = mod * sy, s2 = mod * sz;
    const float r = q.x, x = q.y, y = q.z, z = q.w;
    // R columns (glm::mat3 constructor fills column by column)
    const float R00 = 1.f - 2.f * (y * y + z * z), R01 = 2.f * (x * y - r * z), R02 = 2.f * (x * z + r * y);
    const float R10 = 2.f * (x * y + r * z), R11 = 1.f - 2.f * (x * x + z * z), R12 = 2.f * (y * z - r * x);
    const float R20 = 2.f * (x * z - r * y), R21 = 2.f * (y * z + r * x), R22 = 1.f - 2.f * (x * x + y * y);
    // M = S * R: M[j][i] = S[0][i]*R[j][0] + S[1][i]*R[j][1] + S[2][i]*R[j][2], S diagonal (zeros kept)
    float M[3][3];
    const float Rc[3][3] = {{R00, R01, R02}, {R10, R11, R12}, {R20, R21, R22}};
    const float S[3][3] = {{s0, 0.f, 0.f}, {0.f, s1, 0.f}, {0.f, 0.f, s2}};
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int i = 0; i < 3; ++i) M[j][i] = S[0][i] * Rc[j][0] + S[1][i] * Rc[j][1] + S[2][i] * Rc[j][2];
    // Sigma = M^T M: Sigma[j][i] = M[i][0]*M[j][0] + M[i][1]*M[j][1] + M[i][2]*M[j][2]
    auto sig = [&](int j, int i) { return M[i][0] * M[j][0] + M[i][1] * M[j][1] + M[i][2] * M[j][2]; };
    c[0] = sig(0, 0);
    c[1] = sig(0, 1);
    c[2] = sig(0, 2);
    c[3] = sig(1, 1);
    c[4] = sig(1, 2);
    c[5] = sig(2, 2);
}

// cov = T^T Vrk T with T = W J (forward.cu:113-126 / :174-188); J has a zero third column.
// T[j][i] = W[0][i]*J[j][0] + W[1][i]*J[j][1] + W[2][i]*J[j][2]; W[c] = (v[c], v[c+4], v[c+8]).
__device__ __forceinline__ float3 cov2d_from_J(const float* v, const float J0[3], const float J1[3], const float* c3)
{
    const float W[3][3] = {{v[0], v[4], v[8]}, {v[1], v[5], v[9]}, {v[2], v[6], v[10]}};
    float T0[3], T1[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        T0[i] = W[0][i] * J0[0] + W[1][i] * J0[1] + W[2][i] * J0[2];
        T1[i] = W[0][i] * J1[0] + W[1][i] * J1[1] + W[2][i] * J1[2];
    }
    const float V[3][3] = {{c3[0], c3[1], c3[2]}, {c3[1], c3[3], c3[4]}, {c3[2], c3[4], c3[5]}};
    // B = T^T * Vrk: B[j][i] = T[i][0]*V[j][0] + T[i][1]*V[j][1] + T[i][2]*V[j][2], rows i = 0, 1
    float B0[3], B1[3];  // B[j][0], B[j][1]
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        B0[j] = T0[0] * V[j][0] + T0[1] * V[j][1] + T0[2] * V[j][2];
        B1[j] = T1[0] * V[j][0] + T1[1] * V[j][1] + T1[2] * V[j][2];
    }
    // cov = B * T: cov[j][i] = B[0][i]*T[j][0] + B[1][i]*T[j][1] + B[2][i]*T[j][2]
    float c00 = B0[0] * T0[0] + B0[1] * T0[1] + B0[2] * T0[2];
    const float c01 = B1[0] * T0[0] + B1[1] * T0[1] + B1[2] * T0[2];
    float c11 = B1[0] * T1[0] + B1[1] * T1[1] + B1[2] * T1[2];
    c00 += 0.3f;
    c11 += 0.3f;
    return {c00, c01, c11};
}

// The inputs preprocess_point reads, loaded up front. The camera matrices are wave-uniform (SGPRs after
// readfirstlane).
struct PreIn {
    float v[16], pm[16];
    float sx, sy, sz, opacity;
    float4 q;
};
template <int CAM>
__device__ __forceinline__ void load_pre_in(const PreprocessArgs& a, int idx, bool valid, PreIn& in)
{
#pragma unroll
    for (int k = 0; k < 16; ++k) in.v[k] = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, a.viewmatrix[k])));
    if constexpr (CAM != CAM_LONLAT) {
#pragma unroll
        for (int k = 0; k < 16; ++k) in.pm[k] = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, a.projmatrix[k])));
    }
    in.sx = in.sy = in.sz = in.opacity = 0.f;
    in.q = make_float4(0.f, 0.f, 0.f, 0.f);
    if (valid) {
        in.opacity = a.opacities[idx];
        if (a.cov3D_precomp == nullptr) {
            in.sx = a.scales[3 * idx], in.sy = a.scales[3 * idx + 1], in.sz = a.scales[3 * idx + 2];
            if ((reinterpret_cast<uintptr_t>(a.rotations) & 15u) == 0) in.q = reinterpret_cast<const float4*>(a.rotations)[idx];
            else in.q = make_float4(a.rotations[4 * idx], a.rotations[4 * idx + 1], a.rotations[4 * idx + 2], a.rotations[4 * idx + 3]);
        }
    }
}

// What one Gaussian's preprocess produces (forward.cu:693-702); rec = the 64-B render record (raster_common.h)
struct PreOut {
    float4 rec[SPLAT_F4];
    int rad;
    uint32_t area;
    uint8_t clamp_bits;
    float depth;
};

// One Gaussian, forward.cu:593-703 (lonlat) / :231-340 (pinhole). Returns false for a culled Gaussian (the caller
// then writes radius 0, no tiles, the culled sort key).
// shv: the Gaussian's SH row in registers when sh16, else the row is read from a.shs.
// The view direction (forward.cu:37-38) and, from the SH row in registers, the colour (sh_eval.h) and the backward's
// dRGB/ddir: preprocess_point's sh16 colour, restated for rows staged after the geometry (the same expressions, so
// the same bits).
__device__ __forceinline__ void sh16_colour(const PreprocessArgs& a, int idx, float3 p_orig, const float* shv,
                                            float rgb[3], uint8_t& clamp_bits)
{
    const float3 cp = {a.campos[0], a.campos[1], a.campos[2]};
    float dx = p_orig.x - cp.x, dy = p_orig.y - cp.y, dz = p_orig.z - cp.z;
    const float len = sqrtf(dx * dx + dy * dy + dz * dz);
    dx = dx / len;
    dy = dy / len;
    dz = dz / len;
    sh_to_rgb(a.D, dx, dy, dz, shv, rgb, clamp_bits);
#if OMR_SH_JAC
    float gx[3], gy[3], gz[3];
    sh_dir_grad(a.D, dx, dy, dz, [&](int k, int ch) { return shv[3 * k + ch]; }, gx, gy, gz);
    float* j = a.g.sh_jac + (size_t)idx * 9;
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) j[ch] = gx[ch], j[3 + ch] = gy[ch], j[6 + ch] = gz[ch];
#endif
}

// sh16_late: the SH row is not in shv yet; the caller stages it for the visible lanes and fills o.rec[2].xyz and
// o.clamp_bits with sh16_colour afterwards.
template <int CAM>
__device__ __forceinline__ bool preprocess_point(const PreprocessArgs& a, const PreIn& in, int idx, float3 p_orig,
                                                 bool sh16, const float (&shv)[48], PreOut& o, bool sh16_late = false)
{
    const float* v = in.v;
    const float3 t = transformPoint4x3(p_orig, v);
    float2 point_image;
    float depth;
    float J0[3], J1[3];  // columns 0 and 1 of the glm J (column 2 is zero)

    if constexpr (CAM == CAM_LONLAT) {
        // too_close (auxiliary.h:198-220)
        const float rr = t.x * t.x + t.y * t.y + t.z * t.z;
        if (rr <= 0.04f) return false;
        const float r = sqrtf(rr);
        // point3ToLonlatScreen (auxiliary.h:236-248)
        const float inv_r = 1.0f / (r + 0.0000001f);
        const float lon = omni::atan2f_(t.x, t.z);
        const float lat = omni::asinf_(t.y * inv_r);
        point_image = {ndc2Pix(lon * INV_PI, a.W), ndc2Pix(lat * TWO_INV_PI, a.H)};
        depth = r;
        // computeCov2DLonlat Jacobian (forward.cu:147-167)
        const float trxztrxz = t.x * t.x + t.z * t.z;
        const float trxztrxz_inv = 1.0f / (trxztrxz + 0.0000001f);
        const float trxz = sqrtf(trxztrxz);
        const float trxz_inv = 1.0f / (trxz + 0.0000001f);
        const float trtr = trxztrxz + t.y * t.y;
        const float trtr_inv = 1.0f / (trtr + 0.0000001f);
        const float W_div_2pi = (float)a.W * 0.5f * INV_PI;
        const float H_div_pi = (float)a.H * INV_PI;
        J0[0] = W_div_2pi * t.z * trxztrxz_inv;
        J0[1] = 0.0f;
        J0[2] = -W_div_2pi * t.x * trxztrxz_inv;
        J1[0] = -H_div_pi * t.x * t.y * trxz_inv * trtr_inv;
        J1[1] = H_div_pi * trxz * trtr_inv;
        J1[2] = -H_div_pi * t.z * t.y * trxz_inv * trtr_inv;
    } else {
        // in_frustum (auxiliary.h:166-196)
        if (t.z <= 0.2f) {
            if (a.prefiltered) atomicOr(a.error_flag, 1);
            return false;
        }
        const float4 p_hom = transformPoint4x4(p_orig, in.pm);
        const float p_w = 1.0f / (p_hom.w + 0.0000001f);
        point_image = {ndc2Pix(p_hom.x * p_w, a.W), ndc2Pix(p_hom.y * p_w, a.H)};
        depth = t.z;
        // computeCov2D (forward.cu:92-106)
        const float limx = 1.3f * a.tan_fovx;
        const float limy = 1.3f * a.tan_fovy;
        const float txtz = t.x / t.z;
        const float tytz = t.y / t.z;
        const float tx = fminf(limx, fmaxf(-limx, txtz)) * t.z;
        const float ty = fminf(limy, fmaxf(-limy, tytz)) * t.z;
        J0[0] = a.focal_x / t.z;
        J0[1] = 0.0f;
        J0[2] = -(a.focal_x * tx) / (t.z * t.z);
        J1[0] = 0.0f;
        J1[1] = a.focal_y / t.z;
        J1[2] = -(a.focal_y * ty) / (t.z * t.z);
    }

    float c3[6];
    if (a.cov3D_precomp != nullptr) {
#pragma unroll
        for (int k = 0; k < 6; ++k) c3[k] = a.cov3D_precomp[6 * idx + k];
    } else {
        cov3d_from_scale_rot(in.sx, in.sy, in.sz, a.scale_modifier, in.q, c3);
    }
    const float3 cov = cov2d_from_J(v, J0, J1, c3);

    // conic and radius (forward.cu:660-674)
    const float det = (cov.x * cov.z - cov.y * cov.y);
    if (det == 0.0f) return false;
    const float det_inv = 1.f / det;
    const float3 conic = {cov.z * det_inv, -cov.y * det_inv, cov.x * det_inv};
    const float mid = 0.5f * (cov.x + cov.z);
    const float lambda1 = mid + sqrtf(fmaxf(0.1f, mid * mid - det));
    const float lambda2 = mid - sqrtf(fmaxf(0.1f, mid * mid - det));
    const float my_radius = ceilf(3.f * sqrtf(fmaxf(lambda1, lambda2)));
    const int rad = (int)my_radius;
    uint32_t x0, y0, x1, y1;
    getRect(point_image, rad, a.gx, a.gy, x0, y0, x1, y1);
    const uint32_t area = (y1 - y0) * (x1 - x0);
    if (area == 0) return false;

    float rgb[3] = {0.f, 0.f, 0.f};
    uint8_t clamp_bits = 0;
    if (a.colors_precomp == nullptr) {
        const float3 cp = {a.campos[0], a.campos[1], a.campos[2]};
        float dx = p_orig.x - cp.x, dy = p_orig.y - cp.y, dz = p_orig.z - cp.z;
        const float len = sqrtf(dx * dx + dy * dy + dz * dz);
        dx = dx / len;
        dy = dy / len;
        dz = dz / len;
        if (sh16) {
            if (!sh16_late) {
                sh_to_rgb(a.D, dx, dy, dz, shv, rgb, clamp_bits);
#if OMR_SH_JAC
                // the backward's dRGB/ddir from the row in registers (sh_eval.h: sh_dir_grad; gaussian_bwd reads these
                // 36 B instead of the 192-B row)
                float gx[3], gy[3], gz[3];
                sh_dir_grad(a.D, dx, dy, dz, [&](int k, int ch) { return shv[3 * k + ch]; }, gx, gy, gz);
                float* j = a.g.sh_jac + (size_t)idx * 9;
#pragma unroll
                for (int ch = 0; ch < 3; ++ch) j[ch] = gx[ch], j[3 + ch] = gy[ch], j[6 + ch] = gz[ch];
#endif
            }
        } else {
            sh_to_rgb(a.D, dx, dy, dz, a.shs + (size_t)idx * a.M * 3, rgb, clamp_bits);
        }
    } else {
        rgb[0] = a.colors_precomp[3 * idx];
        rgb[1] = a.colors_precomp[3 * idx + 1];
        rgb[2] = a.colors_precomp[3 * idx + 2];
    }
    o.rec[0] = {point_image.x, point_image.y, depth, 0.0f};  // .w (slot base) is written by emit
    o.rec[1] = {conic.x, conic.y, conic.z, in.opacity};
    o.rec[2] = {rgb[0], rgb[1], rgb[2], __builtin_bit_cast(float, x1 - x0)};
    o.rec[3] = {__builtin_bit_cast(float, x0), __builtin_bit_cast(float, y0), __builtin_bit_cast(float, x1),
                __builtin_bit_cast(float, y1)};
    o.rad = rad;
    o.area = area;
    o.clamp_bits = clamp_bits;
    o.depth = depth;
    return true;
}

// The per-Gaussian outputs of one lane besides the colour (rec[2].xyz, clamped) and the render record: radius,
// tiles_touched, the row binning's rect word and band constants, the first depth-sort key / value, conic + opacity.
__device__ __forceinline__ void store_geometry(const PreprocessArgs& a, int idx, bool vis, const PreOut& o)
{
    const GeomState& g = a.g;
    a.radii[idx] = vis ? o.rad : 0;
    g.tiles_touched[idx] = vis ? o.area : 0u;
    const uint32_t x0 = __builtin_bit_cast(uint32_t, o.rec[3].x), y0 = __builtin_bit_cast(uint32_t, o.rec[3].y);
    const uint32_t wd = __builtin_bit_cast(uint32_t, o.rec[3].z) - x0;
    // the row binning's rect word (fields sized for BIN_MAX_GRID tiles a side); views past that carve no rect
    // and no bin_rec (GeomState::carve)
    if (g.rect)
        g.rect[idx] = vis ? make_uint2((__builtin_bit_cast(uint32_t, o.rec[3].w) - y0) | (y0 << RECT_ROWS_BITS) |
                                           (wd << 21),
                                       x0)
                          : make_uint2(0u, 0u);
    if (vis && g.bin_rec) {  // the binning's band-mask constants (bin.hip: the columns pass reads them per (Gaussian, row))
        float4 r0, r1;
        band_row_consts(band_consts(o.rec[1]), make_float2(o.rec[0].x, o.rec[0].y), r0, r1);
        g.bin_rec[2 * (size_t)idx] = r0;
        g.bin_rec[2 * (size_t)idx + 1] = r1;
    }
    g.key_a[idx] = vis ? __float_as_uint(o.depth) : 0xFFFFFFFFu;  // culled Gaussians sort last, emit nothing
    g.val_a[idx] = (uint32_t)idx;
    if (vis) g.conic_op[idx] = o.rec[1];  // the backward's per-Gaussian factors (raw_row_to_grads)
}

// scratch words later kernels expect zeroed (counters, tile ranges / costs, sort scratch), and the sh_jac key of the
// inputs: the first kernel of the forward does both, so there are no memset launches
__device__ __forceinline__ void preprocess_prologue(const PreprocessArgs& a)
{
    const size_t gtid = (size_t)blockIdx.x * blockDim.x + threadIdx.x, nth = (size_t)gridDim.x * blockDim.x;
#pragma unroll
    for (int z = 0; z < PRE_ZERO_SPANS; ++z)
        for (size_t i = gtid; i < a.zero[z].n; i += nth) a.zero[z].p[i] = 0u;
    // sh_jac stored (preprocess_point's sh16 rows; the host carved it on the same condition): the key of the inputs
    // ([6] keeps the same key for omr_debug_set_sh_jac, which clears and restores [5])
    if (gtid == 0) {
        const uint32_t key = sh_jac_stored(a.colors_precomp, a.M, a.shs)
                                 ? sh_jac_key(a.shs, a.means3D, __float_as_uint(a.campos[0]),
                                              __float_as_uint(a.campos[1]), __float_as_uint(a.campos[2]))
                                 : 0u;
        a.g.counters[5] = key;
        a.g.counters[6] = key;
    }
}

// One wave per 64 consecutive Gaussians. The wave reads its 64 SH rows (12 KiB) and writes its
// 64 render records (4 KiB) as contiguous spans through LDS (wave_rows.h). Equirect views request the SH rows before
// the projection math so their latency overlaps it; pinhole views request only the rows of the visible points, after
// the geometry (below). (Staging the rows by LDS-DMA instead, with the geometry computed while
// they land, measured no faster — the kernel streams at ~4.2 TB/s either way: profiles/r04c_ab_preprocess_dma.txt;
// the code is kept in profiles/r04_pruned_experiments.patch.)
//
// Pinhole views (round 6) read the SH rows lane by lane into registers instead: a frustum leaves few lanes of a wave
// with a row to read (12 % at E pinhole), so the per-lane loads touch few lines, and the wave's LDS image only
// stages the render records (5 KiB instead of 13): the kernel is no longer held at 3 waves per SIMD by LDS.
// OMR_PRE_PINHOLE_SPAN=1 (A/B builds) keeps the staged spans for pinhole views too.
#ifndef OMR_PRE_PINHOLE_SPAN
#define OMR_PRE_PINHOLE_SPAN 0
#endif
#ifndef OMR_PRE_PIN_MINW
#define OMR_PRE_PIN_MINW 1
#endif
// OMR_PRE_PIN_GLOBAL=1 (A/B builds): pinhole lanes evaluate the colour from the SH row in global memory (no 48
// registers for it, no early request)
#ifndef OMR_PRE_PIN_GLOBAL
#define OMR_PRE_PIN_GLOBAL 0
#endif
// OMR_PRE_LON_LANE=1 / OMR_PRE_LON_GLOBAL=1 (A/B builds): the same two forms for equirect views
#ifndef OMR_PRE_LON_LANE
#define OMR_PRE_LON_LANE 0
#endif
#ifndef OMR_PRE_LON_GLOBAL
#define OMR_PRE_LON_GLOBAL 0
#endif
template <int CAM>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(CAM == CAM_LONLAT ? 1 : OMR_PRE_PIN_MINW)))
void preprocess_kernel(PreprocessArgs a)
{
    constexpr int SH_F4 = 12;  // 16 coefficients x 3 channels
    // colour from the SH row in global memory / SH rows as staged spans (else: per-lane rows in registers)
    constexpr bool global_colour = CAM == CAM_LONLAT ? OMR_PRE_LON_GLOBAL : OMR_PRE_PIN_GLOBAL;
    constexpr bool span_rows =
        !global_colour && (CAM == CAM_LONLAT ? !OMR_PRE_LON_LANE : (bool)OMR_PRE_PINHOLE_SPAN);
    constexpr int IMG_F4 = span_rows ? stage_f4<SH_F4>() : stage_f4<SPLAT_F4>();
    static_assert(IMG_F4 >= stage_f4<SPLAT_F4>(), "the image also stages the render records");
    __shared__ float4 s_stage[4][IMG_F4];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    preprocess_prologue(a);
    const int wave_first = (int)(blockIdx.x * 256u + wv * 64u);
    if (wave_first >= a.P) return;  // wave-uniform
    const int idx = wave_first + (int)lane;
    const bool valid = idx < a.P;
    float4* stage = s_stage[wv];
    GeomState& g = a.g;

    const float3 p_orig = valid ? make_float3(a.means3D[3 * idx], a.means3D[3 * idx + 1], a.means3D[3 * idx + 2])
                                : make_float3(0.f, 0.f, 0.f);
    const bool sh16 = a.colors_precomp == nullptr && a.M == 16 && (reinterpret_cast<uintptr_t>(a.shs) & 15u) == 0;
    const int nf4 = (3 * (a.D + 1) * (a.D + 1) + 3) >> 2;
    float shv[48];
    PreIn in;
    load_pre_in<CAM>(a, idx, valid, in);
    // Every view requests the SH rows before the projection, into registers, and parks them in LDS after it, so the
    // loads' latency overlaps the projection (the 48 VGPRs are free: the LDS image caps the kernel at 3 waves per
    // SIMD). Waiting for them before the projection (wave_rows_load) cost C 0.024 ms of the kernel's 0.092: without
    // the rows it took 0.068 ms (profiles/r05v_ab.txt). Equirect views see every point: every valid lane's row. A
    // frustum culls most of a pinhole view's scene (88 % at E pinhole), so there only the rows of the lanes whose mean
    // lies in front of the near plane and inside the 1.3x widened view cone (the cov2D clamp's, forward.cu:92-106) are
    // requested: a prediction from the mean alone. A visible lane outside it (a large Gaussian whose mean is off-view)
    // reads its row itself after the projection.
    uint64_t fetch_rows = __ballot(valid);
    if constexpr (CAM != CAM_LONLAT) {
        const float tz = in.v[2] * p_orig.x + in.v[6] * p_orig.y + in.v[10] * p_orig.z + in.v[14];
        const float tx = in.v[0] * p_orig.x + in.v[4] * p_orig.y + in.v[8] * p_orig.z + in.v[12];
        const float ty = in.v[1] * p_orig.x + in.v[5] * p_orig.y + in.v[9] * p_orig.z + in.v[13];
        const bool near = valid && tz > 0.2f && fabsf(tx) <= 1.3f * a.tan_fovx * tz && fabsf(ty) <= 1.3f * a.tan_fovy * tz;
        fetch_rows = __ballot(near);
    }
    rowv4 early[SH_F4];
    // every load issued so far lands before the rows are requested, on both sides of the branch below: loads retire
    // in order on vmcnt, and a later wait for one of them would otherwise have to count the rows in (the wait
    // counter merges the branch's sides conservatively), i.e. wait for the rows too
    asm volatile("" ::"v"(in.opacity), "v"(in.sx), "v"(in.sy), "v"(in.sz), "v"(in.q.x), "v"(in.q.y), "v"(in.q.z),
                 "v"(in.q.w), "v"(p_orig.x), "v"(p_orig.y), "v"(p_orig.z));
    const bool fetched = !global_colour && ((fetch_rows >> lane) & 1u);
    if constexpr (span_rows) {
        if (sh16 && fetch_rows) {
            wave_rows_fetch<SH_F4>(reinterpret_cast<const float4*>(a.shs) + (size_t)wave_first * SH_F4, fetch_rows,
                                   nf4, lane, early);
        }
    } else {
        if (sh16 && fetched) {  // the lane's own row (columns past nf4 are never read)
            const rowv4* row = reinterpret_cast<const rowv4*>(a.shs) + (size_t)idx * SH_F4;
#pragma unroll
            for (int q = 0; q < SH_F4; ++q) early[q] = q < nf4 ? row[q] : rowv4{0.f, 0.f, 0.f, 0.f};
        }
    }
    PreOut o;
    const bool vis = valid && preprocess_point<CAM>(a, in, idx, p_orig, sh16, shv, o, sh16);
    if constexpr (global_colour) {
        if (sh16 && vis) {
            float rgb[3];
            sh16_colour(a, idx, p_orig, a.shs + (size_t)idx * 48, rgb, o.clamp_bits);
            o.rec[2].x = rgb[0], o.rec[2].y = rgb[1], o.rec[2].z = rgb[2];
        }
    } else if constexpr (!span_rows) {
        if (sh16 && vis) {
            if (!fetched) {  // a visible lane outside the prediction: its row after the projection
                const rowv4* row = reinterpret_cast<const rowv4*>(a.shs) + (size_t)idx * SH_F4;
#pragma unroll
                for (int q = 0; q < SH_F4; ++q) early[q] = q < nf4 ? row[q] : rowv4{0.f, 0.f, 0.f, 0.f};
            }
#pragma unroll
            for (int q = 0; q < SH_F4; ++q) {
                shv[4 * q] = early[q].x, shv[4 * q + 1] = early[q].y, shv[4 * q + 2] = early[q].z;
                shv[4 * q + 3] = early[q].w;
            }
            float rgb[3];
            sh16_colour(a, idx, p_orig, shv, rgb, o.clamp_bits);
            o.rec[2].x = rgb[0], o.rec[2].y = rgb[1], o.rec[2].z = rgb[2];
        }
    }
    if (span_rows && sh16) {
        const uint64_t rows = __ballot(vis);
        if (rows) {  // wave-uniform
            wave_rows_park<SH_F4>(early, stage, lane);
            wave_sync();
#pragma unroll
            for (int q = 0; q < SH_F4; ++q) {
                const float4 v = q < nf4 ? stage[lane * stage_stride<SH_F4>() + q] : make_float4(0.f, 0.f, 0.f, 0.f);
                shv[4 * q] = v.x, shv[4 * q + 1] = v.y, shv[4 * q + 2] = v.z, shv[4 * q + 3] = v.w;
            }
            if constexpr (CAM != CAM_LONLAT) {
                if (vis && !((fetch_rows >> lane) & 1u)) {  // a visible lane outside the prediction: its own row
                    const float4* row = reinterpret_cast<const float4*>(a.shs) + (size_t)idx * SH_F4;
#pragma unroll
                    for (int q = 0; q < SH_F4; ++q) {
                        const float4 v = q < nf4 ? row[q] : make_float4(0.f, 0.f, 0.f, 0.f);
                        shv[4 * q] = v.x, shv[4 * q + 1] = v.y, shv[4 * q + 2] = v.z, shv[4 * q + 3] = v.w;
                    }
                }
            }
            wave_sync();  // the image is reused for the records below
            if (vis) {
                float rgb[3];
                sh16_colour(a, idx, p_orig, shv, rgb, o.clamp_bits);
                o.rec[2].x = rgb[0], o.rec[2].y = rgb[1], o.rec[2].z = rgb[2];
            }
        }
    }
    if (valid) {
        store_geometry(a, idx, vis, o);
        if (vis) g.clamped[idx] = o.clamp_bits;
    }
    // the render record of a visible Gaussian (culled records are never read)
    const uint64_t rec_rows = __ballot(vis);
    if (vis) {
#pragma unroll
        for (int j = 0; j < SPLAT_F4; ++j) stage[lane * stage_stride<SPLAT_F4>() + j] = o.rec[j];
    }
    wave_sync();
    wave_rows_store<SPLAT_F4>(g.splat + (size_t)wave_first * SPLAT_F4, rec_rows, stage, lane);
}

__global__ void mark_frustum_kernel(int P, const float* means3D, const float* viewmatrix, bool* present)
{
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= P) return;
    const float3 p = {means3D[3 * idx], means3D[3 * idx + 1], means3D[3 * idx + 2]};
    present[idx] = transformPoint4x3(p, viewmatrix).z > 0.2f;  // checkFrustum, rasterizer_impl.cu:66-78
}

__global__ void mark_all_kernel(int P, bool* present)  // markAllVisible, rasterizer_impl.cu:82-90
{
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx < P) present[idx] = true;
}

}  // namespace

void launch_preprocess(int camera_type, const PreprocessArgs& a, hipStream_t s)
{
    if (a.P <= 0) return;
    const dim3 grid(div_up(a.P, 256));
    if (camera_type == CAM_LONLAT) preprocess_kernel<CAM_LONLAT><<<grid, 256, 0, s>>>(a);
    else preprocess_kernel<CAM_PINHOLE><<<grid, 256, 0, s>>>(a);
}

void launch_mark_visible(int camera_type, int P, const float* means3D, const float* viewmatrix, const float* projmatrix,
                         bool* present, hipStream_t s)
{
    (void)projmatrix;
    if (P <= 0) return;
    const dim3 grid(div_up(P, 256));
    if (camera_type == CAM_LONLAT) mark_all_kernel<<<grid, 256, 0, s>>>(P, present);
    else mark_frustum_kernel<<<grid, 256, 0, s>>>(P, means3D, viewmatrix, present);
}

}  // namespace omr

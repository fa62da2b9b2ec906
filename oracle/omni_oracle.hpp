// omni_oracle.hpp — CPU restatement of the OmniGS tile rasterizer (reference: raikuma/OmniGS-fork @ 2025-03-04,
// cuda_rasterizer/*). TEST INFRASTRUCTURE ONLY: this file is the parity checker for the HIP path and the
// cpu_baseline of bench.py. Nothing in the product (omnigs-fork_amd/) includes, links or calls it.
//
// PARITY STATUS: "parity unpinned" in the strict sense — the reference is CUDA-only (no nvcc, no glm here),
// ships no tests and no golden vectors, so it cannot be run to produce fixtures.
// The restatement is pinned instead by (tests/test_oracle_*.py):
//   * known answers taken from the reference's own files: examples/simple_cloud.cpp:130-226 (3 Gaussians,
//     analytic lonlat centres at 2000x1000) and the closed-form lonlat Jacobian of supp.pdf App. A;
//   * finite differences of the double instantiation of this file (backward vs forward);
//   * an independent PyTorch-autograd model of preprocess + blending written separately (tests/torch_model.py).
//
// Every function cites the reference file:line it follows. Arithmetic follows the reference expression by
// expression (left-to-right evaluation, glm column-major conventions) so that, compiled with
// -ffp-contract=off, the float instantiation is bit-reproducible; the transcendentals that decide tile
// membership come from omnigs-fork_amd/csrc/omni_math.h (see that header for why).
//
// Template parameter R = float (parity, fixtures, cpu baseline) or double (finite-difference checks).
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <utility>
#include <vector>

#include "../omnigs-fork_amd/csrc/omni_math.h"

#ifdef _OPENMP
#include <omp.h>
#endif

namespace oracle {

constexpr int BLOCK_X = 16;  // cuda_rasterizer/config.h:26
constexpr int BLOCK_Y = 16;  // config.h:27
constexpr int BLOCK_SIZE = BLOCK_X * BLOCK_Y;  // auxiliary.h:28
constexpr int NUM_CHANNELS = 3;  // config.h:25

// ---------------------------------------------------------------------------------------------------------
// Scalar helpers per precision
// ---------------------------------------------------------------------------------------------------------
template <typename R> struct Math;
template <> struct Math<float> {
#ifdef OMR_ORACLE_LIBM_TRIG
    // liboracle_libm.so (oracle/Makefile): glibc's atan2f / asinf, an implementation independent of omni_math.h (as
    // libdevice's is for the reference, auxiliary.h:240-241), so oracle/contraction.py can measure what the choice
    // of transcendental implementation changes in the tile rects, keys and point list
    static float atan2(float y, float x) { return ::atan2f(y, x); }
    static float asin(float x) { return ::asinf(x); }
#else
    static float atan2(float y, float x) { return omni::atan2f_(y, x); }
    static float asin(float x) { return omni::asinf_(x); }
#endif
    static float sqrt(float x) { return std::sqrt(x); }
    static float exp(float x) { return std::exp(x); }
    static float ceil(float x) { return std::ceil(x); }
};
template <> struct Math<double> {
    static double atan2(double y, double x) { return std::atan2(y, x); }
    static double asin(double x) { return std::asin(x); }
    static double sqrt(double x) { return std::sqrt(x); }
    static double exp(double x) { return std::exp(x); }
    static double ceil(double x) { return std::ceil(x); }
};
template <typename R> R fmax_(R a, R b) { return std::fmax(a, b); }
template <typename R> R fmin_(R a, R b) { return std::fmin(a, b); }

// float bit pattern used by the sort key (rasterizer_impl.cu:133)
inline uint32_t float_bits(float f)
{
    uint32_t u;
    std::memcpy(&u, &f, 4);
    return u;
}

template <typename R> struct V2 { R x, y; };
template <typename R> struct V3 {
    R x, y, z;
    V3 operator+(const V3& o) const { return {x + o.x, y + o.y, z + o.z}; }
    V3 operator-(const V3& o) const { return {x - o.x, y - o.y, z - o.z}; }
    V3& operator+=(const V3& o) { x += o.x; y += o.y; z += o.z; return *this; }
};
template <typename R> V3<R> operator*(R s, const V3<R>& v) { return {s * v.x, s * v.y, s * v.z}; }
template <typename R> V3<R> operator/(const V3<R>& v, R s) { return {v.x / s, v.y / s, v.z / s}; }
template <typename R> R dot3(const V3<R>& a, const V3<R>& b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
template <typename R> struct V4 { R x, y, z, w; };

// glm::mat3 semantics: m[col][row]; the 9-argument constructor fills column by column.
template <typename R> struct M3 {
    R m[3][3];
    static M3 cols(R a0, R a1, R a2, R b0, R b1, R b2, R c0, R c1, R c2)
    {
        M3 r;
        r.m[0][0] = a0; r.m[0][1] = a1; r.m[0][2] = a2;
        r.m[1][0] = b0; r.m[1][1] = b1; r.m[1][2] = b2;
        r.m[2][0] = c0; r.m[2][1] = c1; r.m[2][2] = c2;
        return r;
    }
    static M3 identity() { return cols(1, 0, 0, 0, 1, 0, 0, 0, 1); }
    R* operator[](int c) { return m[c]; }
    const R* operator[](int c) const { return m[c]; }
};
// glm operator*(mat3, mat3): Result[j][i] = A[0][i]*B[j][0] + A[1][i]*B[j][1] + A[2][i]*B[j][2]
template <typename R> M3<R> operator*(const M3<R>& A, const M3<R>& B)
{
    M3<R> r;
    for (int j = 0; j < 3; ++j)
        for (int i = 0; i < 3; ++i) r.m[j][i] = A.m[0][i] * B.m[j][0] + A.m[1][i] * B.m[j][1] + A.m[2][i] * B.m[j][2];
    return r;
}
template <typename R> M3<R> operator*(R s, const M3<R>& A)
{
    M3<R> r;
    for (int j = 0; j < 3; ++j)
        for (int i = 0; i < 3; ++i) r.m[j][i] = s * A.m[j][i];
    return r;
}
template <typename R> M3<R> transpose(const M3<R>& A)
{
    M3<R> r;
    for (int j = 0; j < 3; ++j)
        for (int i = 0; i < 3; ++i) r.m[j][i] = A.m[i][j];
    return r;
}
template <typename R> V3<R> col(const M3<R>& A, int c) { return {A.m[c][0], A.m[c][1], A.m[c][2]}; }

// SH constants, auxiliary.h:32-49
template <typename R> struct SH {
    static constexpr R C0 = R(0.28209479177387814);
    static constexpr R C1 = R(0.4886025119029199);
    static constexpr R C2[5] = {R(1.0925484305920792), R(-1.0925484305920792), R(0.31539156525252005),
                                R(-1.0925484305920792), R(0.5462742152960396)};
    static constexpr R C3[7] = {R(-0.5900435899266435), R(2.890611442640554), R(-0.4570457994644658),
                                R(0.3731763325901154), R(-0.4570457994644658), R(1.445305721320277),
                                R(-0.5900435899266435)};
};
template <typename R> constexpr R R_1_PI = R(0.318309886183790671537767526745028724);  // M_1_PIf32
template <typename R> constexpr R R_2_PI = R(0.636619772367581343075535053490057448);  // M_2_PIf32

// auxiliary.h:51-54 — computed in double, rounded to R
template <typename R> R ndc2Pix(R v, int S) { return (R)((((double)v + 1.0) * S - 1.0) * 0.5); }

struct Rect { uint32_t minx, miny, maxx, maxy; };
// auxiliary.h:56-66
template <typename R> Rect getRect(V2<R> p, int max_radius, uint32_t gx, uint32_t gy)
{
    auto clampi = [](uint32_t g, int v) { return std::min<uint32_t>(g, (uint32_t)std::max(0, v)); };
    Rect r;
    r.minx = clampi(gx, (int)((p.x - (R)max_radius) / (R)BLOCK_X));
    r.miny = clampi(gy, (int)((p.y - (R)max_radius) / (R)BLOCK_Y));
    // BLOCK_X is the macro 16, so p.x + max_radius + BLOCK_X - 1 is ((p.x + r) + 16) - 1 in float
    r.maxx = clampi(gx, (int)((p.x + (R)max_radius + (R)BLOCK_X - R(1)) / (R)BLOCK_X));
    r.maxy = clampi(gy, (int)((p.y + (R)max_radius + (R)BLOCK_Y - R(1)) / (R)BLOCK_Y));
    return r;
}

// auxiliary.h:85-93
template <typename R> V3<R> transformPoint4x3(const V3<R>& p, const R* m)
{
    return {m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12], m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13],
            m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14]};
}
// auxiliary.h:95-104
template <typename R> V4<R> transformPoint4x4(const V3<R>& p, const R* m)
{
    return {m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12], m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13],
            m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14], m[3] * p.x + m[7] * p.y + m[11] * p.z + m[15]};
}
// auxiliary.h:116-124
template <typename R> V3<R> transformVec4x3Transpose(const V3<R>& p, const R* m)
{
    return {m[0] * p.x + m[1] * p.y + m[2] * p.z, m[4] * p.x + m[5] * p.y + m[6] * p.z,
            m[8] * p.x + m[9] * p.y + m[10] * p.z};
}
// auxiliary.h:134-144
template <typename R> V3<R> dnormvdv(const V3<R>& v, const V3<R>& dv)
{
    R sum2 = v.x * v.x + v.y * v.y + v.z * v.z;
    R invsum32 = R(1) / Math<R>::sqrt(sum2 * sum2 * sum2);
    V3<R> r;
    r.x = ((+sum2 - v.x * v.x) * dv.x - v.y * v.x * dv.y - v.z * v.x * dv.z) * invsum32;
    r.y = (-v.x * v.y * dv.x + (sum2 - v.y * v.y) * dv.y - v.z * v.y * dv.z) * invsum32;
    r.z = (-v.x * v.z * dv.x - v.y * v.z * dv.y + (sum2 - v.z * v.z) * dv.z) * invsum32;
    return r;
}

// auxiliary.h:166-196 (prefiltered trap replaced by an exception)
template <typename R> bool in_frustum(const V3<R>& p_orig, const R* viewmatrix, const R* projmatrix, bool prefiltered, V3<R>& p_view)
{
    V4<R> p_hom = transformPoint4x4(p_orig, projmatrix);
    (void)p_hom;
    p_view = transformPoint4x3(p_orig, viewmatrix);
    if (p_view.z <= R(0.2f)) {
        if (prefiltered) throw std::runtime_error("Point is filtered although prefiltered is set. This shouldn't happen!");
        return false;
    }
    return true;
}

// auxiliary.h:198-220
template <typename R> bool too_close(const V3<R>& p_orig, const R* viewmatrix, V4<R>& pr_view)
{
    V3<R> p_view = transformPoint4x3(p_orig, viewmatrix);
    R rr = p_view.x * p_view.x + p_view.y * p_view.y + p_view.z * p_view.z;
    if (rr <= R(0.04f)) return true;
    R r = Math<R>::sqrt(rr);
    pr_view = {p_view.x, p_view.y, p_view.z, r};
    return false;
}

// auxiliary.h:236-248
template <typename R> V2<R> point3ToLonlatScreen(const V4<R>& pt)
{
    R inv_r = R(1) / (pt.w + R(0.0000001f));
    R lon = Math<R>::atan2(pt.x, pt.z);
    R lat = Math<R>::asin(pt.y * inv_r);
    return {lon * R_1_PI<R>, lat * R_2_PI<R>};
}

// ---------------------------------------------------------------------------------------------------------
// Forward per-Gaussian math
// ---------------------------------------------------------------------------------------------------------

// forward.cu:30-83
template <typename R>
V3<R> computeColorFromSH(int idx, int deg, int max_coeffs, const R* means, const R* campos, const R* shs, uint8_t* clamped)
{
    using S = SH<R>;
    V3<R> pos = {means[3 * idx], means[3 * idx + 1], means[3 * idx + 2]};
    V3<R> cp = {campos[0], campos[1], campos[2]};
    V3<R> dir = pos - cp;
    dir = dir / Math<R>::sqrt(dot3(dir, dir));  // glm::length
    const R* b = shs + (size_t)idx * max_coeffs * 3;
    auto sh = [&](int k) { return V3<R>{b[3 * k], b[3 * k + 1], b[3 * k + 2]}; };
    V3<R> result = S::C0 * sh(0);
    if (deg > 0) {
        R x = dir.x, y = dir.y, z = dir.z;
        result = result - (S::C1 * y) * sh(1) + (S::C1 * z) * sh(2) - (S::C1 * x) * sh(3);
        if (deg > 1) {
            R xx = x * x, yy = y * y, zz = z * z;
            R xy = x * y, yz = y * z, xz = x * z;
            result = result + (S::C2[0] * xy) * sh(4) + (S::C2[1] * yz) * sh(5) +
                     (S::C2[2] * (R(2) * zz - xx - yy)) * sh(6) + (S::C2[3] * xz) * sh(7) + (S::C2[4] * (xx - yy)) * sh(8);
            if (deg > 2) {
                result = result + (S::C3[0] * y * (R(3) * xx - yy)) * sh(9) + (S::C3[1] * xy * z) * sh(10) +
                         (S::C3[2] * y * (R(4) * zz - xx - yy)) * sh(11) +
                         (S::C3[3] * z * (R(2) * zz - R(3) * xx - R(3) * yy)) * sh(12) +
                         (S::C3[4] * x * (R(4) * zz - xx - yy)) * sh(13) + (S::C3[5] * z * (xx - yy)) * sh(14) +
                         (S::C3[6] * x * (xx - R(3) * yy)) * sh(15);
            }
        }
    }
    result += V3<R>{R(0.5f), R(0.5f), R(0.5f)};
    clamped[3 * idx + 0] = result.x < 0;
    clamped[3 * idx + 1] = result.y < 0;
    clamped[3 * idx + 2] = result.z < 0;
    return {fmax_(result.x, R(0)), fmax_(result.y, R(0)), fmax_(result.z, R(0))};
}

template <typename R> M3<R> viewW(const R* v)  // forward.cu:108-111 / 169-172
{
    return M3<R>::cols(v[0], v[4], v[8], v[1], v[5], v[9], v[2], v[6], v[10]);
}
template <typename R> M3<R> vrk(const R* c)  // forward.cu:115-118
{
    return M3<R>::cols(c[0], c[1], c[2], c[1], c[3], c[4], c[2], c[4], c[5]);
}

// forward.cu:86-127 (pinhole)
template <typename R>
V3<R> computeCov2D(const V3<R>& mean, R focal_x, R focal_y, R tan_fovx, R tan_fovy, const R* cov3D, const R* viewmatrix)
{
    V3<R> t = transformPoint4x3(mean, viewmatrix);
    const R limx = R(1.3f) * tan_fovx;
    const R limy = R(1.3f) * tan_fovy;
    const R txtz = t.x / t.z;
    const R tytz = t.y / t.z;
    t.x = fmin_(limx, fmax_(-limx, txtz)) * t.z;
    t.y = fmin_(limy, fmax_(-limy, tytz)) * t.z;
    M3<R> J = M3<R>::cols(focal_x / t.z, R(0), -(focal_x * t.x) / (t.z * t.z), R(0), focal_y / t.z,
                          -(focal_y * t.y) / (t.z * t.z), 0, 0, 0);
    M3<R> W = viewW(viewmatrix);
    M3<R> T = W * J;
    M3<R> Vrk = vrk(cov3D);
    M3<R> cov = transpose(T) * transpose(Vrk) * T;
    cov[0][0] += R(0.3f);
    cov[1][1] += R(0.3f);
    return {cov[0][0], cov[0][1], cov[1][1]};
}

// lonlat Jacobian entries, forward.cu:147-162 (identical in backward.cu:340-360)
template <typename R> struct LonlatJ {
    R dpx_dtx, dpx_dtz, dpy_dtx, dpy_dty, dpy_dtz;
};
template <typename R> LonlatJ<R> lonlatJ(const V3<R>& t, int width, int height)
{
    R trxztrxz = t.x * t.x + t.z * t.z;
    R trxztrxz_inv = R(1) / (trxztrxz + R(0.0000001f));
    R trxz = Math<R>::sqrt(trxztrxz);
    R trxz_inv = R(1) / (trxz + R(0.0000001f));
    R trtr = trxztrxz + t.y * t.y;
    R trtr_inv = R(1) / (trtr + R(0.0000001f));
    R W_div_2pi = (R)width * R(0.5f) * R_1_PI<R>;
    R H_div_pi = (R)height * R_1_PI<R>;
    LonlatJ<R> j;
    j.dpx_dtx = W_div_2pi * t.z * trxztrxz_inv;
    j.dpx_dtz = -W_div_2pi * t.x * trxztrxz_inv;
    j.dpy_dtx = -H_div_pi * t.x * t.y * trxz_inv * trtr_inv;
    j.dpy_dty = H_div_pi * trxz * trtr_inv;
    j.dpy_dtz = -H_div_pi * t.z * t.y * trxz_inv * trtr_inv;
    return j;
}

// forward.cu:130-189
template <typename R> V3<R> computeCov2DLonlat(const V3<R>& mean, int width, int height, const R* cov3D, const R* viewmatrix)
{
    V3<R> t = transformPoint4x3(mean, viewmatrix);
    LonlatJ<R> j = lonlatJ(t, width, height);
    M3<R> J = M3<R>::cols(j.dpx_dtx, R(0), j.dpx_dtz, j.dpy_dtx, j.dpy_dty, j.dpy_dtz, R(0), R(0), R(0));
    M3<R> W = viewW(viewmatrix);
    M3<R> T = W * J;
    M3<R> Vrk = vrk(cov3D);
    M3<R> cov = transpose(T) * transpose(Vrk) * T;
    cov[0][0] += R(0.3f);
    cov[1][1] += R(0.3f);
    return {cov[0][0], cov[0][1], cov[1][1]};
}

// forward.cu:194-228
template <typename R> void computeCov3D(const V3<R>& scale, R mod, const V4<R>& rot, R* cov3D)
{
    M3<R> S = M3<R>::identity();
    S[0][0] = mod * scale.x;
    S[1][1] = mod * scale.y;
    S[2][2] = mod * scale.z;
    V4<R> q = rot;  // not normalised (forward.cu:203)
    R r = q.x, x = q.y, y = q.z, z = q.w;
    M3<R> Rm = M3<R>::cols(R(1) - R(2) * (y * y + z * z), R(2) * (x * y - r * z), R(2) * (x * z + r * y),
                           R(2) * (x * y + r * z), R(1) - R(2) * (x * x + z * z), R(2) * (y * z - r * x),
                           R(2) * (x * z - r * y), R(2) * (y * z + r * x), R(1) - R(2) * (x * x + y * y));
    M3<R> M = S * Rm;
    M3<R> Sigma = transpose(M) * M;
    cov3D[0] = Sigma[0][0];
    cov3D[1] = Sigma[0][1];
    cov3D[2] = Sigma[0][2];
    cov3D[3] = Sigma[1][1];
    cov3D[4] = Sigma[1][2];
    cov3D[5] = Sigma[2][2];
}

// ---------------------------------------------------------------------------------------------------------
// Rasterizer state (rasterizer_impl.h:37-102, but as plain vectors: the oracle owns its buffers)
// ---------------------------------------------------------------------------------------------------------
template <typename R> struct Args {
    int P = 0, D = 0, M = 0;
    const R* background = nullptr;
    int width = 0, height = 0;
    const R* means3D = nullptr;
    const R* shs = nullptr;
    const R* colors_precomp = nullptr;
    const R* opacities = nullptr;
    const R* scales = nullptr;
    R scale_modifier = 1;
    const R* rotations = nullptr;
    const R* cov3D_precomp = nullptr;
    const R* viewmatrix = nullptr;
    const R* projmatrix = nullptr;
    const R* campos = nullptr;
    R tan_fovx = 0, tan_fovy = 0;
    bool prefiltered = false;
    int camera_type = 3;
    bool render_depth = false;
};

template <typename R> struct State {
    Args<R> a;
    // copies of the inputs (so backward can run after the caller's arrays are gone)
    std::vector<R> bg, means3D, shs, colors_precomp, opac, scales, rots, cov3D_precomp, view, proj, campos;
    // GeometryState
    std::vector<R> depths;
    std::vector<uint8_t> clamped;
    std::vector<int> radii;
    std::vector<V2<R>> means2D;
    std::vector<R> cov3D;
    std::vector<V4<R>> conic_opacity;
    std::vector<R> rgb;
    std::vector<uint32_t> tiles_touched, point_offsets;
    // BinningState
    std::vector<uint64_t> keys;      // sorted
    std::vector<uint32_t> point_list;  // sorted
    // ImageState
    std::vector<R> final_T;
    std::vector<uint32_t> n_contrib;
    std::vector<uint32_t> ranges;  // 2 per tile
    int num_rendered = 0;
    std::vector<R> out_color;
    uint32_t gx = 0, gy = 0;
};

template <typename T> static void copy_in(std::vector<T>& dst, const T* src, size_t n)
{
    if (src == nullptr) { dst.clear(); return; }
    dst.assign(src, src + n);
}

// rasterizer_impl.cu:47-62
inline uint32_t getHigherMsb(uint32_t n)
{
    uint32_t msb = sizeof(n) * 4;
    uint32_t step = msb;
    while (step > 1) {
        step /= 2;
        if (n >> msb) msb += step;
        else msb -= step;
    }
    if (n >> msb) msb++;
    return msb;
}

// forward.cu:593-703 (lonlat) and forward.cu:231-340 (pinhole), one Gaussian
template <typename R> void preprocess_one(State<R>& s, int idx, R focal_x, R focal_y)
{
    const Args<R>& a = s.a;
    s.radii[idx] = 0;
    s.tiles_touched[idx] = 0;
    V3<R> p_orig = {a.means3D[3 * idx], a.means3D[3 * idx + 1], a.means3D[3 * idx + 2]};
    V2<R> point_image;
    R depth;
    const R* cov3D;
    V3<R> cov;
    if (a.camera_type == 3) {
        V4<R> p_view;
        if (too_close(p_orig, a.viewmatrix, p_view)) return;
        V2<R> p_proj = point3ToLonlatScreen(p_view);
        if (a.cov3D_precomp != nullptr) cov3D = a.cov3D_precomp + idx * 6;
        else {
            V3<R> sc = {a.scales[3 * idx], a.scales[3 * idx + 1], a.scales[3 * idx + 2]};
            V4<R> ro = {a.rotations[4 * idx], a.rotations[4 * idx + 1], a.rotations[4 * idx + 2], a.rotations[4 * idx + 3]};
            computeCov3D(sc, a.scale_modifier, ro, &s.cov3D[6 * idx]);
            cov3D = &s.cov3D[6 * idx];
        }
        cov = computeCov2DLonlat(p_orig, a.width, a.height, cov3D, a.viewmatrix);
        point_image = {ndc2Pix(p_proj.x, a.width), ndc2Pix(p_proj.y, a.height)};
        depth = p_view.w;
    } else {
        V3<R> p_view;
        if (!in_frustum(p_orig, a.viewmatrix, a.projmatrix, a.prefiltered, p_view)) return;
        V4<R> p_hom = transformPoint4x4(p_orig, a.projmatrix);
        R p_w = R(1) / (p_hom.w + R(0.0000001f));
        V3<R> p_proj = {p_hom.x * p_w, p_hom.y * p_w, p_hom.z * p_w};
        if (a.cov3D_precomp != nullptr) cov3D = a.cov3D_precomp + idx * 6;
        else {
            V3<R> sc = {a.scales[3 * idx], a.scales[3 * idx + 1], a.scales[3 * idx + 2]};
            V4<R> ro = {a.rotations[4 * idx], a.rotations[4 * idx + 1], a.rotations[4 * idx + 2], a.rotations[4 * idx + 3]};
            computeCov3D(sc, a.scale_modifier, ro, &s.cov3D[6 * idx]);
            cov3D = &s.cov3D[6 * idx];
        }
        cov = computeCov2D(p_orig, focal_x, focal_y, a.tan_fovx, a.tan_fovy, cov3D, a.viewmatrix);
        point_image = {ndc2Pix(p_proj.x, a.width), ndc2Pix(p_proj.y, a.height)};
        depth = p_view.z;
    }
    // forward.cu:660-674
    R det = (cov.x * cov.z - cov.y * cov.y);
    if (det == R(0)) return;
    R det_inv = R(1) / det;
    V3<R> conic = {cov.z * det_inv, -cov.y * det_inv, cov.x * det_inv};
    R mid = R(0.5f) * (cov.x + cov.z);
    R lambda1 = mid + Math<R>::sqrt(fmax_(R(0.1f), mid * mid - det));
    R lambda2 = mid - Math<R>::sqrt(fmax_(R(0.1f), mid * mid - det));
    R my_radius = Math<R>::ceil(R(3) * Math<R>::sqrt(fmax_(lambda1, lambda2)));
    Rect rc = getRect(point_image, (int)my_radius, s.gx, s.gy);
    if ((rc.maxx - rc.minx) * (rc.maxy - rc.miny) == 0) return;
    if (a.colors_precomp == nullptr) {
        V3<R> result = computeColorFromSH(idx, a.D, a.M, a.means3D, a.campos, a.shs, s.clamped.data());
        s.rgb[idx * 3 + 0] = result.x;
        s.rgb[idx * 3 + 1] = result.y;
        s.rgb[idx * 3 + 2] = result.z;
    }
    s.depths[idx] = depth;
    s.radii[idx] = (int)my_radius;
    s.means2D[idx] = point_image;
    s.conic_opacity[idx] = {conic.x, conic.y, conic.z, a.opacities[idx]};
    s.tiles_touched[idx] = (rc.maxy - rc.miny) * (rc.maxx - rc.minx);
}

// forward.cu:346-467 (renderCUDA) and :472-590 (renderDepthCUDA), one tile; per-pixel semantics are
// independent of the block batching and of the block-vote early exit, so pixels are walked one by one.
template <typename R> void render_tile(State<R>& s, uint32_t tx, uint32_t ty, const R* features, bool depth_mode)
{
    const int W = s.a.width, H = s.a.height;
    const uint32_t t = ty * s.gx + tx;
    const uint32_t rx = s.ranges[2 * t], ry = s.ranges[2 * t + 1];
    for (int ly = 0; ly < BLOCK_Y; ++ly)
        for (int lx = 0; lx < BLOCK_X; ++lx) {
            const uint32_t px = tx * BLOCK_X + lx, py = ty * BLOCK_Y + ly;
            if (!(px < (uint32_t)W && py < (uint32_t)H)) continue;
            const uint32_t pix_id = W * py + px;
            const V2<R> pixf = {(R)px, (R)py};
            R T = 1;
            uint32_t contributor = 0, last_contributor = 0;
            R C[NUM_CHANNELS] = {0, 0, 0};
            for (uint32_t k = rx; k < ry; ++k) {
                contributor++;
                const uint32_t id = s.point_list[k];
                const V2<R> xy = s.means2D[id];
                const V2<R> d = {xy.x - pixf.x, xy.y - pixf.y};
                const V4<R> con_o = s.conic_opacity[id];
                const R power = R(-0.5f) * (con_o.x * d.x * d.x + con_o.z * d.y * d.y) - con_o.y * d.x * d.y;
                if (power > R(0)) continue;
                const R alpha = fmin_(R(0.99f), con_o.w * Math<R>::exp(power));
                if (alpha < R(1.0f / 255.0f)) continue;
                const R test_T = T * (R(1) - alpha);
                if (test_T < R(0.0001f)) break;  // done = true
                for (int ch = 0; ch < NUM_CHANNELS; ++ch) {
                    const R f = depth_mode ? s.depths[id] : features[id * NUM_CHANNELS + ch];
                    C[ch] += f * alpha * T;
                }
                T = test_T;
                last_contributor = contributor;
            }
            s.final_T[pix_id] = T;
            s.n_contrib[pix_id] = last_contributor;
            for (int ch = 0; ch < NUM_CHANNELS; ++ch)
                s.out_color[(size_t)ch * H * W + pix_id] = C[ch] + T * s.a.background[ch];
        }
}

// rasterizer_impl.cu:540-697 (LonlatRasterizer::forward) / :250-433 (Rasterizer::forward).
// Returns num_rendered; out_color is s.out_color ([3,H,W]); radii is s.radii.
template <typename R> int forward(State<R>& s, const Args<R>& in)
{
    s.a = in;
    Args<R>& a = s.a;
    const int P = a.P;
    const size_t N = (size_t)a.width * a.height;
    // keep private copies of all inputs (backward may run after the caller freed them)
    copy_in(s.bg, a.background, 3);
    copy_in(s.means3D, a.means3D, 3 * (size_t)P);
    copy_in(s.shs, a.shs, (size_t)P * a.M * 3);
    copy_in(s.colors_precomp, a.colors_precomp, 3 * (size_t)P);
    copy_in(s.opac, a.opacities, (size_t)P);
    copy_in(s.scales, a.scales, 3 * (size_t)P);
    copy_in(s.rots, a.rotations, 4 * (size_t)P);
    copy_in(s.cov3D_precomp, a.cov3D_precomp, 6 * (size_t)P);
    copy_in(s.view, a.viewmatrix, 16);
    copy_in(s.proj, a.projmatrix, 16);
    copy_in(s.campos, a.campos, 3);
    auto rp = [](std::vector<R>& v) -> const R* { return v.empty() ? nullptr : v.data(); };
    a.background = rp(s.bg); a.means3D = rp(s.means3D); a.shs = rp(s.shs); a.colors_precomp = rp(s.colors_precomp);
    a.opacities = rp(s.opac); a.scales = rp(s.scales); a.rotations = rp(s.rots); a.cov3D_precomp = rp(s.cov3D_precomp);
    a.viewmatrix = rp(s.view); a.projmatrix = rp(s.proj); a.campos = rp(s.campos);

    s.gx = (a.width + BLOCK_X - 1) / BLOCK_X;
    s.gy = (a.height + BLOCK_Y - 1) / BLOCK_Y;
    const uint32_t T = s.gx * s.gy;
    s.out_color.assign(3 * N, R(0));
    s.radii.assign(P, 0);
    s.depths.assign(P, R(0));
    s.clamped.assign(3 * (size_t)P, 0);
    s.means2D.assign(P, V2<R>{0, 0});
    s.cov3D.assign(6 * (size_t)P, R(0));
    s.conic_opacity.assign(P, V4<R>{0, 0, 0, 0});
    s.rgb.assign(3 * (size_t)P, R(0));
    s.tiles_touched.assign(P, 0);
    s.point_offsets.assign(P, 0);
    s.final_T.assign(N, R(0));
    s.n_contrib.assign(N, 0);
    s.ranges.assign(2 * (size_t)T, 0);
    s.keys.clear();
    s.point_list.clear();
    s.num_rendered = 0;
    if (P == 0) return 0;  // rasterize_points.cu:97 — all-zero image, empty buffers
    if (a.camera_type != 1 && a.camera_type != 3) throw std::runtime_error("[CudaRasterizer]Invalid camera_type");

    const R focal_y = (R)a.height / (R(2) * a.tan_fovy);  // rasterizer_impl.cu:275-276
    const R focal_x = (R)a.width / (R(2) * a.tan_fovx);

    // exceptions must not escape an OpenMP region: record and rethrow after it
    int prefiltered_violation = 0;
#pragma omp parallel for schedule(static) reduction(| : prefiltered_violation)
    for (int i = 0; i < P; ++i) {
        try {
            preprocess_one(s, i, focal_x, focal_y);
        } catch (const std::runtime_error&) {
            prefiltered_violation |= 1;
        }
    }
    if (prefiltered_violation)
        throw std::runtime_error("Point is filtered although prefiltered is set. This shouldn't happen!");

    // InclusiveSum (rasterizer_impl.cu:622)
    uint64_t acc = 0;
    for (int i = 0; i < P; ++i) {
        acc += s.tiles_touched[i];
        s.point_offsets[i] = (uint32_t)acc;
    }
    const int num_rendered = (int)s.point_offsets[P - 1];
    s.num_rendered = num_rendered;

    // duplicateWithKeys (rasterizer_impl.cu:94-140): every Gaussian writes its own slot range, so the loop is
    // parallel over Gaussians with the reference's per-Gaussian row-major emission order
    std::vector<uint64_t> keys_unsorted(num_rendered);
    std::vector<uint32_t> vals_unsorted(num_rendered);
#pragma omp parallel for schedule(dynamic, 1024)
    for (int idx = 0; idx < P; ++idx) {
        if (s.radii[idx] > 0) {
            uint32_t off = (idx == 0) ? 0 : s.point_offsets[idx - 1];
            Rect rc = getRect(s.means2D[idx], s.radii[idx], s.gx, s.gy);
            for (uint32_t y = rc.miny; y < rc.maxy; y++)
                for (uint32_t x = rc.minx; x < rc.maxx; x++) {
                    uint64_t key = (uint64_t)(y * s.gx + x);
                    key <<= 32;
                    key |= float_bits((float)s.depths[idx]);
                    keys_unsorted[off] = key;
                    vals_unsorted[off] = idx;
                    off++;
                }
        }
    }
    // SortPairs (rasterizer_impl.cu:656-661): stable LSD radix on bits [0, 32+bit). Its permutation is that of a
    // stable sort by the masked key (bits above 32+bit are zero because tile < T <= 2^bit), i.e. by
    // (tile, depth bits) with ties in emission order. Computed as a stable counting sort by tile (per-thread
    // contiguous chunks, so placement keeps emission order), then a stable sort by depth bits inside each tile:
    // the same permutation, in parallel.
    std::vector<uint32_t> perm(num_rendered);
    {
        const int nth = omp_get_max_threads();
        std::vector<uint32_t> cnt((size_t)nth * T, 0u);
        std::vector<uint32_t> tile_start(T + 1, 0u);
        const size_t L = (size_t)num_rendered;
        auto chunk = [&](int t, size_t& lo, size_t& hi) { lo = L * t / nth; hi = L * (t + 1) / nth; };
#pragma omp parallel num_threads(nth)
        {
            const int t = omp_get_thread_num();
            size_t lo, hi;
            chunk(t, lo, hi);
            uint32_t* c = &cnt[(size_t)t * T];
            for (size_t i = lo; i < hi; ++i) c[keys_unsorted[i] >> 32]++;
#pragma omp barrier
#pragma omp single
            {
                uint32_t run = 0;
                for (uint32_t tile = 0; tile < T; ++tile) {
                    tile_start[tile] = run;
                    for (int q = 0; q < nth; ++q) {
                        const uint32_t v = cnt[(size_t)q * T + tile];
                        cnt[(size_t)q * T + tile] = run;
                        run += v;
                    }
                }
                tile_start[T] = run;
            }
            for (size_t i = lo; i < hi; ++i) perm[c[keys_unsorted[i] >> 32]++] = (uint32_t)i;
        }
#pragma omp parallel for schedule(dynamic, 16)
        for (int tile = 0; tile < (int)T; ++tile)
            std::stable_sort(perm.begin() + tile_start[tile], perm.begin() + tile_start[tile + 1],
                             [&](uint32_t l, uint32_t r) {
                                 return (uint32_t)keys_unsorted[l] < (uint32_t)keys_unsorted[r];
                             });
    }
    s.keys.resize(num_rendered);
    s.point_list.resize(num_rendered);
#pragma omp parallel for schedule(static)
    for (int i = 0; i < num_rendered; ++i) {
        s.keys[i] = keys_unsorted[perm[i]];
        s.point_list[i] = vals_unsorted[perm[i]];
    }
    // identifyTileRanges (rasterizer_impl.cu:145-167)
    for (int idx = 0; idx < num_rendered; ++idx) {
        uint32_t currtile = (uint32_t)(s.keys[idx] >> 32);
        if (idx == 0) s.ranges[2 * currtile] = 0;
        else {
            uint32_t prevtile = (uint32_t)(s.keys[idx - 1] >> 32);
            if (currtile != prevtile) {
                s.ranges[2 * prevtile + 1] = idx;
                s.ranges[2 * currtile] = idx;
            }
        }
        if (idx == num_rendered - 1) s.ranges[2 * currtile + 1] = num_rendered;
    }
    // render (rasterizer_impl.cu:683, :398-430): lonlat never renders depth
    const bool depth_mode = a.render_depth && a.camera_type == 1;
    const R* features = a.colors_precomp != nullptr ? a.colors_precomp : s.rgb.data();
#pragma omp parallel for schedule(dynamic, 4)
    for (int t = 0; t < (int)T; ++t) render_tile(s, t % s.gx, t / s.gx, features, depth_mode);
    return num_rendered;
}

// ---------------------------------------------------------------------------------------------------------
// Backward
// ---------------------------------------------------------------------------------------------------------
template <typename R> struct Grads {
    std::vector<R> dmean2D;  // [P,3]
    std::vector<R> dconic;   // [P,4] (slots 0,1,3 used)
    std::vector<R> dopacity; // [P]
    std::vector<R> dcolor;   // [P,3]
    std::vector<R> dmean3D;  // [P,3]
    std::vector<R> dcov3D;   // [P,6]
    std::vector<R> dsh;      // [P,M,3]
    std::vector<R> dscale;   // [P,3]
    std::vector<R> drot;     // [P,4]
    void zero(int P, int M)
    {
        dmean2D.assign(3 * (size_t)P, 0); dconic.assign(4 * (size_t)P, 0); dopacity.assign(P, 0);
        dcolor.assign(3 * (size_t)P, 0); dmean3D.assign(3 * (size_t)P, 0); dcov3D.assign(6 * (size_t)P, 0);
        dsh.assign((size_t)P * M * 3, 0); dscale.assign(3 * (size_t)P, 0); drot.assign(4 * (size_t)P, 0);
    }
};

// backward.cu:671-843, one tile. Accumulation is sequential (tiles in order, pixels in thread-rank order,
// instances back to front), i.e. one fixed order of the reference's float atomicAdds.
template <typename R>
void render_backward_tile(const State<R>& s, uint32_t tx, uint32_t ty, const R* colors, const R* dL_dpixels, Grads<R>& g)
{
    const int W = s.a.width, H = s.a.height;
    const uint32_t t = ty * s.gx + tx;
    const uint32_t rx = s.ranges[2 * t], ry = s.ranges[2 * t + 1];
    const R ddelx_dx = (R)(0.5 * W);
    const R ddely_dy = (R)(0.5 * H);
    const R* bg = s.a.background;
    for (int ly = 0; ly < BLOCK_Y; ++ly)
        for (int lx = 0; lx < BLOCK_X; ++lx) {
            const uint32_t px = tx * BLOCK_X + lx, py = ty * BLOCK_Y + ly;
            if (!(px < (uint32_t)W && py < (uint32_t)H)) continue;
            const uint32_t pix_id = W * py + px;
            const V2<R> pixf = {(R)px, (R)py};
            const R T_final = s.final_T[pix_id];
            R T = T_final;
            uint32_t contributor = ry - rx;
            const uint32_t last_contributor = s.n_contrib[pix_id];
            R accum_rec[NUM_CHANNELS] = {0, 0, 0};
            R dL_dpixel[NUM_CHANNELS];
            for (int i = 0; i < NUM_CHANNELS; ++i) dL_dpixel[i] = dL_dpixels[(size_t)i * H * W + pix_id];
            R last_alpha = 0;
            R last_color[NUM_CHANNELS] = {0, 0, 0};
            for (uint32_t k = ry; k-- > rx;) {
                contributor--;
                if (contributor >= last_contributor) continue;
                const uint32_t gid = s.point_list[k];
                const V2<R> xy = s.means2D[gid];
                const V2<R> d = {xy.x - pixf.x, xy.y - pixf.y};
                const V4<R> con_o = s.conic_opacity[gid];
                const R power = R(-0.5f) * (con_o.x * d.x * d.x + con_o.z * d.y * d.y) - con_o.y * d.x * d.y;
                if (power > R(0)) continue;
                const R G = Math<R>::exp(power);
                const R alpha = fmin_(R(0.99f), con_o.w * G);
                if (alpha < R(1.0f / 255.0f)) continue;
                T = T / (R(1) - alpha);
                const R dchannel_dcolor = alpha * T;
                R dL_dalpha = 0;
                for (int ch = 0; ch < NUM_CHANNELS; ++ch) {
                    const R c = colors[gid * NUM_CHANNELS + ch];
                    accum_rec[ch] = last_alpha * last_color[ch] + (R(1) - last_alpha) * accum_rec[ch];
                    last_color[ch] = c;
                    const R dL_dchannel = dL_dpixel[ch];
                    dL_dalpha += (c - accum_rec[ch]) * dL_dchannel;
                    g.dcolor[gid * NUM_CHANNELS + ch] += dchannel_dcolor * dL_dchannel;
                }
                dL_dalpha *= T;
                last_alpha = alpha;
                R bg_dot_dpixel = 0;
                for (int i = 0; i < NUM_CHANNELS; ++i) bg_dot_dpixel += bg[i] * dL_dpixel[i];
                dL_dalpha += (-T_final / (R(1) - alpha)) * bg_dot_dpixel;
                const R dL_dG = con_o.w * dL_dalpha;
                const R gdx = G * d.x;
                const R gdy = G * d.y;
                const R dG_ddelx = -gdx * con_o.x - gdy * con_o.y;
                const R dG_ddely = -gdy * con_o.z - gdx * con_o.y;
                g.dmean2D[3 * gid + 0] += dL_dG * dG_ddelx * ddelx_dx;
                g.dmean2D[3 * gid + 1] += dL_dG * dG_ddely * ddely_dy;
                g.dconic[4 * gid + 0] += R(-0.5f) * gdx * d.x * dL_dG;
                g.dconic[4 * gid + 1] += R(-0.5f) * gdx * d.y * dL_dG;
                g.dconic[4 * gid + 3] += R(-0.5f) * gdy * d.y * dL_dG;
                g.dopacity[gid] += G * dL_dalpha;
            }
        }
}

// dL/dconic -> dL/dcov2D -> dL/dcov3D and dL/dT, shared by backward.cu:213-265 and :391-443
template <typename R> struct Cov2DBack {
    R dL_dT00, dL_dT01, dL_dT02, dL_dT10, dL_dT11, dL_dT12;
};
template <typename R>
Cov2DBack<R> cov2d_backward_common(const M3<R>& T, const M3<R>& Vrk, const V3<R>& dL_dconic, R* dL_dcov)
{
    M3<R> cov2D = transpose(T) * transpose(Vrk) * T;
    R a = cov2D[0][0] += R(0.3f);
    R b = cov2D[0][1];
    R c = cov2D[1][1] += R(0.3f);
    R denom = a * c - b * b;
    R dL_da = 0, dL_db = 0, dL_dc = 0;
    R denom2inv = R(1) / ((denom * denom) + R(0.0000001f));
    if (denom2inv != R(0)) {
        dL_da = denom2inv * (-c * c * dL_dconic.x + R(2) * b * c * dL_dconic.y + (denom - a * c) * dL_dconic.z);
        dL_dc = denom2inv * (-a * a * dL_dconic.z + R(2) * a * b * dL_dconic.y + (denom - a * c) * dL_dconic.x);
        dL_db = denom2inv * R(2) * (b * c * dL_dconic.x - (denom + R(2) * b * b) * dL_dconic.y + a * b * dL_dconic.z);
        dL_dcov[0] = (T[0][0] * T[0][0] * dL_da + T[0][0] * T[1][0] * dL_db + T[1][0] * T[1][0] * dL_dc);
        dL_dcov[3] = (T[0][1] * T[0][1] * dL_da + T[0][1] * T[1][1] * dL_db + T[1][1] * T[1][1] * dL_dc);
        dL_dcov[5] = (T[0][2] * T[0][2] * dL_da + T[0][2] * T[1][2] * dL_db + T[1][2] * T[1][2] * dL_dc);
        dL_dcov[1] = R(2) * T[0][0] * T[0][1] * dL_da + (T[0][0] * T[1][1] + T[0][1] * T[1][0]) * dL_db + R(2) * T[1][0] * T[1][1] * dL_dc;
        dL_dcov[2] = R(2) * T[0][0] * T[0][2] * dL_da + (T[0][0] * T[1][2] + T[0][2] * T[1][0]) * dL_db + R(2) * T[1][0] * T[1][2] * dL_dc;
        dL_dcov[4] = R(2) * T[0][2] * T[0][1] * dL_da + (T[0][1] * T[1][2] + T[0][2] * T[1][1]) * dL_db + R(2) * T[1][1] * T[1][2] * dL_dc;
    } else {
        for (int i = 0; i < 6; i++) dL_dcov[i] = 0;
    }
    Cov2DBack<R> o;
    o.dL_dT00 = R(2) * (T[0][0] * Vrk[0][0] + T[0][1] * Vrk[0][1] + T[0][2] * Vrk[0][2]) * dL_da +
                (T[1][0] * Vrk[0][0] + T[1][1] * Vrk[0][1] + T[1][2] * Vrk[0][2]) * dL_db;
    o.dL_dT01 = R(2) * (T[0][0] * Vrk[1][0] + T[0][1] * Vrk[1][1] + T[0][2] * Vrk[1][2]) * dL_da +
                (T[1][0] * Vrk[1][0] + T[1][1] * Vrk[1][1] + T[1][2] * Vrk[1][2]) * dL_db;
    o.dL_dT02 = R(2) * (T[0][0] * Vrk[2][0] + T[0][1] * Vrk[2][1] + T[0][2] * Vrk[2][2]) * dL_da +
                (T[1][0] * Vrk[2][0] + T[1][1] * Vrk[2][1] + T[1][2] * Vrk[2][2]) * dL_db;
    o.dL_dT10 = R(2) * (T[1][0] * Vrk[0][0] + T[1][1] * Vrk[0][1] + T[1][2] * Vrk[0][2]) * dL_dc +
                (T[0][0] * Vrk[0][0] + T[0][1] * Vrk[0][1] + T[0][2] * Vrk[0][2]) * dL_db;
    o.dL_dT11 = R(2) * (T[1][0] * Vrk[1][0] + T[1][1] * Vrk[1][1] + T[1][2] * Vrk[1][2]) * dL_dc +
                (T[0][0] * Vrk[1][0] + T[0][1] * Vrk[1][1] + T[0][2] * Vrk[1][2]) * dL_db;
    o.dL_dT12 = R(2) * (T[1][0] * Vrk[2][0] + T[1][1] * Vrk[2][1] + T[1][2] * Vrk[2][2]) * dL_dc +
                (T[0][0] * Vrk[2][0] + T[0][1] * Vrk[2][1] + T[0][2] * Vrk[2][2]) * dL_db;
    return o;
}

// backward.cu:156-292 (pinhole computeCov2DCUDA), one Gaussian
template <typename R>
void computeCov2D_backward(const State<R>& s, int idx, const R* cov3Ds, R h_x, R h_y, Grads<R>& g)
{
    const R* view_matrix = s.a.viewmatrix;
    const R* cov3D = cov3Ds + 6 * idx;
    V3<R> mean = {s.a.means3D[3 * idx], s.a.means3D[3 * idx + 1], s.a.means3D[3 * idx + 2]};
    V3<R> dL_dconic = {g.dconic[4 * idx], g.dconic[4 * idx + 1], g.dconic[4 * idx + 3]};
    V3<R> t = transformPoint4x3(mean, view_matrix);
    const R limx = R(1.3f) * s.a.tan_fovx;
    const R limy = R(1.3f) * s.a.tan_fovy;
    const R txtz = t.x / t.z;
    const R tytz = t.y / t.z;
    t.x = fmin_(limx, fmax_(-limx, txtz)) * t.z;
    t.y = fmin_(limy, fmax_(-limy, tytz)) * t.z;
    const R x_grad_mul = txtz < -limx || txtz > limx ? R(0) : R(1);
    const R y_grad_mul = tytz < -limy || tytz > limy ? R(0) : R(1);
    M3<R> J = M3<R>::cols(h_x / t.z, R(0), -(h_x * t.x) / (t.z * t.z), R(0), h_y / t.z, -(h_y * t.y) / (t.z * t.z), 0, 0, 0);
    M3<R> W = viewW(view_matrix);
    M3<R> Vrk = vrk(cov3D);
    M3<R> T = W * J;
    Cov2DBack<R> b = cov2d_backward_common(T, Vrk, dL_dconic, &g.dcov3D[6 * idx]);
    R dL_dJ00 = W[0][0] * b.dL_dT00 + W[0][1] * b.dL_dT01 + W[0][2] * b.dL_dT02;
    R dL_dJ02 = W[2][0] * b.dL_dT00 + W[2][1] * b.dL_dT01 + W[2][2] * b.dL_dT02;
    R dL_dJ11 = W[1][0] * b.dL_dT10 + W[1][1] * b.dL_dT11 + W[1][2] * b.dL_dT12;
    R dL_dJ12 = W[2][0] * b.dL_dT10 + W[2][1] * b.dL_dT11 + W[2][2] * b.dL_dT12;
    R tz = R(1) / t.z;
    R tz2 = tz * tz;
    R tz3 = tz2 * tz;
    R dL_dtx = x_grad_mul * -h_x * tz2 * dL_dJ02;
    R dL_dty = y_grad_mul * -h_y * tz2 * dL_dJ12;
    R dL_dtz = -h_x * tz2 * dL_dJ00 - h_y * tz2 * dL_dJ11 + (R(2) * h_x * t.x) * tz3 * dL_dJ02 + (R(2) * h_y * t.y) * tz3 * dL_dJ12;
    V3<R> dL_dmean = transformVec4x3Transpose(V3<R>{dL_dtx, dL_dty, dL_dtz}, view_matrix);
    g.dmean3D[3 * idx + 0] = dL_dmean.x;
    g.dmean3D[3 * idx + 1] = dL_dmean.y;
    g.dmean3D[3 * idx + 2] = dL_dmean.z;
}

// backward.cu:297-485 (computeCov2DLonLatCUDA), one Gaussian; also returns dpx_dt / dpy_dt
template <typename R>
void computeCov2DLonLat_backward(const State<R>& s, int idx, const R* cov3Ds, Grads<R>& g, V3<R>& dpx_dt, V3<R>& dpy_dt)
{
    const R* view_matrix = s.a.viewmatrix;
    const int width = s.a.width, height = s.a.height;
    const R* cov3D = cov3Ds + 6 * idx;
    V3<R> mean = {s.a.means3D[3 * idx], s.a.means3D[3 * idx + 1], s.a.means3D[3 * idx + 2]};
    V3<R> dL_dconic = {g.dconic[4 * idx], g.dconic[4 * idx + 1], g.dconic[4 * idx + 3]};
    V3<R> t = transformPoint4x3(mean, view_matrix);
    R txtx = t.x * t.x;
    R tyty = t.y * t.y;
    R tztz = t.z * t.z;
    R txtytz = t.x * t.y * t.z;
    R trxztrxz = txtx + tztz;
    R trxztrxz_inv = R(1) / (trxztrxz + R(0.0000001f));
    R trxztrxztrxztrxz_inv = trxztrxz_inv * trxztrxz_inv;
    R trxz = Math<R>::sqrt(trxztrxz);
    R trxz_inv = R(1) / (trxz + R(0.0000001f));
    R trtr = trxztrxz + tyty;
    R trtr_inv = R(1) / (trtr + R(0.0000001f));
    R trtrtrtr_inv = trtr_inv * trtr_inv;
    R trxz_trtrtrtr_inv = trxz_inv * trtrtrtr_inv;
    R trxztrxztrxz_trtrtrtr_inv = trxztrxz_inv * trxz_trtrtrtr_inv;
    R tyty_minus_trxztrxz = tyty - trxztrxz;
    R W_div_2pi = (R)width * R(0.5f) * R_1_PI<R>;
    R H_div_pi = (R)height * R_1_PI<R>;
    R dpx_dtx = W_div_2pi * t.z * trxztrxz_inv;
    R dpx_dtz = -W_div_2pi * t.x * trxztrxz_inv;
    R dpy_dtx = -H_div_pi * t.x * t.y * trxz_inv * trtr_inv;
    R dpy_dty = H_div_pi * trxz * trtr_inv;
    R dpy_dtz = -H_div_pi * t.z * t.y * trxz_inv * trtr_inv;
    dpx_dt = {dpx_dtx, R(0), dpx_dtz};
    dpy_dt = {dpy_dtx, dpy_dty, dpy_dtz};
    M3<R> J = M3<R>::cols(dpx_dtx, R(0), dpx_dtz, dpy_dtx, dpy_dty, dpy_dtz, R(0), R(0), R(0));
    M3<R> W = viewW(view_matrix);
    M3<R> Vrk = vrk(cov3D);
    M3<R> T = W * J;
    Cov2DBack<R> b = cov2d_backward_common(T, Vrk, dL_dconic, &g.dcov3D[6 * idx]);
    R dL_dJ00 = W[0][0] * b.dL_dT00 + W[0][1] * b.dL_dT01 + W[0][2] * b.dL_dT02;
    R dL_dJ02 = W[2][0] * b.dL_dT00 + W[2][1] * b.dL_dT01 + W[2][2] * b.dL_dT02;
    R dL_dJ10 = W[0][0] * b.dL_dT10 + W[0][1] * b.dL_dT11 + W[0][2] * b.dL_dT12;
    R dL_dJ11 = W[1][0] * b.dL_dT10 + W[1][1] * b.dL_dT11 + W[1][2] * b.dL_dT12;
    R dL_dJ12 = W[2][0] * b.dL_dT10 + W[2][1] * b.dL_dT11 + W[2][2] * b.dL_dT12;
    R temp1 = H_div_pi * tyty_minus_trxztrxz * trxz_trtrtrtr_inv;
    R temp2 = H_div_pi * txtytz * (trtr + R(2) * trxztrxz) * trxztrxztrxz_trtrtrtr_inv;
    R temp3 = W_div_2pi * (txtx - tztz) * trxztrxztrxztrxz_inv;
    R temp4 = W_div_2pi * R(2) * t.x * t.z * trxztrxztrxztrxz_inv;
    R temp5 = H_div_pi * t.y * trxztrxztrxz_trtrtrtr_inv;
    R dL_dtx = -dL_dJ00 * temp4 + dL_dJ02 * temp3 + dL_dJ10 * temp5 * (R(2) * txtx * trxztrxz - tztz * trtr) +
               dL_dJ11 * t.x * temp1 + dL_dJ12 * temp2;
    R dL_dty = dL_dJ10 * t.x * temp1 - dL_dJ11 * H_div_pi * R(2) * trxz * t.y * trtrtrtr_inv + dL_dJ12 * t.z * temp1;
    R dL_dtz = dL_dJ00 * temp3 + dL_dJ02 * temp4 + dL_dJ10 * temp2 + dL_dJ11 * t.z * temp1 +
               dL_dJ12 * temp5 * (R(2) * tztz * trxztrxz - txtx * trtr);
    V3<R> dL_dmean = transformVec4x3Transpose(V3<R>{dL_dtx, dL_dty, dL_dtz}, view_matrix);
    g.dmean3D[3 * idx + 0] = dL_dmean.x;
    g.dmean3D[3 * idx + 1] = dL_dmean.y;
    g.dmean3D[3 * idx + 2] = dL_dmean.z;
}

// backward.cu:30-151 (SH backward), one Gaussian. glm expressions are evaluated left to right:
// (C * y) * sh[k] is scalar*vec3; C * sh[k] * a * b is ((vec3 * a) * b).
template <typename R> void computeColorFromSH_backward(const State<R>& s, int idx, Grads<R>& g)
{
    using S = SH<R>;
    const int deg = s.a.D, max_coeffs = s.a.M;
    V3<R> pos = {s.a.means3D[3 * idx], s.a.means3D[3 * idx + 1], s.a.means3D[3 * idx + 2]};
    V3<R> cp = {s.a.campos[0], s.a.campos[1], s.a.campos[2]};
    V3<R> dir_orig = pos - cp;
    V3<R> dir = dir_orig / Math<R>::sqrt(dot3(dir_orig, dir_orig));
    const R* b = s.a.shs + (size_t)idx * max_coeffs * 3;
    auto sh = [&](int k) { return V3<R>{b[3 * k], b[3 * k + 1], b[3 * k + 2]}; };
    auto vs = [](V3<R> v, R f) { return V3<R>{v.x * f, v.y * f, v.z * f}; };  // vec3 * scalar
    V3<R> dL_dRGB = {g.dcolor[3 * idx], g.dcolor[3 * idx + 1], g.dcolor[3 * idx + 2]};
    dL_dRGB.x *= s.clamped[3 * idx + 0] ? R(0) : R(1);
    dL_dRGB.y *= s.clamped[3 * idx + 1] ? R(0) : R(1);
    dL_dRGB.z *= s.clamped[3 * idx + 2] ? R(0) : R(1);
    V3<R> dRGBdx = {0, 0, 0}, dRGBdy = {0, 0, 0}, dRGBdz = {0, 0, 0};
    R x = dir.x, y = dir.y, z = dir.z;
    R* dsh = g.dsh.data() + (size_t)idx * max_coeffs * 3;
    auto put = [&](int k, R coef) {
        V3<R> v = coef * dL_dRGB;
        dsh[3 * k] = v.x; dsh[3 * k + 1] = v.y; dsh[3 * k + 2] = v.z;
    };
    put(0, S::C0);
    if (deg > 0) {
        put(1, -S::C1 * y);
        put(2, S::C1 * z);
        put(3, -S::C1 * x);
        dRGBdx = -S::C1 * sh(3);
        dRGBdy = -S::C1 * sh(1);
        dRGBdz = S::C1 * sh(2);
        if (deg > 1) {
            R xx = x * x, yy = y * y, zz = z * z;
            R xy = x * y, yz = y * z, xz = x * z;
            put(4, S::C2[0] * xy);
            put(5, S::C2[1] * yz);
            put(6, S::C2[2] * (R(2) * zz - xx - yy));
            put(7, S::C2[3] * xz);
            put(8, S::C2[4] * (xx - yy));
            dRGBdx += (S::C2[0] * y) * sh(4) + (S::C2[2] * R(2) * -x) * sh(6) + (S::C2[3] * z) * sh(7) + (S::C2[4] * R(2) * x) * sh(8);
            dRGBdy += (S::C2[0] * x) * sh(4) + (S::C2[1] * z) * sh(5) + (S::C2[2] * R(2) * -y) * sh(6) + (S::C2[4] * R(2) * -y) * sh(8);
            dRGBdz += (S::C2[1] * y) * sh(5) + (S::C2[2] * R(2) * R(2) * z) * sh(6) + (S::C2[3] * x) * sh(7);
            if (deg > 2) {
                put(9, S::C3[0] * y * (R(3) * xx - yy));
                put(10, S::C3[1] * xy * z);
                put(11, S::C3[2] * y * (R(4) * zz - xx - yy));
                put(12, S::C3[3] * z * (R(2) * zz - R(3) * xx - R(3) * yy));
                put(13, S::C3[4] * x * (R(4) * zz - xx - yy));
                put(14, S::C3[5] * z * (xx - yy));
                put(15, S::C3[6] * x * (xx - R(3) * yy));
                dRGBdx += (vs(vs(vs(S::C3[0] * sh(9), R(3)), R(2)), xy) + vs(S::C3[1] * sh(10), yz) +
                           vs(vs(S::C3[2] * sh(11), R(-2)), xy) + vs(vs(vs(S::C3[3] * sh(12), R(-3)), R(2)), xz) +
                           vs(S::C3[4] * sh(13), (R(-3) * xx + R(4) * zz - yy)) + vs(vs(S::C3[5] * sh(14), R(2)), xz) +
                           vs(vs(S::C3[6] * sh(15), R(3)), (xx - yy)));
                dRGBdy += (vs(vs(S::C3[0] * sh(9), R(3)), (xx - yy)) + vs(S::C3[1] * sh(10), xz) +
                           vs(S::C3[2] * sh(11), (R(-3) * yy + R(4) * zz - xx)) + vs(vs(vs(S::C3[3] * sh(12), R(-3)), R(2)), yz) +
                           vs(vs(S::C3[4] * sh(13), R(-2)), xy) + vs(vs(S::C3[5] * sh(14), R(-2)), yz) +
                           vs(vs(vs(S::C3[6] * sh(15), R(-3)), R(2)), xy));
                dRGBdz += (vs(S::C3[1] * sh(10), xy) + vs(vs(vs(S::C3[2] * sh(11), R(4)), R(2)), yz) +
                           vs(vs(S::C3[3] * sh(12), R(3)), (R(2) * zz - xx - yy)) + vs(vs(vs(S::C3[4] * sh(13), R(4)), R(2)), xz) +
                           vs(S::C3[5] * sh(14), (xx - yy)));
            }
        }
    }
    V3<R> dL_ddir = {dot3(dRGBdx, dL_dRGB), dot3(dRGBdy, dL_dRGB), dot3(dRGBdz, dL_dRGB)};
    V3<R> dL_dmean = dnormvdv(dir_orig, dL_ddir);
    g.dmean3D[3 * idx + 0] += dL_dmean.x;
    g.dmean3D[3 * idx + 1] += dL_dmean.y;
    g.dmean3D[3 * idx + 2] += dL_dmean.z;
}

// backward.cu:489-552 (computeCov3D backward), one Gaussian
template <typename R> void computeCov3D_backward(const State<R>& s, int idx, Grads<R>& g)
{
    V3<R> scale = {s.a.scales[3 * idx], s.a.scales[3 * idx + 1], s.a.scales[3 * idx + 2]};
    R mod = s.a.scale_modifier;
    V4<R> q = {s.a.rotations[4 * idx], s.a.rotations[4 * idx + 1], s.a.rotations[4 * idx + 2], s.a.rotations[4 * idx + 3]};
    R r = q.x, x = q.y, y = q.z, z = q.w;
    M3<R> Rm = M3<R>::cols(R(1) - R(2) * (y * y + z * z), R(2) * (x * y - r * z), R(2) * (x * z + r * y),
                           R(2) * (x * y + r * z), R(1) - R(2) * (x * x + z * z), R(2) * (y * z - r * x),
                           R(2) * (x * z - r * y), R(2) * (y * z + r * x), R(1) - R(2) * (x * x + y * y));
    M3<R> S = M3<R>::identity();
    V3<R> sv = mod * scale;
    S[0][0] = sv.x;
    S[1][1] = sv.y;
    S[2][2] = sv.z;
    M3<R> M = S * Rm;
    const R* d = &g.dcov3D[6 * idx];
    M3<R> dL_dSigma = M3<R>::cols(d[0], R(0.5f) * d[1], R(0.5f) * d[2], R(0.5f) * d[1], d[3], R(0.5f) * d[4],
                                  R(0.5f) * d[2], R(0.5f) * d[4], d[5]);
    M3<R> dL_dM = R(2) * M * dL_dSigma;  // (2*M) * dL_dSigma
    M3<R> Rt = transpose(Rm);
    M3<R> dL_dMt = transpose(dL_dM);
    R* ds = &g.dscale[3 * idx];
    ds[0] = dot3(col(Rt, 0), col(dL_dMt, 0));
    ds[1] = dot3(col(Rt, 1), col(dL_dMt, 1));
    ds[2] = dot3(col(Rt, 2), col(dL_dMt, 2));
    for (int k = 0; k < 3; ++k) dL_dMt[0][k] *= sv.x;
    for (int k = 0; k < 3; ++k) dL_dMt[1][k] *= sv.y;
    for (int k = 0; k < 3; ++k) dL_dMt[2][k] *= sv.z;
    R* dq = &g.drot[4 * idx];
    dq[0] = R(2) * z * (dL_dMt[0][1] - dL_dMt[1][0]) + R(2) * y * (dL_dMt[2][0] - dL_dMt[0][2]) + R(2) * x * (dL_dMt[1][2] - dL_dMt[2][1]);
    dq[1] = R(2) * y * (dL_dMt[1][0] + dL_dMt[0][1]) + R(2) * z * (dL_dMt[2][0] + dL_dMt[0][2]) + R(2) * r * (dL_dMt[1][2] - dL_dMt[2][1]) - R(4) * x * (dL_dMt[2][2] + dL_dMt[1][1]);
    dq[2] = R(2) * x * (dL_dMt[1][0] + dL_dMt[0][1]) + R(2) * r * (dL_dMt[2][0] - dL_dMt[0][2]) + R(2) * z * (dL_dMt[1][2] + dL_dMt[2][1]) - R(4) * y * (dL_dMt[2][2] + dL_dMt[0][0]);
    dq[3] = R(2) * r * (dL_dMt[0][1] - dL_dMt[1][0]) + R(2) * x * (dL_dMt[2][0] + dL_dMt[0][2]) + R(2) * y * (dL_dMt[1][2] + dL_dMt[2][1]) - R(4) * z * (dL_dMt[1][1] + dL_dMt[0][0]);
}

// backward.cu:557-608 (pinhole preprocessCUDA backward) and :613-669 (preprocessLonLatCUDA), one Gaussian
template <typename R>
void preprocess_backward_one(const State<R>& s, int idx, const V3<R>& dpx_dt, const V3<R>& dpy_dt, Grads<R>& g)
{
    V3<R> m = {s.a.means3D[3 * idx], s.a.means3D[3 * idx + 1], s.a.means3D[3 * idx + 2]};
    const R dm2x = g.dmean2D[3 * idx], dm2y = g.dmean2D[3 * idx + 1];
    V3<R> dL_dmean;
    if (s.a.camera_type == 3) {
        R dsx_dpx = R(2) / (R)s.a.width;
        R dsy_dpy = R(2) / (R)s.a.height;
        R dL_dpx = dm2x * dsx_dpx;
        R dL_dpy = dm2y * dsy_dpy;
        R dL_dtx = dL_dpx * dpx_dt.x + dL_dpy * dpy_dt.x;
        R dL_dty = dL_dpx * dpx_dt.y + dL_dpy * dpy_dt.y;
        R dL_dtz = dL_dpx * dpx_dt.z + dL_dpy * dpy_dt.z;
        dL_dmean = transformVec4x3Transpose(V3<R>{dL_dtx, dL_dty, dL_dtz}, s.a.viewmatrix);
    } else {
        const R* proj = s.a.projmatrix;
        V4<R> m_hom = transformPoint4x4(m, proj);
        R m_w = R(1) / (m_hom.w + R(0.0000001f));
        R mul1 = (proj[0] * m.x + proj[4] * m.y + proj[8] * m.z + proj[12]) * m_w * m_w;
        R mul2 = (proj[1] * m.x + proj[5] * m.y + proj[9] * m.z + proj[13]) * m_w * m_w;
        dL_dmean.x = (proj[0] * m_w - proj[3] * mul1) * dm2x + (proj[1] * m_w - proj[3] * mul2) * dm2y;
        dL_dmean.y = (proj[4] * m_w - proj[7] * mul1) * dm2x + (proj[5] * m_w - proj[7] * mul2) * dm2y;
        dL_dmean.z = (proj[8] * m_w - proj[11] * mul1) * dm2x + (proj[9] * m_w - proj[11] * mul2) * dm2y;
    }
    g.dmean3D[3 * idx + 0] += dL_dmean.x;
    g.dmean3D[3 * idx + 1] += dL_dmean.y;
    g.dmean3D[3 * idx + 2] += dL_dmean.z;
    if (s.a.shs) computeColorFromSH_backward(s, idx, g);
    if (s.a.scales) computeCov3D_backward(s, idx, g);
}

// rasterizer_impl.cu:701-795 (LonlatRasterizer::backward) / :437-535 (Rasterizer::backward).
// dL_dpix is [3,H,W]. Grads are zero-initialised first, as RasterizeGaussiansBackwardCUDA does
// (src/rasterize_points.cu:200-208). With nthreads > 1 the render backward accumulates into per-thread
// buffers which are then summed in thread order (same algorithm, different float summation order).
template <typename R> void backward(const State<R>& s, const R* dL_dpix, Grads<R>& g, int nthreads = 1)
{
    const int P = s.a.P;
    g.zero(P, s.a.M);
    if (P == 0) return;
    const R* colors = s.a.colors_precomp != nullptr ? s.a.colors_precomp : s.rgb.data();
    const int T = (int)(s.gx * s.gy);
    if (nthreads <= 1) {
        for (int t = 0; t < T; ++t) render_backward_tile(s, t % s.gx, t / s.gx, colors, dL_dpix, g);
    } else {
        std::vector<Grads<R>> part(nthreads);
#pragma omp parallel num_threads(nthreads)
        {
            int tid = 0;
#ifdef _OPENMP
            tid = omp_get_thread_num();
#endif
            Grads<R>& pg = part[tid];
            pg.dmean2D.assign(3 * (size_t)P, 0); pg.dconic.assign(4 * (size_t)P, 0);
            pg.dopacity.assign(P, 0); pg.dcolor.assign(3 * (size_t)P, 0);
#pragma omp for schedule(dynamic, 4)
            for (int t = 0; t < T; ++t) render_backward_tile(s, t % s.gx, t / s.gx, colors, dL_dpix, pg);
        }
        for (int tid = 0; tid < nthreads; ++tid) {
            for (size_t i = 0; i < g.dmean2D.size(); ++i) g.dmean2D[i] += part[tid].dmean2D[i];
            for (size_t i = 0; i < g.dconic.size(); ++i) g.dconic[i] += part[tid].dconic[i];
            for (size_t i = 0; i < g.dopacity.size(); ++i) g.dopacity[i] += part[tid].dopacity[i];
            for (size_t i = 0; i < g.dcolor.size(); ++i) g.dcolor[i] += part[tid].dcolor[i];
        }
    }
    const R* cov3D_ptr = s.a.cov3D_precomp != nullptr ? s.a.cov3D_precomp : s.cov3D.data();
    const R focal_y = (R)s.a.height / (R(2) * s.a.tan_fovy);
    const R focal_x = (R)s.a.width / (R(2) * s.a.tan_fovx);
#pragma omp parallel for schedule(static) num_threads(nthreads)
    for (int idx = 0; idx < P; ++idx) {
        if (!(s.radii[idx] > 0)) continue;
        V3<R> dpx_dt = {0, 0, 0}, dpy_dt = {0, 0, 0};
        if (s.a.camera_type == 3) computeCov2DLonLat_backward(s, idx, cov3D_ptr, g, dpx_dt, dpy_dt);
        else computeCov2D_backward(s, idx, cov3D_ptr, focal_x, focal_y, g);
        preprocess_backward_one(s, idx, dpx_dt, dpy_dt, g);
    }
}

// rasterize_points.cu:287-319 / rasterizer_impl.cu:66-90
template <typename R> void markVisible(int P, const R* means3D, const R* viewmatrix, const R* projmatrix, int camera_type, uint8_t* present)
{
    for (int i = 0; i < P; ++i) {
        if (camera_type == 3) { present[i] = 1; continue; }
        V3<R> p = {means3D[3 * i], means3D[3 * i + 1], means3D[3 * i + 2]};
        V3<R> pv;
        present[i] = in_frustum(p, viewmatrix, projmatrix, false, pv) ? 1 : 0;
    }
}

}  // namespace oracle

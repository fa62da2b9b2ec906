// sh_eval.h — spherical-harmonics evaluation shared by the forward preprocess, the per-Gaussian backward and the
// view-parallel SH-gradient reconstruction (preprocess.hip, gaussian_bwd.hip). One implementation, so the colour,
// its clamp bits and the basis values come out bit-identical wherever they are recomputed.
#pragma once

#include "raster_common.h"

namespace omr {

constexpr float SH_C0 = 0.28209479177387814f;  // auxiliary.h:32-49
constexpr float SH_C1 = 0.4886025119029199f;
constexpr float SH_C2[5] = {1.0925484305920792f, -1.0925484305920792f, 0.31539156525252005f, -1.0925484305920792f,
                            0.5462742152960396f};
constexpr float SH_C3[7] = {-0.5900435899266435f, 2.890611442640554f, -0.4570457994644658f, 0.3731763325901154f,
                            -0.4570457994644658f, 1.445305721320277f, -0.5900435899266435f};

// the unit view direction of forward.cu:37-38 / backward.cu:40-41: normalize(mean - campos)
__device__ __forceinline__ void sh_direction(float px, float py, float pz, const float* campos, float& x, float& y,
                                             float& z)
{
    const float dx = px - campos[0], dy = py - campos[1], dz = pz - campos[2];
    const float len = sqrtf(dx * dx + dy * dy + dz * dz);
    x = dx / len;
    y = dy / len;
    z = dz / len;
}

// forward.cu:30-83, one channel at a time (glm vec3 ops are componentwise, same order)
__device__ __forceinline__ void sh_to_rgb(int deg, float x, float y, float z, const float* sh, float out[3],
                                          uint8_t& clamp_bits)
{
    clamp_bits = 0;
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
        auto s = [&](int k) { return sh[3 * k + ch]; };
        float res = SH_C0 * s(0);
        if (deg > 0) {
            res = res - SH_C1 * y * s(1) + SH_C1 * z * s(2) - SH_C1 * x * s(3);
            if (deg > 1) {
                const float xx = x * x, yy = y * y, zz = z * z;
                const float xy = x * y, yz = y * z, xz = x * z;
                res = res + SH_C2[0] * xy * s(4) + SH_C2[1] * yz * s(5) + SH_C2[2] * (2.0f * zz - xx - yy) * s(6) +
                      SH_C2[3] * xz * s(7) + SH_C2[4] * (xx - yy) * s(8);
                if (deg > 2) {
                    res = res + SH_C3[0] * y * (3.0f * xx - yy) * s(9) + SH_C3[1] * xy * z * s(10) +
                          SH_C3[2] * y * (4.0f * zz - xx - yy) * s(11) +
                          SH_C3[3] * z * (2.0f * zz - 3.0f * xx - 3.0f * yy) * s(12) +
                          SH_C3[4] * x * (4.0f * zz - xx - yy) * s(13) + SH_C3[5] * z * (xx - yy) * s(14) +
                          SH_C3[6] * x * (xx - 3.0f * yy) * s(15);
                }
            }
        }
        res += 0.5f;
        if (res < 0) clamp_bits |= (uint8_t)(1u << ch);
        out[ch] = fmaxf(res, 0.0f);
    }
}

// dRGB/ddir of backward.cu:56-112 per channel (gx = dRGB/dx etc.), s(k, ch) = coefficient k of channel ch. They depend
// on the SH row and the view direction only, so the forward evaluates them where it has the row in registers
// (preprocess.hip, stored as GeomState::sh_jac) and gaussian_bwd reads 36 B instead of the 192-B row; both sites run this
// one function, compiled without contraction, so the values are the same bits either way.
template <class S>
__device__ __forceinline__ void sh_dir_grad(int deg, float x, float y, float z, S s, float gx[3], float gy[3],
                                            float gz[3])
{
    const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
        gx[ch] = gy[ch] = gz[ch] = 0.f;
        if (deg > 0) {
            gx[ch] = -SH_C1 * s(3, ch);
            gy[ch] = -SH_C1 * s(1, ch);
            gz[ch] = SH_C1 * s(2, ch);
            if (deg > 1) {
                gx[ch] += SH_C2[0] * y * s(4, ch) + SH_C2[2] * 2.f * -x * s(6, ch) + SH_C2[3] * z * s(7, ch) +
                          SH_C2[4] * 2.f * x * s(8, ch);
                gy[ch] += SH_C2[0] * x * s(4, ch) + SH_C2[1] * z * s(5, ch) + SH_C2[2] * 2.f * -y * s(6, ch) +
                          SH_C2[4] * 2.f * -y * s(8, ch);
                gz[ch] += SH_C2[1] * y * s(5, ch) + SH_C2[2] * 2.f * 2.f * z * s(6, ch) + SH_C2[3] * x * s(7, ch);
                if (deg > 2) {
                    gx[ch] += (SH_C3[0] * s(9, ch) * 3.f * 2.f * xy + SH_C3[1] * s(10, ch) * yz +
                               SH_C3[2] * s(11, ch) * -2.f * xy + SH_C3[3] * s(12, ch) * -3.f * 2.f * xz +
                               SH_C3[4] * s(13, ch) * (-3.f * xx + 4.f * zz - yy) + SH_C3[5] * s(14, ch) * 2.f * xz +
                               SH_C3[6] * s(15, ch) * 3.f * (xx - yy));
                    gy[ch] += (SH_C3[0] * s(9, ch) * 3.f * (xx - yy) + SH_C3[1] * s(10, ch) * xz +
                               SH_C3[2] * s(11, ch) * (-3.f * yy + 4.f * zz - xx) +
                               SH_C3[3] * s(12, ch) * -3.f * 2.f * yz + SH_C3[4] * s(13, ch) * -2.f * xy +
                               SH_C3[5] * s(14, ch) * -2.f * yz + SH_C3[6] * s(15, ch) * -3.f * 2.f * xy);
                    gz[ch] += (SH_C3[1] * s(10, ch) * xy + SH_C3[2] * s(11, ch) * 4.f * 2.f * yz +
                               SH_C3[3] * s(12, ch) * 3.f * (2.f * zz - xx - yy) + SH_C3[4] * s(13, ch) * 4.f * 2.f * xz +
                               SH_C3[5] * s(14, ch) * (xx - yy));
                }
            }
        }
    }
}

// dRGB/dsh_k of backward.cu:56-112 (the SH basis values): coef[k] for k < (deg+1)^2, zero beyond
__device__ __forceinline__ void sh_basis(int deg, float x, float y, float z, float coef[16])
{
#pragma unroll
    for (int k = 0; k < 16; ++k) coef[k] = 0.f;
    coef[0] = SH_C0;
    const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
    if (deg > 0) {
        coef[1] = -SH_C1 * y;
        coef[2] = SH_C1 * z;
        coef[3] = -SH_C1 * x;
        if (deg > 1) {
            coef[4] = SH_C2[0] * xy;
            coef[5] = SH_C2[1] * yz;
            coef[6] = SH_C2[2] * (2.f * zz - xx - yy);
            coef[7] = SH_C2[3] * xz;
            coef[8] = SH_C2[4] * (xx - yy);
            if (deg > 2) {
                coef[9] = SH_C3[0] * y * (3.f * xx - yy);
                coef[10] = SH_C3[1] * xy * z;
                coef[11] = SH_C3[2] * y * (4.f * zz - xx - yy);
                coef[12] = SH_C3[3] * z * (2.f * zz - 3.f * xx - 3.f * yy);
                coef[13] = SH_C3[4] * x * (4.f * zz - xx - yy);
                coef[14] = SH_C3[5] * z * (xx - yy);
                coef[15] = SH_C3[6] * x * (xx - 3.f * yy);
            }
        }
    }
}

}  // namespace omr

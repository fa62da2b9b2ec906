// omni_math.h — float transcendentals shared bit-for-bit by the gfx950 kernels and the CPU oracle.
//
// Why this exists: tile membership of a Gaussian is decided by float expressions such as
// (int)((p.x - r) / 16) where p.x comes from atan2f/asinf (reference cuda_rasterizer/auxiliary.h:236-248).
// CUDA libdevice, ROCm OCML and glibc implement atan2f/asinf differently, so the same input can land on a
// different tile when p.x is within an ulp of a tile boundary. To make radii / rects / sort keys bit-exact
// between the HIP path and the oracle, both call these implementations, built only from +,-,*,/ and sqrt
// (all IEEE correctly rounded on gfx950 with -fhip-fp32-correctly-rounded-divide-sqrt, and on x86 SSE), and
// both are compiled without FMA contraction (-ffp-contract=off).
//
// Accuracy (tests/test_math.py checks it against libm in double): atan2f <= 3 ulp, asinf <= 3 ulp over the
// domain the rasterizer uses. Algorithms: Cephes-style minimax polynomials (public domain, S. Moshier),
// restated here.
#pragma once

#if defined(__HIPCC__)
#define OMNI_HD __host__ __device__ __forceinline__
#else
#define OMNI_HD inline
#endif

namespace omni {

#if defined(__clang__)
#pragma clang fp contract(off)
#endif

// atan(x) for x in [0, 1].
OMNI_HD float atan_unit(float x)
{
    // reduce to |x| <= tan(pi/8)
    float y0 = 0.0f;
    if (x > 0.41421356237309504880f) {
        y0 = 0.78539816339744830962f;
        x = (x - 1.0f) / (x + 1.0f);
    }
    const float z = x * x;
    float p = 8.05374449538e-2f;
    p = p * z - 1.38776856032e-1f;
    p = p * z + 1.99777106478e-1f;
    p = p * z - 3.33329491539e-1f;
    const float y = p * z * x + x;
    return y0 + y;
}

// IEEE-style atan2f(y, x) including signed zeros; NaN in -> NaN out.
OMNI_HD float atan2f_(float y, float x)
{
    if (y != y || x != x) return y + x;
    const float ay = y < 0.0f ? -y : y;
    const float ax = x < 0.0f ? -x : x;
    const bool y_neg = (y < 0.0f) || (y == 0.0f && 1.0f / y < 0.0f);
    const bool x_neg = (x < 0.0f) || (x == 0.0f && 1.0f / x < 0.0f);
    float a;
    if (ay == 0.0f && ax == 0.0f) {
        a = x_neg ? 3.14159265358979323846f : 0.0f;
    } else if (ax == ay) {
        a = 0.78539816339744830962f;
        if (x_neg) a = 2.35619449019234492885f;
    } else {
        // inputs of the rasterizer are finite; inf/inf handled by the ratio path (NaN)
        if (ay > ax) {
            a = 1.57079632679489661923f - atan_unit(ax / ay);
        } else {
            a = atan_unit(ay / ax);
        }
        if (x_neg) a = 3.14159265358979323846f - a;
    }
    return y_neg ? -a : a;
}

// asinf(x); |x| > 1 -> NaN.
OMNI_HD float asinf_(float x)
{
    const bool neg = x < 0.0f;
    const float a = neg ? -x : x;
    if (a > 1.0f || x != x) return (x - x) / (x - x);  // NaN
    if (a < 1.0e-4f) return x;
    float z, w;
    bool big = false;
    if (a > 0.5f) {
        z = 0.5f * (1.0f - a);
        w = __builtin_sqrtf(z);
        big = true;
    } else {
        w = a;
        z = a * a;
    }
    float p = 4.2163199048e-2f;
    p = p * z + 2.4181311049e-2f;
    p = p * z + 4.5470025998e-2f;
    p = p * z + 7.4953002686e-2f;
    p = p * z + 1.6666752422e-1f;
    float r = p * z * w + w;
    if (big) {
        r = r + r;
        r = 1.57079632679489661923f - r;
    }
    return neg ? -r : r;
}

}  // namespace omni

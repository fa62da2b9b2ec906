// ambiguity.hpp — how much of a result the missing reference run could still move (TEST INFRASTRUCTURE ONLY).
//
// The oracle is a restatement: no run of the CUDA reference pins it. Where the reference's own
// arithmetic could decide differently from ours, a parity claim rests on the restatement alone. This counts those
// places on a forward the oracle has just run (SURVEY.md §7 "Hard parts" 1, VERDICT r1 "quantify the unpinned
// residual"):
//
//  * rect-ambiguous Gaussians: lonlat pixel centres come from atan2f / asinf (auxiliary.h:236-248), which CUDA
//    libdevice, ROCm OCML, glibc and our shared omni_math.h may round differently (<= 3 ulp measured against glibc,
//    tests/test_math.py). A Gaussian whose getRect (auxiliary.h:56-66) changes when lon or lat moves by up to
//    `ulps` ulp (every combination) could own other tiles -> other keys and point lists in the reference;
//  * threshold pixels: a blend decision within `eps` (relative) of a threshold, alpha at 1/255
//    (forward.cu:436-437) or T (1 - alpha) at 1e-4 (:440-444), where exp implementations (libdevice expf, v_exp_f32,
//    glibc expf) may decide differently; such a pixel can differ by one Gaussian's contribution;
//  * flip-affected Gaussians: the Gaussians whose own decision sits at a threshold somewhere. When it flips, that
//    Gaussian gains or loses the whole pixel term of its gradient; every other Gaussian of the pixel changes by a
//    term scaled by the flipped alpha (~1/255) or by the transmittance at saturation (~1e-4), inside the bar.
// The parity tests use the last set to bound which gradient entries may fall outside the bar.
#pragma once

#include <cmath>
#include <cstring>
#include <vector>

#include "omni_oracle.hpp"

namespace oracle {

struct Ambiguity {
    int64_t rect_gaussians = 0;   // lonlat Gaussians whose tile rect moves under +-ulps of atan2 / asin
    int64_t alpha_pixels = 0;     // pixels with an alpha decision within eps of 1/255
    int64_t sat_pixels = 0;       // pixels with a T(1 - alpha) decision within eps of 1e-4
    int64_t flip_gaussians = 0;   // Gaussians whose own blend decision sits at a threshold
    std::vector<uint8_t> flip;    // [P] 1 = flip-affected
};

inline float step_ulps(float v, int k)
{
    for (; k > 0; --k) v = std::nextafter(v, INFINITY);
    for (; k < 0; ++k) v = std::nextafter(v, -INFINITY);
    return v;
}

// getRect of a lonlat Gaussian for lon / lat moved by (dl, db) ulp (forward.cu:630-640 order of operations)
inline Rect lonlat_rect_perturbed(const State<float>& s, int idx, int dl, int db)
{
    const Args<float>& a = s.a;
    V3<float> p_orig = {a.means3D[3 * idx], a.means3D[3 * idx + 1], a.means3D[3 * idx + 2]};
    V4<float> pv;
    too_close(p_orig, a.viewmatrix, pv);
    const float inv_r = 1.0f / (pv.w + 0.0000001f);
    const float lon = step_ulps(Math<float>::atan2(pv.x, pv.z), dl);
    const float lat = step_ulps(Math<float>::asin(pv.y * inv_r), db);
    const V2<float> p_proj = {lon * R_1_PI<float>, lat * R_2_PI<float>};
    const V2<float> pix = {ndc2Pix(p_proj.x, a.width), ndc2Pix(p_proj.y, a.height)};
    return getRect(pix, s.radii[idx], s.gx, s.gy);
}

inline Ambiguity ambiguity_scan(const State<float>& s, double eps, int ulps)
{
    Ambiguity out;
    const Args<float>& a = s.a;
    const int P = a.P, W = a.width, H = a.height;
    out.flip.assign(P, 0);
    if (P == 0) return out;
    if (a.camera_type == 3) {
        int64_t n = 0;
#pragma omp parallel for schedule(dynamic, 4096) reduction(+ : n)
        for (int i = 0; i < P; ++i) {
            if (s.radii[i] <= 0) continue;
            const Rect base = lonlat_rect_perturbed(s, i, 0, 0);
            bool moved = false;
            for (int dl = -ulps; dl <= ulps && !moved; ++dl)
                for (int db = -ulps; db <= ulps && !moved; ++db) {
                    const Rect r = lonlat_rect_perturbed(s, i, dl, db);
                    moved = r.minx != base.minx || r.maxx != base.maxx || r.miny != base.miny || r.maxy != base.maxy;
                }
            n += moved ? 1 : 0;
        }
        out.rect_gaussians = n;
    }
    // blend decisions, walked exactly as render_tile (forward.cu:346-467), in double so the window is not itself
    // blurred by float rounding
    const uint32_t T = s.gx * s.gy;
    int64_t na = 0, ns = 0;
    std::vector<std::vector<uint32_t>> marked(T);
#pragma omp parallel for schedule(dynamic, 4) reduction(+ : na, ns)
    for (int t = 0; t < (int)T; ++t) {
        const uint32_t tx = t % s.gx, ty = t / s.gx;
        const uint32_t rx = s.ranges[2 * t], ry = s.ranges[2 * t + 1];
        for (int ly = 0; ly < BLOCK_Y; ++ly)
            for (int lx = 0; lx < BLOCK_X; ++lx) {
                const uint32_t px = tx * BLOCK_X + lx, py = ty * BLOCK_Y + ly;
                if (!(px < (uint32_t)W && py < (uint32_t)H)) continue;
                double Tr = 1.0;
                bool amb_a = false, amb_s = false;
                for (uint32_t k = rx; k < ry; ++k) {
                    const uint32_t id = s.point_list[k];
                    const double dx = (double)s.means2D[id].x - px, dy = (double)s.means2D[id].y - py;
                    const V4<float> co = s.conic_opacity[id];
                    const double power = -0.5 * (co.x * dx * dx + co.z * dy * dy) - co.y * dx * dy;
                    if (power > 0) continue;
                    const double alpha = std::fmin(0.99, co.w * std::exp(power));
                    if (std::fabs(alpha - 1.0 / 255.0) < eps / 255.0) {
                        amb_a = true;
                        marked[t].push_back(id);
                    }
                    if (alpha < 1.0 / 255.0) continue;
                    const double test_T = Tr * (1.0 - alpha);
                    if (std::fabs(test_T - 1e-4) < eps * 1e-4) {
                        amb_s = true;
                        marked[t].push_back(id);
                    }
                    if (test_T < 1e-4) break;
                    Tr = test_T;
                }
                na += amb_a ? 1 : 0;
                ns += amb_s ? 1 : 0;
            }
    }
    out.alpha_pixels = na;
    out.sat_pixels = ns;
    for (const auto& v : marked)
        for (uint32_t id : v) out.flip[id] = 1;
    for (int i = 0; i < P; ++i) out.flip_gaussians += out.flip[i];
    return out;
}

}  // namespace oracle

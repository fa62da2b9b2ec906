// ambiguity.hpp — how much of a result the missing reference run could still move (TEST INFRASTRUCTURE ONLY).
//
// The oracle is a restatement: no run of the CUDA reference pins it. Where the reference AS
// COMPILED could decide differently from the restatement, a parity claim rests on the restatement alone. Two
// effects separate them:
//   1. transcendental implementations: libdevice atan2f / asinf / expf vs the shared omni_math.h and v_exp_f32;
//   2. FMA contraction: nvcc's default --fmad=true (no -fmad flag in /root/reference/CMakeLists.txt:60-85) fuses
//      mul+add pairs the oracle (-ffp-contract=off) rounds twice: transformPoint4x3 / 4x4 (auxiliary.h:85-104),
//      too_close's rr (auxiliary.h:206), the cov2D products (forward.cu:86-228), det / mid / lambda
//      (forward.cu:660-674), the falloff power (forward.cu:434, backward.cu:774). oracle/contraction.py measures
//      the effect with two contracted builds of this oracle (GCC and LLVM fuse different multiplies).
// This file bounds both from the restatement's own forward, per decision, with explicit error windows, and
// returns the sets the parity tests excuse (tests/helpers.py: reference_allowance):
//
//  * rect-ambiguous Gaussians: getRect (auxiliary.h:56-66) changes when the pixel centre moves by k_pos ulp (or, for
//    lonlat, lon / lat by atan_ulps ulp), or when the radius ceil(3 sqrt(lambda_max)) (forward.cu:672) sits within
//    its rounding window of an integer and radius +-1 moves the rect. Such a Gaussian may own other tiles in the
//    reference: pixels of the tiles it gains or loses where it reaches alpha >= 1/255 are marked (PX_RECT);
//  * order-ambiguous pairs: same-tile neighbours of the sorted list whose depths (the sort key's low 32 bits,
//    rasterizer_impl.cu:133) differ by less than the sum of their depth rounding windows may sort the other way;
//    a pixel where two members of such a run both blend is marked (PX_ORDER);
//  * threshold pixels: a blend decision inside its window — alpha at 1/255 (forward.cu:436-437), power at 0
//    (:434-435), T (1 - alpha) at 1e-4 (:440-444). The window of power is the rounding bound of its evaluation from
//    rounded conic and centre: (kappa_g + k_eval eps) S + u G, S = a dx^2 / 2 + c dy^2 / 2 + |b dx dy|,
//    G = |a dx + b dy| + |b dx + c dy|, u = k_pos ulp of the centre, kappa_g = k_eval eps (|ac| + b^2) / |ac - b^2|
//    (the conic's condition); plus eps_exp for the exp implementations. T's window accumulates, over every blended
//    Gaussian in front, the relative change of its factor (1 - alpha): alpha (power window + eps_exp) / (1 - alpha);
//  * per flagged pixel, a bound on the colour change the flagged decisions can make (Allowance::bound, any channel):
//    each flipped term moves the pixel by at most its blend weight alpha T times the colour span 2 cmax (cmax = the
//    largest |colour| of the scene and background): alpha ~1/255 for an alpha flip, the opacity for a power-0 flip,
//    alpha_a alpha_b for an order swap, the transmittance ~1e-4 at saturation, the Gaussian's reach for a rect;
//  * flip Gaussians: the Gaussians owning any such decision. When one flips, that Gaussian gains or loses a whole
//    pixel term (or swaps its order with its pair) and its gradient may leave the bar;
//  * exposed Gaussians (G_EXPOSED): the ones blending behind such a decision (alpha, power 0, order, rect) and the
//    ones blending IN FRONT of it. Behind, their pixel term scales by the flipped alpha (~1/255 for a threshold
//    flip); in front, the colour accumulated behind them (accum_rec, backward.cu:745-760) gains or loses the flipped
//    term, which moves their dL/dalpha at that pixel by the same order. Small against the Gaussian's total, unless
//    its pixel terms cancel; the parity tests give them a wider bar (tests/helpers.py). The front half was found by
//    oracle/contraction.py's libm variant (glibc atan2f / asinf, round 6): a Gaussian in front of a neighbour's
//    alpha flip left the strict bar by 1.1x at A and B. A saturation flip only moves terms of transmittance ~1e-4
//    and exposes no one.
#pragma once

#include <cmath>
#include <cstring>
#include <vector>

#include "omni_oracle.hpp"

namespace oracle {

// pixel flags (Allowance::pixel)
enum : uint8_t { PX_ALPHA = 1, PX_SAT = 2, PX_ZERO = 4, PX_ORDER = 8, PX_RECT = 16 };
// Gaussian flags (Allowance::flip)
// G_RUN: member of an order-ambiguous run of some tile's list (its position may change; its result only where two
// members blend at one pixel, G_ORDER)
// G_RADIUS: the radius output (forward.cu:672) may differ by one in the reference (with or without a rect change)
enum : uint8_t { G_THRESHOLD = 1, G_ORDER = 2, G_RECT = 4, G_EXPOSED = 8, G_RUN = 16, G_RADIUS = 32 };

struct AllowanceParams {
    double eps_exp = 1e-5;  // relative window of alpha and T for the exp implementations
    int atan_ulps = 3;      // lonlat: ulps of atan2f / asinf (tests/test_math.py: <= 3 against glibc)
    double k_eval = 8.0;    // ulps (of the evaluated terms) for a contracted vs uncontracted expression
    double k_pos = 4.0;     // ulps of the pixel centre coordinates
    double k_depth = 8.0;   // ulps of the largest term of the view transform, for the depth key
};

// the nine per-pixel gradient terms of one (pixel, Gaussian) pair that backward.cu:671-843 accumulates:
// dL_dmean2D x, y; dL_dconic a, b, c; dL_dopacity; dL_dcolor r, g, b
constexpr int NTERM = 9;

struct Allowance {
    int64_t rect_gaussians = 0;    // flip & G_RECT
    int64_t radius_gaussians = 0;  // radius within its rounding window of an integer (a subset may move the rect)
    int64_t alpha_pixels = 0, sat_pixels = 0, zero_pixels = 0, order_pixels = 0, rect_pixels = 0;
    int64_t order_pairs = 0;       // adjacent same-tile instances whose order the reference may swap
    int64_t flip_gaussians = 0;    // Gaussians with any flag
    int64_t threshold_gaussians = 0, order_gaussians = 0, exposed_gaussians = 0;
    int64_t any_pixels = 0;
    std::vector<uint8_t> flip;     // [P] G_* flags
    std::vector<uint8_t> pixel;    // [H*W] PX_* flags
    std::vector<float> bound;      // [H*W] largest colour change the flagged decisions can make (per channel)
    // [P * NTERM], only with an upstream gradient: per Gaussian, the summed magnitude of the pixel terms its own
    // flagged decisions can add, remove or rescale (owner_term below) — what an owner's gradient may move by
    std::vector<float> term;
};

// |term| of Gaussian `id` at pixel (px, py) if it blends there with alpha `al` = o G behind transmittance T, a bound
// on each of the NTERM terms of backward.cu:745-770. The accumulated colour behind it (accum_rec) and the background
// term are bounded by the scene's colour span (cmax): |c - accum_rec| <= |c| + cmax.
inline void owner_term(const State<float>& s, uint32_t id, double px, double py, double al, double G, double T,
                       double T_final, const double* dLp, double cmax, double bg_dot, const float* features,
                       double scale, float* acc)
{
    const double dx = (double)s.means2D[id].x - px, dy = (double)s.means2D[id].y - py;
    const V4<float> co = s.conic_opacity[id];
    double dLda = 0.0;
    for (int ch = 0; ch < 3; ++ch) dLda += (std::fabs((double)features[3 * id + ch]) + cmax) * dLp[ch];
    dLda = T * dLda + T_final / std::fmax(1.0 - al, 1e-2) * bg_dot;
    const double dG = (double)co.w * dLda;
    const double W2 = 0.5 * s.a.width, H2 = 0.5 * s.a.height;
    acc[0] += (float)(scale * dG * G * std::fabs((double)co.x * dx + (double)co.y * dy) * W2);
    acc[1] += (float)(scale * dG * G * std::fabs((double)co.z * dy + (double)co.y * dx) * H2);
    acc[2] += (float)(scale * 0.5 * G * dx * dx * dG);
    acc[3] += (float)(scale * 0.5 * G * std::fabs(dx * dy) * dG);
    acc[4] += (float)(scale * 0.5 * G * dy * dy * dG);
    acc[5] += (float)(scale * G * dLda);
    for (int ch = 0; ch < 3; ++ch) acc[6 + ch] += (float)(scale * al * T * dLp[ch]);
}

constexpr double EPS32 = 5.9604644775390625e-08;  // 2^-24

inline float step_ulps(float v, int k)
{
    for (; k > 0; --k) v = std::nextafter(v, INFINITY);
    for (; k < 0; ++k) v = std::nextafter(v, -INFINITY);
    return v;
}
inline double ulp_of(float v) { return (double)std::nextafter(std::fabs(v), INFINITY) - std::fabs(v); }

// getRect of a lonlat Gaussian for lon / lat moved by (dl, db) ulp (forward.cu:630-640 order of operations)
inline Rect lonlat_rect_perturbed(const State<float>& s, int idx, int dl, int db, int radius)
{
    const Args<float>& a = s.a;
    V3<float> p_orig = {a.means3D[3 * idx], a.means3D[3 * idx + 1], a.means3D[3 * idx + 2]};
    V4<float> pv = {0.f, 0.f, 0.f, 0.f};
    too_close(p_orig, a.viewmatrix, pv);
    const float inv_r = 1.0f / (pv.w + 0.0000001f);
    const float lon = step_ulps(Math<float>::atan2(pv.x, pv.z), dl);
    const float lat = step_ulps(Math<float>::asin(pv.y * inv_r), db);
    const V2<float> p_proj = {lon * R_1_PI<float>, lat * R_2_PI<float>};
    const V2<float> pix = {ndc2Pix(p_proj.x, a.width), ndc2Pix(p_proj.y, a.height)};
    return getRect(pix, radius, s.gx, s.gy);
}

inline bool same_rect(const Rect& p, const Rect& q)
{
    return p.minx == q.minx && p.maxx == q.maxx && p.miny == q.miny && p.maxy == q.maxy;
}

// rounding window of the depth key of a visible Gaussian: the view transform's components carry an absolute error
// of ~k_depth eps x their largest term (auxiliary.h:85-93); lonlat depth = |p_view| (auxiliary.h:206-213)
inline double depth_window(const State<float>& s, int idx, const AllowanceParams& prm)
{
    const Args<float>& a = s.a;
    const float* m = a.viewmatrix;
    const double p[3] = {a.means3D[3 * idx], a.means3D[3 * idx + 1], a.means3D[3 * idx + 2]};
    double tmax = 0.0;
    for (int i = 0; i < 3; ++i) {
        if (a.camera_type != 3 && i != 2) continue;  // pinhole depth = p_view.z
        const double t = std::fabs(m[i] * p[0]) + std::fabs(m[4 + i] * p[1]) + std::fabs(m[8 + i] * p[2]) +
                         std::fabs((double)m[12 + i]);
        tmax = std::fmax(tmax, t);
    }
    return prm.k_depth * EPS32 * tmax + 2.0 * EPS32 * std::fabs((double)s.depths[idx]);
}

// x = 3 sqrt(lambda_max) (forward.cu:663-672) and its rounding window, from the conic (the inverse of cov2D)
inline void radius_window(const V4<float>& co, const AllowanceParams& prm, double& x, double& dx)
{
    const double dc = (double)co.x * co.z - (double)co.y * co.y;
    const double a = co.z / dc, b = -co.y / dc, c = co.x / dc;  // cov2D
    const double det = a * c - b * b, mid = 0.5 * (a + c);
    const double arg = mid * mid - det;
    const double sq = std::sqrt(std::fmax(0.1, arg));
    const double lam = mid + sq;
    x = 3.0 * std::sqrt(std::fmax(lam, mid - sq));
    double dlam = prm.k_eval * EPS32 * mid;
    if (arg > 0.1) dlam += prm.k_eval * EPS32 * (mid * mid + std::fabs(det)) / (2.0 * sq);
    dx = 3.0 * dlam / (2.0 * std::sqrt(std::fmax(lam, 1e-30))) + prm.k_eval * EPS32 * x;
}

// dL_dpix ([3, H, W], may be NULL): also fill Allowance::term, the owners' gradient bound in pixel-term space
inline Allowance allowance_scan(const State<float>& s, const AllowanceParams& prm, const float* dL_dpix = nullptr)
{
    Allowance out;
    const Args<float>& a = s.a;
    const int P = a.P, W = a.width, H = a.height;
    out.flip.assign(P, 0);
    out.pixel.assign((size_t)W * H, 0);
    out.bound.assign((size_t)W * H, 0.f);
    if (P == 0) return out;
    const uint32_t T = s.gx * s.gy;
    const float* features = a.colors_precomp != nullptr ? a.colors_precomp : s.rgb.data();
    double cmax = 0.0;
    for (int ch = 0; ch < 3; ++ch) cmax = std::fmax(cmax, std::fabs((double)a.background[ch]));
    for (int i = 0; i < P; ++i)
        if (s.radii[i] > 0)
            for (int ch = 0; ch < 3; ++ch) cmax = std::fmax(cmax, std::fabs((double)features[3 * i + ch]));
    const double span = 2.0 * cmax;

    // per Gaussian: depth window, conic condition, centre window; rect / radius ambiguity
    std::vector<double> dwin(P, 0.0), kappa(P, 0.0), upos(P, 0.0);
    std::vector<Rect> alt_rect(P);  // the union of the rects the reference could use (rect-ambiguous ones)
    int64_t n_rect = 0, n_rad = 0;
#pragma omp parallel for schedule(dynamic, 4096) reduction(+ : n_rect, n_rad)
    for (int i = 0; i < P; ++i) {
        if (s.radii[i] <= 0) continue;
        dwin[i] = depth_window(s, i, prm);
        const V4<float> co = s.conic_opacity[i];
        const double ac = (double)co.x * co.z, bb = (double)co.y * co.y;
        kappa[i] = prm.k_eval * EPS32 * (std::fabs(ac) + bb) / std::fmax(std::fabs(ac - bb), 1e-300);
        const V2<float> m2 = s.means2D[i];
        upos[i] = prm.k_pos * std::fmax(ulp_of(m2.x), ulp_of(m2.y));
        // radius window
        double x, dx;
        radius_window(co, prm, x, dx);
        const int r0 = s.radii[i];
        int rlo = r0, rhi = r0;
        if ((int)std::ceil(x - dx) != r0 || (int)std::ceil(x + dx) != r0) {
            n_rad += 1;
            out.flip[i] |= G_RADIUS;
            rlo = std::min(r0, (int)std::ceil(x - dx));
            rhi = std::max(r0, (int)std::ceil(x + dx));
        }
        const Rect base = getRect(m2, r0, s.gx, s.gy);
        Rect un = base;
        bool moved = false;  // some candidate rect differs (grown or shrunk)
        auto widen = [&](const Rect& r) {
            moved = moved || !same_rect(r, base);
            un.minx = std::min(un.minx, r.minx); un.miny = std::min(un.miny, r.miny);
            un.maxx = std::max(un.maxx, r.maxx); un.maxy = std::max(un.maxy, r.maxy);
        };
        for (int rad = rlo; rad <= rhi; ++rad)
            for (int sx = -1; sx <= 1; ++sx)
                for (int sy = -1; sy <= 1; ++sy) {
                    const V2<float> p = {(float)(m2.x + sx * upos[i]), (float)(m2.y + sy * upos[i])};
                    widen(getRect(p, rad, s.gx, s.gy));
                }
        if (a.camera_type == 3)
            for (int dl = -prm.atan_ulps; dl <= prm.atan_ulps; ++dl)
                for (int db = -prm.atan_ulps; db <= prm.atan_ulps; ++db)
                    for (int rad = rlo; rad <= rhi; ++rad) widen(lonlat_rect_perturbed(s, i, dl, db, rad));
        alt_rect[i] = un;
        if (moved) {
            out.flip[i] = (uint8_t)(out.flip[i] | G_RECT);
            n_rect += 1;
        }
    }
    out.rect_gaussians = n_rect;
    out.radius_gaussians = n_rad;

    // per tile: order runs of the sorted list (consecutive instances whose depths are within the summed windows)
    // and the rect-ambiguous Gaussians that may join the tile; then every pixel is walked as render_tile
    // (forward.cu:346-467) in double, decisions tested against their windows
    std::vector<std::vector<int>> gx_extra(T);  // rect-ambiguous Gaussians that may reach tile t but are not listed
    for (int i = 0; i < P; ++i) {
        if (!(out.flip[i] & G_RECT)) continue;
        const Rect base = getRect(s.means2D[i], s.radii[i], s.gx, s.gy), un = alt_rect[i];
        for (uint32_t ty = un.miny; ty < un.maxy; ++ty)
            for (uint32_t tx = un.minx; tx < un.maxx; ++tx) {
                const bool in_base = tx >= base.minx && tx < base.maxx && ty >= base.miny && ty < base.maxy;
                if (!in_base) gx_extra[ty * s.gx + tx].push_back(i);
            }
    }
    int64_t na = 0, ns = 0, nz = 0, no = 0, nr = 0, npairs = 0, nany = 0;
    std::vector<std::vector<std::pair<uint32_t, uint8_t>>> marked(T);
    std::vector<std::vector<uint32_t>> term_id(dL_dpix ? T : 0);  // per tile: flagged (pixel, Gaussian) terms
    std::vector<std::vector<float>> term_val(dL_dpix ? T : 0);
#pragma omp parallel for schedule(dynamic, 4) reduction(+ : na, ns, nz, no, nr, npairs, nany)
    for (int t = 0; t < (int)T; ++t) {
        const uint32_t tx = t % s.gx, ty = t / s.gx;
        const uint32_t rx = s.ranges[2 * t], ry = s.ranges[2 * t + 1];
        std::vector<uint32_t> front_buf;
        const uint32_t n = ry - rx;
        std::vector<uint32_t> run(n);  // run id of each position: consecutive positions in one run may swap
        uint32_t rid = 0;
        for (uint32_t k = 0; k < n; ++k) {
            if (k > 0) {
                const uint32_t i0 = s.point_list[rx + k - 1], i1 = s.point_list[rx + k];
                const double gap = std::fabs((double)s.depths[i1] - (double)s.depths[i0]);
                if (gap <= dwin[i0] + dwin[i1]) {
                    npairs += 1;
                    marked[t].push_back({i0, G_RUN});
                    marked[t].push_back({i1, G_RUN});
                } else {
                    rid += 1;
                }
            }
            run[k] = rid;
        }
        for (int ly = 0; ly < BLOCK_Y; ++ly)
            for (int lx = 0; lx < BLOCK_X; ++lx) {
                const uint32_t px = tx * BLOCK_X + lx, py = ty * BLOCK_Y + ly;
                if (!(px < (uint32_t)W && py < (uint32_t)H)) continue;
                uint8_t pf = 0;
                double Tr = 1.0, errT = 0.0, bnd = 0.0, last_alpha = 0.0, T_before_last = 1.0;
                uint32_t last_run = ~0u, last_run_id = 0;
                bool behind = false;  // a decision in front of this position is ambiguous (alpha, power 0, order, rect)
                double last_G = 0.0;
                // the Gaussians blended so far at this pixel: a flagged decision behind them exposes them too
                std::vector<uint32_t>& front = front_buf;
                front.clear();
                size_t front_marked = 0;
                auto expose_front = [&](uint32_t except) {
                    for (; front_marked < front.size(); ++front_marked)
                        if (front[front_marked] != except) marked[t].push_back({front[front_marked], G_EXPOSED});
                };
                double dLp[3] = {0, 0, 0}, bg_dot = 0.0, T_fin = 0.0;
                if (dL_dpix) {
                    const size_t pid = (size_t)py * W + px;
                    for (int ch = 0; ch < 3; ++ch) {
                        dLp[ch] = std::fabs((double)dL_dpix[(size_t)ch * H * W + pid]);
                        bg_dot += (double)a.background[ch] * dL_dpix[(size_t)ch * H * W + pid];
                    }
                    bg_dot = std::fabs(bg_dot);
                    T_fin = s.final_T[pid];
                }
                // the pixel term of `id` may appear, vanish or be rescaled by `scale` in the reference
                auto add_term = [&](uint32_t id, double al, double G, double Tt, double scale) {
                    if (!dL_dpix) return;
                    term_id[t].push_back(id);
                    const size_t o = term_val[t].size();
                    term_val[t].resize(o + NTERM, 0.f);
                    owner_term(s, id, px, py, al, G, Tt, T_fin, dLp, cmax, bg_dot, features, scale, &term_val[t][o]);
                };
                auto eval = [&](uint32_t id, double& power, double& dp) {
                    const double dx = (double)s.means2D[id].x - px, dy = (double)s.means2D[id].y - py;
                    const V4<float> co = s.conic_opacity[id];
                    power = -0.5 * (co.x * dx * dx + co.z * dy * dy) - co.y * dx * dy;
                    const double S = 0.5 * std::fabs(co.x) * dx * dx + 0.5 * std::fabs(co.z) * dy * dy +
                                     std::fabs(co.y * dx * dy);
                    const double G = std::fabs(co.x * dx + co.y * dy) + std::fabs(co.y * dx + co.z * dy);
                    dp = (kappa[id] + prm.k_eval * EPS32) * S + upos[id] * G;
                };
                // a rect-ambiguous Gaussian that may join the tile (below) may blend at any depth: T's window starts
                // with the factor it can bring
                for (int id : gx_extra[t]) {
                    double power, dp;
                    eval((uint32_t)id, power, dp);
                    const float o = s.conic_opacity[id].w;
                    if (power - dp <= 0.0 && power + dp >= -std::log(255.0 * o) - prm.eps_exp) {
                        const double ax = std::fmin(0.99, o * std::exp(std::fmin(0.0, power + dp)));
                        errT += ax / std::fmax(1.0 - ax, 1e-2);
                    }
                }
                for (uint32_t k = 0; k < n; ++k) {
                    const uint32_t id = s.point_list[rx + k];
                    double power, dp;
                    eval(id, power, dp);
                    const V4<float> co = s.conic_opacity[id];
                    if (std::fabs(power) <= dp && power + dp > 0.0) {  // power > 0 skip (forward.cu:434-435)
                        pf |= PX_ZERO;
                        marked[t].push_back({id, G_THRESHOLD});
                        expose_front(id);
                        bnd += span * Tr * std::fmin(0.99, (double)co.w);
                        const double Gz = std::exp(std::fmin(power, 0.0));
                        const double az = std::fmin(0.99, co.w * Gz);
                        add_term(id, az, Gz, Tr, 1.0);
                        errT += az / std::fmax(1.0 - az, 1e-2);  // T behind it moves by that factor either way
                    }
                    if (power > 0) continue;
                    const double thr = -std::log(255.0 * co.w);  // alpha = o exp(power) = 1/255
                    if (std::fabs(power - thr) <= dp + prm.eps_exp) {
                        pf |= PX_ALPHA;
                        marked[t].push_back({id, G_THRESHOLD});
                        expose_front(id);
                        bnd += span * Tr * (1.0 / 255.0) * std::exp(dp + prm.eps_exp);
                        // blended or not, T behind it moves by the flipped factor (1 - alpha): a later saturation test
                        // (T (1 - alpha) at 1e-4) within that much of its threshold may flip too (found by
                        // oracle/contraction.py's libm variant at E: an alpha flip 170 positions in front of one)
                        const double af = (1.0 / 255.0) * std::exp(dp + prm.eps_exp);
                        errT += af / (1.0 - af);
                        const double Ga = std::exp(std::fmin(power + dp + prm.eps_exp, 0.0));
                        add_term(id, std::fmin(0.99, co.w * Ga), Ga, Tr, 1.0);
                    }
                    const double alpha = std::fmin(0.99, co.w * std::exp(power));
                    if (alpha < 1.0 / 255.0) {
                        behind = behind || (pf & (PX_ALPHA | PX_ZERO));
                        continue;
                    }
                    if (behind) marked[t].push_back({id, G_EXPOSED});
                    if (out.flip[id] & G_RECT) {  // a rect-ambiguous Gaussian may leave a tile on its rect's edge
                        const Rect b = getRect(s.means2D[id], s.radii[id], s.gx, s.gy);
                        if (tx == b.minx || tx + 1 == b.maxx || ty == b.miny || ty + 1 == b.maxy) {
                            pf |= PX_RECT;
                            bnd += span * Tr * alpha;
                            add_term(id, alpha, std::exp(power), Tr, 1.0);
                            expose_front(id);
                            errT += alpha / std::fmax(1.0 - alpha, 1e-2);
                        }
                    }
                    behind = behind || (pf & (PX_ALPHA | PX_ZERO | PX_ORDER | PX_RECT));
                    // order: a second blended member of the same run
                    const bool pair_prev = last_run == run[k];
                    if (pair_prev) {
                        pf |= PX_ORDER;
                        marked[t].push_back({id, G_ORDER});
                        marked[t].push_back({last_run_id, G_ORDER});
                        expose_front(last_run_id);
                        // swapping a, b moves (alpha_a alpha_b T_a)(c_a - c_b); T after both is unchanged
                        bnd += span * (Tr / std::fmax(1.0 - last_alpha, 1e-2)) * last_alpha * alpha;
                        // swapped, b's transmittance grows by 1 / (1 - alpha_a), a's shrinks by (1 - alpha_b), and
                        // both accumulated colours change: each term moves by at most itself times that factor
                        add_term(id, alpha, std::exp(power), Tr, 1.0 + last_alpha / std::fmax(1.0 - last_alpha, 1e-2));
                        add_term(last_run_id, last_alpha, last_G, T_before_last, 1.0 + alpha);
                    }
                    front.push_back(id);
                    last_run = run[k];
                    last_run_id = id;
                    last_alpha = alpha;
                    last_G = std::exp(power);
                    const double test_T = Tr * (1.0 - alpha);
                    // relative error of T (1 - alpha): each blended factor (1 - alpha_j) moves by alpha_j dalpha_j /
                    // (1 - alpha_j) relative (dalpha = alpha dp, plus the exp implementations' eps_exp); the 1 / (1 -
                    // alpha) factor matters for opaque Gaussians (found by oracle/contraction.py's libm variant at E:
                    // a pixel 303 Gaussians deep whose saturation test flipped outside the window without it)
                    const double errk = errT + alpha * (dp + prm.eps_exp) / std::fmax(1.0 - alpha, 1e-2);
                    if (std::fabs(test_T - 1e-4) <= (prm.eps_exp + errk) * 1e-4) {
                        pf |= PX_SAT;
                        marked[t].push_back({id, G_THRESHOLD});
                        bnd += span * Tr;  // this term and everything behind carry transmittance <= Tr
                        add_term(id, alpha, std::exp(power), Tr, 1.0);
                    }
                    if (test_T < 1e-4) {
                        // the run's previous member blended and this one saturates: swapped, the other one may
                        // end the pixel, which moves T and the colour by up to the transmittance before the pair
                        if (pair_prev) {
                            pf |= PX_ORDER;
                            bnd += span * T_before_last;
                        }
                        break;
                    }
                    T_before_last = Tr;
                    Tr = test_T;
                    errT = errk;
                }
                // a rect-ambiguous Gaussian that may join this tile in the reference and reaches the pixel
                for (int id : gx_extra[t]) {
                    double power, dp;
                    eval((uint32_t)id, power, dp);
                    const float o = s.conic_opacity[id].w;
                    if (power - dp <= 0.0 && power + dp >= -std::log(255.0 * o) - prm.eps_exp) {
                        pf |= PX_RECT;
                        expose_front(~0u);  // it may blend at any depth: every blended Gaussian may lie in front
                        bnd += span * std::fmin(0.99, o * std::exp(std::fmin(0.0, power + dp)));
                        // it may blend at any depth position: transmittance <= 1
                        const double Gr = std::exp(std::fmin(0.0, power + dp));
                        add_term((uint32_t)id, std::fmin(0.99, o * Gr), Gr, 1.0, 1.0);
                    }
                }
                na += (pf & PX_ALPHA) ? 1 : 0;
                ns += (pf & PX_SAT) ? 1 : 0;
                nz += (pf & PX_ZERO) ? 1 : 0;
                no += (pf & PX_ORDER) ? 1 : 0;
                nr += (pf & PX_RECT) ? 1 : 0;
                nany += pf ? 1 : 0;
                out.pixel[(size_t)py * W + px] = pf;
                out.bound[(size_t)py * W + px] = (float)bnd;
            }
    }
    out.alpha_pixels = na;
    out.sat_pixels = ns;
    out.zero_pixels = nz;
    out.order_pixels = no;
    out.rect_pixels = nr;
    out.order_pairs = npairs;
    out.any_pixels = nany;
    for (const auto& v : marked)
        for (const auto& e : v) out.flip[e.first] |= e.second;
    if (dL_dpix) {
        out.term.assign((size_t)P * NTERM, 0.f);
        for (uint32_t t = 0; t < T; ++t)
            for (size_t k = 0; k < term_id[t].size(); ++k)
                for (int j = 0; j < NTERM; ++j) out.term[(size_t)term_id[t][k] * NTERM + j] += term_val[t][k * NTERM + j];
    }
    for (int i = 0; i < P; ++i) {
        out.flip_gaussians += (out.flip[i] & (G_THRESHOLD | G_ORDER | G_RECT)) != 0;
        out.threshold_gaussians += (out.flip[i] & G_THRESHOLD) != 0;
        out.order_gaussians += (out.flip[i] & G_ORDER) != 0;
        out.exposed_gaussians += (out.flip[i] & (G_THRESHOLD | G_ORDER | G_RECT | G_EXPOSED)) == G_EXPOSED;
    }
    return out;
}

// The owners' gradient bound in the outputs' own space. The preprocess backward (backward.cu:297-485 lonlat /
// :156-292 pinhole, :613-669 / :557-608, SH :30-151, cov3D :489-552) is linear in the nine pixel-term sums of a
// Gaussian at the forward's state, so |change of an output| <= sum_c |J[output][c]| term[c], J taken column by
// column by running that backward on unit inputs. For each of the n Gaussians ids[i], out[i * K ...] holds, in
// this order: dmean2D (3), dcolor (3), dopacity (1), dmean3D (3), dcov3D (6), dsh (M * 3), dscale (3), drot (4);
// K = 23 + 3 M. `term` is Allowance::term ([P * NTERM]).
inline int owner_grad_bound(const State<float>& s, const float* term, const int32_t* ids, int n, float* out)
{
    const int P = s.a.P, M = s.a.M;
    const int K = 23 + 3 * M;
    Grads<float> g;
    g.zero(P, M);
    const float* cov3D_ptr = s.a.cov3D_precomp != nullptr ? s.a.cov3D_precomp : s.cov3D.data();
    const float focal_y = (float)s.a.height / (2.0f * s.a.tan_fovy);
    const float focal_x = (float)s.a.width / (2.0f * s.a.tan_fovx);
    for (int i = 0; i < n; ++i) {
        const int idx = ids[i];
        float* o = out + (size_t)i * K;
        for (int k = 0; k < K; ++k) o[k] = 0.f;
        if (idx < 0 || idx >= P) return -1;
        const float* tm = term + (size_t)idx * NTERM;
        o[0] = tm[0]; o[1] = tm[1];
        o[3] = tm[6]; o[4] = tm[7]; o[5] = tm[8];
        o[6] = tm[5];
        if (!(s.radii[idx] > 0)) continue;
        for (int c = 0; c < NTERM; ++c) {
            if (tm[c] == 0.f) continue;
            float in[NTERM] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
            in[c] = 1.f;
            g.dmean2D[3 * idx] = in[0]; g.dmean2D[3 * idx + 1] = in[1]; g.dmean2D[3 * idx + 2] = 0.f;
            g.dconic[4 * idx] = in[2]; g.dconic[4 * idx + 1] = in[3]; g.dconic[4 * idx + 3] = in[4];
            g.dopacity[idx] = in[5];
            g.dcolor[3 * idx] = in[6]; g.dcolor[3 * idx + 1] = in[7]; g.dcolor[3 * idx + 2] = in[8];
            V3<float> dpx_dt = {0, 0, 0}, dpy_dt = {0, 0, 0};
            if (s.a.camera_type == 3) computeCov2DLonLat_backward(s, idx, cov3D_ptr, g, dpx_dt, dpy_dt);
            else computeCov2D_backward(s, idx, cov3D_ptr, focal_x, focal_y, g);
            preprocess_backward_one(s, idx, dpx_dt, dpy_dt, g);
            const double w = tm[c];
            float* q = o + 7;
            for (int k = 0; k < 3; ++k) *q++ += (float)(w * std::fabs((double)g.dmean3D[3 * idx + k]));
            for (int k = 0; k < 6; ++k) *q++ += (float)(w * std::fabs((double)g.dcov3D[6 * idx + k]));
            for (int k = 0; k < 3 * M; ++k) *q++ += (float)(w * std::fabs((double)g.dsh[(size_t)idx * M * 3 + k]));
            for (int k = 0; k < 3; ++k) *q++ += (float)(w * std::fabs((double)g.dscale[3 * idx + k]));
            for (int k = 0; k < 4; ++k) *q++ += (float)(w * std::fabs((double)g.drot[4 * idx + k]));
        }
    }
    return K;
}

}  // namespace oracle

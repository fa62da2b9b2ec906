// oracle_capi.cpp — ctypes surface of the CPU oracle (TEST INFRASTRUCTURE ONLY; see omni_oracle.hpp).
// Loaded by tests/ (parity checker, fixture generator) and by bench.py's cpu_baseline leg. Never by the product.
#include <cstdio>
#include <cstring>
#include <string>

#include "ambiguity.hpp"
#include "omni_oracle.hpp"

namespace {

struct Handle {
    bool dbl = false;
    oracle::State<float> sf;
    oracle::State<double> sd;
    oracle::Grads<float> gf;
    oracle::Grads<double> gd;
    std::vector<uint64_t> tmp_u64;
};

template <typename R>
int run_forward(oracle::State<R>& s, int P, int D, int M, const R* bg, int W, int H, const R* means3D, const R* shs,
                const R* colors_precomp, const R* opacities, const R* scales, R scale_modifier, const R* rotations,
                const R* cov3D_precomp, const R* viewmatrix, const R* projmatrix, const R* campos, R tan_fovx, R tan_fovy,
                int prefiltered, int camera_type, int render_depth, char* err, int errlen)
{
    oracle::Args<R> a;
    a.P = P; a.D = D; a.M = M; a.background = bg; a.width = W; a.height = H;
    a.means3D = means3D; a.shs = shs; a.colors_precomp = colors_precomp; a.opacities = opacities;
    a.scales = scales; a.scale_modifier = scale_modifier; a.rotations = rotations; a.cov3D_precomp = cov3D_precomp;
    a.viewmatrix = viewmatrix; a.projmatrix = projmatrix; a.campos = campos; a.tan_fovx = tan_fovx; a.tan_fovy = tan_fovy;
    a.prefiltered = prefiltered != 0; a.camera_type = camera_type; a.render_depth = render_depth != 0;
    try {
        return oracle::forward(s, a);
    } catch (const std::exception& e) {
        if (err && errlen > 0) std::snprintf(err, errlen, "%s", e.what());
        return -1;
    }
}

template <typename R> const void* field(Handle* h, oracle::State<R>& s, oracle::Grads<R>& g, const std::string& n, int64_t& count, int& esize)
{
    esize = sizeof(R);
#define F(name, vec, es)                \
    if (n == name) {                    \
        count = (int64_t)(vec).size();  \
        esize = es;                     \
        return (vec).data();            \
    }
    F("out_color", s.out_color, sizeof(R));
    F("depths", s.depths, sizeof(R));
    F("clamped", s.clamped, 1);
    F("radii", s.radii, 4);
    F("cov3D", s.cov3D, sizeof(R));
    F("rgb", s.rgb, sizeof(R));
    F("tiles_touched", s.tiles_touched, 4);
    F("point_offsets", s.point_offsets, 4);
    F("point_list", s.point_list, 4);
    F("keys", s.keys, 8);
    F("final_T", s.final_T, sizeof(R));
    F("n_contrib", s.n_contrib, 4);
    F("ranges", s.ranges, 4);
    F("dmean2D", g.dmean2D, sizeof(R));
    F("dconic", g.dconic, sizeof(R));
    F("dopacity", g.dopacity, sizeof(R));
    F("dcolor", g.dcolor, sizeof(R));
    F("dmean3D", g.dmean3D, sizeof(R));
    F("dcov3D", g.dcov3D, sizeof(R));
    F("dsh", g.dsh, sizeof(R));
    F("dscale", g.dscale, sizeof(R));
    F("drot", g.drot, sizeof(R));
#undef F
    if (n == "means2D") { count = 2 * (int64_t)s.means2D.size(); return s.means2D.data(); }
    if (n == "conic_opacity") { count = 4 * (int64_t)s.conic_opacity.size(); return s.conic_opacity.data(); }
    (void)h;
    count = -1;
    return nullptr;
}

}  // namespace

extern "C" {

int oracle_allowance_terms(void* hv, const double* prm, uint8_t* flip_out, uint8_t* pixel_out, float* bound_out,
                           int64_t* counts, const float* dL_dpix, float* term_out);

void* oracle_new(int dbl)
{
    Handle* h = new Handle();
    h->dbl = dbl != 0;
    return h;
}

void oracle_free(void* h) { delete static_cast<Handle*>(h); }

int oracle_forward_f32(void* hv, int P, int D, int M, const float* bg, int W, int H, const float* means3D, const float* shs,
                       const float* colors_precomp, const float* opacities, const float* scales, float scale_modifier,
                       const float* rotations, const float* cov3D_precomp, const float* viewmatrix, const float* projmatrix,
                       const float* campos, float tan_fovx, float tan_fovy, int prefiltered, int camera_type, int render_depth,
                       char* err, int errlen)
{
    Handle* h = static_cast<Handle*>(hv);
    return run_forward<float>(h->sf, P, D, M, bg, W, H, means3D, shs, colors_precomp, opacities, scales, scale_modifier,
                              rotations, cov3D_precomp, viewmatrix, projmatrix, campos, tan_fovx, tan_fovy, prefiltered,
                              camera_type, render_depth, err, errlen);
}

int oracle_forward_f64(void* hv, int P, int D, int M, const double* bg, int W, int H, const double* means3D, const double* shs,
                       const double* colors_precomp, const double* opacities, const double* scales, double scale_modifier,
                       const double* rotations, const double* cov3D_precomp, const double* viewmatrix, const double* projmatrix,
                       const double* campos, double tan_fovx, double tan_fovy, int prefiltered, int camera_type, int render_depth,
                       char* err, int errlen)
{
    Handle* h = static_cast<Handle*>(hv);
    return run_forward<double>(h->sd, P, D, M, bg, W, H, means3D, shs, colors_precomp, opacities, scales, scale_modifier,
                               rotations, cov3D_precomp, viewmatrix, projmatrix, campos, tan_fovx, tan_fovy, prefiltered,
                               camera_type, render_depth, err, errlen);
}

int oracle_backward(void* hv, const void* dL_dpix, int nthreads)
{
    Handle* h = static_cast<Handle*>(hv);
    if (h->dbl) oracle::backward(h->sd, static_cast<const double*>(dL_dpix), h->gd, nthreads);
    else oracle::backward(h->sf, static_cast<const float*>(dL_dpix), h->gf, nthreads);
    return 0;
}

// element count of a named array (and its element size in bytes), -1 if unknown
int64_t oracle_size(void* hv, const char* name, int* esize)
{
    Handle* h = static_cast<Handle*>(hv);
    int64_t c = -1;
    int es = 0;
    if (h->dbl) field(h, h->sd, h->gd, name, c, es);
    else field(h, h->sf, h->gf, name, c, es);
    if (esize) *esize = es;
    return c;
}

int oracle_get(void* hv, const char* name, void* dst)
{
    Handle* h = static_cast<Handle*>(hv);
    int64_t c = -1;
    int es = 0;
    const void* p = h->dbl ? field(h, h->sd, h->gd, name, c, es) : field(h, h->sf, h->gf, name, c, es);
    if (c < 0) return -1;
    if (c > 0) std::memcpy(dst, p, (size_t)c * es);
    return 0;
}

int oracle_num_rendered(void* hv)
{
    Handle* h = static_cast<Handle*>(hv);
    return h->dbl ? h->sd.num_rendered : h->sf.num_rendered;
}

void oracle_set_threads(int n)
{
#ifdef _OPENMP
    omp_set_num_threads(n);
#else
    (void)n;
#endif
}

int oracle_max_threads(void)
{
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

uint32_t oracle_higher_msb(uint32_t n) { return oracle::getHigherMsb(n); }
float oracle_atan2f(float y, float x) { return omni::atan2f_(y, x); }
float oracle_asinf(float x) { return omni::asinf_(x); }

void oracle_mark_visible(int P, const float* means3D, const float* viewmatrix, const float* projmatrix, int camera_type, uint8_t* present)
{
    oracle::markVisible<float>(P, means3D, viewmatrix, projmatrix, camera_type, present);
}

// ambiguity.hpp (allowance_scan) on the last float forward. prm: eps_exp, atan_ulps, k_eval, k_pos, k_depth.
// counts (13): rect_gaussians, radius_gaussians, alpha_pixels, sat_pixels, zero_pixels, order_pixels, rect_pixels,
// order_pairs, flip_gaussians, threshold_gaussians, order_gaussians, any_pixels, exposed_gaussians. flip_out [P] G_* flags,
// pixel_out [H*W] PX_* flags, bound_out [H*W] the largest colour change of those decisions (any may be NULL).
int oracle_allowance(void* hv, const double* prm, uint8_t* flip_out, uint8_t* pixel_out, float* bound_out,
                     int64_t* counts)
{
    return oracle_allowance_terms(hv, prm, flip_out, pixel_out, bound_out, counts, nullptr, nullptr);
}

// oracle_allowance, plus (dL_dpix [3, H, W] given) the owners' pixel-term bound Allowance::term into term_out
// [P * 9]; both NULL skips it
int oracle_allowance_terms(void* hv, const double* prm, uint8_t* flip_out, uint8_t* pixel_out, float* bound_out,
                           int64_t* counts, const float* dL_dpix, float* term_out)
{
    Handle* h = static_cast<Handle*>(hv);
    if (h->dbl) return -1;
    oracle::AllowanceParams p;
    p.eps_exp = prm[0];
    p.atan_ulps = (int)prm[1];
    p.k_eval = prm[2];
    p.k_pos = prm[3];
    p.k_depth = prm[4];
    const oracle::Allowance a = oracle::allowance_scan(h->sf, p, term_out ? dL_dpix : nullptr);
    const int64_t c[13] = {a.rect_gaussians, a.radius_gaussians, a.alpha_pixels, a.sat_pixels, a.zero_pixels,
                           a.order_pixels, a.rect_pixels, a.order_pairs, a.flip_gaussians, a.threshold_gaussians,
                           a.order_gaussians, a.any_pixels, a.exposed_gaussians};
    std::memcpy(counts, c, sizeof(c));
    if (flip_out && !a.flip.empty()) std::memcpy(flip_out, a.flip.data(), a.flip.size());
    if (pixel_out && !a.pixel.empty()) std::memcpy(pixel_out, a.pixel.data(), a.pixel.size());
    if (bound_out && !a.bound.empty()) std::memcpy(bound_out, a.bound.data(), a.bound.size() * sizeof(float));
    if (term_out && !a.term.empty()) std::memcpy(term_out, a.term.data(), a.term.size() * sizeof(float));
    return 0;
}

// ambiguity.hpp owner_grad_bound on the last float forward: per Gaussian ids[i], the K = 23 + 3 M output-space
// bounds. Returns K, or -1.
int oracle_owner_grad_bound(void* hv, const float* term, const int32_t* ids, int n, float* out)
{
    Handle* h = static_cast<Handle*>(hv);
    if (h->dbl) return -1;
    return oracle::owner_grad_bound(h->sf, term, ids, n, out);
}

}  // extern "C"

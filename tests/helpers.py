"""Shared test helpers: run the same scene through the oracle (CPU, test infrastructure) and the HIP path."""
from __future__ import annotations

import os

import numpy as np

import _omnigs

omr = _omnigs.load()
scene = omr.scene


def make_case(P, width, height, camera_type, seed, view_index=0, sh_degree=3, spread=None):
    """Seeded synthetic scene. `spread` rescales the distance range (small images want fewer, bigger Gaussians)."""
    g = scene.make_gaussians(P, seed)
    if spread is not None:
        g.scales = (g.scales * spread).astype(np.float32)
    g.sh_degree = sh_degree
    cam = scene.make_camera(camera_type, width, height, view_index)
    dL = scene.upstream_grad(height, width, seed + 1000)
    return g, cam, dL


def oracle_run(g, cam, dL=None, bg=(0.0, 0.0, 0.0), double=False, colors_precomp=None, cov3D_precomp=None,
               render_depth=False, prefiltered=False, nthreads=1, scale_modifier=1.0):
    import oracle as O

    o = O.Oracle(double)
    use_cov = cov3D_precomp is not None
    use_col = colors_precomp is not None
    L = o.forward(background=np.asarray(bg, dtype=np.float64), means3D=g.means3D, opacity=g.opacity,
                  scales=None if use_cov else g.scales, rotations=None if use_cov else g.rotations,
                  shs=None if use_col else g.shs, colors_precomp=colors_precomp, cov3D_precomp=cov3D_precomp,
                  viewmatrix=cam.viewmatrix, projmatrix=cam.projmatrix, campos=cam.campos, width=cam.width,
                  height=cam.height, sh_degree=g.sh_degree, tanfovx=cam.tanfovx, tanfovy=cam.tanfovy,
                  camera_type=cam.camera_type, render_depth=render_depth, prefiltered=prefiltered,
                  scale_modifier=scale_modifier)
    grads = o.backward(dL, nthreads) if dL is not None else None
    return o, L, grads


def hip_run(g, cam, dL=None, bg=(0.0, 0.0, 0.0), colors_precomp=None, cov3D_precomp=None, render_depth=False,
            prefiltered=False, device="cuda", sh_misalign=False, skip_dsh=False, scale_modifier=1.0):
    """The HIP path on one view. sh_misalign: the SH tensor starts 4 B past a 16-B boundary (a view into a larger
    buffer), so the kernels take their unaligned-row paths; skip_dsh: the backward does not write dL_dsh."""
    import torch

    R = omr.rasterizer
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).to(device)

    def t_sh(a):
        if not sh_misalign:
            return t(a)
        flat = torch.zeros(a.size + 1, dtype=torch.float32, device=device)
        v = flat[1:].view(a.shape)
        v.copy_(torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)))
        assert v.data_ptr() % 16 != 0
        return v
    use_cov = cov3D_precomp is not None
    use_col = colors_precomp is not None
    empty = torch.empty(0, device=device)
    bg_t = t(np.asarray(bg))
    args = dict(background=bg_t, means3D=t(g.means3D), colors=t(colors_precomp) if use_col else empty,
                opacity=t(g.opacity), scales=empty if use_cov else t(g.scales),
                rotations=empty if use_cov else t(g.rotations), scale_modifier=scale_modifier,
                cov3D_precomp=t(cov3D_precomp) if use_cov else empty, viewmatrix=t(cam.viewmatrix),
                projmatrix=t(cam.projmatrix), tan_fovx=cam.tanfovx, tan_fovy=cam.tanfovy, image_height=cam.height,
                image_width=cam.width, sh=empty if use_col else t_sh(g.shs), degree=g.sh_degree, campos=t(cam.campos),
                prefiltered=prefiltered, camera_type=cam.camera_type, render_depth=render_depth)
    num_rendered, color, radii, geomB, binB, imgB = R.RasterizeGaussiansCUDA(**args)
    out = dict(L=num_rendered, color=color, radii=radii, geom=geomB, binning=binB, img=imgB)
    out["state"] = R.debug_state(g.P, num_rendered, cam.width, cam.height, geomB, binB, imgB)
    if dL is not None:
        grads = R.RasterizeGaussiansBackwardCUDA(
            bg_t, args["means3D"], radii, args["colors"], args["scales"], args["rotations"], scale_modifier,
            args["cov3D_precomp"],
            args["viewmatrix"], args["projmatrix"], cam.tanfovx, cam.tanfovy, t(dL), args["sh"], g.sh_degree,
            args["campos"], geomB, num_rendered, binB, imgB, cam.camera_type, skip_dsh=skip_dsh)
        names = ["dmean2D", "dcolor", "dopacity", "dmean3D", "dcov3D", "dsh", "dscale", "drot"]
        out["grads"] = dict(zip(names, grads))
    import torch as _t

    _t.cuda.synchronize()
    return out


# ---- parity bars against the reference AS COMPILED -------------------------------------------
# The oracle restates the reference without FMA contraction and with the shared omni_math.h transcendentals; the
# reference binary contracts mul+add (nvcc --fmad=true) and uses libdevice. oracle/ambiguity.hpp bounds, from the
# oracle's own forward, every decision the two could take differently (tile rects, depth order of near-equal keys,
# alpha / power / saturation thresholds) and what each can change: the colour of a flagged pixel, and the gradient
# of a Gaussian owning a flagged decision (its flagged pixel terms through the linear preprocess backward,
# ambiguity.hpp: owner_grad_bound). The bars below allow exactly that, and tests/test_contraction_allowance.py checks
# on CPU that two FMA-contracted builds of the oracle (GCC, LLVM) stay inside them; the HIP path (bit-exact
# integers, v_exp in the blend loops) is held to the same bars, and its consumption of them is recorded per case
# (parity_residuals) and capped by a budget.
WIDE_RTOL, WIDE_ATOL_FRAC = 1e-2, 1e-3  # gradients of Gaussians blending behind a flagged decision
GRAD_NAMES = ("dmean2D", "dcolor", "dopacity", "dmean3D", "dcov3D", "dsh", "dscale", "drot")


def reference_allowance(o, dL=None):
    """oracle/ambiguity.hpp on o's (float) forward: dict(counts, pixel flags [H,W], bound [H,W] (largest colour
    change of the flagged decisions), flags [P] (G_* bits), owners [P] (Gaussians owning a flagged decision),
    exposed [P] (Gaussians blending behind one: the wide gradient bar), t_bound [H,W] (the same for final_T)). With
    the upstream gradient dL [3,H,W] also owner_ids [n] and owner_bound {name: [n, k]}: how far each owner's
    gradient may move (ambiguity.hpp: owner_term, owner_grad_bound). Without dL, owners have no gradient bar."""
    res = o.allowance(dL=dL)
    counts, flip, pix, bound = res[:4]
    P = o.P
    vis = o.get("radii") > 0
    rgb = o.get("rgb").reshape(P, 3)[vis] if vis.any() else np.zeros((1, 3), np.float32)
    cmax = max(float(np.abs(rgb).max()) if rgb.size else 0.0, float(np.abs(o.background).max()), 1e-6)
    owners = (flip & 7) != 0
    out = dict(counts=counts, pixel=pix, bound=bound, t_bound=bound / (2.0 * cmax), flags=flip, owners=owners,
               exposed=(flip & 8) != 0)
    if dL is not None:
        ids = np.nonzero(owners)[0].astype(np.int32)
        out["owner_ids"] = ids
        out["owner_bound"] = o.owner_grad_bound(res[4], ids)
    return out


def check_image(test_img, ref_img, allow, what="out_color", bound_key="bound"):
    """|test - ref| <= 1e-4 (north_star) everywhere, plus the flagged pixels' own bound where the reference as
    compiled may decide differently. test_img / ref_img: [..., H, W] (channels reduced by max)."""
    err = np.abs(np.asarray(test_img, np.float64) - np.asarray(ref_img, np.float64))
    if err.ndim == 3:
        err = err.max(0)
    bad = err > 1e-4 + allow[bound_key]
    if bad.any():
        ys, xs = np.nonzero(bad)
        raise AssertionError(f"{what}: {int(bad.sum())} pixels over 1e-4 + allowance (first ({xs[0]},{ys[0]}): err "
                             f"{err[ys[0], xs[0]]:.3g}, flags {int(allow['pixel'][ys[0], xs[0]])}, allowance "
                             f"{float(allow[bound_key][ys[0], xs[0]]):.3g})")
    return int((err > 1e-4).sum())


def grad_residuals(test, ref, allow, P, names=None):
    """How much of the gradient allowance `test` uses against `ref`, per tensor and in total: entries outside the
    strict grad_close bar, the Gaussians they belong to, how many of those are owners (held to their owner bound)
    or exposed (held to the wide bar), the largest fraction of an owner's bound used, and the entries outside every
    bar (`unexplained`, must be 0). An owner that is also exposed gets the wide bar plus its owner bound."""
    names = list(names or [n for n in GRAD_NAMES if n in ref])
    owners, exposed = allow["owners"], allow["exposed"]
    ob = allow.get("owner_bound")
    row_of = None
    if ob is not None:
        row_of = np.full(P, -1, np.int64)
        row_of[allow["owner_ids"]] = np.arange(len(allow["owner_ids"]))
    tot = dict(entries_outside_strict=0, gaussians_outside_strict=0, owner_gaussians_used=0,
               exposed_gaussians_used=0, unexplained=0, owner_bound_max_use=0.0)
    per, first_bad = {}, None
    for name in names:
        a = np.asarray(test[name], np.float64).reshape(P, -1)
        b = np.asarray(ref[name], np.float64).reshape(P, -1)
        scale = np.abs(b).max() if b.size else 0.0
        err = np.abs(a - b)
        lim = 1e-3 * np.abs(b) + 1e-4 * scale
        lim_w = WIDE_RTOL * np.abs(b) + WIDE_ATOL_FRAC * scale
        out = err > lim
        rows = out.any(axis=1)
        ok = ~out
        # exposed (not owners): the wide bar
        ok |= (exposed & ~owners)[:, None] & (err <= lim_w)
        used_owner, use_max = np.zeros(P, bool), 0.0
        if owners.any() and ob is not None:
            orow = np.nonzero(owners & rows)[0]
            if len(orow):
                bnd = ob[name].reshape(len(allow["owner_ids"]), -1)[row_of[orow]].astype(np.float64)
                base = np.where(exposed[orow][:, None], lim_w[orow], lim[orow])
                bar = base + bnd
                e = err[orow]
                ok[orow] |= e <= bar
                over = e > base
                used_owner[orow] = over.any(axis=1)
                if over.any():
                    use_max = float(((e - base) / np.maximum(bnd, 1e-38))[over].max())
        bad = ~ok
        d = dict(entries_outside_strict=int(out.sum()), gaussians_outside_strict=int(rows.sum()),
                 owner_gaussians_used=int((rows & owners).sum()),
                 exposed_gaussians_used=int((rows & exposed & ~owners).sum()), unexplained=int(bad.sum()),
                 owner_bound_max_use=use_max)
        per[name] = d
        for k in tot:
            tot[k] = max(tot[k], d[k]) if k == "owner_bound_max_use" else tot[k] + d[k]
        if bad.any() and first_bad is None:
            i = int(np.nonzero(bad.any(axis=1))[0][0])
            first_bad = (f"{name}: {int(bad.any(axis=1).sum())} Gaussians outside the bar (first {i}: "
                         f"{a[i]} vs {b[i]}, owner {bool(owners[i])}, exposed {bool(exposed[i])})")
    tot["per_tensor"] = per
    tot["first_unexplained"] = first_bad
    return tot


def check_grads(test, ref, allow, P, names=None):
    """grad_close per element; the wide bar (WIDE_RTOL, WIDE_ATOL_FRAC) on the Gaussians blending behind a flagged
    decision; on the Gaussians owning one, their bar plus their owner bound (reference_allowance with dL). Returns
    grad_residuals()."""
    r = grad_residuals(test, ref, allow, P, names)
    if r["unexplained"]:
        if allow.get("owner_bound") is None and allow["owners"].any():
            raise AssertionError("owners need reference_allowance(o, dL) for a gradient bar; " + str(r["first_unexplained"]))
        raise AssertionError(r["first_unexplained"])
    return r


# How much of the allowance the HIP path may use, per case (parity_residuals keys). The default scales with the
# case; the BASELINE configs carry their own (tests/test_gpu_parity.py: CONFIG_BUDGETS), set from the measured
# consumption (profiles/r04_parity_residuals.json) with headroom, at or below what the FMA-contracted proxies of the
# reference need (profiles/ambiguity.json), so a regression that pushes pixels or Gaussians into the allowance fails.
def default_budget(P, pixels):
    return dict(pixels_over_1e4=max(2, pixels // 100000), final_T_over_1e4=max(2, pixels // 100000),
                n_contrib_mismatches=max(4, pixels // 50000), gaussians_outside_strict=max(4, P // 50000),
                owner_gaussians_used=max(2, P // 100000), exposed_gaussians_used=max(2, P // 100000))


def record_residuals(rec, budget=None):
    """Append the case's residual record to $OMR_PARITY_RESIDUALS (JSON lines; tests/test_gpu_parity.py writes one
    per comparison) and assert it stays inside `budget` (default_budget when None)."""
    import json

    rec = dict(rec)
    rec["case"] = os.environ.get("PYTEST_CURRENT_TEST", "?").split(" ")[0]
    b = budget if budget is not None else default_budget(rec.get("P", 0), rec.get("pixels", 0))
    rec["budget"] = b
    path = os.environ.get("OMR_PARITY_RESIDUALS")
    if path:
        with open(path, "a") as f:
            f.write(json.dumps(rec) + "\n")
    over = {k: (rec.get(k, 0), v) for k, v in b.items() if rec.get(k, 0) > v}
    assert not over, f"parity residual over budget (used, budget): {over}"
    return rec


def oracle_threads() -> int:
    """Threads for the oracle at the full BASELINE sizes: the box's CPU share (16) or this container's CPUs."""
    return max(1, min(16, os.cpu_count() or 1))


def to_np(x):
    return x.detach().cpu().numpy()


def grad_close(a, b, rtol=1e-3, atol_frac=1e-4, elementwise=False):
    """Per-element |a-b| <= rtol*|b| + atol_frac*max|b| (documented gradient tolerance: north_star 1e-3 rel, with an
    absolute floor at 1e-4 of the tensor's largest entry for entries that cancel to ~0). elementwise=True returns the
    boolean array of entries inside the bar instead."""
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    scale = np.abs(b).max() if b.size else 0.0
    err = np.abs(a - b)
    lim = rtol * np.abs(b) + atol_frac * scale
    bad = err > lim
    if elementwise:
        return ~bad
    return (not bad.any()), (float(err.max()) if err.size else 0.0), int(bad.sum())


# SH constants of cuda_rasterizer/auxiliary.h:32-49 (the test-side model of omr_sh_grad_from_colors)
_C0, _C1 = 0.28209479177387814, 0.4886025119029199
_C2 = (1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792, 0.5462742152960396)
_C3 = (-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154, -0.4570457994644658,
       1.445305721320277, -0.5900435899266435)


def sh_basis_np(deg, x, y, z):
    """SH basis values [..., 16] of forward.cu:30-83 / backward.cu:56-112 (zeros beyond (deg+1)^2), float64."""
    c = np.zeros(x.shape + (16,))
    c[..., 0] = _C0
    if deg > 0:
        c[..., 1], c[..., 2], c[..., 3] = -_C1 * y, _C1 * z, -_C1 * x
    if deg > 1:
        xx, yy, zz = x * x, y * y, z * z
        c[..., 4], c[..., 5] = _C2[0] * x * y, _C2[1] * y * z
        c[..., 6], c[..., 7], c[..., 8] = _C2[2] * (2 * zz - xx - yy), _C2[3] * x * z, _C2[4] * (xx - yy)
    if deg > 2:
        c[..., 9] = _C3[0] * y * (3 * xx - yy)
        c[..., 10] = _C3[1] * x * y * z
        c[..., 11] = _C3[2] * y * (4 * zz - xx - yy)
        c[..., 12] = _C3[3] * z * (2 * zz - 3 * xx - 3 * yy)
        c[..., 13] = _C3[4] * x * (4 * zz - xx - yy)
        c[..., 14] = _C3[5] * z * (xx - yy)
        c[..., 15] = _C3[6] * x * (xx - 3 * yy)
    return c


def sh_grad_from_colors_np(means3D, shs, deg, campos_all, dcolors_all):
    """Sum over views of dL/dsh rebuilt from each view's colour gradient (model of omr_sh_grad_from_colors):
    dL/dsh_k = basis_k(dir_v) * dRGB_v, dRGB_v zeroed where the forward clamped the colour (backward.cu:30-151)."""
    m = np.asarray(means3D, np.float64)
    sh = np.asarray(shs, np.float64)
    out = np.zeros_like(sh)
    for cp, dc in zip(np.asarray(campos_all, np.float64), np.asarray(dcolors_all, np.float64)):
        d = m - cp
        d /= np.linalg.norm(d, axis=1, keepdims=True)
        basis = sh_basis_np(deg, d[:, 0], d[:, 1], d[:, 2])
        rgb = np.einsum("pk,pkc->pc", basis, sh[:, :16]) + 0.5
        dm = np.where(rgb < 0, 0.0, dc)
        out[:, :16] += basis[:, :, None] * dm[:, None, :]
    return out

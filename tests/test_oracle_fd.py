"""Finite-difference checks of the oracle's backward (double instantiation of oracle/omni_oracle.hpp).

Loss = sum(dL_dout * out_color). The analytic gradients are the reference's (backward.cu, restated) and the
forward is the reference's (forward.cu, restated), so agreement pins the restated backward — including the
lonlat second-derivative terms of backward.cu:455-475 (supp.pdf App. A) — against its own forward.

Scenes avoid the non-differentiable spots of the forward: opacities <= 0.9 (alpha never reaches the 0.99
clamp, which the reference's backward ignores), few overlapping Gaussians (no T < 1e-4 cut-off), and central
differences with h = 1e-6 so that the 1/255 threshold and the tile rects practically never flip.
Tolerance: |fd - analytic| <= 2e-4 * max|analytic of that tensor| + 1e-3 * |analytic| per element.
"""
import numpy as np
import pytest

import oracle as O
from helpers import scene

H_STEP = 1e-6


def _scene(P, W, H, cam_type, seed, deg, view=0):
    rng = np.random.default_rng(seed)
    g = scene.make_gaussians(P, seed)
    if cam_type == scene.CAMERA_LONLAT:
        # spread around the sphere, 2-5 m away, big enough to cover several pixels at this resolution
        d = rng.standard_normal((P, 3))
        d /= np.linalg.norm(d, axis=1, keepdims=True)
        d[:, 1] *= 0.6  # keep away from the poles
        d /= np.linalg.norm(d, axis=1, keepdims=True)
        means = d * rng.uniform(2, 5, (P, 1))
    else:
        means = np.c_[rng.uniform(-1, 1, P), rng.uniform(-0.5, 0.5, P), rng.uniform(2, 4, P)]
    g.means3D = means.astype(np.float64)
    g.scales = np.exp(rng.uniform(np.log(0.05), np.log(0.2), (P, 3)))
    q = rng.standard_normal((P, 4))
    g.rotations = q / np.linalg.norm(q, axis=1, keepdims=True)
    g.opacity = rng.uniform(0.2, 0.9, (P, 1))
    g.shs = rng.standard_normal((P, 16, 3)) * 0.3
    g.shs[:, 0, :] += 1.0  # keep colours away from the clamp at 0
    g.sh_degree = deg
    cam = scene.make_camera(cam_type, W, H, view)
    dL = rng.standard_normal((3, H, W))
    return g, cam, dL


def _loss_and_grads(g, cam, dL, **over):
    o = O.Oracle(double=True)
    kw = dict(background=np.array([0.1, 0.2, 0.3]), means3D=g.means3D, opacity=g.opacity, scales=g.scales,
              rotations=g.rotations, shs=g.shs, viewmatrix=cam.viewmatrix.astype(np.float64),
              projmatrix=cam.projmatrix.astype(np.float64), campos=cam.campos.astype(np.float64), width=cam.width,
              height=cam.height, sh_degree=g.sh_degree, tanfovx=cam.tanfovx, tanfovy=cam.tanfovy,
              camera_type=cam.camera_type)
    kw.update(over)
    o.forward(**kw)
    img = o.get("out_color").reshape(3, cam.height, cam.width)
    return float((img * dL).sum()), o, kw


def _check(name, an, fd):
    an, fd = np.asarray(an, np.float64), np.asarray(fd, np.float64)
    lim = 2e-4 * np.abs(an).max() + 1e-3 * np.abs(an)
    bad = np.abs(an - fd) > lim
    assert not bad.any(), f"{name}: max |fd-an| = {np.abs(an - fd).max():.3e}, max|an| = {np.abs(an).max():.3e}"


@pytest.mark.parametrize("cam_type,deg", [(scene.CAMERA_LONLAT, 3), (scene.CAMERA_LONLAT, 1),
                                          (scene.CAMERA_PINHOLE, 3), (scene.CAMERA_PINHOLE, 0)])
def test_fd_all_parameters(cam_type, deg, oracle_mod):
    W, H = (64, 32) if cam_type == scene.CAMERA_LONLAT else (48, 36)
    g, cam, dL = _scene(12, W, H, cam_type, 100 + deg + cam_type, deg, view=1)
    _, o, kw = _loss_and_grads(g, cam, dL)
    grads = o.backward(dL)
    assert (o.get("radii") > 0).sum() >= 8

    def fd(param, idx):
        base = kw[param].copy()
        out = []
        for sgn in (+1, -1):
            arr = base.copy()
            arr[idx] += sgn * H_STEP
            out.append(_loss_and_grads(g, cam, dL, **{param: arr})[0])
        return (out[0] - out[1]) / (2 * H_STEP)

    checks = [("means3D", "dmean3D", 3), ("scales", "dscale", 3), ("rotations", "drot", 4),
              ("opacity", "dopacity", 1)]
    for param, gname, k in checks:
        an = grads[gname].reshape(-1, k)
        fdv = np.array([[fd(param, (i, c)) for c in range(k)] for i in range(g.P)])
        _check(param, an, fdv)
    nk = (deg + 1) ** 2
    an = grads["dsh"][:, :nk, :]
    fdv = np.array([[[fd("shs", (i, c, ch)) for ch in range(3)] for c in range(nk)] for i in range(4)])
    _check("shs", an[:4], fdv)
    assert (grads["dsh"][:, nk:, :] == 0).all()


def test_fd_cov3D_precomp_and_colors_precomp(oracle_mod):
    g, cam, dL = _scene(10, 64, 32, scene.CAMERA_LONLAT, 7, 3)
    o0 = O.Oracle(double=True)
    o0.forward(background=np.zeros(3), means3D=g.means3D, opacity=g.opacity, scales=g.scales, rotations=g.rotations,
               shs=g.shs, viewmatrix=cam.viewmatrix.astype(np.float64), projmatrix=cam.projmatrix.astype(np.float64),
               campos=cam.campos.astype(np.float64), width=64, height=32, sh_degree=3, camera_type=3)
    cov = o0.get("cov3D").reshape(-1, 6)
    colors = np.random.default_rng(3).uniform(0.1, 0.9, (g.P, 3))
    _, o, kw = _loss_and_grads(g, cam, dL, scales=None, rotations=None, shs=None, cov3D_precomp=cov,
                               colors_precomp=colors)
    grads = o.backward(dL)

    def fd(param, idx):
        vals = []
        for sgn in (+1, -1):
            arr = kw[param].copy()
            arr[idx] += sgn * H_STEP
            vals.append(_loss_and_grads(g, cam, dL, scales=None, rotations=None, shs=None,
                                        **{**{"cov3D_precomp": cov, "colors_precomp": colors}, param: arr})[0])
        return (vals[0] - vals[1]) / (2 * H_STEP)

    _check("colors_precomp", grads["dcolor"], np.array([[fd("colors_precomp", (i, c)) for c in range(3)]
                                                         for i in range(g.P)]))
    # dL/dcov3D is w.r.t. the 6 stored entries; off-diagonal entries appear twice in the symmetric matrix
    # (backward.cu:418-422 doubles them), which is exactly the derivative w.r.t. the stored value
    _check("cov3D_precomp", grads["dcov3D"], np.array([[fd("cov3D_precomp", (i, c)) for c in range(6)]
                                                        for i in range(g.P)]))
    _check("means3D(cov,col)", grads["dmean3D"], np.array([[fd("means3D", (i, c)) for c in range(3)]
                                                           for i in range(g.P)]))

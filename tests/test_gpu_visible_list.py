"""gaussian_bwd over the visible list (gaussian_bwd.hip: gaussian_bwd_list_kernel): after a
forward whose depth sort set the culled Gaussians aside (every pinhole view by default), the backward writes every
Gaussian's outputs as a culled one's in index order and then runs the per-Gaussian chain densely over the depth-sorted
visible Gaussians. Its arithmetic is the index-order wave kernel's, so every gradient must be bit-identical to the
backward after the plain depth sort (which gives the same visible order, so the same forward and render backward).
Covered: pinhole with the stored dRGB/ddir, pinhole reading the SH rows (flag cleared), 9-coefficient SH rows (the
per-float path), precomputed colours, and a lonlat view forced onto the culled-aside sort."""
import numpy as np
import pytest
import torch

from helpers import make_case, omr, scene
from test_gpu_sh_jac import _backward, _forward

pytestmark = pytest.mark.gpu

R = omr.rasterizer
LON, PIN = scene.CAMERA_LONLAT, scene.CAMERA_PINHOLE


def _grads_with_mode(mode, g, cam, dL, colors=None, clear_jac=False):
    old = R.debug_depth_sort_mode(mode)
    try:
        args, fwd = _forward(g, cam, colors)
        geomB = fwd[3]
        vis = R.debug_counters(g.P, geomB)["visible"]
        if clear_jac:
            R.debug_set_sh_jac(g.P, geomB, False)
        grads = _backward(g, cam, args, fwd, dL)
        radii = fwd[2].cpu().numpy()
    finally:
        R.debug_depth_sort_mode(old)
    return grads, vis, radii


@pytest.mark.parametrize("case", ["pinhole_jac", "pinhole_sh_rows", "pinhole_M9", "pinhole_colors", "lonlat_forced"])
def test_visible_list_backward_is_bitwise_the_wave_kernel(case):
    cam_t = LON if case == "lonlat_forced" else PIN
    g, cam, dL = make_case(20000, 320, 180, cam_t, 71, view_index=1, spread=1.0)
    colors = None
    if case == "pinhole_M9":
        g.shs = np.ascontiguousarray(g.shs[:, :9, :])
        g.sh_degree = 2
    if case == "pinhole_colors":
        colors = np.random.default_rng(72).uniform(0, 1, (g.P, 3)).astype(np.float32)
    clear = case == "pinhole_sh_rows"
    ref, vis_ref, radii = _grads_with_mode(1, g, cam, dL, colors, clear)  # plain sort: the index-order wave kernel
    out, vis, radii2 = _grads_with_mode(2, g, cam, dL, colors, clear)     # culled aside: the visible list
    assert vis_ref is None, "the plain sort publishes no visible list"
    nvis = int((radii > 0).sum())
    assert vis == nvis and 0 < nvis <= g.P, (vis, nvis, g.P)
    if cam_t == PIN:
        assert nvis < g.P, "the pinhole view culls part of the scene"
    assert np.array_equal(radii, radii2)
    for k, (a, b) in enumerate(zip(out, ref)):
        assert a.shape == b.shape, k
        assert torch.equal(a, b), f"gradient {k}: max |diff| {float((a - b).abs().max())}"

"""The backward's SH direction gradient from the forward's stored dRGB/ddir (GeomState::sh_jac) against the path that
reads the SH rows: one forward, the backward run twice on its buffers, once with the stored
values and once with the flag cleared (omr_debug_set_sh_jac), so the kernel reads the 192-B SH rows and evaluates
sh_eval.h: sh_dir_grad itself. Both sites run that one function without contraction, so every gradient must be
bit-identical. The stored values are also checked against the oracle transitively by tests/test_gpu_parity.py,
whose backward takes them by default."""
import numpy as np
import pytest
import torch

from helpers import make_case, omr, scene

pytestmark = pytest.mark.gpu

R = omr.rasterizer


def _forward(g, cam, colors=None):
    dev = torch.device("cuda", 0)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).to(dev)  # noqa: E731
    empty = torch.empty(0, device=dev)
    args = dict(background=t(np.zeros(3)), means3D=t(g.means3D), colors=empty if colors is None else t(colors),
                opacity=t(g.opacity), scales=t(g.scales), rotations=t(g.rotations), scale_modifier=1.0,
                cov3D_precomp=empty, viewmatrix=t(cam.viewmatrix), projmatrix=t(cam.projmatrix), tan_fovx=cam.tanfovx,
                tan_fovy=cam.tanfovy, image_height=cam.height, image_width=cam.width,
                sh=t(g.shs) if colors is None else empty, degree=g.sh_degree, campos=t(cam.campos), prefiltered=False,
                camera_type=cam.camera_type, render_depth=False)
    return args, R.RasterizeGaussiansCUDA(**args)


def _backward(g, cam, args, fwd, dL):
    num_rendered, _, radii, geomB, binB, imgB = fwd
    grads = R.RasterizeGaussiansBackwardCUDA(
        args["background"], args["means3D"], radii, args["colors"], args["scales"], args["rotations"], 1.0,
        args["cov3D_precomp"], args["viewmatrix"], args["projmatrix"], cam.tanfovx, cam.tanfovy,
        torch.from_numpy(np.ascontiguousarray(dL, dtype=np.float32)).to(args["means3D"].device), args["sh"],
        g.sh_degree, args["campos"], geomB, num_rendered, binB, imgB, cam.camera_type)
    torch.cuda.synchronize()
    return [x.clone() for x in grads]


@pytest.mark.parametrize("camera,deg", [(scene.CAMERA_LONLAT, 3), (scene.CAMERA_PINHOLE, 3), (scene.CAMERA_LONLAT, 1)])
def test_stored_direction_gradient_matches_sh_row_path_bitwise(camera, deg):
    g, cam, dL = make_case(3000, 256, 128, camera, 21, view_index=2, sh_degree=deg, spread=2.0)
    args, fwd = _forward(g, cam)
    geomB = fwd[3]
    assert R.debug_counters(g.P, geomB)["sh_jac"], "a 16-coefficient forward stores dRGB/ddir"
    with_jac = _backward(g, cam, args, fwd, dL)
    R.debug_set_sh_jac(g.P, geomB, False)
    assert not R.debug_counters(g.P, geomB)["sh_jac"]
    from_rows = _backward(g, cam, args, fwd, dL)
    names = ["dmean2D", "dcolor", "dopacity", "dmean3D", "dcov3D", "dsh", "dscale", "drot"]
    for n, a, b in zip(names, with_jac, from_rows):
        assert torch.equal(a, b), n
    assert torch.count_nonzero(with_jac[3]) > 0  # the direction term reaches dL/dmean3D


def test_precomputed_colours_store_no_direction_gradient():
    g, cam, dL = make_case(500, 128, 64, scene.CAMERA_LONLAT, 22, view_index=1, spread=3.0)
    colors = np.random.default_rng(5).random((g.P, 3)).astype(np.float32)
    _, fwd = _forward(g, cam, colors=colors)
    assert not R.debug_counters(g.P, fwd[3])["sh_jac"]


@pytest.mark.parametrize("camera", [scene.CAMERA_LONLAT, scene.CAMERA_PINHOLE])
def test_sh_row_path_alone_matches_the_oracle(camera):
    """The backward's own dRGB/ddir evaluation (the MC == 16 row-reading path, flag cleared) against the oracle, not
    only against the stored path: a wrong sh_dir_grad shared by both sites would fail here."""
    from helpers import grad_close, oracle_run, to_np

    g, cam, dL = make_case(2000, 256, 128, camera, 23, view_index=3, spread=2.0)
    args, fwd = _forward(g, cam)
    R.debug_set_sh_jac(g.P, fwd[3], False)
    grads = _backward(g, cam, args, fwd, dL)
    _, L, og = oracle_run(g, cam, dL)
    assert fwd[0] == L
    for name, idx in (("dmean3D", 3), ("dsh", 5), ("dopacity", 2), ("dscale", 6), ("drot", 7)):
        ok, emax, nbad = grad_close(to_np(grads[idx]), og[name])
        assert ok, (name, emax, nbad)


def test_backward_with_other_inputs_recomputes_the_direction_gradient():
    """sh_jac is keyed to the forward's SH array, means and campos (raster_common.h: sh_jac_key): a backward handed
    another camera position uses its own inputs, as the reference's backward does (backward.cu:56-112), and equals
    the row-reading path on those inputs bit for bit."""
    g, cam, dL = make_case(2000, 256, 128, scene.CAMERA_LONLAT, 24, view_index=1, spread=2.0)
    args, fwd = _forward(g, cam)
    geomB = fwd[3]
    key = R.debug_counters(g.P, geomB)["sh_jac_key"]
    assert key != 0
    same = _backward(g, cam, args, fwd, dL)
    moved = dict(args, campos=args["campos"] + torch.tensor([0.05, -0.02, 0.03], device=args["campos"].device))
    other = _backward(g, cam, moved, fwd, dL)
    R.debug_set_sh_jac(g.P, geomB, False)
    other_rows = _backward(g, cam, moved, fwd, dL)
    R.debug_set_sh_jac(g.P, geomB, True)
    assert R.debug_counters(g.P, geomB)["sh_jac_key"] == key  # restored
    for a, b in zip(other, other_rows):
        assert torch.equal(a, b)
    assert not torch.equal(other[5], same[5])  # dL/dsh depends on the view direction
    # a copy of the SH array (another pointer, the same values) also takes the row path: the same bits
    copied = dict(args, sh=args["sh"].clone())
    for a, b in zip(_backward(g, cam, copied, fwd, dL), same):
        assert torch.equal(a, b)

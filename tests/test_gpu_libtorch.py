"""The LibTorch drop-in (librasterize_points.so, reference rasterize_points.h symbols) on the GPU: results are
bitwise identical to the Python boundary (same C ABI underneath) and meet the oracle parity bar."""
import numpy as np
import pytest
import torch

from helpers import grad_close, hip_run, make_case, oracle_run, scene, to_np

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cam_type", [scene.CAMERA_LONLAT, scene.CAMERA_PINHOLE])
def test_libtorch_boundary_matches_python_boundary_and_oracle(cam_type, omr):
    W, H = (128, 64) if cam_type == scene.CAMERA_LONLAT else (160, 90)
    g, cam, dL = make_case(1000, W, H, cam_type, 41, spread=3.0)
    m = omr.rasterizer.libtorch_boundary()
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).cuda()
    e = torch.empty(0, device="cuda")
    bg = torch.zeros(3, device="cuda")
    nr, color, radii, gb, bb, ib = m.RasterizeGaussiansCUDA(
        bg, t(g.means3D), e, t(g.opacity), t(g.scales), t(g.rotations), 1.0, e, t(cam.viewmatrix), t(cam.projmatrix),
        cam.tanfovx, cam.tanfovy, H, W, t(g.shs), g.sh_degree, t(cam.campos), False, cam_type, False)
    grads = m.RasterizeGaussiansBackwardCUDA(bg, t(g.means3D), radii, e, t(g.scales), t(g.rotations), 1.0, e,
                                             t(cam.viewmatrix), t(cam.projmatrix), cam.tanfovx, cam.tanfovy, t(dL),
                                             t(g.shs), g.sh_degree, t(cam.campos), gb, nr, bb, ib, cam_type)
    torch.cuda.synchronize()
    h = hip_run(g, cam, dL)
    assert nr == h["L"]
    assert torch.equal(color, h["color"]) and torch.equal(radii, h["radii"])
    names = ["dmean2D", "dcolor", "dopacity", "dmean3D", "dcov3D", "dsh", "dscale", "drot"]
    for name, a in zip(names, grads):
        assert torch.equal(a, h["grads"][name]), name  # deterministic backward: bitwise equal
    o, L, og = oracle_run(g, cam, dL)
    assert nr == L
    assert np.abs(to_np(color) - o.get("out_color").reshape(3, H, W)).max() <= 1e-4
    ok, emax, nbad = grad_close(to_np(grads[3]), og["dmean3D"])
    assert ok, (emax, nbad)
    present = m.markVisible(t(g.means3D), t(cam.viewmatrix), t(cam.projmatrix), cam_type)
    assert present.dtype == torch.bool and present.shape == (g.P,)


def test_libtorch_boundary_errors(omr):
    m = omr.rasterizer.libtorch_boundary()
    e = torch.empty(0, device="cuda")
    with pytest.raises(RuntimeError, match="num_points, 3"):
        m.RasterizeGaussiansCUDA(e, torch.zeros(4, 2, device="cuda"), e, e, e, e, 1.0, e, e, e, 0.0, 0.0, 32, 64, e,
                                 3, e, False, 3, False)
    with pytest.raises(RuntimeError, match="Invalid camera_type"):
        m.RasterizeGaussiansCUDA(torch.zeros(3, device="cuda"), torch.zeros(4, 3, device="cuda"), e,
                                 torch.ones(4, 1, device="cuda"), torch.ones(4, 3, device="cuda"),
                                 torch.ones(4, 4, device="cuda"), 1.0, e, torch.eye(4, device="cuda"),
                                 torch.eye(4, device="cuda"), 0.0, 0.0, 32, 64, torch.zeros(4, 16, 3, device="cuda"),
                                 3, torch.zeros(3, device="cuda"), False, 2, False)

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


@pytest.mark.parametrize("cam_type", [scene.CAMERA_LONLAT, scene.CAMERA_PINHOLE])
def test_libtorch_boundary_takes_non_contiguous_inputs(cam_type, omr):
    """rasterize_points.cu:113-130 takes .contiguous() of every input; the reference host passes a transposed
    viewmatrix view (world_view_transform_ = EigenMatrix2TorchTensor(Tcw).transpose(0, 1),
    gaussian_keyframe.cpp:137-140, passed by gaussian_renderer.cpp:68,201). Non-contiguous views of the same
    values — a transposed viewmatrix / projmatrix, means3D and scales as column slices of wider tensors, a strided
    SH — give results bitwise equal to the contiguous call, forward and backward."""
    W, H = (128, 64) if cam_type == scene.CAMERA_LONLAT else (160, 90)
    g, cam, dL = make_case(1500, W, H, cam_type, 43, spread=3.0)
    m = omr.rasterizer.libtorch_boundary()
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).cuda()
    e = torch.empty(0, device="cuda")
    bg = torch.zeros(3, device="cuda")

    def wide(a):  # the same values as a column slice of a [P, k + 2] tensor (row stride k + 2)
        w = torch.zeros(a.shape[0], a.shape[1] + 2, device="cuda")
        w[:, 1:1 + a.shape[1]] = t(a)
        v = w[:, 1:1 + a.shape[1]]
        assert not v.is_contiguous()
        return v

    vm_nc = t(cam.viewmatrix.T).t()
    pm_nc = t(cam.projmatrix.T).t()
    assert not vm_nc.is_contiguous() and torch.equal(vm_nc, t(cam.viewmatrix))
    sh_nc = t(np.ascontiguousarray(g.shs.transpose(0, 2, 1))).transpose(1, 2)
    assert not sh_nc.is_contiguous()

    def run(means, scales, vm, pm, sh):
        nr, color, radii, gb, bb, ib = m.RasterizeGaussiansCUDA(
            bg, means, e, t(g.opacity), scales, t(g.rotations), 1.0, e, vm, pm, cam.tanfovx, cam.tanfovy, H, W, sh,
            g.sh_degree, t(cam.campos), False, cam_type, False)
        grads = m.RasterizeGaussiansBackwardCUDA(bg, means, radii, e, scales, t(g.rotations), 1.0, e, vm, pm,
                                                 cam.tanfovx, cam.tanfovy, t(dL), sh, g.sh_degree, t(cam.campos), gb,
                                                 nr, bb, ib, cam_type)
        torch.cuda.synchronize()
        return nr, color, radii, grads

    a = run(t(g.means3D), t(g.scales), t(cam.viewmatrix), t(cam.projmatrix), t(g.shs))
    b = run(wide(g.means3D), wide(g.scales), vm_nc, pm_nc, sh_nc)
    assert a[0] == b[0] and torch.equal(a[1], b[1]) and torch.equal(a[2], b[2])
    for x, y in zip(a[3], b[3]):
        assert torch.equal(x, y)

"""The view-parallel SH-gradient rebuild (omr_sh_grad_from_colors, parallel.allreduce_compact_) on the GPU.

For several views of the same Gaussians, the HIP backward gives per-view dL/dsh and dL/dcolors. Summing the
per-view dL/dsh in view order must equal, bit for bit, the rebuild from the per-view dL/dcolors and camera
positions (same SH arithmetic, sh_eval.h, same products, same summation order); it must also match the float64
numpy model of tests/helpers.py.
"""
import numpy as np
import pytest
import torch

from helpers import grad_close, hip_run, make_case, omr, scene, sh_grad_from_colors_np, to_np

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cam_type,deg", [(scene.CAMERA_LONLAT, 3), (scene.CAMERA_PINHOLE, 3),
                                          (scene.CAMERA_LONLAT, 1)])
def test_sh_rebuild_equals_sum_of_views(cam_type, deg):
    R = omr.rasterizer
    views = (0, 3, 5)
    W, H = (256, 128) if cam_type == scene.CAMERA_LONLAT else (160, 90)
    dsh_sum, dcolors, campos = None, [], []
    g = None
    for v in views:
        g, cam, dL = make_case(3000, W, H, cam_type, 91, view_index=v, sh_degree=deg, spread=2.0)
        h = hip_run(g, cam, dL)
        dsh = h["grads"]["dsh"]
        dsh_sum = dsh.clone() if dsh_sum is None else dsh_sum + dsh
        dcolors.append(h["grads"]["dcolor"])
        campos.append(torch.from_numpy(cam.campos).cuda())
    dev = dsh_sum.device
    means = torch.from_numpy(g.means3D).to(dev)
    shs = torch.from_numpy(g.shs).to(dev)
    rebuilt = R.sh_grad_from_colors(means, shs, deg, torch.stack(campos), torch.stack(dcolors))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(to_np(rebuilt), to_np(dsh_sum))
    # the packed layout parallel.allreduce_compact_ gathers: [n, P+1, 3], campos as row P of each view
    packed = torch.cat([torch.stack(dcolors), torch.stack(campos)[:, None, :]], dim=1).contiguous()
    np.testing.assert_array_equal(to_np(R.sh_grad_from_colors_packed(means, shs, deg, packed)), to_np(dsh_sum))
    model =sh_grad_from_colors_np(g.means3D, g.shs, deg, to_np(torch.stack(campos)), to_np(torch.stack(dcolors)))
    ok, emax, nbad = grad_close(to_np(rebuilt), model)
    assert ok, (emax, nbad)


def test_sh_rebuild_argument_checks():
    R = omr.rasterizer
    m = torch.zeros((10, 3), device="cuda")
    sh = torch.zeros((10, 16, 3), device="cuda")
    with pytest.raises(R.RasterizerError):
        R.sh_grad_from_colors(m, sh, 3, torch.zeros((2, 3), device="cuda"), torch.zeros((3, 10, 3), device="cuda"))


@pytest.mark.parametrize("cam_type", [scene.CAMERA_LONLAT, scene.CAMERA_PINHOLE])
def test_colors_event_fires_when_colour_gradients_are_final(cam_type):
    """parallel.CompactExchange's overlap: the backward records colors_event once dL_dcolors is final (row sums),
    before the per-Gaussian backward. A side stream that waits on the event and copies dL_dcolors right away must see
    the final values; skip_dsh leaves dL_dsh unwritten and every other output equal to the plain backward."""
    R = omr.rasterizer
    W, H = (512, 256) if cam_type == scene.CAMERA_LONLAT else (320, 180)
    g, cam, dL = make_case(20000, W, H, cam_type, 17, view_index=2)
    ref = hip_run(g, cam, dL)
    dev = torch.device("cuda")
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).to(dev)
    m, sc, rot, sh, op = t(g.means3D), t(g.scales), t(g.rotations), t(g.shs), t(g.opacity)
    vm, pm, cp, bg, dl = t(cam.viewmatrix), t(cam.projmatrix), t(cam.campos), torch.zeros(3, device=dev), t(dL)
    e = torch.empty(0, device=dev)
    nr, color, radii, gb, bb, ib = R.RasterizeGaussiansCUDA(bg, m, e, op, sc, rot, 1.0, e, vm, pm, cam.tanfovx,
                                                            cam.tanfovy, H, W, sh, g.sh_degree, cp, False,
                                                            cam.camera_type, False)
    ev = torch.cuda.Event()
    side = torch.cuda.Stream(dev)
    grads = R.RasterizeGaussiansBackwardCUDA(bg, m, radii, e, sc, rot, 1.0, e, vm, pm, cam.tanfovx, cam.tanfovy, dl,
                                             sh, g.sh_degree, cp, gb, nr, bb, ib, cam.camera_type,
                                             colors_event=ev, skip_dsh=True)
    with torch.cuda.stream(side):
        side.wait_event(ev)
        early = grads[1].clone()
    torch.cuda.synchronize()
    assert grads[5] is None
    np.testing.assert_array_equal(to_np(early), to_np(ref["grads"]["dcolor"]))
    for i, name in enumerate(["dmean2D", "dcolor", "dopacity", "dmean3D", "dcov3D"]):
        np.testing.assert_array_equal(to_np(grads[i]), to_np(ref["grads"][name]), err_msg=name)
    np.testing.assert_array_equal(to_np(grads[6]), to_np(ref["grads"]["dscale"]))
    np.testing.assert_array_equal(to_np(grads[7]), to_np(ref["grads"]["drot"]))
    # the event is consumed by that call: a second backward without one records nothing and must still work
    again = R.RasterizeGaussiansBackwardCUDA(bg, m, radii, e, sc, rot, 1.0, e, vm, pm, cam.tanfovx, cam.tanfovy, dl,
                                             sh, g.sh_degree, cp, gb, nr, bb, ib, cam.camera_type)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(to_np(again[5]), to_np(ref["grads"]["dsh"]))

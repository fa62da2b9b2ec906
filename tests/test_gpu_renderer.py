"""Renderer glue (renderer.py, reference gaussian_renderer.cpp renderLonlat/render + gaussian_model.cpp activations)
end-to-end on the GPU: raw parameters -> activations -> HIP rasterizer -> loss -> autograd -> raw-parameter grads.

The oracle renders the exact activated float32 tensors the GPU saw; its activated-space gradients are chained to the
raw parameters in float64 torch on the CPU (exact chain rule), then compared at the north_star tolerances.
"""
import types

import numpy as np
import pytest
import torch

from helpers import grad_close, make_case, omr, oracle_run, scene, to_np

pytestmark = pytest.mark.gpu
RD = omr.renderer


def _raw_params(g, device, seed):
    rng = np.random.default_rng(seed)
    f32 = lambda a: torch.tensor(np.ascontiguousarray(a, dtype=np.float32), device=device, requires_grad=True)
    o = np.clip(g.opacity.astype(np.float64), 1e-6, 1 - 1e-6)
    rot = g.rotations * rng.uniform(0.5, 2.0, size=(g.P, 1))  # unnormalised: exercises the normalize grad
    return RD.GaussianModelParams(f32(g.means3D), f32(g.shs[:, :1]), f32(g.shs[:, 1:]), f32(np.log(o / (1 - o))),
                                  f32(np.log(g.scales)), f32(rot), g.sh_degree, 3)


def _viewpoint(cam, device, fovx=0.0, fovy=0.0):
    t = lambda a: torch.tensor(np.ascontiguousarray(a, dtype=np.float32), device=device)
    return RD.Viewpoint(t(cam.viewmatrix), t(cam.projmatrix), t(cam.campos), fovx, fovy)


def _activated(pc):
    with torch.no_grad():
        return types.SimpleNamespace(means3D=to_np(pc.get_xyz()), scales=to_np(pc.get_scaling_activation()),
                                     rotations=to_np(pc.get_rotation_activation()),
                                     opacity=to_np(pc.get_opacity_activation()), shs=to_np(pc.get_features()),
                                     sh_degree=pc.active_sh_degree, P=pc.xyz.shape[0])


def _chain_to_raw(pc, og):
    """Oracle activated-space grads -> raw-parameter grads (float64 autograd of the same activations, CPU)."""
    d = lambda t: t.detach().cpu().double().requires_grad_(True)
    sc, rot, op, dc, rest = d(pc.scaling), d(pc.rotation), d(pc.opacity), d(pc.features_dc), d(pc.features_rest)
    outs = [torch.exp(sc), torch.nn.functional.normalize(rot), torch.sigmoid(op), torch.cat([dc, rest], 1)]
    gouts = [torch.from_numpy(og[k].astype(np.float64)).reshape(o.shape)
             for k, o in zip(["dscale", "drot", "dopacity", "dsh"], outs)]
    gs = torch.autograd.grad(outs, [sc, rot, op, dc, rest], gouts)
    return dict(xyz=og["dmean3D"], scaling=gs[0].numpy(), rotation=gs[1].numpy(), opacity=gs[2].numpy(),
                features_dc=gs[3].numpy(), features_rest=gs[4].numpy())


@pytest.mark.parametrize("cam_type", [scene.CAMERA_LONLAT, scene.CAMERA_PINHOLE])
def test_render_end_to_end_raw_param_grads(cam_type):
    W, H = (192, 96) if cam_type == scene.CAMERA_LONLAT else (160, 120)
    g, cam, dL = make_case(1500, W, H, cam_type, 77, spread=3.0)
    pc = _raw_params(g, "cuda", 5)
    bg = torch.tensor([0.1, 0.2, 0.3], device="cuda")
    pipe = RD.PipelineParams()
    if cam_type == scene.CAMERA_LONLAT:
        image, vsp, vis, radii = RD.render_lonlat(_viewpoint(cam, "cuda"), H, W, pc, pipe, bg)
        tanfov = (0.0, 0.0)
    else:
        fovx, fovy = 2 * np.arctan(cam.tanfovx), 2 * np.arctan(cam.tanfovy)
        image, vsp, vis, radii = RD.render(_viewpoint(cam, "cuda", fovx, fovy), H, W, pc, pipe, bg)
        tanfov = (float(np.tan(np.float32(fovx) * np.float32(0.5))), float(np.tan(np.float32(fovy) * np.float32(0.5))))
    assert image.shape == (3, H, W) and vsp.shape == (g.P, 3) and radii.shape == (g.P,)
    assert torch.equal(vis, radii > 0)
    (image * torch.from_numpy(dL).cuda()).sum().backward()
    torch.cuda.synchronize()

    act = _activated(pc)
    cam_o = types.SimpleNamespace(**{k: getattr(cam, k) for k in ("viewmatrix", "projmatrix", "campos", "width",
                                                                   "height", "camera_type")},
                                  tanfovx=tanfov[0], tanfovy=tanfov[1])
    o, L, og = oracle_run(act, cam_o, dL, bg=(0.1, 0.2, 0.3))
    assert np.abs(to_np(image) - o.get("out_color").reshape(3, H, W)).max() <= 1e-4
    # Gaussians surround the camera: the 360° view sees most, the 90° pinhole about a sixth
    assert vis.sum().item() > (0.3 if cam_type == scene.CAMERA_LONLAT else 0.1) * g.P
    ok, emax, nbad = grad_close(to_np(vsp.grad), og["dmean2D"])
    assert ok, ("viewspace_points", emax, nbad)
    want = _chain_to_raw(pc, og)
    for name, ref in want.items():
        got = to_np(getattr(pc, name).grad)
        ok, emax, nbad = grad_close(got, np.asarray(ref).reshape(got.shape))
        assert ok, (name, emax, nbad)


def test_render_lonlat_convert_shs_and_cov3D_paths_agree():
    """pipe.convert_SHs (torch eval_sh) and pipe.compute_cov3D (torch covariance) reach the same image and grads as
    the in-kernel SH / covariance path (gaussian_renderer.cpp:225-256)."""
    W, H = 128, 64
    g, cam, dL = make_case(800, W, H, scene.CAMERA_LONLAT, 91, spread=3.0)
    dl = torch.from_numpy(dL).cuda()
    bg = torch.zeros(3, device="cuda")
    outs = {}
    for key, pipe in [("kernel", RD.PipelineParams()), ("sh", RD.PipelineParams(convert_SHs=True)),
                      ("cov", RD.PipelineParams(compute_cov3D=True))]:
        pc = _raw_params(g, "cuda", 5)
        image, vsp, vis, radii = RD.render_lonlat(_viewpoint(cam, "cuda"), H, W, pc, pipe, bg)
        (image * dl).sum().backward()
        outs[key] = (to_np(image), {n: to_np(p.grad) for n, p in
                                    zip(["xyz", "dc", "rest", "opacity", "scaling", "rotation"], pc.parameters())},
                     to_np(radii))
    img0, g0, r0 = outs["kernel"]
    for key in ("sh", "cov"):
        img, gr, r = outs[key]
        assert np.array_equal(r, r0), key
        assert np.abs(img - img0).max() <= 1e-4, key
        for n in g0:
            ok, emax, nbad = grad_close(gr[n], g0[n], rtol=2e-3, atol_frac=2e-4)
            assert ok, (key, n, emax, nbad)


def test_render_override_color():
    W, H = 96, 48
    g, cam, dL = make_case(400, W, H, scene.CAMERA_LONLAT, 13, spread=4.0)
    pc = _raw_params(g, "cuda", 1)
    col = torch.rand(g.P, 3, device="cuda", requires_grad=True)
    image, vsp, vis, radii = RD.render_lonlat(_viewpoint(cam, "cuda"), H, W, pc, RD.PipelineParams(),
                                              torch.zeros(3, device="cuda"), override_color=col)
    (image * torch.from_numpy(dL).cuda()).sum().backward()
    act = _activated(pc)
    o, L, og = oracle_run(act, cam, dL, colors_precomp=to_np(col))
    assert np.abs(to_np(image) - o.get("out_color").reshape(3, H, W)).max() <= 1e-4
    ok, emax, nbad = grad_close(to_np(col.grad), og["dcolor"])
    assert ok, (emax, nbad)
    assert pc.features_dc.grad is None or float(pc.features_dc.grad.abs().max()) == 0.0

"""Host-side renderer glue on the CPU (no GPU): the torch activations and the convert_SHs / compute_cov3D helpers of
renderer.py agree with the oracle's preprocess intermediates (cov3D, rgb) on the same Gaussians."""
import numpy as np
import torch

from helpers import make_case, omr, oracle_run, scene

RD = omr.renderer


def _pc(g):
    t = lambda a: torch.tensor(np.ascontiguousarray(a, dtype=np.float32))
    o = np.clip(g.opacity.astype(np.float64), 1e-6, 1 - 1e-6)
    return RD.GaussianModelParams(t(g.means3D), t(g.shs[:, :1]), t(g.shs[:, 1:]), t(np.log(o / (1 - o))),
                                  t(np.log(g.scales)), t(g.rotations * 1.7), 3, 3)


def test_covariance_activation_matches_oracle_cov3D():
    g, cam, _ = make_case(500, 128, 64, scene.CAMERA_LONLAT, 3, spread=3.0)
    pc = _pc(g)
    g.scales = pc.get_scaling_activation().numpy()
    g.rotations = pc.get_rotation_activation().numpy()
    o, L, _ = oracle_run(g, cam)
    vis = o.get("radii") > 0
    ref = o.get("cov3D").reshape(g.P, 6)[vis]
    got = pc.get_covariance_activation().numpy()[vis]
    assert np.abs(got - ref).max() <= 1e-6 * np.abs(ref).max() + 1e-12
    # reference getCovarianceActivation(int scaling_modifier = 1): the renderer's modifier never reaches it
    assert torch.equal(pc.get_covariance_activation(1), pc.get_covariance_activation())


def test_eval_sh_matches_oracle_rgb():
    g, cam, _ = make_case(500, 128, 64, scene.CAMERA_LONLAT, 4, spread=3.0)
    for deg in (0, 1, 2, 3):
        g.sh_degree = deg
        o, L, _ = oracle_run(g, cam)
        vis = o.get("radii") > 0
        pc = _pc(g)
        pc.active_sh_degree = deg
        feats = pc.get_features()
        shs_view = feats.transpose(1, 2).reshape(-1, 3, 16)
        d = pc.xyz - torch.tensor(cam.campos, dtype=torch.float32).repeat(g.P, 1)
        d = d / d.norm(dim=1, keepdim=True)
        rgb = torch.clamp_min(RD.eval_sh(deg, shs_view, d) + 0.5, 0.0).numpy()
        ref = o.get("rgb").reshape(g.P, 3)
        assert np.abs(rgb[vis] - ref[vis]).max() <= 2e-6, deg


def test_activations_follow_reference():
    g, _, _ = make_case(50, 64, 32, scene.CAMERA_LONLAT, 5)
    pc = _pc(g)
    np.testing.assert_allclose(pc.get_scaling_activation().numpy(), g.scales, rtol=1e-6)
    np.testing.assert_allclose(pc.get_opacity_activation().numpy(), np.clip(g.opacity, 1e-6, 1 - 1e-6), rtol=1e-5)
    np.testing.assert_allclose(pc.get_rotation_activation().numpy(), g.rotations, atol=1e-6)
    assert pc.get_features().shape == (50, 16, 3)

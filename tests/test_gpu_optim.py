"""The training step after the backward on the GPU (csrc/optim.hip through the C ABI), against LibTorch's own Adam
(tests/golden/optim/adam_*.npz, made by make_adam_golden.py) and the CPU oracle (oracle/optim_oracle.py).

Bars: parameters 2e-6 relative (float order and expf/sqrtf ulps differ from LibTorch's CPU kernels); moments 1e-5
relative with a floor of 1e-5 x the group's largest moment (sums of gradients of both signs cancel); everything
densifyAndPrune copies or reorders is bit-exact; the split positions / scalings it computes are 1e-6 relative.
"""
import os
import sys

import numpy as np
import pytest
import torch

from helpers import omr, to_np

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import optim_oracle as OO  # noqa: E402

OPT, RD = omr.optim, omr.renderer
GOLDEN = [os.path.join(ROOT, "tests", "golden", "optim", n) for n in ("adam_deg3_P61.npz", "adam_deg1_P67.npz")]


def _cuda(a, grad=False):
    return torch.tensor(np.ascontiguousarray(a), dtype=torch.float32, device="cuda", requires_grad=grad)


def _model(params, grad=False):
    t = [_cuda(p, grad) for p in params]
    return RD.GaussianModelParams(t[0], t[1], t[2], t[3], t[4], t[5], 3, 3)


def _check(p, m, v, ref_p, ref_m, ref_v, what):
    assert p.shape == ref_p.shape, what
    if ref_p.size == 0:
        return
    np.testing.assert_allclose(p, ref_p, rtol=2e-6, atol=2e-7, err_msg=f"param {what}")
    for name, x, ref in (("exp_avg", m, ref_m), ("exp_avg_sq", v, ref_v)):
        np.testing.assert_allclose(x, ref, rtol=1e-5, atol=1e-5 * max(np.abs(ref).max(), 1e-30),
                                   err_msg=f"{name} {what}")


def _raster_grads(d, s):
    return {"dL_dmeans3D": _cuda(d[f"act_grad{s}_0"]), "dL_dsh": _cuda(d[f"act_grad{s}_1"]),
            "dL_dopacity": _cuda(d[f"act_grad{s}_2"]), "dL_dscales": _cuda(d[f"act_grad{s}_3"]),
            "dL_drotations": _cuda(d[f"act_grad{s}_4"])}


@pytest.mark.parametrize("path", GOLDEN)
@pytest.mark.parametrize("mode", ["raster", "raw"])
def test_adam_matches_libtorch_golden(path, mode):
    """mode raster: the fused activation backward + Adam on the rasterizer's gradients; mode raw: Adam on the raw
    gradients LibTorch's autograd produced (what .grad holds in the reference)."""
    d = np.load(path)
    steps = int(d["steps"])
    model = _model([d[f"param{k}"] for k in range(6)], grad=(mode == "raw"))
    opt = OPT.GaussianOptimizer(model, OPT.OptimizationParams())
    for s in range(steps):
        opt.lr = [float(x) for x in d["lrs"][s]]
        if mode == "raster":
            opt.step(raster_grads=_raster_grads(d, s))
        else:
            for k, p in enumerate(opt.params()):
                p.grad = _cuda(d[f"raw_grad{s}_{k}"])
            opt.step()
            opt.zero_grad()
    torch.cuda.synchronize()
    assert opt.steps == [steps] * 6
    for k, p in enumerate(opt.params()):
        _check(to_np(p), to_np(opt.exp_avg[k]), to_np(opt.exp_avg_sq[k]), d[f"out_param{k}"], d[f"out_exp_avg{k}"],
               d[f"out_exp_avg_sq{k}"], f"group {k}")


def _random_params(P, Mr, seed):
    rng = np.random.default_rng(seed)
    f = np.float32
    return [rng.normal(0, 1, (P, 3)).astype(f), rng.normal(0, 0.5, (P, 1, 3)).astype(f),
            rng.normal(0, 0.2, (P, Mr, 3)).astype(f), rng.normal(0, 2, (P, 1)).astype(f),
            rng.normal(-4, 1.5, (P, 3)).astype(f), rng.normal(0, 1, (P, 4)).astype(f)]


@pytest.mark.parametrize("P,Mr", [(100003, 15), (4097, 3), (777, 0), (1, 8)])
def test_adam_raster_grads_vs_oracle(P, Mr):
    """Sizes with ragged 16-B chunks in every group (3P, 3*Mr*P not multiples of 4), SH degrees 3, 1, 0, 2."""
    rng = np.random.default_rng(P + Mr)
    params = _random_params(P, Mr, P)
    model = _model(params)
    opt = OPT.GaussianOptimizer(model, OPT.OptimizationParams(), spatial_lr_scale=2.5)
    ref = [p.copy() for p in params]
    ms = [np.zeros_like(p) for p in ref]
    vs = [np.zeros_like(p) for p in ref]
    for s in range(3):
        opt.update_learning_rate(1000 * s)
        g = {"dL_dmeans3D": rng.normal(0, 1e-4, (P, 3)), "dL_dsh": rng.normal(0, 1e-4, (P, Mr + 1, 3)),
             "dL_dopacity": rng.normal(0, 1e-3, (P, 1)), "dL_dscales": rng.normal(0, 1e-3, (P, 3)),
             "dL_drotations": rng.normal(0, 1e-4, (P, 4))}
        g = {k: v.astype(np.float32) for k, v in g.items()}
        g["dL_dmeans3D"][rng.random(P) < 0.5] = 0
        opt.step(raster_grads={k: _cuda(v) for k, v in g.items()})
        raw = OO.activation_backward(ref, g)
        for k in range(6):
            OO.adam_step(ref[k], ms[k], vs[k], raw[k], opt.lr[k], s + 1)
    torch.cuda.synchronize()
    for k, p in enumerate(opt.params()):
        _check(to_np(p), to_np(opt.exp_avg[k]), to_np(opt.exp_avg_sq[k]), ref[k], ms[k], vs[k], f"group {k}")


def test_adam_skips_groups_without_grad():
    params = _random_params(1000, 15, 3)
    model = _model(params, grad=True)
    opt = OPT.GaussianOptimizer(model, OPT.OptimizationParams())
    model.opacity.grad = torch.full_like(model.opacity, 1e-3)
    opt.step()
    torch.cuda.synchronize()
    assert opt.steps == [0, 0, 0, 1, 0, 0]
    for k, p in enumerate(opt.params()):
        if k == 3:
            assert not np.array_equal(to_np(p), params[k])
        else:
            np.testing.assert_array_equal(to_np(p), params[k])
            assert not to_np(opt.exp_avg[k]).any()


def test_adam_rejects_misaligned_and_bad_shapes():
    params = _random_params(64, 15, 4)
    model = _model(params)
    opt = OPT.GaussianOptimizer(model, OPT.OptimizationParams())
    bad = torch.zeros(64 * 3 + 1, device="cuda")[1:].view(64, 3)  # 4-byte offset
    g = {"dL_dmeans3D": bad, "dL_dsh": torch.zeros(64, 16, 3, device="cuda"), "dL_dopacity": torch.zeros(64, 1, device="cuda"),
         "dL_dscales": torch.zeros(64, 3, device="cuda"), "dL_drotations": torch.zeros(64, 4, device="cuda")}
    with pytest.raises(omr.rasterizer.RasterizerError, match="aligned"):
        opt.step(raster_grads=g)
    g["dL_dmeans3D"] = torch.zeros(64, 3, device="cuda")
    g["dL_dsh"] = torch.zeros(64, 4, 3, device="cuda")
    with pytest.raises(omr.rasterizer.RasterizerError, match="dL_dsh"):
        opt.step(raster_grads=g)


def test_densification_stats_vs_oracle():
    P = 50001
    rng = np.random.default_rng(5)
    model = _model(_random_params(P, 15, 5))
    opt = OPT.GaussianOptimizer(model, OPT.OptimizationParams())
    accum, denom, mr = np.zeros((P, 1), np.float32), np.zeros((P, 1), np.float32), np.zeros(P, np.float32)
    for s in range(3):
        radii = rng.integers(-2, 30, P).astype(np.int32)
        vg = rng.normal(0, 1e-3, (P, 3)).astype(np.float32)
        opt.add_densification_stats(_cuda(vg), torch.tensor(radii, device="cuda"))
        OO.densification_stats(radii, vg, accum, denom, mr)
    torch.cuda.synchronize()
    np.testing.assert_allclose(to_np(opt.xyz_gradient_accum), accum, rtol=1e-6)
    np.testing.assert_array_equal(to_np(opt.denom), denom)
    np.testing.assert_array_equal(to_np(opt.max_radii2D), mr)


def _densify_case(P, Mr, seed, max_grad, min_op, extent, max_screen, by_ext):
    rng = np.random.default_rng(seed)
    params = _random_params(P, Mr, seed)
    model = _model(params)
    opt = OPT.GaussianOptimizer(model, OPT.OptimizationParams())
    ea = [rng.random(p.shape).astype(np.float32) for p in params]
    es = [rng.random(p.shape).astype(np.float32) for p in params]
    accum = (rng.random((P, 1)) * 4e-3).astype(np.float32)
    denom = rng.integers(0, 5, (P, 1)).astype(np.float32)
    accum[denom == 0] = 0
    exist = rng.integers(0, 1000, P).astype(np.int32)
    mr = (rng.random(P) * 40).astype(np.float32)
    opt.exp_avg = [_cuda(a) for a in ea]
    opt.exp_avg_sq = [_cuda(a) for a in es]
    opt.xyz_gradient_accum, opt.denom, opt.max_radii2D = _cuda(accum), _cuda(denom), _cuda(mr)
    opt.exist_since_iter = torch.tensor(exist, device="cuda")
    ref = OO.ModelState(params, ea, es, exist, accum, denom, mr)
    normals = rng.normal(size=(2 * P, 3)).astype(np.float32)
    info = opt.densify_and_prune(max_grad, min_op, extent, max_screen, by_ext, normals=_cuda(normals))
    S = ref.densify_and_prune(max_grad, min_op, extent, max_screen, by_ext, 0.01, normals)
    torch.cuda.synchronize()
    return opt, ref, info, S


@pytest.mark.parametrize("P,Mr,max_screen,by_ext,extent", [(30001, 15, 20, True, 5.0), (5000, 3, 0, True, 5.0),
                                                           (5000, 15, 20, False, 5.0), (4099, 0, 20, True, 0.3)])
def test_densify_and_prune_vs_oracle(P, Mr, max_screen, by_ext, extent):
    opt, ref, info, S = _densify_case(P, Mr, 7 + P, 2e-4, 0.005, extent, max_screen, by_ext)
    assert info["splits_selected"] == S
    assert info["P_new"] == ref.P == opt.P
    assert info["clones"] > 0 and S > 0
    np.testing.assert_array_equal(to_np(opt.exist_since_iter), ref.exist)
    n_fixed = ref.P - 2 * info["splits_kept"]  # kept originals + clones: pure copies
    for k, p in enumerate(opt.params()):
        got, want = to_np(p), ref.params[k]
        assert got.shape == want.shape, k
        if k in (0, 4):  # split copies: positions and scalings are computed
            np.testing.assert_array_equal(got[:n_fixed], want[:n_fixed])
            np.testing.assert_allclose(got[n_fixed:], want[n_fixed:], rtol=1e-6, atol=1e-6)
        else:
            np.testing.assert_array_equal(got, want)
        np.testing.assert_array_equal(to_np(opt.exp_avg[k]), ref.exp_avg[k])
        np.testing.assert_array_equal(to_np(opt.exp_avg_sq[k]), ref.exp_avg_sq[k])
    for t in (opt.xyz_gradient_accum, opt.denom, opt.max_radii2D):
        assert t.shape[0] == ref.P and not t.any()


def test_densify_nothing_selected_and_all_pruned():
    opt, ref, info, S = _densify_case(2000, 15, 3, 1e9, 0.0, 5.0, 0, True)  # nothing to do
    assert info == {"P_new": 2000, "clones": 0, "splits_selected": 0, "splits_kept": 0}
    np.testing.assert_array_equal(to_np(opt.exist_since_iter), ref.exist)
    opt, ref, info, S = _densify_case(2000, 15, 3, 2e-4, 1.1, 5.0, 0, True)  # every opacity < 1.1: all pruned
    assert info["P_new"] == 0 == ref.P and opt.P == 0


@pytest.mark.parametrize("ceiling", [1.0, 0.01])
def test_reset_opacity_vs_oracle(ceiling):
    P = 10000
    params = _random_params(P, 15, 9)
    model = _model(params)
    opt = OPT.GaussianOptimizer(model, OPT.OptimizationParams())
    opt.exp_avg[3].fill_(1.0)
    opt.exp_avg_sq[3].fill_(1.0)
    opt.reset_opacity(ceiling)
    o, m, v = params[3].copy(), np.ones_like(params[3]), np.ones_like(params[3])
    OO.reset_opacity(o, m, v, ceiling)
    torch.cuda.synchronize()
    np.testing.assert_allclose(to_np(model.opacity), o, rtol=1e-5, atol=1e-5)
    assert not opt.exp_avg[3].any() and not opt.exp_avg_sq[3].any()


@pytest.mark.parametrize("masked,skip_bottom_ratio", [(False, 0.0), (True, 0.063)],
                         ids=["plain", "mask_skip_bottom"])
def test_fused_train_step_matches_autograd_reference_composition(masked, skip_bottom_ratio):
    """trainer.train_step (no autograd: fused loss, rasterizer backward, fused activation backward + Adam) reaches
    the same parameters as the reference's composition: torch activations -> rasterizer autograd -> masked image,
    optional bottom crop, l1/ssim loss in torch (gaussian_mapper.cpp:387-413, loss_utils.h; oracle/loss_oracle.py)
    -> loss.backward() -> Adam on .grad (raw mode). 0.063 is the skip_bottom_ratio of the reference's
    cfg/lonlat/360roam_lonlat.yaml (8 of 128 rows here)."""
    import loss_oracle as LO
    from helpers import make_case, scene

    W, H = 256, 128
    g, cam, _ = make_case(3000, W, H, scene.CAMERA_LONLAT, 21, spread=2.0)
    rng = np.random.default_rng(1)
    o = np.clip(g.opacity.astype(np.float64), 1e-4, 1 - 1e-4)
    params = [g.means3D, g.shs[:, :1], g.shs[:, 1:], np.log(o / (1 - o)), np.log(g.scales),
              g.rotations * rng.uniform(0.5, 2.0, (g.P, 1))]
    params = [np.ascontiguousarray(p, dtype=np.float32) for p in params]
    gt = torch.tensor(rng.random((3, H, W)), dtype=torch.float32, device="cuda")
    mask = None
    if masked:  # an undistortion mask: black border columns, the rest 1 (gaussian_mapper.cpp:389)
        mask = torch.ones((1, H, W), device="cuda")
        mask[:, :, :9] = 0.0
        mask[:, :, W - 7:] = 0.0
    bg = torch.zeros(3, device="cuda")
    t = lambda a: torch.tensor(np.ascontiguousarray(a, dtype=np.float32), device="cuda")  # noqa: E731
    vp = RD.Viewpoint(t(cam.viewmatrix), t(cam.projmatrix), t(cam.campos))
    args = OPT.OptimizationParams()

    # fused
    m1 = _model(params)
    opt1 = OPT.GaussianOptimizer(m1, args)
    state = omr.trainer.TrainStep()
    # reference composition
    m2 = _model(params, grad=True)
    opt2 = OPT.GaussianOptimizer(m2, args)
    for it in range(3):
        for opt in (opt1, opt2):
            opt.update_learning_rate(it)
        terms, img1, radii1 = omr.trainer.train_step(opt1, vp, H, W, gt, bg, lambda_dssim=0.2, state=state,
                                                     mask=mask, skip_bottom_ratio=skip_bottom_ratio)
        img2, vsp, vis, radii2 = RD.render_lonlat(vp, H, W, m2, RD.PipelineParams(), bg)
        loss = LO.training_loss(img2, gt, 0.2, mask=mask, skip_bottom_ratio=skip_bottom_ratio)
        loss.backward()
        opt2.add_densification_stats(vsp.grad, radii2)
        opt2.step()
        opt2.zero_grad()
        torch.cuda.synchronize()
        assert abs(float(terms[0]) - float(loss.detach())) <= 1e-5 * abs(float(loss.detach())) + 1e-7
        assert torch.equal(radii1, radii2)
    for k, (p1, p2) in enumerate(zip(opt1.params(), opt2.params())):
        # the two paths take different float routes to the same gradient. Adam (eps 1e-15) normalises magnitudes, so
        # an element whose gradient is at rounding-noise level may move by +-lr either way: compare the parameter
        # moves and allow such elements to be rare
        d1, d2 = to_np(p1) - params[k], to_np(p2) - params[k]
        bad = np.abs(d1 - d2) > 2e-3 * np.abs(d2).max() + 1e-9
        assert bad.mean() <= 1e-3, (k, int(bad.sum()), d1.size)
    np.testing.assert_allclose(to_np(opt1.xyz_gradient_accum), to_np(opt2.xyz_gradient_accum), rtol=2e-3,
                               atol=1e-3 * float(opt2.xyz_gradient_accum.abs().max()))
    np.testing.assert_array_equal(to_np(opt1.denom), to_np(opt2.denom))


@pytest.mark.parametrize("P,cam,deg", [(5000, "lonlat", 3), (4999, "pinhole", 3), (1023, "pinhole", 1),
                                       (6, "lonlat", 0)])
def test_activate_matches_the_torch_activations(P, cam, deg):
    """omr_activate (optim.hip: activate_kernel) against gaussian_model.cpp:54-77's torch expressions: the SH
    concatenation, sigmoid and exp bit for bit; normalize within an ulp of torch's (its norm reduction may sum the
    four squares in another order). Lonlat and pinhole scenes, P not a multiple of 4 (ragged 16-B SH chunks), SH
    degrees 3 / 1 / 0."""
    from helpers import make_case, scene

    g, _, _ = make_case(P, 64, 32, scene.CAMERA_LONLAT if cam == "lonlat" else scene.CAMERA_PINHOLE, 31 + P)
    rng = np.random.default_rng(2)
    o = np.clip(g.opacity.astype(np.float64), 1e-4, 1 - 1e-4)
    nsh = (deg + 1) ** 2
    params = [g.means3D, g.shs[:, :1], g.shs[:, 1:nsh], np.log(o / (1 - o)), np.log(g.scales),
              g.rotations * rng.uniform(0.5, 2.0, (g.P, 1))]
    m = _model([np.ascontiguousarray(p, dtype=np.float32) for p in params])
    opt = OPT.GaussianOptimizer(m, OPT.OptimizationParams())
    act = opt.activate()
    again = opt.activate(act)  # reuses the buffers
    assert all(again[k] is act[k] for k in ("shs", "opacity", "scales", "rotations"))
    torch.cuda.synchronize()
    assert act["xyz"] is m.xyz
    assert torch.equal(act["shs"], torch.cat([m.features_dc, m.features_rest], dim=1))
    assert torch.equal(act["opacity"], torch.sigmoid(m.opacity))
    assert torch.equal(act["scales"], torch.exp(m.scaling))
    ref = torch.nn.functional.normalize(m.rotation)
    torch.testing.assert_close(act["rotations"], ref, rtol=2.4e-7, atol=0)



@pytest.mark.parametrize("P,Mr", [(100003, 15), (4097, 3), (777, 0), (1, 8)])
def test_adam_step_activate_equals_step_then_activate(P, Mr):
    """omr_adam_step_activate (trainer.train_step's Adam launch) writes exactly omr_activate's outputs of the updated
    parameters, and updates parameters and moments exactly as omr_adam_step does; activate_cached then reuses them
    and recomputes after the parameters change outside Adam (a torch in-place op, resetOpacity, densification)."""
    rng = np.random.default_rng(P + 7 * Mr)
    params = _random_params(P, Mr, P + 1)
    opt1 = OPT.GaussianOptimizer(_model(params), OPT.OptimizationParams())
    opt2 = OPT.GaussianOptimizer(_model(params), OPT.OptimizationParams())
    act1 = {}
    for s in range(2):
        g = {"dL_dmeans3D": rng.normal(0, 1e-4, (P, 3)), "dL_dsh": rng.normal(0, 1e-4, (P, Mr + 1, 3)),
             "dL_dopacity": rng.normal(0, 1e-3, (P, 1)), "dL_dscales": rng.normal(0, 1e-3, (P, 3)),
             "dL_drotations": rng.normal(0, 1e-4, (P, 4))}
        g = {k: _cuda(v) for k, v in g.items()}
        opt1.step(raster_grads=g, act_out=act1)
        opt2.step(raster_grads=g)
    act2 = opt2.activate()
    torch.cuda.synchronize()
    for k in range(6):
        for a, b in ((opt1.params()[k], opt2.params()[k]), (opt1.exp_avg[k], opt2.exp_avg[k]),
                     (opt1.exp_avg_sq[k], opt2.exp_avg_sq[k])):
            assert torch.equal(a, b), k
    for k in ("shs", "opacity", "scales", "rotations"):
        assert torch.equal(act1[k], act2[k]), k
    assert act1["xyz"] is opt1.model.xyz

    # cached: the same tensors, untouched (a launch would rewrite the same bits: poison them to see it does not run)
    act1["opacity"].fill_(-1.0)
    again = opt1.activate_cached(act1)
    torch.cuda.synchronize()
    assert again is act1 and bool((act1["opacity"] == -1.0).all())
    # a torch in-place op on a parameter: recomputed
    opt1.model.opacity.add_(0.5)
    opt1.activate_cached(act1)
    torch.cuda.synchronize()
    assert torch.equal(act1["opacity"], torch.sigmoid(opt1.model.opacity))
    # resetOpacity (a raw-pointer write): recomputed
    opt1.reset_opacity(0.01)
    act1["opacity"].fill_(-1.0)
    opt1.activate_cached(act1)
    torch.cuda.synchronize()
    assert torch.equal(act1["opacity"], torch.sigmoid(opt1.model.opacity))
    # a parameter replaced by a NEW tensor (same shape, version 0, possibly the freed block's address): recomputed
    opt1.model.opacity = opt1.model.opacity.detach().clone() + 0.25
    act1["opacity"].fill_(-1.0)
    opt1.activate_cached(act1)
    torch.cuda.synchronize()
    assert torch.equal(act1["opacity"], torch.sigmoid(opt1.model.opacity))
    # a write torch does not version (through .data): invisible to the key, so invalidate() is the contract
    v0 = opt1.model.scaling._version
    opt1.model.scaling.data.copy_(opt1.model.scaling.data * 0.5)
    assert opt1.model.scaling._version == v0
    opt1.invalidate()
    act1["scales"].fill_(-1.0)
    opt1.activate_cached(act1)
    torch.cuda.synchronize()
    assert torch.equal(act1["scales"], torch.exp(opt1.model.scaling))


@pytest.mark.parametrize("P,Mr", [(4099, 15), (513, 3)])
def test_adam_step_activate_without_the_sh_row_walk(P, Mr):
    """omr_debug_adam_sh_rows(0) (OMR_ADAM_SH_ROWS=0, the A/B switch): f_dc and f_rest step as two gathering groups and
    the activated SH array is copied after the launch. Same bits as the row walk, and train steps still run (ADVICE
    r05: the switch used to make every omr_adam_step_activate with SH outputs fail)."""
    rng = np.random.default_rng(P)
    params = _random_params(P, Mr, P + 3)
    opts = [OPT.GaussianOptimizer(_model(params), OPT.OptimizationParams()) for _ in range(2)]
    acts = [{}, {}]
    old = omr.rasterizer.debug_adam_sh_rows(1)
    try:
        for s in range(2):
            g = {"dL_dmeans3D": rng.normal(0, 1e-4, (P, 3)), "dL_dsh": rng.normal(0, 1e-4, (P, Mr + 1, 3)),
                 "dL_dopacity": rng.normal(0, 1e-3, (P, 1)), "dL_dscales": rng.normal(0, 1e-3, (P, 3)),
                 "dL_drotations": rng.normal(0, 1e-4, (P, 4))}
            g = {k: _cuda(v) for k, v in g.items()}
            for k, (opt, act) in enumerate(zip(opts, acts)):
                omr.rasterizer.debug_adam_sh_rows(1 - k)
                opt.step(raster_grads=g, act_out=act)
        torch.cuda.synchronize()
    finally:
        omr.rasterizer.debug_adam_sh_rows(old)
    for k in range(6):
        assert torch.equal(opts[0].params()[k], opts[1].params()[k]), k
        assert torch.equal(opts[0].exp_avg_sq[k], opts[1].exp_avg_sq[k]), k
    for k in ("shs", "opacity", "scales", "rotations"):
        assert torch.equal(acts[0][k], acts[1][k]), k
    m = opts[1].model
    assert torch.equal(acts[1]["shs"], torch.cat([m.features_dc, m.features_rest], dim=1))
    with pytest.raises(omr.rasterizer.RasterizerError):
        omr.rasterizer.debug_adam_sh_rows(2)


def test_adam_step_activate_rejects_outputs_of_groups_that_do_not_step():
    params = _random_params(64, 15, 5)
    opt = OPT.GaussianOptimizer(_model(params), OPT.OptimizationParams())
    L = omr.rasterizer.lib()
    import ctypes as C
    out = opt._act_buffers({})
    g = [torch.zeros_like(p) for p in opt.params()]
    g[1] = g[2] = torch.zeros((64, 16, 3), device="cuda")
    g[3] = None  # opacity does not step: its activated output would be stale
    lr = (C.c_float * 6)(*opt.lr)
    st = (C.c_int64 * 6)(*[1] * 6)
    rc = L.omr_adam_step_activate(64, 15, OPT._p6(opt.params()), OPT._p6(opt.exp_avg), OPT._p6(opt.exp_avg_sq),
                                  OPT._p6(g), lr, st, 0.9, 0.999, 1e-15, out["shs"].data_ptr(),
                                  out["opacity"].data_ptr(), out["scales"].data_ptr(), out["rotations"].data_ptr(),
                                  None, None, 0, None, None, None, omr.rasterizer._stream(torch.device("cuda")))
    assert rc != 0
    assert "does not step" in L.omr_last_error().decode()


def test_adam_step_with_densification_stats_equals_the_separate_call():
    """step(..., densify_stats=(dL_dmeans2D, radii)) (the statistics as extra blocks of the Adam launch) updates
    xyz_gradient_accum / denom / max_radii2D bit for bit as add_densification_stats, and Adam as without them."""
    P, Mr = 70001, 15
    rng = np.random.default_rng(9)
    params = _random_params(P, Mr, 12)
    opt1 = OPT.GaussianOptimizer(_model(params), OPT.OptimizationParams())
    opt2 = OPT.GaussianOptimizer(_model(params), OPT.OptimizationParams())
    act1, act2 = {}, {}
    for s in range(2):
        g = {"dL_dmeans3D": rng.normal(0, 1e-4, (P, 3)), "dL_dsh": rng.normal(0, 1e-4, (P, Mr + 1, 3)),
             "dL_dopacity": rng.normal(0, 1e-3, (P, 1)), "dL_dscales": rng.normal(0, 1e-3, (P, 3)),
             "dL_drotations": rng.normal(0, 1e-4, (P, 4))}
        g = {k: _cuda(v) for k, v in g.items()}
        vgrad = _cuda(rng.normal(0, 1e-3, (P, 3)))
        radii = torch.tensor(rng.integers(-1, 40, P), dtype=torch.int32, device="cuda")
        opt1.step(raster_grads=g, act_out=act1, densify_stats=(vgrad, radii))
        opt2.add_densification_stats(vgrad, radii)
        opt2.step(raster_grads=g, act_out=act2)
    torch.cuda.synchronize()
    for a, b in ((opt1.xyz_gradient_accum, opt2.xyz_gradient_accum), (opt1.denom, opt2.denom),
                 (opt1.max_radii2D, opt2.max_radii2D)):
        assert torch.equal(a, b)
    for k in range(6):
        assert torch.equal(opt1.params()[k], opt2.params()[k]), k
    with pytest.raises(omr.rasterizer.RasterizerError, match="act_out"):
        opt1.step(raster_grads=g, densify_stats=(vgrad, radii))

"""The optimizer / densification oracle (oracle/optim_oracle.py) on CPU.

* Pinned to LibTorch: the oracle's activation backward + Adam reproduce the fixtures that LibTorch's own C++ Adam and
  autograd produced (tests/golden/make_adam_golden.py), step by step.
* expon_lr follows exponLrFunc (gaussian_model.cpp:1140-1152).
* densify_and_prune: structural checks of the reference's clone -> split -> prune sequence (parity unpinned: no run
  of the reference is possible here).
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import optim_oracle as O  # noqa: E402

GOLDEN = [os.path.join(ROOT, "tests", "golden", "optim", n) for n in ("adam_deg3_P61.npz", "adam_deg1_P67.npz")]


def load_golden(path):
    d = np.load(path)
    steps = int(d["steps"])
    return d, steps


def act_dict(d, s):
    return {"dL_dmeans3D": d[f"act_grad{s}_0"], "dL_dsh": d[f"act_grad{s}_1"], "dL_dopacity": d[f"act_grad{s}_2"],
            "dL_dscales": d[f"act_grad{s}_3"], "dL_drotations": d[f"act_grad{s}_4"]}


@pytest.mark.parametrize("path", GOLDEN)
def test_activation_backward_matches_libtorch_autograd(path):
    d, steps = load_golden(path)
    params = [d[f"param{k}"].copy() for k in range(6)]
    ms = [np.zeros_like(p) for p in params]
    vs = [np.zeros_like(p) for p in params]
    for s in range(steps):
        raw = O.activation_backward(params, act_dict(d, s))
        for k in range(6):
            ref = d[f"raw_grad{s}_{k}"]  # normalize's backward cancels: floor at 1e-5 of the group's scale
            np.testing.assert_allclose(raw[k], ref, rtol=2e-6, atol=1e-5 * np.abs(ref).max(), err_msg=f"step {s} group {k}")
        for k in range(6):
            O.adam_step(params[k], ms[k], vs[k], d[f"raw_grad{s}_{k}"], float(d["lrs"][s, k]), s + 1)


@pytest.mark.parametrize("path", GOLDEN)
def test_adam_matches_libtorch(path):
    """Adam on LibTorch's own raw gradients reproduces LibTorch's parameters and moments."""
    d, steps = load_golden(path)
    params = [d[f"param{k}"].copy() for k in range(6)]
    ms = [np.zeros_like(p) for p in params]
    vs = [np.zeros_like(p) for p in params]
    for s in range(steps):
        for k in range(6):
            O.adam_step(params[k], ms[k], vs[k], d[f"raw_grad{s}_{k}"], float(d["lrs"][s, k]), s + 1)
    for k in range(6):
        check_state(params[k], ms[k], vs[k], d, k)


def check_state(p, m, v, d, k):
    """Bars vs LibTorch: parameters 1e-6 relative; moments 1e-5 relative with a floor at 1e-5 of the group's
    largest moment (a moment that sums gradients of both signs cancels)."""
    np.testing.assert_allclose(p, d[f"out_param{k}"], rtol=1e-6, atol=1e-7, err_msg=f"param {k}")
    for name, x in (("exp_avg", m), ("exp_avg_sq", v)):
        ref = d[f"out_{name}{k}"]
        np.testing.assert_allclose(x, ref, rtol=1e-5, atol=1e-5 * np.abs(ref).max(), err_msg=f"{name} {k}")


def test_adam_zero_gradient_still_moves_with_eps_1e15():
    """Invisible Gaussians (zero gradient this step) keep moving on their first moment, as in LibTorch."""
    p, m, v = np.ones(4, np.float32), np.full(4, 1e-3, np.float32), np.full(4, 1e-6, np.float32)
    O.adam_step(p, m, v, np.zeros(4, np.float32), 0.01, 5)
    assert np.all(p < 1)


def test_expon_lr():
    sys.path[:0] = [ROOT]
    import _omnigs

    opt = _omnigs.load().optim
    f = np.float32
    # endpoints and midpoint of the log-linear schedule (position_lr_* of cfg/lonlat/360roam_lonlat.yaml)
    assert opt.expon_lr(0, 1.6e-4, 1.6e-6, 0, 0.01, 30000) == pytest.approx(1.6e-4, rel=1e-6)
    assert opt.expon_lr(30000, 1.6e-4, 1.6e-6, 0, 0.01, 30000) == pytest.approx(1.6e-6, rel=1e-5)
    assert opt.expon_lr(60000, 1.6e-4, 1.6e-6, 0, 0.01, 30000) == pytest.approx(1.6e-6, rel=1e-5)
    assert opt.expon_lr(15000, 1.6e-4, 1.6e-6, 0, 0.01, 30000) == pytest.approx(1.6e-5, rel=1e-5)
    assert opt.expon_lr(-1, 1.6e-4, 1.6e-6) == 0.0
    assert opt.expon_lr(10, 0.0, 0.0) == 0.0
    # delay branch: sin ramp from lr_delay_mult
    v = opt.expon_lr(0, 1.0, 1.0, 100, 0.01, 1000)
    assert v == pytest.approx(0.01, rel=1e-6)
    assert opt.expon_lr(50, 1.0, 1.0, 100, 0.01, 1000) == pytest.approx(float(f(0.01) + f(0.99) * np.sin(f(np.pi / 4))),
                                                                     rel=1e-6)


def _model(P, Mr, seed):
    rng = np.random.default_rng(seed)
    f = np.float32
    params = [rng.normal(0, 1, (P, 3)).astype(f), rng.normal(0, 0.5, (P, 1, 3)).astype(f),
              rng.normal(0, 0.2, (P, Mr, 3)).astype(f), rng.normal(0, 2, (P, 1)).astype(f),
              rng.normal(-4, 1.5, (P, 3)).astype(f), rng.normal(0, 1, (P, 4)).astype(f)]
    ea = [rng.random(p.shape).astype(f) for p in params]
    es = [rng.random(p.shape).astype(f) for p in params]
    accum = (rng.random(P) * 4e-3).astype(f)
    denom = rng.integers(0, 5, P).astype(f)
    accum[denom == 0] = 0
    return O.ModelState(params, ea, es, np.arange(P, dtype=np.int32), accum, denom, rng.random(P).astype(f) * 40)


def test_densify_sequence_structure():
    st = _model(500, 15, 3)
    src = _model(500, 15, 3)
    rng = np.random.default_rng(9)
    normals = rng.normal(size=(2 * 500, 3)).astype(np.float32)
    S = st.densify_and_prune(2e-4, 0.005, 5.0, 20, True, 0.01, normals)
    with np.errstate(invalid="ignore", divide="ignore"):
        grads = np.nan_to_num(src.accum[:, 0] / src.denom[:, 0])
    maxs = np.exp(src.params[4]).max(1)
    clone = (grads >= 2e-4) & (maxs <= 0.05)
    split = (grads >= 2e-4) & (maxs > 0.05)
    assert S == split.sum() and S > 0 and clone.sum() > 0
    # statistics reset, moments of new points zero, exist_since_iter carried
    assert not st.accum.any() and not st.denom.any() and not st.max_radii.any()
    # originals first (index order, own parameters and moments), then the unpruned clones with zero moments
    ok = (O._sigmoid(src.params[3])[:, 0] >= np.float32(0.005)) & ~(maxs > np.float32(0.5))
    orig = np.nonzero(~split & ok)[0]
    clones = np.nonzero(clone & ok)[0]
    np.testing.assert_array_equal(st.exist[: len(orig)], orig)
    np.testing.assert_array_equal(st.exist[len(orig): len(orig) + len(clones)], clones)
    for k in range(6):
        np.testing.assert_array_equal(st.params[k][: len(orig)], src.params[k][orig])
        np.testing.assert_array_equal(st.exp_avg[k][: len(orig)], src.exp_avg[k][orig])
        np.testing.assert_array_equal(st.params[k][len(orig): len(orig) + len(clones)], src.params[k][clones])
        assert not st.exp_avg[k][len(orig):].any() and not st.exp_avg_sq[k][len(orig):].any()
    rest = st.exist[len(orig) + len(clones):]
    assert len(rest) % 2 == 0 and np.isin(rest, np.nonzero(split)[0]).all()
    np.testing.assert_array_equal(rest[: len(rest) // 2], rest[len(rest) // 2:])
    # every surviving point passes the opacity test
    assert (O._sigmoid(st.params[3]) >= np.float32(0.005)).all()


def test_reset_opacity_reference_bound_is_one():
    o = np.array([[-5.0], [0.0], [4.0]], np.float32)
    m, v = np.ones_like(o), np.ones_like(o)
    o2 = o.copy()
    O.reset_opacity(o2, m, v)  # ones_like(...) bound: value round-trips, moments reset
    np.testing.assert_allclose(o2, o, atol=1e-5)
    assert not m.any() and not v.any()
    o3 = o.copy()
    O.reset_opacity(o3, m, v, ceiling=0.01)
    np.testing.assert_allclose(o3[1:], np.log(np.float32(0.01) / np.float32(0.99)), rtol=1e-5)
    np.testing.assert_allclose(o3[0], o[0], atol=1e-5)


def test_optimizer_host_rejects_cpu_tensors():
    sys.path[:0] = [ROOT]
    import torch

    import _omnigs

    omr = _omnigs.load()
    m = omr.renderer.GaussianModelParams(torch.zeros(4, 3), torch.zeros(4, 1, 3), torch.zeros(4, 15, 3),
                                         torch.zeros(4, 1), torch.zeros(4, 3), torch.zeros(4, 4))
    with pytest.raises(omr.rasterizer.RasterizerError, match="HIP device"):
        omr.optim.GaussianOptimizer(m, omr.optim.OptimizationParams())

"""Golden fixtures (tests/golden/*.npz, made by tests/golden/make_golden.py from the validated oracle):

* CPU: the scene generator still produces the fixture's inputs (SHA-256) and the oracle still reproduces every
  stored intermediate / output / gradient (integers exactly, floats to 1e-6) — guards both against drift;
* GPU (marked gpu): the HIP path through the C ABI against the fixtures, with the parity bar of
  test_gpu_parity.py (bit-exact integers and geometry, 1e-4 colour, gradient tolerance of helpers.grad_close).
"""
import glob
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FILES = sorted(glob.glob(os.path.join(GOLDEN, "*.npz")))
NAMES = [os.path.basename(f)[:-4] for f in FILES]
INT_KEYS = ["radii", "tiles_touched", "point_list", "ranges", "n_contrib"]
GEOM_KEYS = ["means2D", "conic_opacity", "depths"]
GRAD_KEYS = ["dL_dmeans2D", "dL_dcolors", "dL_dopacity", "dL_dmeans3D", "dL_dcov3D", "dL_dsh", "dL_dscales",
             "dL_drotations"]


def _load(name):
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def test_fixtures_present():
    assert len(FILES) >= 4


@pytest.mark.parametrize("name", NAMES)
def test_oracle_reproduces_fixture(name, oracle_mod):
    import make_golden as MG

    fx = _load(name)
    g, cam, dL, bg = MG.inputs_of(name)
    assert MG.input_digest(g, cam, dL, bg) == str(fx["input_sha256"])
    now = MG.compute(name)
    assert int(now["num_rendered"]) == int(fx["num_rendered"])
    for k in INT_KEYS:
        np.testing.assert_array_equal(now[k], fx[k], err_msg=k)
    for k in GEOM_KEYS + ["out_color", "final_T"] + GRAD_KEYS:
        np.testing.assert_allclose(now[k], fx[k], rtol=1e-6, atol=1e-7, err_msg=k)


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_hip_matches_fixture(name):
    import make_golden as MG
    from helpers import grad_close, hip_run, to_np

    fx = _load(name)
    g, cam, dL, bg = MG.inputs_of(name)
    h = hip_run(g, cam, dL, bg=tuple(float(x) for x in bg))
    st = {k: to_np(v) for k, v in h["state"].items()}
    assert h["L"] == int(fx["num_rendered"])
    np.testing.assert_array_equal(to_np(h["radii"]), fx["radii"])
    vis = fx["radii"] > 0
    np.testing.assert_array_equal(st["tiles_touched"].astype(np.uint32), fx["tiles_touched"])
    for k in GEOM_KEYS:
        np.testing.assert_array_equal(st[k][vis], fx[k][vis], err_msg=k)
    np.testing.assert_array_equal(st["point_list"].astype(np.uint32), fx["point_list"])
    np.testing.assert_array_equal(st["ranges"].astype(np.uint32), fx["ranges"])
    assert np.abs(to_np(h["color"]) - fx["out_color"]).max() <= 1e-4
    same = (st["n_contrib"].astype(np.uint32).reshape(fx["n_contrib"].shape) == fx["n_contrib"]).mean()
    assert same >= 0.9999
    names = dict(dL_dmeans2D="dmean2D", dL_dcolors="dcolor", dL_dopacity="dopacity", dL_dmeans3D="dmean3D",
                 dL_dcov3D="dcov3D", dL_dsh="dsh", dL_dscales="dscale", dL_drotations="drot")
    for k, hk in names.items():
        ok, emax, nbad = grad_close(to_np(h["grads"][hk]), fx[k])
        assert ok, (k, emax, nbad)

"""omni_math.h transcendentals (shared by the HIP preprocess and the oracle) against libm in double."""
import numpy as np

import oracle as O


def _ulp_err(got, ref):
    ref32 = np.float32(ref)
    sp = np.spacing(np.abs(ref32)).astype(np.float64)
    sp = np.where(sp == 0, np.spacing(np.float32(0)), sp)
    return np.abs(np.float64(got) - ref) / sp


def test_atan2_ulps(oracle_mod):
    L = O.lib()
    rng = np.random.default_rng(0)
    ys = np.concatenate([rng.uniform(-20, 20, 20000), rng.uniform(-1e-3, 1e-3, 2000), [0.0, -0.0, 1.0, -1.0, 3.0]])
    xs = np.concatenate([rng.uniform(-20, 20, 20000), rng.uniform(-1e-3, 1e-3, 2000), [1.0, -1.0, 0.0, -0.0, 3.0]])
    worst = 0.0
    for y, x in zip(ys.astype(np.float32), xs.astype(np.float32)):
        got = L.oracle_atan2f(float(y), float(x))
        ref = np.arctan2(np.float64(y), np.float64(x))
        worst = max(worst, float(_ulp_err(got, ref)))
    assert worst <= 3.0, worst


def test_atan2_signed_zeros_and_axes(oracle_mod):
    L = O.lib()
    assert L.oracle_atan2f(0.0, 1.0) == 0.0
    assert np.isclose(L.oracle_atan2f(0.0, -1.0), np.pi, rtol=0, atol=3e-7)
    assert np.isclose(L.oracle_atan2f(1.0, 0.0), np.pi / 2, rtol=0, atol=2e-7)
    assert np.isclose(L.oracle_atan2f(-1.0, 0.0), -np.pi / 2, rtol=0, atol=2e-7)
    assert np.copysign(1.0, L.oracle_atan2f(-0.0, 1.0)) < 0


def test_asin_ulps(oracle_mod):
    L = O.lib()
    rng = np.random.default_rng(1)
    xs = np.concatenate([rng.uniform(-1, 1, 20000), rng.uniform(-1e-3, 1e-3, 2000), [0.0, 0.5, -0.5, 1.0, -1.0,
                                                                                    0.99999994]])
    worst = 0.0
    for x in xs.astype(np.float32):
        got = L.oracle_asinf(float(x))
        worst = max(worst, float(_ulp_err(got, np.arcsin(np.float64(x)))))
    assert worst <= 3.0, worst
    assert np.isnan(L.oracle_asinf(1.0000001))

"""GPU unit test of the wave64 gradient reductions of wave_ops.h (cross-row-first v_permlane16/32_swap, and the
LDS-transposed ones the render backward uses). Column sums of a [64, 9] block must
match a float64 reference to f32 rounding."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


MODES = [dict(), dict(lds=True)]


@pytest.mark.parametrize("mode", MODES, ids=["rows", "lds"])
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_wave_sum_matches_column_sums(seed, mode, omr):
    import torch

    rng = np.random.default_rng(seed)
    x = rng.standard_normal((64, 9)).astype(np.float32)
    if seed == 2:  # sparse: most lanes zero, as when few pixels of a wave contribute
        x[rng.uniform(size=x.shape) < 0.85] = 0.0
    got = omr.rasterizer.debug_wave_sum(torch.from_numpy(x).cuda(), **mode).cpu().numpy()
    ref = x.astype(np.float64).sum(axis=0)
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("mode", MODES, ids=["rows", "lds"])
def test_wave_sum_lane_identity(mode, omr):
    import torch

    # value c of lane l = (c + 1) * 1000 + l: distinguishes every (lane, column) contribution exactly in f32
    x = np.array([[(c + 1) * 1000 + l for c in range(9)] for l in range(64)], dtype=np.float32)
    got = omr.rasterizer.debug_wave_sum(torch.from_numpy(x).cuda(), **mode).cpu().numpy()
    ref = x.astype(np.float64).sum(axis=0)
    np.testing.assert_array_equal(got, ref)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_wave_sum_pair_matches_column_sums(seed, omr):
    """wave_sum9x2_stored (render_bwd.hip): two instances' rows summed in one pass."""
    import torch

    rng = np.random.default_rng(10 + seed)
    x = rng.standard_normal((2, 64, 9)).astype(np.float32)
    if seed == 2:
        x[rng.uniform(size=x.shape) < 0.85] = 0.0
    got = omr.rasterizer.debug_wave_sum_pair(torch.from_numpy(x).cuda()).cpu().numpy()
    np.testing.assert_allclose(got, x.astype(np.float64).sum(axis=1), rtol=1e-5, atol=1e-5)


def test_wave_sum_pair_lane_identity(omr):
    import torch

    x = np.array([[[(i * 9 + c + 1) * 1000 + l for c in range(9)] for l in range(64)] for i in range(2)],
                 dtype=np.float32)
    got = omr.rasterizer.debug_wave_sum_pair(torch.from_numpy(x).cuda()).cpu().numpy()
    np.testing.assert_array_equal(got, x.astype(np.float64).sum(axis=1))

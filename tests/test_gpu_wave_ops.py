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


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_dpp_wave_scans(seed, omr):
    """raster_common.h: wave_incl_sum_u32 / wave_incl_max_u32 (row_shr + row_bcast DPP; every block scan of the sorts,
    look-back scans and row binning) and tile_wave.h: wave_max_u32, against numpy on full 64-lane waves."""
    import torch

    rng = np.random.default_rng(seed)
    hi = [1 << 20, 1 << 31, 4][seed]  # seed 1: large values (wrapping u32 sums), seed 2: many equal values
    x = rng.integers(0, hi, size=(2, 64), dtype=np.uint64).astype(np.uint32)
    got = omr.rasterizer.debug_wave_scans(torch.from_numpy(x.view(np.int32)).cuda()).cpu().numpy().view(np.uint32)
    np.testing.assert_array_equal(got[0], np.cumsum(x[0], dtype=np.uint64).astype(np.uint32))
    np.testing.assert_array_equal(got[1], np.maximum.accumulate(x[1]))
    np.testing.assert_array_equal(got[2], np.full(64, x[1].max(), dtype=np.uint32))

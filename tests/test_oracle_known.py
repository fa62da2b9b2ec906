"""Known-answer tests of the CPU oracle, pinned to the reference's own files (no golden vectors exist there):

* examples/simple_cloud.cpp:36-37,96-102,130-168,225-226 — 3 Gaussians, identity pose, 2000x1000 lonlat,
  raw scaling -0.3, raw opacity 5, D = 0: projected centres, colours and depths are analytic;
* an isotropic Gaussian on the equator: cov2D = s^2 diag((W/2pi d)^2, (H/pi d)^2) + 0.3 (forward.cu:147-188);
* getHigherMsb (rasterizer_impl.cu:47-62) on the tile counts of every BASELINE config;
* sort / range invariants of duplicateWithKeys + SortPairs + identifyTileRanges (rasterizer_impl.cu:94-167);
* rasterize_points.cu edge cases: P = 0 -> zero image; all culled -> background.
"""
import math

import numpy as np
import pytest

import oracle as O
from helpers import make_case, oracle_run, scene

LON, PIN = scene.CAMERA_LONLAT, scene.CAMERA_PINHOLE
SH_C0 = 0.28209479177387814


def _simple_cloud(dist):
    """simple_cloud.cpp: points, colours; createFromPcd sets f_dc = RGB2SH(colour), rotation (1,0,0,0)."""
    pts = np.array([[dist, -5 * dist, dist], [-dist, 0.5 * dist, -0.7 * dist], [dist, dist, -dist]], np.float32)
    cols = np.array([[1, 0, 0], [0, 1, 0], [0, 0, 1]], np.float32)
    P = 3
    sh = np.zeros((P, 16, 3), np.float32)
    sh[:, 0, :] = (cols - 0.5) / SH_C0
    g = scene.Gaussians(means3D=pts, scales=np.full((P, 3), math.exp(-0.3), np.float32),
                        rotations=np.tile(np.array([1, 0, 0, 0], np.float32), (P, 1)),
                        opacity=np.full((P, 1), 1 / (1 + math.exp(-5)), np.float32), shs=sh, sh_degree=0)
    Tcw = np.eye(4)
    cam = scene.Camera(LON, 2000, 1000, Tcw.T.astype(np.float32), Tcw.T.astype(np.float32), np.zeros(3, np.float32))
    return g, cam, cols


@pytest.mark.parametrize("dist", [1.0, 2.5])
def test_simple_cloud_centres_colours_depths(dist, oracle_mod):
    g, cam, cols = _simple_cloud(dist)
    o, L, _ = oracle_run(g, cam)
    W, H = cam.width, cam.height
    m2 = o.get("means2D").reshape(3, 2)
    p = g.means3D.astype(np.float64)
    r = np.linalg.norm(p, axis=1)
    lon = np.arctan2(p[:, 0], p[:, 2])
    lat = np.arcsin(p[:, 1] / r)
    px = ((lon / math.pi + 1) * W - 1) * 0.5
    py = ((lat * 2 / math.pi + 1) * H - 1) * 0.5
    np.testing.assert_allclose(m2[:, 0], px, atol=2e-3)
    np.testing.assert_allclose(m2[:, 1], py, atol=2e-3)
    np.testing.assert_allclose(o.get("depths"), r, rtol=1e-6)
    np.testing.assert_allclose(o.get("rgb").reshape(3, 3), cols, atol=1e-6)  # D = 0: C0 * RGB2SH(c) + 0.5 = c
    assert (o.get("radii") > 0).all() and L > 0
    # at each centre pixel the Gaussian dominates: colour ~ alpha_max * c (alpha clamps at 0.99)
    img = o.get("out_color").reshape(3, H, W)
    for k in range(3):
        x, y = int(round(px[k])), int(round(py[k]))
        assert img[:, y, x].argmax() == cols[k].argmax()
        assert img[:, y, x].max() > 0.9


@pytest.mark.parametrize("W,H,d,s", [(512, 256, 4.0, 0.05), (2048, 1024, 7.0, 0.02), (333, 171, 3.0, 0.1)])
def test_equator_isotropic_conic(W, H, d, s, oracle_mod):
    g = scene.Gaussians(means3D=np.array([[0, 0, d]], np.float32), scales=np.full((1, 3), s, np.float32),
                        rotations=np.array([[1, 0, 0, 0]], np.float32), opacity=np.array([[0.8]], np.float32),
                        shs=np.zeros((1, 16, 3), np.float32), sh_degree=0)
    Tcw = np.eye(4)
    cam = scene.Camera(LON, W, H, Tcw.T.astype(np.float32), Tcw.T.astype(np.float32), np.zeros(3, np.float32))
    o, _, _ = oracle_run(g, cam)
    m2 = o.get("means2D")
    np.testing.assert_allclose(m2, [(W - 1) / 2, (H - 1) / 2], atol=1e-4)
    a = s * s * (W / (2 * math.pi * d)) ** 2 + 0.3
    c = s * s * (H / (math.pi * d)) ** 2 + 0.3
    con = o.get("conic_opacity")
    np.testing.assert_allclose(con[[0, 2]], [1 / a, 1 / c], rtol=2e-5)
    assert abs(con[1]) < 1e-6 * max(1 / a, 1 / c)
    lam = max(a, c)
    assert o.get("radii")[0] == math.ceil(3 * math.sqrt(lam))


@pytest.mark.parametrize("T,expect", [(1, 1), (512, 10), (2048, 12), (8192, 14), (32768, 16), (8160, 13), (9, 4)])
def test_get_higher_msb(T, expect, oracle_mod):
    assert O.lib().oracle_higher_msb(T) == expect


def test_sort_invariants_and_ranges(oracle_mod):
    g, cam, _ = make_case(10000, 512, 256, LON, scene.BASE_SEED)
    o, L, _ = oracle_run(g, cam)
    keys = o.get("keys")
    pl = o.get("point_list")
    assert len(keys) == L == len(pl) == int(o.get("tiles_touched").astype(np.int64).sum())
    assert (keys[1:] >= keys[:-1]).all()
    tile = (keys >> np.uint64(32)).astype(np.int64)
    depth = (keys & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    np.testing.assert_array_equal(depth, o.get("depths").astype(np.float32).view(np.uint32)[pl])
    same = tile[1:] == tile[:-1]
    # ties in (tile, depth) keep ascending Gaussian index (stable radix sort of the emission order)
    tie = same & (depth[1:] == depth[:-1])
    assert (pl[1:][tie] > pl[:-1][tie]).all()
    # ranges cover exactly each tile's run
    rng = o.get("ranges").reshape(-1, 2)
    gx, gy = 32, 16
    assert rng.shape[0] == gx * gy
    counts = np.bincount(tile, minlength=gx * gy)
    np.testing.assert_array_equal(rng[:, 1] - rng[:, 0], counts)
    nz = counts > 0
    np.testing.assert_array_equal(tile[rng[nz, 0]], np.nonzero(nz)[0])


def test_two_stage_binning_reproduces_reference_order(oracle_mod):
    """The gfx950 binning (depth sort of Gaussians, emission in depth order, stable tile sort) yields exactly the
    reference's SortPairs permutation — checked here in numpy against the oracle's 64-bit-key sort."""
    g, cam, _ = make_case(5000, 333, 171, LON, 31, view_index=3, spread=1.5)
    o, L, _ = oracle_run(g, cam)
    P = g.P
    radii = o.get("radii")
    depth_bits = o.get("depths").astype(np.float32).view(np.uint32)
    order = np.argsort(np.where(radii > 0, depth_bits, np.uint32(0xFFFFFFFF)), kind="stable")
    keys = o.get("keys")
    tile_of = {}
    pl = o.get("point_list")
    tiles_sorted = (keys >> np.uint64(32)).astype(np.int64)
    # per Gaussian, the set of tiles it was emitted to (from the reference order itself)
    for t_, gid in zip(tiles_sorted, pl):
        tile_of.setdefault(int(gid), []).append(int(t_))
    em_tiles, em_vals = [], []
    for gid in order:
        if radii[gid] > 0:
            ts = sorted(tile_of[int(gid)])  # row-major emission = ascending tile id within the rect
            em_tiles += ts
            em_vals += [gid] * len(ts)
    em_tiles, em_vals = np.array(em_tiles), np.array(em_vals)
    assert len(em_vals) == L
    perm = np.argsort(em_tiles, kind="stable")
    np.testing.assert_array_equal(em_vals[perm], pl)
    del P


def test_empty_scene_is_zero_image(oracle_mod):
    g, cam, dL = make_case(0, 64, 32, LON, 1)
    o, L, gr = oracle_run(g, cam, dL, bg=(1, 1, 1))
    assert L == 0
    assert (o.get("out_color") == 0).all()


def test_all_culled_is_background(oracle_mod):
    g, cam, dL = make_case(50, 64, 32, LON, 2)
    g.means3D = (g.means3D * 1e-3).astype(np.float32)
    o, L, gr = oracle_run(g, cam, dL, bg=(0.25, 0.5, 1.0))
    assert L == 0
    img = o.get("out_color").reshape(3, 32, 64)
    np.testing.assert_array_equal(img[1], 0.5)
    for v in gr.values():
        assert (v == 0).all()


def test_pinhole_culls_behind_camera(oracle_mod):
    g, cam, _ = make_case(2000, 160, 90, PIN, 3)
    o, _, _ = oracle_run(g, cam)
    z = (np.c_[g.means3D.astype(np.float64), np.ones(g.P)] @ cam.viewmatrix.astype(np.float64))[:, 2]
    radii = o.get("radii")
    assert (radii[z <= 0.19] == 0).all()


def test_invalid_camera_type_raises(oracle_mod):
    g, cam, _ = make_case(10, 64, 32, LON, 4)
    cam.camera_type = 2
    with pytest.raises(RuntimeError, match="Invalid camera_type"):
        oracle_run(g, cam)


def test_prefiltered_cull_raises(oracle_mod):
    g, cam, _ = make_case(100, 64, 32, PIN, 5)
    with pytest.raises(RuntimeError, match="prefiltered"):
        oracle_run(g, cam, prefiltered=True)

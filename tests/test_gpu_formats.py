"""distCUDA2 (csrc/knn.hip) and Gaussian PLY I/O (csrc/formats.hip) on the GPU against oracle/formats_oracle.py.

Bars: distCUDA2 bit-exact (both sides keep the exact three smallest float32 squared distances); PLY files
byte-identical to the savePly layout; loaded tensors bit-exact.
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
import formats_oracle as FO  # noqa: E402

F = omr.formats


def _pts(kind, P, seed):
    rng = np.random.default_rng(seed)
    if kind == "normal":
        p = rng.normal(size=(P, 3))
    elif kind == "clustered":  # SLAM-like: dense clusters far from the origin plus sparse outliers
        c = rng.normal(size=(max(P // 500, 1), 3)) * 20 + 50
        p = c[rng.integers(0, len(c), P)] + rng.normal(size=(P, 3)) * 0.05
        p[: P // 100] = rng.uniform(-100, 100, size=(P // 100, 3))
    elif kind == "duplicates":
        p = rng.normal(size=(P, 3))
        p[1::3] = p[0::3][: len(p[1::3])]
    elif kind == "plane":  # z = 0 everywhere: a degenerate Morton axis
        p = rng.normal(size=(P, 3))
        p[:, 2] = 0
    else:
        raise ValueError(kind)
    return np.ascontiguousarray(p, dtype=np.float32)


@pytest.mark.parametrize("P", [1, 2, 3, 4, 5, 63, 64, 65, 100, 4097])
def test_dist2_small_exact(P):
    p = _pts("normal", P, P)
    got = to_np(F.distCUDA2(torch.from_numpy(p).cuda()))
    with np.errstate(over="ignore"):
        want = FO.dist2(p)
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("kind,P", [("normal", 200003), ("clustered", 150000), ("duplicates", 30000),
                                    ("plane", 20000)])
def test_dist2_large_exact(kind, P):
    p = _pts(kind, P, 11)
    got = to_np(F.distCUDA2(torch.from_numpy(p).cuda()))
    np.testing.assert_array_equal(got, FO.dist2(p))


def test_dist2_empty_and_cpu_rejected():
    assert F.distCUDA2(torch.zeros((0, 3), device="cuda")).shape == (0,)
    with pytest.raises(omr.rasterizer.RasterizerError, match="HIP"):
        F.distCUDA2(torch.zeros((4, 3)))


def test_create_from_pcd():
    P = 5000
    p = _pts("clustered", P, 2)
    col = np.random.default_rng(2).random((P, 3)).astype(np.float32)
    m = F.create_from_pcd(torch.from_numpy(p).cuda(), torch.from_numpy(col).cuda(), 3)
    torch.cuda.synchronize()
    d2 = np.maximum(FO.dist2(p), np.float32(1e-7))
    np.testing.assert_allclose(to_np(m.scaling), np.repeat(np.log(np.sqrt(d2))[:, None], 3, 1), rtol=1e-6)
    np.testing.assert_allclose(to_np(m.features_dc)[:, 0], (col - 0.5) / 0.28209479177387814, rtol=1e-6)
    assert m.features_rest.shape == (P, 15, 3) and not m.features_rest.any()
    assert torch.equal(m.rotation, torch.tensor([[1.0, 0, 0, 0]], device="cuda").expand(P, 4))
    np.testing.assert_allclose(to_np(torch.sigmoid(m.opacity)), 0.1, rtol=1e-6)


def _model(P, Mr, seed):
    rng = np.random.default_rng(seed)
    arrs = [rng.normal(size=(P, 3)), rng.normal(size=(P, 1, 3)), rng.normal(size=(P, Mr, 3)), rng.normal(size=(P, 1)),
            rng.normal(size=(P, 3)), rng.normal(size=(P, 4))]
    arrs = [np.ascontiguousarray(a, dtype=np.float32) for a in arrs]
    deg = int(round(np.sqrt(Mr + 1))) - 1
    return arrs, omr.renderer.GaussianModelParams(*[torch.from_numpy(a).cuda() for a in arrs], deg, deg)


@pytest.mark.parametrize("P,Mr", [(1000, 15), (257, 3), (5, 0), (0, 15)])
def test_save_ply_bytes_match_saveply_layout(tmp_path, P, Mr):
    arrs, m = _model(P, Mr, P + Mr)
    path = str(tmp_path / "m.ply")
    F.save_ply(m, path)
    assert open(path, "rb").read() == FO.ply_bytes(*arrs)


@pytest.mark.parametrize("deg", [3, 1])
def test_load_ply_roundtrip(tmp_path, deg):
    Mr = (deg + 1) ** 2 - 1
    arrs, m = _model(3001, Mr, 5)
    path = str(tmp_path / "m.ply")
    with open(path, "wb") as fh:
        fh.write(FO.ply_bytes(*arrs))
    got = F.load_ply(path, deg)
    torch.cuda.synchronize()
    assert got.active_sh_degree == deg and got.max_sh_degree == deg
    for a, t in zip(arrs, got.parameters()):
        np.testing.assert_array_equal(to_np(t), a)
    F.save_ply(got, str(tmp_path / "again.ply"))
    assert open(str(tmp_path / "again.ply"), "rb").read() == open(path, "rb").read()


@pytest.mark.parametrize("fmt,dtype,leading", [("binary_little_endian", "float", True), ("ascii", "float", True),
                                               ("binary_big_endian", "float", False),
                                               ("binary_little_endian", "double", False)])
def test_load_ply_other_layouts(tmp_path, fmt, dtype, leading):
    """tinyply requests properties by name: permuted order, extra properties, other elements, ascii / big-endian
    files and wider types load to the same tensors."""
    arrs, _ = _model(777, 15, 8)
    table, names = FO.ply_columns(*arrs)
    order = np.random.default_rng(1).permutation(len(names))
    path = str(tmp_path / "c.ply")
    FO.ply_write_custom(path, table, names, fmt=fmt, dtype=dtype, order=order, extra=2, leading_element=leading)
    got = F.load_ply(path, 3)
    torch.cuda.synchronize()
    for a, t in zip(arrs, got.parameters()):
        np.testing.assert_array_equal(to_np(t), a)


def test_load_ply_errors(tmp_path):
    with pytest.raises(omr.rasterizer.RasterizerError, match="Fail to open ply file"):
        F.load_ply(str(tmp_path / "missing.ply"), 3)
    arrs, _ = _model(10, 3, 1)  # degree-1 file read as degree 3: f_rest_9.. missing
    path = str(tmp_path / "d1.ply")
    with open(path, "wb") as fh:
        fh.write(FO.ply_bytes(*arrs))
    with pytest.raises(omr.rasterizer.RasterizerError, match="f_rest_9"):
        F.load_ply(path, 3)
    with open(path, "r+b") as fh:  # truncate the data
        fh.truncate(len(FO.ply_bytes(*arrs)) - 100)
    with pytest.raises(omr.rasterizer.RasterizerError, match="truncated"):
        F.load_ply(path, 1)

"""distCUDA2 / PLY oracle (oracle/formats_oracle.py) on CPU: known answers, brute force vs k-d tree, the savePly
byte layout (tinyply.h:664-703 header, gaussian_model.cpp:974-1070 records)."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import formats_oracle as FO  # noqa: E402


def test_dist2_known_answers():
    # unit square corners in z = 0: every corner has neighbours at 1, 1, sqrt(2) -> (1 + 1 + 2) / 3
    sq = np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0], [1, 1, 0]], np.float32)
    np.testing.assert_array_equal(FO.dist2(sq), np.full(4, np.float32(4.0) / np.float32(3.0)))
    # duplicates are distance 0 to each other
    d = FO.dist2(np.array([[0, 0, 0]] * 4 + [[5, 5, 5]], np.float32))
    assert (d[:4] == 0).all() and d[4] == np.float32(75.0)
    # fewer than 4 points: FLT_MAX fills the missing neighbours (the sum overflows to inf, as the reference)
    with np.errstate(over="ignore"):
        assert np.isinf(FO.dist2(np.zeros((2, 3), np.float32))).all()
        assert FO.dist2(np.zeros((0, 3), np.float32)).shape == (0,)


def test_dist2_brute_force_matches_kdtree():
    rng = np.random.default_rng(3)
    p = np.concatenate([rng.normal(size=(5000, 3)), rng.normal(size=(2500, 3)) * 0.01 + 3.0]).astype(np.float32)
    p[100:110] = p[200]  # duplicates
    np.testing.assert_array_equal(FO.dist2(p, brute=False), FO.dist2(p, brute=True))


def test_ply_bytes_layout():
    P, Mr = 2, 1
    xyz = np.arange(6, dtype=np.float32).reshape(P, 3)
    f_dc = np.arange(6, dtype=np.float32).reshape(P, 1, 3) + 10
    f_rest = np.arange(6, dtype=np.float32).reshape(P, Mr, 3) + 20
    op = np.array([[0.5], [0.25]], np.float32)
    sc = -np.arange(6, dtype=np.float32).reshape(P, 3)
    rot = np.arange(8, dtype=np.float32).reshape(P, 4) + 30
    b = FO.ply_bytes(xyz, f_dc, f_rest, op, sc, rot)
    head = ("ply\nformat binary_little_endian 1.0\nelement vertex 2\n" +
            "".join(f"property float {n}\n" for n in ["x", "y", "z", "nx", "ny", "nz", "f_dc_0", "f_dc_1", "f_dc_2",
                                                       "f_rest_0", "f_rest_1", "f_rest_2", "opacity", "scale_0",
                                                       "scale_1", "scale_2", "rot_0", "rot_1", "rot_2", "rot_3"]) +
            "end_header\n").encode()
    assert b[:len(head)] == head
    rec = np.frombuffer(b[len(head):], "<f4").reshape(P, 20)
    np.testing.assert_array_equal(rec[0], [0, 1, 2, 0, 0, 0, 10, 11, 12, 20, 21, 22, 0.5, 0, -1, -2, 30, 31, 32, 33])
    names, table = FO.ply_parse(b)
    assert len(names) == 20 and np.array_equal(table, rec)
    # degree 3: 62 properties, 248 B per vertex (gaussian_model.cpp:974-1070)
    b3 = FO.ply_bytes(xyz, f_dc, np.zeros((P, 15, 3), np.float32), op, sc, rot)
    names, table = FO.ply_parse(b3)
    assert len(names) == 62 and table.shape == (2, 62)


def test_ply_channel_major_sh():
    """f_rest_{c*Mr + k} = features_rest[p][k][c] (features.transpose(1, 2).flatten(1))."""
    Mr = 15
    fr = np.arange(45, dtype=np.float32).reshape(1, Mr, 3)
    table, names = FO.ply_columns(np.zeros((1, 3), np.float32), np.zeros((1, 1, 3), np.float32), fr,
                                  np.zeros((1, 1), np.float32), np.zeros((1, 3), np.float32),
                                  np.zeros((1, 4), np.float32))
    for c in range(3):
        for k in range(Mr):
            assert table[0, names.index(f"f_rest_{c * Mr + k}")] == fr[0, k, c]


@pytest.mark.parametrize("fmt,dtype", [("ascii", "float"), ("binary_big_endian", "double")])
def test_custom_writer_formats_parse(tmp_path, fmt, dtype):
    table = np.arange(12, dtype=np.float32).reshape(3, 4)
    p = tmp_path / "x.ply"
    FO.ply_write_custom(str(p), table, ["a", "b", "c", "d"], fmt=fmt, dtype=dtype, order=[3, 1, 0, 2], extra=1)
    txt = open(p, "rb").read()
    assert txt.startswith(b"ply\nformat " + fmt.encode()) and b"property " + dtype.encode() + b" d\n" in txt

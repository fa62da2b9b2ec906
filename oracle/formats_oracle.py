"""CPU restatement of distCUDA2 and the Gaussian PLY format (TEST INFRASTRUCTURE ONLY).

Used by tests/ as the checker for omnigs-fork_amd/csrc/knn.hip and formats.hip; the product never imports it.

  * dist2            simple_knn.cu:145-183 computes, for every point, the mean of its 3 smallest squared distances
                     to other points (box pruning never drops one of them). Restated as brute force in float32:
                     d = dx*dx + dy*dy + dz*dz, the three smallest ascending, (b0 + b1 + b2) / 3, FLT_MAX for
                     missing neighbours (P < 4). For large P the candidates come from scipy's k-d tree (8 nearest
                     in float64) and are re-measured in float32. Parity unpinned: the reference ships no KNN tests.
  * ply_bytes        the file GaussianModel::savePly (gaussian_model.cpp:974-1070) writes through tinyply: header as
                     tinyply.h:664-703, interleaved float32 records, zero normals, channel-major SH.
  * ply_write_custom files in other layouts (property order, extra properties, ascii, big-endian, doubles) that
                     loadPly accepts because tinyply requests properties by name.
"""
from __future__ import annotations

import numpy as np

FLT_MAX = np.float32(np.finfo(np.float32).max)
f32 = np.float32


def _mean3(best):
    best = np.sort(best.astype(f32), axis=1)
    return ((best[:, 0] + best[:, 1]) + best[:, 2]) / f32(3.0)


def _sqd(p, q):
    d = (q - p).astype(f32)
    return d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1] + d[..., 2] * d[..., 2]


def dist2(points, chunk=512, brute=None):
    p = np.asarray(points, f32).reshape(-1, 3)
    P = p.shape[0]
    out = np.zeros(P, f32)
    if P == 0:
        return out
    if (brute is None and P > 6000) or brute is False:
        return _dist2_kdtree(p)
    for s in range(0, P, chunk):
        q = p[s:s + chunk]
        d = _sqd(q[:, None, :], p[None, :, :])
        d[np.arange(q.shape[0]), np.arange(s, s + q.shape[0])] = np.inf
        k = min(3, P - 1)
        best = np.full((q.shape[0], 3), FLT_MAX, f32)
        if k > 0:
            best[:, :k] = np.partition(d, k - 1, axis=1)[:, :k]
        out[s:s + chunk] = _mean3(best)
    return out


def _dist2_kdtree(p):
    from scipy.spatial import cKDTree

    P = p.shape[0]
    _, idx = cKDTree(p.astype(np.float64)).query(p.astype(np.float64), k=min(9, P))
    cand = p[idx]  # [P, k, 3]
    d = _sqd(p[:, None, :], cand)
    d[idx == np.arange(P)[:, None]] = np.inf
    best = np.partition(d, 2, axis=1)[:, :3]
    return _mean3(best)


def _names(Mr):
    n = ["x", "y", "z", "nx", "ny", "nz", "f_dc_0", "f_dc_1", "f_dc_2"]
    n += [f"f_rest_{i}" for i in range(3 * Mr)]
    n += ["opacity", "scale_0", "scale_1", "scale_2", "rot_0", "rot_1", "rot_2", "rot_3"]
    return n


def ply_columns(xyz, f_dc, f_rest, opacity, scaling, rotation):
    """[P, 17 + 3 Mr] float32 table in savePly's property order."""
    P = xyz.shape[0]
    Mr = f_rest.shape[1]
    cols = [xyz.reshape(P, 3), np.zeros((P, 3), f32), f_dc.reshape(P, 1, 3).transpose(0, 2, 1).reshape(P, 3),
            f_rest.reshape(P, Mr, 3).transpose(0, 2, 1).reshape(P, 3 * Mr), opacity.reshape(P, 1),
            scaling.reshape(P, 3), rotation.reshape(P, 4)]
    return np.concatenate(cols, axis=1).astype(f32), _names(Mr)


def ply_bytes(xyz, f_dc, f_rest, opacity, scaling, rotation) -> bytes:
    table, names = ply_columns(xyz, f_dc, f_rest, opacity, scaling, rotation)
    head = "ply\nformat binary_little_endian 1.0\n" + f"element vertex {table.shape[0]}\n"
    head += "".join(f"property float {n}\n" for n in names) + "end_header\n"
    return head.encode("ascii") + table.astype("<f4").tobytes()


def ply_write_custom(path, table, names, fmt="binary_little_endian", dtype="float", order=None, extra=0,
                     comments=("written by tests",), leading_element=False):
    """Write `table` ([P, n] with column names) as a PLY in another layout: permuted property `order`, `extra`
    additional float properties, ascii / big-endian format, double properties, a leading non-vertex element."""
    P = table.shape[0]
    order = list(range(table.shape[1])) if order is None else list(order)
    cols = [table[:, j] for j in order]
    cnames = [names[j] for j in order]
    rng = np.random.default_rng(0)
    for e in range(extra):
        cols.append(rng.normal(size=P).astype(f32))
        cnames.append(f"extra_{e}")
    data = np.stack(cols, axis=1) if cols else np.zeros((P, 0), f32)
    np_t = {"float": "f4", "double": "f8"}[dtype]
    head = f"ply\nformat {fmt} 1.0\n" + "".join(f"comment {c}\n" for c in comments)
    if leading_element:
        head += "element camera 2\nproperty float fx\nproperty uchar id\n"
    head += f"element vertex {P}\n" + "".join(f"property {dtype} {n}\n" for n in cnames)
    head += "element face 0\nproperty list uchar int vertex_indices\nend_header\n"
    with open(path, "wb") as fh:
        fh.write(head.encode("ascii"))
        if fmt == "ascii":
            if leading_element:
                fh.write(b"1.5 3\n2.5 4\n")
            for row in data:
                fh.write((" ".join(repr(float(v)) for v in row) + "\n").encode("ascii"))
        else:
            end = "<" if fmt == "binary_little_endian" else ">"
            if leading_element:
                for v, i in ((1.5, 3), (2.5, 4)):
                    fh.write(np.array([v], end + "f4").tobytes() + bytes([i]))
            fh.write(data.astype(end + np_t).tobytes())


def ply_parse(path_or_bytes):
    """Minimal reader of savePly files: returns (names, table float32 [P, n])."""
    raw = path_or_bytes if isinstance(path_or_bytes, (bytes, bytearray)) else open(path_or_bytes, "rb").read()
    end = raw.index(b"end_header\n") + len(b"end_header\n")
    names, P = [], 0
    for line in raw[:end].decode("ascii").splitlines():
        t = line.split()
        if t[:2] == ["element", "vertex"]:
            P = int(t[2])
        elif t and t[0] == "property":
            names.append(t[2])
    table = np.frombuffer(raw[end:end + 4 * P * len(names)], "<f4").reshape(P, len(names))
    return names, table

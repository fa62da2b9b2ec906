"""Gaussian model formats on gfx950.

  * distCUDA2(points)                   third_party/simple-knn/spatial.cu:15-25 (simple_knn.cu:185-220)
  * create_from_pcd(points, colors)     GaussianModel::createFromPcd (gaussian_model.cpp:120-185)
  * load_ply(path, max_sh_degree)       GaussianModel::loadPly (gaussian_model.cpp:860-972)
  * save_ply(model, path)               GaussianModel::savePly (gaussian_model.cpp:974-1070)

The KNN, the PLY (de)interleave and the SH transposes run in libomnigs_raster.so (csrc/knn.hip,
csrc/formats.hip); torch only allocates.
"""
from __future__ import annotations

import ctypes as C
import os

import torch

from . import rasterizer as R
from .renderer import GaussianModelParams

SH_C0 = 0.28209479177387814


def _p6(ts):
    return (C.c_void_p * 6)(*[None if t is None or t.numel() == 0 else t.data_ptr() for t in ts])


def distCUDA2(points: torch.Tensor) -> torch.Tensor:
    """Mean squared distance of every point to its 3 nearest other points (exact), float32 [P]."""
    if points.device.type != "cuda":
        raise R.RasterizerError("distCUDA2 needs a HIP tensor (no CPU path)")
    pts = points.detach().contiguous().float()
    if pts.dim() != 2 or pts.shape[1] != 3:
        raise R.RasterizerError("points must be [P,3]")
    P = int(pts.shape[0])
    out = torch.zeros((P,), dtype=torch.float32, device=pts.device)
    if P == 0:
        return out
    L = R.lib()
    scratch = torch.empty(int(L.omr_dist2_scratch_bytes(P)), dtype=torch.uint8, device=pts.device)
    R._check(L.omr_dist2(P, pts.data_ptr(), out.data_ptr(), scratch.data_ptr(), R._stream(pts.device)), "distCUDA2")
    return out


def create_from_pcd(points: torch.Tensor, colors: torch.Tensor, max_sh_degree: int = 3) -> GaussianModelParams:
    """createFromPcd: SH DC from RGB2SH(colors) (sh_utils.h:138-141), rest zero; scales log(sqrt(max(dist2, 1e-7)))
    on all three axes; identity rotations; opacity inverse_sigmoid(0.1)."""
    dev = points.device
    xyz = points.detach().contiguous().float().clone()
    P = xyz.shape[0]
    M = (max_sh_degree + 1) ** 2
    f_dc = ((colors.detach().float().to(dev) - 0.5) / SH_C0).reshape(P, 1, 3).contiguous()
    f_rest = torch.zeros((P, M - 1, 3), device=dev)
    dist2 = torch.clamp_min(distCUDA2(xyz), 0.0000001)
    scales = torch.log(torch.sqrt(dist2)).unsqueeze(1).repeat(1, 3).contiguous()
    rots = torch.zeros((P, 4), device=dev)
    rots[:, 0] = 1
    op = 0.1 * torch.ones((P, 1), device=dev)
    opacity = torch.log(op / (1 - op))
    return GaussianModelParams(xyz, f_dc, f_rest, opacity, scales, rots, 0, max_sh_degree)


def load_ply(path: str, max_sh_degree: int = 3, device="cuda") -> GaussianModelParams:
    """loadPly: active_sh_degree = max_sh_degree afterwards (:971)."""
    L = R.lib()
    h = C.c_void_p()
    n = C.c_int64()
    R._check(L.omr_ply_open(os.fsencode(path), int(max_sh_degree), C.byref(h), C.byref(n)), "loadPly")
    try:
        P, Mr = int(n.value), (max_sh_degree + 1) ** 2 - 1
        dev = torch.device(device)
        ts = [torch.empty(s, dtype=torch.float32, device=dev)
              for s in ((P, 3), (P, 1, 3), (P, Mr, 3), (P, 1), (P, 3), (P, 4))]
        R._check(L.omr_ply_read(h, _p6(ts), R._stream(dev)), "loadPly")
    finally:
        L.omr_ply_close(h)
    return GaussianModelParams(*ts, max_sh_degree, max_sh_degree)


def save_ply(model: GaussianModelParams, path: str):
    ts = [t.detach().contiguous().float() for t in model.parameters()]
    if any(t.device.type != "cuda" for t in ts):
        raise R.RasterizerError("save_ply needs the model on a HIP device")
    P, Mr = int(ts[0].shape[0]), int(ts[2].shape[1])
    R._check(R.lib().omr_ply_save(os.fsencode(path), P, Mr, _p6(ts), R._stream(ts[0].device)), "savePly")

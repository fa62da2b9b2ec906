"""View-parallel data parallelism for the rasterizer.

One process per GPU; every rank holds all P Gaussians, renders its own view (rank k -> view k) and runs the
rasterizer backward; the per-Gaussian gradients of all views are then summed with ONE all-reduce of a flat
buffer over RCCL (torch.distributed backend "nccl" is RCCL on ROCm; gloo on CPU for tests).

The reference has no parallelism at all (one view per Adam step on one GPU, gaussian_mapper.cpp:301); this is
the added axis. Gradients are taken w.r.t. the rasterizer's inputs (activated parameters): the chain rule
through exp/normalize/sigmoid is per Gaussian and linear in the incoming gradient, so it commutes with the
sum over views and is applied once after the reduction instead of once per view.

Flat buffer layout (float32, one segment per tensor, each contiguous — 59 floats = 236 B per Gaussian):
    [ means3D 3P | opacity P | scales 3P | rotations 4P | sh 3MP ]
The rasterizer backward writes straight into these views (RasterizeGaussiansBackwardCUDA(out=...)), so there
is no pack/unpack copy before or after the collective.

Two exchanges give the same summed gradients (up to the order of the float additions):
  * allreduce_          one RCCL all-reduce of the whole 236 B/Gaussian buffer;
  * allreduce_compact_  (default in bench.py) all-reduce of the first 44 B/Gaussian (xyz, opacity, scale,
                        rotation) and an all-gather of each view's colour gradient (12 B/Gaussian) and camera
                        position; every rank then rebuilds the summed SH gradient with the backward's own SH
                        arithmetic (omr_sh_grad_from_colors). Per rank on a ring of n: 2(n-1)/n * 236 B/G vs
                        2(n-1)/n * 44 + (n-1) * 12 B/G — at n = 8, 413 vs 161 MB for 1 M Gaussians, at n = 2 236 vs
                        56 MB. xGMI is point-to-point (a 2-GPU job has ONE link), so bytes are the scaling cost.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.distributed as dist

SEGMENTS = ("dL_dmeans3D", "dL_dopacity", "dL_dscales", "dL_drotations", "dL_dsh")
REDUCED_FLOATS = 11  # per Gaussian ahead of the SH segment: xyz 3, opacity 1, scales 3, rotations 4


@dataclass
class DistInfo:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0

    @property
    def enabled(self) -> bool:
        return self.world_size > 1


class GradBuffer:
    """Flat gradient buffer with per-tensor views matching RasterizeGaussiansBackwardCUDA's outputs."""

    def __init__(self, P: int, M: int, device, dtype=torch.float32):
        self.P, self.M = P, M
        sizes = [3 * P, P, 3 * P, 4 * P, 3 * M * P]
        shapes = [(P, 3), (P, 1), (P, 3), (P, 4), (P, M, 3)]
        self.flat = torch.empty(sum(sizes), dtype=dtype, device=device)
        self.views = {}
        off = 0
        for name, n, shp in zip(SEGMENTS, sizes, shapes):
            self.views[name] = self.flat[off:off + n].view(shp)
            off += n
        self.extra = {}  # scratch outputs that are not reduced (dL_dmeans2D, dL_dcolors, dL_dcov3D)

    def out_dict(self, device):
        P = self.P
        if not self.extra:
            self.extra = dict(dL_dmeans2D=torch.empty((P, 3), device=device),
                              dL_dcolors=torch.empty((P, 3), device=device),
                              dL_dcov3D=torch.empty((P, 6), device=device))
        d = dict(self.views)
        d.update(self.extra)
        return d

    @property
    def nbytes(self) -> int:
        return self.flat.numel() * self.flat.element_size()


def allreduce_(buf: GradBuffer, info: DistInfo, average: bool = False, bucket_bytes: int = 0):
    """Sum (or mean) the flat buffer over all ranks in place. bucket_bytes > 0 splits it into equal buckets
    (one collective each); 0 = a single collective — RCCL's multi-channel rings already spread one large
    message over the xGMI links, so fewer, larger calls are the default."""
    if not info.enabled:
        return
    flat = buf.flat
    if bucket_bytes and bucket_bytes < buf.nbytes:
        n = max(1, bucket_bytes // flat.element_size())
        for s in range(0, flat.numel(), n):
            dist.all_reduce(flat[s:s + n], op=dist.ReduceOp.SUM)
    else:
        dist.all_reduce(flat, op=dist.ReduceOp.SUM)
    if average:
        flat.div_(info.world_size)


def allreduce_compact_(buf: GradBuffer, info: DistInfo, dL_dcolors: torch.Tensor, campos: torch.Tensor, rebuild,
                       average: bool = False):
    """Sum over ranks with the compact SH exchange (module docstring): all-reduce the 11 non-SH floats per
    Gaussian, all-gather every rank's dL_dcolors [P,3] and campos [3], then
    rebuild(campos_all [n,3], dcolors_all [n,P,3], out=dL_dsh view) writes the summed SH gradient. `rebuild` is
    rasterizer.sh_grad_from_colors bound to the (replicated) means3D / SH / degree; tests pass a CPU model."""
    if not info.enabled:
        return
    n, P = info.world_size, buf.P
    prefix = buf.flat[:REDUCED_FLOATS * P]
    dist.all_reduce(prefix, op=dist.ReduceOp.SUM)
    dc = dL_dcolors.contiguous().view(P, 3)
    cp = campos.contiguous().view(3).to(dc.dtype)
    if dist.get_backend() == "nccl":
        dcolors_all = torch.empty((n, P, 3), dtype=dc.dtype, device=dc.device)
        campos_all = torch.empty((n, 3), dtype=dc.dtype, device=dc.device)
        dist.all_gather_into_tensor(dcolors_all, dc)
        dist.all_gather_into_tensor(campos_all, cp)
    else:
        parts = [torch.empty_like(dc) for _ in range(n)]
        cps = [torch.empty_like(cp) for _ in range(n)]
        dist.all_gather(parts, dc)
        dist.all_gather(cps, cp)
        dcolors_all, campos_all = torch.stack(parts), torch.stack(cps)
    rebuild(campos_all, dcolors_all, out=buf.views["dL_dsh"])
    if average:
        buf.flat.div_(n)

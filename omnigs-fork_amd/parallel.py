"""View-parallel data parallelism for the rasterizer.

One process per GPU; every rank holds all P Gaussians, renders its own view (rank k -> view k) and runs the
rasterizer backward; the per-Gaussian gradients of all views are then summed with ONE all-reduce of a flat
buffer over RCCL (torch.distributed backend "nccl" is RCCL on ROCm; gloo on CPU for tests).

The reference has no parallelism at all (one view per Adam step on one GPU, gaussian_mapper.cpp:301); this is
the added axis. Gradients are taken w.r.t. the rasterizer's inputs (activated parameters): the chain rule
through exp/normalize/sigmoid is per Gaussian and linear in the incoming gradient, so it commutes with the
sum over views and is applied once after the reduction instead of once per view.

Flat buffer layout (float32, one segment per tensor, each contiguous — 59 floats = 236 B per Gaussian):
    [ means3D 3P | sh 3MP | opacity P | scales 3P | rotations 4P ]
The rasterizer backward writes straight into these views (RasterizeGaussiansBackwardCUDA(out=...)), so there
is no pack/unpack copy before or after the collective.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.distributed as dist

SEGMENTS = ("dL_dmeans3D", "dL_dsh", "dL_dopacity", "dL_dscales", "dL_drotations")


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
        sizes = [3 * P, 3 * M * P, P, 3 * P, 4 * P]
        shapes = [(P, 3), (P, M, 3), (P, 1), (P, 3), (P, 4)]
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

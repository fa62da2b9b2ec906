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
  * allreduce_compact_  all-reduce of the first 44 B/Gaussian (xyz, opacity, scale,
                        rotation) and ONE all-gather of each view's colour gradient (12 B/Gaussian) with its camera
                        position appended as an extra row; every rank then rebuilds the summed SH gradient with the backward's own SH
                        arithmetic (omr_sh_grad_from_colors). Per rank on a ring of n: 2(n-1)/n * 236 B/G vs
                        2(n-1)/n * 44 + (n-1) * 12 B/G — at n = 8, 413 vs 161 MB for 1 M Gaussians, at n = 2 236 vs
                        56 MB. xGMI is point-to-point (a 2-GPU job has ONE link), so bytes are the scaling cost.
  * CompactExchange     (default in bench.py) the compact exchange overlapped with the backward: the row sums write
                        dL_dcolors before the per-Gaussian backward runs, the backward records an event there
                        (omr_backward_colors_event), and the colour all-gather starts on a side stream as soon as it
                        fires; the per-view dL_dsh is not written at all (skip_dsh), since the rebuild replaces it.
                        ar_chunks = k > 1 also pipelines the 44 B/G all-reduce: the per-Gaussian backward runs over k
                        Gaussian ranges with an event after each (omr_backward_chunk_events) and each range is
                        reduced on the side stream once final.
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
    # test-only: run the exchange's collectives even at world size 1 (tests/test_gpu_rccl_one_rank.py executes the
    # RCCL calls on a one-GPU box, where a 1-rank communicator makes every collective an identity)
    force_exchange: bool = False

    @property
    def enabled(self) -> bool:
        return self.world_size > 1 or self.force_exchange


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
        # dL_dcolors lives in the first P rows of a [P + 1, 3] tensor whose last row takes the camera position, so the
        # compact exchange gathers both with one collective (allreduce_compact_)
        self.colors_ext = None

    def out_dict(self, device):
        P = self.P
        if not self.extra:
            self.colors_ext = torch.empty((P + 1, 3), dtype=self.flat.dtype, device=device)
            self.extra = dict(dL_dmeans2D=torch.empty((P, 3), device=device),
                              dL_dcolors=self.colors_ext[:P],
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
                       average: bool = False, rebuild_packed=None):
    """Sum over ranks with the compact SH exchange (module docstring): all-reduce the 11 non-SH floats per
    Gaussian, all-gather every rank's dL_dcolors [P,3] with its campos [3] appended as row P (one collective), then
    rebuild the summed SH gradient into the dL_dsh view, either as
    rebuild_packed(packed_all [n,P+1,3], out=...) (rasterizer.sh_grad_from_colors_packed bound to the replicated
    means3D / SH / degree) or rebuild(campos_all [n,3], dcolors_all [n,P,3], out=...) (tests pass a CPU model)."""
    if not info.enabled:
        return
    n, P = info.world_size, buf.P
    prefix = buf.flat[:REDUCED_FLOATS * P]
    dist.all_reduce(prefix, op=dist.ReduceOp.SUM)
    ext = buf.colors_ext
    if ext is None or dL_dcolors.data_ptr() != ext.data_ptr():  # colours not written into the packed tensor
        ext = torch.empty((P + 1, 3), dtype=dL_dcolors.dtype, device=dL_dcolors.device)
        ext[:P].copy_(dL_dcolors.reshape(P, 3))
    ext[P].copy_(campos.reshape(3).to(ext.dtype))
    if dist.get_backend() == "nccl":
        packed_all = torch.empty((n, P + 1, 3), dtype=ext.dtype, device=ext.device)
        dist.all_gather_into_tensor(packed_all, ext)
    else:
        parts = [torch.empty_like(ext) for _ in range(n)]
        dist.all_gather(parts, ext)
        packed_all = torch.stack(parts)
    if rebuild_packed is not None:
        rebuild_packed(packed_all, out=buf.views["dL_dsh"])
    else:
        rebuild(packed_all[:, P].contiguous(), packed_all[:, :P].contiguous(), out=buf.views["dL_dsh"])
    if average:
        buf.flat.div_(n)


class CompactExchange:
    """allreduce_compact_ with the colour all-gather overlapped with the rest of the backward (module docstring).

    Per step: call the backward with **backward_kwargs(campos) (event + skip_dsh; campos = this step's camera
    position, copied into the gathered row P on the current stream BEFORE the backward is queued, so the all-gather
    behind the event sees it), then start() (queues the all-gather on a side stream behind the event), then finish()
    (all-reduce of the 44 B/G prefix on the current stream once the backward is done, then the SH rebuild behind both
    collectives). Over gloo (CPU rehearsals), or when `overlap` is False (e.g. a host that cannot pass the event), it
    falls back to allreduce_compact_ inside finish(). A trainer whose ranks change viewpoint every step must pass
    each step's campos: the SH rebuild evaluates the view directions from it."""

    def __init__(self, buf: GradBuffer, info: DistInfo, campos: torch.Tensor, rebuild_packed, device,
                 overlap: bool = True, any_backend: bool = False, ar_chunks: int = 1):
        self.buf, self.info, self.rebuild_packed = buf, info, rebuild_packed
        P = buf.P
        buf.out_dict(device)  # creates colors_ext [P + 1, 3]
        self.set_campos(campos)
        # any_backend: also overlap over gloo (ranks sharing one GPU in tests and `bench.py --rehearse`: the same
        # event / side-stream / collective sequence as over RCCL, with gloo's host copies)
        self.overlap = bool(overlap and info.enabled and (any_backend or dist.get_backend() == "nccl"))
        if self.overlap:
            self.event = torch.cuda.Event()
            self.comm = torch.cuda.Stream(device)
            self.packed_all = torch.empty((info.world_size, P + 1, 3), dtype=buf.colors_ext.dtype, device=device)
        # ar_chunks > 1: the 44 B/G all-reduce runs per Gaussian range on the side stream behind the colour all-gather,
        # each range as soon as the backward's per-Gaussian kernel has finished it (chunk events; DESIGN.md §6 on
        # when that can pay)
        self.ar_chunks = int(ar_chunks) if self.overlap else 1
        self.chunk_events, self.ranges = [], []
        if self.ar_chunks > 1:
            from . import rasterizer as _R  # the ranges the library uses (omr_backward_chunk_begin)

            self.chunk_events = [torch.cuda.Event() for _ in range(self.ar_chunks)]
            self.ranges = _R.backward_chunk_ranges(P, self.ar_chunks)

    def set_campos(self, campos: torch.Tensor):
        """This step's camera position: stream-ordered copy into row P of the gathered tensor (current stream)."""
        self.campos = campos
        self.buf.colors_ext[self.buf.P].copy_(campos.reshape(3).to(self.buf.colors_ext.dtype))

    def backward_kwargs(self, campos: torch.Tensor | None = None) -> dict:
        """Keyword arguments of this step's RasterizeGaussiansBackwardCUDA call; campos: this step's camera position
        (None = unchanged since the last step). Call before queueing the backward."""
        if campos is not None:
            self.set_campos(campos)
        if not self.overlap:
            return {}
        kw = dict(colors_event=self.event, skip_dsh=True)
        if self.chunk_events:
            kw["chunk_events"] = self.chunk_events
        return kw

    def start(self):
        if not self.overlap:
            return
        with torch.cuda.stream(self.comm):
            self.comm.wait_event(self.event)
            if dist.get_backend() == "nccl":
                dist.all_gather_into_tensor(self.packed_all, self.buf.colors_ext)
            else:  # gloo: list form
                dist.all_gather(list(self.packed_all.unbind(0)), self.buf.colors_ext)
            for ev, (b, e) in zip(self.chunk_events, self.ranges):  # ar_chunks > 1: each range once it is final
                self.comm.wait_event(ev)
                if e > b:
                    for name in SEGMENTS[:4]:
                        dist.all_reduce(self.buf.views[name][b:e], op=dist.ReduceOp.SUM)

    def finish(self):
        if not self.info.enabled:
            return
        if not self.overlap:
            allreduce_compact_(self.buf, self.info, self.buf.colors_ext[:self.buf.P], self.campos, None,
                               rebuild_packed=self.rebuild_packed)
            return
        if not self.chunk_events:
            dist.all_reduce(self.buf.flat[:REDUCED_FLOATS * self.buf.P], op=dist.ReduceOp.SUM)
        torch.cuda.current_stream().wait_stream(self.comm)
        self.rebuild_packed(self.packed_all, out=self.buf.views["dL_dsh"])


# ---- the scaling model of DESIGN.md §6, for a SCALE record to be checked against mechanically -------------------
# RCCL's bus bandwidth over xGMI, per link direction after protocol overhead: the ONE assumption of the model
# (uncertain by up to 2x; a SCALE record outside that band points at RCCL's behaviour)
XGMI_LINK_GBPS = 55.0
# links a ring of n ranks spreads one message over (a 2-GPU job has one link; 4 GPUs three; 8 GPUs six of seven)
XGMI_RING_LINKS = {2: 1, 4: 3, 8: 6}
HBM_GBPS = 6300.0  # achievable HBM bandwidth (MI355X_MICROARCH.md), for the SH rebuild's passes


def bus_gbps(n: int) -> float:
    return XGMI_LINK_GBPS * XGMI_RING_LINKS.get(n, max(1, min(n - 1, 6)))


def predict_step_ms(n: int, P: int, compute_ms_per_rank, gbwd_ms: float, exchange: str = "compact") -> dict:
    """step(n) = max over ranks of forward + backward, plus the exchange's tail past the per-Gaussian
    backward it overlaps. compact: t_AR = 2 (n-1)/n 44 B P / B(n), t_AG = (n-1) 12 B P / B(n) (each rank receives the
    n-1 other views' colour gradients), tail = (t_AR + t_AG - t_gbwd)+ + t_rebuild (n 12 + 384 B/G over HBM); flat:
    one all-reduce of 236 B/G after the backward. Returns the model's terms in ms."""
    n = int(n)
    comp = max(compute_ms_per_rank) if compute_ms_per_rank else 0.0
    if n <= 1:
        return dict(step_ms=comp, t_ar_ms=0.0, t_ag_ms=0.0, tail_ms=0.0, bus_GBps=None)
    B = bus_gbps(n) * 1e9
    if exchange == "compact":
        t_ar = 2 * (n - 1) / n * 44 * P / B * 1e3
        t_ag = (n - 1) * 12 * P / B * 1e3
        t_rb = (n * 12 + 384) * P / (HBM_GBPS * 1e9) * 1e3
        tail = max(0.0, t_ar + t_ag - gbwd_ms) + t_rb
    else:
        t_ar = 2 * (n - 1) / n * 236 * P / B * 1e3
        t_ag = 0.0
        tail = t_ar
    return dict(step_ms=comp + tail, t_ar_ms=t_ar, t_ag_ms=t_ag, tail_ms=tail, bus_GBps=B / 1e9)

"""View-parallel data parallelism (omnigs-fork_amd/parallel.py) on CPU with gloo, world_size 2.

Each rank renders its own view of the same Gaussians (gradients from the CPU oracle standing in for the HIP
backward, which needs a GPU), writes them into the flat GradBuffer views and all-reduces. Checked: the reduced
buffer equals the sum of the per-view gradients computed sequentially (SURVEY.md §8(e) parity), for a single
collective and for bucketed collectives, and the mean variant.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _view_grads(view):
    import sys

    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
    import _omnigs

    _omnigs.load()
    from helpers import make_case, oracle_run

    g, cam, dL = make_case(300, 64, 32, 3, 77, view_index=view, spread=3.0)
    _, _, gr = oracle_run(g, cam, dL)
    return {"dL_dmeans3D": gr["dmean3D"], "dL_dsh": gr["dsh"], "dL_dopacity": gr["dopacity"],
            "dL_dscales": gr["dscale"], "dL_drotations": gr["drot"]}


def _worker(rank, world, port, bucket, average, q):
    import sys

    sys.path[:0] = [ROOT]
    import torch
    import torch.distributed as dist

    import _omnigs

    par = _omnigs.load().parallel
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        grads = _view_grads(rank)
        buf = par.GradBuffer(300, 16, torch.device("cpu"))
        for k, v in buf.views.items():
            v.copy_(torch.from_numpy(grads[k]))
        par.allreduce_(buf, par.DistInfo(rank, world, rank), average=average, bucket_bytes=bucket)
        q.put((rank, {k: v.numpy().copy() for k, v in buf.views.items()}))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("bucket,average", [(0, False), (4096, False), (0, True)])
def test_allreduce_equals_sum_of_views(bucket, average, oracle_mod):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, bucket, average, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    g0, g1 = _view_grads(0), _view_grads(1)
    for k in g0:
        ref = g0[k] + g1[k]
        if average:
            ref = ref / 2
        for r in (0, 1):
            np.testing.assert_allclose(res[r][k], ref, rtol=1e-6, atol=1e-9, err_msg=f"{k} rank {r}")


def test_gradbuffer_layout():
    import sys

    sys.path[:0] = [ROOT]
    import torch

    import _omnigs

    par = _omnigs.load().parallel
    b = par.GradBuffer(10, 16, torch.device("cpu"))
    assert b.flat.numel() == 10 * 59  # 236 B per Gaussian
    off = 0
    for k in par.SEGMENTS:
        v = b.views[k]
        assert v.is_contiguous() and v.data_ptr() == b.flat.data_ptr() + 4 * off
        off += v.numel()

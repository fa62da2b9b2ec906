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
            "dL_dscales": gr["dscale"], "dL_drotations": gr["drot"], "dL_dcolors": gr["dcolor"],
            "campos": cam.campos, "means3D": g.means3D, "shs": g.shs, "deg": g.sh_degree}


def _worker(rank, world, port, bucket, average, q, compact=False):
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
        info = par.DistInfo(rank, world, rank)
        if compact:
            sys.path[:0] = [os.path.join(ROOT, "tests")]
            from helpers import sh_grad_from_colors_np

            def rebuild(campos_all, dcolors_all, out):
                out.copy_(torch.from_numpy(sh_grad_from_colors_np(grads["means3D"], grads["shs"], grads["deg"],
                                                                  campos_all.numpy(), dcolors_all.numpy())))

            if compact == "cx":  # parallel.CompactExchange: over gloo it takes the non-overlapped path
                def rebuild_packed(pk, out):
                    rebuild(pk[:, buf.P].contiguous(), pk[:, :buf.P].contiguous(), out)

                cx = par.CompactExchange(buf, info, torch.from_numpy(grads["campos"]), rebuild_packed,
                                         torch.device("cpu"))
                assert not cx.overlap and cx.backward_kwargs() == {}
                buf.colors_ext[:buf.P].copy_(torch.from_numpy(grads["dL_dcolors"]))  # the backward's output slot
                cx.start()
                cx.finish()
            else:
                par.allreduce_compact_(buf, info, torch.from_numpy(grads["dL_dcolors"]),
                                       torch.from_numpy(grads["campos"]), rebuild, average=average)
        else:
            par.allreduce_(buf, info, average=average, bucket_bytes=bucket)
        q.put((rank, {k: v.numpy().copy() for k, v in buf.views.items()}))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("bucket,average,compact", [(0, False, False), (4096, False, False), (0, True, False),
                                                    (0, False, True), (0, True, True), (0, False, "cx")])
def test_allreduce_equals_sum_of_views(bucket, average, compact, oracle_mod):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, bucket, average, q, compact)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    g0, g1 = _view_grads(0), _view_grads(1)
    for k in ("dL_dmeans3D", "dL_dsh", "dL_dopacity", "dL_dscales", "dL_drotations"):
        ref = g0[k] + g1[k]
        if average:
            ref = ref / 2
        # the compact exchange rebuilds the SH sum in float64 here (the HIP rebuild is checked bitwise on the GPU)
        rtol, atol = (1e-5, 1e-8) if compact and k == "dL_dsh" else (1e-6, 1e-9)
        for r in (0, 1):
            np.testing.assert_allclose(res[r][k], ref, rtol=rtol, atol=atol, err_msg=f"{k} rank {r}")
    if compact:  # every rank holds the identical sum
        for k in res[0]:
            np.testing.assert_array_equal(res[0][k], res[1][k])


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


def test_scaling_model_matches_design_table():
    """parallel.predict_step_ms restates DESIGN.md §6's model (bench.py reports it at N > 1 as `predicted`): config D
    at P = 1 M with 1.11 ms per-rank compute and gaussian_bwd 0.11 ms — t_AR / t_AG as in the DESIGN table, and a
    single GPU is just its compute."""
    import _omnigs

    par = _omnigs.load().parallel
    P = 1_000_000
    one = par.predict_step_ms(1, P, [1.11], 0.11)
    assert one["step_ms"] == 1.11 and one["tail_ms"] == 0.0
    for n, ar, ag in ((2, 0.80, 0.22), (4, 0.40, 0.22), (8, 0.23, 0.25)):
        r = par.predict_step_ms(n, P, [1.11] * n, 0.11)
        assert abs(r["t_ar_ms"] - ar) < 0.01 and abs(r["t_ag_ms"] - ag) < 0.01, (n, r)
        assert r["step_ms"] > 1.11 and r["tail_ms"] >= r["t_ar_ms"] + r["t_ag_ms"] - 0.11
    flat = par.predict_step_ms(8, P, [1.11] * 8, 0.11, exchange="flat")
    assert flat["step_ms"] > par.predict_step_ms(8, P, [1.11] * 8, 0.11)["step_ms"]

"""The view-parallel exchange over REAL RCCL on a one-GPU box.

A 1-rank `nccl` process group (RCCL on ROCm), initialised as bench.py does (`device_id=`), with the test-only
DistInfo.force_exchange so the exchange code runs at world size 1. Over one rank every collective is an identity, so
after each exchange the gradient buffer must equal, bit for bit, the same view's backward without any exchange:

  * allreduce_            one all_reduce of the flat 236 B/G buffer (and in buckets);
  * allreduce_compact_    all_reduce of the 44 B/G prefix + all_gather_into_tensor of the packed colour gradients,
                          then the SH gradient rebuilt from them (omr_sh_grad_from_colors_packed);
  * CompactExchange       the overlapped form: the backward's colours event, the all-gather on a side stream waiting on
                          it, skip_dsh, the all-reduce on the compute stream, the stream join and the rebuild; with
                          ar_chunks 1 and 3 (per-range all-reduces behind the backward's chunk events).

The child process runs everything (a process group per process); the parent checks the results.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _worker(port, q):
    import torch
    import torch.distributed as dist

    sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
    import _omnigs
    from helpers import make_case, scene

    omr = _omnigs.load()
    R, par = omr.rasterizer, omr.parallel
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    out_q = {"backend": dist.get_backend(), "nccl_version": ".".join(map(str, torch.cuda.nccl.version()))}
    try:
        g, cam, dL = make_case(7000, 256, 128, scene.CAMERA_LONLAT, 41, view_index=3, spread=2.0)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).to(dev)  # noqa: E731
        m, sh = t(g.means3D), t(g.shs)
        op, sc, rot = t(g.opacity), t(g.scales), t(g.rotations)
        vm, pm, cp, bg, e = t(cam.viewmatrix), t(cam.projmatrix), t(cam.campos), torch.zeros(3, device=dev), \
            torch.empty(0, device=dev)
        info = par.DistInfo(0, 1, 0, force_exchange=True)
        assert info.enabled

        def backward(buf, **kw):
            nr, color, radii, gb, bb, ib = R.RasterizeGaussiansCUDA(bg, m, e, op, sc, rot, 1.0, e, vm, pm,
                                                                    cam.tanfovx, cam.tanfovy, cam.height, cam.width,
                                                                    sh, g.sh_degree, cp, False, cam.camera_type, False)
            out = buf.out_dict(dev)
            R.RasterizeGaussiansBackwardCUDA(bg, m, radii, e, sc, rot, 1.0, e, vm, pm, cam.tanfovx, cam.tanfovy,
                                             t(dL), sh, g.sh_degree, cp, gb, nr, bb, ib, cam.camera_type, out=out, **kw)

        rebuild = lambda pk, out: R.sh_grad_from_colors_packed(m, sh, g.sh_degree, pk, out=out)  # noqa: E731
        ref = par.GradBuffer(g.P, g.shs.shape[1], dev)
        backward(ref)  # no exchange at all
        torch.cuda.synchronize()
        res = {"ref": ref.flat.cpu().numpy()}

        buf = par.GradBuffer(g.P, g.shs.shape[1], dev)
        backward(buf)
        par.allreduce_(buf, info)
        torch.cuda.synchronize()
        res["allreduce"] = buf.flat.cpu().numpy()
        par.allreduce_(buf, info, bucket_bytes=1 << 20)  # buckets: identity again
        torch.cuda.synchronize()
        res["allreduce_buckets"] = buf.flat.cpu().numpy()

        buf = par.GradBuffer(g.P, g.shs.shape[1], dev)
        backward(buf)
        buf.views["dL_dsh"].fill_(float("nan"))  # the rebuild must write every SH gradient element
        par.allreduce_compact_(buf, info, buf.colors_ext[:g.P], cp, None, rebuild_packed=rebuild)
        torch.cuda.synchronize()
        res["compact"] = buf.flat.cpu().numpy()

        for chunks in (1, 3):
            buf = par.GradBuffer(g.P, g.shs.shape[1], dev)
            cx = par.CompactExchange(buf, info, cp, rebuild, dev, ar_chunks=chunks)
            assert cx.overlap and cx.ar_chunks == chunks  # nccl: the overlapped path
            for step in range(2):  # the event, the side stream and the buffers are reused across steps
                buf.views["dL_dsh"].fill_(float("nan"))
                backward(buf, **cx.backward_kwargs(cp))
                cx.start()
                cx.finish()
            torch.cuda.synchronize()
            res[f"overlap_{chunks}"] = buf.flat.cpu().numpy()
        out_q.update(res)
        out_q["P"] = g.P
    finally:
        dist.destroy_process_group()
    q.put(out_q)


def test_exchange_over_rccl_one_rank_is_bitwise_identity():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(port, q))
    p.start()
    res = q.get(timeout=300)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert res["backend"] == "nccl"
    print(f"RCCL {res['nccl_version']} over backend {res['backend']}")
    ref = res["ref"]
    assert np.isfinite(ref).all()
    for k in ("allreduce", "allreduce_buckets", "compact", "overlap_1", "overlap_3"):
        np.testing.assert_array_equal(res[k], ref, err_msg=k)

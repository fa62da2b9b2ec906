"""parallel.CompactExchange's overlapped path on ONE GPU: 2 ranks over gloo, both on cuda:0 (any_backend=True runs
the same event / side-stream / collective sequence the RCCL path runs). Each rank renders its own view and calls the
backward with the colours event and skip_dsh; after start() / finish() both ranks must hold, bit for bit, the sum of
the two views' 44 B/G gradients and the SH gradient rebuilt from both views' colour gradients, which equals the sum
of the per-view SH gradients (tests/test_gpu_parallel.py)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _case(view):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
    from helpers import make_case, scene

    return make_case(6000, 256, 128, scene.CAMERA_LONLAT, 23, view_index=view, spread=2.0)


def _worker(rank, world, port, q, move_view=False, ar_chunks=1):
    import torch
    import torch.distributed as dist

    sys.path[:0] = [ROOT]
    import _omnigs

    omr = _omnigs.load()
    R, par = omr.rasterizer, omr.parallel
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        g, cam, dL = _case(rank)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).to(dev)  # noqa: E731
        m, sh = t(g.means3D), t(g.shs)
        vm, pm, cp, bg, e = t(cam.viewmatrix), t(cam.projmatrix), t(cam.campos), torch.zeros(3, device=dev), \
            torch.empty(0, device=dev)
        buf = par.GradBuffer(g.P, g.shs.shape[1], dev)
        out = buf.out_dict(dev)
        cx = par.CompactExchange(buf, par.DistInfo(rank, world, 0), cp,
                                 lambda pk, out: R.sh_grad_from_colors_packed(m, sh, g.sh_degree, pk, out=out), dev,
                                 any_backend=True, ar_chunks=ar_chunks)
        assert cx.overlap and cx.ar_chunks == ar_chunks
        for step in range(2):  # twice: the event and the buffers are reused across steps
            if move_view and step == 1:  # the second step renders another viewpoint (rank + 2): campos changes
                g, cam, dL = _case(rank + 2)
                vm, pm, cp = t(cam.viewmatrix), t(cam.projmatrix), t(cam.campos)
            nr, color, radii, gb, bb, ib = R.RasterizeGaussiansCUDA(bg, m, e, t(g.opacity), t(g.scales),
                                                                    t(g.rotations), 1.0, e, vm, pm, cam.tanfovx,
                                                                    cam.tanfovy, cam.height, cam.width, sh,
                                                                    g.sh_degree, cp, False, cam.camera_type, False)
            R.RasterizeGaussiansBackwardCUDA(bg, m, radii, e, t(g.scales), t(g.rotations), 1.0, e, vm, pm,
                                             cam.tanfovx, cam.tanfovy, t(dL), sh, g.sh_degree, cp, gb, nr, bb, ib,
                                             cam.camera_type, out=out, **cx.backward_kwargs(cp))
            cx.start()
            cx.finish()
        torch.cuda.synchronize()
        q.put((rank, {k: v.cpu().numpy() for k, v in buf.views.items()}))
    finally:
        dist.destroy_process_group()


def _run(move_view, ar_chunks=1):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, move_view, ar_chunks)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for k in res[0]:
        np.testing.assert_array_equal(res[0][k], res[1][k], err_msg=k)  # identical replicas
    import torch

    sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
    from helpers import hip_run, to_np

    views = (2, 3) if move_view else (0, 1)  # the last step's views
    h = [hip_run(*_case(v)) for v in views]
    names = {"dL_dmeans3D": "dmean3D", "dL_dopacity": "dopacity", "dL_dscales": "dscale", "dL_drotations": "drot",
             "dL_dsh": "dsh"}
    for k, n in names.items():
        ref = (h[0]["grads"][n] + h[1]["grads"][n]).reshape(res[0][k].shape)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(res[0][k], to_np(ref), err_msg=k)


def test_overlapped_compact_exchange_sums_views_bitwise():
    _run(move_view=False)


def test_overlapped_exchange_follows_a_moving_camera():
    """the gathered camera position must be each step's (the SH rebuild evaluates view directions from
    it); the second step renders other viewpoints and must equal the per-view sums of THAT step bitwise."""
    _run(move_view=True)


def test_pipelined_all_reduce_over_gaussian_ranges_sums_views_bitwise():
    """ar_chunks = 3 runs the per-Gaussian backward over three Gaussian ranges (omr_backward_chunk_
    events) and all-reduces each range's 44 B/G on the side stream as soon as its event fires; the replicas must
    equal the per-view sums bit for bit, as with one all-reduce."""
    import _omnigs

    ranges = _omnigs.load().rasterizer.backward_chunk_ranges(6000, 3)
    assert ranges == [(0, 1792), (1792, 3840), (3840, 6000)]  # multiples of 256, covering [0, P)
    _run(move_view=True, ar_chunks=3)

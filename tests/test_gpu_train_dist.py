"""View-parallel training step (trainer.train_step with dist_info) on ONE GPU: 2 ranks over gloo, both on cuda:0
(the exchange path of bench.py --rehearse). Each rank renders its own view; after the compact exchange every rank
must take the same Adam step: parameters identical on both ranks, and bitwise equal to a single-process step on the
summed gradients of both views.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _setup(view, dev):
    import torch

    sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
    import _omnigs

    omr = _omnigs.load()
    from helpers import make_case

    g, cam, _ = make_case(4000, 192, 96, omr.scene.CAMERA_LONLAT, 5, view_index=view, spread=2.0)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).to(dev)  # noqa: E731
    model = omr.renderer.GaussianModelParams.from_activated(t(g.means3D), t(g.scales), t(g.rotations),
                                                            t(g.opacity).reshape(-1, 1), t(g.shs), 3)
    for name in ("xyz", "features_dc", "features_rest", "opacity", "scaling", "rotation"):
        setattr(model, name, getattr(model, name).contiguous())
    vp = omr.renderer.Viewpoint(t(cam.viewmatrix), t(cam.projmatrix), t(cam.campos))
    gen = torch.Generator(device=dev).manual_seed(100 + view)
    gt = torch.rand((3, 96, 192), device=dev, generator=gen)
    return omr, model, vp, gt


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        omr, model, vp, gt = _setup(rank, dev)
        opt = omr.optim.GaussianOptimizer(model, omr.optim.OptimizationParams())
        info = omr.parallel.DistInfo(rank, world, 0)
        state = omr.trainer.TrainStep()
        bg = torch.zeros(3, device=dev)
        for it in range(2):
            omr.trainer.train_step(opt, vp, 96, 192, gt, bg, state=state, dist_info=info)
        opt.sync_densification_stats(info)
        torch.cuda.synchronize()
        q.put((rank, [p.cpu().numpy() for p in opt.params()], opt.denom.cpu().numpy()))
    finally:
        dist.destroy_process_group()


def test_view_parallel_train_step_replicas_agree_with_summed_views():
    import torch

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (ps, den)) for r, ps, den in (q.get(timeout=300) for _ in procs))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for a, b in zip(res[0][0], res[1][0]):
        np.testing.assert_array_equal(a, b)  # replicas identical
    np.testing.assert_array_equal(res[0][1], res[1][1])
    # single process: both views' rasterizer gradients summed, then one Adam step per iteration
    dev = torch.device("cuda", 0)
    omr, model, vp0, gt0 = _setup(0, dev)
    _, _, vp1, gt1 = _setup(1, dev)
    opt = omr.optim.GaussianOptimizer(model, omr.optim.OptimizationParams())
    R = omr.rasterizer
    bg = torch.zeros(3, device=dev)
    for it in range(2):
        total = None
        # the trainer's activations (omr_activate), checked here against torch's independent expressions
        # (gaussian_model.cpp:54-77) so this test does not rest on the kernel it is comparing the trainer with
        a = opt.activate()
        m = opt.model
        assert torch.equal(a["shs"], torch.cat([m.features_dc, m.features_rest], dim=1))
        assert torch.equal(a["opacity"], torch.sigmoid(m.opacity))
        assert torch.equal(a["scales"], torch.exp(m.scaling))
        torch.testing.assert_close(a["rotations"], torch.nn.functional.normalize(m.rotation), rtol=2.4e-7, atol=0)
        shs = a["shs"]
        act = (a["xyz"], a["opacity"], a["scales"], a["rotations"])
        for vp, gt in ((vp0, gt0), (vp1, gt1)):
            nr, img, radii, gb, bb, ib = R.RasterizeGaussiansCUDA(bg, act[0], None, act[1], act[2], act[3], 1.0, None,
                                                                  vp.world_view_transform, vp.full_proj_transform,
                                                                  0.0, 0.0, 96, 192, shs, 3, vp.camera_center, False,
                                                                  R.CAMERA_LONLAT)
            _, dimg = omr.losses.l1_ssim_loss_and_grad(img, gt, 0.2)
            gr = R.RasterizeGaussiansBackwardCUDA(bg, act[0], radii, None, act[2], act[3], 1.0, None,
                                                  vp.world_view_transform, vp.full_proj_transform, 0.0, 0.0, dimg,
                                                  shs, 3, vp.camera_center, gb, nr, bb, ib, R.CAMERA_LONLAT)
            d = {"dL_dmeans3D": gr[3], "dL_dsh": gr[5], "dL_dopacity": gr[2], "dL_dscales": gr[6],
                 "dL_drotations": gr[7]}
            total = d if total is None else {k: total[k] + d[k] for k in d}
        opt.step(raster_grads={k: v.contiguous() for k, v in total.items()})
    torch.cuda.synchronize()
    for k, (p, ref) in enumerate(zip(opt.params(), res[0][0])):
        # bitwise: the compact exchange sums two views exactly as the single process does (all-reduce of two floats;
        # the SH rebuild equals the sum of the per-view SH gradients bit for bit, tests/test_gpu_parallel.py), and
        # every kernel is deterministic
        np.testing.assert_array_equal(ref, p.detach().cpu().numpy(), err_msg=f"parameter group {k}")

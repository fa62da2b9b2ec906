"""Config D (1 M Gaussians, eight equirect views, one per GPU; BASELINE.json) and config E (5 M Gaussians, a mixed
batch: four 4096x2048 equirect views on ranks 0-3, four 1920x1080 pinhole views on ranks 4-7, as bench.py places
them) through the real exchange code: eight ranks over gloo, all on cuda:0 (the one-GPU box's stand-in for the 8-GPU node the driver's scaling run uses). Each
rank renders its view of the config's scene, runs the HIP backward into its GradBuffer and calls
parallel.allreduce_compact_ (the exchange bench.py runs at N > 1: all-reduce of the 44 B/G xyz / opacity / scale /
rotation gradients, all-gather of every view's colour gradient and camera position, SH gradient rebuilt on every
rank), and through the overlapped parallel.CompactExchange that bench.py runs by default (colour all-gather on a side
stream behind the backward's colours event, dL_dsh not written by the backward; ar_chunks 1 and 3, the latter
all-reducing the 44 B/G per Gaussian range behind the chunk events). Every exchange is checked
against the eight per-view HIP gradients computed one after another in this process:
  * every rank holds the same buffer, bit for bit;
  * the 44 B/G part equals the per-view sum to float32 summation-order error (gloo's ring adds the eight views in
    another order than a sequential loop: |diff| <= 8 ulp of the sum of magnitudes);
  * the SH part equals, bit for bit, the rebuild from the eight gathered colour gradients in view order, and that
    rebuild equals the sequential sum of the per-view SH gradients bit for bit (same arithmetic, same order).
"""
import hashlib
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORLD = 8
NAMES = {"dL_dmeans3D": "dmean3D", "dL_dopacity": "dopacity", "dL_dscales": "dscale", "dL_drotations": "drot"}


def _scene_name(config, rank):
    """bench.py's placement: config E puts the second half of the ranks on pinhole views of the same scene."""
    if config == "E":
        return "E" if rank < WORLD // 2 else "E_pinhole"
    return config


MODES = ("call", "overlap1", "overlap3")  # allreduce_compact_ after the backward; CompactExchange, ar_chunks 1 / 3


def _worker(rank, world, port, q, tmpdir, config):
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
        g, cam, dL = omr.scene.config_scene(_scene_name(config, rank), view_index=rank)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).to(dev)  # noqa: E731
        m, sh = t(g.means3D), t(g.shs)
        vm, pm, cp, bg, e = t(cam.viewmatrix), t(cam.projmatrix), t(cam.campos), torch.zeros(3, device=dev), \
            torch.empty(0, device=dev)
        op, sc, rot, dLt = t(g.opacity), t(g.scales), t(g.rotations), t(dL)
        info = par.DistInfo(rank, world, 0)
        rebuild = lambda pk, out: R.sh_grad_from_colors_packed(m, sh, g.sh_degree, pk, out=out)  # noqa: E731
        digests = {}
        for mode in MODES:
            buf = par.GradBuffer(g.P, g.shs.shape[1], dev)
            buf.flat.fill_(float("nan"))  # every element must be written by the backward or the exchange
            out = buf.out_dict(dev)
            cx = None
            if mode != "call":
                cx = par.CompactExchange(buf, info, cp, rebuild, dev, any_backend=True, ar_chunks=int(mode[-1]))
                assert cx.overlap and cx.ar_chunks == int(mode[-1])
            nr, color, radii, gb, bb, ib = R.RasterizeGaussiansCUDA(bg, m, e, op, sc, rot, 1.0, e, vm, pm, cam.tanfovx,
                                                                    cam.tanfovy, cam.height, cam.width, sh,
                                                                    g.sh_degree, cp, False, cam.camera_type, False)
            R.RasterizeGaussiansBackwardCUDA(bg, m, radii, e, sc, rot, 1.0, e, vm, pm, cam.tanfovx, cam.tanfovy, dLt,
                                             sh, g.sh_degree, cp, gb, nr, bb, ib, cam.camera_type, out=out,
                                             **(cx.backward_kwargs(cp) if cx else {}))
            if cx is None:
                torch.cuda.synchronize()
                par.allreduce_compact_(buf, info, out["dL_dcolors"], cp, None, rebuild_packed=rebuild)
            else:
                cx.start()
                cx.finish()
            torch.cuda.synchronize()
            flat = buf.flat.cpu().numpy()
            if rank == 0:
                np.save(os.path.join(tmpdir, f"flat0_{mode}.npy"), flat)
            digests[mode] = hashlib.sha1(flat.tobytes()).hexdigest()
            del buf, out, cx, gb, bb, ib
        q.put((rank, digests))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("config", ["D", "E"])
def test_config_eight_ranks_compact_exchange(config, tmp_path, capsys):
    """allreduce_compact_ after the backward and the overlapped CompactExchange (ar_chunks 1, 3) at eight ranks."""
    import queue
    import time

    import torch

    t0 = time.monotonic()

    def progress(what):  # a line past pytest's capture every half minute: config E runs for minutes without output
        with capsys.disabled():
            print(f"\n  [{config}, {time.monotonic() - t0:.0f} s] {what}", flush=True)

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, WORLD, port, q, str(tmp_path), config)) for r in range(WORLD)]
    for p in procs:
        p.start()
    digests, last = {}, time.monotonic()
    while len(digests) < WORLD:
        try:
            r, d = q.get(timeout=30)
            digests[r] = d
        except queue.Empty:
            assert time.monotonic() - t0 < 600, f"{WORLD - len(digests)} ranks silent after 600 s"
        if time.monotonic() - last >= 30:
            progress(f"{len(digests)} of {WORLD} ranks done")
            last = time.monotonic()
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for mode in MODES:
        per_rank = {r: d[mode] for r, d in digests.items()}
        assert len(set(per_rank.values())) == 1, (mode, per_rank)  # identical replicas, bit for bit

    sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
    from helpers import hip_run, omr, to_np

    R, par = omr.rasterizer, omr.parallel
    sums, mags, dsh_seq, dcolors, campos = None, None, None, [], []
    for v in range(WORLD):
        progress(f"sequential reference, view {v}")
        g, cam, dL = omr.scene.config_scene(_scene_name(config, v), view_index=v)
        h = hip_run(g, cam, dL)
        gr = h["grads"]
        part = np.concatenate([to_np(gr[NAMES[k]]).reshape(g.P, -1) for k in NAMES], axis=1).astype(np.float64)
        sums = part if sums is None else sums + part
        mags = np.abs(part) if mags is None else mags + np.abs(part)
        dsh_seq = gr["dsh"].clone() if dsh_seq is None else dsh_seq + gr["dsh"]
        dcolors.append(gr["dcolor"].clone())
        campos.append(torch.from_numpy(cam.campos).cuda())
        del h, gr
    P = g.P
    dev = dsh_seq.device
    packed = torch.cat([torch.stack(dcolors), torch.stack(campos)[:, None, :]], dim=1).contiguous()
    rebuilt = R.sh_grad_from_colors_packed(torch.from_numpy(g.means3D).to(dev), torch.from_numpy(g.shs).to(dev),
                                           g.sh_degree, packed)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(to_np(rebuilt), to_np(dsh_seq))
    tol = 8 * np.finfo(np.float32).eps * mags + np.finfo(np.float32).tiny
    for mode in MODES:
        buf = par.GradBuffer(P, g.shs.shape[1], torch.device("cpu"))
        buf.flat.copy_(torch.from_numpy(np.load(os.path.join(str(tmp_path), f"flat0_{mode}.npy"))))
        assert not torch.isnan(buf.flat).any(), mode
        got = np.concatenate([buf.views[k].numpy().reshape(P, -1) for k in NAMES], axis=1).astype(np.float64)
        bad = np.abs(got - sums) > tol
        assert not bad.any(), f"{mode}: {int(bad.sum())} entries of the 44 B/G sum off by more than 8 ulp"
        np.testing.assert_array_equal(buf.views["dL_dsh"].numpy(), to_np(rebuilt), err_msg=mode)

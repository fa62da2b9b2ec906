#!/usr/bin/env python3
"""bench.py — BASELINE.json metric: Mpixels/s of one rasterizer forward + backward, 1M Gaussians @ 2048x1024
equirect (config C), on 1/2/4/8 MI355X (config D: one view per GPU + RCCL all-reduce of the Gaussian gradients).

A "step" = RasterizeGaussiansCUDA + RasterizeGaussiansBackwardCUDA on one view with a fixed upstream gradient
(BASELINE.md §2), plus, for N > 1, the sum all-reduce of the flat per-Gaussian gradient buffer (236 B/Gaussian).
Inputs are synthetic (SplitMix64) and resident in HBM before timing starts.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 --master-port P \
        bench.py --gpus N --steps K --warmup W

`python bench.py --gpus N` with N > 1 and no WORLD_SIZE in the environment launches the N ranks itself (a child
torch.distributed.run, before anything touches the GPU) and exits with its status.

Rank 0 prints ONE JSON line (the driver's contract), with `roofline` for the dominant kernel (the stage with the
largest measured time; HIP events on the launch stream over the timed region) and, at N = 1, `cpu_baseline` (the CPU
oracle on a bounded sample: medians of >= 10 runs, all cores and one thread).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, Chip-level parameters)
VALU_PEAK_TFLOPS = 157.3  # MI355X f32 vector peak with v_pk_fma_f32 (MI355X_MICROARCH.md, MFMA/VALU peak table)
# VALU issue roofline: 256 CUs x 4 SIMDs, each issuing one wave64 VALU instruction per 2 cycles at 2.4 GHz
# (MI355X_MICROARCH.md: "issues each VALU instruction over 2 cycles")
VALU_SIMDS = 1024
VALU_ISSUE_PER_SIMD = 1.2e9


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--config", default="C", help="scene config of omnigs-fork_amd/scene.py (default C)")
    p.add_argument("--gaussians", type=int, default=None, help="override P (testing only)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=45.0,
                   help="CPU-oracle time budget per leg (runs stop early past it, after at least 3)")
    p.add_argument("--cpu-threads", type=int, default=None)
    p.add_argument("--bucket-mb", type=float, default=0.0, help="all-reduce bucket size (0 = one collective)")
    p.add_argument("--exchange", choices=["compact", "flat"], default="compact",
                   help="N > 1 gradient exchange: compact = all-reduce of the 44 B/G non-SH gradients + all-gather of "
                        "12 B/G colour gradients and an SH rebuild (parallel.allreduce_compact_); flat = one "
                        "all-reduce of all 236 B/G")
    p.add_argument("--ar-chunks", type=int, default=1,
                   help="compact exchange: all-reduce the 44 B/G gradients per Gaussian range, each as soon as the "
                        "backward finishes it (1 = one all-reduce after the backward; DESIGN.md §6)")
    p.add_argument("--boundary", choices=["ctypes", "libtorch"], default="ctypes",
                   help="ctypes: Python host on the C ABI (writes grads into the flat all-reduce buffer); libtorch: "
                        "the rasterize_points.h drop-in (librasterize_points.so) through its pybind module")
    p.add_argument("--rehearse", action="store_true",
                   help="multi-rank rehearsal on a one-GPU box: every rank on cuda:0, gloo instead of RCCL "
                        "(exercises the N > 1 code path; numbers are not a scaling measurement)")
    p.add_argument("--scene", default=None, help="override the scene of this rank (e.g. E_pinhole)")
    p.add_argument("--no-train-step", action="store_true",
                   help="skip the extra whole-training-iteration timing (N = 1 only; not part of `value`)")
    p.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "pmc_latest.json"))
    p.add_argument("--ambiguity-json", default=os.path.join(ROOT, "profiles", "ambiguity.json"),
                   help="parity allowance counts per config and the FMA-contracted reference proxies' differences "
                        "(oracle/contraction.py), reported as "
                        "config.ambiguous")
    p.add_argument("--cpu-runs", type=int, default=10, help="CPU-oracle runs per baseline leg (median reported)")
    p.add_argument("--cpu-single-config", default="B",
                   help="config of the one-thread CPU leg (one thread at config C takes ~30 s per run)")
    p.add_argument("--dist-check", action="store_true",
                   help="no GPU: only the N-rank launch and rendezvous (gloo), checking the world size; for tests")
    return p.parse_args()


def free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_ranks(n: int) -> int:
    """`bench.py --gpus N` run directly (no WORLD_SIZE): start N ranks under torch.distributed.run as a child process
    (nothing here has touched the GPU) and return its exit status."""
    import subprocess

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "4")
    print(f"[bench] launching {n} ranks: {' '.join(cmd[1:6])} ...", file=sys.stderr, flush=True)
    return subprocess.run(cmd, env=env).returncode


def dist_check(args) -> int:
    """--dist-check: the multi-rank path without a GPU (gloo): world size, ranks, per-rank timing gather."""
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
        world = dist.get_world_size()
    if world != args.gpus:
        print(f"[bench] world size {world} != --gpus {args.gpus}", file=sys.stderr)
        return 3
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    per_rank = [torch.zeros(1, dtype=torch.float64) for _ in range(world)]
    if world > 1:
        dist.all_gather(per_rank, t)
    else:
        per_rank = [t]
    if rank == 0:
        print(json.dumps({"n_gpus": world, "ranks_seen": world, "per_rank": [float(x.item()) for x in per_rank]}),
              flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


def stage_bytes(stage, P, V, L, N, T, M=16, D=3, rows=None):
    """Algorithmic HBM bytes of one launch of each stage (SURVEY.md §8(d) accounting). rows = the row
    binning's row-slot count M_r (bin.hip; None: sort.hip's emit + tile sort + ranges)."""
    sh = 12 * (D + 1) ** 2
    kb = 2 if T <= 65536 else 4  # tile-id bytes: 16-bit keys up to 65536 tiles (capi.hip: keys16)
    if rows is not None:
        # bin.hip, all timed as tile_sort: the rows pass reads each visible rank's row offset and depth-ordered rect
        # word twice (hist, scatter) and its Gaussian index once (28 B) and writes M_r row entries (Gaussian, width |
        # x0, first instance slot: 12 B); the columns pass reads the entries' slot and width (hist, 8 B) and the whole
        # entry plus its Gaussian's 32-B bin record (scatter, 44 B), writes the point list and row_valid (5 B per
        # instance) and the ranges (8 B per tile)
        binning = 28 * V + 64 * rows + 5 * L + 8 * T
        emit, tile_sort, tile_ranges = 0, binning, 16 * T  # tile_ranges: the render schedule (tile_order) only
    else:
        emit = 8 * P + 12 * V + (kb + 4) * L
        tile_sort = 2 * 2 * (kb + 4) * L           # 2 passes x (tile id + point-list entry, read + write)
        tile_ranges = kb * L + 16 * T
    return {
        # + the 8-B rect word, the 32-B bin record and the 36-B dRGB/ddir (sh_jac) for gaussian_bwd
        "preprocess": 32 * P + (40 + sh + 45 + 40 + 36) * V,
        "depth_sort": 4 * 2 * 8 * P,               # 4 passes x (key+value read + write)
        # order, tiles_touched (index order) and row_first; sort path: tiles_touched in depth order and offsets; row
        # path: the 8-B rect words in depth order (read and written) and row_offsets
        "scan": 12 * P + (8 * P if rows is None else 20 * P),
        "emit": emit,
        "tile_sort": tile_sort,
        "tile_ranges": tile_ranges,
        "render_forward": 40 * L + 20 * N + 8 * T,
        "render_backward": 40 * L + 20 * N + 8 * T + 88 * V,
        # tiles_touched + row_first + row_valid bytes + one 36-B sum row written per Gaussian; the marked 36-B
        # instance rows it reads depend on the scene and are not counted
        "row_sums": 8 * P + L + 36 * P,
        # reads radii 4P + (row sums 36, xyz 12, scale 12, rot 16, the forward's dRGB/ddir 36 in place of the SH row,
        # clamped 1) per visible Gaussian; writes every gradient output: 3+3+1+3+6+3*M(coeffs)+3+4 floats per Gaussian
        "gaussian_backward": 4 * P + (36 + 12 + 12 + 16 + 36 + 1) * V + (92 + 12 * M) * P,
    }.get(stage, 0)


def survey_step_bytes(P, V, L, N, T, camera_type):
    """algorithmic bytes of one fwd+bwd of one view as the reference's kernels move them (SH in the
    rasterizer, D = 3): B = 364 P + 1068 V + 124 L + 40 N + 32 T (lonlat), 340 P + 1020 V + ... (pinhole: no
    dpx_dt / dpy_dt)."""
    if camera_type == 1:
        return 340 * P + 1020 * V + 124 * L + 40 * N + 32 * T
    return 364 * P + 1068 * V + 124 * L + 40 * N + 32 * T


def workload_text(cfg_name, config, world, P, W, H, camera_type, sh_degree, exchange="compact"):
    cam = lambda w, h, t: f"{w}x{h} " + ("equirect (camera_type=3)" if t == 3 else "pinhole (camera_type=1)")
    if config == "E" and world > 1:
        views = (f"{cam(4096, 2048, 3)} on ranks 0-{world // 2 - 1}, {cam(1920, 1080, 1)} on ranks "
                 f"{world // 2}-{world - 1}")
    else:
        views = cam(W, H, camera_type)
    text = f"{cfg_name}: {P} Gaussians, {views}, SH degree {sh_degree}, one view per GPU"
    if world > 1 and exchange == "compact":
        text += (", RCCL gradient exchange: all-reduce of 44 B/Gaussian + all-gather of 12 B/Gaussian/view colour "
                 "gradients, SH gradient rebuilt on every rank")
    elif world > 1:
        text += ", RCCL sum all-reduce of 236 B/Gaussian gradients"
    return text


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


CPU_VARIANT = "fast"  # oracle/Makefile: -O3 -march=x86-64-v3; the parity build is -O2


def _oracle_leg(O, g, cam, dL, threads, runs, seconds):
    """Median seconds of `runs` oracle fwd+bwd passes (stopping early once `seconds` is spent, after >= 3 runs)."""
    import numpy as np

    O.set_threads(threads)
    times = []
    t_start = time.perf_counter()
    while len(times) < runs:
        t0 = time.perf_counter()
        o = O.Oracle(False, CPU_VARIANT)
        o.forward(background=np.zeros(3), means3D=g.means3D, opacity=g.opacity, scales=g.scales,
                  rotations=g.rotations, shs=g.shs, viewmatrix=cam.viewmatrix, projmatrix=cam.projmatrix,
                  campos=cam.campos, width=cam.width, height=cam.height, sh_degree=g.sh_degree,
                  camera_type=cam.camera_type)
        o.backward(dL, nthreads=threads)
        times.append(time.perf_counter() - t0)
        del o
        if len(times) >= 3 and time.perf_counter() - t_start > seconds:
            break
    return float(np.median(times)), times


def cpu_baseline(omr, g, cam, dL, seconds, threads, runs, single_config):
    """The CPU oracle (oracle/, a port: the reference has no CPU path, rasterize_points.cu:87 hard-codes kCUDA) timed
    on this host: all-core leg on the bench workload itself, one-thread leg on a smaller config (bounded sample)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O  # test infrastructure: the CPU restatement, timed as the baseline only

    O.build()
    med, times = _oracle_leg(O, g, cam, dL, threads, runs, seconds)
    N = cam.width * cam.height
    out = {"value": round(N / med / 1e6, 4), "unit": "Mpixels/s", "cores": threads, "kind": "port",
           "cpu_model": cpu_model(), "build": "oracle/_build/liboracle_fast.so (g++ -O3 -march=x86-64-v3 -fopenmp)",
           "sample": f"median of {len(times)} fwd+bwd of the bench view ({cam.width}x{cam.height}, P={g.P}, same "
                     f"scene as the GPU run) on {threads} OpenMP threads: {med:.2f} s (min {min(times):.2f}, max "
                     f"{max(times):.2f}); oracle/ restatement, no CPU reference exists"}
    if single_config:
        g1, cam1, dL1 = omr.scene.config_scene(single_config)
        med1, t1 = _oracle_leg(O, g1, cam1, dL1, 1, runs, seconds)
        out["single_thread"] = {
            "value": round(cam1.width * cam1.height / med1 / 1e6, 4), "unit": "Mpixels/s", "cores": 1,
            "sample": f"median of {len(t1)} fwd+bwd of config {single_config} ({cam1.width}x{cam1.height}, "
                      f"P={g1.P}) on one thread: {med1:.2f} s"}
    # config A (10 k Gaussians @ 512x256, the reference's own CPU-runnable case) on one thread and
    # on all cores
    gA, camA, dLA = omr.scene.config_scene("A")
    NA = camA.width * camA.height
    out["config_A"] = {}
    for leg, th in (("single_thread", 1), ("all_cores", threads)):
        mA, tA = _oracle_leg(O, gA, camA, dLA, th, runs, seconds)
        out["config_A"][leg] = {"value": round(NA / mA / 1e6, 4), "unit": "Mpixels/s", "cores": th,
                                "sample": f"median of {len(tA)} fwd+bwd of config A (512x256, P={gA.P}): {mA:.3f} s"}
    O.set_threads(1)
    return out


def main():
    args = parse()
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        return launch_ranks(args.gpus)
    if args.dist_check:
        return dist_check(args)
    import numpy as np
    import torch
    import torch.distributed as dist

    import _omnigs

    omr = _omnigs.load()
    R, scene, par = omr.rasterizer, omr.scene, omr.parallel

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    info = par.DistInfo(rank, world, local)
    if args.rehearse:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if args.rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
        seen = dist.get_world_size()
        if seen != args.gpus:
            print(f"[bench] error: --gpus {args.gpus} but the process group has {seen} ranks", file=sys.stderr)
            return 3
    elif args.gpus != 1:
        print(f"[bench] error: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        return 3
    if os.environ.get("OMR_LIB_PATH") and rank == 0:
        print(f"[bench] warning: OMR_LIB_PATH selects {os.environ['OMR_LIB_PATH']}", file=sys.stderr)

    # config D is config C's scene rendered one view per GPU: the same Gaussians for every N (weak scaling)
    cfg_name = "D" if (world > 1 and args.config == "C") else args.config
    # config E is a mixed batch (BASELINE.json): the first half of the ranks render 4096x2048 equirect views, the
    # second half 1920x1080 pinhole views; every other config is one camera type
    scene_name = args.config
    if args.config == "E" and world > 1 and rank >= world // 2:
        scene_name = "E_pinhole"
    if args.scene:
        scene_name = args.scene
    g, cam, dL = scene.config_scene(scene_name, view_index=rank % 8, P=args.gaussians)
    P, W, H = g.P, cam.width, cam.height
    M = g.shs.shape[1]
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).to(dev)
    means3D, opacity, scales, rots, shs = t(g.means3D), t(g.opacity), t(g.scales), t(g.rotations), t(g.shs)
    view, proj, campos, bg = t(cam.viewmatrix), t(cam.projmatrix), t(cam.campos), torch.zeros(3, device=dev)
    dL_dout = t(dL)
    empty = torch.empty(0, device=dev)
    grads = par.GradBuffer(P, M, dev)
    out = grads.out_dict(dev)
    bucket = int(args.bucket_mb * 1024 * 1024)
    stats = {}
    stream = torch.cuda.current_stream(dev)
    compute_events = []  # per step: (start, end of this rank's forward + backward), before the exchange
    record = {"on": False}
    COMPUTE_EVENT_STEPS = 3

    LT = R.libtorch_boundary() if args.boundary == "libtorch" else None

    def step_libtorch():
        nr, color, radii, gb, bb, ib = LT.RasterizeGaussiansCUDA(
            bg, means3D, empty, opacity, scales, rots, 1.0, empty, view, proj, cam.tanfovx, cam.tanfovy, H, W, shs,
            g.sh_degree, campos, False, cam.camera_type, False)
        gr = LT.RasterizeGaussiansBackwardCUDA(bg, means3D, radii, empty, scales, rots, 1.0, empty, view, proj,
                                               cam.tanfovx, cam.tanfovy, dL_dout, shs, g.sh_degree, campos, gb, nr, bb,
                                               ib, cam.camera_type)
        if world > 1:  # the drop-in allocates its own gradient tensors: gather them into the flat buffer
            for name, idx in (("dL_dmeans3D", 3), ("dL_dsh", 5), ("dL_dopacity", 2), ("dL_dscales", 6),
                              ("dL_drotations", 7), ("dL_dcolors", 1)):
                (out if name == "dL_dcolors" else grads.views)[name].copy_(gr[idx])
        return nr, radii, gb, ib

    # compact exchange: the colour all-gather overlaps the backward's per-Gaussian stage (parallel.CompactExchange);
    # the LibTorch boundary has no event hook, so it exchanges after the backward
    cx = None
    if world > 1 and args.exchange == "compact":
        cx = par.CompactExchange(grads, info, campos,
                                 lambda pk, out: R.sh_grad_from_colors_packed(means3D, shs, g.sh_degree, pk, out=out),
                                 dev, overlap=LT is None, any_backend=args.rehearse, ar_chunks=args.ar_chunks)
    bwd_kwargs = cx.backward_kwargs() if cx is not None else {}

    def exchange():
        if cx is not None:
            cx.start()
            cx.finish()
        elif world > 1:
            par.allreduce_(grads, info, average=False, bucket_bytes=bucket)

    def step():
        # per-rank compute time (N > 1) from the first COMPUTE_EVENT_STEPS timed steps only: every event record ends
        # in a system-scope release (an L2 writeback, ~5 us of GPU idle), so timing every step would
        # slow the steps it measures
        timed = record["on"] and len(compute_events) < COMPUTE_EVENT_STEPS
        if timed:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record(stream)
        if LT is not None:
            nr, radii, gb, ib = step_libtorch()
        else:
            nr, color, radii, gb, bb, ib = R.RasterizeGaussiansCUDA(
                bg, means3D, empty, opacity, scales, rots, 1.0, empty, view, proj, cam.tanfovx, cam.tanfovy, H, W,
                shs, g.sh_degree, campos, False, cam.camera_type, False)
            R.RasterizeGaussiansBackwardCUDA(bg, means3D, radii, empty, scales, rots, 1.0, empty, view, proj,
                                             cam.tanfovx, cam.tanfovy, dL_dout, shs, g.sh_degree, campos, gb, nr, bb,
                                             ib, cam.camera_type, out=out, **bwd_kwargs)
        if timed:
            ev[1].record(stream)
            compute_events.append(ev)
        exchange()
        stats["L"] = nr
        stats["radii"] = radii
        stats["img"] = ib
        stats["geom"] = gb

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    V = int((stats["radii"] > 0).sum().item()) if args.warmup else None
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    # per-stage pass (untimed): HIP events at every stage boundary, which cost a few us of GPU idle each; it picks
    # the dominant stage (the largest: render_backward at A-D, the tile sort at E equirect, gaussian_backward at E
    # pinhole). The timed pass then records events around that kernel only (the roofline's live launch duration)
    # and, at N > 1, two per step around this rank's forward + backward (per-rank compute time).
    R.profile_reset()
    R.profile_enable(True)
    for _ in range(min(args.steps, 10)):
        step()
    torch.cuda.synchronize(dev)
    R.profile_enable(False)
    prof = R.profile_read()
    stage_avg = {k: (ms / c if c else 0.0) for k, (ms, c) in prof.items()}
    ranked = sorted((k for k in stage_avg if stage_avg[k] > 0), key=lambda k: -stage_avg[k])
    dom = ranked[0]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    R.profile_reset()
    # The roofline kernel's launches are timed live on every LIVE_EVERY-th timed step (every step: sampling every
    # 4th measured no faster, 1718-1721 vs 1721-1724 MP/s). OMR_BENCH_LIVE=0 (diagnostic only: profiles/gaps.py): no
    # events in the timed loop; the roofline then falls back to the per-stage pass's average.
    live_on = os.environ.get("OMR_BENCH_LIVE", "1") != "0"
    LIVE_EVERY = 1
    R.profile_enable(live_on, stages=[dom])
    R.runtime_stats_reset()
    torch.cuda.reset_peak_memory_stats(dev)
    mem0 = torch.cuda.memory_stats(dev)
    record["on"] = world > 1
    t0 = time.perf_counter()
    for i in range(args.steps):
        R.profile_set_on(live_on and i % LIVE_EVERY == 0)
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    record["on"] = False
    mem1 = torch.cuda.memory_stats(dev)
    host_stats = R.runtime_stats()
    R.profile_enable(False)
    live = R.profile_read()
    if compute_events:
        compute_ms = sum(a.elapsed_time(b) for a, b in compute_events) / len(compute_events)
    else:  # N = 1: the whole step is this rank's forward + backward
        compute_ms = elapsed / args.steps * 1e3
    if V is None:
        V = int((stats["radii"] > 0).sum().item())
    if world > 1:
        e = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
        cm = torch.tensor([compute_ms], dtype=torch.float64, device=dev)
        per_rank = [torch.zeros_like(cm) for _ in range(world)]
        dist.all_gather(per_rank, cm)
        per_rank_ms = [round(float(x.item()), 4) for x in per_rank]
    else:
        per_rank_ms = [round(compute_ms, 4)]

    ms_per_step = elapsed / args.steps * 1e3
    # whole-job pixels per step: every rank's view (ranks of a mixed config render different resolutions)
    pix = torch.tensor([float(W * H)], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(pix, op=dist.ReduceOp.SUM)
    value = float(pix.item()) / (elapsed / args.steps) / 1e6
    L, N = int(stats["L"]), W * H
    T = ((W + 15) // 16) * ((H + 15) // 16)

    # dominant kernel: the largest stage of the per-stage pass; its launch duration from the timed pass (HIP events
    # on the launch stream around that kernel alone)
    pmc, pmc_file, pmc_sq_file = {}, None, None
    try:
        with open(args.traffic_json) as f:
            pj = json.load(f)
        if pj.get("config") == cfg_name and pj.get("P") == P:
            pmc = pj.get("kernels", {})
            pmc_file = pj.get("kernel_stats_file")
            pmc_sq_file = pj.get("sq_file")
    except (OSError, ValueError):
        pass

    # the row binning (bin.hip) runs for views of at most 1024 tiles a side; its algorithmic bytes need its row slots
    gxy = ((W + 15) // 16, (H + 15) // 16)
    rows_slots = R.debug_counters(P, stats["geom"])["row_slots"] if max(gxy) <= 1024 else None

    def stage_entry(k, live_ok=True):
        b = stage_bytes(k, P, V, L, N, T, M, g.sh_degree, rows_slots)
        ms_l, cnt_l = live.get(k, (0.0, 0))
        ms_k = ms_l / cnt_l if (cnt_l and live_ok) else stage_avg[k]
        ach = b / (ms_k * 1e-3) / 1e9 if ms_k > 0 else 0.0
        tr = pmc.get(k, {}).get("hbm_bytes_per_launch")
        lo = pmc.get(k, {}).get("hbm_bytes_lower")
        # the committed rocprofv3 average of the same kernel over the timed loop of a profiled bench run
        # (profiles/<tag>_kernel_stats_timed.csv, profiles/pmc_summarize.py: timed_window): `frac_rocprof` recomputes
        # `frac` from it as algorithmic bytes / avg / peak
        rp = pmc.get(k, {}).get("rocprof_avg_ms")
        ach_rp = b / (rp * 1e-3) / 1e9 if rp else None
        # VALU roofline beside the HBM one: the kernel's VALU wave-instructions per launch (committed SQ pass of the
        # same tree, profiles/<tag>_sq.csv via pmc_latest.json) over what the chip issues in its launch time
        sq = pmc.get(k, {}).get("sq") or {}
        vi = sq.get("valu_insts_per_launch")
        vfrac = vi / (VALU_SIMDS * VALU_ISSUE_PER_SIMD * ms_k * 1e-3) if (vi and ms_k > 0) else None
        # traffic = (2 FETCH + WRITE): exact for 16-B/lane streams, an upper bound for gathers, which
        # profiles/calib_fetch.hip shows FETCH counting 1:1 (traffic_lower = FETCH + WRITE)
        return {"stage": k, "avg_launch_ms": round(ms_k, 4), "timed_launches": int(cnt_l) if live_ok else 0,
                "algorithmic_bytes_per_launch": b,
                "achieved_GBps": round(ach, 2), "frac": round(ach / HBM_PEAK_GBS, 5), "traffic": tr,
                "traffic_lower": lo, "traffic_over_algorithmic": round(tr / b, 3) if (tr and b) else None,
                "traffic_lower_over_algorithmic": round(lo / b, 3) if (lo and b) else None,
                "avg_launch_ms_rocprof": rp, "frac_rocprof": round(ach_rp / HBM_PEAK_GBS, 5) if ach_rp else None,
                "rocprof_file": pmc_file if rp else None,
                "valu_issue_frac": round(vfrac, 4) if vfrac else None,
                "valu_insts_per_launch": vi, "sq_file": pmc_sq_file if vi else None}

    d = stage_entry(dom)
    survey_b = survey_step_bytes(P, V, L, N, T, cam.camera_type)
    algo_total = sum(stage_bytes(s, P, V, L, N, T, M, g.sh_degree, rows_slots) for s in stage_avg)
    # VALU secondary: pixel-instance evaluations = the forward's (instance, 16x4 band) pairs x 64,
    # at nominal 20 flop (forward) / 60 flop (backward) each, against the f32 vector peak; the backward evaluates at
    # most the forward's pairs (it stops at each band's last contributor), so its figure is an upper bound
    evals = int(R.debug_tile_cost(W, H, stats["img"]).sum().item()) * 64
    valu = {"peak_tflops": VALU_PEAK_TFLOPS, "pixel_evals": evals}
    for k, fl in (("render_forward", 20), ("render_backward", 60)):
        ms_k = stage_avg.get(k, 0.0)
        tf = evals * fl / (ms_k * 1e-3) / 1e12 if ms_k > 0 else 0.0
        valu[k] = {"flop_per_eval": fl, "tflops": round(tf, 2), "frac": round(tf / VALU_PEAK_TFLOPS, 4)}
    ambiguous = None
    try:
        with open(args.ambiguity_json) as f:
            amb = json.load(f).get("configs", {}).get(scene_name if world == 1 else cfg_name)
        if amb:  # oracle/contraction.py: the allowance counts and, per FMA-contracted build, what actually changed
            keep = ("num_rendered_delta", "depths_changed", "point_list_positions_changed", "pixels_over_1e-4",
                    "image_max_abs_err", "grad_entries_outside_bar", "grad_entries_on_owners")
            ambiguous = {"allowance": amb.get("allowance"),
                         "contracted_reference_proxies": {
                             v: dict({k: r.get(k) for k in keep},
                                     unexplained=sum(x for k, x in r.items() if k.endswith("_unexplained")))
                             for v, r in amb.get("variants", {}).items()},
                         "source": os.path.relpath(args.ambiguity_json, ROOT)}
    except (OSError, ValueError, AttributeError):
        pass
    delta = lambda k: int(mem1.get(k, 0) - mem0.get(k, 0))
    result = {
        "metric": "Mpixels/s fwd+bwd, 1M Gaussians @ 2048x1024 equirect; 1/2/4/8 GPU",
        "value": round(value, 3),
        "unit": "Mpixels/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (SplitMix64 scene, SURVEY.md §8(d)); random-init Gaussians, fixed dL/dout",
        "config": {"workload": workload_text(cfg_name, args.config, world, P, W, H, cam.camera_type, g.sh_degree,
                                               args.exchange),
                   "P": P, "V": V, "L": L, "N": N, "T": T, "width": W, "height": H, "row_slots": rows_slots,
                   "binning": "rows then columns (bin.hip)" if rows_slots is not None else "emit + radix tile sort",
                   "parallelism": f"view-parallel dp{world}", "boundary": args.boundary,
                   "exchange": args.exchange if world > 1 else None,
                   "ar_chunks": args.ar_chunks if world > 1 and args.exchange == "compact" else None,
                   "ambiguous": ambiguous},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": d["achieved_GBps"], "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": d["frac"], "traffic": d["traffic"],
                     "algorithmic_bytes_per_launch": d["algorithmic_bytes_per_launch"],
                     "avg_launch_ms": d["avg_launch_ms"], "timed_launches": d["timed_launches"],
                     "avg_launch_ms_rocprof": d["avg_launch_ms_rocprof"], "frac_rocprof": d["frac_rocprof"],
                     "rocprof_file": d["rocprof_file"],
                     # the VALU issue roofline of the same kernel (SQ_INSTS_VALU over 1024 SIMDs x 1.2 G/s x launch
                     # time): what the render kernels can actually be driven towards
                     "valu_issue_frac": d["valu_issue_frac"], "valu_insts_per_launch": d["valu_insts_per_launch"],
                     "valu_issue_peak": f"{VALU_SIMDS} SIMDs x {VALU_ISSUE_PER_SIMD / 1e9:.1f} G wave-instructions/s",
                     "sq_file": d["sq_file"],
                     "step_algorithmic_GBps": round(algo_total / (ms_per_step * 1e-3) / 1e9, 2),
                     "step_algorithmic_bytes": int(algo_total),
                     # SURVEY.md §8(d)'s whole-step formula (the reference's own kernels' compulsory bytes, its 324 B/G
                     # zero-fill and atomic RMW included) beside the per-stage accounting above
                     "step_survey_B_bytes": survey_b,
                     "step_survey_B_GBps": round(survey_b / (ms_per_step * 1e-3) / 1e9, 2),
                     "step_survey_B_frac": round(survey_b / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                     "top_stages": [stage_entry(k) for k in ranked[:3]]},
        "stages_ms": {k: round(v, 4) for k, v in stage_avg.items()},
        "valu_secondary": valu,
        "ranks": {"seen": world, "compute_ms_per_rank": per_rank_ms,
                  "imbalance_max_over_mean": round(max(per_rank_ms) / (sum(per_rank_ms) / len(per_rank_ms)), 4)
                  if sum(per_rank_ms) > 0 else None,
                  "backend": (dist.get_backend() if world > 1 else None)},
        "host": {"library": R.loaded_library(), "runtime_stats_timed": host_stats,
                 "torch_allocator_timed": {"device_mallocs": delta("num_device_alloc"),
                                           "device_frees": delta("num_device_free"),
                                           "alloc_retries": delta("num_alloc_retries"),
                                           "peak_reserved_bytes": int(mem1.get("reserved_bytes.all.peak", 0))}},
    }
    if world == 1 and rank == 0 and not args.no_cpu_baseline:
        threads = args.cpu_threads or int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
        try:
            result["cpu_baseline"] = cpu_baseline(omr, g, cam, dL, args.cpu_seconds, threads, args.cpu_runs,
                                                  args.cpu_single_config)
        except Exception as ex:  # the GPU number stands on its own; report why the baseline is missing
            result["cpu_baseline"] = {"value": None, "error": repr(ex)}
    if world == 1 and rank == 0 and not args.no_train_step:
        try:
            result["train_step"] = train_step_timing(omr, g, cam, dev, steps=10, warmup=3)
        except Exception as ex:  # informational only
            result["train_step"] = {"error": repr(ex)}
    if world > 1:
        # DESIGN.md §6's model from this run's own per-rank compute and gaussian_bwd stage time (parallel.py:
        # predict_step_ms, link bandwidth parallel.XGMI_LINK_GBPS): the driver's SCALE record can be checked against
        # it. Efficiency as the driver computes it, value(N) / (N value(1)), with value(1) = rank 0's view alone.
        pr = par.predict_step_ms(world, P, per_rank_ms, stage_avg.get("gaussian_backward", 0.0), args.exchange)
        p0 = torch.tensor([float(W * H)], dtype=torch.float64, device=dev)
        dist.broadcast(p0, 0)
        pix0 = float(p0.item())
        single = pix0 / (per_rank_ms[0] * 1e-3) / 1e6 if per_rank_ms[0] > 0 else None
        pred_value = float(pix.item()) / (pr["step_ms"] * 1e-3) / 1e6 if pr["step_ms"] > 0 else None
        result["predicted"] = {"ms_per_step": round(pr["step_ms"], 4), "value": round(pred_value, 3) if pred_value else None,
                               "efficiency": round(pred_value / (world * single), 4) if (pred_value and single) else None,
                               "measured_efficiency_vs_rank0_compute": round(value / (world * single), 4) if single else None,
                               "terms_ms": {k: (round(v, 4) if isinstance(v, float) else v) for k, v in pr.items()},
                               "xgmi_link_GBps_assumed": par.XGMI_LINK_GBPS, "model": "DESIGN.md §6"}
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


def train_step_timing(omr, g, cam, dev, steps, warmup):
    """Extra, informational (not `value`): one whole training iteration without autograd on the same scene and
    view (trainer.train_step: activations -> rasterizer forward -> fused L1+SSIM loss and dloss/dimage ->
    rasterizer backward -> densification stats -> fused activation-backward + Adam over the six groups). The
    reference's derived anchor for its whole training step is ~23 MP/s on an RTX 3090."""
    import numpy as np
    import torch

    t = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).to(dev)  # noqa: E731
    model = omr.renderer.GaussianModelParams.from_activated(t(g.means3D), t(g.scales), t(g.rotations),
                                                            t(g.opacity).reshape(-1, 1), t(g.shs), g.sh_degree)
    for name in ("xyz", "features_dc", "features_rest", "opacity", "scaling", "rotation"):
        setattr(model, name, getattr(model, name).contiguous())
    opt = omr.optim.GaussianOptimizer(model, omr.optim.OptimizationParams())
    vp = omr.renderer.Viewpoint(t(cam.viewmatrix), t(cam.projmatrix), t(cam.campos))
    gen = torch.Generator(device=dev).manual_seed(5)
    gt = torch.rand((3, cam.height, cam.width), device=dev, generator=gen)
    bg = torch.zeros(3, device=dev)
    state = omr.trainer.TrainStep()

    def it(k):
        opt.update_learning_rate(k)
        return omr.trainer.train_step(opt, vp, cam.height, cam.width, gt, bg, cam.camera_type, 0.2, state=state)

    for k in range(warmup):
        it(k)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(steps):
        terms, _, _ = it(warmup + k)
    torch.cuda.synchronize(dev)
    ms = (time.perf_counter() - t0) / steps * 1e3
    return {"ms": round(ms, 4), "Mpixels_s": round(cam.width * cam.height / (ms * 1e-3) / 1e6, 2),
            "iterations_s": round(1e3 / ms, 1), "loss": round(float(terms[0]), 6),
            "includes": "fwd + fused L1/SSIM loss + bwd + densification stats + fused Adam (6 groups)"}


if __name__ == "__main__":
    sys.exit(main())

"""bench.py's multi-rank launch without a GPU: `bench.py --gpus N` started directly (no WORLD_SIZE) spawns N ranks
itself under torch.distributed.run, every rank checks the process group holds N ranks, and rank 0 prints one JSON
line with n_gpus = N (the driver's contract); `--dist-check` stops there (gloo, no HIP library)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       timeout=180, env=env, cwd="/tmp")
    return r


def test_self_launch_two_ranks():
    r = _run("--gpus", "2", "--dist-check")
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["ranks_seen"] == 2 and d["per_rank"] == [1.0, 2.0]


def test_world_size_mismatch_fails():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-check"],
                       capture_output=True, text=True, timeout=120, env=env, cwd="/tmp")
    assert r.returncode != 0

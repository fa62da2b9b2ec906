#!/usr/bin/env python3
"""Whole training iterations of bench.py's train_step at a config (default C), for a rocprofv3 kernel trace:
    rocprofv3 --kernel-trace --stats -d DIR -o run -- python3 profiles/train_prof.py [--config C] [--steps 10]
Prints one JSON line (ms per iteration, from the host clock around the timed iterations); profiles/train_summarize.py
turns the trace into per-kernel times per iteration."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    a = ap.parse_args()
    import torch

    import _omnigs
    import bench

    omr = _omnigs.load()
    g, cam, _ = omr.scene.config_scene(a.config)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    r = bench.train_step_timing(omr, g, cam, dev, steps=a.steps, warmup=a.warmup)
    r.update(config=a.config, steps=a.steps, warmup=a.warmup)
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()

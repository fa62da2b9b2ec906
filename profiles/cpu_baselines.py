#!/usr/bin/env python3
"""CPU baselines of SURVEY.md §8(d): the oracle/ restatement (the reference has no CPU path) timed on configs A and
B, single-thread and all-core (the box's CPU share), fwd + bwd of one view. Host cores only; run on the GPU box:
    python profiles/cpu_baselines.py [threads]"""
import json
import os
import platform
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]


def main():
    import _omnigs

    omr = _omnigs.load()
    import bench

    threads = int(sys.argv[1]) if len(sys.argv) > 1 else min(16, os.cpu_count() or 1)
    cpu = next((l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")),
               platform.processor())
    out = {"cpu": cpu, "nproc": os.cpu_count(), "results": []}
    for cfg in ("A", "B"):
        g, cam, dL = omr.scene.config_scene(cfg)
        for t in (1, threads):
            r = bench.cpu_baseline(g, cam, dL, seconds=5.0, threads=t)
            out["results"].append({"config": cfg, "threads": t, "Mpixels_s": r["value"], "sample": r["sample"]})
            print(json.dumps(out["results"][-1]), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()

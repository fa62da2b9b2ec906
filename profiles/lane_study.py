#!/usr/bin/env python3
"""Lane-mapping study of the render kernels on a BASELINE config (CPU; profiles/lane_study.cpp does the counting).

Runs the oracle forward on the config's bench view, dumps means2D / conic_opacity / point_list / ranges, and counts
the wave steps and lane use of three lane mappings (16x4 bands = the current kernels, 4x4 blocks walked by 16-lane
groups, and the same grouped by 8x8 quadrants), forward and backward.

    python profiles/lane_study.py [C] [--threads 8]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config", nargs="?", default="C")
    ap.add_argument("--threads", type=int, default=8)
    args = ap.parse_args()
    import _omnigs
    import oracle as O

    exe = os.path.join(tempfile.gettempdir(), "lane_study")
    subprocess.run(["g++", "-O2", "-fopenmp", "-o", exe, os.path.join(ROOT, "profiles", "lane_study.cpp")],
                   check=True)
    O.set_threads(args.threads)
    g, cam, _ = _omnigs.load().scene.config_scene(args.config)
    o, L, _ = O.run_scene(g, cam)
    with tempfile.TemporaryDirectory() as d:
        np.array([cam.width, cam.height], np.int32).tofile(os.path.join(d, "dims.bin"))
        for k in ("means2D", "conic_opacity", "point_list", "ranges"):
            o.get(k).tofile(os.path.join(d, f"{k}.bin"))
        env = dict(os.environ, OMP_NUM_THREADS=str(args.threads))
        out = subprocess.run([exe, d], check=True, capture_output=True, text=True, env=env).stdout
    res = json.loads(out)
    res.update(config=args.config, L=int(L))
    print(json.dumps(res))


if __name__ == "__main__":
    main()

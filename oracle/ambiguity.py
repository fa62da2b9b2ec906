#!/usr/bin/env python3
"""Boundary-ambiguity counts of the BASELINE configs (TEST INFRASTRUCTURE; oracle/ambiguity.hpp).

For each config's bench view, runs the oracle forward and counts what the missing reference run could still move:
lonlat Gaussians whose tile rect changes under +-3 ulp of atan2f / asinf, pixels with a blend decision within 1e-5
of a threshold, and the Gaussians whose own decision sits there. Writes profiles/ambiguity.json, which bench.py
reports as config.ambiguous (the bench itself never runs the oracle for this).

    python oracle/ambiguity.py [A B C E_pinhole E] [--threads N]
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="*", default=["A", "B", "C", "E_pinhole", "E"])
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 1)
    ap.add_argument("--eps", type=float, default=1e-5)
    ap.add_argument("--ulps", type=int, default=3)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "ambiguity.json"))
    args = ap.parse_args()
    import numpy as np

    import _omnigs
    import oracle as O

    scene = _omnigs.load().scene
    O.build()
    O.set_threads(args.threads)
    try:
        with open(args.out) as f:
            doc = json.load(f)
    except (OSError, ValueError):
        doc = {}
    doc.setdefault("configs", {})
    doc["method"] = ("oracle/ambiguity.hpp on the oracle forward of each config's bench view (view 0): "
                     f"rect_gaussians = lonlat Gaussians whose getRect changes under +-{args.ulps} ulp of atan2f/asinf; "
                     f"alpha_pixels / saturation_pixels = pixels with a blend decision within {args.eps} (relative) of "
                     "alpha = 1/255 / T(1-alpha) = 1e-4; flip_gaussians = Gaussians whose own decision sits there")
    for name in args.configs:
        t0 = time.time()
        g, cam, _ = scene.config_scene(name)
        o = O.Oracle(False)
        L = o.forward(background=np.zeros(3), means3D=g.means3D, opacity=g.opacity, scales=g.scales,
                      rotations=g.rotations, shs=g.shs, viewmatrix=cam.viewmatrix, projmatrix=cam.projmatrix,
                      campos=cam.campos, width=cam.width, height=cam.height, sh_degree=g.sh_degree,
                      tanfovx=cam.tanfovx, tanfovy=cam.tanfovy, camera_type=cam.camera_type)
        counts, _ = o.ambiguity(args.eps, args.ulps)
        V = int((o.get("radii") > 0).sum())
        counts.update(P=g.P, V=V, L=int(L), pixels=cam.width * cam.height)
        doc["configs"][name] = counts
        print(name, counts, f"{time.time() - t0:.1f} s", flush=True)
        del o
    # config D = config C's scene, one view per GPU: the same counts per view as C's view 0
    if "C" in doc["configs"]:
        doc["configs"]["D"] = dict(doc["configs"]["C"], note="view 0 of the config-C scene (one of D's eight views)")
    with open(args.out, "w") as f:
        json.dump(doc, f, indent=1)


if __name__ == "__main__":
    main()

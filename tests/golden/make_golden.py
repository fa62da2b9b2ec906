#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ from the CPU oracle (oracle/, validated by
tests/test_oracle_known.py, test_oracle_fd.py and test_torch_model.py — the reference itself cannot be built or
run here: CUDA-only).

Each fixture stores the inputs (or, for config A, the SHA-256 of the inputs regenerated from the seeded scene
generator), every intermediate the reference exposes in its scratch state (radii, pixel centres, conics, depths,
tiles_touched, sorted point_list, tile ranges, final_T, n_contrib) and all outputs and gradients.

    python tests/golden/make_golden.py            # rewrite all fixtures
"""
import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]

import _omnigs  # noqa: E402

_omnigs.load()
from helpers import make_case, oracle_run, scene  # noqa: E402

LON, PIN = scene.CAMERA_LONLAT, scene.CAMERA_PINHOLE

# name: (P, W, H, camera, seed, view, sh_degree, scale multiplier, bg, store_inputs)
CASES = {
    "lonlat_64_64x32": (64, 64, 32, LON, 11, 0, 3, 8.0, (0.0, 0.0, 0.0), True),
    "lonlat_1k_128x64_white": (1000, 128, 64, LON, 12, 1, 3, 3.0, (1.0, 1.0, 1.0), True),
    "pinhole_1k_160x90": (1000, 160, 90, PIN, 16, 0, 3, 3.0, (0.0, 0.0, 0.0), True),
    "lonlat_A_10k_512x256": (10000, 512, 256, LON, scene.BASE_SEED, 0, 3, 1.0, (0.0, 0.0, 0.0), False),
}


def inputs_of(name):
    P, W, H, cam_t, seed, view, deg, mult, bg, _ = CASES[name]
    g, cam, dL = make_case(P, W, H, cam_t, seed, view_index=view, sh_degree=deg, spread=mult)
    return g, cam, dL, np.asarray(bg, np.float32)


def input_digest(g, cam, dL, bg):
    h = hashlib.sha256()
    for a in (g.means3D, g.scales, g.rotations, g.opacity, g.shs, cam.viewmatrix, cam.projmatrix, cam.campos, dL, bg):
        h.update(np.ascontiguousarray(a, np.float32).tobytes())
    return h.hexdigest()


def compute(name):
    g, cam, dL, bg = inputs_of(name)
    o, L, gr = oracle_run(g, cam, dL, bg=tuple(float(x) for x in bg))
    P, W, H = g.P, cam.width, cam.height
    out = dict(
        num_rendered=np.array(L, np.int64), width=np.array(W), height=np.array(H),
        camera_type=np.array(cam.camera_type), sh_degree=np.array(g.sh_degree),
        input_sha256=np.array(input_digest(g, cam, dL, bg)),
        out_color=o.get("out_color").reshape(3, H, W), radii=o.get("radii"),
        means2D=o.get("means2D").reshape(P, 2), conic_opacity=o.get("conic_opacity").reshape(P, 4),
        depths=o.get("depths"), tiles_touched=o.get("tiles_touched"), point_list=o.get("point_list"),
        ranges=o.get("ranges").reshape(-1, 2), final_T=o.get("final_T").reshape(H, W),
        n_contrib=o.get("n_contrib").reshape(H, W),
        dL_dmeans2D=gr["dmean2D"], dL_dcolors=gr["dcolor"], dL_dopacity=gr["dopacity"], dL_dmeans3D=gr["dmean3D"],
        dL_dcov3D=gr["dcov3D"], dL_dsh=gr["dsh"], dL_dscales=gr["dscale"], dL_drotations=gr["drot"],
    )
    if CASES[name][-1]:
        out.update(means3D=g.means3D, scales=g.scales, rotations=g.rotations, opacity=g.opacity, shs=g.shs,
                   viewmatrix=cam.viewmatrix, projmatrix=cam.projmatrix, campos=cam.campos,
                   tanfov=np.array([cam.tanfovx, cam.tanfovy], np.float32), dL_dout=dL, background=bg)
    return out


def main():
    for name in CASES:
        path = os.path.join(HERE, f"{name}.npz")
        np.savez_compressed(path, **compute(name))
        print(f"wrote {path} ({os.path.getsize(path) / 1e6:.2f} MB)")


if __name__ == "__main__":
    main()

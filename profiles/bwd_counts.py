#!/usr/bin/env python3
"""Diagnostic (variant build with -DOMR_BWD_COUNT): how much of render_backward's (instance, band) work finds a
contributing pixel. GPU box: OMR_LIB_PATH=omnigs-fork_amd/lib/exp/count.so python profiles/bwd_counts.py [config]"""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import _omnigs

    omr = _omnigs.load()
    R = omr.rasterizer
    L = R.lib()
    L.omr_debug_bwd_counts.argtypes = [C.c_void_p, C.c_int]
    g, cam, dL = omr.scene.config_scene(sys.argv[1] if len(sys.argv) > 1 else "C")
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).cuda()  # noqa: E731
    e = torch.empty(0, device="cuda")
    args = (t(g.means3D), t(g.opacity), t(g.scales), t(g.rotations), t(g.shs))
    bg = torch.zeros(3, device="cuda")
    nr, color, radii, gb, bb, ib = R.RasterizeGaussiansCUDA(bg, args[0], e, args[1], args[2], args[3], 1.0, e,
                                                            t(cam.viewmatrix), t(cam.projmatrix), cam.tanfovx,
                                                            cam.tanfovy, cam.height, cam.width, args[4], g.sh_degree,
                                                            t(cam.campos), False, cam.camera_type)
    buf = (C.c_uint64 * 5)()
    L.omr_debug_bwd_counts(buf, 1)
    R.RasterizeGaussiansBackwardCUDA(bg, args[0], radii, e, args[2], args[3], 1.0, e, t(cam.viewmatrix),
                                     t(cam.projmatrix), cam.tanfovx, cam.tanfovy, t(dL), args[4], g.sh_degree,
                                     t(cam.campos), gb, nr, bb, ib, cam.camera_type)
    torch.cuda.synchronize()
    L.omr_debug_bwd_counts(buf, 0)
    staged, evals, hits, anyc, lanes = (int(x) for x in buf)
    print(json.dumps({"L": nr, "staged_instances": staged, "band_evals": evals, "band_evals_with_contrib": hits,
                      "instances_with_contrib": anyc, "hit_frac": round(hits / max(evals, 1), 4),
                      "any_frac": round(anyc / max(staged, 1), 4),
                      "contrib_pixel_pairs": lanes, "lanes_per_hit_band": round(lanes / max(hits, 1), 2)}))


if __name__ == "__main__":
    main()

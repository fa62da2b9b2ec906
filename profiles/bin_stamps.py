#!/usr/bin/env python3
"""Phase timeline of the row binning's columns scatter (diagnostic; GPU box):
    OMR_LIB_PATH=omnigs-fork_amd/lib/exp/binstamps.so python profiles/bin_stamps.py [config]
Needs a build with -DOMR_BIN_STAMPS (omnigs-fork_amd/csrc/build_variant.sh binstamps -DOMR_BIN_STAMPS). Runs three
forwards of the bench scene, reads the per-block, per-chunk s_memrealtime stamps (100 MHz) of cols_scatter_kernel's
phases and prints the mean / median duration of each phase and of a whole chunk iteration."""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PHASES = ["stage owners", "owner map", "expand + band masks", "rank", "sort in LDS", "write-out + ranges",
          "end barrier"]


def main():
    import torch

    import _omnigs

    omr = _omnigs.load()
    R, scene = omr.rasterizer, omr.scene
    cfg = sys.argv[1] if len(sys.argv) > 1 else "E"
    g, cam, _ = scene.config_scene(cfg, view_index=0)
    dev = torch.device("cuda", 0)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).to(dev)  # noqa: E731
    empty = torch.empty(0, device=dev)
    for _ in range(3):
        R.RasterizeGaussiansCUDA(torch.zeros(3, device=dev), t(g.means3D), empty, t(g.opacity), t(g.scales),
                                 t(g.rotations), 1.0, empty, t(cam.viewmatrix), t(cam.projmatrix), cam.tanfovx,
                                 cam.tanfovy, cam.height, cam.width, t(g.shs), g.sh_degree, t(cam.campos), False,
                                 cam.camera_type, False)
    torch.cuda.synchronize()
    lib = R.lib()
    lib.omr_debug_bin_stamps.argtypes = [C.c_void_p, C.c_size_t]
    buf = np.zeros((1024, 16, 8), dtype=np.uint64)
    rc = lib.omr_debug_bin_stamps(buf.ctypes.data_as(C.c_void_p), buf.nbytes)
    assert rc == 0, rc
    st = buf.astype(np.int64)
    ok = (st[:, :, 0] > 0) & (st[:, :, 7] >= st[:, :, 0])
    out = {"config": cfg, "chunks_sampled": int(ok.sum()), "unit": "us", "phases": {}}
    for p, name in enumerate(PHASES):
        d = (st[:, :, p + 1] - st[:, :, p])[ok] / 100.0
        out["phases"][name] = {"mean": round(float(d.mean()), 3), "median": round(float(np.median(d)), 3)}
    tot = (st[:, :, 7] - st[:, :, 0])[ok] / 100.0
    out["iteration"] = {"mean": round(float(tot.mean()), 3), "median": round(float(np.median(tot)), 3)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

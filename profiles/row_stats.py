#!/usr/bin/env python3
"""Gradient-row statistics of a bench scene (diagnostic; GPU box): one forward, then the distribution of tiles_touched
(= each Gaussian's gradient rows), the huge Gaussians' share (more than ROW_SUM_HUGE = 256 rows: summed by
huge_row_sums, gaussian_bwd.hip) and the largest.   python profiles/row_stats.py [config]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


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
    out = R.RasterizeGaussiansCUDA(torch.zeros(3, device=dev), t(g.means3D), empty, t(g.opacity), t(g.scales),
                                   t(g.rotations), 1.0, empty, t(cam.viewmatrix), t(cam.projmatrix), cam.tanfovx,
                                   cam.tanfovy, cam.height, cam.width, t(g.shs), g.sh_degree, t(cam.campos), False,
                                   cam.camera_type, False)
    num_rendered, geom, binning, img = out[0], out[3], out[4], out[5]
    P = g.means3D.shape[0]
    st = R.debug_state(P, 0, cam.width, cam.height, geom, binning, img)
    tt = st["tiles_touched"].cpu().numpy().astype(np.int64)
    huge = tt > 256
    qs = [50, 90, 99, 99.9]
    res = {"config": cfg, "P": int(P), "rows": int(tt.sum()), "num_rendered": int(num_rendered),
           "visible": int((tt > 0).sum()), "rows_percentiles": {str(q): float(np.percentile(tt[tt > 0], q)) for q in qs},
           "huge_gaussians": int(huge.sum()), "huge_rows": int(tt[huge].sum()), "max_rows": int(tt.max()),
           "huge_rows_hist": {f"{lo}-{hi}": int(((tt > lo) & (tt <= hi)).sum())
                              for lo, hi in [(256, 1024), (1024, 4096), (4096, 16384), (16384, 1 << 30)]},
           "counters": R.debug_counters(P, geom)}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()

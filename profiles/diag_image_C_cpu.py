"""CPU side of the config-C forward-image diagnosis (GPU side: profiles/diag_image_C.py).
For every pixel where |HIP - oracle| > 1e-4 it re-blends the pixel's tile list in float64 from the (bit-exact)
oracle geometry and reports whether a blend decision sits at a threshold: an alpha within 1e-5 relative of 1/255
(skip test, forward.cu:436-437) or a T*(1-alpha) within 1e-5 relative of 1e-4 (saturation test, :440-444)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import oracle as O  # noqa: E402
from helpers import oracle_run, scene  # noqa: E402

O.set_threads(os.cpu_count() or 1)
d = np.load(os.path.join(ROOT, "gpurun_out", "diag_C.npz"))
g, cam, _ = scene.config_scene("C")
o, L, _ = oracle_run(g, cam, None)
W, H, P = cam.width, cam.height, g.P
img_o = o.get("out_color").reshape(3, H, W)
err = np.abs(d["color"] - img_o).max(0)
nc_o, nc_h = o.get("n_contrib").reshape(H, W), d["n_contrib"].astype(np.uint32).reshape(H, W)
bad = np.argwhere(err > 1e-4)
print(f"L {L} (hip {int(d['L'])}); pixels > 1e-4: {len(bad)} of {W*H}; n_contrib differs on {(nc_o != nc_h).sum()}")
print("n_contrib differs on bad pixels:", sum(int(nc_o[y, x] != nc_h[y, x]) for y, x in bad))
pl = o.get("point_list"); rg = o.get("ranges").reshape(-1, 2)
m2 = o.get("means2D").reshape(P, 2).astype(np.float64); co = o.get("conic_opacity").reshape(P, 4).astype(np.float64)
rgb = o.get("rgb").reshape(P, 3).astype(np.float64)
gx = (W + 15) // 16
for y, x in bad[np.argsort(-err[bad[:, 0], bad[:, 1]])][:20]:
    t = (y // 16) * gx + x // 16
    ids = pl[rg[t, 0]:rg[t, 1]]
    dx, dy = m2[ids, 0] - x, m2[ids, 1] - y
    power = -0.5 * (co[ids, 0] * dx * dx + co[ids, 2] * dy * dy) - co[ids, 1] * dx * dy
    alpha = np.minimum(0.99, co[ids, 3] * np.exp(power))
    T, near_a, near_t = 1.0, 0, 0
    for k in range(len(ids)):
        if power[k] > 0: continue
        a = alpha[k]
        if abs(a - 1 / 255) < 1e-5 * (1 / 255): near_a += 1
        if a < 1 / 255: continue
        tt = T * (1 - a)
        if abs(tt - 1e-4) < 1e-5 * 1e-4: near_t += 1
        if tt < 1e-4: break
        T = tt
    print(f"pix ({x},{y}) err {err[y, x]:.2e} n_contrib o/h {nc_o[y, x]}/{nc_h[y, x]} "
          f"final_T o/h {o.get('final_T').reshape(H, W)[y, x]:.3e}/{d['final_T'].reshape(H, W)[y, x]:.3e} "
          f"alpha@1/255 {near_a} T@1e-4 {near_t} list {len(ids)}")

#!/usr/bin/env python3
"""Wave timeline of the render kernels (diagnostic; GPU box):
    OMR_LIB_PATH=omnigs-fork_amd/lib/exp/stamps.so python profiles/wave_timeline.py [config]
Needs a build with -DOMR_STAMPS (omnigs-fork_amd/csrc/build_variant.sh stamps -DOMR_STAMPS ...). Runs one
forward + backward of the bench scene, reads the per-wave [start, end, HW_ID|XCC_ID, unit] stamps and prints, per
kernel: duration, wave lifetime distribution, and the mean number of resident waves per SIMD over time."""
import ctypes as C
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
    cfg = sys.argv[1] if len(sys.argv) > 1 else "C"
    g, cam, dL = scene.config_scene(cfg, view_index=0)
    dev = torch.device("cuda", 0)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).to(dev)
    args = dict(bg=torch.zeros(3, device=dev), means3D=t(g.means3D), opacity=t(g.opacity), scales=t(g.scales),
                rots=t(g.rotations), shs=t(g.shs), view=t(cam.viewmatrix), proj=t(cam.projmatrix),
                campos=t(cam.campos))
    empty = torch.empty(0, device=dev)
    dL_dout = t(dL)
    W, H = cam.width, cam.height
    for it in range(3):
        nr, color, radii, gb, bb, ib = R.RasterizeGaussiansCUDA(
            args["bg"], args["means3D"], empty, args["opacity"], args["scales"], args["rots"], 1.0, empty,
            args["view"], args["proj"], cam.tanfovx, cam.tanfovy, H, W, args["shs"], g.sh_degree, args["campos"],
            False, cam.camera_type, False)
        R.RasterizeGaussiansBackwardCUDA(args["bg"], args["means3D"], radii, empty, args["scales"], args["rots"], 1.0,
                                         empty, args["view"], args["proj"], cam.tanfovx, cam.tanfovy, dL_dout,
                                         args["shs"], g.sh_degree, args["campos"], gb, nr, bb, ib, cam.camera_type)
    torch.cuda.synchronize()
    lib = R.lib()
    lib.omr_debug_stamps.argtypes = [C.c_int, C.c_void_p, C.c_int]
    out = {}
    for which, name in ((0, "render_forward"), (1, "render_backward")):
        n = 1 << 17
        buf = np.zeros((n, 4), dtype=np.uint64)
        rc = lib.omr_debug_stamps(which, buf.ctypes.data_as(C.c_void_p), n)
        assert rc == 0, rc
        used = buf[buf[:, 1] > 0]
        t0, t1 = used[:, 0].astype(np.int64), used[:, 1].astype(np.int64)
        base = t0.min()
        s, e = (t0 - base) * 10.0, (t1 - base) * 10.0  # ns (100 MHz)
        life = e - s
        hw = used[:, 2] & 0xFFFFFFFF
        xcc = used[:, 2] >> 32
        simd = (hw >> 4) & 3
        cu = (hw >> 8) & 15
        sh = (hw >> 12) & 1
        se = (hw >> 13) & 7
        key = ((xcc * 8 + se) * 2 + sh) * 16 * 4 + cu * 4 + simd
        nsimd = len(np.unique(key))
        dur = e.max()
        grid = np.linspace(0, dur, 200)
        conc = np.array([((s <= x) & (e > x)).sum() for x in grid]) / max(nsimd, 1)
        print(f"{name}: waves {len(used)} on {nsimd} SIMDs, span {dur / 1e3:.1f} us; lifetime mean "
              f"{life.mean() / 1e3:.1f} p50 {np.median(life) / 1e3:.1f} max {life.max() / 1e3:.1f} us; "
              f"start max {s.max() / 1e3:.1f} us; resident waves/SIMD mean {conc.mean():.2f} max {conc.max():.2f}")
        print("  waves/SIMD over time (10 samples):", np.round(conc[::20], 2).tolist())
        out[name] = used
    np.savez(os.path.join(ROOT, "gpurun_out", "wave_timeline.npz"), **out)


if __name__ == "__main__":
    main()

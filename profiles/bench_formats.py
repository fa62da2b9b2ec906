#!/usr/bin/env python3
"""distCUDA2 and PLY I/O at config C's model size (P = 1 M Gaussians, SH degree 3).
distCUDA2 is timed with HIP events; PLY save / load wall-clock includes the file system (page cache).
GPU box: python profiles/bench_formats.py [P]"""
import json
import os
import sys
import tempfile
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import _omnigs

    omr = _omnigs.load()
    F = omr.formats
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    g = torch.Generator(device="cuda").manual_seed(0)
    out = {"P": P}
    for kind in ("normal", "clustered"):
        pts = torch.randn((P, 3), device="cuda", generator=g)
        if kind == "clustered":
            centers = torch.randn((P // 500, 3), device="cuda", generator=g) * 20 + 50
            pts = centers[torch.randint(0, P // 500, (P,), device="cuda", generator=g)] + pts * 0.05
        for _ in range(2):
            F.distCUDA2(pts)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(5):
            F.distCUDA2(pts)
        e.record()
        torch.cuda.synchronize()
        out[f"dist2_{kind}_ms"] = round(s.elapsed_time(e) / 5, 3)
    t = [torch.randn(sh, device="cuda", generator=g) for sh in ((P, 3), (P, 1, 3), (P, 15, 3), (P, 1), (P, 3), (P, 4))]
    m = omr.renderer.GaussianModelParams(*t, 3, 3)
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "m.ply")
        F.save_ply(m, path)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        F.save_ply(m, path)
        t1 = time.perf_counter()
        m2 = F.load_ply(path, 3)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        size = os.path.getsize(path)
        assert all(torch.equal(a, b) for a, b in zip(m.parameters(), m2.parameters()))
    out.update(ply_bytes=size, ply_save_ms=round((t1 - t0) * 1e3, 1), ply_load_ms=round((t2 - t1) * 1e3, 1),
               ply_save_MBps=round(size / (t1 - t0) / 1e6), ply_load_MBps=round(size / (t2 - t1) / 1e6))
    print(json.dumps(out))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""A/B of two builds of omr_l1_ssim_loss (default lib vs omnigs-fork_amd/lib/exp/ssim_tiled.so): bitwise dL/dimg,
loss values and timing. GPU box: python profiles/ssim_ab.py [H W]"""
import ctypes as C
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(path):
    L = C.CDLL(path)
    L.omr_l1_ssim_scratch_floats.restype = C.c_size_t
    L.omr_l1_ssim_scratch_floats.argtypes = [C.c_int] * 3
    L.omr_l1_ssim_loss.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_float, C.c_void_p,
                                   C.c_void_p, C.c_void_p, C.c_void_p]
    return L


def run(L, img, gt, lam, reps=20):
    Cn, H, W = img.shape
    grad = torch.empty_like(img)
    out3 = torch.empty(3, device="cuda")
    scratch = torch.empty(int(L.omr_l1_ssim_scratch_floats(Cn, H, W)), device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    f = lambda: L.omr_l1_ssim_loss(img.data_ptr(), gt.data_ptr(), Cn, H, W, lam, grad.data_ptr(), out3.data_ptr(),  # noqa: E731
                                   scratch.data_ptr(), st)
    for _ in range(3):
        assert f() == 0
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        f()
    e.record()
    torch.cuda.synchronize()
    return grad.clone(), out3.clone(), s.elapsed_time(e) / reps


def main():
    import glob

    H, W = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (1024, 2048)
    g = torch.Generator(device="cuda").manual_seed(0)
    base = load(os.path.join(ROOT, "omnigs-fork_amd", "lib", "libomnigs_raster.so"))
    variants = {os.path.basename(p)[:-3]: load(p) for p in sorted(glob.glob(os.path.join(ROOT, "omnigs-fork_amd", "lib",
                                                                                          "exp", "*.so")))}
    res = {}
    for shape in ((3, H, W), (3, 2048, 4096), (3, 91, 157), (1, 16, 16), (3, 5, 300)):
        img = torch.rand(shape, device="cuda", generator=g)
        gt = torch.rand(shape, device="cuda", generator=g)
        a = run(base, img, gt, 0.2)
        r = {"base_ms": round(a[2], 4), "loss": [float(x) for x in a[1]]}
        for name, L in variants.items():
            b = run(L, img, gt, 0.2)
            r[name] = {"ms": round(b[2], 4), "grad_bitwise_equal": bool(torch.equal(a[0], b[0])),
                       "loss": [float(x) for x in b[1]]}
        res[str(shape)] = r
    print(json.dumps(res))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Fused L1 + SSIM loss (omr_l1_ssim_loss) vs the reference's torch formulation (loss_utils.h: five depthwise
11x11 conv2d + autograd), forward + backward on one [3,H,W] image (default 2048x1024, config C). GPU box:
    python profiles/bench_loss.py [H W]"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timeit(fn, steps=20, warmup=5):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


def main():
    import _omnigs

    L = _omnigs.load().losses
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import loss_oracle as LO  # the reference formulation in torch (timed beside the fused kernel)
    H, W = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (1024, 2048)
    g = torch.Generator(device="cuda").manual_seed(0)
    gt = torch.rand((3, H, W), device="cuda", generator=g)
    img = torch.rand((3, H, W), device="cuda", generator=g).requires_grad_(True)
    lam = 0.2

    def fused():
        img.grad = None
        loss, _ = L.l1_ssim_loss(img, gt, lam)
        loss.backward()

    def reference():
        img.grad = None
        loss = (1.0 - lam) * LO.l1_loss(img, gt) + lam * (1.0 - LO.ssim(img, gt))
        loss.backward()

    t_f, t_r = timeit(fused), timeit(reference)
    n = 3 * H * W
    print(json.dumps({"loss": "(1-l)*L1 + l*(1-SSIM) fwd+bwd", "shape": [3, H, W], "fused_ms": round(t_f, 4),
                      "torch_reference_ms": round(t_r, 4), "speedup": round(t_r / t_f, 2),
                      "fused_GBps_12B_per_px": round(12 * n / (t_f * 1e-3) / 1e9, 1)}))


if __name__ == "__main__":
    main()

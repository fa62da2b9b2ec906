"""The reference's training loss restated in torch (TEST INFRASTRUCTURE ONLY).

include/loss_utils.h:31-129 (l1_loss, gaussian window, ssim with five depthwise 11x11 conv2d and zero padding) as
gaussian_mapper.cpp:391-413 combines them, including the undistortion mask and the skip-bottom crop. Used by
tests/ (checker of the fused HIP loss csrc/ssim.hip and of trainer.train_step) and by profiles/bench_loss.py
(the reference formulation timed beside the fused kernel). The product never imports it.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def l1_loss(network_output: torch.Tensor, gt: torch.Tensor) -> torch.Tensor:
    """loss_utils.h:31-34."""
    return torch.abs(network_output - gt).mean()


def gaussian(window_size: int, sigma: float, device, dtype=torch.float32) -> torch.Tensor:
    """loss_utils.h:54-67."""
    x = torch.arange(window_size, dtype=dtype, device=device) - window_size // 2
    g = torch.exp(-(x * x) / (2.0 * sigma * sigma))
    return g / g.sum()


def ssim(img1: torch.Tensor, img2: torch.Tensor, window_size: int = 11, size_average: bool = True) -> torch.Tensor:
    """loss_utils.h:69-129 ([C,H,W] images, depthwise 11x11 Gaussian window sigma 1.5, zero padding)."""
    channel = img1.shape[-3]
    g = gaussian(window_size, 1.5, img1.device, torch.float32).unsqueeze(1)
    window = (g @ g.t()).to(img1.dtype).expand(channel, 1, window_size, window_size).contiguous()
    pad = window_size // 2
    conv = lambda x: F.conv2d(x, window, padding=pad, groups=channel)  # noqa: E731
    mu1, mu2 = conv(img1), conv(img2)
    mu1_sq, mu2_sq, mu1_mu2 = mu1 * mu1, mu2 * mu2, mu1 * mu2
    sigma1_sq = conv(img1 * img1) - mu1_sq
    sigma2_sq = conv(img2 * img2) - mu2_sq
    sigma12 = conv(img1 * img2) - mu1_mu2
    C1, C2 = 0.01 ** 2, 0.03 ** 2
    ssim_map = ((2 * mu1_mu2 + C1) * (2 * sigma12 + C2)) / ((mu1_sq + mu2_sq + C1) * (sigma1_sq + sigma2_sq + C2))
    return ssim_map.mean() if size_average else ssim_map.mean(1).mean(1).mean(1)


def skip_bottom_rows(height: int, ratio: float) -> int:
    """gaussian_mapper.cpp:396: (int)std::round(image_height * skip_bottom_ratio_) (round half away from zero)."""
    return int(math.floor(height * ratio + 0.5))


def training_loss(rendered: torch.Tensor, gt: torch.Tensor, lambda_dssim: float, mask=None,
                  skip_bottom_ratio: float = 0.0) -> torch.Tensor:
    """gaussian_mapper.cpp:387-413: masked image, optional bottom crop, (1 - l) L1 + l (1 - SSIM)."""
    img = rendered * mask if mask is not None else rendered
    if skip_bottom_ratio > 0.0:
        pix = skip_bottom_rows(img.shape[1], skip_bottom_ratio)
        img, gt = img[:, 0:img.shape[1] - pix, :], gt[:, 0:gt.shape[1] - pix, :]
    return (1.0 - lambda_dssim) * l1_loss(img, gt) + lambda_dssim * (1.0 - ssim(img, gt))

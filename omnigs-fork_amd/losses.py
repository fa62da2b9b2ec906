"""Training loss of OmniGS on the gfx950 library: (1 - lambda) * L1 + lambda * (1 - SSIM).

Mirrors include/loss_utils.h:31-129 (l1_loss, ssim) as combined by gaussian_trainer.cpp:88-90 and
gaussian_mapper.cpp:403-412. `l1_ssim_loss` runs the fused HIP kernel (omr_l1_ssim_loss, csrc/ssim.hip): one pass
computes the loss and d loss / d image, and the autograd backward scales that gradient. There is no torch
formulation here: the reference's formulas in torch are the tests' checker (oracle/loss_oracle.py).
"""
from __future__ import annotations

import torch

from . import rasterizer as R


def l1_ssim_loss_and_grad(image: torch.Tensor, gt: torch.Tensor, lambda_dssim: float, grad_out=None):
    """The fused kernel without autograd: returns (terms = tensor([loss, l1, ssim]), dloss/dimage [C,H,W])."""
    if image.device.type != "cuda" or gt.device.type != "cuda":
        raise R.RasterizerError("l1_ssim_loss needs HIP tensors (the fused loss has no CPU path)")
    img = image.detach().contiguous().float()
    ref = gt.detach().contiguous().float()
    if img.shape != ref.shape or img.dim() != 3:
        raise R.RasterizerError("image and gt must both be [C,H,W]")
    Cn, H, W = (int(s) for s in img.shape)
    L = R.lib()
    grad = torch.empty_like(img) if grad_out is None else grad_out
    if grad.shape != img.shape or not grad.is_contiguous() or grad.dtype != torch.float32:
        raise R.RasterizerError("grad_out must be a contiguous float32 tensor shaped like image")
    out3 = torch.empty(3, dtype=torch.float32, device=img.device)
    scratch = torch.empty(int(L.omr_l1_ssim_scratch_floats(Cn, H, W)), dtype=torch.float32, device=img.device)
    rc = L.omr_l1_ssim_loss(img.data_ptr(), ref.data_ptr(), Cn, H, W, float(lambda_dssim), grad.data_ptr(),
                            out3.data_ptr(), scratch.data_ptr(), R._stream(img.device))
    R._check(rc, "l1_ssim_loss")
    return out3, grad


class _FusedL1SSIM(torch.autograd.Function):
    @staticmethod
    def forward(ctx, image, gt, lambda_dssim):
        out3, grad = l1_ssim_loss_and_grad(image, gt, lambda_dssim)
        ctx.save_for_backward(grad)
        ctx.mark_non_differentiable(out3)
        return out3[0], out3

    @staticmethod
    def backward(ctx, grad_loss, _grad_terms):
        (grad,) = ctx.saved_tensors
        return grad * grad_loss, None, None


def l1_ssim_loss(image: torch.Tensor, gt: torch.Tensor, lambda_dssim: float):
    """(1 - lambda) * l1_loss(image, gt) + lambda * (1 - ssim(image, gt)), fused. Returns (loss, terms) where
    terms = tensor([loss, l1, ssim]) (no gradient; for logging like gaussian_trainer.cpp:99-110)."""
    return _FusedL1SSIM.apply(image, gt, float(lambda_dssim))

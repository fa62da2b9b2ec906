"""One training iteration with no autograd graph (SURVEY.md §8(f) ranks 1-3 put together).

GaussianMapper::trainForOneIteration (gaussian_mapper.cpp:338-488), minus the SLAM bookkeeping:
  activations (gaussian_model.cpp:54-77) -> RasterizeGaussiansCUDA -> fused L1 + SSIM loss and dloss/dimage
  (loss_utils.h, csrc/ssim.hip) -> RasterizeGaussiansBackwardCUDA -> Adam on the rasterizer's activated-space
  gradients with the activation backward fused (csrc/optim.hip), which also writes the next forward's activated
  tensors and does max_radii2D + addDensificationStats in the same launch.
The reference reaches the same state through torch autograd (loss.backward()) and torch::optim::Adam;
tests/test_gpu_optim.py checks the two agree. Densification / opacity reset stay with the caller, as in the
reference's loop (:436-452), through GaussianOptimizer.densify_and_prune / reset_opacity.
"""
from __future__ import annotations

import math
from typing import Optional

import numpy as np
import torch

from . import losses
from . import optim as O
from . import rasterizer as R
from .parallel import DistInfo, GradBuffer, allreduce_compact_


class TrainStep:
    """Reusable buffers for train_step (the gradient buffer is sized once per P, the activated tensors' buffers
    likewise)."""

    def __init__(self):
        self.buf: Optional[GradBuffer] = None
        self.dimg: Optional[torch.Tensor] = None
        self.act: dict = {}


def skip_bottom_rows(image_height: int, skip_bottom_ratio: float) -> int:
    """gaussian_mapper.cpp:396: (int)std::round(image_height * skip_bottom_ratio_), half away from zero."""
    return int(math.floor(image_height * skip_bottom_ratio + 0.5))


def train_step(opt: O.GaussianOptimizer, viewpoint, image_height: int, image_width: int, gt_image: torch.Tensor,
               bg_color: torch.Tensor, camera_type: int = R.CAMERA_LONLAT, lambda_dssim: float = 0.2,
               densification_stats: bool = True, state: Optional[TrainStep] = None,
               dist_info: Optional[DistInfo] = None, mask: Optional[torch.Tensor] = None,
               skip_bottom_ratio: float = 0.0):
    """Render `viewpoint`, take the loss against gt_image, backpropagate and step Adam. Returns
    (terms = tensor([loss, l1, ssim]), rendered image, radii).

    The loss is the reference's (gaussian_mapper.cpp:387-413): the rendered image times `mask` (the undistortion
    mask, broadcast over channels; None = all ones), and with skip_bottom_ratio > 0 the bottom
    round(H * ratio) rows of image and gt left out of L1 and SSIM (cfg/lonlat/360roam_lonlat.yaml uses 0.063).
    d loss / d image is the fused kernel's gradient on the kept rows, zero on the skipped ones, times the mask.

    View-parallel (dist_info.world_size > 1): every rank renders its own view of the replicated
    Gaussians; the compact exchange (parallel.allreduce_compact_) sums the rasterizer gradients over the views and
    every rank then takes the same Adam step on the same sums, so the replicas stay identical without a parameter
    broadcast (the kernels are deterministic). Densification statistics stay per rank until
    GaussianOptimizer.sync_densification_stats() at a densification iteration (the sums commute)."""
    pc = opt.model
    state = state or TrainStep()
    P, Mr = opt.P, opt.Mr
    dev = pc.xyz.device
    # the activations (cat / sigmoid / exp / normalize): written by the previous step's Adam launch
    # (omr_adam_step_activate), else one omr_activate launch (first step, after densification / opacity reset)
    act = opt.activate_cached(state.act)
    means3D, shs, opacity, scales, rotations = act["xyz"], act["shs"], act["opacity"], act["scales"], act["rotations"]
    if camera_type == R.CAMERA_PINHOLE:  # std::tan(FoV * 0.5f) in float (gaussian_renderer.cpp:58-59)
        tanfovx = float(np.tan(np.float32(viewpoint.FoVx) * np.float32(0.5)))
        tanfovy = float(np.tan(np.float32(viewpoint.FoVy) * np.float32(0.5)))
    else:
        tanfovx = tanfovy = 0.0
    vm, pm, cp = viewpoint.world_view_transform, viewpoint.full_proj_transform, viewpoint.camera_center
    nr, image, radii, geom, binning, img = R.RasterizeGaussiansCUDA(
        bg_color, means3D, None, opacity, scales, rotations, 1.0, None, vm, pm, tanfovx, tanfovy, image_height,
        image_width, shs, pc.active_sh_degree, cp, False, camera_type)
    if state.dimg is None or state.dimg.shape != image.shape:
        state.dimg = torch.empty_like(image)
    masked = image * mask if mask is not None else image
    if skip_bottom_ratio > 0.0:
        kept = image_height - skip_bottom_rows(image_height, skip_bottom_ratio)
        if kept <= 0 or kept == image_height:
            # pix == 0 makes the reference's Slice(0, -pix) empty (kept == H here), which its conv2d rejects, and so
            # is a crop of every row
            raise ValueError(f"skip_bottom_ratio {skip_bottom_ratio} keeps {kept} of {image_height} rows")
        dtop = torch.empty((image.shape[0], kept, image_width), dtype=image.dtype, device=dev)
        terms, _ = losses.l1_ssim_loss_and_grad(masked[:, :kept], gt_image[:, :kept], lambda_dssim, grad_out=dtop)
        state.dimg[:, :kept].copy_(dtop)
        state.dimg[:, kept:].zero_()
        dimg = state.dimg
    else:
        terms, dimg = losses.l1_ssim_loss_and_grad(masked, gt_image, lambda_dssim, grad_out=state.dimg)
    if mask is not None:
        dimg.mul_(mask)
    if state.buf is None or state.buf.P != P or state.buf.M != Mr + 1:
        state.buf = GradBuffer(P, Mr + 1, dev)
    out = state.buf.out_dict(dev)
    R.RasterizeGaussiansBackwardCUDA(bg_color, means3D, radii, None, scales, rotations, 1.0, None, vm, pm, tanfovx,
                                     tanfovy, dimg, shs, pc.active_sh_degree, cp, geom, nr, binning, img, camera_type,
                                     out=out)
    if dist_info is not None and dist_info.enabled:
        allreduce_compact_(state.buf, dist_info, out["dL_dcolors"], cp,
                           lambda c, d, out: R.sh_grad_from_colors(means3D, shs, pc.active_sh_degree, c, d, out=out),
                           rebuild_packed=lambda pk, out: R.sh_grad_from_colors_packed(means3D, shs,
                                                                                      pc.active_sh_degree, pk, out=out))
    # Adam + the next step's activations + max_radii2D / addDensificationStats (this rank's own dL_dmeans2D, which the
    # exchange leaves alone) in one launch
    opt.step(raster_grads=out, act_out=state.act,
             densify_stats=(out["dL_dmeans2D"], radii) if densification_stats else None)
    return terms, image, radii

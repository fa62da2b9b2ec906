"""Renderer glue: GaussianRenderer::renderLonlat / ::render (src/gaussian_renderer.cpp:30-290) and the model
activations they use (src/gaussian_model.cpp:54-90), on the gfx950 rasterizer.

Returns the reference's tuple (rendered_image, viewspace_points, visibility_filter, radii); gradients flow to
the raw model parameters through torch.autograd (exp / normalize / sigmoid / cat are cheap elementwise torch
ops; everything per-pixel runs in libomnigs_raster.so).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

from . import rasterizer as R

SH_C0 = 0.28209479177387814
SH_C1 = 0.4886025119029199
SH_C2 = (1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792, 0.5462742152960396)
SH_C3 = (-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154, -0.4570457994644658,
         1.445305721320277, -0.5900435899266435)


@dataclass
class GaussianModelParams:
    """The trainable tensors of GaussianModel (include/gaussian_model.h), raw (pre-activation)."""
    xyz: torch.Tensor            # [P,3]
    features_dc: torch.Tensor    # [P,1,3]
    features_rest: torch.Tensor  # [P,(max_deg+1)^2-1,3]
    opacity: torch.Tensor        # [P,1] logit
    scaling: torch.Tensor        # [P,3] log
    rotation: torch.Tensor       # [P,4] unnormalised (r,x,y,z)
    active_sh_degree: int = 3
    max_sh_degree: int = 3

    # gaussian_model.cpp:54-77
    def get_scaling_activation(self):
        return torch.exp(self.scaling)

    def get_rotation_activation(self):
        return torch.nn.functional.normalize(self.rotation)

    def get_xyz(self):
        return self.xyz

    def get_features(self):
        return torch.cat([self.features_dc, self.features_rest], dim=1)

    def get_opacity_activation(self):
        return torch.sigmoid(self.opacity)

    def get_covariance_activation(self, scaling_modifier: int = 1):
        """build_rotation + build_scaling_rotation + strip_symmetric (gaussian_model.cpp:79-108,
        general_utils.h:34-58). The reference's modifier is an `int` defaulting to 1 and the renderer calls it
        without one (gaussian_renderer.cpp:94, :226), so the precomputed-cov3D path ignores scaling_modifier."""
        s = int(scaling_modifier) * self.get_scaling_activation()
        q = self.rotation / torch.sqrt((self.rotation * self.rotation).sum(-1, keepdim=True))
        r, x, y, z = q.unbind(-1)
        Rm = torch.stack([
            torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y)], -1),
            torch.stack([2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x)], -1),
            torch.stack([2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)], -1)], -2)
        Lm = Rm * s[:, None, :]
        S = Lm @ Lm.transpose(1, 2)
        return torch.stack([S[:, 0, 0], S[:, 0, 1], S[:, 0, 2], S[:, 1, 1], S[:, 1, 2], S[:, 2, 2]], -1)

    @staticmethod
    def from_activated(means3D, scales, rotations, opacity, shs, sh_degree=3):
        """Raw parameters whose activations equal the given (activated) tensors."""
        P = means3D.shape[0]
        o = torch.clamp(opacity, 1e-7, 1 - 1e-7)
        return GaussianModelParams(means3D.clone(), shs[:, :1].clone(), shs[:, 1:].clone(), torch.log(o / (1 - o)),
                                   torch.log(scales), rotations.clone(), sh_degree,
                                   int(round(math.sqrt(shs.shape[1]))) - 1 if P else sh_degree)

    def parameters(self):
        return [self.xyz, self.features_dc, self.features_rest, self.opacity, self.scaling, self.rotation]


@dataclass
class Viewpoint:
    """The camera fields of GaussianKeyframe the renderer reads (gaussian_keyframe.cpp:132-163)."""
    world_view_transform: torch.Tensor  # Tcw^T
    full_proj_transform: torch.Tensor   # (P Tcw)^T
    camera_center: torch.Tensor         # [3]
    FoVx: float = 0.0
    FoVy: float = 0.0
    RwcT: Optional[torch.Tensor] = None


@dataclass
class PipelineParams:
    convert_SHs: bool = False   # cfg/lonlat/*.yaml: 0
    compute_cov3D: bool = False  # cfg/lonlat/*.yaml: 0


def eval_sh(deg: int, sh: torch.Tensor, dirs: torch.Tensor) -> torch.Tensor:
    """sh_utils::eval_sh: sh [..., C, (deg+1)^2], dirs [..., 3] -> [..., C]."""
    result = SH_C0 * sh[..., 0]
    if deg > 0:
        x, y, z = dirs[..., 0:1], dirs[..., 1:2], dirs[..., 2:3]
        result = result - SH_C1 * y * sh[..., 1] + SH_C1 * z * sh[..., 2] - SH_C1 * x * sh[..., 3]
        if deg > 1:
            xx, yy, zz, xy, yz, xz = x * x, y * y, z * z, x * y, y * z, x * z
            result = (result + SH_C2[0] * xy * sh[..., 4] + SH_C2[1] * yz * sh[..., 5] +
                      SH_C2[2] * (2.0 * zz - xx - yy) * sh[..., 6] + SH_C2[3] * xz * sh[..., 7] +
                      SH_C2[4] * (xx - yy) * sh[..., 8])
            if deg > 2:
                result = (result + SH_C3[0] * y * (3 * xx - yy) * sh[..., 9] + SH_C3[1] * xy * z * sh[..., 10] +
                          SH_C3[2] * y * (4 * zz - xx - yy) * sh[..., 11] +
                          SH_C3[3] * z * (2 * zz - 3 * xx - 3 * yy) * sh[..., 12] +
                          SH_C3[4] * x * (4 * zz - xx - yy) * sh[..., 13] + SH_C3[5] * z * (xx - yy) * sh[..., 14] +
                          SH_C3[6] * x * (xx - 3 * yy) * sh[..., 15])
    return result


def _render(cam: Viewpoint, image_height: int, image_width: int, pc: GaussianModelParams, pipe: PipelineParams,
            bg_color: torch.Tensor, override_color: Optional[torch.Tensor], scaling_modifier: float,
            camera_type: int, render_depth: bool):
    xyz = pc.get_xyz()
    screenspace_points = torch.zeros_like(xyz, requires_grad=True)
    try:
        screenspace_points.retain_grad()
    except RuntimeError:
        pass
    if camera_type == R.CAMERA_PINHOLE:  # std::tan(FoV * 0.5f) in float (gaussian_renderer.cpp:58-59)
        tanfovx = float(np.tan(np.float32(cam.FoVx) * np.float32(0.5)))
        tanfovy = float(np.tan(np.float32(cam.FoVy) * np.float32(0.5)))
    else:
        tanfovx = tanfovy = 0.0
    settings = R.GaussianRasterizationSettings(image_height, image_width, tanfovx, tanfovy, bg_color, scaling_modifier,
                                               cam.world_view_transform, cam.full_proj_transform, cam.RwcT,
                                               pc.active_sh_degree, cam.camera_center, False, camera_type,
                                               render_depth)
    rasterizer = R.GaussianRasterizer(settings)
    scales = rotations = cov3D_precomp = None
    if pipe.compute_cov3D:
        cov3D_precomp = pc.get_covariance_activation()
    else:
        scales, rotations = pc.get_scaling_activation(), pc.get_rotation_activation()
    shs = colors_precomp = None
    if override_color is not None:
        colors_precomp = override_color
    elif pipe.convert_SHs:
        feats = pc.get_features()
        shs_view = feats.transpose(1, 2).reshape(-1, 3, (pc.max_sh_degree + 1) ** 2)
        dir_pp = xyz - cam.camera_center.repeat(feats.shape[0], 1)
        dir_pp = dir_pp / dir_pp.norm(dim=1, keepdim=True)
        colors_precomp = torch.clamp_min(eval_sh(pc.active_sh_degree, shs_view, dir_pp) + 0.5, 0.0)
    else:
        shs = pc.get_features()
    image, radii = rasterizer(xyz, screenspace_points, pc.get_opacity_activation(), shs=shs,
                              colors_precomp=colors_precomp, scales=scales, rotations=rotations,
                              cov3D_precomp=cov3D_precomp)
    return image, screenspace_points, radii > 0, radii


def render_lonlat(viewpoint_camera: Viewpoint, image_height: int, image_width: int, pc: GaussianModelParams,
                  pipe: PipelineParams, bg_color: torch.Tensor, override_color: Optional[torch.Tensor] = None,
                  scaling_modifier: float = 1.0):
    """GaussianRenderer::renderLonlat (gaussian_renderer.cpp:167-290)."""
    return _render(viewpoint_camera, image_height, image_width, pc, pipe, bg_color, override_color, scaling_modifier,
                   R.CAMERA_LONLAT, False)


def render(viewpoint_camera: Viewpoint, image_height: int, image_width: int, pc: GaussianModelParams,
           pipe: PipelineParams, bg_color: torch.Tensor, override_color: Optional[torch.Tensor] = None,
           render_depth: bool = False, scaling_modifier: float = 1.0):
    """GaussianRenderer::render (gaussian_renderer.cpp:30-160), pinhole."""
    return _render(viewpoint_camera, image_height, image_width, pc, pipe, bg_color, override_color, scaling_modifier,
                   R.CAMERA_PINHOLE, render_depth)

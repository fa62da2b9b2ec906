"""GaussianModel's optimizer, learning-rate schedule and densification on gfx950.

Mirrors, with the reference's names and argument meaning:
  * GaussianModel::trainingSetup          gaussian_model.cpp:485-518   -> GaussianOptimizer.__init__
  * GaussianModel::updateLearningRate     :520-532, exponLrFunc :1140-1152 -> update_learning_rate / expon_lr
  * set{Position,Feature,Opacity,Scaling,Rotation}LearningRate :541-562
  * optimizer_->step(); zero_grad(true)   gaussian_mapper.cpp:484-488  -> step() / zero_grad()
  * addDensificationStats + max_radii2D   gaussian_model.cpp:839-853, gaussian_mapper.cpp:427-434
  * densifyAndPrune (clone, split, prune) gaussian_model.cpp:619-837    -> densify_and_prune
  * resetOpacity                          gaussian_model.cpp:564-592    -> reset_opacity

All arithmetic runs in libomnigs_raster.so (csrc/optim.hip): one Adam launch for the six groups, either on the raw
gradients autograd leaves in .grad (step()) or straight on the rasterizer backward's gradients w.r.t. the activated
tensors (step(raster_grads=...)), applying the activation backward (cat / sigmoid / exp / normalize) in registers —
the training step then needs no autograd graph at all. torch allocates memory and draws the split samples.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

from . import rasterizer as R

GROUPS = ("xyz", "features_dc", "features_rest", "opacity", "scaling", "rotation")


@dataclass
class OptimizationParams:
    """GaussianOptimizationParams as the reference's lonlat configs set them (cfg/lonlat/360roam_lonlat.yaml:55-78)."""
    iterations: int = 32010
    position_lr_init: float = 0.00016
    position_lr_final: float = 0.0000016
    position_lr_delay_mult: float = 0.01
    position_lr_max_steps: int = 30000
    feature_lr: float = 0.0025
    opacity_lr: float = 0.05
    scaling_lr: float = 0.005
    rotation_lr: float = 0.001
    percent_dense: float = 0.01
    lambda_dssim: float = 0.2
    densification_interval: int = 100
    opacity_reset_interval: int = 3000
    prune_big_point_after_iter: int = 0
    densify_min_opacity: float = 0.005
    densify_from_iter: int = 500
    densify_until_iter: int = 15000
    densify_grad_threshold: float = 0.0002
    prune_by_extent: bool = True


def expon_lr(step: int, lr_init: float, lr_final: float, lr_delay_steps: int = 0, lr_delay_mult: float = 1.0,
             max_steps: int = 1000000) -> float:
    """GaussianModel::exponLrFunc (gaussian_model.cpp:1140-1152), in the reference's float arithmetic."""
    f = np.float32
    lr_init, lr_final = f(lr_init), f(lr_final)
    if step < 0 or (lr_init == 0 and lr_final == 0):
        return 0.0
    if lr_delay_steps > 0:
        c = np.clip(f(step) / f(lr_delay_steps), f(0), f(1))
        delay_rate = f(lr_delay_mult) + (f(1) - f(lr_delay_mult)) * np.sin(f(np.pi / 2) * c)
    else:
        delay_rate = f(1)
    t = np.clip(f(step) / f(max_steps), f(0), f(1))
    log_lerp = np.exp(np.log(lr_init) * (f(1) - t) + np.log(lr_final) * t)
    return float(f(delay_rate * log_lerp))


def _p6(ts):
    return (C.c_void_p * 6)(*[None if t is None or t.numel() == 0 else t.data_ptr() for t in ts])


def _check_dev(t: torch.Tensor, name: str, dtype=torch.float32):
    if t.device.type != "cuda":
        raise R.RasterizerError(f"{name} must be on a HIP device (got {t.device}); the optimizer has no CPU path")
    if t.dtype != dtype:
        raise R.RasterizerError(f"{name} must be {dtype} (got {t.dtype})")
    if not t.is_contiguous():
        raise R.RasterizerError(f"{name} must be contiguous")


class GaussianOptimizer:
    """torch::optim::Adam over GaussianModel's six parameter groups plus the densification state, as
    GaussianModel::trainingSetup builds them (gaussian_model.cpp:485-518). `model` is a
    renderer.GaussianModelParams; its tensors are updated in place by step() and replaced by densify_and_prune()."""

    def __init__(self, model, args: OptimizationParams, spatial_lr_scale: float = 1.0, betas=(0.9, 0.999),
                 eps: float = 1e-15):
        self.model = model
        self.args = args
        self.spatial_lr_scale = float(spatial_lr_scale)
        self.percent_dense = args.percent_dense
        self.betas = (float(betas[0]), float(betas[1]))
        self.eps = float(eps)
        self.lr = [args.position_lr_init * self.spatial_lr_scale, args.feature_lr, args.feature_lr / 20.0,
                   args.opacity_lr, args.scaling_lr, args.rotation_lr]
        # get_expon_lr_func arguments (:514-517); lr_delay_steps_ stays at its constructor value 0 (:26)
        self.lr_init = args.position_lr_init * self.spatial_lr_scale
        self.lr_final = args.position_lr_final * self.spatial_lr_scale
        self.lr_delay_steps = 0
        self.lr_delay_mult = args.position_lr_delay_mult
        self.max_steps = args.position_lr_max_steps
        params = self.params()
        for name, p in zip(GROUPS, params):
            _check_dev(p, name)
        self.steps = [0] * 6
        self.exp_avg = [torch.zeros_like(p) for p in params]
        self.exp_avg_sq = [torch.zeros_like(p) for p in params]
        P, dev = params[0].shape[0], params[0].device
        self.xyz_gradient_accum = torch.zeros((P, 1), device=dev)
        self.denom = torch.zeros((P, 1), device=dev)
        self.max_radii2D = torch.zeros((P,), device=dev)
        self.exist_since_iter = torch.zeros((P,), dtype=torch.int32, device=dev)
        self._plan = None
        self._act_key = None  # what the last activated outputs were computed from (activate_cached)

    # ---- parameters ------------------------------------------------------------------------------------------
    def params(self):
        m = self.model
        return [m.xyz, m.features_dc, m.features_rest, m.opacity, m.scaling, m.rotation]

    def _set_params(self, ps):
        m = self.model
        m.xyz, m.features_dc, m.features_rest, m.opacity, m.scaling, m.rotation = ps

    @property
    def P(self) -> int:
        return self.model.xyz.shape[0]

    @property
    def Mr(self) -> int:
        return self.model.features_rest.shape[1]

    # ---- learning rates (gaussian_model.cpp:520-562) ---------------------------------------------------------
    def update_learning_rate(self, step: int) -> float:
        lr = expon_lr(step, self.lr_init, self.lr_final, self.lr_delay_steps, self.lr_delay_mult, self.max_steps)
        self.lr[0] = lr
        return lr

    def set_position_learning_rate(self, lr: float):
        self.lr[0] = lr * self.spatial_lr_scale

    def set_feature_learning_rate(self, lr: float):
        self.lr[1], self.lr[2] = lr, lr / 20.0

    def set_opacity_learning_rate(self, lr: float):
        self.lr[3] = lr

    def set_scaling_learning_rate(self, lr: float):
        self.lr[4] = lr

    def set_rotation_learning_rate(self, lr: float):
        self.lr[5] = lr

    # ---- the renderer's activations (gaussian_model.cpp:54-77) ----------------------------------------------------
    def _act_buffers(self, out: Optional[dict]) -> dict:
        ps = self.params()
        P, Mr, dev = self.P, self.Mr, ps[0].device
        shapes = dict(shs=(P, Mr + 1, 3), opacity=(P, 1), scales=(P, 3), rotations=(P, 4))
        out = {} if out is None else out
        for k, shp in shapes.items():
            t = out.get(k)
            if t is None or tuple(t.shape) != shp or t.device != dev:
                out[k] = torch.empty(shp, dtype=torch.float32, device=dev)
        out["xyz"] = ps[0]
        return out

    def _key(self, out: dict):
        """The activated outputs in `out` are current while the parameters are the same tensor OBJECTS (the key holds
        them, so a new tensor at a reused address never matches), untouched by torch in-place ops (their _version),
        and no raw-pointer write other than Adam's (reset_opacity, densify) happened. Writes torch does not version
        (through `p.data`, e.g. p.data.copy_ when loading a checkpoint) are invisible here: call invalidate()."""
        ps = self.params()
        return (id(out), tuple(ps), tuple((p.data_ptr(), p._version, tuple(p.shape)) for p in ps),
                tuple(out[k].data_ptr() for k in ("shs", "opacity", "scales", "rotations")))

    @staticmethod
    def _same_key(a, b) -> bool:
        return (a is not None and b is not None and a[0] == b[0] and len(a[1]) == len(b[1])
                and all(x is y for x, y in zip(a[1], b[1])) and a[2:] == b[2:])

    def invalidate(self):
        """Forget that the activated outputs are current: the next activate_cached() recomputes them. Needed after
        any write to the parameters that torch does not version (p.data.copy_, raw-pointer writes by other code)."""
        self._act_key = None

    def activate(self, out: Optional[dict] = None) -> dict:
        """cat(features_dc, features_rest), sigmoid(opacity), exp(scaling), normalize(rotation) in one launch
        (omr_activate), into the tensors of `out` (keys shs, opacity, scales, rotations; reused when their shapes
        match, else allocated). xyz is passed through. Returns the dict."""
        out = self._act_buffers(out)
        ps = self.params()
        rc = R.lib().omr_activate(self.P, self.Mr, _p6(ps), out["shs"].data_ptr(), out["opacity"].data_ptr(),
                                  out["scales"].data_ptr(), out["rotations"].data_ptr(), R._stream(ps[0].device))
        R._check(rc, "omr_activate")
        self._act_key = self._key(out)
        return out

    def activate_cached(self, out: dict) -> dict:
        """`out` as activate() would fill it, launching omr_activate only when the last step(act_out=out) (or
        activate(out)) did not already leave the activations of the current parameters there."""
        if self._act_key is not None and all(k in out for k in ("shs", "opacity", "scales", "rotations")):
            out["xyz"] = self.params()[0]
            if self._same_key(self._key(out), self._act_key):
                return out
        return self.activate(out)

    # ---- Adam ------------------------------------------------------------------------------------------------
    def step(self, raster_grads: Optional[dict] = None, act_out: Optional[dict] = None, densify_stats=None):
        """optimizer_->step(). Without arguments: Adam on each parameter's .grad (groups whose .grad is None are
        skipped, as adam.cpp does). With raster_grads = the rasterizer backward's outputs (dL_dmeans3D, dL_dsh,
        dL_dopacity, dL_dscales, dL_drotations — e.g. parallel.GradBuffer.views), the activation backward is fused
        into the same launch and no .grad is needed. With act_out (a dict as activate() fills; raster_grads
        required) the same launch also writes the activations of the updated parameters there
        (omr_adam_step_activate), and activate_cached(act_out) then has nothing to do; densify_stats =
        (viewspace_grad, radii) (act_out required) folds add_densification_stats into that launch too."""
        if act_out is not None and raster_grads is None:
            raise R.RasterizerError("step(act_out=...) needs raster_grads")
        if densify_stats is not None and act_out is None:
            raise R.RasterizerError("step(densify_stats=...) needs act_out (omr_adam_step_activate)")
        ps = self.params()
        P, Mr = self.P, self.Mr
        if raster_grads is not None:
            g = raster_grads
            grads = [g["dL_dmeans3D"], g["dL_dsh"], g["dL_dsh"], g["dL_dopacity"], g["dL_dscales"], g["dL_drotations"]]
            for name, t in zip(("dL_dmeans3D", "dL_dsh", "dL_dsh", "dL_dopacity", "dL_dscales", "dL_drotations"), grads):
                _check_dev(t, name)
            if grads[1].numel() != P * (Mr + 1) * 3:
                raise R.RasterizerError(f"dL_dsh has {grads[1].numel()} floats, expected P*(Mr+1)*3 = {P * (Mr + 1) * 3}")
            active = [True] * 6
            kind = 1
        else:
            grads = [p.grad for p in ps]
            active = [gr is not None for gr in grads]
            for name, gr, p in zip(GROUPS, grads, ps):
                if gr is not None:
                    _check_dev(gr, name + ".grad")
                    if gr.shape != p.shape:
                        raise R.RasterizerError(f"{name}.grad shape {tuple(gr.shape)} != {tuple(p.shape)}")
            kind = 0
        for k in range(6):
            if active[k]:
                self.steps[k] += 1
        use = lambda ts: [t if active[k] else None for k, t in enumerate(ts)]  # noqa: E731
        lr = (C.c_float * 6)(*self.lr)
        st = (C.c_int64 * 6)(*[max(s, 1) for s in self.steps])
        stream = R._stream(ps[0].device)
        if act_out is not None:
            act_out = self._act_buffers(act_out)
            stats = [None, None, 0, None, None, None]
            if densify_stats is not None:
                vgrad, radii = self._stats_inputs(*densify_stats)
                stats = [radii.data_ptr(), vgrad.data_ptr(), vgrad.shape[1], self.xyz_gradient_accum.data_ptr(),
                         self.denom.data_ptr(), self.max_radii2D.data_ptr()]
            rc = R.lib().omr_adam_step_activate(P, Mr, _p6(ps), _p6(self.exp_avg), _p6(self.exp_avg_sq), _p6(grads), lr,
                                                st, self.betas[0], self.betas[1], self.eps, act_out["shs"].data_ptr(),
                                                act_out["opacity"].data_ptr(), act_out["scales"].data_ptr(),
                                                act_out["rotations"].data_ptr(), *stats, stream)
            R._check(rc, "omr_adam_step_activate")
            self._act_key = self._key(act_out)
            return
        rc = R.lib().omr_adam_step(P, Mr, _p6(use(ps)), _p6(self.exp_avg), _p6(self.exp_avg_sq), _p6(use(grads)), kind,
                                   lr, st, self.betas[0], self.betas[1], self.eps, stream)
        R._check(rc, "omr_adam_step")
        self._act_key = None  # the parameters moved

    def zero_grad(self):
        """zero_grad(true): gradients are set to None."""
        for p in self.params():
            p.grad = None

    # ---- densification (gaussian_model.cpp:564-853) -----------------------------------------------------------
    def _stats_inputs(self, viewspace_grad: torch.Tensor, radii: torch.Tensor):
        _check_dev(viewspace_grad, "viewspace_grad")
        _check_dev(radii, "radii", torch.int32)
        if viewspace_grad.shape[0] != self.P or radii.numel() != self.P or viewspace_grad.dim() != 2 \
                or viewspace_grad.shape[1] < 2:
            raise R.RasterizerError("viewspace_grad [P, >=2] / radii [P] do not match the model's P")
        return viewspace_grad, radii

    def add_densification_stats(self, viewspace_grad: torch.Tensor, radii: torch.Tensor):
        """max_radii2D[vis] = max(max_radii2D[vis], radii[vis]) (gaussian_mapper.cpp:429-432) and
        addDensificationStats (gaussian_model.cpp:839-853) for vis = radii > 0. viewspace_grad is the means2D
        gradient [P,3] (viewspace_point_tensor.grad(), or the rasterizer backward's dL_dmeans2D)."""
        _check_dev(viewspace_grad, "viewspace_grad")
        _check_dev(radii, "radii", torch.int32)
        P = self.P
        if viewspace_grad.shape[0] != P or radii.numel() != P:
            raise R.RasterizerError("viewspace_grad / radii do not match the model's P")
        rc = R.lib().omr_densification_stats(P, radii.data_ptr(), viewspace_grad.data_ptr(), viewspace_grad.shape[1],
                                             self.xyz_gradient_accum.data_ptr(), self.denom.data_ptr(),
                                             self.max_radii2D.data_ptr(), R._stream(radii.device))
        R._check(rc, "omr_densification_stats")

    def sync_densification_stats(self, dist_info=None):
        """View-parallel training: sum xyz_gradient_accum / denom and take the max of max_radii2D over the ranks
        (SURVEY.md §8(e)), so every replica densifies identically. Call before densify_and_prune."""
        import torch.distributed as dist

        if dist_info is None or not dist_info.enabled:
            return
        dist.all_reduce(self.xyz_gradient_accum, op=dist.ReduceOp.SUM)
        dist.all_reduce(self.denom, op=dist.ReduceOp.SUM)
        dist.all_reduce(self.max_radii2D, op=dist.ReduceOp.MAX)

    def densify_and_prune(self, max_grad: float, min_opacity: float, extent: float, max_screen_size: int,
                          prune_by_extent: bool = True, normals: Optional[torch.Tensor] = None,
                          generator: Optional[torch.Generator] = None) -> dict:
        """densifyAndPrune (gaussian_model.cpp:812-837). The split samples are standard normals drawn with torch
        (the reference's at::normal, :751) unless `normals` [2*S,3] is given; view-parallel replicas must pass the
        same samples (or identically seeded generators) to stay identical. Returns the plan's counts."""
        ps = self.params()
        P, Mr, dev = self.P, self.Mr, ps[0].device
        L = R.lib()
        nbytes = int(L.omr_densify_plan_bytes(P))
        if self._plan is None or self._plan.numel() < nbytes:
            self._plan = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=dev)
        counts = (C.c_int64 * 4)()
        stream = R._stream(dev)
        rc = L.omr_densify_plan(P, self.xyz_gradient_accum.data_ptr(), self.denom.data_ptr(), ps[4].data_ptr(),
                                ps[3].data_ptr(), float(max_grad), float(min_opacity), float(extent),
                                float(self.percent_dense), int(max_screen_size), int(bool(prune_by_extent)),
                                self._plan.data_ptr(), counts, stream)
        R._check(rc, "omr_densify_plan")
        P_new, n_clone, n_split_sel, n_split_kept = (int(c) for c in counts)
        if normals is None:
            normals = torch.randn((2 * n_split_sel, 3), device=dev, generator=generator)
        else:
            _check_dev(normals, "normals")
            if normals.numel() < 6 * n_split_sel:
                raise R.RasterizerError(f"normals needs {2 * n_split_sel} rows of 3")
        shapes = [(P_new,) + tuple(p.shape[1:]) for p in ps]
        new_p = [torch.empty(s, device=dev) for s in shapes]
        new_m = [torch.empty(s, device=dev) for s in shapes]
        new_v = [torch.empty(s, device=dev) for s in shapes]
        new_exist = torch.empty((P_new,), dtype=torch.int32, device=dev)
        if P_new:  # (everything pruned: nothing to write)
            rc = L.omr_densify_apply(P, Mr, self._plan.data_ptr(), _p6(ps), _p6(self.exp_avg), _p6(self.exp_avg_sq),
                                     self.exist_since_iter.data_ptr(), normals.data_ptr() if normals.numel() else None,
                                     _p6(new_p), _p6(new_m), _p6(new_v), new_exist.data_ptr(), stream)
            R._check(rc, "omr_densify_apply")
        for old, new in zip(ps, new_p):
            new.requires_grad_(old.requires_grad)
        self._set_params(new_p)
        self._act_key = None
        self.exp_avg, self.exp_avg_sq, self.exist_since_iter = new_m, new_v, new_exist
        # densificationPostfix resets the statistics (:728-730)
        self.xyz_gradient_accum = torch.zeros((P_new, 1), device=dev)
        self.denom = torch.zeros((P_new, 1), device=dev)
        self.max_radii2D = torch.zeros((P_new,), device=dev)
        return {"P_new": P_new, "clones": n_clone, "splits_selected": n_split_sel, "splits_kept": n_split_kept}

    def reset_opacity(self, ceiling: float = 1.0):
        """resetOpacity (gaussian_model.cpp:564-572). The reference bounds sigmoid(opacity) by
        ones_like(sigmoid(opacity) * 0.01) = 1, so only the opacity group's Adam moments reset (the value round-trips
        through inverse_sigmoid(sigmoid(.))); ceiling=0.01 gives the 3DGS reset the expression was meant to be."""
        op = self.model.opacity
        rc = R.lib().omr_reset_opacity(self.P, op.data_ptr(), self.exp_avg[3].data_ptr(), self.exp_avg_sq[3].data_ptr(),
                                       float(ceiling), R._stream(op.device))
        R._check(rc, "omr_reset_opacity")
        self._act_key = None

"""CPU restatement of the training step after the rasterizer backward (TEST INFRASTRUCTURE ONLY).

Used by tests/ as the parity checker for omnigs-fork_amd/csrc/optim.hip; the product never imports it. numpy,
float32 arithmetic in the reference's operation order:

  * adam_step            torch::optim::Adam::step, LibTorch adam.cpp (the reference pins LibTorch 2.0.1,
                         README.md:29; groups / eps from gaussian_model.cpp:485-518). Pinned against LibTorch's own
                         Adam by tests/golden/make_adam_golden.py.
  * activation_backward  autograd of the renderer's activations (gaussian_model.cpp:54-77: cat, sigmoid, exp,
                         torch::nn::functional::normalize), also pinned by the LibTorch golden.
  * densification_stats  addDensificationStats (gaussian_model.cpp:839-853) + max_radii2D (gaussian_mapper.cpp:427-432)
  * densify_and_prune    densifyAndPrune (gaussian_model.cpp:812-837) as the reference sequences it: densifyAndClone
                         (:779-810) -> densificationPostfix (:671-731) -> densifyAndSplit (:733-777) -> prunePoints
                         (:619-669). Parity unpinned (the reference cannot run here); restated step by step, unlike
                         the kernel's classify / scan / scatter.
  * reset_opacity        resetOpacity (gaussian_model.cpp:564-572)
"""
from __future__ import annotations

import numpy as np

f32 = np.float32


def adam_step(p, m, v, g, lr, step, beta1=0.9, beta2=0.999, eps=1e-15):
    """One Adam step on float32 arrays (in place); step is the count after its increment."""
    bc1 = 1.0 - beta1 ** step
    bc2 = 1.0 - beta2 ** step
    m *= f32(beta1)
    m += f32(1.0 - beta1) * g
    v *= f32(beta2)
    v += f32(1.0 - beta2) * g * g
    denom = np.sqrt(v) / f32(np.sqrt(bc2)) + f32(eps)
    p += f32(-(lr / bc1)) * (m / denom)


def activation_backward(params, raster_grads):
    """Raw-parameter gradients from the rasterizer's gradients w.r.t. the activated tensors.
    params: [xyz, f_dc, f_rest, opacity, scaling, rotation]; raster_grads: dict of dL_dmeans3D, dL_dsh [P,M,3],
    dL_dopacity, dL_dscales, dL_drotations."""
    xyz, f_dc, f_rest, op, sc, rot = params
    g = raster_grads
    dsh = np.asarray(g["dL_dsh"], f32).reshape(xyz.shape[0], -1, 3)
    y = f32(1) / (f32(1) + np.exp(-op))
    gop = np.asarray(g["dL_dopacity"], f32).reshape(op.shape) * (f32(1) - y) * y
    gsc = np.asarray(g["dL_dscales"], f32).reshape(sc.shape) * np.exp(sc)
    gr = np.asarray(g["dL_drotations"], f32).reshape(rot.shape)
    nrm = np.sqrt((rot * rot).sum(-1, keepdims=True))
    d = np.maximum(nrm, f32(1e-12))
    dot = (gr * rot).sum(-1, keepdims=True)
    gn = np.where(nrm >= f32(1e-12), (-dot / (d * d)) / nrm, f32(0))
    grot = gr / d + rot * gn
    return [np.asarray(g["dL_dmeans3D"], f32).reshape(xyz.shape), dsh[:, :1].copy(), dsh[:, 1:].copy(), gop, gsc,
            grot.astype(f32)]


def densification_stats(radii, vgrad, accum, denom, max_radii):
    vis = radii > 0
    max_radii[vis] = np.maximum(max_radii[vis], radii[vis].astype(f32))
    gx, gy = vgrad[vis, 0], vgrad[vis, 1]
    accum[vis, 0] += np.sqrt(gx * gx + gy * gy)
    denom[vis, 0] += f32(1)


def _sigmoid(x):
    return f32(1) / (f32(1) + np.exp(-x))


def build_rotation(r):
    """general_utils.h:34-59"""
    n = np.sqrt(r[:, 0] * r[:, 0] + r[:, 1] * r[:, 1] + r[:, 2] * r[:, 2] + r[:, 3] * r[:, 3])
    q = r / n[:, None]
    w, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    R = np.zeros((r.shape[0], 3, 3), f32)
    R[:, 0, 0] = 1 - 2 * (y * y + z * z)
    R[:, 0, 1] = 2 * (x * y - w * z)
    R[:, 0, 2] = 2 * (x * z + w * y)
    R[:, 1, 0] = 2 * (x * y + w * z)
    R[:, 1, 1] = 1 - 2 * (x * x + z * z)
    R[:, 1, 2] = 2 * (y * z - w * x)
    R[:, 2, 0] = 2 * (x * z - w * y)
    R[:, 2, 1] = 2 * (y * z + w * x)
    R[:, 2, 2] = 1 - 2 * (x * x + y * y)
    return R


class ModelState:
    """The arrays densifyAndPrune touches: params (6 groups), Adam moments, exist_since_iter, statistics."""

    def __init__(self, params, exp_avg, exp_avg_sq, exist, accum, denom, max_radii):
        self.params = [np.array(p, f32) for p in params]
        self.exp_avg = [np.array(a, f32) for a in exp_avg]
        self.exp_avg_sq = [np.array(a, f32) for a in exp_avg_sq]
        self.exist = np.array(exist, np.int32)
        self.accum = np.array(accum, f32).reshape(-1, 1)
        self.denom = np.array(denom, f32).reshape(-1, 1)
        self.max_radii = np.array(max_radii, f32).reshape(-1)

    @property
    def P(self):
        return self.params[0].shape[0]

    def _postfix(self, new_params, new_exist):  # densificationPostfix (:671-731)
        for k in range(6):
            self.exp_avg[k] = np.concatenate([self.exp_avg[k], np.zeros_like(new_params[k])])
            self.exp_avg_sq[k] = np.concatenate([self.exp_avg_sq[k], np.zeros_like(new_params[k])])
            self.params[k] = np.concatenate([self.params[k], new_params[k]])
        self.exist = np.concatenate([self.exist, new_exist])
        self.accum = np.zeros((self.P, 1), f32)
        self.denom = np.zeros((self.P, 1), f32)
        self.max_radii = np.zeros((self.P,), f32)

    def _prune(self, mask):  # prunePoints (:619-669)
        keep = ~mask
        for k in range(6):
            self.params[k] = self.params[k][keep]
            self.exp_avg[k] = self.exp_avg[k][keep]
            self.exp_avg_sq[k] = self.exp_avg_sq[k][keep]
        self.exist = self.exist[keep]
        self.accum, self.denom, self.max_radii = self.accum[keep], self.denom[keep], self.max_radii[keep]

    def densify_and_prune(self, max_grad, min_opacity, extent, max_screen_size, prune_by_extent, percent_dense,
                          normals):
        """normals: [2 S, 3] standard normal samples for the S split-selected Gaussians (batch-major)."""
        with np.errstate(invalid="ignore", divide="ignore"):
            grads = self.accum / self.denom
        grads[np.isnan(grads)] = 0
        bound = f32(percent_dense) * f32(extent)
        # densifyAndClone (:779-810)
        maxs = np.exp(self.params[4]).max(1)
        sel = (np.abs(grads[:, 0]) >= f32(max_grad)) & (maxs <= bound)
        self._postfix([p[sel] for p in self.params], self.exist[sel])
        # densifyAndSplit (:733-777), N = 2
        n0 = grads.shape[0]
        padded = np.zeros(self.P, f32)
        padded[:n0] = grads[:, 0]
        maxs = np.exp(self.params[4]).max(1)
        sel = (padded >= f32(max_grad)) & (maxs > bound)
        S = int(sel.sum())
        stds = np.tile(np.exp(self.params[4][sel]), (2, 1))
        samples = np.asarray(normals, f32).reshape(-1, 3)[:2 * S] * stds
        rots = np.tile(build_rotation(self.params[5][sel]), (2, 1, 1))
        new_xyz = np.einsum("nij,nj->ni", rots, samples).astype(f32) + np.tile(self.params[0][sel], (2, 1))
        new_sc = np.log(np.tile(np.exp(self.params[4][sel]), (2, 1)) / f32(1.6))
        new = [new_xyz, np.tile(self.params[1][sel], (2, 1, 1)), np.tile(self.params[2][sel], (2, 1, 1)),
               np.tile(self.params[3][sel], (2, 1)), new_sc, np.tile(self.params[5][sel], (2, 1))]
        self._postfix(new, np.tile(self.exist[sel], 2))
        self._prune(np.concatenate([sel, np.zeros(2 * S, bool)]))
        # prune (:824-834); max_radii2D was just reset by densificationPostfix
        prune = (_sigmoid(self.params[3]) < f32(min_opacity)).reshape(-1)
        if max_screen_size:
            big_vs = self.max_radii > max_screen_size
            big_ws = (np.exp(self.params[4]).max(1) > f32(0.1) * f32(extent)) if prune_by_extent else \
                np.zeros_like(big_vs)
            prune = prune | big_vs | big_ws
        self._prune(prune)
        return S


def reset_opacity(opacity, exp_avg, exp_avg_sq, ceiling=1.0):
    """resetOpacity (gaussian_model.cpp:564-572); the reference's bound is ones_like(...) = 1."""
    x = np.minimum(_sigmoid(opacity), f32(ceiling))
    opacity[...] = np.log(x / (f32(1) - x))
    exp_avg[...] = 0
    exp_avg_sq[...] = 0

"""Synthetic Gaussian scenes and camera poses.

Deterministic, platform independent (numpy uint64 SplitMix64), so the oracle, the HIP path, the fixtures and
bench.py all see identical inputs for a given (config, seed).

Conventions follow the reference host:
  * viewmatrix = Tcw^T stored row-major, i.e. Tcw column-major (gaussian_keyframe.cpp:136-140);
  * projmatrix = (P · Tcw)^T with P from GaussianKeyframe::getProjectionMatrix (gaussian_keyframe.cpp:197-225);
  * campos = camera centre = inverse(viewmatrix)[3, :3] (gaussian_keyframe.cpp:163);
  * activated parameters, as GaussianRenderer::renderLonlat feeds them (gaussian_renderer.cpp:167-290):
    scales = exp(.), rotations = normalize(.), opacity = sigmoid(.), shs = cat(f_dc, f_rest) -> [P, 16, 3].
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass

import numpy as np

GOLDEN = np.uint64(0x9E3779B97F4A7C15)
M1 = np.uint64(0xBF58476D1CE4E5B9)
M2 = np.uint64(0x94D049BB133111EB)
BASE_SEED = 0x0A1B2C3D

CAMERA_PINHOLE = 1
CAMERA_LONLAT = 3


_CHUNK = 1 << 20  # values per worker task of the threaded generator


def _pool():
    global _POOL
    if _POOL is None:
        from concurrent.futures import ThreadPoolExecutor

        _POOL = ThreadPoolExecutor(max_workers=max(1, min(16, os.cpu_count() or 1)))
    return _POOL


_POOL = None


class SplitMix64:
    """Sequential SplitMix64 stream; uniform = (x >> 40) * 2^-24, normal = Box-Muller (cos branch).

    Value j of the stream (0-based) is mix(seed + (j + 1) * GOLDEN), so any slice can be computed on its own: long
    draws are split over a thread pool (numpy releases the GIL in its loops) with results identical to one
    sequential pass."""

    def __init__(self, seed: int):
        self.state = np.uint64(seed & 0xFFFFFFFFFFFFFFFF)

    @staticmethod
    def _mix(state, first: int, n: int) -> np.ndarray:
        with np.errstate(over="ignore"):
            k = np.arange(first + 1, first + n + 1, dtype=np.uint64)
            z = state + k * GOLDEN
            z = (z ^ (z >> np.uint64(30))) * M1
            z = (z ^ (z >> np.uint64(27))) * M2
            return z ^ (z >> np.uint64(31))

    def _draw(self, n: int, per_value: int, fn) -> np.ndarray:
        """n outputs, each from `per_value` consecutive stream values; fn maps the u64 slice to the outputs."""
        state = self.state
        with np.errstate(over="ignore"):
            self.state = self.state + np.uint64(n * per_value) * GOLDEN
        if n * per_value <= _CHUNK:
            return fn(self._mix(state, 0, n * per_value))
        out = np.empty(n, dtype=np.float64 if fn is not None else np.uint64)
        step = _CHUNK // per_value

        def work(i0):
            i1 = min(n, i0 + step)
            out[i0:i1] = fn(self._mix(state, i0 * per_value, (i1 - i0) * per_value))

        list(_pool().map(work, range(0, n, step)))
        return out

    def next_u64(self, n: int) -> np.ndarray:
        state = self.state
        with np.errstate(over="ignore"):
            self.state = self.state + np.uint64(n) * GOLDEN
        return self._mix(state, 0, n)

    @staticmethod
    def _uniform(x: np.ndarray) -> np.ndarray:
        return (x >> np.uint64(40)).astype(np.float64) * (1.0 / (1 << 24))

    @staticmethod
    def _normal(x: np.ndarray) -> np.ndarray:
        u = SplitMix64._uniform(x)
        u1 = 1.0 - u[0::2]  # (0, 1]
        u2 = u[1::2]
        return np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * math.pi * u2)

    def uniform(self, n: int) -> np.ndarray:
        return self._draw(n, 1, self._uniform)

    def normal(self, n: int) -> np.ndarray:
        return self._draw(n, 2, self._normal)


@dataclass
class Gaussians:
    means3D: np.ndarray    # [P,3] f32
    scales: np.ndarray     # [P,3] f32 (activated)
    rotations: np.ndarray  # [P,4] f32 (normalised, (r,x,y,z))
    opacity: np.ndarray    # [P,1] f32 (activated)
    shs: np.ndarray        # [P,16,3] f32
    sh_degree: int = 3

    @property
    def P(self) -> int:
        return self.means3D.shape[0]


def make_gaussians(P: int, seed: int) -> Gaussians:
    g = SplitMix64(seed)
    d = g.normal(3 * P).reshape(P, 3)
    d /= np.maximum(np.linalg.norm(d, axis=1, keepdims=True), 1e-12)
    r = 2.0 + 10.0 * g.uniform(P)
    means = d * r[:, None]
    lo, hi = math.log(0.01), math.log(0.08)
    scales = np.exp(lo + (hi - lo) * g.uniform(3 * P)).reshape(P, 3)
    q = g.normal(4 * P).reshape(P, 4)
    q /= np.maximum(np.linalg.norm(q, axis=1, keepdims=True), 1e-12)
    opac = 1.0 / (1.0 + np.exp(-1.5 * g.normal(P)))
    sh = g.normal(P * 16 * 3).reshape(P, 16, 3)
    sh[:, 0, :] *= 0.8
    sh[:, 1:, :] *= 0.15
    f32 = lambda a: np.ascontiguousarray(a, dtype=np.float32)
    return Gaussians(f32(means), f32(scales), f32(q), f32(opac.reshape(P, 1)), f32(sh), 3)


def upstream_grad(H: int, W: int, seed: int, scale: float = 1e-3) -> np.ndarray:
    """dL/dout_color ~ scale * N(0,1), [3,H,W] f32."""
    return np.ascontiguousarray((scale * SplitMix64(seed).normal(3 * H * W)).reshape(3, H, W), dtype=np.float32)


@dataclass
class Camera:
    camera_type: int
    width: int
    height: int
    viewmatrix: np.ndarray  # [4,4] f32 = Tcw^T
    projmatrix: np.ndarray  # [4,4] f32 = (P Tcw)^T (identity-free for lonlat; unused there)
    campos: np.ndarray      # [3] f32
    tanfovx: float = 0.0
    tanfovy: float = 0.0


def yaw_pose(k: int, n: int = 8, radius: float = 0.3):
    """View k of the §8(d) ring: centre 0.3·(cos 2πk/n, 0, sin 2πk/n), yaw 2πk/n about +y. Returns (Rwc, c)."""
    th = 2.0 * math.pi * k / n
    c = np.array([radius * math.cos(th), 0.0, radius * math.sin(th)]) if k else np.zeros(3)
    Rwc = np.array([[math.cos(th), 0.0, math.sin(th)], [0.0, 1.0, 0.0], [-math.sin(th), 0.0, math.cos(th)]])
    return Rwc, c


def world_view(Rwc: np.ndarray, c: np.ndarray) -> np.ndarray:
    Tcw = np.eye(4)
    Tcw[:3, :3] = Rwc.T
    Tcw[:3, 3] = -Rwc.T @ c
    return Tcw


def projection_matrix(znear: float, zfar: float, fovx: float, fovy: float) -> np.ndarray:
    """GaussianKeyframe::getProjectionMatrix (gaussian_keyframe.cpp:197-225)."""
    tan_y, tan_x = math.tan(fovy / 2), math.tan(fovx / 2)
    top, right = tan_y * znear, tan_x * znear
    bottom, left = -top, -right
    P = np.zeros((4, 4))
    P[0, 0] = 2.0 * znear / (right - left)
    P[1, 1] = 2.0 * znear / (top - bottom)
    P[0, 2] = (right + left) / (right - left)
    P[1, 2] = (top + bottom) / (top - bottom)
    P[3, 2] = 1.0
    P[2, 2] = zfar / (zfar - znear)
    P[2, 3] = -(zfar * znear) / (zfar - znear)
    return P


def make_camera(camera_type: int, width: int, height: int, view_index: int = 0,
                tanfovx: float | None = None, tanfovy: float | None = None) -> Camera:
    Rwc, c = yaw_pose(view_index)
    Tcw = world_view(Rwc, c)
    view = Tcw.T
    if camera_type == CAMERA_PINHOLE:
        tx = 1.0 if tanfovx is None else tanfovx
        ty = (height / width) * tx if tanfovy is None else tanfovy
        Pm = projection_matrix(0.01, 100.0, 2 * math.atan(tx), 2 * math.atan(ty))
        proj = (Pm @ Tcw).T
    else:
        tx = ty = 0.0
        proj = Tcw.T  # lonlat ignores projmatrix (rasterizer_impl.cu:540-697); full_proj with P = I
    f32 = lambda a: np.ascontiguousarray(a, dtype=np.float32)
    return Camera(camera_type, width, height, f32(view), f32(proj), f32(c), float(tx), float(ty))


# BASELINE.json configs (index = config position; seed = 0x0A1B2C3D + index)
CONFIGS = {
    "A": dict(index=0, P=10_000, width=512, height=256, camera_type=CAMERA_LONLAT),
    "B": dict(index=1, P=100_000, width=1024, height=512, camera_type=CAMERA_LONLAT),
    "C": dict(index=2, P=1_000_000, width=2048, height=1024, camera_type=CAMERA_LONLAT),
    "D": dict(index=3, P=1_000_000, width=2048, height=1024, camera_type=CAMERA_LONLAT),
    "E": dict(index=4, P=5_000_000, width=4096, height=2048, camera_type=CAMERA_LONLAT),
    "E_pinhole": dict(index=4, P=5_000_000, width=1920, height=1080, camera_type=CAMERA_PINHOLE),
}


def config_scene(name: str, view_index: int = 0, P: int | None = None):
    cfg = CONFIGS[name]
    seed = BASE_SEED + cfg["index"]
    g = make_gaussians(cfg["P"] if P is None else P, seed)
    cam = make_camera(cfg["camera_type"], cfg["width"], cfg["height"], view_index)
    dL = upstream_grad(cfg["height"], cfg["width"], seed + 1000 + view_index)
    return g, cam, dL

"""ctypes wrapper of the CPU oracle (TEST INFRASTRUCTURE ONLY).

Used by tests/ as the parity checker and fixture generator, and by bench.py's cpu_baseline leg. The product
(omnigs-fork_amd/) never imports this module.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")
# builds of the same sources (oracle/Makefile): "base" is the parity checker (no FMA contraction); "fma_gcc" /
# "fma_clang" contract mul+add into FMA as nvcc compiles the reference (oracle/contraction.py); "fast" is the
# -O3 timing build of bench.py's cpu_baseline; "libm" is "base" with glibc's atan2f / asinf instead of omni_math.h's
# (an independent implementation of the transcendentals the tile rects depend on, oracle/contraction.py)
VARIANTS = {"base": "liboracle.so", "fma_gcc": "liboracle_fma_gcc.so", "fma_clang": "liboracle_fma_clang.so",
            "fast": "liboracle_fast.so", "libm": "liboracle_libm.so"}
_libs = {}

_F32 = {"out_color", "depths", "cov3D", "rgb", "final_T", "means2D", "conic_opacity", "dmean2D", "dconic",
        "dopacity", "dcolor", "dmean3D", "dcov3D", "dsh", "dscale", "drot"}
_DT = {"clamped": np.uint8, "radii": np.int32, "tiles_touched": np.uint32, "point_offsets": np.uint32,
       "point_list": np.uint32, "keys": np.uint64, "n_contrib": np.uint32, "ranges": np.uint32}


def build() -> str:
    """Compile oracle/_build/liboracle.so (make) if missing or stale."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib(variant: str = "base"):
    if variant not in _libs:
        path = os.path.join(_HERE, "_build", VARIANTS[variant])
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        vp, i, f, d = C.c_void_p, C.c_int, C.c_float, C.c_double
        L.oracle_new.restype = vp
        L.oracle_new.argtypes = [i]
        L.oracle_free.argtypes = [vp]
        common = [i, i, i, vp, i, i, vp, vp, vp, vp, vp]
        L.oracle_forward_f32.argtypes = [vp] + common + [f, vp, vp, vp, vp, vp, f, f, i, i, i, C.c_char_p, i]
        L.oracle_forward_f64.argtypes = [vp] + common + [d, vp, vp, vp, vp, vp, d, d, i, i, i, C.c_char_p, i]
        L.oracle_backward.argtypes = [vp, vp, i]
        L.oracle_size.restype = C.c_int64
        L.oracle_size.argtypes = [vp, C.c_char_p, C.POINTER(C.c_int)]
        L.oracle_get.argtypes = [vp, C.c_char_p, vp]
        L.oracle_num_rendered.argtypes = [vp]
        L.oracle_set_threads.argtypes = [i]
        L.oracle_higher_msb.restype = C.c_uint32
        L.oracle_higher_msb.argtypes = [C.c_uint32]
        L.oracle_atan2f.restype = f
        L.oracle_atan2f.argtypes = [f, f]
        L.oracle_asinf.restype = f
        L.oracle_asinf.argtypes = [f]
        L.oracle_mark_visible.argtypes = [i, vp, vp, vp, i, vp]
        L.oracle_allowance.argtypes = [vp, C.POINTER(C.c_double), vp, vp, vp, C.POINTER(C.c_int64)]
        L.oracle_allowance_terms.argtypes = [vp, C.POINTER(C.c_double), vp, vp, vp, C.POINTER(C.c_int64), vp, vp]
        L.oracle_owner_grad_bound.argtypes = [vp, vp, vp, i, vp]
        _libs[variant] = L
    return _libs[variant]


def _ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


class Oracle:
    """One rasterizer instance (geometry/binning/image state kept between forward and backward)."""

    def __init__(self, double: bool = False, variant: str = "base"):
        self.double = double
        self.variant = variant
        self.dtype = np.float64 if double else np.float32
        self.L = lib(variant)
        self.h = self.L.oracle_new(1 if double else 0)
        self._keep = []

    def __del__(self):
        try:
            if self.h:
                self.L.oracle_free(self.h)
        except Exception:
            pass

    def _arr(self, a):
        if a is None:
            return None
        a = np.ascontiguousarray(a, dtype=self.dtype)
        self._keep.append(a)
        return a

    def forward(self, *, background, means3D, opacity, scales=None, rotations=None, shs=None, colors_precomp=None,
                cov3D_precomp=None, viewmatrix, projmatrix, campos, width, height, sh_degree=3,
                scale_modifier=1.0, tanfovx=0.0, tanfovy=0.0, prefiltered=False, camera_type=3, render_depth=False):
        self._keep = []
        self.background = np.asarray(background, dtype=np.float64).reshape(3)
        P = int(means3D.shape[0])
        M = 0 if shs is None or shs.shape[0] == 0 else int(shs.shape[1])
        args = [self._arr(x) for x in (background, means3D, shs, colors_precomp, opacity, scales)]
        rest = [self._arr(x) for x in (rotations, cov3D_precomp, viewmatrix, projmatrix, campos)]
        err = C.create_string_buffer(512)
        fn = self.L.oracle_forward_f64 if self.double else self.L.oracle_forward_f32
        L = fn(self.h, P, int(sh_degree), M, _ptr(args[0]), int(width), int(height), _ptr(args[1]), _ptr(args[2]),
               _ptr(args[3]), _ptr(args[4]), _ptr(args[5]), scale_modifier, _ptr(rest[0]), _ptr(rest[1]),
               _ptr(rest[2]), _ptr(rest[3]), _ptr(rest[4]), tanfovx, tanfovy, int(prefiltered), int(camera_type),
               int(render_depth), err, 512)
        if L < 0:
            raise RuntimeError(err.value.decode())
        self.P, self.M, self.W, self.H = P, M, int(width), int(height)
        return L

    def get(self, name: str) -> np.ndarray:
        es = C.c_int(0)
        n = self.L.oracle_size(self.h, name.encode(), C.byref(es))
        if n < 0:
            raise KeyError(name)
        dt = _DT.get(name, self.dtype)
        out = np.empty(n, dtype=dt)
        if n:
            self.L.oracle_get(self.h, name.encode(), _ptr(out))
        return out

    def backward(self, dL_dout: np.ndarray, nthreads: int = 1):
        d = np.ascontiguousarray(dL_dout, dtype=self.dtype)
        self.L.oracle_backward(self.h, _ptr(d), int(nthreads))
        P, M = self.P, self.M
        return dict(dmean2D=self.get("dmean2D").reshape(P, 3), dconic=self.get("dconic").reshape(P, 4),
                    dopacity=self.get("dopacity").reshape(P, 1), dcolor=self.get("dcolor").reshape(P, 3),
                    dmean3D=self.get("dmean3D").reshape(P, 3), dcov3D=self.get("dcov3D").reshape(P, 6),
                    dsh=self.get("dsh").reshape(P, M, 3), dscale=self.get("dscale").reshape(P, 3),
                    drot=self.get("drot").reshape(P, 4))

    # what the reference as compiled may decide differently (oracle/ambiguity.hpp); the parity tests excuse
    # exactly these pixels and Gaussians (tests/helpers.py: reference_allowance)
    ALLOWANCE_DEFAULTS = dict(eps_exp=1e-5, atan_ulps=3, k_eval=8.0, k_pos=4.0, k_depth=8.0)
    ALLOWANCE_COUNTS = ("rect_gaussians", "radius_gaussians", "alpha_pixels", "saturation_pixels", "zero_power_pixels",
                        "order_pixels", "rect_pixels", "order_pairs", "flip_gaussians", "threshold_gaussians",
                        "order_gaussians", "allowed_pixels", "exposed_gaussians")
    PX = dict(alpha=1, saturation=2, zero_power=4, order=8, rect=16)
    G = dict(threshold=1, order=2, rect=4, exposed=8, run=16, radius=32)

    def allowance(self, dL=None, **kw):
        """ambiguity.hpp's allowance_scan on the last (float) forward. Returns (counts dict, flip [P] uint8 of G flags,
        pixel [H, W] uint8 of PX flags, bound [H, W] float32: the largest colour change those decisions can make),
        and with the upstream gradient dL [3, H, W] a fifth item, term [P, 9]: per Gaussian the summed magnitude of
        the pixel terms its flagged decisions can move (dmean2D x y, dconic a b c, dopacity, dcolor r g b)."""
        if self.double:
            raise RuntimeError("allowance needs a float forward")
        prm = dict(self.ALLOWANCE_DEFAULTS, **kw)
        pv = (C.c_double * 5)(prm["eps_exp"], prm["atan_ulps"], prm["k_eval"], prm["k_pos"], prm["k_depth"])
        flip = np.zeros(self.P, dtype=np.uint8)
        pix = np.zeros(self.W * self.H, dtype=np.uint8)
        bound = np.zeros(self.W * self.H, dtype=np.float32)
        counts = (C.c_int64 * 13)()
        d = term = None
        if dL is not None:
            d = np.ascontiguousarray(dL, dtype=np.float32).reshape(3, self.H, self.W)
            term = np.zeros((self.P, 9), dtype=np.float32)
        if self.L.oracle_allowance_terms(self.h, pv, _ptr(flip), _ptr(pix), _ptr(bound), counts, _ptr(d),
                                         _ptr(term)) != 0:
            raise RuntimeError("allowance failed")
        out = {k: int(counts[i]) for i, k in enumerate(self.ALLOWANCE_COUNTS)}
        out.update(prm)
        res = (out, flip, pix.reshape(self.H, self.W), bound.reshape(self.H, self.W))
        return res + (term,) if dL is not None else res

    OWNER_BOUND_LAYOUT = (("dmean2D", 3), ("dcolor", 3), ("dopacity", 1), ("dmean3D", 3), ("dcov3D", 6), ("dsh", None),
                          ("dscale", 3), ("drot", 4))

    def owner_grad_bound(self, term: np.ndarray, ids: np.ndarray) -> dict:
        """ambiguity.hpp owner_grad_bound: for the Gaussians `ids`, the bound on every output gradient element that
        their flagged pixel terms `term` ([P, 9], allowance(dL)) can carry, through the linear preprocess backward at
        this forward's state. Returns {name: [len(ids), k]} in the rasterizer's output layouts."""
        ids = np.ascontiguousarray(ids, dtype=np.int32)
        term = np.ascontiguousarray(term, dtype=np.float32)
        K = 23 + 3 * self.M
        out = np.zeros((len(ids), K), dtype=np.float32)
        if len(ids) and self.L.oracle_owner_grad_bound(self.h, _ptr(term), _ptr(ids), len(ids), _ptr(out)) != K:
            raise RuntimeError("owner_grad_bound failed")
        res, c = {}, 0
        for name, k in self.OWNER_BOUND_LAYOUT:
            k = 3 * self.M if k is None else k
            res[name] = out[:, c:c + k]
            c += k
        return res

    def ambiguity(self, **kw):
        """allowance() as (counts, boolean [P] mask of the Gaussians owning an ambiguous decision)."""
        counts, flip, _, _ = self.allowance(**kw)
        return counts, (flip & 7) != 0

    @property
    def num_rendered(self) -> int:
        return self.L.oracle_num_rendered(self.h)


def set_threads(n: int):
    """OpenMP threads of every loaded build (each links its own OpenMP runtime)."""
    lib()
    for L in _libs.values():
        L.oracle_set_threads(int(n))


def run_scene(g, cam, dL=None, bg=(0.0, 0.0, 0.0), double=False, nthreads=1, variant="base", **kw):
    """Convenience: forward (+ backward if dL given) on a scene.Gaussians / scene.Camera pair."""
    o = Oracle(double, variant)
    L = o.forward(background=np.asarray(bg, dtype=np.float64), means3D=g.means3D, opacity=g.opacity,
                  scales=kw.pop("scales", g.scales), rotations=kw.pop("rotations", g.rotations),
                  shs=kw.pop("shs", g.shs), viewmatrix=cam.viewmatrix, projmatrix=cam.projmatrix, campos=cam.campos,
                  width=cam.width, height=cam.height, sh_degree=kw.pop("sh_degree", g.sh_degree),
                  tanfovx=cam.tanfovx, tanfovy=cam.tanfovy, camera_type=cam.camera_type, **kw)
    grads = o.backward(dL, nthreads) if dL is not None else None
    return o, L, grads

"""Python host mirror of the OmniGS rasterizer boundary, on the gfx950 C ABI (include/omnigs_raster.h).

Mirrors, name for name and argument for argument:
  * include/rasterize_points.h:29-80      -> RasterizeGaussiansCUDA / RasterizeGaussiansBackwardCUDA / markVisible
  * include/gaussian_rasterizer.h:32-141  -> GaussianRasterizationSettings / GaussianRasterizerFunction /
    src/gaussian_rasterizer.cpp:24-223       rasterize_gaussians / GaussianRasterizer

PyTorch here is plumbing only: it owns device memory (the three scratch byte tensors, outputs) and the current
HIP stream. All compute runs in libomnigs_raster.so. There is no CPU fallback: if the HIP library is missing
or a tensor is not on a HIP device, calls raise.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, field
from typing import Optional

import torch

CAMERA_PINHOLE = 1
CAMERA_LONLAT = 3

_HERE = os.path.dirname(os.path.abspath(__file__))
# OMR_LIB_PATH selects another build of the same C ABI (kernel experiments); default: the in-tree library
LIB_PATH = os.environ.get("OMR_LIB_PATH") or os.path.join(_HERE, "lib", "libomnigs_raster.so")
_ALLOC_FN = C.CFUNCTYPE(C.c_void_p, C.c_void_p, C.c_size_t)
_lib = None


class RasterizerError(RuntimeError):
    pass


def lib() -> C.CDLL:
    """Load libomnigs_raster.so (built by __graft_entry__.build() / `make -C omnigs-fork_amd/csrc`)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RasterizerError(f"HIP rasterizer library not built: {LIB_PATH} (run __graft_entry__.build())")
        L = C.CDLL(LIB_PATH)
        vp, i, f, b, sz = C.c_void_p, C.c_int, C.c_float, C.c_bool, C.c_size_t
        L.omr_last_error.restype = C.c_char_p
        L.omr_abi_version.restype = i
        L.omr_rasterizer_mark_visible.argtypes = [i, vp, vp, vp, vp, vp]
        L.omr_lonlat_mark_visible.argtypes = [i, vp, vp]
        allocs = [_ALLOC_FN, vp, _ALLOC_FN, vp, _ALLOC_FN, vp]
        L.omr_rasterizer_forward.argtypes = allocs + [i, i, i, vp, i, i, vp, vp, vp, vp, vp, f, vp, vp, vp, vp, vp, f, f,
                                                      b, vp, vp, b, vp, C.POINTER(i)]
        L.omr_lonlat_forward.argtypes = allocs + [i, i, i, vp, i, i, vp, vp, vp, vp, vp, f, vp, vp, vp, vp, b, vp, vp, vp,
                                                  C.POINTER(i)]
        L.omr_rasterizer_backward.argtypes = [i, i, i, i, vp, i, i, vp, vp, vp, vp, f, vp, vp, vp, vp, vp, f, f, vp, vp,
                                              vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]
        L.omr_lonlat_backward.argtypes = [i, i, i, i, vp, i, i, vp, vp, vp, vp, f, vp, vp, vp, vp, vp, vp, vp, vp, vp,
                                          vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]
        for n in ("omr_geometry_bytes",):
            getattr(L, n).restype = sz
            getattr(L, n).argtypes = [i]
        L.omr_image_bytes.restype = sz
        L.omr_image_bytes.argtypes = [i, i]
        L.omr_binning_bytes.restype = sz
        L.omr_binning_bytes.argtypes = [i, i, i]
        L.omr_forward_status.argtypes = [vp, i, vp]
        L.omr_backward_colors_event.argtypes = [vp]
        L.omr_backward_colors_event.restype = None
        L.omr_backward_chunk_events.argtypes = [i, vp]
        L.omr_backward_chunk_events.restype = None
        L.omr_backward_chunk_begin.argtypes = [i, i, i]
        L.omr_backward_chunk_begin.restype = i
        L.omr_debug_point_list.argtypes = [vp, i, i, i, vp, vp]
        L.omr_debug_point_list_raw.argtypes = [vp, i, i, i, vp, vp]
        L.omr_debug_ranges.argtypes = [vp, i, i, vp, vp]
        L.omr_debug_image_state.argtypes = [vp, i, i, vp, vp, vp]
        L.omr_debug_tile_cost.argtypes = [vp, i, i, vp, vp]
        L.omr_debug_counters.argtypes = [vp, i, vp, vp]
        L.omr_debug_depth_sort_mode.restype = i
        L.omr_debug_depth_sort_mode.argtypes = [i]
        L.omr_debug_binning_mode.restype = i
        L.omr_debug_binning_mode.argtypes = [i]
        L.omr_debug_ssim_mode.restype = i
        L.omr_debug_ssim_mode.argtypes = [i]
        L.omr_debug_bwd_bands.restype = i
        L.omr_debug_bwd_bands.argtypes = [i]
        L.omr_debug_adam_sh_rows.restype = i
        L.omr_debug_adam_sh_rows.argtypes = [i]
        L.omr_debug_set_sh_jac.restype = i
        L.omr_debug_set_sh_jac.argtypes = [vp, i, i, vp]
        L.omr_debug_geometry.argtypes = [vp, i, vp, vp, vp, vp, vp, vp]
        L.omr_debug_wave_sum9.argtypes = [vp, vp, vp]
        L.omr_debug_wave_sum9_lds.argtypes = [vp, vp, vp]
        L.omr_debug_wave_sum9x2.argtypes = [vp, vp, vp]
        L.omr_debug_wave_scans.argtypes = [vp, vp, vp]
        L.omr_profile_enable.argtypes = [i]
        L.omr_sh_grad_from_colors.argtypes = [i, i, i, i, vp, vp, vp, vp, vp, vp]
        L.omr_sh_grad_from_colors_packed.restype = i
        L.omr_sh_grad_from_colors_packed.argtypes = [i, i, i, i, vp, vp, vp, vp, vp]
        L.omr_l1_ssim_scratch_floats.restype = sz
        L.omr_l1_ssim_scratch_floats.argtypes = [i, i, i]
        L.omr_l1_ssim_loss.argtypes = [vp, vp, i, i, i, f, vp, vp, vp, vp]
        P6 = C.c_void_p * 6
        L.omr_adam_step.argtypes = [i, i, P6, P6, P6, P6, i, C.c_float * 6, C.c_int64 * 6, f, f, f, vp]
        L.omr_adam_step_activate.argtypes = [i, i, P6, P6, P6, P6, C.c_float * 6, C.c_int64 * 6, f, f, f, vp, vp, vp,
                                             vp, vp, vp, i, vp, vp, vp, vp]
        L.omr_densification_stats.argtypes = [i, vp, vp, i, vp, vp, vp, vp]
        L.omr_activate.argtypes = [i, i, P6, vp, vp, vp, vp, vp]
        L.omr_densify_plan_bytes.restype = sz
        L.omr_densify_plan_bytes.argtypes = [i]
        L.omr_densify_plan.argtypes = [i, vp, vp, vp, vp, f, f, f, f, i, i, vp, C.c_int64 * 4, vp]
        L.omr_densify_apply.argtypes = [i, i, vp, P6, P6, P6, vp, vp, P6, P6, P6, vp, vp]
        L.omr_reset_opacity.argtypes = [i, vp, vp, vp, f, vp]
        L.omr_dist2_scratch_bytes.restype = sz
        L.omr_dist2_scratch_bytes.argtypes = [i]
        L.omr_dist2.argtypes = [i, vp, vp, vp, vp]
        L.omr_ply_open.argtypes = [C.c_char_p, i, C.POINTER(vp), C.POINTER(C.c_int64)]
        L.omr_ply_read.argtypes = [vp, P6, vp]
        L.omr_ply_close.argtypes = [vp]
        L.omr_ply_close.restype = None
        L.omr_ply_save.argtypes = [C.c_char_p, i, i, P6, vp]
        L.omr_profile_set_mask.argtypes = [C.c_uint32]
        L.omr_profile_read.restype = i
        L.omr_profile_read.argtypes = [C.POINTER(C.c_double), C.POINTER(C.c_uint64), i]
        L.omr_profile_stage_name.restype = C.c_char_p
        L.omr_profile_stage_name.argtypes = [i]
        L.omr_runtime_stats.restype = i
        L.omr_runtime_stats.argtypes = [C.POINTER(C.c_uint64), i]
        L.omr_runtime_stat_name.restype = C.c_char_p
        L.omr_runtime_stat_name.argtypes = [i]
        L.omr_runtime_stats_reset.restype = None
        _lib = L
    return _lib


def libtorch_boundary():
    """The LibTorch drop-in (lib/librasterize_points.so: the reference's rasterize_points.h C++ symbols) through
    its pybind11 module — the same functions a C++ LibTorch host links against."""
    import importlib
    import sys

    libdir = os.path.join(_HERE, "lib")
    if libdir not in sys.path:
        sys.path.insert(0, libdir)
    try:
        return importlib.import_module("_rasterize_points")
    except ImportError as e:
        raise RasterizerError(f"LibTorch drop-in not built ({e}); run __graft_entry__.build()") from e


def _check(rc: int, what: str):
    if rc != 0:
        msg = lib().omr_last_error().decode(errors="replace")
        raise RasterizerError(f"{what} failed (status {rc}): {msg}")


def _ptr(t: Optional[torch.Tensor]):
    """Device pointer of a tensor; None / empty -> NULL ("absent", as data_ptr() of an empty tensor)."""
    if t is None or t.numel() == 0:
        return None
    return t.data_ptr()


def _dev_f32(t: Optional[torch.Tensor], name: str, dev: Optional[torch.device] = None,
             numel: Optional[int] = None) -> Optional[torch.Tensor]:
    """A present input as a contiguous float32 tensor on `dev` (the device of means3D) holding `numel` elements: the
    kernels get raw device pointers, so a host tensor, one on another GPU or a short one would fault there."""
    if t is None or t.numel() == 0:
        return None
    if t.device.type != "cuda":
        raise RasterizerError(f"{name} must be on a HIP device (got {t.device}); the rasterizer has no CPU path")
    if dev is not None and t.device != dev:
        raise RasterizerError(f"{name} must be on {dev} (the device of means3D), got {t.device}")
    if t.dtype != torch.float32:
        raise RasterizerError(f"{name} must be float32 (got {t.dtype})")
    if numel is not None and t.numel() != numel:
        raise RasterizerError(f"{name} must hold {numel} elements, got {t.numel()} (shape {tuple(t.shape)})")
    return t.contiguous()


def _check_sh(sh, P):
    if sh is not None and sh.numel() != 0 and (sh.dim() != 3 or sh.shape[0] != P or sh.shape[2] != 3):
        raise RasterizerError(f"sh must be [P, M, 3] with P = {P}, got {tuple(sh.shape)}")


def _stream(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


class _ByteBuffer:
    """Allocation callback backed by a torch uint8 tensor (plays the role of resizeFunctional,
    src/rasterize_points.cu:41-47).

    The callback closes over a one-element list, not over `self`: a closure that referenced the buffer object would
    form a reference cycle (object -> callback -> closure -> object), so every step's scratch tensors (0.7 GB at
    config C, 7.6 GB at E) would wait for Python's cyclic GC instead of returning to the caching allocator when the
    caller drops them, and the allocator would keep calling hipMalloc for new blocks."""

    def __init__(self, device: torch.device):
        holder = [torch.empty(0, dtype=torch.uint8, device=device)]

        def _cb(ctx, nbytes):
            try:
                holder[0] = torch.empty(int(nbytes), dtype=torch.uint8, device=device)
                return holder[0].data_ptr()
            except Exception:  # out of memory -> NULL -> OMR_ERR_ALLOCATION
                return None

        self._holder = holder
        self.fn = _ALLOC_FN(_cb)

    @property
    def tensor(self) -> torch.Tensor:
        return self._holder[0]


def RasterizeGaussiansCUDA(background, means3D, colors, opacity, scales, rotations, scale_modifier, cov3D_precomp,
                           viewmatrix, projmatrix, tan_fovx, tan_fovy, image_height, image_width, sh, degree, campos,
                           prefiltered, camera_type=CAMERA_PINHOLE, render_depth=False):
    """rasterize_points.cu:49-164. Returns (num_rendered, out_color[3,H,W], radii[P] i32, geomBuffer,
    binningBuffer, imgBuffer)."""
    if means3D.ndim != 2 or means3D.shape[1] != 3:
        raise RasterizerError("means3D must have dimensions (num_points, 3)")
    if camera_type not in (CAMERA_PINHOLE, CAMERA_LONLAT):
        raise RasterizerError("[CudaRasterizer]Invalid camera_type")
    dev = means3D.device
    P, H, W = int(means3D.shape[0]), int(image_height), int(image_width)
    geom, binning, img = _ByteBuffer(dev), _ByteBuffer(dev), _ByteBuffer(dev)
    if P == 0:
        out_color = torch.zeros((3, H, W), dtype=torch.float32, device=dev)
        radii = torch.zeros((0,), dtype=torch.int32, device=dev)
        return 0, out_color, radii, geom.tensor, binning.tensor, img.tensor
    m = _dev_f32(means3D, "means3D")
    if H <= 0 or W <= 0:
        raise RasterizerError(f"image_height and image_width must be positive, got {H} x {W}")
    _check_sh(sh, P)
    M = int(sh.shape[1]) if sh is not None and sh.numel() != 0 and sh.shape[0] != 0 else 0
    bg, shc, col, op = (_dev_f32(background, "background", dev, 3), _dev_f32(sh, "sh", dev),
                        _dev_f32(colors, "colors", dev, 3 * P), _dev_f32(opacity, "opacity", dev, P))
    sc, rot, cov = (_dev_f32(scales, "scales", dev, 3 * P), _dev_f32(rotations, "rotations", dev, 4 * P),
                    _dev_f32(cov3D_precomp, "cov3D_precomp", dev, 6 * P))
    vm, pm, cp = (_dev_f32(viewmatrix, "viewmatrix", dev, 16),
                  _dev_f32(projmatrix, "projmatrix", dev, 16 if camera_type == CAMERA_PINHOLE else None),
                  _dev_f32(campos, "campos", dev, 3))
    out_color = torch.empty((3, H, W), dtype=torch.float32, device=dev)  # every pixel is written
    radii = torch.empty((P,), dtype=torch.int32, device=dev)  # every Gaussian is written
    nr = C.c_int(0)
    L = lib()
    if camera_type == CAMERA_PINHOLE:
        rc = L.omr_rasterizer_forward(geom.fn, None, binning.fn, None, img.fn, None, P, int(degree), M, _ptr(bg), W, H,
                                      _ptr(m), _ptr(shc), _ptr(col), _ptr(op), _ptr(sc), float(scale_modifier),
                                      _ptr(rot), _ptr(cov), _ptr(vm), _ptr(pm), _ptr(cp), float(tan_fovx),
                                      float(tan_fovy), bool(prefiltered), out_color.data_ptr(), radii.data_ptr(),
                                      bool(render_depth), _stream(dev), C.byref(nr))
    else:
        rc = L.omr_lonlat_forward(geom.fn, None, binning.fn, None, img.fn, None, P, int(degree), M, _ptr(bg), W, H,
                                  _ptr(m), _ptr(shc), _ptr(col), _ptr(op), _ptr(sc), float(scale_modifier), _ptr(rot),
                                  _ptr(cov), _ptr(vm), _ptr(cp), bool(prefiltered), out_color.data_ptr(),
                                  radii.data_ptr(), _stream(dev), C.byref(nr))
    _check(rc, "RasterizeGaussiansCUDA")
    return int(nr.value), out_color, radii, geom.tensor, binning.tensor, img.tensor


def backward_chunk_ranges(P, n):
    """The Gaussian ranges [begin, end) of a backward run with n chunk events (omr_backward_chunk_begin)."""
    L = lib()
    b = [int(L.omr_backward_chunk_begin(int(P), int(n), k)) for k in range(int(n) + 1)]
    return [(b[k], b[k + 1]) for k in range(int(n))]


def RasterizeGaussiansBackwardCUDA(background, means3D, radii, colors, scales, rotations, scale_modifier, cov3D_precomp,
                                   viewmatrix, projmatrix, tan_fovx, tan_fovy, dL_dout_color, sh, degree, campos,
                                   geomBuffer, R, binningBuffer, imageBuffer, camera_type=CAMERA_PINHOLE, out=None,
                                   colors_event=None, skip_dsh=False, chunk_events=None):
    """rasterize_points.cu:166-285. Returns (dL_dmeans2D, dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dcov3D, dL_dsh,
    dL_dscales, dL_drotations).

    Extensions for a data-parallel host (parallel.CompactExchange):
      `out`          optional dict of preallocated, contiguous float32 tensors keyed by those names, written in place
                     (every element is written): the gradients land inside one flat all-reduce buffer;
      `colors_event` a torch.cuda.Event recorded on the stream as soon as dL_dcolors is final (after the row sums,
                     before the per-Gaussian backward): the colour all-gather can wait on it and overlap the rest;
      `skip_dsh`     dL_dsh is not written (returned as None): the compact exchange rebuilds the summed SH gradient
                     from the gathered colour gradients, so the per-view one would be overwritten unread;
      `chunk_events` a list of n torch.cuda.Events: the per-Gaussian backward runs over the n Gaussian ranges of
                     backward_chunk_ranges(P, n) and event k is recorded once range k's gradients are final."""
    if camera_type not in (CAMERA_PINHOLE, CAMERA_LONLAT):
        raise RasterizerError("[CudaRasterizer]Invalid camera_type")
    if means3D.ndim != 2 or means3D.shape[1] != 3:
        raise RasterizerError("means3D must have dimensions (num_points, 3)")
    dev = means3D.device
    P = int(means3D.shape[0])
    if dL_dout_color.dim() != 3 or dL_dout_color.shape[0] != 3 or min(dL_dout_color.shape[1:]) <= 0:
        raise RasterizerError(f"dL_dout_color must be [3, H, W], got {tuple(dL_dout_color.shape)}")
    H, W = int(dL_dout_color.shape[1]), int(dL_dout_color.shape[2])
    _check_sh(sh, P)
    M = int(sh.shape[1]) if sh is not None and sh.numel() != 0 and sh.shape[0] != 0 else 0
    if int(R) < 0:
        raise RasterizerError(f"R (num_rendered) must be >= 0, got {R}")
    if P != 0:
        if radii is None or radii.dim() != 1 or radii.shape[0] != P or radii.dtype != torch.int32 or radii.device != dev:
            raise RasterizerError(f"radii must be the forward's [P] int32 tensor on {dev} with P = {P}, got "
                                  f"{None if radii is None else (tuple(radii.shape), radii.dtype, radii.device)}")
        for name, b in (("geomBuffer", geomBuffer), ("binningBuffer", binningBuffer), ("imageBuffer", imageBuffer)):
            if b.dtype != torch.uint8 or (b.numel() != 0 and b.device != dev):
                raise RasterizerError(f"{name} must be the forward's uint8 buffer on {dev}")
        if geomBuffer.numel() == 0 or imageBuffer.numel() == 0:
            raise RasterizerError("geomBuffer / imageBuffer are empty: pass the buffers the forward returned")
        need = int(lib().omr_image_bytes(W, H))
        if imageBuffer.numel() != need:
            raise RasterizerError(f"dL_dout_color is [3, {H}, {W}] but imageBuffer ({imageBuffer.numel()} bytes) was "
                                  f"sized by the forward for a different view ({need} bytes for this one)")
        if int(R) > 0 and binningBuffer.numel() < int(lib().omr_binning_bytes(int(R), W, H)):
            raise RasterizerError(f"binningBuffer ({binningBuffer.numel()} bytes) is too small for R = {R} instances "
                                  f"of a {W} x {H} view")
    shapes = dict(dL_dmeans2D=(P, 3), dL_dcolors=(P, 3), dL_dopacity=(P, 1), dL_dmeans3D=(P, 3), dL_dcov3D=(P, 6),
                  dL_dsh=(P, M, 3), dL_dscales=(P, 3), dL_drotations=(P, 4))
    o = {}
    for k, shp in shapes.items():
        if k == "dL_dsh" and skip_dsh:
            o[k] = None
            continue
        t = None if out is None else out.get(k)
        if t is None:
            t = (torch.zeros if P == 0 else torch.empty)(shp, dtype=torch.float32, device=dev)
        elif tuple(t.shape) != shp or not t.is_contiguous() or t.dtype != torch.float32:
            raise RasterizerError(f"out[{k}] must be a contiguous float32 tensor of shape {shp}")
        o[k] = t
    if P != 0:
        L = lib()
        args_common = dict(bg=_dev_f32(background, "background", dev, 3), m=_dev_f32(means3D, "means3D"),
                           shc=_dev_f32(sh, "sh", dev), col=_dev_f32(colors, "colors", dev, 3 * P),
                           sc=_dev_f32(scales, "scales", dev, 3 * P), rot=_dev_f32(rotations, "rotations", dev, 4 * P),
                           cov=_dev_f32(cov3D_precomp, "cov3D_precomp", dev, 6 * P),
                           vm=_dev_f32(viewmatrix, "viewmatrix", dev, 16), cp=_dev_f32(campos, "campos", dev, 3),
                           dl=_dev_f32(dL_dout_color, "dL_dout_color", dev))
        a = args_common
        rad = radii.contiguous()
        gb, bb, ib = geomBuffer.data_ptr(), binningBuffer.data_ptr() if binningBuffer.numel() else None, imageBuffer.data_ptr()
        if colors_event is not None:
            if colors_event.cuda_event == 0:  # torch creates the HIP event at its first record
                colors_event.record(torch.cuda.current_stream(dev))
            L.omr_backward_colors_event(C.c_void_p(colors_event.cuda_event))
        if chunk_events:
            for ev in chunk_events:
                if ev.cuda_event == 0:
                    ev.record(torch.cuda.current_stream(dev))
            arr = (C.c_void_p * len(chunk_events))(*[ev.cuda_event for ev in chunk_events])
            L.omr_backward_chunk_events(len(chunk_events), arr)
        if camera_type == CAMERA_PINHOLE:
            pm = _dev_f32(projmatrix, "projmatrix", dev, 16)
            rc = L.omr_rasterizer_backward(P, int(degree), M, int(R), _ptr(a["bg"]), W, H, _ptr(a["m"]), _ptr(a["shc"]),
                                           _ptr(a["col"]), _ptr(a["sc"]), float(scale_modifier), _ptr(a["rot"]),
                                           _ptr(a["cov"]), _ptr(a["vm"]), _ptr(pm), _ptr(a["cp"]), float(tan_fovx),
                                           float(tan_fovy), rad.data_ptr(), gb, bb, ib, _ptr(a["dl"]),
                                           o["dL_dmeans2D"].data_ptr(), None, o["dL_dopacity"].data_ptr(),
                                           o["dL_dcolors"].data_ptr(), o["dL_dmeans3D"].data_ptr(),
                                           o["dL_dcov3D"].data_ptr(), _ptr(o["dL_dsh"]), o["dL_dscales"].data_ptr(),
                                           o["dL_drotations"].data_ptr(), _stream(dev))
        else:
            rc = L.omr_lonlat_backward(P, int(degree), M, int(R), _ptr(a["bg"]), W, H, _ptr(a["m"]), _ptr(a["shc"]),
                                       _ptr(a["col"]), _ptr(a["sc"]), float(scale_modifier), _ptr(a["rot"]),
                                       _ptr(a["cov"]), _ptr(a["vm"]), _ptr(a["cp"]), rad.data_ptr(), gb, bb, ib,
                                       _ptr(a["dl"]), o["dL_dmeans2D"].data_ptr(), None, o["dL_dopacity"].data_ptr(),
                                       o["dL_dcolors"].data_ptr(), o["dL_dmeans3D"].data_ptr(),
                                       o["dL_dcov3D"].data_ptr(), _ptr(o["dL_dsh"]), o["dL_dscales"].data_ptr(),
                                       o["dL_drotations"].data_ptr(), None, None, _stream(dev))
        _check(rc, "RasterizeGaussiansBackwardCUDA")
    return (o["dL_dmeans2D"], o["dL_dcolors"], o["dL_dopacity"], o["dL_dmeans3D"], o["dL_dcov3D"], o["dL_dsh"],
            o["dL_dscales"], o["dL_drotations"])


def sh_grad_from_colors(means3D, sh, degree, campos_all, dcolors_all, out=None):
    """Extension for view-parallel DP (parallel.allreduce_compact_): the sum over n views of dL/dsh, rebuilt from
    each view's dL_dcolors ([n,P,3], the backward's second output) and camera position ([n,3]) with the backward's
    own SH arithmetic (omr_sh_grad_from_colors). Returns dL_dsh [P,M,3] (written into `out` if given)."""
    m, shc = _dev_f32(means3D, "means3D"), _dev_f32(sh, "sh")
    cp, dc = _dev_f32(campos_all, "campos_all"), _dev_f32(dcolors_all, "dcolors_all")
    P, M = int(m.shape[0]), int(shc.shape[1])
    n = int(cp.shape[0])
    if tuple(dc.shape) != (n, P, 3) or tuple(cp.shape) != (n, 3):
        raise RasterizerError("dcolors_all must be [n,P,3] and campos_all [n,3]")
    if out is None:
        out = torch.empty((P, M, 3), dtype=torch.float32, device=m.device)
    elif tuple(out.shape) != (P, M, 3) or not out.is_contiguous() or out.dtype != torch.float32:
        raise RasterizerError(f"out must be a contiguous float32 tensor of shape {(P, M, 3)}")
    rc = lib().omr_sh_grad_from_colors(P, int(degree), M, n, _ptr(m), _ptr(shc), _ptr(cp), _ptr(dc), out.data_ptr(),
                                       _stream(m.device))
    _check(rc, "sh_grad_from_colors")
    return out


def sh_grad_from_colors_packed(means3D, sh, degree, packed, out=None):
    """sh_grad_from_colors with both inputs in one [n, P+1, 3] tensor: rows 0..P-1 of view v are its dL_dcolors, row
    P its camera position (what parallel.allreduce_compact_ gathers with one collective)."""
    m, shc, pk = _dev_f32(means3D, "means3D"), _dev_f32(sh, "sh"), _dev_f32(packed, "packed")
    P, M = int(m.shape[0]), int(shc.shape[1])
    if pk.dim() != 3 or tuple(pk.shape[1:]) != (P + 1, 3):
        raise RasterizerError("packed must be [n, P+1, 3]")
    n = int(pk.shape[0])
    if out is None:
        out = torch.empty((P, M, 3), dtype=torch.float32, device=m.device)
    elif tuple(out.shape) != (P, M, 3) or not out.is_contiguous() or out.dtype != torch.float32:
        raise RasterizerError(f"out must be a contiguous float32 tensor of shape {(P, M, 3)}")
    rc = lib().omr_sh_grad_from_colors_packed(P, int(degree), M, n, _ptr(m), _ptr(shc), _ptr(pk), out.data_ptr(),
                                              _stream(m.device))
    _check(rc, "sh_grad_from_colors_packed")
    return out


def markVisible(means3D, viewmatrix, projmatrix, camera_type=CAMERA_PINHOLE):
    """rasterize_points.cu:287-319: bool [P]; pinhole = view-space z > 0.2, lonlat = all True."""
    dev = means3D.device
    P = int(means3D.shape[0])
    present = torch.zeros((P,), dtype=torch.bool, device=dev)
    if P == 0:
        return present
    if camera_type == CAMERA_PINHOLE:
        m, vm, pm = _dev_f32(means3D, "means3D"), _dev_f32(viewmatrix, "viewmatrix"), _dev_f32(projmatrix, "projmatrix")
        rc = lib().omr_rasterizer_mark_visible(P, _ptr(m), _ptr(vm), _ptr(pm), present.data_ptr(), _stream(dev))
    elif camera_type == CAMERA_LONLAT:
        rc = lib().omr_lonlat_mark_visible(P, present.data_ptr(), _stream(dev))
    else:
        raise RasterizerError("[CudaRasterizer]Invalid camera_type")
    _check(rc, "markVisible")
    return present


# --------------------------------------------------------------------------------------------------------------
# Autograd glue: include/gaussian_rasterizer.h:32-141, src/gaussian_rasterizer.cpp:24-223
# --------------------------------------------------------------------------------------------------------------
@dataclass
class GaussianRasterizationSettings:
    image_height: int
    image_width: int
    tanfovx: float
    tanfovy: float
    bg: torch.Tensor
    scale_modifier: float
    viewmatrix: torch.Tensor
    projmatrix: torch.Tensor
    RwcT: Optional[torch.Tensor]
    sh_degree: int
    campos: torch.Tensor
    prefiltered: bool
    camera_type: int = CAMERA_PINHOLE
    render_depth: bool = False


class GaussianRasterizerFunction(torch.autograd.Function):
    """gaussian_rasterizer.cpp:35-171."""

    @staticmethod
    def forward(ctx, means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp, settings):
        s = settings
        num_rendered, color, radii, geomBuffer, binningBuffer, imgBuffer = RasterizeGaussiansCUDA(
            s.bg, means3D, colors_precomp, opacities, scales, rotations, s.scale_modifier, cov3Ds_precomp,
            s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, s.image_height, s.image_width, sh, s.sh_degree,
            s.campos, s.prefiltered, int(s.camera_type), s.render_depth)
        ctx.settings = s
        ctx.num_rendered = num_rendered
        ctx.save_for_backward(colors_precomp, means3D, scales, rotations, cov3Ds_precomp, radii, sh, geomBuffer,
                              binningBuffer, imgBuffer)
        ctx.mark_non_differentiable(radii)
        return color, radii

    @staticmethod
    def backward(ctx, grad_out_color, grad_radii):
        s = ctx.settings
        colors_precomp, means3D, scales, rotations, cov3Ds_precomp, radii, sh, geomBuffer, binningBuffer, imgBuffer = \
            ctx.saved_tensors
        g = RasterizeGaussiansBackwardCUDA(s.bg, means3D, radii, colors_precomp, scales, rotations, s.scale_modifier,
                                           cov3Ds_precomp, s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy,
                                           grad_out_color.contiguous(), sh, s.sh_degree, s.campos, geomBuffer,
                                           ctx.num_rendered, binningBuffer, imgBuffer, int(s.camera_type))
        dmeans2D, dcolors, dopacity, dmeans3D, dcov3D, dsh, dscales, drot = g
        # gaussian_rasterizer.cpp:159-169: (means3D, means2D, sh, colors, opacity, scales, rotations, cov3D, settings)
        return (dmeans3D, dmeans2D, dsh, dcolors, dopacity, dscales, drot, dcov3D, None)


def rasterize_gaussians(means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp, settings):
    """gaussian_rasterizer.h:87-106."""
    return GaussianRasterizerFunction.apply(means3D, means2D, sh, colors_precomp, opacities, scales, rotations,
                                            cov3Ds_precomp, settings)


class GaussianRasterizer(torch.nn.Module):
    """gaussian_rasterizer.h:108-141 / gaussian_rasterizer.cpp:24-32, :173-223."""

    def __init__(self, raster_settings: GaussianRasterizationSettings):
        super().__init__()
        self.raster_settings = raster_settings

    def markVisibleGaussians(self, positions):
        with torch.no_grad():
            s = self.raster_settings
            return markVisible(positions, s.viewmatrix, s.projmatrix)  # pinhole test, as the reference

    def forward(self, means3D, means2D, opacities, shs=None, colors_precomp=None, scales=None, rotations=None,
                cov3D_precomp=None):
        has_shs, has_col = shs is not None, colors_precomp is not None
        has_s, has_r, has_cov = scales is not None, rotations is not None, cov3D_precomp is not None
        if (not has_shs and not has_col) or (has_shs and has_col):
            raise RasterizerError("Please provide excatly one of either SHs or precomputed colors!")
        if ((not has_s or not has_r) and not has_cov) or ((has_s or has_r) and has_cov):
            raise RasterizerError("Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!")
        dev = means3D.device
        empty = lambda: torch.empty(0, dtype=torch.float32, device=dev)
        color, radii = rasterize_gaussians(means3D, means2D, shs if has_shs else empty(),
                                           colors_precomp if has_col else empty(), opacities,
                                           scales if has_s else empty(), rotations if has_r else empty(),
                                           cov3D_precomp if has_cov else empty(), self.raster_settings)
        return color, radii


# --------------------------------------------------------------------------------------------------------------
# Introspection (tests): intermediate state of a forward, read back from the private scratch layout
# --------------------------------------------------------------------------------------------------------------
def debug_state(P, R, width, height, geomBuffer, binningBuffer, imgBuffer):
    dev = geomBuffer.device
    gx, gy = (width + 15) // 16, (height + 15) // 16
    N = width * height
    out = dict(
        means2D=torch.empty((P, 2), dtype=torch.float32, device=dev),
        conic_opacity=torch.empty((P, 4), dtype=torch.float32, device=dev),
        rgb=torch.empty((P, 3), dtype=torch.float32, device=dev),
        depths=torch.empty((P,), dtype=torch.float32, device=dev),
        tiles_touched=torch.empty((P,), dtype=torch.int32, device=dev),
        point_list=torch.empty((max(R, 0),), dtype=torch.int32, device=dev),
        ranges=torch.empty((gx * gy, 2), dtype=torch.int32, device=dev),
        final_T=torch.empty((N,), dtype=torch.float32, device=dev),
        n_contrib=torch.empty((N,), dtype=torch.int32, device=dev),
    )
    L, st = lib(), _stream(dev)
    if P > 0:
        _check(L.omr_debug_geometry(geomBuffer.data_ptr(), P, out["means2D"].data_ptr(),
                                    out["conic_opacity"].data_ptr(), out["rgb"].data_ptr(), out["depths"].data_ptr(),
                                    out["tiles_touched"].data_ptr(), st), "debug_geometry")
        if R > 0:
            _check(L.omr_debug_point_list(binningBuffer.data_ptr(), R, width, height, out["point_list"].data_ptr(), st),
                   "debug_point_list")
        _check(L.omr_debug_ranges(imgBuffer.data_ptr(), width, height, out["ranges"].data_ptr(), st), "debug_ranges")
        _check(L.omr_debug_image_state(imgBuffer.data_ptr(), width, height, out["final_T"].data_ptr(),
                                       out["n_contrib"].data_ptr(), st), "debug_image_state")
    return out


def debug_point_masks(R, width, height, binningBuffer) -> torch.Tensor:
    """Each point-list entry's band mask (top 4 bits: the tile's 16x4 bands the instance can reach), int32 [R]."""
    out = torch.empty((max(R, 0),), dtype=torch.int32, device=binningBuffer.device)
    if R > 0:
        _check(lib().omr_debug_point_list_raw(binningBuffer.data_ptr(), R, width, height, out.data_ptr(),
                                              _stream(binningBuffer.device)), "debug_point_list_raw")
    return (out >> 28) & 15


def debug_tile_cost(width, height, imgBuffer) -> torch.Tensor:
    """The forward's per-tile count of (instance, 16x4 band) evaluations, int32 [T] (render_fwd.hip: `work`)."""
    T = ((width + 15) // 16) * ((height + 15) // 16)
    out = torch.empty((T,), dtype=torch.int32, device=imgBuffer.device)
    _check(lib().omr_debug_tile_cost(imgBuffer.data_ptr(), width, height, out.data_ptr(), _stream(imgBuffer.device)),
           "debug_tile_cost")
    return out


def debug_counters(P, geomBuffer) -> dict:
    """The forward's count words (omr_debug_counters): num_rendered, the row binning's row slots M, ..."""
    out = torch.zeros((8,), dtype=torch.int32, device=geomBuffer.device)
    _check(lib().omr_debug_counters(geomBuffer.data_ptr(), int(P), out.data_ptr(), _stream(geomBuffer.device)),
           "debug_counters")
    c = [int(v) & 0xFFFFFFFF for v in out.cpu().tolist()]
    return {"num_rendered": c[0], "prefiltered_flag": c[1], "huge": c[2], "error": c[3], "row_slots": c[4],
            "sh_jac": c[5] != 0, "sh_jac_key": c[5]}


def debug_depth_sort_mode(mode: int) -> int:
    """The forward's depth sort, process-wide (omr_debug_depth_sort_mode): 0 by size and camera type, 1 the plain
    4 x 8-bit radix sort, 2 the sort that sets culled Gaussians aside first, 3 the sort by counting (views of at most
    2^18 Gaussians; the default up to 12288). Returns the previous mode."""
    rc = int(lib().omr_debug_depth_sort_mode(int(mode)))
    if rc < 0:
        raise RasterizerError(f"debug_depth_sort_mode({mode}): {lib().omr_last_error().decode()}")
    return rc


def debug_binning_mode(mode: int) -> int:
    """The forward's binning, process-wide (omr_debug_binning_mode): 0 by view, 1 the row binning wherever the grid
    allows it, 2 the emit + radix tile sort. A forward and its backward must run under the same mode. Returns the
    previous mode."""
    rc = int(lib().omr_debug_binning_mode(int(mode)))
    if rc < 0:
        raise RasterizerError(f"debug_binning_mode({mode}): {lib().omr_last_error().decode()}")
    return rc


def debug_ssim_mode(mode: int) -> int:
    """The fused loss's kernel, process-wide (omr_debug_ssim_mode): 0 by image size, 1 tiled, 2 streaming. Returns the
    previous mode."""
    rc = int(lib().omr_debug_ssim_mode(int(mode)))
    if rc < 0:
        raise RasterizerError(f"debug_ssim_mode({mode}): {lib().omr_last_error().decode()}")
    return rc


def debug_bwd_bands(mode: int) -> int:
    """The render backward's mapping, process-wide (omr_debug_bwd_bands): 0 by view (two waves of two bands per unit
    when every unit is resident at once), 2 or 4 forced. Returns the previous mode."""
    rc = int(lib().omr_debug_bwd_bands(int(mode)))
    if rc < 0:
        raise RasterizerError(f"debug_bwd_bands({mode}): {lib().omr_last_error().decode()}")
    return rc


def debug_adam_sh_rows(enabled: int) -> int:
    """Adam's f_dc + f_rest row walk, process-wide (omr_debug_adam_sh_rows): 1 on (default), 0 the two gathering
    groups (the activated SH output then comes from a separate copy launch). Returns the previous value."""
    rc = int(lib().omr_debug_adam_sh_rows(int(enabled)))
    if rc < 0:
        raise RasterizerError(f"debug_adam_sh_rows({enabled}): {lib().omr_last_error().decode()}")
    return rc


def debug_set_sh_jac(P, geomBuffer, enabled: bool):
    """Clears or restores the key by which the backward takes the forward's stored dRGB/ddir (omr_debug_set_sh_jac)."""
    _check(lib().omr_debug_set_sh_jac(geomBuffer.data_ptr(), int(P), 1 if enabled else 0, _stream(geomBuffer.device)),
           "debug_set_sh_jac")


# --------------------------------------------------------------------------------------------------------------
# Stage timing: HIP events recorded by the library on the launch stream (omr_profile_*)
# --------------------------------------------------------------------------------------------------------------
NUM_STAGES = 10


def profile_enable(on: bool = True, stages=None):
    """Record per-stage HIP events; `stages` (names) limits recording to those stages (None = all)."""
    mask = 0xFFFFFFFF
    if stages is not None:
        names = [lib().omr_profile_stage_name(i).decode() for i in range(NUM_STAGES)]
        mask = sum(1 << names.index(s) for s in stages)
    lib().omr_profile_set_mask(mask)
    lib().omr_profile_enable(1 if on else 0)


def profile_set_on(on: bool):
    """Turn the stage profiler on or off, keeping the stage mask (one cheap call per step)."""
    lib().omr_profile_enable(1 if on else 0)


def profile_reset():
    lib().omr_profile_reset()


def profile_read() -> dict:
    """{stage_name: (total_ms, launches)} accumulated since the last reset (waits for the recorded events)."""
    tot = (C.c_double * NUM_STAGES)()
    cnt = (C.c_uint64 * NUM_STAGES)()
    n = lib().omr_profile_read(tot, cnt, NUM_STAGES)
    return {lib().omr_profile_stage_name(i).decode(): (float(tot[i]), int(cnt[i])) for i in range(n)}


NUM_RUNTIME_STATS = 9


def runtime_stats() -> dict:
    """Host-side counters of the library since load or the last reset (omr_runtime_stats): forwards, backwards,
    first-call syncs, capacity-hint back-half re-runs, host wait (ns) for num_rendered and for the backward's error
    word, allocation callbacks and bytes, look-back give-ups."""
    buf = (C.c_uint64 * NUM_RUNTIME_STATS)()
    n = lib().omr_runtime_stats(buf, NUM_RUNTIME_STATS)
    return {lib().omr_runtime_stat_name(i).decode(): int(buf[i]) for i in range(n)}


def runtime_stats_reset():
    lib().omr_runtime_stats_reset()


def forward_status(geomBuffer: torch.Tensor, P: int) -> None:
    """For forward-only callers: raises RasterizerError if the forward's device-side binning (emit, tile sort) failed
    after RasterizeGaussiansCUDA returned (a decoupled look-back gave up: the view rendered background only). A
    backward on the same buffers reports the same failure itself. Synchronises the current stream."""
    _check(lib().omr_forward_status(geomBuffer.data_ptr(), int(P), _stream(geomBuffer.device)), "forward_status")


def loaded_library() -> str:
    """Absolute path of the HIP library this process loaded (OMR_LIB_PATH or the in-tree build)."""
    lib()
    return os.path.realpath(LIB_PATH)


def debug_wave_sum(x: torch.Tensor, lds: bool = False) -> torch.Tensor:
    """Column sums of a [64, 9] float32 device tensor through a wave reduction of wave_ops.h: the cross-row-first
    wave_sum9_rows (default; the row sums') or wave_sum9_lds (lds=True, the render backward's unpaired one)."""
    x = _dev_f32(x, "x")
    assert tuple(x.shape) == (64, 9)
    out = torch.empty(9, dtype=torch.float32, device=x.device)
    fn = lib().omr_debug_wave_sum9_lds if lds else lib().omr_debug_wave_sum9
    _check(fn(x.data_ptr(), out.data_ptr(), _stream(x.device)), "debug_wave_sum")
    return out


def debug_wave_scans(x: torch.Tensor) -> torch.Tensor:
    """The DPP wave scans of raster_common.h on a [2, 64] int32 device tensor (u32 bits): returns [3, 64] = the
    inclusive sum of x[0], the inclusive max of x[1], and the wave max of x[1] on every lane."""
    if not x.is_cuda or x.dtype != torch.int32 or tuple(x.shape) != (2, 64):
        raise ValueError("x must be a [2, 64] int32 tensor on the HIP device")
    x = x.contiguous()
    out = torch.empty((3, 64), dtype=torch.int32, device=x.device)
    _check(lib().omr_debug_wave_scans(x.data_ptr(), out.data_ptr(), _stream(x.device)), "debug_wave_scans")
    return out


def debug_wave_sum_pair(x: torch.Tensor) -> torch.Tensor:
    """Column sums of two [64, 9] float32 blocks (x: [2, 64, 9] on the device) through wave_sum9x2_stored, the
    render backward's paired reduction: returns [2, 9]."""
    x = _dev_f32(x, "x")
    assert tuple(x.shape) == (2, 64, 9)
    out = torch.empty((2, 9), dtype=torch.float32, device=x.device)
    _check(lib().omr_debug_wave_sum9x2(x.data_ptr(), out.data_ptr(), _stream(x.device)), "debug_wave_sum_pair")
    return out

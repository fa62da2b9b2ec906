"""C-ABI library checks that need no GPU: the library loads, exports every entry point include/omnigs_raster.h
declares, and the host-side logic (argument validation, scratch sizing, P = 0 early return) behaves."""
import ctypes as C
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "omnigs_raster.h")


def _declared():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(omr_[a-z0-9_]+)\s*\(", text)) - {"omr_alloc_fn"})


def test_header_declares_reference_entry_points():
    names = _declared()
    for n in ["omr_rasterizer_mark_visible", "omr_rasterizer_forward", "omr_rasterizer_backward",
              "omr_lonlat_mark_visible", "omr_lonlat_forward", "omr_lonlat_backward"]:
        assert n in names


def test_library_exports_every_declared_symbol(omr):
    lib = omr.rasterizer.lib()
    out = subprocess.run(["nm", "-D", "--defined-only", omr.rasterizer.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r" T (omr_\w+)", out))
    for n in _declared():
        assert n in exported, n
        assert getattr(lib, n) is not None


def test_abi_version_and_sizes(omr):
    lib = omr.rasterizer.lib()
    assert lib.omr_abi_version() == 1
    g0, g1 = lib.omr_geometry_bytes(1000), lib.omr_geometry_bytes(2000)
    assert g1 > g0 > 1000 * 93  # 64-B render record + clamped, tiles_touched, sort keys/values, offsets, radii
    assert lib.omr_image_bytes(64, 32) >= 64 * 32 * 8 + 8 * 8
    b0, b1 = lib.omr_binning_bytes(0, 64, 32), lib.omr_binning_bytes(1000, 64, 32)
    assert b1 - b0 >= 1000 * (16 + 36)  # keys/values ping-pong + one gradient row per instance


def test_invalid_camera_type_and_empty_scene_without_gpu(omr):
    lib = omr.rasterizer.lib()
    nr = C.c_int(-1)
    alloc = omr.rasterizer._ALLOC_FN(lambda ctx, n: None)
    # P = 0 returns before touching the device (rasterize_points.cu:97)
    rc = lib.omr_lonlat_forward(alloc, None, alloc, None, alloc, None, 0, 3, 16, None, 64, 32, None, None, None, None,
                                None, 1.0, None, None, None, None, False, None, None, None, C.byref(nr))
    assert rc == 0 and nr.value == 0
    # missing inputs are rejected by the host validation, before any allocation or launch
    rc = lib.omr_lonlat_forward(alloc, None, alloc, None, alloc, None, 10, 3, 16, None, 64, 32, None, None, None, None,
                                None, 1.0, None, None, None, None, False, None, None, None, C.byref(nr))
    assert rc == 1
    assert b"missing" in lib.omr_last_error()
    rc = lib.omr_lonlat_backward(10, 3, 16, 0, None, 64, 32, None, None, None, None, 1.0, None, None, None, None,
                                 None, None, None, None, None, None, None, None, None, None, None, None, None, None,
                                 None, None, None)
    assert rc == 1


def test_python_boundary_rejects_cpu_tensors(omr):
    import torch

    R = omr.rasterizer
    t = torch.zeros(4, 3)
    with pytest.raises(R.RasterizerError, match="HIP device"):
        R.RasterizeGaussiansCUDA(torch.zeros(3), t, torch.empty(0), torch.ones(4, 1), torch.ones(4, 3),
                                 torch.ones(4, 4), 1.0, torch.empty(0), torch.eye(4), torch.eye(4), 0.0, 0.0, 32, 64,
                                 torch.zeros(4, 16, 3), 3, torch.zeros(3), False, 3)
    with pytest.raises(R.RasterizerError, match="num_points, 3"):
        R.RasterizeGaussiansCUDA(torch.zeros(3), torch.zeros(4, 2), None, None, None, None, 1.0, None, None, None,
                                 0.0, 0.0, 32, 64, None, 3, None, False, 3)
    with pytest.raises(R.RasterizerError, match="Invalid camera_type"):
        R.RasterizeGaussiansCUDA(torch.zeros(3), t, None, None, None, None, 1.0, None, None, None, 0.0, 0.0, 32, 64,
                                 None, 3, None, False, 2)


def test_autograd_wrapper_argument_rules(omr):
    import torch

    R = omr.rasterizer
    s = R.GaussianRasterizationSettings(32, 64, 0.0, 0.0, torch.zeros(3), 1.0, torch.eye(4), torch.eye(4), None, 3,
                                        torch.zeros(3), False, R.CAMERA_LONLAT)
    rast = R.GaussianRasterizer(s)
    m = torch.zeros(4, 3)
    with pytest.raises(R.RasterizerError, match="excatly one of either SHs"):
        rast(m, m, torch.ones(4, 1), scales=torch.ones(4, 3), rotations=torch.ones(4, 4))
    with pytest.raises(R.RasterizerError, match="scale/rotation pair"):
        rast(m, m, torch.ones(4, 1), shs=torch.zeros(4, 16, 3), scales=torch.ones(4, 3))


def test_libtorch_dropin_exports_reference_symbols(omr):
    """librasterize_points.so exports the reference's three C++ functions with identical signatures
    (include/rasterize_points.h:29-80 of the reference), so a LibTorch host links it unchanged."""
    path = os.path.join(os.path.dirname(omr.rasterizer.LIB_PATH), "librasterize_points.so")
    out = subprocess.run(["nm", "-DC", "--defined-only", path], capture_output=True, text=True, check=True).stdout
    T, F = "at::Tensor const&", "float"
    expect = [
        f"RasterizeGaussiansCUDA({T}, {T}, {T}, {T}, {T}, {T}, {F}, {T}, {T}, {T}, {F}, {F}, int, int, {T}, int, {T}, "
        "bool, int, bool)",
        f"RasterizeGaussiansBackwardCUDA({T}, {T}, {T}, {T}, {T}, {T}, {F}, {T}, {T}, {T}, {F}, {F}, {T}, {T}, int, "
        f"{T}, {T}, int, {T}, {T}, int)",
        "markVisible(at::Tensor&, at::Tensor&, at::Tensor&, int)",
    ]
    for sig in expect:
        assert sig in out, sig
    m = omr.rasterizer.libtorch_boundary()
    assert hasattr(m, "RasterizeGaussiansCUDA") and hasattr(m, "markVisible")


def test_runtime_stats_without_gpu(omr):
    """omr_runtime_stats: the host-side counters bench.py reports (first-call syncs, back-half re-runs, host waits,
    allocation callbacks, look-back give-ups) are named, start at zero after a reset, and count the host-validated
    calls that never reach the device."""
    R = omr.rasterizer
    R.runtime_stats_reset()
    st = R.runtime_stats()
    assert list(st) == ["forwards", "backwards", "first_call_syncs", "back_half_reruns", "count_wait_ns",
                        "backward_wait_ns", "alloc_calls", "alloc_bytes", "lookback_errors"]
    assert all(v == 0 for v in st.values())
    assert R.loaded_library().endswith("libomnigs_raster.so")


def test_scratch_buffers_free_without_cyclic_gc(omr):
    """The allocation callbacks' byte buffers must not sit in a reference cycle: otherwise each step's scratch
    tensors (0.7 GB at config C, 7.6 GB at E) outlive the step until Python's cyclic GC runs, and the caching
    allocator has to hipMalloc fresh blocks every step (bench.py reports device_mallocs in the timed region)."""
    import gc
    import weakref

    import torch

    gc.disable()
    try:
        b = omr.rasterizer._ByteBuffer(torch.device("cpu"))
        ref = weakref.ref(b)
        assert b.fn(None, 64)
        t = b.tensor
        assert t.numel() == 64
        del b
        assert ref() is None
    finally:
        gc.enable()


def test_kernel_switches_without_gpu(omr):
    """omr_debug_depth_sort_mode / omr_debug_ssim_mode / omr_debug_binning_mode (process-wide switches between
    kernels that give the same results): each returns the previous mode, rejects a mode outside its range (0..3,
    0..2, 0..2) with -1 and a message, and is restored."""
    R = omr.rasterizer
    for setter, top in ((R.debug_depth_sort_mode, 3), (R.debug_ssim_mode, 2), (R.debug_binning_mode, 2)):
        old = setter(2)
        try:
            assert setter(1) == 2
            assert setter(top) == 1
            assert setter(0) == top
            with pytest.raises(R.RasterizerError, match="mode"):
                setter(top + 1)
            assert setter(0) == 0  # the bad call changed nothing
        finally:
            setter(old)

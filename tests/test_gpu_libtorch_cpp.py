"""The reference host's LibTorch caller, in C++, over the drop-in.

tests/cpp/reference_host_caller.cpp restates /root/reference/src/gaussian_rasterizer.cpp:35-224 on
include/rasterize_points.h: a torch::autograd::Function that saves geomBuffer / binningBuffer / imgBuffer and R
(num_rendered) in its forward (:78-98), restores them in its backward (:109-131) and maps the drop-in's 8 gradients
onto its 9 inputs (:159-169). It links lib/librasterize_points.so and LibTorch only, runs forward, loss =
sum(color * dL), loss.backward() through LibTorch's engine, and writes the results as raw files. Here they are
compared bitwise with the ctypes path (same deterministic kernels underneath) and against the oracle's bars.
"""
import os
import subprocess

import numpy as np
import pytest

from helpers import grad_close, hip_run, make_case, oracle_run, scene, to_np

pytestmark = pytest.mark.gpu

EXE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cpp", "build", "reference_host_caller")


def _write_case(d, g, cam, dL):
    os.makedirs(d, exist_ok=True)
    arrays = {"means3D": g.means3D, "shs": g.shs, "opacity": g.opacity, "scales": g.scales, "rotations": g.rotations,
              "viewmatrix": cam.viewmatrix, "projmatrix": cam.projmatrix, "campos": cam.campos,
              "bg": np.zeros(3), "dL_dcolor": dL}
    for k, a in arrays.items():
        np.ascontiguousarray(a, dtype=np.float32).tofile(os.path.join(d, k + ".f32"))
    with open(os.path.join(d, "params.txt"), "w") as f:
        f.write(f"P {g.P}\nW {cam.width}\nH {cam.height}\nsh_degree {g.sh_degree}\nM {g.shs.shape[1]}\n"
                f"tanfovx {cam.tanfovx!r}\ntanfovy {cam.tanfovy!r}\ncamera_type {cam.camera_type}\n")


def _read(d, name, shape, dtype=np.float32):
    ext = ".i32" if dtype == np.int32 else ".f32"
    return np.fromfile(os.path.join(d, name + ext), dtype=dtype).reshape(shape)


@pytest.mark.parametrize("cam_type,P,W,H", [(scene.CAMERA_LONLAT, 1500, 128, 64),
                                            (scene.CAMERA_PINHOLE, 1500, 160, 90),
                                            (scene.CAMERA_LONLAT, 100_000, 1024, 512)])
def test_cpp_autograd_function_over_dropin(tmp_path, cam_type, P, W, H, omr):
    assert os.path.exists(EXE), f"{EXE} missing: run __graft_entry__.build()"
    g, cam, dL = make_case(P, W, H, cam_type, 77, view_index=2, spread=3.0 if P < 10_000 else None)
    case, out = str(tmp_path / "case"), str(tmp_path / "out")
    _write_case(case, g, cam, dL)
    os.makedirs(out)
    r = subprocess.run([EXE, case, out], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert '"refused": 2' in r.stdout, r.stdout  # both exactly-one-of checks throw (gaussian_rasterizer.cpp:190-196)

    color = _read(out, "color", (3, H, W))
    radii = _read(out, "radii", (g.P,), np.int32)
    got = {"dmean3D": _read(out, "dmean3D", (g.P, 3)), "dmean2D": _read(out, "dmean2D", (g.P, 3)),
           "dsh": _read(out, "dsh", g.shs.shape), "dopacity": _read(out, "dopacity", (g.P, 1)),
           "dscale": _read(out, "dscale", (g.P, 3)), "drot": _read(out, "drot", (g.P, 4))}

    # bitwise against the ctypes boundary: same kernels, fixed-order sums
    h = hip_run(g, cam, dL)
    np.testing.assert_array_equal(color, to_np(h["color"]))
    np.testing.assert_array_equal(radii, to_np(h["radii"]))
    for name, a in got.items():
        np.testing.assert_array_equal(a.reshape(-1), to_np(h["grads"][name]).reshape(-1), err_msg=name)

    # the oracle's bars
    o, L, og = oracle_run(g, cam, dL, nthreads=8)
    np.testing.assert_array_equal(radii, o.get("radii"))
    assert np.abs(color - o.get("out_color").reshape(3, H, W)).max() <= 1e-4
    for name in ("dmean3D", "dsh", "dopacity", "dscale", "drot"):
        ok, emax, nbad = grad_close(got[name].reshape(og[name].shape), og[name])
        assert ok, (name, emax, nbad)

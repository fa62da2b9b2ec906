"""Caller mistakes at the two host boundaries (the LibTorch drop-in, include/rasterize_points.h, and the Python host on
the C ABI) are reported as RuntimeError before any kernel sees a pointer, and the process stays healthy: the next
good call gives the same result as before. The reference checks means3D's shape only (rasterize_points.cu:72-75);
the kernels take raw device pointers, so a host tensor, a tensor on another device, a short tensor or a gradient
image of another view would otherwise be a memory fault, not an error."""
import numpy as np
import pytest
import torch

from helpers import make_case, scene

pytestmark = pytest.mark.gpu


def _inputs(cam_type):
    W, H = (128, 64) if cam_type == scene.CAMERA_LONLAT else (160, 90)
    g, cam, dL = make_case(800, W, H, cam_type, 77, spread=3.0)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).cuda()  # noqa: E731
    d = dict(bg=torch.zeros(3, device="cuda"), means=t(g.means3D), op=t(g.opacity), sc=t(g.scales),
             rot=t(g.rotations), vm=t(cam.viewmatrix), pm=t(cam.projmatrix), sh=t(g.shs), cp=t(cam.campos), dL=t(dL),
             e=torch.empty(0, device="cuda"))
    return g, cam, d


def _fwd(api, g, cam, d, cam_type, **over):
    x = dict(d)
    x.update(over)
    return api.RasterizeGaussiansCUDA(x["bg"], x["means"], x["e"], x["op"], x["sc"], x["rot"], 1.0, x["e"], x["vm"],
                                      x["pm"], cam.tanfovx, cam.tanfovy, cam.height, cam.width, x["sh"], g.sh_degree,
                                      x["cp"], False, cam_type, False)


def _bwd(api, g, cam, d, cam_type, fwd, **over):
    nr, _, radii, gb, bb, ib = fwd
    x = dict(d, radii=radii, nr=nr, gb=gb, bb=bb, ib=ib)
    x.update(over)
    return api.RasterizeGaussiansBackwardCUDA(x["bg"], x["means"], x["radii"], x["e"], x["sc"], x["rot"], 1.0, x["e"],
                                              x["vm"], x["pm"], cam.tanfovx, cam.tanfovy, x["dL"], x["sh"],
                                              g.sh_degree, x["cp"], x["gb"], x["nr"], x["bb"], x["ib"], cam_type)


@pytest.mark.parametrize("boundary", ["libtorch", "ctypes"])
@pytest.mark.parametrize("cam_type", [scene.CAMERA_LONLAT, scene.CAMERA_PINHOLE])
def test_bad_inputs_raise_and_the_process_stays_healthy(boundary, cam_type, omr):
    api = omr.rasterizer.libtorch_boundary() if boundary == "libtorch" else omr.rasterizer
    g, cam, d = _inputs(cam_type)
    good = _fwd(api, g, cam, d, cam_type)
    good_grads = _bwd(api, g, cam, d, cam_type, good)
    torch.cuda.synchronize()
    P = g.P

    # forward: a host tensor, a short tensor, a mis-shaped SH array
    with pytest.raises(RuntimeError, match="sh"):
        _fwd(api, g, cam, d, cam_type, sh=d["sh"].cpu())
    with pytest.raises(RuntimeError, match="opacity"):
        _fwd(api, g, cam, d, cam_type, op=d["op"][: P // 2])
    with pytest.raises(RuntimeError, match="sh"):
        _fwd(api, g, cam, d, cam_type, sh=d["sh"].reshape(P, 48)[:, :45].reshape(P, 15, 3)[: P - 1])
    with pytest.raises(RuntimeError, match="rotations"):
        _fwd(api, g, cam, d, cam_type, rot=d["rot"][:, :3].contiguous())
    with pytest.raises(RuntimeError, match="viewmatrix"):
        _fwd(api, g, cam, d, cam_type, vm=d["vm"].cpu())

    # backward: a CPU SH array, a gradient image of another shape, int64 radii, radii of another length,
    # empty scratch buffers, a too-large R
    with pytest.raises(RuntimeError, match="sh"):
        _bwd(api, g, cam, d, cam_type, good, sh=d["sh"].cpu())
    with pytest.raises(RuntimeError, match="dL_dout_color"):
        _bwd(api, g, cam, d, cam_type, good, dL=d["dL"][:, :-16, :].contiguous())
    with pytest.raises(RuntimeError, match="dL_dout_color"):
        _bwd(api, g, cam, d, cam_type, good, dL=d["dL"][:2].contiguous())
    with pytest.raises(RuntimeError, match="dL_dout_color"):
        _bwd(api, g, cam, d, cam_type, good, dL=d["dL"].cpu())
    with pytest.raises(RuntimeError, match="radii"):
        _bwd(api, g, cam, d, cam_type, good, radii=good[2].to(torch.int64))
    with pytest.raises(RuntimeError, match="radii"):
        _bwd(api, g, cam, d, cam_type, good, radii=good[2][:-1])
    with pytest.raises(RuntimeError, match="empty"):
        _bwd(api, g, cam, d, cam_type, good, gb=torch.empty(0, dtype=torch.uint8, device="cuda"))
    with pytest.raises(RuntimeError, match="binningBuffer"):
        _bwd(api, g, cam, d, cam_type, good, nr=good[0] * 4 + 100000)
    with pytest.raises(RuntimeError):
        _bwd(api, g, cam, d, cam_type, good, nr=-1)

    # the next good calls reproduce the first ones bit for bit
    again = _fwd(api, g, cam, d, cam_type)
    again_grads = _bwd(api, g, cam, d, cam_type, again)
    torch.cuda.synchronize()
    assert again[0] == good[0]
    assert torch.equal(again[1], good[1]) and torch.equal(again[2], good[2])
    for a, b in zip(again_grads, good_grads):
        assert torch.equal(a, b)

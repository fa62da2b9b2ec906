"""Oracle (line-by-line restatement of the reference) vs an independent PyTorch-autograd model (torch_model.py)
on small scenes, in float64: forward image and the gradients of sum(dL * image) w.r.t. every input."""
import numpy as np
import pytest
import torch

import oracle as O
import torch_model as TM
from helpers import scene
from test_oracle_fd import _scene


@pytest.mark.parametrize("cam_type,deg,seed", [(scene.CAMERA_LONLAT, 3, 1), (scene.CAMERA_LONLAT, 2, 2),
                                               (scene.CAMERA_PINHOLE, 3, 3), (scene.CAMERA_PINHOLE, 1, 4)])
def test_oracle_matches_torch_autograd(cam_type, deg, seed, oracle_mod):
    W, H = (64, 32) if cam_type == scene.CAMERA_LONLAT else (48, 36)
    g, cam, dL = _scene(24, W, H, cam_type, 300 + seed, deg, view=seed % 8 if cam_type == scene.CAMERA_LONLAT else 0)
    bg = np.array([0.1, 0.2, 0.3])
    o = O.Oracle(double=True)
    o.forward(background=bg, means3D=g.means3D, opacity=g.opacity, scales=g.scales, rotations=g.rotations,
              shs=g.shs, viewmatrix=cam.viewmatrix.astype(np.float64), projmatrix=cam.projmatrix.astype(np.float64),
              campos=cam.campos.astype(np.float64), width=W, height=H, sh_degree=deg, tanfovx=cam.tanfovx,
              tanfovy=cam.tanfovy, camera_type=cam_type)
    grads = o.backward(dL)
    img_o = o.get("out_color").reshape(3, H, W)

    tt = lambda a: torch.tensor(np.asarray(a, np.float64), requires_grad=True)
    m, s, q, op, sh = tt(g.means3D), tt(g.scales), tt(g.rotations), tt(g.opacity), tt(g.shs)
    img_t = TM.render(m, s, q, op, sh, torch.tensor(cam.viewmatrix, dtype=torch.float64),
                      torch.tensor(cam.projmatrix, dtype=torch.float64), torch.tensor(cam.campos, dtype=torch.float64),
                      W, H, deg, cam_type, torch.tensor(bg), cam.tanfovx, cam.tanfovy)
    # the reference writes its guards as float literals (0.3f, 1e-7f, 0.2f) that the double oracle keeps
    np.testing.assert_allclose(img_t.detach().numpy(), img_o, rtol=0, atol=1e-7)
    (img_t * torch.tensor(dL)).sum().backward()
    pairs = [("dmean3D", m), ("dscale", s), ("drot", q), ("dopacity", op), ("dsh", sh)]
    for name, t in pairs:
        ref = t.grad.numpy()
        got = grads[name].reshape(ref.shape)
        np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-7 * max(1.0, np.abs(ref).max()), err_msg=name)

"""Fused L1 + SSIM loss (csrc/ssim.hip) against the reference formula (include/loss_utils.h:31-129,
gaussian_trainer.cpp:88-90; restated in oracle/loss_oracle.py) evaluated by torch autograd in float64 on the CPU: loss value and d loss / d image,
on image sizes that are not multiples of the 16x16 tile or of the 54-column strip (border handling of the zero
padding), through both kernels (tiled; streaming, the one the training step's image sizes take), which must give
bitwise the same gradient."""
import numpy as np
import pytest
import torch

from helpers import grad_close, omr, to_np

pytestmark = pytest.mark.gpu


def _reference(img, gt, lam):
    import loss_oracle as L  # oracle/: the reference formula in torch (test infrastructure)

    x = img.detach().double().cpu().requires_grad_(True)
    y = gt.detach().double().cpu()
    loss = (1.0 - lam) * L.l1_loss(x, y) + lam * (1.0 - L.ssim(x, y))
    loss.backward()
    return float(loss.detach()), to_np(x.grad), float(L.l1_loss(x, y).detach()), float(L.ssim(x, y).detach())


@pytest.fixture(params=["tiled", "stream"])
def ssim_kernel(request):
    old = omr.rasterizer.debug_ssim_mode(1 if request.param == "tiled" else 2)
    yield request.param
    omr.rasterizer.debug_ssim_mode(old)


@pytest.mark.parametrize("C,H,W,lam,seed", [(3, 64, 96, 0.2, 0), (3, 130, 70, 0.2, 1), (1, 33, 17, 0.5, 2),
                                            (3, 16, 16, 1.0, 3), (2, 75, 131, 0.2, 4)])
def test_fused_l1_ssim_matches_reference(C, H, W, lam, seed, ssim_kernel):
    g = torch.Generator().manual_seed(seed)
    gt = torch.rand((C, H, W), generator=g)
    img = (gt + 0.1 * torch.randn((C, H, W), generator=g)).clamp(0, 1)
    img_d = img.cuda().requires_grad_(True)
    loss, terms = omr.losses.l1_ssim_loss(img_d, gt.cuda(), lam)
    loss.backward()
    ref_loss, ref_grad, ref_l1, ref_ssim = _reference(img, gt, lam)
    t = to_np(terms)
    assert abs(float(loss.detach()) - ref_loss) < 1e-5, (float(loss.detach()), ref_loss)
    assert abs(t[1] - ref_l1) < 1e-6 and abs(t[2] - ref_ssim) < 1e-5, (t, ref_l1, ref_ssim)
    ok, emax, nbad = grad_close(to_np(img_d.grad), ref_grad, rtol=1e-3, atol_frac=1e-4)
    assert ok, (emax, nbad)


def test_fused_loss_is_deterministic():
    g = torch.Generator().manual_seed(5)
    gt = torch.rand((3, 200, 300), generator=g).cuda()
    img = torch.rand((3, 200, 300), generator=g).cuda()
    runs = []
    for _ in range(2):
        x = img.clone().requires_grad_(True)
        loss, _ = omr.losses.l1_ssim_loss(x, gt, 0.2)
        loss.backward()
        runs.append((float(loss.detach()), to_np(x.grad)))
    assert runs[0][0] == runs[1][0]
    np.testing.assert_array_equal(runs[0][1], runs[1][1])


@pytest.mark.parametrize("C,H,W", [(3, 200, 300), (1, 97, 163), (3, 1024, 2048)])
def test_tiled_and_streaming_kernels_agree_bitwise(C, H, W):
    """The same dL/dimg bits from both kernels (same tap order, fused multiply-adds, ssim_partials); the loss terms
    differ only in their block partial sums' grouping."""
    g = torch.Generator().manual_seed(11)
    gt = torch.rand((C, H, W), generator=g).cuda()
    img = (gt.cpu() + 0.05 * torch.randn((C, H, W), generator=g)).clamp(0, 1).cuda()
    R = omr.rasterizer
    res = {}
    old = R.debug_ssim_mode(1)
    try:
        for mode in (1, 2):
            R.debug_ssim_mode(mode)
            terms, grad = omr.losses.l1_ssim_loss_and_grad(img, gt, 0.2)
            res[mode] = (to_np(terms), to_np(grad))
    finally:
        R.debug_ssim_mode(old)
    np.testing.assert_array_equal(res[1][1], res[2][1])
    np.testing.assert_allclose(res[1][0], res[2][0], rtol=1e-6, atol=1e-7)

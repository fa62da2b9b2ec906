"""Independent PyTorch (float64, CPU, autograd) model of the reference rasterizer's forward semantics.

Written from the math, not from the glm code: standard EWA covariance J Rcw Sigma Rcw^T J^T with J the
Jacobian of the lonlat (or pinhole) projection, Sigma = R S^2 R^T, SH colours, per-tile membership from the
reference's getRect, front-to-back blending with the reference's skip rules (power > 0, alpha < 1/255,
T < 1e-4 stop). Gradients come from torch.autograd. TEST INFRASTRUCTURE: cross-checks the oracle (which
transcribes the reference line by line) against an independent formulation of the same semantics.
"""
from __future__ import annotations

import math

import torch

SH_C0 = 0.28209479177387814
SH_C1 = 0.4886025119029199
SH_C2 = [1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792, 0.5462742152960396]
SH_C3 = [-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154, -0.4570457994644658,
         1.445305721320277, -0.5900435899266435]


def quat_to_rot(q):
    r, x, y, z = q.unbind(-1)
    return torch.stack([
        torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y)], -1),
        torch.stack([2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x)], -1),
        torch.stack([2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)], -1)], -2)


def sh_color(shs, dirs, deg):
    x, y, z = dirs.unbind(-1)
    res = SH_C0 * shs[:, 0]
    if deg > 0:
        res = res - SH_C1 * y[:, None] * shs[:, 1] + SH_C1 * z[:, None] * shs[:, 2] - SH_C1 * x[:, None] * shs[:, 3]
    if deg > 1:
        xx, yy, zz, xy, yz, xz = x * x, y * y, z * z, x * y, y * z, x * z
        terms = [xy, yz, 2 * zz - xx - yy, xz, xx - yy]
        for k in range(5):
            res = res + SH_C2[k] * terms[k][:, None] * shs[:, 4 + k]
    if deg > 2:
        terms = [y * (3 * xx - yy), xy * z, y * (4 * zz - xx - yy), z * (2 * zz - 3 * xx - 3 * yy),
                 x * (4 * zz - xx - yy), z * (xx - yy), x * (xx - 3 * yy)]
        for k in range(7):
            res = res + SH_C3[k] * terms[k][:, None] * shs[:, 9 + k]
    return torch.clamp_min(res + 0.5, 0.0)


def render(means3D, scales, rotations, opacity, shs, view, proj, campos, W, H, deg, camera_type, bg,
           tanfovx=0.0, tanfovy=0.0):
    """Returns the [3,H,W] image. `view`/`proj` are the reference's tensors (Tcw^T, (P Tcw)^T)."""
    Tcw = view.T
    Rcw, tcw = Tcw[:3, :3], Tcw[:3, 3]
    t = means3D @ Rcw.T + tcw
    tx, ty, tz = t.unbind(-1)
    if camera_type == 3:
        rr = (t * t).sum(-1)
        keep = rr > 0.04
        r = torch.sqrt(rr)
        lon = torch.atan2(tx, tz)
        lat = torch.asin(ty / (r + 1e-7))
        px = ((lon / math.pi + 1) * W - 1) * 0.5
        py = ((lat * 2 / math.pi + 1) * H - 1) * 0.5
        rho2 = tx * tx + tz * tz
        rho = torch.sqrt(rho2)
        a, b = W / (2 * math.pi), H / math.pi
        J = torch.zeros(len(t), 2, 3, dtype=t.dtype)
        J[:, 0, 0] = a * tz / (rho2 + 1e-7)
        J[:, 0, 2] = -a * tx / (rho2 + 1e-7)
        J[:, 1, 0] = -b * tx * ty / ((rho + 1e-7) * (rho2 + ty * ty + 1e-7))
        J[:, 1, 1] = b * rho / (rho2 + ty * ty + 1e-7)
        J[:, 1, 2] = -b * tz * ty / ((rho + 1e-7) * (rho2 + ty * ty + 1e-7))
        depth = r
    else:
        keep = tz > 0.2
        ph = torch.cat([means3D, torch.ones_like(means3D[:, :1])], 1) @ proj
        pw = 1.0 / (ph[:, 3] + 1e-7)
        px = ((ph[:, 0] * pw + 1) * W - 1) * 0.5
        py = ((ph[:, 1] * pw + 1) * H - 1) * 0.5
        fx, fy = W / (2 * tanfovx), H / (2 * tanfovy)
        limx, limy = 1.3 * tanfovx, 1.3 * tanfovy
        txc = torch.clamp(tx / tz, -limx, limx) * tz
        tyc = torch.clamp(ty / tz, -limy, limy) * tz
        J = torch.zeros(len(t), 2, 3, dtype=t.dtype)
        J[:, 0, 0] = fx / tz
        J[:, 0, 2] = -fx * txc / (tz * tz)
        J[:, 1, 1] = fy / tz
        J[:, 1, 2] = -fy * tyc / (tz * tz)
        depth = tz
    R = quat_to_rot(rotations)
    S2 = torch.diag_embed(scales * scales)
    Sigma = R @ S2 @ R.transpose(-1, -2)
    JW = J @ Rcw
    cov = JW @ Sigma @ JW.transpose(-1, -2) + 0.3 * torch.eye(2, dtype=t.dtype)
    det = cov[:, 0, 0] * cov[:, 1, 1] - cov[:, 0, 1] ** 2
    conic = torch.stack([cov[:, 1, 1] / det, -cov[:, 0, 1] / det, cov[:, 0, 0] / det], -1)
    with torch.no_grad():
        mid = 0.5 * (cov[:, 0, 0] + cov[:, 1, 1])
        lam = mid + torch.sqrt(torch.clamp_min(mid * mid - det, 0.1))
        radius = torch.ceil(3 * torch.sqrt(lam)).to(torch.int64)
        gx, gy = (W + 15) // 16, (H + 15) // 16
        x0 = torch.clamp(torch.trunc((px - radius) / 16), 0, gx).to(torch.int64)
        y0 = torch.clamp(torch.trunc((py - radius) / 16), 0, gy).to(torch.int64)
        x1 = torch.clamp(torch.trunc((px + radius + 15) / 16), 0, gx).to(torch.int64)
        y1 = torch.clamp(torch.trunc((py + radius + 15) / 16), 0, gy).to(torch.int64)
        vis = keep & (det != 0) & ((x1 - x0) * (y1 - y0) > 0)
        order = sorted([i for i in range(len(t)) if vis[i]], key=lambda i: (float(depth[i].float()), i))
    dirs = means3D - campos
    dirs = dirs / dirs.norm(dim=-1, keepdim=True)
    col = sh_color(shs, dirs, deg)
    ys, xs = torch.meshgrid(torch.arange(H, dtype=t.dtype), torch.arange(W, dtype=t.dtype), indexing="ij")
    tile_x, tile_y = (xs // 16).to(torch.int64), (ys // 16).to(torch.int64)
    T = torch.ones(H, W, dtype=t.dtype)
    C = torch.zeros(3, H, W, dtype=t.dtype)
    done = torch.zeros(H, W, dtype=torch.bool)
    for i in order:
        inrect = (tile_x >= x0[i]) & (tile_x < x1[i]) & (tile_y >= y0[i]) & (tile_y < y1[i])
        dx, dy = px[i] - xs, py[i] - ys
        power = -0.5 * (conic[i, 0] * dx * dx + conic[i, 2] * dy * dy) - conic[i, 1] * dx * dy
        alpha = torch.clamp_max(opacity[i, 0] * torch.exp(power), 0.99)
        ok = inrect & ~done & (power <= 0) & (alpha >= 1 / 255)
        test_T = T * (1 - alpha)
        stop = ok & (test_T < 1e-4)
        done = done | stop
        ok = ok & ~stop
        C = C + torch.where(ok, alpha * T, torch.zeros_like(T))[None] * col[i][:, None, None]
        T = torch.where(ok, test_T, T)
    return C + T[None] * bg[:, None, None]

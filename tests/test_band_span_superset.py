"""The emit kernel's per-band span test (raster_common.h: band_mask_span) must keep every band the per-row test
(band_mask_of) keeps: a band mask may only be conservative, since a dropped band would drop pixels from the render.
Both are restated here in float32 on random anisotropic Gaussians and tiles around them (host-side property check of
the math; the GPU parity tests check the kernels' images and gradients)."""
import numpy as np

f32 = np.float32


def _consts(a, b, c, o):
    t = f32(2) * f32(np.log(f32(255) * o)) * f32(1.002) + f32(0.02)
    ra = f32(1) / a
    return t, -b * ra, (a * c - b * b) * ra, a


def _row_mask(t, k, dd, a, x, y, tx, ty):
    x0 = f32(tx * 16)
    lo, hi, dy0 = x - (x0 + f32(15)), x - x0, y - f32(ty * 16)
    m = 0
    for bb in range(4):
        for r in range(4):
            dy = dy0 - f32(4 * bb + r)
            kdy = k * dy
            e = np.clip(kdy, lo, hi) - kdy
            if a * e * e + dd * dy * dy <= t:
                m |= 1 << bb
                break
    return m


def _span_mask(t, k, dd, a, x, y, tx, ty):
    A = a * k * k + dd
    kdt, ak, adt, at, inv_a = k * np.sqrt(t / dd), a * k, a * dd, A * t, f32(1) / A
    x0 = f32(tx * 16)
    lo, hi = x - (x0 + f32(15)), x - x0
    lt, lb = np.clip(kdt, lo, hi), np.clip(-kdt, lo, hi)
    dt, db = at - adt * lt * lt, at - adt * lb * lb
    if not dt >= 0:
        return 0
    y2 = (ak * lt + np.sqrt(dt)) * inv_a
    y1 = (ak * lb - np.sqrt(max(db, f32(0)))) * inv_a
    y2 += f32(0.02) + f32(2e-6) * abs(y2)
    y1 -= f32(0.02) + f32(2e-6) * abs(y1)
    dy0 = y - f32(ty * 16)
    return sum(1 << b for b in range(4) if dy0 - f32(4 * b + 3) <= y2 and dy0 - f32(4 * b) >= y1)


def test_span_mask_keeps_every_band_the_row_test_keeps():
    rng = np.random.default_rng(7)
    n = extra = 0
    with np.errstate(all="ignore"):
        for _ in range(3000):
            s = 10 ** rng.uniform(-0.5, 2.5)
            sx, sy, th = s * 10 ** rng.uniform(-1, 1), s, rng.uniform(0, np.pi)
            R = np.array([[np.cos(th), -np.sin(th)], [np.sin(th), np.cos(th)]])
            Ci = np.linalg.inv(R @ np.diag([sx * sx + 0.3, sy * sy + 0.3]) @ R.T)
            a, b, c = f32(Ci[0, 0]), f32(Ci[0, 1]), f32(Ci[1, 1])
            o = f32(rng.uniform(0.004, 1.0))
            x, y = f32(rng.uniform(0, 4096)), f32(rng.uniform(0, 2048))
            t, k, dd, a = _consts(a, b, c, o)
            r = 3 * np.sqrt(max(sx, sy) ** 2 + 0.3)
            for _ in range(4):
                tx = int(np.clip((x + rng.uniform(-r, r)) // 16, 0, 255))
                ty = int(np.clip((y + rng.uniform(-r, r)) // 16, 0, 127))
                m_row, m_span = _row_mask(t, k, dd, a, x, y, tx, ty), _span_mask(t, k, dd, a, x, y, tx, ty)
                assert m_row & ~m_span == 0, (a, b, c, o, x, y, tx, ty, m_row, m_span)
                n += 1
                extra += bin(m_span & ~m_row).count("1")
    assert extra <= 0.01 * n  # barely looser than the row test: the render kernels do no noticeable extra work

"""Synthetic stereo pairs ("Synthetic generator").

The reference ships no data (``.gitignore:2-3`` ignores ``data/``), so every benchmark and
most parity cases use Gaussian-smoothed uniform texture with a known horizontal shift.
Pure numpy (separable Gaussian, sigma=1.0, truncate=4.0 like scipy's default) so the
generator runs identically here and on the GPU box.
"""

import numpy as np


def _gauss_kernel(sigma=1.0, truncate=4.0):
    r = int(truncate * sigma + 0.5)
    x = np.arange(-r, r + 1, dtype=np.float64)
    k = np.exp(-0.5 * (x / sigma) ** 2)
    return k / k.sum()


def _smooth(a, sigma=1.0):
    k = _gauss_kernel(sigma)
    r = len(k) // 2
    out = a.astype(np.float64)
    for axis in (0, 1):
        pad = [(0, 0), (0, 0)]
        pad[axis] = (r, r)
        p = np.pad(out, pad, mode='reflect')
        acc = np.zeros_like(out)
        for t in range(len(k)):
            sl = [slice(None), slice(None)]
            sl[axis] = slice(t, t + out.shape[axis])
            acc += k[t] * p[tuple(sl)]
        out = acc
    return out


def texture(h, w, seed, sigma=1.0):
    """uint8 texture of shape (h, w): uniform noise, smoothed, stretched to [0, 255]."""
    rng = np.random.default_rng(seed)
    raw = rng.integers(0, 256, size=(h, w)).astype(np.float64)
    s = _smooth(raw, sigma)
    lo, hi = s.min(), s.max()
    return np.rint((s - lo) * (255.0 / (hi - lo))).astype(np.uint8)


def stereo_pair(h, w, seed=0, dx=2, max_disp=None, sinusoidal=False):
    """Return (img1, img2), uint8 (h, w): img2 is img1's texture shifted by dx columns.

    With ``sinusoidal=True`` the shift varies smoothly in [0, max_disp] across the image
    (the "realism" runs of SURVEY.md section 8d)."""
    if max_disp is None:
        max_disp = max(dx, 8)
    tex = texture(h + 8, w + 8 + max_disp, seed)
    img1 = tex[4:4 + h, 4:4 + w].copy()
    if not sinusoidal:
        img2 = tex[4:4 + h, 4 + dx:4 + dx + w].copy()
    else:
        yy, xx = np.mgrid[0:h, 0:w]
        d = np.rint(0.5 * max_disp * (1.0 + np.sin(2 * np.pi * xx / max(w, 1)) *
                                      np.cos(2 * np.pi * yy / max(h, 1)))).astype(np.int64)
        img2 = tex[4 + yy, 4 + xx + d].astype(np.uint8)
    return img1, img2

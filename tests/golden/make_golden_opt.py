"""Golden fixtures of the Gauss-Seidel post-processing loops, made by the REFERENCE code.

Run in the build container only (``/root/reference`` does not exist on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_opt.py

``misc/optimize_loop.py`` and ``misc/opt_loop.py`` import nothing but numpy, so they are
imported unchanged from ``/root/reference`` and run as they are: ``optimize_loop`` (with its
``image_threshold`` and the backward sweep's row alternation), ``make_weight`` (numpy's
``np.exp``), ``optimize_loop_bilateral_horizon`` / ``_vertical`` (numpy's pairwise sums).
Only inputs and outputs are written (tests/golden/opt_*.npz), never reference source.
"""

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get('DM_REFERENCE', '/root/reference')
sys.path.insert(0, REF)
sys.dont_write_bytecode = True

from misc.optimize_loop import optimize_loop  # noqa: E402
from misc.opt_loop import (make_weight, optimize_loop_bilateral_horizon,  # noqa: E402
                           optimize_loop_bilateral_vertical)


def smooth_map(rng, h, w, lo=-1.0, hi=11.0):
    """A disparity-like float64 map: smooth ramp + noise spanning [lo, hi]."""
    y, x = np.mgrid[0:h, 0:w]
    m = 5.0 + 4.0 * np.sin(x / 5.0) * np.cos(y / 7.0) + rng.normal(0, 1.0, (h, w))
    return np.clip(m, lo, hi)


def opt_case(name, h, w, e, size, seed, alpha=0.008, nan=False):
    rng = np.random.default_rng(seed)
    img = rng.uniform(-2.0, 12.0, (h, w))
    if nan:
        img[h // 2, w // 3] = np.nan
    coef = rng.uniform(0.0, 2.0, (h, w))
    out, err = optimize_loop(img.copy(), coef, alpha, e, list(size))
    np.savez_compressed(os.path.join(HERE, 'opt_%s.npz' % name), img=img, coef=coef,
                        alpha=np.float64(alpha), exclusion=np.int64(e), size=np.array(size),
                        out=out, error=np.float64(err))
    print(name, out.shape, float(err))


def bilat_case(name, h, w, e, size, seed, sigma, coef_shape=None):
    rng = np.random.default_rng(seed)
    guide = smooth_map(rng, h, w)
    img = guide + rng.normal(0, 0.3, (h, w))
    coef = rng.uniform(0.2, 1.5, coef_shape or (h, w))
    gw, cwm = make_weight(guide, e, list(size), sigma)
    rec = {'guide': guide, 'img': img, 'coef': coef, 'exclusion': np.int64(e), 'size': np.array(size),
           'sigma': np.asarray(sigma), 'sigma_int': np.int64(np.asarray(sigma).dtype.kind == 'i'),
           'gauss': gw, 'color': cwm}
    a = img.copy()
    out_h, err_h = optimize_loop_bilateral_horizon(a, cwm, gw, coef, 0.008, e, list(size))
    rec['out_h'], rec['error_h'] = out_h.copy(), np.float64(err_h)
    b = img.copy()
    out_v, err_v = optimize_loop_bilateral_vertical(b, cwm, gw, coef, 0.008, e, list(size))
    rec['out_v'], rec['error_v'] = out_v.copy(), np.float64(err_v)
    np.savez_compressed(os.path.join(HERE, 'opt_%s.npz' % name), **rec)
    print(name, cwm.shape, float(err_h), float(err_v))


def main():
    opt_case('loop_24x31_e1', 24, 31, 1, (24, 31), seed=1)
    opt_case('loop_20x22_e3_sub', 20, 22, 3, (18, 17), seed=2)
    opt_case('loop_13x15_e0', 13, 15, 0, (12, 14), seed=3, alpha=0.05)
    opt_case('loop_17x16_e2_nan', 17, 16, 2, (17, 16), seed=4, nan=True)
    opt_case('loop_5x9_e2_empty', 5, 9, 2, (5, 9), seed=5)
    bilat_case('bilat_26x29_e1', 26, 29, 1, (26, 29), seed=11, sigma=np.array([5, 5]))
    bilat_case('bilat_24x27_e2_float', 24, 27, 2, (22, 27), seed=12, sigma=[2.5, 3.0])
    bilat_case('bilat_30x28_e3', 30, 28, 3, (30, 28), seed=13, sigma=np.array([5, 5]))
    bilat_case('bilat_22x23_e6', 22, 23, 6, (22, 23), seed=14, sigma=np.array([4, 6]))
    bilat_case('bilat_9x11_e0', 9, 11, 0, (9, 11), seed=15, sigma=np.array([3, 3]), coef_shape=(4, 5))


if __name__ == '__main__':
    main()

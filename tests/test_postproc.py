"""Gauss-Seidel post-processing: misc/optimize_loop.py and
misc/opt_loop.py.

CPU: the oracle against the reference-made goldens (tests/golden/opt_*.npz,
make_golden_opt.py), the pinned exp, and the dependency-level schedules of dm_gs_schedule
(a host-only entry of the HIP library) executed level by level in numpy -- each level's
updates all read the state before any of them writes -- against the sequential loops.
GPU: the mirrors (misc.optimize_loop / misc.opt_loop) through the C ABI against the oracle
and the goldens.

Tolerances: maps, errors and weights are bit-exact against the oracle (same pinned exp);
against the goldens optimize_loop is bit-exact (no transcendental), the bilateral sweeps are
bit-exact on the golden weights, and the weights themselves (numpy's np.exp vs the pinned
dm_exp) agree within TOL_W relative; maps swept with our own weights within TOL_MAP.
"""
import glob
import math
import os
from decimal import Decimal, getcontext

import numpy as np
import pytest

from oracle import oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, 'golden')
TOL_W = 5e-16     # relative, weights: <= 2 ulp between np.exp and dm_exp
TOL_MAP = 1e-12   # absolute, maps swept with dm_exp weights vs np.exp weights
TOL_ERR = 1e-12   # relative, the error sums on those maps


def gold(kind):
    return sorted(glob.glob(os.path.join(GOLD, 'opt_%s_*.npz' % kind)))


def sigma_of(z):
    s = z['sigma']
    return s if int(z['sigma_int']) else [float(v) for v in s]


def same(a, b):
    return np.array_equal(a, b, equal_nan=True)


def same_err(a, b):
    return (np.isnan(a) and np.isnan(b)) or a == b


# ---------------------------------------------------------------------------------------
# oracle vs reference goldens
# ---------------------------------------------------------------------------------------
@pytest.mark.parametrize('path', gold('loop'), ids=os.path.basename)
def test_oracle_optimize_loop_golden(path):
    z = np.load(path)
    out, err = O.optimize_loop(z['img'], z['coef'], float(z['alpha']), int(z['exclusion']), list(z['size']))
    assert same(out, z['out'])
    assert same_err(err, z['error'])


@pytest.mark.parametrize('path', gold('bilat'), ids=os.path.basename)
def test_oracle_bilateral_golden(path):
    z = np.load(path)
    e, size = int(z['exclusion']), list(z['size'])
    g, c = O.make_weight(z['guide'], e, size, sigma_of(z))
    assert g.shape == z['gauss'].shape and c.shape == z['color'].shape
    np.testing.assert_allclose(g, z['gauss'], rtol=TOL_W, atol=0)
    np.testing.assert_allclose(c, z['color'], rtol=TOL_W, atol=0)
    for vert, key in ((False, 'h'), (True, 'v')):
        out, err = O.opt_loop_bilateral(z['img'], z['color'], z['gauss'], z['coef'], e, size, vert)
        assert same(out, z['out_' + key]), key
        assert err == z['error_' + key]
        out2, err2 = O.opt_loop_bilateral(z['img'], c, g, z['coef'], e, size, vert)
        np.testing.assert_allclose(out2, z['out_' + key], rtol=0, atol=TOL_MAP)
        assert abs(err2 - z['error_' + key]) <= TOL_ERR * abs(z['error_' + key])


def test_pinned_exp_accuracy():
    getcontext().prec = 50
    rng = np.random.default_rng(7)
    xs = np.concatenate([rng.uniform(-745.0, 709.7, 3000), -rng.uniform(0, 40, 3000), rng.uniform(-1, 0, 3000)])
    worst = 0.0
    for x in xs:
        v = O.exp(x)
        ex = Decimal(float(x)).exp()
        ulp = math.ulp(float(ex)) if float(ex) > 0 else 5e-324
        worst = max(worst, float(abs(Decimal(v) - ex) / Decimal(ulp)))
        assert abs(v - np.exp(x)) <= 2 * ulp
    assert worst < 0.75
    assert np.isnan(O.exp(float('nan'))) and O.exp(710.0) == math.inf and O.exp(-746.0) == 0.0
    assert O.exp(0.0) == 1.0 and O.exp(-0.0) == 1.0


# ---------------------------------------------------------------------------------------
# schedules (host-only entry of the HIP library; no GPU)
# ---------------------------------------------------------------------------------------
def _cell(kind, s, s0, s1, e):
    nj = s1 - 2 * e - 1
    o, k = divmod(s, nj)
    if kind == 1:  # BWD4: the reference's alternating row
        return ((e + o) if k & 1 else (s0 - 1 - (e + o))), s1 - 1 - (e + k)
    return e + o, e + k


def _upd4(m, coef, alpha, r, c):
    """one update of optimize_loop.py:20-25 on the current state (python floats/np.float64)."""
    sum_d = m[r, c - 1] + m[r, c + 1] + m[r - 1, c] + m[r + 1, c]
    a = coef[r, c]
    return (-a * m[r, c] + alpha * sum_d) / (-a + 4.0 * alpha)


def _updb(m, cwm, gw, a, K, e, r, c):
    """one update of opt_loop.py:25-33."""
    sub = m[r - e:r + e + 1, c - e:c + e + 1]
    cw = cwm[r - e, c - e]
    b = sub[e, e] - K
    return (-a * b + (gw * cw * sub).sum()) / (-a + (gw * cw).sum())


def _run_levels(kind, m, s0, s1, e, fn):
    from deepmatching_stereo_matching_amd import postproc
    order, off = postproc.host_schedule(kind, m.shape[0], m.shape[1], s0, s1, e)
    n = max(0, s0 - 2 * e - 1) * max(0, s1 - 2 * e - 1)
    assert sorted(order.tolist()) == list(range(n))
    for l in range(len(off) - 1):
        cells = [_cell(kind, int(s), s0, s1, e) for s in order[off[l]:off[l + 1]]]
        assert len(set(cells)) == len(cells)
        vals = [fn(m, r, c) for r, c in cells]      # every read before any write of the level
        for (r, c), v in zip(cells, vals):
            m[r, c] = v
    return len(off) - 1


@pytest.mark.parametrize('h,w,s0,s1,e', [(24, 31, 24, 31, 1), (20, 22, 18, 17, 3), (13, 15, 12, 14, 0),
                                         (40, 9, 40, 9, 1), (7, 7, 7, 7, 3)])
def test_schedule_optimize_loop(h, w, s0, s1, e):
    rng = np.random.default_rng(h * 100 + w)
    img = O.image_threshold(rng.uniform(-2, 12, (h, w)))
    coef = rng.uniform(0, 2, (h, w))
    ref, _ = O.optimize_loop(img, coef, 0.008, e, (s0, s1))
    m = img.copy()
    nl_f = _run_levels(0, m, s0, s1, e, lambda mm, r, c: _upd4(mm, coef, 0.008, r, c))
    nl_b = _run_levels(1, m, s0, s1, e, lambda mm, r, c: _upd4(mm, coef, 0.008, r, c))
    assert same(m, ref)
    n = max(0, s0 - 2 * e - 1) * max(0, s1 - 2 * e - 1)
    if n:  # the schedule is parallel: far fewer levels than updates
        assert nl_f <= (s0 - 2 * e - 1) + (s1 - 2 * e - 1) and nl_b < n or n < 4


@pytest.mark.parametrize('path', gold('bilat'), ids=os.path.basename)
def test_schedule_bilateral(path):
    z = np.load(path)
    e, size = int(z['exclusion']), list(z['size'])
    coef = z['coef']
    for vert, key in ((False, 'h'), (True, 'v')):
        c0 = coef[e, e]
        cp, cm = (coef[e + 1, e], coef[e - 1, e]) if vert else (coef[e, e + 1], coef[e, e - 1])
        a = -(c0 - (cp + cm) / 2.0)
        K = (cp - cm) / 2.0 / (-2.0 * c0 + cp + cm)
        m = z['img'].copy()
        _run_levels(2, m, size[0], size[1], e, lambda mm, r, c: _updb(mm, z['color'], z['gauss'], a, K, e, r, c))
        assert same(m, z['out_' + key]), key


def test_schedule_rejects_bad_shapes():
    from deepmatching_stereo_matching_amd import postproc
    with pytest.raises(IndexError):   # the backward sweep reads row s0 - e == h
        postproc.host_schedule(1, 10, 10, 10, 10, 0)
    with pytest.raises(ValueError):
        postproc.host_schedule(0, 10, 10, 12, 10, 1)
    order, off = postproc.host_schedule(2, 5, 5, 5, 5, 2)   # no update: empty schedule
    assert len(order) == 0 and list(off) == [0]


# ---------------------------------------------------------------------------------------
# GPU: the mirrors through the C ABI
# ---------------------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize('path', gold('loop'), ids=os.path.basename)
def test_gpu_optimize_loop_golden(path):
    from deepmatching_stereo_matching_amd.misc.optimize_loop import optimize_loop
    z = np.load(path)
    img = z['img'].copy()
    out, err = optimize_loop(img, z['coef'], float(z['alpha']), int(z['exclusion']), list(z['size']))
    assert same(img, z['img'])          # the reference sweeps a thresholded copy
    assert same(out, z['out'])
    assert same_err(err, z['error'])


@pytest.mark.gpu
@pytest.mark.parametrize('h,w,e,size', [(300, 257, 1, None), (211, 190, 3, (200, 181)), (64, 80, 0, (63, 79))])
def test_gpu_optimize_loop_oracle(h, w, e, size):
    from deepmatching_stereo_matching_amd.misc.optimize_loop import optimize_loop
    rng = np.random.default_rng(h + w + e)
    img = rng.uniform(-2, 12, (h, w))
    img[rng.integers(0, h, 5), rng.integers(0, w, 5)] = np.nan
    coef = rng.uniform(0, 2, (h, w))
    size = size or (h, w)
    ref, rerr = O.optimize_loop(img, coef, 0.008, e, size)
    out, err = optimize_loop(img, coef, 0.008, e, size)
    assert same(out, ref)
    assert same_err(err, rerr)


@pytest.mark.gpu
@pytest.mark.parametrize('path', gold('bilat'), ids=os.path.basename)
def test_gpu_bilateral_golden(path):
    from deepmatching_stereo_matching_amd.misc import opt_loop as M
    z = np.load(path)
    e, size = int(z['exclusion']), list(z['size'])
    g, c = M.make_weight(z['guide'], e, size, sigma_of(z))
    og, oc = O.make_weight(z['guide'], e, size, sigma_of(z))
    assert same(g, og) and same(c, oc)                      # pinned exp: bit-exact vs oracle
    np.testing.assert_allclose(c, z['color'], rtol=TOL_W, atol=0)
    for fn, key in ((M.optimize_loop_bilateral_horizon, 'h'), (M.optimize_loop_bilateral_vertical, 'v')):
        img = z['img'].copy()
        out, err = fn(img, z['color'], z['gauss'], z['coef'], 0.008, e, size)
        assert out is img                                   # in place, as the reference
        assert same(img, z['out_' + key]) and err == z['error_' + key]
        img2 = z['img'].copy()
        out2, err2 = fn(img2, c, g, z['coef'], 0.008, e, size)
        ref2, rerr2 = O.opt_loop_bilateral(z['img'], oc, og, z['coef'], e, size, key == 'v')
        assert same(out2, ref2) and err2 == rerr2


@pytest.mark.gpu
@pytest.mark.parametrize('h,w,e', [(160, 150, 3), (97, 120, 2)])
def test_gpu_bilateral_oracle_torch(h, w, e):
    """device-resident loop (torch tensors in place), several sweeps as optimize_looper does"""
    import torch
    from deepmatching_stereo_matching_amd.misc import opt_loop as M
    rng = np.random.default_rng(h * w)
    y, x = np.mgrid[0:h, 0:w]
    guide = 5 + 4 * np.sin(x / 9.0) * np.cos(y / 11.0) + rng.normal(0, 1, (h, w))
    coef = rng.uniform(0.2, 1.5, (h, w))
    sigma = np.array([5, 5])
    og, oc = O.make_weight(guide, e, (h, w), sigma)
    dev = torch.device('cuda', 0)
    tg = torch.from_numpy(guide).to(dev)
    g, c = M.make_weight(tg, e, (h, w), sigma)
    assert isinstance(c, torch.Tensor) and same(c.cpu().numpy(), oc) and same(g.cpu().numpy(), og)
    ref = guide.copy()
    timg = tg.clone()
    tcoef = torch.from_numpy(coef).to(dev)
    for it in range(3):
        ref, rerr = O.opt_loop_bilateral(ref, oc, og, coef, e, (h, w), it % 2 == 1)
        fn = M.optimize_loop_bilateral_vertical if it % 2 else M.optimize_loop_bilateral_horizon
        out, err = fn(timg, c, g, tcoef, 0.008, e, (h, w))
        assert out is timg
        assert float(err) == rerr
    assert same(timg.cpu().numpy(), ref)


@pytest.mark.gpu
def test_gpu_image_threshold_and_errors():
    from deepmatching_stereo_matching_amd.misc.optimize_loop import image_threshold, optimize_loop
    from deepmatching_stereo_matching_amd.misc.opt_loop import make_weight, optimize_loop_bilateral_horizon
    a = np.array([[-5.0, 0.0, 3.5], [10.0, 11.0, np.nan]])
    assert same(image_threshold(a), O.image_threshold(a))
    assert same(image_threshold(a, threshold=[-3, 3]), O.image_threshold(a, (-3, 3)))
    with pytest.raises(IndexError):     # backward sweep reads row s0 - e == h (python IndexError)
        optimize_loop(np.ones((10, 10)), np.ones((10, 10)), 0.008, 0, (10, 10))
    with pytest.raises(IndexError):     # coefficient too small for the swept cells
        optimize_loop(np.ones((10, 10)), np.ones((4, 4)), 0.008, 1, (10, 10))
    g, c = make_weight(np.ones((8, 8)), 1, (8, 8), [2.0, 2.0])
    with pytest.raises(IndexError):     # coefficient[e, e + 1] out of range
        optimize_loop_bilateral_horizon(np.ones((8, 8)), c, g, np.ones((2, 2)), 0.0, 1, (8, 8))
    out, err = optimize_loop(np.full((5, 9), 20.0), np.ones((5, 9)), 0.008, 2, (5, 9))   # no update
    assert same(out, np.full((5, 9), 10.0)) and err == 0.0


# ---------------------------------------------------------------------------------------
# GPU: the pipelined level walks (k_optimize_loop_pf, k_bilateral_pf; DM_GS_PF=0 selects
# the one-lane-per-update kernels) -- every exclusion they instantiate, levels wider than
# one round of the workgroup, and the fallback (e = 6)
# ---------------------------------------------------------------------------------------
def _bilateral_case(n, e, seed):
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:n, 0:n]
    guide = 5 + 4 * np.sin(x / 13.0) * np.cos(y / 7.0) + rng.normal(0, 0.7, (n, n))
    coef = rng.uniform(0.2, 1.5, (n, n))
    return guide, coef


@pytest.mark.gpu
@pytest.mark.parametrize('n,e', [(40, 1), (61, 2), (300, 1), (150, 3), (90, 4), (700, 4), (70, 5), (50, 6),
                                 (800, 2)])
def test_gpu_bilateral_pipelined(n, e, monkeypatch):
    import torch
    from deepmatching_stereo_matching_amd.misc import opt_loop as M
    guide, coef = _bilateral_case(n, e, n + e)
    og, oc = O.make_weight(guide, e, (n, n), [5, 5])
    dev = torch.device('cuda', 0)
    tc, tg = torch.from_numpy(oc).to(dev), torch.from_numpy(og).to(dev)
    tcoef = torch.from_numpy(coef).to(dev)
    for vert in (False, True):
        ref, rerr = O.opt_loop_bilateral(guide, oc, og, coef, e, (n, n), vert)
        fn = M.optimize_loop_bilateral_vertical if vert else M.optimize_loop_bilateral_horizon
        outs = []
        for pf in ('1', '0'):
            monkeypatch.setenv('DM_GS_PF', pf)
            timg = torch.from_numpy(guide).to(dev)
            _, err = fn(timg, tc, tg, tcoef, 0.008, e, (n, n))
            outs.append((timg.cpu().numpy(), float(err)))
        for out, err in outs:
            assert same(out, ref) and err == rerr, (vert, e)


@pytest.mark.gpu
@pytest.mark.parametrize('h,w,e', [(1100, 1100, 1), (33, 1030, 0), (257, 64, 2)])
def test_gpu_optimize_loop_pipelined(h, w, e, monkeypatch):
    from deepmatching_stereo_matching_amd.misc.optimize_loop import optimize_loop
    rng = np.random.default_rng(h * w + e)
    img = rng.uniform(-2, 12, (h, w))
    coef = rng.uniform(0, 2, (h, w))
    size = (h - 1, w - 1) if e == 0 else (h, w)    # e = 0: the backward sweep reads row s0 - e
    ref, rerr = O.optimize_loop(img, coef, 0.008, e, size)
    for pf in ('1', '0'):
        monkeypatch.setenv('DM_GS_PF', pf)
        out, err = optimize_loop(img, coef, 0.008, e, size)
        assert same(out, ref) and same_err(err, rerr), pf

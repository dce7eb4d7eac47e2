"""The CPU oracle against the reference at full C2/C3 tile size (round-3 goldens).

tests/golden/c3_tile_*.npz and c2_tile_*.npz come from tests/golden/make_golden_r03.py, which
ran the unchanged reference (misc/Correlation_map.py:161-173 -> misc/Matching.py:211-222 ->
misc/Calc_difference.py:26-49) on S=128 / S=64 tiles cut from bench.py's own input pairs,
and on the same pyramids cut to k levels with N_map = 2^(k-1) (the
"4-level" / "3-level" pyramids of BASELINE configs C3 / C2).

Tolerances as tests/test_oracle_golden.py: level 0 (float32) and integer correspondences
bit-exact; float64 levels |d| <= 1e-12 (relative, for checksums); sub-pixel and cal_map
|d| <= 1e-9.  Both rectification pows (libm and the kernels' pinned pow14) must hold them.
"""

import hashlib
import os

import numpy as np
import pytest

from oracle import oracle as O

GOLD = os.path.join(os.path.dirname(__file__), 'golden')
TOL_F64 = 1e-12
TOL_SUBPIX = 1e-9
CASES = [('c2_tile_2_5', 'libm'), ('c2_tile_2_5', 'pinned'),
         ('c3_tile_0_0', 'libm'), ('c3_tile_0_0', 'pinned'), ('c3_tile_5_3', 'pinned')]


def _close(a, b, tol):
    assert a.shape == b.shape
    na, nb = np.isnan(a), np.isnan(b)
    assert np.array_equal(na, nb)
    if (~na).any():
        assert np.max(np.abs(a[~na] - b[~na])) <= tol


def truncations(g):
    return sorted(int(k[len('match_k'):]) for k in g if k.startswith('match_k'))


@pytest.fixture(scope='module', params=CASES, ids=lambda c: '%s-%s' % c)
def case(request):
    name, mode = request.param
    g = dict(np.load(os.path.join(GOLD, name + '.npz')))
    ws = int(g['ws'])
    O.set_pow_mode(mode)
    try:
        lev, it, n_map = O.pyramid_stream(g['img1'], g['img2'], ws)
        res = {'match': O.match_stream(g['img1'], g['img2'], ws, lev, sub_pix=False),
               'match_subpix': O.match_stream(g['img1'], g['img2'], ws, lev, sub_pix=True)}
        for k in truncations(g):
            res['match_k%d' % k] = O.match_stream(g['img1'], g['img2'], ws, lev[:k], sub_pix=False)
            res['match_subpix_k%d' % k] = O.match_stream(g['img1'], g['img2'], ws, lev[:k], sub_pix=True)
    finally:
        O.set_pow_mode('libm')
    return g, lev, it, n_map, res


def test_inventory():
    names = {c[0] for c in CASES}
    for n in names:
        g = np.load(os.path.join(GOLD, n + '.npz'))
        assert truncations(g), n
    assert int(np.load(os.path.join(GOLD, 'c3_tile_0_0.npz'))['img1'].shape[0]) == 132


def test_level0_bit_exact():
    """The whole S=128 level-0 volume (268 M float32 values) against the reference's sha256."""
    for name in ('c3_tile_0_0', 'c2_tile_2_5'):
        g = np.load(os.path.join(GOLD, name + '.npz'))
        l0 = O.corr_l0(g['img1'], g['img2'], int(g['ws']))
        assert hashlib.sha256(l0.tobytes()).hexdigest() == str(g['l0_sha'])
        idx = g['l0_sample_idx']
        assert np.array_equal(l0[idx[:, 0], idx[:, 1]], g['l0_sample'], equal_nan=True)


def test_pyramid(case):
    g, lev, it, n_map, _ = case
    assert it == int(g['iteration']) and n_map == int(g['N_map']) and len(lev) == int(g['nlev'])
    for k in range(1, len(lev)):
        s = float(np.nansum(lev[k]))
        assert abs(s - float(g['level%d_sum' % k])) <= TOL_F64 * max(1.0, abs(s))
        if 'level%d' % k in g:
            _close(lev[k], g['level%d' % k], TOL_F64)


def test_match(case):
    g, _, _, _, res = case
    assert np.array_equal(res['match'][:2], g['match'][:2])
    _close(res['match'][2], g['match'][2], TOL_F64)
    _close(res['match_subpix'], g['match_subpix'], TOL_SUBPIX)
    _close(O.cal_map(res['match_subpix'], 'elevation'), g['calmap_elevation'], TOL_SUBPIX)


def test_k_level_pyramid(case):
    """Matching on co_map_list[:k] with N_map = 2^(k-1), as the reference ran it."""
    g, _, _, _, res = case
    for k in truncations(g):
        m, ms = res['match_k%d' % k], res['match_subpix_k%d' % k]
        assert np.array_equal(m[:2], g['match_k%d' % k][:2])
        _close(m[2], g['match_k%d' % k][2], TOL_F64)
        _close(ms, g['match_subpix_k%d' % k], TOL_SUBPIX)
        _close(O.cal_map(ms, 'elevation'), g['calmap_elevation_k%d' % k], TOL_SUBPIX)

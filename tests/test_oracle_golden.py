"""Pin the CPU oracle (oracle/) against golden vectors produced by the reference itself.

tests/golden/*.npz come from tests/golden/make_golden.py, which runs the unchanged
reference modules (misc/Correlation_map.py, misc/Matching.py, misc/Calc_difference.py,
misc/image_cut_solver.py, misc/sub_pix_cal.py) with the repo's pinned matchTemplate.

Tolerances (stated here, used everywhere):
  * level-0 min-max volume (float32)          bit-exact, NaN positions equal
  * integer correspondences (sub_pix=False)   bit-exact
  * float64 levels / scores                   |d| <= 1e-12  (pow is 1-ulp platform-
                                              dependent even inside the reference)
  * sub-pixel coordinates, cal_map            |d| <= 1e-9   (the quadratic vertex divides
                                              by a curvature that can be ~1e-7)
"""

import glob
import hashlib
import os

import numpy as np
import pytest

from oracle import oracle as O

GOLD = os.path.join(os.path.dirname(__file__), 'golden')
PAIRS = sorted(glob.glob(os.path.join(GOLD, 'pair_*.npz')))
TOL_F64 = 1e-12
TOL_SUBPIX = 1e-9


def _close(a, b, tol):
    assert a.shape == b.shape
    na, nb = np.isnan(a), np.isnan(b)
    assert np.array_equal(na, nb)
    if (~na).any():
        assert np.max(np.abs(a[~na] - b[~na])) <= tol


@pytest.fixture(scope='module', params=['libm', 'pinned'])
def pow_mode(request):
    """Both rectification pows must reproduce the reference: libm (numpy's, here) and the
    build's pinned dm_pow14 that the GPU kernels evaluate."""
    O.set_pow_mode(request.param)
    yield request.param
    O.set_pow_mode('libm')


@pytest.fixture(scope='module', params=PAIRS, ids=lambda p: os.path.basename(p)[:-4])
def case(request, pow_mode):
    g = dict(np.load(request.param))
    l0 = O.corr_l0(g['img1'], g['img2'], int(g['ws']), str(g['feature']))
    levels, it, n_map = O.pyramid(l0)
    return g, l0, levels, it, n_map


def test_golden_inventory():
    assert len(PAIRS) >= 12


def test_l0_bit_exact(case):
    g, l0, *_ = case
    assert hashlib.sha256(l0.tobytes()).hexdigest() == str(g['l0_sha'])
    assert int(np.isnan(l0).sum()) == int(g['l0_nan'])
    if 'l0' in g:
        assert np.array_equal(l0, g['l0'], equal_nan=True)
    else:
        idx = g['l0_sample_idx']
        assert np.array_equal(l0[idx[:, 0], idx[:, 1]], g['l0_sample'], equal_nan=True)


def test_pyramid(case):
    g, l0, levels, it, n_map = case
    assert it == int(g['iteration']) and n_map == int(g['N_map'])
    assert len(levels) == int(g['nlev'])
    for k, lv in enumerate(levels):
        if 'level%d' % k in g:
            _close(lv, g['level%d' % k], TOL_F64)
        if 'level%d_sum' % k in g:
            s = float(np.nansum(lv))
            assert abs(s - float(g['level%d_sum' % k])) <= TOL_F64 * max(1.0, abs(s))


def test_match_indices_bit_exact(case):
    g, l0, levels, *_ = case
    m = O.match(levels, sub_pix=False)
    assert np.array_equal(m[:2], g['match'][:2])
    _close(m[2], g['match'][2], TOL_F64)


def test_match_subpix_and_cal_map(case):
    g, l0, levels, *_ = case
    m = O.match(levels, sub_pix=True)
    _close(m, g['match_subpix'], TOL_SUBPIX)
    for mode in ('elevation', 'elevation2', 'distance'):
        _close(O.cal_map(m, mode), g['calmap_' + mode], TOL_SUBPIX)


def test_match_filtered(case):
    g, l0, levels, *_ = case
    for fm in ('median', 'average'):
        if 'match_filter_' + fm in g:
            m = O.match(levels, sub_pix=True, filtering=True, filtering_mode=fm,
                        filtering_num=3)
            _close(m, g['match_filter_' + fm], TOL_SUBPIX)


CUTS = ['cut_44_s16_st12', 'cut_52x40_s16_pad', 'cut_48_s16_pad']
BAD = sorted(glob.glob(os.path.join(GOLD, 'bad_matching_*.npz')))


def cut_modes(g):
    if 'modes' in g:
        return [str(m) for m in g['modes']]
    return ['elevation', 'elevation2', 'distance'][:g['d_map'].shape[0]]


@pytest.mark.parametrize('name', CUTS)
def test_image_cut_solver(name):
    g = np.load(os.path.join(GOLD, name + '.npz'))
    modes = cut_modes(g)
    pad = name.endswith('_pad')
    d_map, score = O.cut_solve(g['img1'], g['img2'], image_size=list(g['image_size']),
                               stride=list(g['stride']), window_size=int(g['ws']),
                               degree_map_mode=modes, padding=pad)
    assert d_map.shape == g['d_map'].shape
    covered = ~np.isnan(score)
    _close(d_map[:, covered], g['d_map'][:, covered], TOL_SUBPIX)
    _close(score[covered], g['score'][covered], TOL_F64)


def test_sub_pix_cal_py():
    g = np.load(os.path.join(GOLD, 'subpixcal_s32.npz'))
    _close(O.sub_pix_cal(g['arr'], g['co_map'], direction=0), g['out_dir0'], TOL_SUBPIX)
    _close(O.sub_pix_cal(g['arr'], g['co_map'], direction=1, ratio=30.), g['out_dir1'],
           TOL_SUBPIX)


@pytest.mark.parametrize('path', BAD, ids=lambda p: os.path.basename(p)[:-4])
def test_atomic_patch_and_bad_matching(path):
    """_create_atomic_patch (Correlation_map.py:51-67) and bad_matching.py:60-70's row
    argmax on the level-0 volume, against the reference's own outputs (bit-exact)."""
    g = np.load(path)
    ws, feat = int(g['ws']), str(g['feature'])
    ap = O.atomic_patch(g['img1'], ws)
    assert ap.dtype == g['atomic_patch'].dtype and np.array_equal(ap, g['atomic_patch'])
    dis = O.bad_matching(O.corr_l0(g['img1'], g['img2'], ws, feat))
    assert np.array_equal(dis, g['dis'])


def test_padding_grid_counts_unpadded_shape():
    """ImageCutSolver counts tiles on the image shape recorded before _padding
    (image_cut_solver.py:46,62): 48x48, S=16 -> one tile, not the padded 52x52's 2x2."""
    g = np.load(os.path.join(GOLD, 'cut_48_s16_pad.npz'))
    assert g['d_map'].shape[1:] == (16, 16)

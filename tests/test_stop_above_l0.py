"""Matching with an N_map that stops the descent above level 0, with sub-pixel refinement
(VERDICT r3 missing #4).

The reference (misc/Matching.py:85-96, :133-134) descends one level per halving of N_map, so
an N_map smaller than 2^(n-1) leaves the final map at level `bottom` > 0; _sub_pix_cal
(:177-209) then still reads co_map_list[0] at (i, j, row, col) of that coarse map.
tests/golden/stop_above_l0_s{16,32}.npz (tests/golden/make_golden_r04.py) and
stop_above_l0_s64.npz (make_golden_r05.py) hold the reference's own outputs for bottom = 1, 2.  CPU: the oracle (oracle.match_from) against them.  GPU:
the mirror's Matching (engine.match_levels + dm_subpix_map_tiles, level 0 on demand) against them and, bit for bit,
against the oracle on the same levels.

Tolerances as tests/test_oracle_golden.py: integer correspondences exact; scores |d| <= 1e-12;
sub-pixel |d| <= 1e-9 (the reference's numpy pow vs the pinned one)."""
import os

import numpy as np
import pytest

from oracle import oracle as O

GOLD = os.path.join(os.path.dirname(__file__), 'golden')
TOL_F64 = 1e-12
TOL_SUBPIX = 1e-9
NAMES = ['stop_above_l0_s16', 'stop_above_l0_s32', 'stop_above_l0_s64']


def _close(a, b, tol):
    assert a.shape == b.shape
    na, nb = np.isnan(a), np.isnan(b)
    assert np.array_equal(na, nb)
    if (~na).any():
        assert np.max(np.abs(a[~na] - b[~na])) <= tol


def _cases(g):
    for b in (1, 2):
        yield 'match_b%d' % b, b, False, False
        yield 'match_subpix_b%d' % b, b, True, False
        if 'match_subpix_filt_b%d' % b in g:
            yield 'match_subpix_filt_b%d' % b, b, True, True


@pytest.fixture(scope='module', params=NAMES)
def gold(request):
    g = dict(np.load(os.path.join(GOLD, request.param + '.npz')))
    levels, it, n_map = O.pyramid(O.corr_l0(g['img1'], g['img2'], int(g['ws'])))
    assert len(levels) == int(g['nlev']) and n_map == int(g['N_map_full'])
    return g, levels


def test_oracle_matches_reference(gold):
    g, levels = gold
    for key, b, sp, filt in _cases(g):
        assert int(g['N_map_b%d' % b]) == 2 ** (len(levels) - 1 - b)
        m = O.match_from(levels, b, sub_pix=sp, filtering=filt)
        assert np.array_equal(np.floor(m[:2]), np.floor(g[key][:2])), key
        if not sp:
            assert np.array_equal(m[:2], g[key][:2]), key      # integer correspondences
        _close(m[2], g[key][2], TOL_F64)
        _close(m, g[key], TOL_SUBPIX)
    # the refinement is not a no-op on these pairs
    assert not np.array_equal(g['match_subpix_b1'], g['match_b1'])


@pytest.mark.gpu
def test_mirror_matches_reference_and_oracle(gold):
    import torch
    from deepmatching_stereo_matching_amd.misc.Correlation_map import Correlation_map
    from deepmatching_stereo_matching_amd.misc.Matching import Matching
    assert torch.cuda.is_available()
    g, _ = gold
    co = Correlation_map(g['img1'], g['img2'], window_size=int(g['ws']))
    co()
    O.set_pow_mode('pinned')
    try:
        levels, _, _ = O.pyramid(O.corr_l0(g['img1'], g['img2'], int(g['ws'])))
        for key, b, sp, filt in _cases(g):
            co.N_map = int(g['N_map_b%d' % b])
            kw = dict(filtering=True, filter_window_size=3, filtering_num=3,
                      filtering_mode='median') if filt else {}
            m = Matching(co, sub_pix=sp, **kw)()
            assert m.shape == g[key].shape, key
            ref = O.match_from(levels, b, sub_pix=sp, filtering=filt)
            assert np.array_equal(m, ref, equal_nan=True), key          # bit-exact vs the oracle
            _close(m, g[key], TOL_SUBPIX)
    finally:
        O.set_pow_mode('libm')


@pytest.mark.gpu
def test_subpix_map_full_level_equals_dm_match_subpix(gold):
    """dm_subpix_map with hm = h0 is dm_match's own sub-pixel step."""
    import torch
    from deepmatching_stereo_matching_amd import engine
    _, levels = gold
    dev = torch.device('cuda', 0)
    lv = [torch.from_numpy(x).to(dev) for x in levels]
    plain = engine.match_levels(lv, sub_pix=False).clone()
    sub = engine.match_levels(lv, sub_pix=True)
    engine.subpix_map(lv[0], plain)
    torch.cuda.synchronize()
    assert torch.equal(plain.view(torch.int64), sub.view(torch.int64))


def test_subpix_map_rejects_bad_shapes():
    from deepmatching_stereo_matching_amd import _lib as L
    try:
        lib = L.load()
    except L.DmUnavailable:
        pytest.skip('library not built')
    # argument checks run before any device work
    assert lib.dm_subpix_map(None, 1, 4, 4, 2, 2, None, None) == L.DM_ERR_ARG
    assert lib.dm_subpix_map(1, 1, 4, 4, 8, 2, 1, None) == L.DM_ERR_ARG
    assert lib.dm_subpix_map(1, 0, 4, 4, 2, 2, 1, None) == L.DM_ERR_ARG

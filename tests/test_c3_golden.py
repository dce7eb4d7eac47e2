"""Reference-owned parity at full C3 (S=128) and C2 (S=64) tile size, on the GPU.

tests/golden/make_golden_r03.py ran the unchanged reference on tiles cut from bench.py's own
input pairs (seed 1000): Correlation_map()() -> Matching(sub_pix False/True)() -> cal_map,
and Matching on the same pyramid cut to k levels with N_map = 2^(k-1) (SURVEY.md section 0;
BASELINE configs C3 "4-level", C2 "3-level").  Here the same tiles go through

  * the drop-in mirror (misc.Correlation_map -> misc.Matching), including the k-level cut
    made the reference's way (co_map_list[:k], N_map = 2^(k-1)) and by del / pop, and
  * the path bench.py times (TileBatch of the bench pair -> DevicePyramid.build ->
    match), with and without --levels k.

Tolerances (as tests/test_oracle_golden.py): the whole level-0 volume and the integer
correspondences bit-exact against the reference; float64 levels |d| <= 1e-12; sub-pixel and
cal_map |d| <= 1e-9 (the kernels' pinned pow14 vs numpy's pow: tools/pow_pin.py measures
the difference, profiles/pow_pin.json).
"""
import hashlib
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), 'golden')
NAMES = ['c3_tile_0_0', 'c3_tile_5_3', 'c2_tile_2_5']
TOL_F64 = 1e-12
TOL_SUBPIX = 1e-9
WS = 5


def _close(a, b, tol):
    a, b = np.asarray(a), np.asarray(b)
    assert a.shape == b.shape, (a.shape, b.shape)
    na, nb = np.isnan(a), np.isnan(b)
    assert np.array_equal(na, nb)
    if (~na).any():
        d = np.max(np.abs(a[~na] - b[~na]))
        assert d <= tol, d


def _indices(m, ref):
    assert np.array_equal(np.asarray(m)[:2], np.asarray(ref)[:2]), \
        '%d pixels differ' % int((np.asarray(m)[:2] != np.asarray(ref)[:2]).any(axis=0).sum())


def truncations(g):
    return sorted(int(k[len('match_k'):]) for k in g if k.startswith('match_k'))


@pytest.fixture(scope='module')
def mirror():
    from deepmatching_stereo_matching_amd.misc import Correlation_map as CM, Matching as MT
    from deepmatching_stereo_matching_amd.misc import Calc_difference as CD
    return CM, MT, CD


@pytest.fixture(scope='module', params=NAMES)
def case(request, mirror):
    CM = mirror[0]
    g = dict(np.load(os.path.join(GOLD, request.param + '.npz')))
    co = CM.Correlation_map(g['img1'], g['img2'], window_size=int(g['ws']))
    co()
    yield g, co
    del co
    torch.cuda.empty_cache()


def test_level0_volume_bit_exact(case):
    """Every level-0 value (dm_corr_volume, float32) against the reference's co_map sha256."""
    from deepmatching_stereo_matching_amd import engine
    g, co = case
    S = g['img1'].shape[0] - WS + 1
    v = co._pyr.volume()[0].cpu().numpy().reshape(S, S, S, S)
    co._pyr._volume = None
    assert hashlib.sha256(v.tobytes()).hexdigest() == str(g['l0_sha'])
    idx = g['l0_sample_idx']
    assert np.array_equal(v[idx[:, 0], idx[:, 1]], g['l0_sample'], equal_nan=True)
    assert isinstance(co._pyr, engine.DevicePyramid)


def test_pyramid(case):
    g, co = case
    assert co.iteration == int(g['iteration']) and co.N_map == int(g['N_map'])
    assert len(co.co_map_list) == int(g['nlev'])
    for k in range(2, len(co.co_map_list)):
        lv = co.co_map_list[k]
        s = float(np.nansum(lv))
        assert abs(s - float(g['level%d_sum' % k])) <= TOL_F64 * max(1.0, abs(s))
        if 'level%d' % k in g:
            _close(lv, g['level%d' % k], TOL_F64)


def test_matching(case, mirror):
    CM, MT, CD = mirror
    g, co = case
    m = MT.Matching(co, sub_pix=False)()
    _indices(m, g['match'])
    _close(m[2], g['match'][2], TOL_F64)
    ms = MT.Matching(co, sub_pix=True)()
    _close(ms, g['match_subpix'], TOL_SUBPIX)
    for mode in ('elevation', 'elevation2', 'distance'):
        if 'calmap_' + mode in g:
            _close(CD.Calc_difference.cal_map(ms, mode=mode), g['calmap_' + mode], TOL_SUBPIX)


def test_k_level_pyramid_reference_way(case, mirror):
    """co_map_list cut to k levels and N_map = 2^(k-1), exactly as the golden was made."""
    CM, MT, CD = mirror
    g, co = case
    full, n_full = co.co_map_list, co.N_map
    try:
        for k in truncations(g):
            co.co_map_list = full[:k]
            co.N_map = 2 ** (k - 1)
            assert isinstance(co.co_map_list, CM.LevelList) and len(co.co_map_list) == k
            m = MT.Matching(co, sub_pix=False)()
            _indices(m, g['match_k%d' % k])
            _close(m[2], g['match_k%d' % k][2], TOL_F64)
            ms = MT.Matching(co, sub_pix=True)()
            _close(ms, g['match_subpix_k%d' % k], TOL_SUBPIX)
            _close(CD.Calc_difference.cal_map(ms, mode='elevation'), g['calmap_elevation_k%d' % k],
                   TOL_SUBPIX)
    finally:
        co.co_map_list, co.N_map = full, n_full


def test_k_level_pyramid_del_and_pop(mirror):
    """The other ways a script cuts a list: del co_map_list[k:] and pop()."""
    CM, MT, CD = mirror
    g = dict(np.load(os.path.join(GOLD, 'c2_tile_2_5.npz')))
    co = CM.Correlation_map(g['img1'], g['img2'], window_size=WS)
    co()
    del co.co_map_list[3:]
    co.N_map = 4
    _indices(MT.Matching(co, sub_pix=False)(), g['match_k3'])
    co.co_map_list.pop()
    co.N_map = 2
    assert len(co.co_map_list) == 2
    _close(MT.Matching(co, sub_pix=True)(), g['match_subpix_k2'], TOL_SUBPIX)
    co.N_map = 8                         # more halvings than levels: the reference's IndexError
    with pytest.raises(IndexError):
        MT.Matching(co)()


def test_k_level_on_plain_levels(mirror):
    """A plain numpy co_map_list (levels uploaded, level 0 materialised) cut to 3 levels."""
    CM, MT, CD = mirror
    g = dict(np.load(os.path.join(GOLD, 'c2_tile_2_5.npz')))
    co = CM.Correlation_map(g['img1'], g['img2'], window_size=WS)
    co()

    class Plain:
        co_map_list = [co.co_map_list[k] for k in range(3)]
        N_map = 4
    _indices(MT.Matching(Plain(), sub_pix=False)(), g['match_k3'])
    _close(MT.Matching(Plain(), sub_pix=True)(), g['match_subpix_k3'], TOL_SUBPIX)

    class NoN:
        co_map_list = Plain.co_map_list
    with pytest.raises(AttributeError):  # the reference reads Co_obj.N_map (Matching.py:96)
        MT.Matching(NoN())()


@pytest.mark.parametrize('S', [128, 64])
def test_bench_path_on_reference_tiles(S):
    """bench.py's timed path (one TileBatch of the bench pair, DevicePyramid.build, match with
    sub-pixel), full pyramid and --levels k, against the reference goldens of its tiles."""
    from deepmatching_stereo_matching_amd import _lib as L
    from deepmatching_stereo_matching_amd import engine
    from deepmatching_stereo_matching_amd.synthetic import stereo_pair
    names = [n for n in NAMES if n.startswith('c3' if S == 128 else 'c2')]
    gs = [dict(np.load(os.path.join(GOLD, n + '.npz'))) for n in names]
    side = 9 * S + WS - 1
    a, b = stereo_pair(side, side, seed=1000, dx=2, max_disp=S // 4, sinusoidal=True)
    org = [tuple(int(x) for x in g['origin']) for g in gs]
    for g, (r, c) in zip(gs, org):       # the generator reproduces the goldens' inputs
        assert np.array_equal(a[r:r + S + WS - 1, c:c + S + WS - 1], g['img1'])
        assert np.array_equal(b[r:r + S + WS - 1, c:c + S + WS - 1], g['img2'])
    dev = torch.device('cuda', 0)
    batch = engine.TileBatch(torch.from_numpy(a).to(dev), torch.from_numpy(b).to(dev), org, S, S, WS,
                             L.DM_TM_CCOEFF_NORMED, dev)
    pyr = engine.DevicePyramid(batch, build=False).build()
    full = pyr.match(sub_pix=True).cpu().numpy()
    for t, g in enumerate(gs):
        _close(full[t], g['match_subpix'], TOL_SUBPIX)
    k = truncations(gs[0])[0]
    pk = engine.DevicePyramid(batch, build=False).build(nlev=k)
    assert len(pk.levels) == k
    mk = pk.match(sub_pix=False, nlev=k).cpu().numpy()
    mks = pk.match(sub_pix=True, nlev=k).cpu().numpy()
    for t, g in enumerate(gs):
        _indices(mk[t], g['match_k%d' % k])
        _close(mks[t], g['match_subpix_k%d' % k], TOL_SUBPIX)

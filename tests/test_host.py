"""Host-side logic that needs no GPU: pyramid plan, tile grid, loaders, the driver flags,
and that the product path refuses to run without the HIP device (no CPU fallback)."""
import os

import numpy as np
import pytest

from deepmatching_stereo_matching_amd import engine
from deepmatching_stereo_matching_amd import _lib as L


@pytest.mark.parametrize('h0,w0,nlev,N', [(32, 32, 6, 32), (16, 64, 5, 16), (64, 16, 5, 16),
                                          (8, 8, 4, 8), (1, 1, 1, 1), (2, 6, 2, 2)])
def test_pyramid_plan(h0, w0, nlev, N):
    assert engine.pyramid_plan(h0, w0) == (nlev, N)


@pytest.mark.parametrize('h0,w0', [(124, 124), (6, 6), (12, 12)])
def test_pyramid_plan_rejects_like_reference(h0, w0):
    # misc/Correlation_map.py:96-103: MaxPool of an odd side cannot be assigned
    with pytest.raises(ValueError, match='broadcast'):
        engine.pyramid_plan(h0, w0)


def test_cut_grid_reference_order():
    # image_cut_solver.py:62 floor rule, :103-113 j outer / i inner
    n, org = engine.cut_grid((164, 164), [32, 32], [32, 32], 5)
    assert n == [4, 4]
    assert org[:5].tolist() == [[0, 0], [32, 0], [64, 0], [96, 0], [0, 32]]
    n, org = engine.cut_grid((1156, 1156), [128, 128], [128, 128], 5)
    assert n == [8, 8] and len(org) == 64
    n, org = engine.cut_grid((44, 44), [16, 16], [12, 12], 5)
    assert n == [2, 2]


def test_cut_grid_no_tile():
    with pytest.raises(IndexError):
        engine.cut_grid((20, 20), [32, 32], [32, 32], 5)


def test_tile_bytes_monotone():
    assert engine.tile_bytes(128, 128) > engine.tile_bytes(64, 64) > 0
    # level 1 dominates: (64*64)^2 float64
    assert engine.tile_bytes(128, 128) >= 8 * (64 * 64) ** 2


def test_no_cpu_fallback():
    import torch
    if torch.cuda.is_available():
        pytest.skip('GPU present')
    with pytest.raises(L.DmUnavailable):
        engine.default_device()
    from deepmatching_stereo_matching_amd.misc.Correlation_map import Correlation_map
    img = np.zeros((20, 20), np.uint8)
    with pytest.raises(L.DmUnavailable):
        Correlation_map(img, img, window_size=5)()


def test_reference_error_conventions():
    from deepmatching_stereo_matching_amd.misc.Correlation_map import Correlation_map
    from deepmatching_stereo_matching_amd.misc.Feature_value import Feature_value
    from deepmatching_stereo_matching_amd.misc.Matching import Matching
    from deepmatching_stereo_matching_amd.misc.Calc_difference import Calc_difference
    with pytest.raises(SystemExit):
        Correlation_map(np.zeros((5, 5), np.uint8), np.zeros((5, 6), np.uint8))
    with pytest.raises(SystemExit):
        Feature_value('cv2.TM_SQDIFF')
    with pytest.raises(SystemExit):
        Matching(object())
    with pytest.raises(SystemExit):
        Calc_difference.cal_map(np.zeros((3, 2, 2)), mode='height')

    class Fake:
        co_map_list = []
    with pytest.raises(AssertionError):
        Matching(Fake(), filtering_mode='mode')


def test_raw_read(tmp_path):
    from deepmatching_stereo_matching_amd.misc.raw_read import RawRead
    a = np.arange(-50, 50, dtype=np.int8).reshape(10, 10)
    p = tmp_path / 'x.raw'
    a.tofile(p)
    out = RawRead.read(str(p), size=(10, 10), rate=2)
    assert out.dtype == np.uint8 and np.array_equal(out, (a * 2).astype(np.uint8))


def test_loader_channels(tmp_path):
    from PIL import Image
    from deepmatching_stereo_matching_amd.misc.loader import Loader
    rng = np.random.default_rng(0)
    rgb = rng.integers(0, 256, (40, 50, 3), dtype=np.uint8)
    p = tmp_path / 'x.png'
    Image.fromarray(rgb).save(p)
    before, after, change = Loader(str(p), start=[5, 6], size=[10, 12], integrated=True)()
    assert np.array_equal(before, rgb[5:15, 6:18, 1])   # cv2 BGR channel 1 = G
    assert np.array_equal(after, rgb[5:15, 6:18, 0])    # cv2 channel 2 = R
    assert np.array_equal(change, rgb[5:15, 6:18, 2])   # cv2 channel 0 = B
    g = rng.integers(0, 256, (30, 30), dtype=np.uint8)
    Image.fromarray(g).save(tmp_path / 'g1.png')
    Image.fromarray(g[::-1]).save(tmp_path / 'g2.png')
    a, b = Loader([str(tmp_path / 'g1.png'), str(tmp_path / 'g2.png')], start=[1, 2], size=[8, 9],
                  integrated=False)()
    assert np.array_equal(a, g[1:9, 2:11]) and np.array_equal(b, g[::-1][1:9, 2:11])


def test_alias_misc_imports_every_mirror_module():
    """Reference scripts import ``misc.<module>`` (deep_dem_mathing.py:11-13,
    optimize_looper.py:21 ``from misc.opt_loop import *``); under alias_misc() every module
    of the reference's misc/ that the mirror re-provides must import, in a fresh
    interpreter (no GPU needed to import)."""
    import subprocess
    import sys
    code = ('import deepmatching_stereo_matching_amd as p; p.alias_misc()\n'
            'from misc.opt_loop import *\n'
            'from misc.optimize_loop import optimize_loop, image_threshold\n'
            'from misc.Correlation_map import Correlation_map, Maxpool\n'
            'from misc.Matching import Matching, Zero_padding\n'
            'from misc.Calc_difference import Calc_difference\n'
            'from misc.Feature_value import Feature_value\n'
            'from misc.image_cut_solver import ImageCutSolver\n'
            'from misc.loader import Loader\n'
            'from misc.raw_read import RawRead\n'
            'from misc.sub_pix_cal import sub_pix_cal\n'
            'assert callable(make_weight) and callable(optimize_loop_bilateral_horizon)\n')
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, '-c', code], cwd=repo, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_atomic_patch_on_host_matches_reference():
    """Correlation_map._create_atomic_patch runs on the host (no device needed) and equals
    the reference's atomic_patch (bad_matching_* fixtures, Correlation_map.py:51-67)."""
    import glob
    from deepmatching_stereo_matching_amd.misc.Correlation_map import Correlation_map
    paths = sorted(glob.glob(os.path.join(os.path.dirname(__file__), 'golden', 'bad_matching_*.npz')))
    assert paths
    for p in paths:
        g = np.load(p)
        co = Correlation_map(g['img1'], g['img2'], window_size=int(g['ws']),
                             feature_name=str(g['feature']))
        co._create_atomic_patch()
        assert co.atomic_patch.dtype == np.uint8
        assert np.array_equal(co.atomic_patch, g['atomic_patch'])
        with pytest.raises(AttributeError):      # no co_map before _create_simple_initial_co_map
            co.co_map


def test_matching_descent_reads_co_map_list_and_n_map():
    """Matching follows the reference's loop (misc/Matching.py:85-149): start at
    co_map_list[-1], one _B per halving of N_map until N == 1, IndexError when N_map asks for
    more levels than the list holds (a k-level cut: co_map_list[:k], N_map = 2^(k-1))."""
    from deepmatching_stereo_matching_amd.misc.Matching import Matching

    def obj(n, N):
        class O:
            co_map_list = [np.zeros((1 << (n - 1 - k),) * 4) for k in range(n)]
            N_map = N
        return O()
    for n in range(2, 9):
        lst, bottom, steps = Matching(obj(n, 2 ** (n - 1)))._descent()
        assert (bottom, steps, len(lst)) == (0, n - 1, n)
    assert Matching(obj(4, 4))._descent()[1:] == (1, 2)     # stops above level 0
    assert Matching(obj(4, 6))._descent()[1:] == (1, 2)     # int(6/2) = 3, int(3/2) = 1
    for N in (16, 1, 0):                                    # never reaches 1 in time
        with pytest.raises(IndexError):
            Matching(obj(4, N))._descent()
    with pytest.raises(IndexError):
        Matching(obj(1, 1))._descent()

    class NoN:
        co_map_list = []
    with pytest.raises(AttributeError):
        Matching(NoN())._descent()


def test_level_list_cuts_like_a_list():
    """co_map_list of the device pyramid: prefix slices stay device-backed, del of a suffix
    and pop() shorten it, other cuts raise (host logic only, a stand-in pyramid)."""
    from deepmatching_stereo_matching_amd.misc.Correlation_map import LevelList

    class Pyr:
        nlev = 5

        def level_shape(self, k):
            return (1 << (4 - k),) * 4

        def level(self, k):
            import torch
            return torch.full((1,) + (1 << (2 * (4 - k)),) * 2, float(k), dtype=torch.float64)
    ll = LevelList(Pyr())
    assert len(ll) == 5 and ll[-1].shape == (1, 1, 1, 1) and ll[4][0, 0, 0, 0] == 4
    v = ll[:3]
    assert isinstance(v, LevelList) and len(v) == 3 and v[-1][0, 0, 0, 0] == 2
    assert isinstance(ll[1:3], list) and len(ll[1:3]) == 2
    assert len(ll[:0]) == 0 and len(ll[:-1]) == 4
    with pytest.raises(IndexError):
        v[3]
    del v[2:]
    assert len(v) == 2 and len(ll) == 5
    assert v.pop()[0, 0, 0, 0] == 1 and len(v) == 1
    with pytest.raises(TypeError):
        del ll[1:3]
    with pytest.raises(TypeError):
        ll.pop(0)
    del ll[4]
    assert len(ll) == 4
    # negative steps: an empty cut deletes nothing; a top suffix taken backwards drops it;
    # any other cut (a plain list would delete those items) raises
    del ll[2:2:-1]
    assert len(ll) == 4
    del ll[:1:-1]                      # items 3, 2: the top suffix from level 2
    assert len(ll) == 2
    with pytest.raises(TypeError):
        del ll[-2::-1]                 # item 0 only: not a top suffix
    del ll[::-2]                       # item 1: the top
    assert len(ll) == 1

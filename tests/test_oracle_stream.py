"""The oracle's streaming mode (level 0 never stored: dmo_corr_level1_stream,
dmo_match_stream, dmo_corr_l0_rows) against its materialising mode, which the reference
goldens pin (test_oracle_golden.py).  Bit-exact, both pow modes, both methods, NaN rows;
this is what lets the GPU tests check a full C5 tile (S = 256) against the oracle."""
import numpy as np
import pytest

from oracle import oracle as O
from deepmatching_stereo_matching_amd.synthetic import stereo_pair


def _same(a, b):
    assert a.shape == b.shape
    assert np.array_equal(a, b, equal_nan=True)


@pytest.mark.parametrize('pow_mode', ['libm', 'pinned'])
@pytest.mark.parametrize('h0,w0,ws,feat,flat', [
    (16, 16, 5, 'cv2.TM_CCOEFF_NORMED', False), (32, 32, 5, 'cv2.TM_CCOEFF_NORMED', True),
    (16, 64, 3, 'cv2.TM_CCOEFF_NORMED', False), (64, 16, 5, 'cv2.TM_CCOEFF', False),
    (32, 32, 7, 'cv2.TM_CCOEFF', True), (64, 64, 5, 'cv2.TM_CCOEFF_NORMED', False),
    (2, 2, 3, 'cv2.TM_CCOEFF_NORMED', False)])
def test_stream_equals_materialised(pow_mode, h0, w0, ws, feat, flat):
    a, b = stereo_pair(h0 + ws - 1, w0 + ws - 1, seed=h0 + 3 * w0 + ws, dx=2, sinusoidal=True)
    if flat:                       # constant patches -> NaN rows (NORMED) / zero rows
        a = a.copy()
        a[3:3 + ws + 2, 4:4 + ws + 3] = 90
    O.set_pow_mode(pow_mode)
    try:
        l0 = O.corr_l0(a, b, ws, feat)
        lev, it, n = O.pyramid(l0)
        slev, sit, sn = O.pyramid_stream(a, b, ws, feat)
        assert (it, n) == (sit, sn) and len(lev) == len(slev)
        for k in range(1, len(lev)):
            _same(slev[k], lev[k])
        for sp in (False, True):
            _same(O.match_stream(a, b, ws, slev, sub_pix=sp, feature=feat), O.match(lev, sub_pix=sp))
        P = h0 * w0
        rows = np.array([0, P - 1, P // 3, 5 % P], dtype=np.int64)
        _same(O.corr_l0_rows(a, b, ws, rows, feat), l0.reshape(P, P)[rows])
    finally:
        O.set_pow_mode('libm')


def test_zncc_formula_pin_is_within_float32_rounding():
    """the kernels' two-multiply ZNCC (pinned) against SURVEY 8(c)'s
    f64-division formula moves level-0 values by float32 rounding only (|d| <= 2^-21 on
    [0, 1], no NaN moved) and, on this tile, no integer correspondence
    (tools/zncc_pin.py measures 8 C3 tiles: profiles/zncc_pin.json)."""
    a, b = stereo_pair(36, 36, seed=0, dx=2, max_disp=8, sinusoidal=True)
    d = O.zncc_formula_diff(a, b, 5)
    assert d['nan_mismatch'] == 0 and d['values'] > 0
    assert d['max_abs'] <= 2.0 ** -21
    res = {}
    for f in ('pinned', 'f64div'):
        O.set_zncc_formula(f)
        try:
            lev, _, _ = O.pyramid_stream(a, b, 5)
            res[f] = O.match_stream(a, b, 5, lev, sub_pix=False)
        finally:
            O.set_zncc_formula('pinned')
    assert np.array_equal(res['pinned'][:2], res['f64div'][:2])

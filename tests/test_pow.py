"""The pinned float64 pow(x, 1.4) (deepmatching_stereo_matching_amd/csrc/dm_pow.h).

Host build via the oracle library (the same header is compiled into the HIP kernels; the
GPU bit-identity is checked in test_gpu_parity.py).  Accuracy is measured against a
60-digit decimal evaluation: every sample within 1 ulp, >= 99.9 % correctly rounded.
"""
import math
from decimal import Decimal, getcontext

import numpy as np
import pytest

from oracle import oracle as O

Y = Decimal(1.4)


def _exact(x):
    getcontext().prec = 60
    return float((Y * Decimal(x).ln()).exp())


def _ulps(a, b):
    return abs(int(np.float64(a).view(np.int64)) - int(np.float64(b).view(np.int64)))


def test_special_values():
    assert O.pow14(0.0) == 0.0 and O.pow14(-0.0) == 0.0
    assert O.pow14(1.0) == 1.0
    assert math.isnan(O.pow14(float('nan')))
    assert math.isnan(O.pow14(-0.5))
    assert O.pow14(float('inf')) == float('inf')
    assert O.pow14(2.0 ** -1074) == 0.0 or O.pow14(2.0 ** -1074) >= 0.0


@pytest.mark.parametrize('kind', ['f32_unit', 'f64_unit', 'wide'])
def test_accuracy(kind):
    rng = np.random.default_rng({'f32_unit': 1, 'f64_unit': 2, 'wide': 3}[kind])
    if kind == 'f32_unit':
        xs = rng.random(3000).astype(np.float32).astype(np.float64)
    elif kind == 'f64_unit':
        xs = rng.random(3000)
    else:
        xs = np.exp2(rng.uniform(-700, 700, 3000)) * rng.random(3000)
    bad = cr = 0
    for x in xs:
        if x == 0:
            continue
        got, ref = O.pow14(x), _exact(x)
        u = _ulps(got, ref)
        bad += u > 1
        cr += u == 0
    assert bad == 0
    assert cr >= 0.999 * len(xs) - 1


def test_agrees_with_libm_mostly():
    rng = np.random.default_rng(5)
    xs = rng.random(20000)
    u = np.array([_ulps(O.pow14(x), math.pow(x, 1.4)) for x in xs])
    assert u.max() <= 1


def _fast_c_table():
    import os
    import re
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                        'deepmatching_stereo_matching_amd', 'csrc', 'dm_pow_tables.h')
    text = open(path).read()
    body = text.split('#define DM_POWF_C_INIT {', 1)[1].split('}', 1)[0]
    return [float.fromhex(h) for h in re.findall(r'-?0x[0-9a-fA-Fp.+-]+', body)]


def test_fast_table_makes_float32_r_exact():
    """The level kernel forms r = M c_i - 1 for float32 inputs with one float32 FMA
    (dm_kernels.hip pow14_zf); that equals the oracle's float64 FMA only because c_i has
    <= 10 significant bits and |r| < 2^-9 (gen_pow_tables.py).  Check both, and the
    exactness itself on every bin's end points and random float32 mantissas."""
    from fractions import Fraction
    cs = _fast_c_table()
    assert len(cs) == 512
    for i, c in enumerate(cs):
        m, e = math.frexp(c)
        assert float(m * 2 ** 10).is_integer(), (i, c)
        for M in (1 + i / 512, 1 + (i + 1) / 512 - 2.0 ** -23):
            assert abs(Fraction(M) * Fraction(c) - 1) < Fraction(1, 512), (i, M)
    rng = np.random.default_rng(7)
    for u in rng.integers(0, 1 << 23, 20000):
        M = 1 + int(u) / 2 ** 23
        i = int(u) >> 14
        exact = Fraction(M) * Fraction(cs[i]) - 1
        assert float(np.float32(float(exact))) == exact   # representable in float32


def _pow14_array(x):
    """The pinned pow on an array (oracle dmo_rectify_f64 in pinned mode)."""
    y = np.ascontiguousarray(x, dtype=np.float64).copy()
    O.set_pow_mode('pinned')
    try:
        O.lib().dmo_rectify_f64(y.ctypes.data_as(O.ctypes.c_void_p), y.size, O.LAM)
    finally:
        O.set_pow_mode('libm')
    return y


def test_pinned_pow_is_monotone():
    """The level kernel pools BEFORE rectifying (MaxPool of pow14(s/4) == pow14 of the MaxPool,
    dm_mfma.h level2_row; the sweeps pool y before r, x, pow14): that is bit-exact only if the
    pinned pow is non-decreasing on adjacent doubles.  Checked where it can break -- both ends
    of every one of the 512 mantissa bins (the c_i table edges) at every exponent of the fast
    path [2^EMIN, 1], plus random points and their successors."""
    emin = -319
    i = np.arange(512, dtype=np.float64)
    lo = 1.0 + i / 512.0                       # first double of bin i
    hi = np.nextafter(1.0 + (i + 1) / 512.0, 0)  # last double of bin i
    xs = []
    for e in range(emin, 1):
        s = np.ldexp(1.0, e)
        for b in (lo, hi):
            v = b * s
            xs.append(np.nextafter(v, 0))
            xs.append(v)
            xs.append(np.nextafter(v, np.inf))
    rng = np.random.default_rng(11)
    r = np.exp2(rng.uniform(emin, 0, 200000))
    x = np.concatenate(xs + [r])
    x = x[(x > 0) & (x <= 1.0)]
    nxt = np.minimum(np.nextafter(x, np.inf), 1.0)
    a, b = _pow14_array(x), _pow14_array(nxt)
    assert np.all(b >= a)
    # and the ends of each bin meet the next bin's start without a step down
    starts = np.concatenate([np.ldexp(lo, e) for e in range(emin, 0)])
    prev = np.nextafter(starts, 0)
    assert np.all(_pow14_array(starts) >= _pow14_array(prev))


def test_pow_pin_vs_libm_within_bound():
    """DESIGN.md section 2 / tools/pow_pin.py (profiles/pow_pin.json: 8 C3 tiles + 1 C5 tile,
    0 of 196,608 correspondences flipped, levels within 7.5e-16 relative, sub-pixel within
    1.5e-14): the kernels' pinned pow14 against libm (numpy's pow, the reference's) on one
    S=32 tile of the same generator -- no integer correspondence moves, float64 levels and
    sub-pixel values move by rounding only."""
    from deepmatching_stereo_matching_amd.synthetic import stereo_pair
    a, b = stereo_pair(36, 36, seed=1000, dx=2, max_disp=8, sinusoidal=True)
    res = {}
    for mode in ('libm', 'pinned'):
        O.set_pow_mode(mode)
        try:
            lev, _, _ = O.pyramid_stream(a, b, 5)
            res[mode] = (lev, O.match_stream(a, b, 5, lev, sub_pix=False),
                         O.match_stream(a, b, 5, lev, sub_pix=True))
        finally:
            O.set_pow_mode('libm')
    (l0, m0, s0), (l1, m1, s1) = res['libm'], res['pinned']
    assert np.array_equal(m0[:2], m1[:2])
    for x, y in zip(l0[1:], l1[1:]):
        assert np.array_equal(np.isnan(x), np.isnan(y))
        ok = ~np.isnan(x) & (x != 0)
        assert np.max(np.abs(x[ok] - y[ok]) / np.abs(x[ok])) <= 4e-15
    assert np.nanmax(np.abs(s0 - s1)) <= 1e-12

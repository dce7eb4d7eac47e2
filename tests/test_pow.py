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

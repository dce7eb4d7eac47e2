"""The pow14 forms the fused kernels evaluate in place of _rectification
(misc/Correlation_map.py:158-159), through dm_pow14_variant (include/dmstereo.h): each equals
the pinned dm_pow14 (the oracle's host build of csrc/dm_pow.h) bit for bit on the domain the
header states, and the two documented out-of-domain results of pow14_q4 hold.

The level kernel pools before it rectifies (level 1 as pow14_q4 of the pooled child sums,
level 2 likewise), so besides monotonicity (test_pow.py) it relies on pow14_q4(s) ==
pow14(s / 4) for every sum it can see: 0, NaN and s / 4 in [2^-319, 1]."""
import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def lib():
    from deepmatching_stereo_matching_amd import _lib as L
    return L


@pytest.fixture(autouse=True)
def pinned():
    O.set_pow_mode('pinned')
    yield
    O.set_pow_mode('libm')


def _dev(lib, variant, xs):
    x = torch.from_numpy(np.ascontiguousarray(xs, dtype=np.float64)).cuda()
    out = torch.empty_like(x)
    lib.check(lib.load().dm_pow14_variant(variant, lib.ptr(x), x.numel(), lib.ptr(out),
                                          lib.stream_handle()), 'dm_pow14_variant')
    torch.cuda.synchronize()
    return out.cpu().numpy()


def _host(xs):
    return np.array([O.pow14(float(v)) for v in xs])


def _same(a, b):
    return np.array_equal(a.view(np.int64), b.view(np.int64)) or (
        np.array_equal(np.isnan(a), np.isnan(b)) and np.array_equal(a[~np.isnan(a)], b[~np.isnan(b)]))


def _bin_edges(emin, emax, rng, nbins=512):
    """both ends of every mantissa bin of the fast path's table at a spread of exponents"""
    out = []
    for e in sorted(set([emin, emin + 1, -127, -126, -64, -8, -2, -1, 0] +
                        list(rng.integers(emin, emax + 1, 8)))):
        if not emin <= e <= emax:
            continue
        for i in range(nbins):
            lo = np.ldexp(1.0 + i / nbins, e)
            hi = np.nextafter(np.ldexp(1.0 + (i + 1) / nbins, e), 0.0)
            out += [lo, hi]
    return np.array([v for v in out if v <= 1.0])


def test_f32_form(lib):
    rng = np.random.default_rng(11)
    xs = np.concatenate([rng.random(60000),
                         np.ldexp(rng.random(20000) + 1.0, -rng.integers(1, 126, 20000)),
                         [0.0, 1.0, 2.0 ** -126, np.nan]]).astype(np.float32)
    xs = xs[(xs == 0) | (xs >= np.float32(2.0 ** -126)) | np.isnan(xs)].astype(np.float64)
    assert _same(_dev(lib, lib.DM_POW_F32, xs), _host(xs))


def test_f32_form_bin_edges(lib):
    xs = _bin_edges(-126, -1, np.random.default_rng(12), 512)
    xs = xs.astype(np.float32).astype(np.float64)
    assert _same(_dev(lib, lib.DM_POW_F32, xs), _host(xs))


def test_q4_is_pow_of_quarter(lib):
    rng = np.random.default_rng(13)
    s = np.concatenate([4.0 * rng.random(60000),
                        4.0 * np.ldexp(rng.random(20000) + 1.0, -rng.integers(1, 318, 20000)),
                        4.0 * _bin_edges(-319, -1, rng, 512)[::7],
                        [0.0, 4.0, np.nan, 4.0 * 2.0 ** -319]])
    assert _same(_dev(lib, lib.DM_POW_Q4, s), _host(s / 4.0))


def test_q4_out_of_domain_is_documented(lib):
    s = np.array([4.0 * 2.0 ** -330, 4.0 * 2.0 ** -1000, 2.0 ** -1074, np.inf])
    got = _dev(lib, lib.DM_POW_Q4, s)
    assert np.all(got[:3] == 0.0), got
    assert np.isnan(got[3])
    # dm_pow14 itself: (2^-330)^1.4 = 2^-462 is a normal double (pow14_q4 diverges there: its
    # callers never go below 2^EMIN); (2^-1000)^1.4 and the quarter of 2^-1074 underflow to 0
    want = _host(s[:3] / 4.0)
    assert want[0] > 0.0 and np.all(want[1:] == 0.0), want


def test_k_form(lib):
    rng = np.random.default_rng(14)
    xs = np.concatenate([rng.random(50000), np.ldexp(rng.random(20000) + 1.0, -rng.integers(1, 319, 20000)),
                         [0.0, 1.0, np.nan, 2.0 ** -319]])
    assert _same(_dev(lib, lib.DM_POW_K, xs), _host(xs))


def test_full_form_everywhere(lib):
    rng = np.random.default_rng(15)
    xs = np.concatenate([rng.random(20000), np.ldexp(rng.random(20000) + 1.0, rng.integers(-1074, 1023, 20000)),
                         [0.0, -0.0, 1.0, np.inf, -1.0, np.nan, 2.0 ** -1074, 2.0 ** -1022, 1.5, 1e300]])
    assert _same(_dev(lib, lib.DM_POW_FULL, xs), _host(xs))


def test_g32_forms_equal_the_gz_forms_everywhere(lib):
    """pow14_q4g / pow14_kg (the pruned level kernel's forms, no gz rows in LDS) equal pow14_q4 /
    pow14_k bit for bit on every double: the domains, zero, NaN, +-inf, negatives, values above
    1 and the rare inputs below 2^-126 (the constant-memory path) and below 2^-319 (0)."""
    rng = np.random.default_rng(16)
    xs = np.concatenate([rng.random(50000), 4.0 * rng.random(50000),
                         np.ldexp(rng.random(40000) + 1.0, rng.integers(-1074, 1023, 40000)),
                         np.ldexp(rng.random(20000) + 1.0, -rng.integers(120, 330, 20000)),
                         4.0 * _bin_edges(-319, -1, rng, 512)[::5],
                         [0.0, -0.0, 1.0, 4.0, np.inf, -np.inf, -1.0, np.nan, 2.0 ** -1074, 2.0 ** -1022,
                          2.0 ** -126, 2.0 ** -127, 4.0 * 2.0 ** -126, 4.0 * 2.0 ** -127, 2.0 ** -319,
                          2.0 ** -320, 4.0 * 2.0 ** -319, 4.0 * 2.0 ** -320, 1.5, 1e300]])
    assert _same(_dev(lib, lib.DM_POW_Q4G, xs), _dev(lib, lib.DM_POW_Q4, xs))
    assert _same(_dev(lib, lib.DM_POW_KG, xs), _dev(lib, lib.DM_POW_K, xs))

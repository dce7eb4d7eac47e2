"""dm_seq_sum (include/dmstereo.h): the error sums of the Gauss-Seidel loops,
`error += abs(img_dis[i, j] - d_new)` (misc/optimize_loop.py:34, misc/opt_loop.py:33), are
float64 sums in sequence order.  The library takes them as exact integer prefix sums between
the steps where the running sum climbs a binade or ties (k_seq_sum_seg); each case here is
checked bit for bit against the plain sequential loop (np.cumsum is that loop: an
accumulate, not numpy's pairwise sum -- pinned on a small case against a Python loop) and
against the library's own dependent-chain kernel (DM_SEQ_SUM=chain).

The cases are built to hit every branch: binade climbs from 0 and from subnormals, chunk
boundaries (8192 terms), exact ties u/2 and 3u/2 at several binades, terms at or above the
binade's top, zeros, NaN and inf, and the sizes of a 1024^2 sweep."""
import math
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def lib():
    from deepmatching_stereo_matching_amd import _lib as L
    return L


def _dev(lib, v, method=None):
    x = torch.from_numpy(np.ascontiguousarray(v, dtype=np.float64)).cuda()
    out = torch.full((1,), -1.0, dtype=torch.float64, device='cuda')
    old = os.environ.pop('DM_SEQ_SUM', None)
    if method:
        os.environ['DM_SEQ_SUM'] = method
    try:
        lib.check(lib.load().dm_seq_sum(lib.ptr(x) if x.numel() else None, x.numel(), lib.ptr(out),
                                        lib.stream_handle()), 'dm_seq_sum')
        torch.cuda.synchronize()
    finally:
        os.environ.pop('DM_SEQ_SUM', None)
        if old is not None:
            os.environ['DM_SEQ_SUM'] = old
    return float(out.cpu().numpy()[0])


def _seq(v):
    v = np.asarray(v, dtype=np.float64)
    return float(np.cumsum(v)[-1]) if v.size else 0.0


def _same(a, b):
    return (math.isnan(a) and math.isnan(b)) or (a == b and math.copysign(1, a) == math.copysign(1, b))


def test_cumsum_is_the_sequential_loop():
    rng = np.random.default_rng(1)
    v = np.abs(rng.standard_normal(5000)) * 10.0 ** rng.integers(-8, 8, 5000)
    s = 0.0
    for x in v:
        s += float(x)
    assert _seq(v) == s


def _cases():
    rng = np.random.default_rng(7)
    n_sweep = 1021 * 1013                   # a 1024^2 sweep at exclusion 1
    ties = [1.0] + [2.0 ** -53] * 700 + [3 * 2.0 ** -53] * 700 + [1.0] + [2.0 ** -52] * 300 + [3 * 2.0 ** -52] * 300
    ties = np.array(ties)
    tie_mix = np.abs(rng.standard_normal(30000))
    tie_mix[::97] = 2.0 ** -50               # ties once the sum is in [2^2, 2^3) .. and beyond
    return {
        'sweep_errors': np.abs(rng.standard_normal(n_sweep)) * 1e-3,
        'sweep_errors_lognormal': np.exp(rng.normal(-6, 3, n_sweep)),
        'log_uniform_range': 10.0 ** rng.uniform(-300, 10, 100000),
        'subnormal_start': np.concatenate([np.full(20000, 5e-324) * rng.integers(0, 9, 20000),
                                           10.0 ** rng.uniform(-310, -300, 20000), rng.random(1000)]),
        'zeros': np.zeros(20000),
        'one_term': np.array([0.3]),
        'chunk_edges': np.concatenate([np.full(8191, 1e-9), [1e3], np.full(8193, 1e-9), [1e6],
                                       np.full(16384, 0.5)]),
        'geometric_climb': 2.0 ** np.arange(-60, 60, dtype=np.float64),
        'top_of_binade': np.concatenate([[1.0], np.full(5000, 2.0 ** -40), [1.0 - 2.0 ** -53], np.full(5000, 2.0 ** -60)]),
        'ties': ties,
        'tie_mix': tie_mix,
        'nan_middle': np.concatenate([rng.random(10000), [np.nan], rng.random(10000)]),
        'inf_then_nan': np.concatenate([rng.random(9000), [np.inf], rng.random(10), [np.nan], rng.random(10)]),
        'inf_only': np.concatenate([rng.random(100), [np.inf], rng.random(9000)]),
        # dm_seq_sum is a public entry point: negative terms (the reference's callers pass abs()
        # values only) are steps of their own, and a negative running sum adds one by one
        'negative_terms': np.where(rng.random(30000) < 0.01, -1.0, 1.0) * np.abs(rng.standard_normal(30000)),
        'negative_sum': np.concatenate([rng.random(5000), [-1e6], rng.random(20000), [2e6], rng.random(9000)]),
        'negative_zero': np.concatenate([[-0.0], rng.random(100), [-0.0, -1e-300]]),
    }


CASES = _cases()


@pytest.mark.parametrize('name', sorted(CASES))
def test_seq_sum_bit_exact(lib, name):
    v = CASES[name]
    want = _seq(v)
    got = _dev(lib, v)
    assert _same(got, want), (name, got, want)


@pytest.mark.parametrize('name', ['sweep_errors', 'ties', 'log_uniform_range', 'nan_middle', 'negative_sum'])
def test_seq_sum_equals_chain_kernel(lib, name):
    v = CASES[name]
    assert _same(_dev(lib, v), _dev(lib, v, 'chain'))


def test_seq_sum_empty(lib):
    assert _same(_dev(lib, np.zeros(0)), 0.0)


def test_seq_sum_random_lengths(lib):
    rng = np.random.default_rng(11)
    for n in (2, 63, 64, 65, 8191, 8192, 8193, 3 * 8192 + 5, 100003):
        v = np.abs(rng.standard_normal(n)) * 10.0 ** rng.integers(-5, 5, n)
        assert _same(_dev(lib, v), _seq(v)), n

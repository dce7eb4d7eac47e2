"""BASELINE config C5 at its full size: the 4096^2 pair of bench.py's c5_split line (16 x 16
tiles of S = 256, ws = 5, the reference's ImageCutSolver loop, misc/image_cut_solver.py:144-179)
through shard.BandSolver, the multi-GPU product path, here without a process group (one rank
solves every tile, in 4 chunks of 64 tiles).

  * BandSolver's [256][3][256][256] results == engine.solve_tiles over all 256 tiles, byte for
    byte (the chunking changes which tiles share a launch, never a result);
  * tiles on either side of every chunk boundary (0, 63 | 64, 127 | 128, 191 | 192, 255) ==
    the same tile solved alone (a batch of one: other launch shapes, other workgroup order);
  * a second solve by the same BandSolver (its TileBatches reused) repeats the first;
  * the stitched maps == engine.stitch of the unchunked results
    (NaN equal to NaN throughout).

Tile-level parity with the oracle at S = 256 is tests/test_c5_tile.py's; this file pins that
the full pair the bench line measures is the same computation.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

S, GRID, WS = 256, 16, 5
MODES = ['elevation']


def _same(x, y):
    assert x.shape == y.shape and x.dtype == y.dtype, (x.shape, y.shape)
    eq = (x == y) | (torch.isnan(x) & torch.isnan(y))
    assert bool(eq.all()), 'differs at %d of %d values' % (int((~eq).sum()), eq.numel())


@pytest.fixture(scope='module')
def pair():
    from deepmatching_stereo_matching_amd.synthetic import stereo_pair
    from deepmatching_stereo_matching_amd import engine
    side = (GRID + 1) * S + WS - 1             # as bench.c5_split makes it
    a, b = stereo_pair(side, side, seed=1000, dx=2, max_disp=S // 4, sinusoidal=True)
    n, org = engine.cut_grid(a.shape, [S, S], [S, S], WS)
    assert list(n) == [GRID, GRID]
    return a, b, n, org


@pytest.fixture(scope='module')
def banded(pair):
    from deepmatching_stereo_matching_amd import shard
    a, b, n, org = pair
    band = shard.BandSolver(a, b, org, S, S, WS, 5, chunks=4)
    assert band.chunks == 4 and [len(i) for i in band.chunk_idx] == [64] * 4
    first = band.solve()
    second = band.solve()
    torch.cuda.synchronize()
    return band, first, second


def test_band_equals_unchunked(pair, banded):
    from deepmatching_stereo_matching_amd import engine
    a, b, n, org = pair
    _, first, second = banded
    whole = engine.solve_tiles(a, b, org, S, S, WS, 5)
    assert first.shape == (GRID * GRID, 3, S, S) and first.dtype == torch.float64
    _same(first, second)
    _same(first, whole)
    d1, o1 = engine.stitch(first, n, S, S, [S, S], MODES)
    d2, o2 = engine.stitch(whole, n, S, S, [S, S], MODES)
    _same(d1, d2)
    _same(o1, o2)


@pytest.mark.parametrize('t', [0, 63, 64, 127, 128, 191, 192, 255])
def test_chunk_boundary_tiles_equal_single_tile(pair, banded, t):
    from deepmatching_stereo_matching_amd import engine
    a, b, n, org = pair
    _, first, _ = banded
    one = engine.solve_tiles(a, b, org[t:t + 1], S, S, WS, 5)
    _same(first[t:t + 1], one)

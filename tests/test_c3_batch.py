"""BASELINE configs C3 (and C2) exactly as bench.py runs them, against the oracle tile by tile.

The bench's input (the 1156^2 synthetic pair of seed 1000; 580^2 for C2) is
cut into 8x8 tiles of S = 128 (S = 64) with ws = 5 and solved as ONE batch through the path bench.py times
(TileBatch -> DevicePyramid.build: stats, the fused level-1/level-2 kernel, levels >= 3 ->
match with sub-pixel, levels 0/1 recomputed on demand -> stitch).  All 64 tiles have their
Matching output compared bit for bit with the oracle's (streaming mode, pinned pow; pinned
to the materialising oracle by tests/test_oracle_stream.py, which the reference goldens
pin), and their part of the stitched elevation map with the oracle's cal_map.
"""
import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu

WS, GRID = 5, 8


def _same(a, b):
    a, b = np.asarray(a), np.asarray(b)
    assert a.shape == b.shape, (a.shape, b.shape)
    assert np.array_equal(a, b, equal_nan=True), 'max |d| = %r' % np.nanmax(np.abs(a - b))


@pytest.mark.parametrize('S', [128, 64])   # C3, C2
def test_c3_batch_vs_oracle(S):
    from deepmatching_stereo_matching_amd import _lib as L
    from deepmatching_stereo_matching_amd import engine
    from deepmatching_stereo_matching_amd.synthetic import stereo_pair
    side = (GRID + 1) * S + WS - 1
    a, b = stereo_pair(side, side, seed=1000, dx=2, max_disp=S // 4, sinusoidal=True)
    dev = torch.device('cuda', 0)
    n, org = engine.cut_grid(a.shape, [S, S], [S, S], WS)
    assert n == [GRID, GRID] and len(org) == 64
    batch = engine.TileBatch(torch.from_numpy(a).to(dev), torch.from_numpy(b).to(dev), org, S, S, WS,
                             L.DM_TM_CCOEFF_NORMED, dev)
    pyr = engine.DevicePyramid(batch, build=False)
    pyr.build()
    match = pyr.match(sub_pix=True)
    dmap, _ = engine.stitch(match, n, S, S, [S, S], ['elevation'])
    match, dmap = match.cpu().numpy(), dmap.cpu().numpy()[0]
    O.set_pow_mode('pinned')
    try:
        for i, j in [(i, j) for j in range(GRID) for i in range(GRID)]:
            t = j * GRID + i                       # reference order: j outer, i inner
            r, c = org[t]
            assert (r, c) == (i * S, j * S)
            ta, tb = a[r:r + S + WS - 1, c:c + S + WS - 1], b[r:r + S + WS - 1, c:c + S + WS - 1]
            lev, _, _ = O.pyramid_stream(ta, tb, WS)
            m = O.match_stream(ta, tb, WS, lev, sub_pix=True)
            _same(match[t], m)
            _same(dmap[r:r + S, c:c + S], O.cal_map(m, 'elevation'))
    finally:
        O.set_pow_mode('libm')

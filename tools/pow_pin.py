"""How far does the kernels' pinned pow14 (csrc/dm_pow.h) move the pyramid and the matches,
against numpy/libm's ``x ** 1.4`` that the reference uses (misc/Correlation_map.py:158-159)?
CPU only (the oracle in its two pow modes, streaming: level 0 is never stored).

Tiles: 8 S=128 tiles of bench.py's C3 pair (1156^2, seed 1000, sinusoidal shift; grid
positions (i, i) on the diagonal) and 1 S=256 tile of its C5 pair (4356^2, seed 1000).

Reports, per tile and in total: float64 values of levels >= 1 that differ and their max
relative difference; integer correspondences (Matching without sub-pixel) that flip, on the
full pyramid and on the 4-level cut (co_map_list[:4], N_map = 8); max |d| of the sub-pixel
output.  Writes profiles/pow_pin.json.

    python tools/pow_pin.py [--tiles 8] [--c5-tiles 1]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from oracle import oracle as O  # noqa: E402
from deepmatching_stereo_matching_amd.synthetic import stereo_pair  # noqa: E402

WS = 5


def solve(a, b, mode, k=4):
    O.set_pow_mode(mode)
    try:
        lev, _, _ = O.pyramid_stream(a, b, WS)
        return (lev, O.match_stream(a, b, WS, lev, sub_pix=False),
                O.match_stream(a, b, WS, lev, sub_pix=True),
                O.match_stream(a, b, WS, lev[:k], sub_pix=False))
    finally:
        O.set_pow_mode('libm')


def compare(a, b, S, where):
    l_lib, m_lib, s_lib, k_lib = solve(a, b, 'libm')
    l_pin, m_pin, s_pin, k_pin = solve(a, b, 'pinned')
    values = differ = 0
    max_rel = 0.0
    for x, y in zip(l_lib[1:], l_pin[1:]):
        ok = ~np.isnan(x)
        assert np.array_equal(np.isnan(x), np.isnan(y))
        d = x[ok] != y[ok]
        values += int(ok.sum())
        differ += int(d.sum())
        if d.any():
            max_rel = max(max_rel, float(np.max(np.abs(x[ok][d] - y[ok][d]) / np.abs(x[ok][d]))))
    return dict(tile=where, S=S, level_values=values, level_values_differ=differ,
                level_max_rel=max_rel, pixels=S * S,
                flips=int((m_lib[:2] != m_pin[:2]).any(axis=0).sum()),
                flips_4level=int((k_lib[:2] != k_pin[:2]).any(axis=0).sum()),
                subpix_max_abs=float(np.nanmax(np.abs(s_lib[:2] - s_pin[:2]))),
                score_max_abs=float(np.nanmax(np.abs(m_lib[2] - m_pin[2]))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--tiles', type=int, default=8)
    ap.add_argument('--c5-tiles', type=int, default=1)
    args = ap.parse_args()
    rows = []
    t0 = time.time()
    S = 128
    side = 9 * S + WS - 1
    a, b = stereo_pair(side, side, seed=1000, dx=2, max_disp=S // 4, sinusoidal=True)
    for i in range(args.tiles):
        r = c = i * S
        rows.append(compare(a[r:r + S + WS - 1, c:c + S + WS - 1], b[r:r + S + WS - 1, c:c + S + WS - 1],
                            S, 'C3 (%d,%d)' % (i, i)))
        print(json.dumps(rows[-1]), flush=True)
    S = 256
    if args.c5_tiles:
        side = 17 * S + WS - 1
        a, b = stereo_pair(side, side, seed=1000, dx=2, max_disp=S // 4, sinusoidal=True)
        for i in range(args.c5_tiles):
            r, c = 7 * S, (7 + i) * S
            rows.append(compare(a[r:r + S + WS - 1, c:c + S + WS - 1], b[r:r + S + WS - 1, c:c + S + WS - 1],
                                S, 'C5 (7,%d)' % (7 + i)))
            print(json.dumps(rows[-1]), flush=True)
    tot = {k: sum(r[k] for r in rows) for k in ('level_values', 'level_values_differ', 'pixels',
                                                 'flips', 'flips_4level')}
    for k in ('level_max_rel', 'subpix_max_abs', 'score_max_abs'):
        tot[k] = max(r[k] for r in rows)
    tot['value_frac'] = tot['level_values_differ'] / tot['level_values']
    tot['flip_rate'] = tot['flips'] / tot['pixels']
    out = {'what': 'pinned pow14 (dm_pow.h, the kernels) vs libm pow (numpy, the reference), '
                   'oracle streaming mode, levels >= 1 and Matching',
           'workload': '%d S=128 tiles of the C3 bench pair + %d S=256 tile(s) of the C5 pair, ws=%d'
                       % (args.tiles, args.c5_tiles, WS),
           'total': tot, 'tiles': rows, 'seconds': round(time.time() - t0, 1)}
    with open(os.path.join(REPO, 'profiles', 'pow_pin.json'), 'w') as f:
        json.dump(out, f, indent=1)
    print(json.dumps(tot))


if __name__ == '__main__':
    main()

"""How far does the pinned (kernel) ZNCC formula move level 0 and the matches, against
SURVEY.md 8(c)'s double-precision formula?  CPU only (the oracle), 8 C3 tiles (S = 128,
ws = 5, seeds 0-7 of the SURVEY 8(d) generator, sinusoidal disparity).

  pinned  y = f32(num) * f32(1/sqrt(f64 dI)); r = clamp(y * f32(1/sqrt(f64 dT)))   (kernels)
  f64div  r = f32(clamp(num / sqrt(f64 dT * f64 dI)))                             

Reports, per tile and in total: level-0 values (after min-max) that differ, their max
float32 ulp distance, NaN mismatches, and the integer correspondences (Matching without
sub-pixel) that flip, plus max |d| of the sub-pixel output.  Writes profiles/zncc_pin.json.

    python tools/zncc_pin.py [--tiles 8] [--tile 128]
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


def solve(a, b, ws, formula):
    O.set_zncc_formula(formula)
    try:
        lev, _, _ = O.pyramid_stream(a, b, ws)
        return O.match_stream(a, b, ws, lev, sub_pix=False), O.match_stream(a, b, ws, lev, sub_pix=True)
    finally:
        O.set_zncc_formula('pinned')


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--tiles', type=int, default=8)
    ap.add_argument('--tile', type=int, default=128)
    args = ap.parse_args()
    S, ws = args.tile, 5
    O.set_pow_mode('libm')
    rows, tot = [], {'voxels': 0, 'values': 0, 'max_ulp': 0, 'max_abs': 0.0, 'nan_mismatch': 0,
                     'pixels': 0, 'flips': 0, 'subpix_max_abs': 0.0}
    t0 = time.time()
    for seed in range(args.tiles):
        a, b = stereo_pair(S + ws - 1, S + ws - 1, seed=seed, dx=2, max_disp=S // 4, sinusoidal=True)
        d = O.zncc_formula_diff(a, b, ws)
        m0, s0 = solve(a, b, ws, 'pinned')
        m1, s1 = solve(a, b, ws, 'f64div')
        flips = int((m0[:2] != m1[:2]).any(axis=0).sum())
        sub = float(np.nanmax(np.abs(s0[:2] - s1[:2])))
        r = dict(seed=seed, voxels=S ** 4, **d, pixels=S * S, flips=flips, subpix_max_abs=sub)
        rows.append(r)
        print(json.dumps(r), flush=True)
        for k in ('voxels', 'values', 'nan_mismatch', 'pixels', 'flips'):
            tot[k] += r[k]
        tot['max_ulp'] = max(tot['max_ulp'], r['max_ulp'])
        tot['max_abs'] = max(tot['max_abs'], r['max_abs'])
        tot['subpix_max_abs'] = max(tot['subpix_max_abs'], sub)
    tot['value_frac'] = tot['values'] / tot['voxels']
    tot['flip_rate'] = tot['flips'] / tot['pixels']
    out = {'what': 'pinned two-multiply ZNCC vs SURVEY 8(c) f64-division ZNCC, oracle, libm pow',
           'workload': '%d tiles S=%d ws=%d, stereo_pair seeds 0..%d, sinusoidal' % (args.tiles, S, ws, args.tiles - 1),
           'total': tot, 'tiles': rows, 'seconds': round(time.time() - t0, 1)}
    with open(os.path.join(REPO, 'profiles', 'zncc_pin.json'), 'w') as f:
        json.dump(out, f, indent=1)
    print(json.dumps(tot))


if __name__ == '__main__':
    main()

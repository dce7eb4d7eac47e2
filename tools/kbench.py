"""Level-kernel timer on the C3 workload: dm_corr_level12 ('l12', level 2 fused) and/or
dm_corr_level1 ('l1'), interleaved rounds in one process (cdna_hip_programming.md section 5.4
rule 24).  Library builds are A/B'd with DM_LIB_PATH (tools/ab3.sh): the kernel variants are
a function of the shape, not of the environment.

    python tools/kbench.py [--variants l12,l1] [--rounds 5] [--tile 128] [--grid 8]
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deepmatching_stereo_matching_amd import _lib as L  # noqa: E402
from deepmatching_stereo_matching_amd import engine  # noqa: E402
from deepmatching_stereo_matching_amd.synthetic import stereo_pair  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--variants', default='l12')
    ap.add_argument('--rounds', type=int, default=5)
    ap.add_argument('--tile', type=int, default=128)
    ap.add_argument('--grid', type=int, default=8)
    ap.add_argument('--ws', type=int, default=5)
    ap.add_argument('--sha', action='store_true', help='print the sha256 of the whole first output')
    args = ap.parse_args()
    S, ws = args.tile, args.ws
    side = (args.grid + 1) * S + ws - 1
    a, b = stereo_pair(side, side, seed=1000, dx=2, max_disp=S // 4, sinusoidal=True)
    dev = torch.device('cuda', 0)
    n, org = engine.cut_grid(a.shape, [S, S], [S, S], ws)
    ia, ib = torch.from_numpy(a).to(dev), torch.from_numpy(b).to(dev)
    lib = L.load()
    P1 = (S // 2) ** 2
    res = {v: [] for v in args.variants.split(',')}
    outs, shas = {}, {}
    for rnd in range(args.rounds + 1):
        for v in res:
            fused = v == 'l12'       # dm_corr_level12 (level 2 fused, level 1 on chip); else level 1
            batch = engine.TileBatch(ia, ib, org, S, S, ws, L.DM_TM_CCOEFF_NORMED, dev)
            pyr = engine.DevicePyramid(batch, build=False).compute_stats()
            P2 = P1 // 4
            l1 = torch.empty((batch.T, P2, P2) if fused else (batch.T, P1, P1),
                             dtype=torch.float64, device=dev)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            if fused:
                L.check(lib.dm_corr_level12(batch.ref(), L.ptr(pyr.stats), None, L.ptr(l1),
                                            L.stream_handle()))
            else:
                L.check(lib.dm_corr_level1(batch.ref(), L.ptr(pyr.stats), L.ptr(l1),
                                           L.stream_handle()))
            e1.record()
            torch.cuda.synchronize()
            if rnd:
                res[v].append(e0.elapsed_time(e1))
            else:
                outs[v] = l1[:2].cpu().numpy()
                if args.sha:
                    import hashlib
                    shas[v] = hashlib.sha256(l1.cpu().numpy().tobytes()).hexdigest()[:16]
            del l1, pyr, batch
    ref = next(iter(outs.values()))
    for v, ts in res.items():
        same = outs[v].shape == ref.shape and np.array_equal(outs[v], ref, equal_nan=True)
        print('%-8s S=%d median %8.3f ms  min %8.3f ms  (%s)  bit-identical to %s: %s%s'
              % (v, S, np.median(ts), np.min(ts), ' '.join('%.2f' % t for t in ts),
                 next(iter(outs)), same, ('  sha256 ' + shas[v]) if v in shas else ''))


if __name__ == '__main__':
    main()

"""C5 strong-scaling forecast from one GPU (diagnostic; never a bench line).

bench.py --config c5 --gpus N shards one 4096^2 pair's 256 tiles round-robin over N ranks
(rank r solves tiles r::N), gathers each rank's (3, S, S) float64 results to rank 0 over
RCCL and rank 0 stitches the map (bench.py PairSolver.step, shard.gather_units_to).  The
driver measures N = 1..8 on an 8-GPU node; this tool measures on ONE GPU the parts that
decide the curve:
  - rank 0's share: the same pipelined solve (2 HIP streams, as bench.py) of tiles 0::N,
    timed over --steps steps after --warmup, for N = 1, 2, 4, 8;
  - rank 0's stitch of the whole map from the gathered (256, 3, S, S) results;
  - the gather itself is priced, not measured (one GPU has no xGMI peer): every peer sends
    its T/N tiles x 3 x S^2 x 8 B over its own link, at --link-gbs (default 50 GB/s, a third
    of the 153 GB/s per-link figure of MI355X_MICROARCH.md, so a pessimistic price).
forecast speed-up(N) = t(1) / (t_share(N) + t_stitch + t_gather(N)), where t(1) is the
one-rank step (which stitches too and gathers nothing).

  python3 tools/c5_share.py [--steps 6 --warmup 2] > gpurun_out/c5_share.json
"""

import argparse
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402
from deepmatching_stereo_matching_amd import engine  # noqa: E402
from deepmatching_stereo_matching_amd import _lib as L  # noqa: E402
from deepmatching_stereo_matching_amd.synthetic import stereo_pair  # noqa: E402


def timed_steps(solver, steps, warmup, stitch):
    """bench.py's pipelined loop for one solver: consecutive solves alternate over two
    streams, each solve's level kernel waits for the previous one's.  stitch: the solve ends
    in engine.stitch of this share (N = 1: the whole map, as bench.py's one-rank step)."""
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    prev = [None]
    k = [0]

    def one():
        st = streams[k[0] % 2]
        k[0] += 1
        with torch.cuda.stream(st):
            m = solver.compute(wait=prev[0])
            prev[0] = solver.last_end
            if stitch:
                engine.stitch(m, solver.n, solver.tile, solver.tile, [solver.tile, solver.tile],
                              ['elevation'])

    for _ in range(warmup):
        one()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        one()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=6)
    ap.add_argument('--warmup', type=int, default=2)
    ap.add_argument('--ranks', default='1,2,4,8')
    ap.add_argument('--link-gbs', type=float, default=50.0)
    args = ap.parse_args()
    tile, grid = bench.CONFIGS['c5']
    side = (grid + 1) * tile + bench.WS - 1
    a, b = stereo_pair(side, side, seed=1000, dx=2, max_disp=tile // 4, sinusoidal=True)
    dev = torch.device('cuda', 0)
    img1, img2 = torch.from_numpy(a).to(dev), torch.from_numpy(b).to(dev)
    full = bench.PairSolver(img1, img2, tile, grid)
    all_origins = full.origins
    T = len(all_origins)
    out = {'what': 'C5 strong-scaling forecast from one GPU (tools/c5_share.py): rank 0 share '
                   'measured, gather priced, stitch measured; diagnostic, not a bench line',
           'tiles': T, 'tile': tile, 'steps': args.steps, 'warmup': args.warmup,
           'link_gbs_assumed': args.link_gbs, 'shares': []}

    # rank 0's stitch of the whole map from the gathered results
    m = full.compute()
    torch.cuda.synchronize()
    ts = []
    for i in range(4):
        t0 = time.perf_counter()
        engine.stitch(m, full.n, tile, tile, [tile, tile], ['elevation'])
        torch.cuda.synchronize()
        if i:
            ts.append((time.perf_counter() - t0) * 1e3)
    t_stitch = sum(ts) / len(ts)
    out['stitch_full_ms'] = round(t_stitch, 3)
    del m

    t1 = None
    for n in [int(x) for x in args.ranks.split(',')]:
        s = bench.PairSolver(img1, img2, tile, grid)
        s.origins = all_origins[0::n]
        s.T = T
        s.batch = engine.TileBatch(img1, img2, s.origins, tile, tile, bench.WS,
                                   L.DM_TM_CCOEFF_NORMED, dev)
        ms = timed_steps(s, args.steps, args.warmup, stitch=(n == 1))
        rec = {'ranks': n, 'rank0_tiles': len(s.origins), 'rank0_solve_ms': round(ms, 3)}
        if n == 1:
            t1 = ms
            rec['step_ms'] = round(ms, 3)
        else:
            peer_bytes = len(s.origins) * 3 * tile * tile * 8
            t_gather = peer_bytes / (args.link_gbs * 1e9) * 1e3
            step = ms + t_gather + t_stitch
            rec.update({'gather_bytes_per_peer': peer_bytes, 'gather_ms_priced': round(t_gather, 3),
                        'step_ms_forecast': round(step, 3),
                        'speedup_forecast': round(t1 / step, 3) if t1 else None,
                        'share_efficiency': round(t1 / (n * ms), 4) if t1 else None})
        out['shares'].append(rec)
        print(json.dumps(rec), file=sys.stderr, flush=True)
        del s
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == '__main__':
    main()

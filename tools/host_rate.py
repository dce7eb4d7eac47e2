"""Is the pipelined bench host-bound?  Host enqueue time vs wall time per pair (diagnostic).

Runs bench.py's step loop (PairSolver on 2 HIP streams, each solve's level kernel waiting
for the previous one's) for --steps pairs and reports the host time spent issuing them
(before the final synchronize) next to the wall time.  When the two are equal the GPU waits
on the host (Python + ctypes issue of ~20 launches and the DevicePyramid allocations per
pair), and the per-pair time is the host's.

    python3 tools/host_rate.py --config c2 [--steps 40 --warmup 5]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='c2', choices=sorted(bench.CONFIGS))
    ap.add_argument('--steps', type=int, default=40)
    ap.add_argument('--warmup', type=int, default=5)
    args = ap.parse_args()
    tile, grid = bench.CONFIGS[args.config]
    side = (grid + 1) * tile + bench.WS - 1
    a, b = bench.stereo_pair(side, side, seed=1000, dx=2, max_disp=tile // 4, sinusoidal=True)
    dev = torch.device('cuda', 0)
    img1, img2 = torch.from_numpy(a).to(dev), torch.from_numpy(b).to(dev)
    s = bench.PairSolver(img1, img2, tile, grid)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    prev = [None]
    k = [0]

    def one():
        s.step(stream=streams[k[0] % 2], wait=prev[0])
        prev[0] = s.last_end
        k[0] += 1

    for _ in range(args.warmup):
        one()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        one()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    rec = {'config': args.config, 'steps': args.steps,
           'host_issue_ms_per_pair': round((t1 - t0) / args.steps * 1e3, 4),
           'wall_ms_per_pair': round((t2 - t0) / args.steps * 1e3, 4)}
    # the issue cost of one solve's pieces, host side only (GPU work left to run)
    torch.cuda.synchronize()
    parts = {}
    for name, fn in (('compute', lambda: s.compute()),):
        ts = []
        for _ in range(10):
            torch.cuda.synchronize()
            u0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - u0)
        parts[name] = round(sorted(ts)[len(ts) // 2] * 1e3, 4)
    torch.cuda.synchronize()
    rec['host_issue_ms_median'] = parts
    print(json.dumps(rec))


if __name__ == '__main__':
    main()

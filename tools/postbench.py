"""Post-processing timer: the Gauss-Seidel loops of
misc/optimize_loop.py and misc/opt_loop.py on an IGARSS-sized disparity map (the driver's
`allowed_error` default is sized for 1000 x 1000, optimize_looper.py:33), on the GPU through
the mirrors with device-resident tensors, next to the sequential C oracle on one host core.

    python tools/postbench.py [--side 1024] [--exclusion 3] [--reps 5]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deepmatching_stereo_matching_amd import _lib as L  # noqa: E402
from deepmatching_stereo_matching_amd import postproc  # noqa: E402
from deepmatching_stereo_matching_amd.misc import opt_loop as M  # noqa: E402
from deepmatching_stereo_matching_amd.misc import optimize_loop as OL  # noqa: E402


def gpu_ms(fn, reps):
    st = torch.cuda.current_stream()
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(reps):
        e0.record(st)
        fn()
        e1.record(st)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return float(np.median(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--side', type=int, default=1024)
    ap.add_argument('--exclusion', type=int, default=3)
    ap.add_argument('--reps', type=int, default=5)
    ap.add_argument('--no-cpu', action='store_true')
    a = ap.parse_args()
    n, e = a.side, a.exclusion
    rng = np.random.default_rng(0)
    y, x = np.mgrid[0:n, 0:n]
    guide = 5 + 4 * np.sin(x / 37.0) * np.cos(y / 23.0) + rng.normal(0, 0.5, (n, n))
    coef = rng.uniform(0.2, 1.5, (n, n))
    sigma = np.array([5, 5])
    dev = torch.device('cuda', 0)
    tg, tc = torch.from_numpy(guide).to(dev), torch.from_numpy(coef).to(dev)
    size = (n, n)
    g, c = M.make_weight(tg, e, size, sigma)
    img = tg.clone()
    upd = (n - 2 * e - 1) ** 2
    # schedules are built once per shape (host C++), then cached on the device
    t0 = time.perf_counter()
    postproc.schedule(L.DM_GS_BILAT, n, n, n, n, e, dev)
    postproc.schedule(L.DM_GS_FWD4, n, n, n, n, 1, dev)
    postproc.schedule(L.DM_GS_BWD4, n, n, n, n, 1, dev)
    sched_ms = (time.perf_counter() - t0) * 1e3
    res = {
        'side': n, 'exclusion': e, 'updates_per_sweep': upd,
        'levels': {'bilat': postproc.schedule(L.DM_GS_BILAT, n, n, n, n, e, dev)[2],
                   'fwd4': postproc.schedule(L.DM_GS_FWD4, n, n, n, n, 1, dev)[2],
                   'bwd4': postproc.schedule(L.DM_GS_BWD4, n, n, n, n, 1, dev)[2]},
        'schedule_build_ms_host': round(sched_ms, 1),
        'gpu_ms': {
            'make_weight': gpu_ms(lambda: M.make_weight(tg, e, size, sigma), a.reps),
            'bilateral_horizon_sweep': gpu_ms(lambda: M.optimize_loop_bilateral_horizon(img, c, g, tc, 0.008, e, size),
                                              a.reps),
            'optimize_loop_e1': gpu_ms(lambda: OL.optimize_loop(img, tc, 0.008, 1, size), a.reps),
        },
    }
    if not a.no_cpu:
        from oracle import oracle as O
        t0 = time.perf_counter()
        og, oc = O.make_weight(guide, e, size, sigma)
        t1 = time.perf_counter()
        O.opt_loop_bilateral(guide, oc, og, coef, e, size, False)
        t2 = time.perf_counter()
        O.optimize_loop(guide, coef, 0.008, 1, size)
        t3 = time.perf_counter()
        res['cpu_oracle_ms_1core'] = {'make_weight': round((t1 - t0) * 1e3, 1),
                                      'bilateral_horizon_sweep': round((t2 - t1) * 1e3, 1),
                                      'optimize_loop_e1': round((t3 - t2) * 1e3, 1)}
    print(json.dumps(res))


if __name__ == '__main__':
    main()

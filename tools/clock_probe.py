"""In-kernel clock of the level kernel under a sustained load (MI355X_MICROARCH.md 'DVFS
give-back' item 6; cdna_hip_programming.md section 5.4 rule 28): back-to-back launches of
dm_corr_level12 on bench.py's pair for --seconds, HIP events around each, then the
per-workgroup stamps of the last launch (a DM_CLOCK_STAMP=1 build: tools/abl_build.sh clk, loaded
through DM_LIB_PATH) give the shader clock while the kernel ran: d(s_memtime) / d(realtime) x
100 MHz per workgroup, median over workgroups.  With the kernel's modelled issue cycles
(profiles/pmc_level1*.json, tools/issue_model.py) that gives the issue occupancy at the clock
the chip actually held: issue cycles / (1024 SIMDs x clock x live time).

    DM_LIB_PATH=ab/libdm_clk.so python tools/clock_probe.py [--tile 128 --grid 8] [--seconds 3]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from deepmatching_stereo_matching_amd import _lib as L  # noqa: E402
from deepmatching_stereo_matching_amd import engine  # noqa: E402
from deepmatching_stereo_matching_amd.synthetic import stereo_pair  # noqa: E402

PMC = {128: 'pmc_level1.json', 64: 'pmc_level1_s64.json', 256: 'pmc_level1_s256.json'}
NB = {128: 2, 64: 4, 256: 1}      # cell blocks per workgroup (DM_C3_NB, DM_C2_NB, DM_C5_NB)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--tile', type=int, default=128)
    ap.add_argument('--grid', type=int, default=8)
    ap.add_argument('--seconds', type=float, default=3.0)
    args = ap.parse_args()
    S, ws = args.tile, 5
    side = (args.grid + 1) * S + ws - 1
    a, b = stereo_pair(side, side, seed=1000, dx=2, max_disp=S // 4, sinusoidal=True)
    dev = torch.device('cuda', 0)
    n, org = engine.cut_grid(a.shape, [S, S], [S, S], ws)
    ia, ib = torch.from_numpy(a).to(dev), torch.from_numpy(b).to(dev)
    lib = L.load()
    fn = getattr(lib, 'dm_diag_clock_stamps', None)
    if fn is None:
        raise SystemExit('this library has no clock stamps: build tools/abl_build.sh clk and set DM_LIB_PATH')
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    fn.restype = ctypes.c_int
    batch = engine.TileBatch(ia, ib, org, S, S, ws, L.DM_TM_CCOEFF_NORMED, dev)
    pyr = engine.DevicePyramid(batch, build=False).compute_stats()
    P2 = (S // 4) ** 2
    l2 = torch.empty((batch.T, P2, P2), dtype=torch.float64, device=dev)
    nwg = batch.T * (S // 4) * (S // 4) // NB[S]
    assert nwg <= 65536, nwg
    times = []
    t_end = time.time() + args.seconds
    while True:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        L.check(lib.dm_corr_level12(batch.ref(), L.ptr(pyr.stats), None, L.ptr(l2), L.stream_handle()))
        e1.record()
        times.append((e0, e1))
        if time.time() > t_end and len(times) >= 8:
            break
        if len(times) % 16 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    ms = [x.elapsed_time(y) for x, y in times]
    st = np.zeros(4 * nwg, dtype=np.uint64)
    L.check(fn(st.ctypes.data, nwg))
    st = st.reshape(nwg, 4).astype(np.float64)
    dt, dr = st[:, 1] - st[:, 0], st[:, 3] - st[:, 2]
    ok = dr > 0
    clk = dt[ok] / dr[ok] * 0.1          # GHz: the real-time counter runs at 100 MHz
    rec = {'tile': S, 'tiles': int(batch.T), 'launches': len(ms), 'seconds': args.seconds,
           'last_ms': round(ms[-1], 4), 'median_ms_last_quarter': round(float(np.median(ms[-max(1, len(ms) // 4):])), 4),
           'workgroups': nwg, 'stamped': int(ok.sum()),
           'clock_ghz_median': round(float(np.median(clk)), 4),
           'clock_ghz_p10_p90': [round(float(np.percentile(clk, 10)), 4), round(float(np.percentile(clk, 90)), 4)],
           'workgroup_us_median': round(float(np.median(dr[ok])) / 100.0, 2)}
    path = os.path.join(REPO, 'profiles', PMC[S])
    if os.path.exists(path):
        d = json.load(open(path))
        cyc = d.get('issue_cycles_per_launch')
        if cyc:
            cyc = cyc * batch.T / d.get('tiles', batch.T)     # the profile's launch may hold more tiles
            t = rec['median_ms_last_quarter'] * 1e-3
            rec['issue_cycles_per_launch'] = cyc
            rec['issue_occupancy_at_in_kernel_clock'] = round(cyc / (1024 * rec['clock_ghz_median'] * 1e9 * t), 4)
            rec['note'] = ('modelled issue cycles of the in-tree ISA; this build adds the stamp '
                           'instructions at workgroup start and end only')
    print(json.dumps(rec))


if __name__ == '__main__':
    main()

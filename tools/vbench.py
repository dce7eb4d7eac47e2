"""Volume-kernel timer: dm_corr_volume on the C3 batch (or --tiles of it), interleaved rounds;
--f16 times the binary16 volume (dm_corr_volume_f16).  Library builds are A/B'd with
DM_LIB_PATH (tools/ab3.sh); "+VAR=value" suffixes of a variant name set environment
variables for that variant (none of the volume kernels reads one any more).

    python tools/vbench.py [--rounds 3] [--tiles 32] [--f16] [--mm]
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

KNOBS = ()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--variants', default='ls')
    ap.add_argument('--rounds', type=int, default=3)
    ap.add_argument('--tile', type=int, default=128)
    ap.add_argument('--tiles', type=int, default=32)
    ap.add_argument('--f16', action='store_true', help='time dm_corr_volume_f16 (binary16, 2 B/voxel)')
    ap.add_argument('--mm', action='store_true',
                    help='min/max already in the stats (one untimed standalone launch first), timed with '
                         'dm_corr_volume_ex(DM_VOLUME_MINMAX_KNOWN)')
    ap.add_argument('--checksum', action='store_true', help='print a checksum of the volume bits')
    args = ap.parse_args()
    S, ws = args.tile, 5
    side = 9 * S + ws - 1
    a, b = stereo_pair(side, side, seed=1000, dx=2, max_disp=S // 4, sinusoidal=True)
    dev = torch.device('cuda', 0)
    n, org = engine.cut_grid(a.shape, [S, S], [S, S], ws)
    org = org[:args.tiles]
    ia, ib = torch.from_numpy(a).to(dev), torch.from_numpy(b).to(dev)
    lib = L.load()
    batch = engine.TileBatch(ia, ib, org, S, S, ws, L.DM_TM_CCOEFF_NORMED, dev)
    pyr = engine.DevicePyramid(batch, build=False).compute_stats()
    vol = torch.empty((batch.T, batch.P, batch.P), dtype=torch.float16 if args.f16 else torch.float32, device=dev)
    fn = lib.dm_corr_volume_f16 if args.f16 else lib.dm_corr_volume
    if args.mm:
        L.check(fn(batch.ref(), L.ptr(pyr.stats), L.ptr(vol), L.stream_handle()))
        flags = (L.DM_VOLUME_F16 if args.f16 else 0) | L.DM_VOLUME_MINMAX_KNOWN

        def fn(b_, st_, v_, s_):   # noqa: F811
            return lib.dm_corr_volume_ex(b_, st_, flags, v_, s_)
    res = {v: [] for v in args.variants.split(',')}
    for rnd in range(args.rounds + 1):
        for v in res:
            for k in KNOBS:
                os.environ.pop(k, None)
            for kv in v.split('+')[1:]:
                k, val = kv.split('=')
                os.environ[k] = val
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            L.check(fn(batch.ref(), L.ptr(pyr.stats), L.ptr(vol), L.stream_handle()))
            e1.record()
            torch.cuda.synchronize()
            if rnd:
                res[v].append(e0.elapsed_time(e1))
    gb = vol.element_size() * vol.numel() / 1e9
    for v, ts in res.items():
        print('%-24s median %8.3f ms  %7.1f GB/s' % (v, np.median(ts), gb / (np.median(ts) * 1e-3)))
    if args.checksum:
        # position-weighted checksum of the last volume's bits, tile by tile on the device: library
        # builds that A/B a kernel variant print the same value iff their volumes are bit-identical
        bits = vol.view(torch.int16 if args.f16 else torch.int32).reshape(vol.shape[0], -1)
        CH = 1 << 26   # elements per chunk (an S = 256 tile holds 2^32)
        base = torch.arange(CH, device=dev, dtype=torch.int64)
        acc = 0
        for t in range(bits.shape[0]):
            for o in range(0, bits.shape[1], CH):
                part = bits[t, o:o + CH].to(torch.int64)
                w = (base[:part.numel()] + (o + 1)) % 1000003
                acc = (acc * 1000033 + int((part * w).sum())) % (1 << 61)
        print('volume checksum %016x' % acc)


if __name__ == '__main__':
    main()

"""Benchmark: correlation-volume G-voxels/s and ms per stereo pair (BASELINE.json metric).

Workload (BASELINE.json configs[2], "C3"): a synthetic 1024x1024 stereo pair (input
1156x1156, so ImageCutSolver's floor rule yields 8x8 tiles of S = 128 = "d"), window 5,
the reference's full 8-level pyramid, backtracking, sub-pixel refinement, elevation
cal_map and stitching -- i.e. ImageCutSolver(img1, img2, image_size=[128,128],
stride=[128,128], window_size=5)() on the GPU.  One step = one pair; inputs are
resident in HBM before the timed region.  V = 64 tiles x 128^4 = 17.18 G voxels/pair.

Multi-GPU (one process per GPU, torch.distributed; `--gpus N` without WORLD_SIZE in the
environment launches N ranks itself through torch.distributed.run before touching the GPU):
  c2/c3  every rank solves its own pair per step (pairs are independent: weak scaling, no
         collective on the data path);
  c4     BASELINE configs[3]: one step is a batch of 64 independent pairs, rank r solves
         pairs r::N (strong scaling over the fixed batch; no collective);
  c5     one 4096^2 pair per step, its 256 tiles sharded over the ranks, results
         all-gathered (RCCL over xGMI) and stitched (strong scaling).
Timing is barrier + synchronize bracketed, max over ranks.  Consecutive pair solves are
pipelined over 2 HIP streams (--streams): a solve's level kernel waits for the previous
solve's level kernel, and the previous pair's latency-bound tail (levels >= 3, matching,
stitch) runs beside it; every step still solves its pair completely inside the timed region.

Also reported: the roofline of the dominant kernel (dm_corr_level12), timed with HIP
events on the launch stream inside the timed steps, the HBM roofline of the level-0
volume kernel (dm_corr_volume, 4 B/voxel written, and its fp16 variant, 2 B/voxel) on the
same batch, the fp16 volume's argmax flip rate, and the CPU oracle's rate on a bounded
sample (rank 0, N=1).
"""

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from deepmatching_stereo_matching_amd import _lib as L  # noqa: E402
from deepmatching_stereo_matching_amd import engine  # noqa: E402
from deepmatching_stereo_matching_amd.synthetic import stereo_pair  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
WS = 5
S = 128
GRID = 8
CONFIGS = {'c2': (64, 8), 'c3': (128, 8), 'c4': (128, 8), 'c5': (256, 16)}   # (tile S, tiles per axis)
C4_PAIRS = 64                  # BASELINE configs[3]: a batch of 64 independent 1024^2 pairs
# Rehearsal of the multi-rank path on a box with fewer GPUs than ranks (tests/test_bench_ranks.py):
# DM_BENCH_BACKEND=gloo and DM_BENCH_ONE_DEVICE=1 put every rank on cuda:0 over gloo.  The
# driver's runs leave both unset: one rank per GPU over RCCL ("nccl").
BACKEND = os.environ.get('DM_BENCH_BACKEND', 'nccl')
ONE_DEVICE = os.environ.get('DM_BENCH_ONE_DEVICE', '0') == '1'
VOLUME_BUDGET = 72e9           # bytes of level-0 volume materialised for its roofline: the whole
                               # C3 batch in float32 (68.7 GB), 8 S=256 tiles in fp16 (whole
                               # rounds of workgroups over the chip, as C5's 256 tiles are)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=5)   # the clock settles after ~3 launches
    ap.add_argument('--streams', type=int, default=2,
                    help='HIP streams consecutive pair solves are pipelined over (1: no overlap)')
    ap.add_argument('--config', choices=sorted(CONFIGS), default='c3',
                    help='BASELINE.json configs: c2 (512^2, S=64), c3 (1024^2, S=128; the metric), '
                         'c4 (64 pairs of c3 per step, sharded over the ranks), c5 (4096^2, S=256)')
    ap.add_argument('--pairs', type=int, default=C4_PAIRS, help='c4: pairs per step (whole job)')
    ap.add_argument('--tile', type=int, default=None)
    ap.add_argument('--grid', type=int, default=None)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--cpu-sample-tiles', type=int, default=16)
    ap.add_argument('--no-volume', action='store_true')
    return ap.parse_args()


class PairSolver:
    """One ImageCutSolver-equivalent pass over a resident pair, with event timing of the
    dominant kernel (dm_corr_level12)."""

    def __init__(self, img1, img2, tile, grid, split=False):
        """split: the pair's tiles are sharded over the ranks (rank r solves tiles r::N) and
        the per-tile results are all-gathered before stitching (RCCL over xGMI); otherwise
        this rank solves every tile of its own pair."""
        from deepmatching_stereo_matching_amd import shard
        self.dev = img1.device
        self.tile = tile
        self.n, origins = engine.cut_grid(tuple(img1.shape), [tile, tile], [tile, tile], WS)
        assert self.n == [grid, grid], self.n
        self.rank, self.world = shard.world() if split else (0, 1)
        self.T = len(origins)
        self.origins = origins[shard.rank_units(self.T, self.rank, self.world)]
        self.batch = engine.TileBatch(img1, img2, self.origins, tile, tile, WS,
                                      L.DM_TM_CCOEFF_NORMED, self.dev)
        self.ev = []

    def step(self, timed=False, stream=None, wait=None):
        """One full solve of the pair on `stream` (default: the current stream).  Every
        device buffer belongs to this step's DevicePyramid, so steps on different streams
        share only the read-only images.  `wait`: event the level kernel waits for (the
        previous solve's level-kernel end when solves are pipelined over streams); this
        solve's level-kernel end is left in self.last_end."""
        if stream is not None:
            with torch.cuda.stream(stream):
                return self.step(timed=timed, wait=wait)
        from deepmatching_stereo_matching_amd import shard
        pyr = engine.DevicePyramid(self.batch, build=False)
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        if timed:
            self.ev.append(ev)
        self.last_end = ev[1]
        pyr.build(events=ev, wait=wait)    # stats, dm_corr_level12 [timed], dm_aggregate levels 3..
        match = pyr.match(sub_pix=True)
        if self.world > 1:
            match = shard._gather_units(match, self.T, self.rank, self.world, match.shape[1:], match.dtype)
        dmap, score = engine.stitch(match, self.n, self.tile, self.tile, [self.tile, self.tile],
                                    ['elevation'])
        return dmap, score

    def level1_ms(self):
        return float(np.mean([a.elapsed_time(b) for a, b in self.ev])) if self.ev else None


def volume_roofline(solver, reps=3, f16=False):
    """HBM roofline of the level-0 volume kernel on the same batch: dm_corr_volume (co_map,
    float32, 4 B per voxel written) or, with f16, the fp16 volume of
    BASELINE config C5 (dm_corr_volume_f16, 2 B per voxel written)."""
    full = solver.batch
    esz = 2 if f16 else 4
    nt = max(1, min(full.T, int(VOLUME_BUDGET // (float(esz) * full.P * full.P))))
    batch = engine.TileBatch(full.img1, full.img2, full.origins_host[:nt], full.h0, full.w0, full.ws,
                             full.method, full.device)
    pyr = engine.DevicePyramid(batch, build=False)
    pyr.compute_stats()
    vol = torch.empty((batch.T, batch.P, batch.P), dtype=torch.float16 if f16 else torch.float32,
                      device=batch.device)
    fn = pyr.lib.dm_corr_volume_f16 if f16 else pyr.lib.dm_corr_volume
    ts = []
    for i in range(reps + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        L.check(fn(batch.ref(), L.ptr(pyr.stats), L.ptr(vol), L.stream_handle()))
        e1.record()
        torch.cuda.synchronize()
        if i:
            ts.append(e0.elapsed_time(e1))
    ms = float(np.mean(ts))
    voxels = batch.T * batch.P * batch.P
    gbs = esz * voxels / (ms * 1e-3) / 1e9
    del vol, pyr
    torch.cuda.empty_cache()
    name = 'dm_corr_volume_f16 (k_volume_ls, binary16)' if f16 else 'dm_corr_volume (k_volume_ls)'
    return {'kernel': name, 'tiles': batch.T, 'tile': batch.h0,
            'ms': round(ms, 3), 'gvox_s': round(voxels / (ms * 1e-3) / 1e9, 1),
            'algorithmic_bytes_per_voxel': esz, 'bound': 'hbm',
            'achieved': round(gbs, 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
            'frac': round(gbs / HBM_PEAK_GBS, 4),
            'traffic': load_traffic(batch.h0, 'volume_f16' if f16 else 'volume')}


def fp16_flip_rate(solver, tiles=2):
    """Argmax flip rate of the fp16-volume pyramid (dm_corr_volume_f16 -> rectify ->
    aggregate -> match) against the float32 path on `tiles` tiles of the workload: the
    fraction of pixels whose integer correspondence differs (C5 fp16 has no
    bit-exact claim, its flip rate is reported)."""
    full = solver.batch
    flips, n = 0, 0
    for t in range(min(tiles, full.T)):   # one tile at a time: its float64 level 0 is 8 B/voxel
        one = engine.TileBatch(full.img1, full.img2, full.origins_host[t:t + 1], full.h0, full.w0,
                               full.ws, full.method, full.device)
        pyr = engine.DevicePyramid(one)
        ref = pyr.match(sub_pix=False)
        lv = pyr.materialized_levels('f16')
        m16 = pyr.match(sub_pix=False, levels=lv)
        flips += int((m16[:, :2] != ref[:, :2]).any(dim=1).sum())
        n += one.P
        del lv, pyr
        torch.cuda.empty_cache()
    return {'tiles': tiles, 'tile': full.h0, 'pixels': n, 'flipped': flips,
            'rate': round(flips / n, 6)}


def cpu_baseline(tiles, tile):
    """The CPU oracle (port of the reference pipeline, OpenMP) on `tiles` tiles of the same
    workload: corr_l0 + pyramid (libm pow) + matching + sub-pixel."""
    from oracle import oracle as O
    a, b = stereo_pair(tile + WS - 1, tiles * tile + WS - 1, seed=1000, dx=2)
    O.set_pow_mode('libm')
    t0 = time.perf_counter()
    for k in range(tiles):
        c0 = k * tile
        l0 = O.corr_l0(a[:, c0:c0 + tile + WS - 1], b[:, c0:c0 + tile + WS - 1], WS)
        levels, _, _ = O.pyramid(l0)
        O.match(levels, sub_pix=True)
        del l0, levels
    dt = time.perf_counter() - t0
    vox = tiles * float(tile) ** 4
    cores = int(os.environ.get('OMP_NUM_THREADS', os.cpu_count() or 1))
    return {'value': round(vox / dt / 1e9, 5), 'unit': 'Gvox/s', 'cores': cores, 'kind': 'port',
            'sample': '%d tiles of S=%d (%.2f G voxels) of the same workload, oracle/dm_oracle.c '
                      '(OpenMP), %.2f s' % (tiles, tile, vox / 1e9, dt),
            # the reference's own Python cannot run on the GPU box (OpenCV and absl are absent
            # from the image); SURVEY.md section 6 timed it in the survey container
            'reference_python': {'value': 0.021, 'unit': 'Gvox/s', 'cores': 8,
                                 'sample': 'one S=128 tile, 12.95 s, reference misc/*.py with the '
                                           'repo cv2 shim, 8-core Xeon (SURVEY.md section 6)'}}


def load_pmc(tile, kernel='level1'):
    """Per-launch PMC figures of a kernel from the committed rocprofv3 passes
    (profiles/pmc_<kernel>.json, tools/profile.sh): HBM bytes (FETCH_SIZE x2 gfx950
    correction + WRITE_SIZE) and, for the level kernel, VALU instructions."""
    path = os.path.join(REPO, 'profiles', 'pmc_%s.json' % kernel)
    try:
        with open(path) as f:
            d = json.load(f)
        if d.get('tile') == tile:
            return d
    except (OSError, ValueError):
        pass
    return {}


def load_traffic(tile, kernel='level1'):
    return load_pmc(tile, kernel).get('hbm_bytes_per_launch')


def level_roofline(solver, tile, l1_ms):
    """Roofline of the dominant kernel, dm_corr_level12 (k_level1_mfq): levels 0 -> 1 -> 2 in
    one pass, level 0 and level 1 never leave the chip.

    It is compute-bound: its physical HBM traffic (PMC, ~1.24 GB per C3 launch) is ~1.5 % of
    what the bandwidth would allow in its run time.  The bound is the vector ALU (float32
    normalisation, float64 pow14 of every pooled child value), so `achieved` / `peak` are
    VALU-busy SIMD-cycles per second against 1024 SIMDs x the clock the kernel ran at, both
    from a committed rocprofv3 --pmc pass (profiles/pmc_level1.json, tools/pmc_valu.sh):
    SQ_ACTIVE_INST_VALU (quad-cycles) x 4 per launch over the live HIP-event time, and the
    effective clock GRBM_GUI_ACTIVE / 8 XCDs / profiled kernel time.  The 4 B/voxel figure of
    SURVEY.md 8(d) (the level-0 volume this kernel does not write) is kept as
    `hbm_equivalent`."""
    vox_launch = solver.batch.T * float(tile) ** 4   # this rank's tiles per launch
    gbs = 4.0 * vox_launch / (l1_ms * 1e-3) / 1e9
    mode = int(os.environ.get('DM_FUSE_L2', str(engine.FUSE_DEFAULT)))
    kname = ('dm_corr_level1 (k_level1_mfq)' if mode == 0
             else 'dm_corr_level12 (k_level1_mfq, level 2 fused)')
    pmc = load_pmc(tile) if solver.batch.T == 64 else {}
    roof = {'kernel': kname, 'bound': 'valu', 'ms': round(l1_ms, 3)}
    busy, cyc = pmc.get('valu_active_cycles_per_launch'), pmc.get('gpu_cycles_per_launch')
    if busy and cyc:
        # the launch's cycle count is taken from the PMC pass (the kernel is deterministic); the
        # live time then gives the clock it ran at in this run, so achieved / peak is the
        # measured VALU-busy fraction
        achieved = busy / (l1_ms * 1e-3) / 1e9          # G SIMD-cycles/s with the VALU busy
        peak = 1024 * cyc / (l1_ms * 1e-3) / 1e9
        roof.update({'achieved': round(achieved, 1), 'peak': round(peak, 1),
                     'unit': 'G VALU-busy SIMD-cycles/s', 'frac': round(achieved / peak, 4),
                     'valu_busy_source': 'SQ_ACTIVE_INST_VALU x4 (one quad-cycle per wave64 VALU '
                                         'instruction) per launch over 1024 SIMDs x GRBM_GUI_ACTIVE/8 '
                                         'cycles per launch, rocprofv3 --pmc (profiles/pmc_level1.json)'})
        for k in ('ta_busy_frac', 'td_busy_frac'):
            if k in pmc:
                roof[k] = pmc[k]
    else:
        roof.update({'achieved': None, 'peak': None, 'unit': 'G VALU-busy SIMD-cycles/s',
                     'frac': None, 'valu_busy_source': 'no PMC pass for this batch shape'})
    if pmc.get('valu_insts_per_launch'):
        # issue-limited estimate: a wave64 VALU instruction occupies a 32-lane SIMD >= 2 cycles
        roof['valu_insts_per_launch'] = pmc['valu_insts_per_launch']
    roof['traffic'] = load_traffic(tile) if pmc else None
    roof['hbm_equivalent'] = {'achieved': round(gbs, 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                              'frac': round(gbs / HBM_PEAK_GBS, 4),
                              'algorithmic': '4 B/voxel x %d level-0 voxels per launch (never '
                                             'written: the volume a materialising kernel would '
                                             'store)' % int(vox_launch)}
    return roof


def launch_ranks(args):
    """`bench.py --gpus N` (N > 1) started without a torch.distributed environment: run
    N ranks (one per GPU) under torch.distributed.run as a CHILD process and return its exit
    status.  This process has not initialised the GPU (torch.cuda.device_count() does not on
    this image), and it never exec()s."""
    import socket
    import subprocess
    n = torch.cuda.device_count()
    if n < args.gpus and not ONE_DEVICE:
        raise SystemExit('bench.py --gpus %d: only %d GPU(s) visible' % (args.gpus, n))
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1',
           '--nproc-per-node', str(args.gpus), '--master-addr', '127.0.0.1',
           '--master-port', str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def make_pairs(args, tile, grid, rank, world):
    """Synthetic input pairs of this rank (SURVEY.md 8(d) generator; seed 1000 + pair index)
    -> (list of (img1, img2) host arrays, pair indices, pairs per step for the whole job)."""
    # ImageCutSolver's floor rule (image_cut_solver.py:62): floor((side - (tile+ws-1)) / tile)
    # tiles per axis, so a grid x grid cut needs side = (grid+1)*tile + ws-1 (1156 for C3)
    side = (grid + 1) * tile + WS - 1
    if args.config == 'c4':
        from deepmatching_stereo_matching_amd import shard
        idx = shard.rank_units(args.pairs, rank, world)
        job_pairs = args.pairs
    elif args.config == 'c5' and world > 1:
        idx, job_pairs = [0], 1       # one pair, tiles split over the ranks
    else:
        idx, job_pairs = [rank], world
    pairs = [stereo_pair(side, side, seed=1000 + i, dx=2, max_disp=tile // 4, sinusoidal=True)
             for i in idx]
    return pairs, idx, job_pairs


def main():
    args = parse()
    if args.gpus > 1 and 'WORLD_SIZE' not in os.environ:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world != args.gpus:
        raise SystemExit('bench.py --gpus %d but WORLD_SIZE=%d' % (args.gpus, world))
    dist = world > 1
    if ONE_DEVICE:   # rehearsal of the multi-rank path on a one-GPU box (tests only)
        local = 0
    if dist:
        import torch.distributed as tdist
        torch.cuda.set_device(local)
        if BACKEND == 'nccl':
            tdist.init_process_group('nccl', device_id=torch.device('cuda', local))
        else:
            tdist.init_process_group(BACKEND)
    dev = torch.device('cuda', local if dist else 0)
    torch.cuda.set_device(dev)
    joined = world
    if dist:   # ranks that actually joined the job
        j = torch.ones(1, dtype=torch.int64, device=dev)
        tdist.all_reduce(j)
        joined = int(j.item())
        if joined != args.gpus:
            raise SystemExit('bench.py --gpus %d: %d ranks joined' % (args.gpus, joined))

    tile, grid = CONFIGS[args.config]
    tile, grid = args.tile or tile, args.grid or grid
    # c5 (BASELINE configs[4]): ONE pair per step, its tiles sharded over the ranks (strong
    # scaling, results all-gathered); c4: a fixed batch of pairs split over the ranks
    # (strong scaling); c2/c3: one pair per rank per step (weak scaling)
    split = args.config == 'c5' and world > 1
    host_pairs, pair_idx, job_pairs = make_pairs(args, tile, grid, rank, world)
    solvers = []
    for a, b in host_pairs:
        img1, img2 = torch.from_numpy(a).to(dev), torch.from_numpy(b).to(dev)
        solvers.append(PairSolver(img1, img2, tile, grid, split=split))
    del host_pairs
    solver = solvers[0] if solvers else None
    voxels = grid * grid * float(tile) ** 4      # per pair

    # --streams S: consecutive pair solves go to S HIP streams round-robin, pipelined: each
    # solve's level kernel waits for the previous solve's level kernel (so level kernels never
    # share the GPU with each other and each one's event time stays its own), while the
    # previous pair's latency-bound tail (levels >= 3, matching on demand, stitch: ~5 % of a
    # solve) runs beside it.  Each solve still solves its pair completely.
    # c5 split over ranks all-gathers inside every solve: its collectives stay on one stream
    # (RCCL operations of one communicator must not race each other on two streams)
    nstreams = 1 if split else max(1, args.streams)
    streams = [torch.cuda.Stream(device=dev) for _ in range(nstreams)] if nstreams > 1 else [None]
    nsolve = [0]
    prev_end = [None]

    def step(timed=False):
        for s in solvers:
            st = streams[nsolve[0] % len(streams)]
            nsolve[0] += 1
            s.step(timed=timed, stream=st, wait=prev_end[0] if st is not None else None)
            prev_end[0] = s.last_end

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if dist:
        tdist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(timed=True)
    torch.cuda.synchronize()
    if dist:
        tdist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        elapsed = float(t.item())

    ms_step = elapsed / args.steps * 1e3
    value = job_pairs * args.steps * voxels / elapsed / 1e9
    l1_ms = solver.level1_ms() if solver else None
    if rank == 0 and solver is None:
        raise SystemExit('rank 0 has no pairs (--pairs < --gpus)')
    if rank == 0:
        roof = level_roofline(solver, tile, l1_ms)
        if args.config == 'c4':
            workload = ('C4: batch of %d independent %dx%d pairs per step (%dx%d tiles of S=%d each), '
                        'ws=%d, full pyramid + sub-pixel + cal_map + stitch'
                        % (job_pairs, grid * tile, grid * tile, grid, grid, tile, WS))
            per_gpu, par = job_pairs / float(world), 'pairs of the batch sharded %d-way' % world
        else:
            workload = ('%s: %dx%d pair, %dx%d tiles of S=%d, ws=%d, full pyramid '
                        '+ sub-pixel + cal_map + stitch'
                        % (args.config.upper(), grid * tile, grid * tile, grid, grid, tile, WS))
            per_gpu = (1.0 / world) if split else 1
            par = ('tiles of one pair sharded %d-way' if split else 'pairs sharded %d-way') % world
        rec = {'metric': 'correlation-volume G-voxels/sec + ms/stereo-pair @1/8 GPU, 1024^2 d=128',
               'value': round(value, 3), 'unit': 'Gvox/s', 'n_gpus': joined, 'steps': args.steps,
               'warmup': args.warmup, 'ms_per_step': round(ms_step, 3),
               'ms_per_pair': round(ms_step / job_pairs * world, 3),
               'higher_is_better': True,
               'scaling': 'strong' if (split or args.config == 'c4') else 'weak',
               'vs_baseline': None, 'dtype': 'u8->i32/f32/f64',
               'data': 'synthetic (Gaussian-smoothed uniform texture, sinusoidal shift)',
               'config': {'workload': workload, 'tile': tile, 'tiles_per_pair': grid * grid,
                          'window_size': WS, 'pairs_per_step': job_pairs,
                          'pairs_per_gpu_per_step': per_gpu, 'parallelism': par,
                          'streams': nstreams},
               'roofline': roof}
        if not args.no_volume:
            rec['volume_kernel_roofline'] = volume_roofline(solver)
            rec['volume_f16_kernel_roofline'] = volume_roofline(solver, f16=True)
            if world == 1:
                rec['fp16_flip_rate'] = fp16_flip_rate(solver)
        if world == 1 and not args.no_cpu_baseline and tile <= 128:   # S=256: 17 GB level 0 per tile on the host
            rec['cpu_baseline'] = cpu_baseline(args.cpu_sample_tiles, tile)
        print(json.dumps(rec))
    if dist:
        tdist.barrier()
        tdist.destroy_process_group()


if __name__ == '__main__':
    main()

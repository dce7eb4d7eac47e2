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
         gathered to rank 0 (RCCL over xGMI), which stitches (strong scaling).
Timing is barrier + synchronize bracketed, max over ranks.  Consecutive pair solves are
pipelined over 2 HIP streams (--streams): a solve's level kernel waits for the previous
solve's level kernel, and the previous pair's latency-bound tail (levels >= 3, matching,
stitch) runs beside it; every step still solves its pair completely inside the timed region.
Every timed solve's stitched maps are kept (on the device) and, after the timed region,
compared bit for bit with the same pair solved again on one stream, un-pipelined
(`step_outputs_identical`, `step_outputs`).  The default c3 line also carries `c5_split`:
one 4096^2 pair per step with its 256 tiles split over the ranks and gathered to rank 0
(north_star's 8-GPU target), with the N = 1 reference solved on rank 0 in the same run.

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

sys.path.insert(0, os.path.join(REPO, 'tools'))
import kernel_hash  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
WS = 5
S = 128
GRID = 8
CONFIGS = {'c2': (64, 8), 'c3': (128, 8), 'c4': (128, 8), 'c5': (256, 16)}   # (tile S, tiles per axis)
C4_PAIRS = 64                  # BASELINE configs[3]: a batch of 64 independent 1024^2 pairs
BASELINE_LEVELS = {'c2': 3, 'c3': 4, 'c4': 4}   # BASELINE configs[1..3]: "3-level" / "4-level pyramid"
SPEC_CLOCK_GHZ = 2.4           # MI355X_MICROARCH.md: max clock (the issue roofline's peak)
# Rehearsal of the multi-rank path on a box with fewer GPUs than ranks (tests/test_bench_ranks.py):
# DM_BENCH_BACKEND=gloo and DM_BENCH_ONE_DEVICE=1 put every rank on cuda:0 over gloo.  The
# driver's runs leave both unset: one rank per GPU over RCCL ("nccl").
BACKEND = os.environ.get('DM_BENCH_BACKEND', 'nccl')
# the c5 split solves each rank's band of tiles in this many chunks, each chunk's gather to rank 0
# overlapping the next chunk's compute (shard.ChunkGather)
C5_CHUNKS = int(os.environ.get('DM_C5_CHUNKS', '4'))
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
    ap.add_argument('--level-stream', type=int, default=0,
                    help='1: the level kernels of all solves run on one stream of their own')
    ap.add_argument('--stats-stream', type=int, default=0,
                    help='1 (with --level-stream 1): stats of all solves on one stream of their own')
    ap.add_argument('--chain-levels', type=int, default=1,
                    help='1: each solve\'s level kernel waits for the previous one (no two level '
                         'kernels on the GPU at once); 0: consecutive level kernels may overlap')
    ap.add_argument('--pair-priority', choices=('normal', 'high'), default='normal',
                    help='priority of the pair streams (stats, levels >= 3, matching, stitch)')
    ap.add_argument('--config', choices=sorted(CONFIGS), default='c3',
                    help='BASELINE.json configs: c2 (512^2, S=64), c3 (1024^2, S=128; the metric), '
                         'c4 (64 pairs of c3 per step, sharded over the ranks), c5 (4096^2, S=256)')
    ap.add_argument('--pairs', type=int, default=C4_PAIRS, help='c4: pairs per step (whole job)')
    ap.add_argument('--tile', type=int, default=None)
    ap.add_argument('--grid', type=int, default=None)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--cpu-sample-tiles', type=int, default=16)
    ap.add_argument('--no-volume', action='store_true')
    ap.add_argument('--levels', type=int, default=None,
                    help='k-level pyramid (BASELINE configs C2 "3-level", C3 "4-level"): build and match '
                         'levels 0..k-1 only, as the reference Matching on co_map_list[:k] with '
                         'N_map = 2^(k-1); default: the full pyramid Correlation_map builds')
    ap.add_argument('--output-hash', action='store_true',
                    help="report sha256 of rank 0's stitched maps of its first pair, solved once "
                         "more after timing (always reported with the step check)")
    ap.add_argument('--no-k-level', action='store_true',
                    help='skip the extra timed pass at BASELINE\'s k-level pyramid')
    ap.add_argument('--no-step-check', action='store_true',
                    help='do not keep the timed solves\' outputs for the bit-for-bit check after timing')
    ap.add_argument('--no-c5-split', action='store_true',
                    help='c3: skip the c5_split sub-line (one 4096^2 pair, tiles split over the ranks)')
    ap.add_argument('--c5-steps', type=int, default=3, help='timed steps of the c5_split sub-line')
    ap.add_argument('--c5-no-group', action='store_true',
                    help='N = 1: run the c5_split sub-line without the one-rank process group (no '
                         'gather, no split_breakdown)')
    return ap.parse_args()


class PairSolver:
    """One ImageCutSolver-equivalent pass over a resident pair, with event timing of the
    dominant kernel (dm_corr_level12)."""

    def __init__(self, img1, img2, tile, grid, split=False, levels=None, chunks=None):
        """split: the pair's tiles are sharded over the ranks of the process group by
        shard.BandSolver -- the product path of ImageCutSolver's tile sharding (rank r solves one
        contiguous band of tiles in `chunks` chunks, each chunk's results gathered to rank 0
        behind the compute; rank 0 stitches the map).  Otherwise this rank solves every tile of
        its own pair in one batch.  levels: k-level pyramid (None: the full pyramid)."""
        from deepmatching_stereo_matching_amd import shard
        self.dev = img1.device
        self.tile = tile
        self.levels = levels
        self.n, origins = engine.cut_grid(tuple(img1.shape), [tile, tile], [tile, tile], WS)
        assert self.n == [grid, grid], self.n
        self.split = bool(split)
        self.T = len(origins)
        if self.split:
            self.band = shard.BandSolver(img1, img2, origins, tile, tile, WS, L.DM_TM_CCOEFF_NORMED,
                                         device=self.dev, chunks=chunks or C5_CHUNKS, dst=0)
            self.rank, self.world = self.band.rank, self.band.size
            self.chunk_idx = self.band.chunk_idx
            self.batches = self.band.batches
            self.origins = origins[self.band.tiles()]
        else:
            self.rank, self.world = 0, 1
            self.chunk_idx = [list(range(self.T))]
            self.origins = origins
            self.batches = [engine.TileBatch(img1, img2, origins, tile, tile, WS, L.DM_TM_CCOEFF_NORMED, self.dev)]
        self.batch = next((b for b in self.batches if b is not None), None)
        self.ev = []        # per timed solve: [(start, end) of each chunk's level kernel]

    def step(self, timed=False, stream=None, wait=None, level_stream=None, stats_stream=None):
        """One full solve of the pair on `stream` (default: the current stream).  Every
        device buffer belongs to this step's DevicePyramids, so steps on different streams
        share only the read-only images.  `wait`: event the level kernel waits for (the
        previous solve's level-kernel end when solves are pipelined over streams); this
        solve's last level-kernel end is left in self.last_end."""
        if stream is not None:
            with torch.cuda.stream(stream):
                return self.step(timed=timed, wait=wait, level_stream=level_stream,
                                 stats_stream=stats_stream)
        if self.split:   # rank 0 receives every tile's (3, S, S) result and stitches
            match = self.start_split(timed=timed, wait=wait, level_stream=level_stream,
                                     stats_stream=stats_stream).result()
            if match is None:
                return None
        else:
            match = self.compute(timed=timed, wait=wait, level_stream=level_stream,
                                 stats_stream=stats_stream)
        return engine.stitch(match, self.n, self.tile, self.tile, [self.tile, self.tile],
                             ['elevation'])

    def start_split(self, timed=False, wait=None, level_stream=None, stats_stream=None):
        """The split solve's band on the current stream through shard.BandSolver.start (each
        chunk's gather issued behind it) -> its ChunkGather; the chunks' level-kernel events
        are kept for level1_ms when timed."""
        evs = []
        g = self.band.start(sub_pix=True, nlev=self.levels, events=evs, wait=wait,
                            level_stream=level_stream, stats_stream=stats_stream)
        if evs:
            self.last_end = evs[-1][1]
        if timed:
            self.ev.append(evs)
        return g

    def compute(self, timed=False, wait=None, level_stream=None, stats_stream=None):
        """This rank's whole pair in one batch: stats, dm_corr_level12 [timed], dm_aggregate
        levels 3.., matching with sub-pixel -> float64 [T][3][S][S] on the current stream."""
        b = self.batch
        pyr = engine.DevicePyramid(b, build=False, stats_stream=stats_stream)
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        self.last_end = ev[1]
        diag = os.environ.get('DM_BENCH_DIAG', '')   # tools only: 'nomatch' / 'l12only' (not a bench line)
        pyr.build(events=ev, wait=wait, nlev=3 if diag == 'l12only' else self.levels, level_stream=level_stream)
        if diag:
            out = torch.zeros((b.T, 3, self.tile, self.tile), dtype=torch.float64, device=self.dev)
        else:
            out = pyr.match(sub_pix=True, nlev=self.levels)
        if timed:
            self.ev.append([ev])
        return out

    def level1_ms(self):
        """Mean over the timed solves of the level-kernel time per solve (summed over its
        chunks)."""
        if not self.ev:
            return None
        return float(np.mean([sum(a.elapsed_time(b) for a, b in evs) for evs in self.ev]))


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
    voxels = batch.T * batch.P * batch.P

    def timed(flags):
        ts = []
        for i in range(reps + 1):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            L.check(pyr.lib.dm_corr_volume_ex(batch.ref(), L.ptr(pyr.stats), flags, L.ptr(vol),
                                              L.stream_handle()))
            e1.record()
            torch.cuda.synchronize()
            if i:
                ts.append(e0.elapsed_time(e1))
        ms = float(np.mean(ts))
        gbs = esz * voxels / (ms * 1e-3) / 1e9
        return ms, gbs

    f = L.DM_VOLUME_F16 if f16 else 0
    ms, gbs = timed(f)          # standalone: computes the per-patch min/max itself
    ms_k, gbs_k = timed(f | L.DM_VOLUME_MINMAX_KNOWN)
    del vol, pyr
    torch.cuda.empty_cache()
    name = 'dm_corr_volume_f16 (k_volume_ls, binary16)' if f16 else 'dm_corr_volume (k_volume_ls)'
    key = 'volume_f16' if f16 else 'volume'
    return {'kernel': name, 'tiles': batch.T, 'tile': batch.h0,
            'ms': round(ms, 3), 'gvox_s': round(voxels / (ms * 1e-3) / 1e9, 1),
            'algorithmic_bytes_per_voxel': esz, 'bound': 'hbm',
            'achieved': round(gbs, 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
            'frac': round(gbs / HBM_PEAK_GBS, 4),
            'traffic': load_traffic(batch.h0, key, batch.T),
            'store_pattern_ceiling': store_ceiling(batch.h0, batch.T, esz, gbs),
            'minmax_known': {
                'what': 'the same volume, per-patch min/max already in the stats workspace (after '
                        'the level kernel, as Correlation_map()() then co_map): dm_corr_volume_ex '
                        'with DM_VOLUME_MINMAX_KNOWN skips the min/max sweep',
                'ms': round(ms_k, 3), 'achieved': round(gbs_k, 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                'frac': round(gbs_k / HBM_PEAK_GBS, 4),
                'traffic': load_traffic(batch.h0, key + '_mm', batch.T),
                'store_pattern_ceiling': store_ceiling(batch.h0, batch.T, esz, gbs_k, mm=True)}}


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


def load_pmc(tile, kernel='level1', tiles=None):
    """Per-launch PMC figures of a kernel from the committed rocprofv3 passes
    (profiles/pmc_<kernel>.json for the C3 shape, pmc_<kernel>_s<tile>.json for others;
    tools/profile.sh): HBM bytes (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE) and, for the
    level kernel, VALU instructions, the issue-cycle model and the clock.  Only a file made on
    the same tile size (and, when given, the same tiles per launch) is used."""
    for name in ('pmc_%s.json' % kernel, 'pmc_%s_s%d.json' % (kernel, tile)):
        try:
            with open(os.path.join(REPO, 'profiles', name)) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        if d.get('tile') == tile and (tiles is None or d.get('tiles', 64) == tiles):
            return d
    return {}


def isa_check(d, key, kind, tile, esz=None, mm=False):
    """Does profile field `key` (an ISA hash recorded when the profile was made) name the kernel
    bytes of the library this process loaded?  -> (ok, note)."""
    sym = kernel_hash.symbol(kind, tile, esz, mm)
    cur = kernel_hash.kernel_hash(sym) if sym else None
    rec = d.get(key)
    if sym is None:
        return False, 'no profiled kernel instance for this shape'
    if cur is None:
        return False, ('kernel instance %s not found in the loaded library (a non-default build? its '
                       'dm_build_config: %s)' % (sym, kernel_hash.build_config()))
    if rec != cur:
        return False, ('stale profile: it was made on kernel ISA %s, the loaded library holds %s '
                       '(re-run tools/pmc_r03.sh / tools/issue_model.py)' % (rec, cur))
    return True, 'profile made on this build (kernel ISA %s)' % cur


def load_traffic(tile, kernel='level1', tiles=None):
    """PMC HBM bytes per launch of the committed profile -- None unless the profile was taken
    on the kernel bytes this process loaded."""
    d = load_pmc(tile, kernel, tiles)
    esz = 2 if 'f16' in kernel else 4
    ok, _ = isa_check(d, 'isa_sha16', 'level' if kernel == 'level1' else 'volume', tile, esz,
                      kernel.endswith('_mm'))
    return d.get('hbm_bytes_per_launch') if ok else None


def store_ceiling(tile, tiles, esz, gbs, mm=False):
    """The rate the volume kernel's own store pattern allows with no arithmetic
    (tools/store_probe.hip, profiles/store_probe.jsonl: the same volume, 16-B nontemporal
    stores per lane, the kernel's patches per wave) and the fraction of it this run reached;
    None for shapes the probe did not run.  The pattern is the instance's (dm_kernels.hip
    launch_volume_ls): w0 = 128 binary16 with the min/max known stores 2 x 512 B of two patch
    maps per instruction ("volh_nt"), w0 = 128 float32 1 KB of one map ("volx_nt"), the others
    4 x 256 B of four maps advancing a row at a time ("vol_nt")."""
    name = 'c%d_f%d' % (3 if tile == 128 else 5, 8 * esz)
    pattern = ('volh_nt' if tile == 128 and esz == 2 and mm else
               'volx_nt' if tile == 128 and esz == 4 else 'vol_nt')
    try:
        with open(os.path.join(REPO, 'profiles', 'store_probe.jsonl')) as f:
            rows = [json.loads(ln) for ln in f if ln.strip()]
    except OSError:
        return None
    for r in rows:
        if r.get('shape') == name and r.get('tiles') == tiles and pattern in r:
            c = r[pattern]['gb_s']
            return {'gb_s': c, 'frac': round(gbs / c, 4), 'best_pattern_gb_s': r['seq']['gb_s'],
                    'source': 'profile: tools/store_probe.hip (profiles/store_probe.jsonl), pattern '
                              '"%s"; best_pattern = each wave streaming a contiguous slab' % pattern}
    return None


def level_roofline(solver, tile, l1_ms):
    """Roofline of the dominant kernel, dm_corr_level12 (k_level1_mfq): levels 0 -> 1 -> 2 in
    one pass, level 0 and level 1 never leave the chip.

    It is bound by vector-instruction issue, not by HBM (its physical traffic, ~1.2 GB per C3
    launch, is ~1.5 % of what the bandwidth allows in its run time) and not by the matrix
    cores.  achieved = the launch's issue cycles / its LIVE time (HIP events around every timed
    launch, on the launch stream); peak = 1024 SIMDs x 2.4 GHz (MI355X_MICROARCH.md max clock).
    The issue cycles per launch are a model (source 'profile'): the kernel's ISA, each
    instruction priced by what tools/valu_probe.hip measured on gfx950 (2.2 cycles for the
    simple VOP2/VOP1 32-bit ops, 4 for float64, packed float32, VOP3 and DPP forms, 11.2 for a
    v_mfma_i32_16x16x32_i8's hold on its SIMD), times how often each block runs (tools/isa_cost.py,
    profiles/pmc_level1.json: the modelled instruction count is checked against the PMC
    SQ_INSTS_VALU of the same build).  clock_ghz_at_full_issue = achieved / 1024: the clock at
    which the live time would mean every SIMD issued on every cycle (MI355X holds 1.7-2.3 GHz
    under this load); issue_occupancy_profiled = the modelled cycles over the cycles of the
    committed PMC pass's own launch (its GRBM_GUI_ACTIVE / 8), a measured busy fraction.
    valu_busy_pmc (SQ_ACTIVE_INST_VALU x 4 / (1024 x cycles)) prices every VALU instruction at
    4 cycles: an upper bound, kept for comparison with round 2."""
    mode = int(os.environ.get('DM_FUSE_L2', str(engine.FUSE_DEFAULT)))
    kern = 'k_level12_strip' if 'strip' in (kernel_hash.symbol('level', tile) or '') else 'k_level1_mfq'
    kname = ('dm_corr_level1 (%s)' % kern if mode == 0
             else 'dm_corr_level12 (%s, level 2 fused)' % kern)
    pmc = load_pmc(tile, 'level1', solver.batch.T)
    peak = 1024 * SPEC_CLOCK_GHZ
    roof = {'kernel': kname, 'bound': 'valu', 'ms': round(l1_ms, 3),
            'unit': 'G SIMD-issue-cycles/s', 'peak': peak}
    # the issue model and the PMC counters are used only when they were made on the kernel
    # bytes this process loaded (tools/kernel_hash.py); otherwise frac is null, with the reason
    model_ok, model_note = isa_check(pmc, 'issue_model_isa_sha16', 'level', tile)
    pmc_ok, pmc_note = isa_check(pmc, 'isa_sha16', 'level', tile)
    roof['isa_check'] = {'issue_model': model_note, 'pmc': pmc_note}
    cyc = pmc.get('issue_cycles_per_launch') if model_ok else None
    if cyc:
        achieved = cyc / (l1_ms * 1e-3) / 1e9
        roof.update({'achieved': round(achieved, 1), 'frac': round(achieved / peak, 4)})
        # the clock at which this live time would keep every SIMD issuing on every cycle
        roof['clock_ghz_at_full_issue'] = round(achieved / 1024, 4)
        if pmc.get('gpu_cycles_per_launch') and pmc_ok:
            # the same model over the profiled launch's own cycles (GRBM_GUI_ACTIVE / 8 XCDs):
            # one run's time and clock, not this run's time with another run's clock
            roof['issue_occupancy_profiled'] = {
                'value': round(cyc / (1024 * pmc['gpu_cycles_per_launch']), 4),
                'clock_ghz': pmc.get('clock_ghz'), 'kernel_ms': pmc.get('kernel_ms_profiled'),
                'source': 'profile: issue cycles / (1024 SIMDs x GRBM_GUI_ACTIVE / 8) of the PMC pass'}
        roof['source'] = {'time': 'live: HIP events around every timed launch on its stream',
                          'issue_cycles_per_launch': 'profile: ' + pmc.get('issue_model_note', ''),
                          'peak': '1024 SIMDs x 2.4 GHz, MI355X_MICROARCH.md'}
    else:
        roof.update({'achieved': None, 'frac': None,
                     'source': {'issue_cycles_per_launch': model_note if not model_ok and pmc
                                else 'no issue model for this batch shape'}})
    if not pmc_ok:
        pmc = {}
    if pmc.get('valu_busy_frac'):
        roof['valu_busy_pmc'] = {'value': pmc['valu_busy_frac'], 'source': 'profile',
                                 'note': 'SQ_ACTIVE_INST_VALU x 4 over 1024 SIMDs x GRBM cycles: '
                                         'every VALU instruction priced at 4 cycles (upper bound)'}
    for k in ('valu_insts_per_launch', 'ta_busy_frac', 'td_busy_frac'):
        if k in pmc:
            roof[k] = pmc[k]
    roof['traffic'] = pmc.get('hbm_bytes_per_launch')
    work = level_work(pmc, solver.batch.T, tile)
    if work:
        roof['work'] = work
    return roof


# float64 pow evaluations per level-0 voxel: the reference rectifies every value of levels 0, 1
# and 2 (misc/Correlation_map.py:141,148: V + V/16 + V/256); the fused kernel pools before it
# rectifies (pow14 is monotone): 4 child pows per level-1 value (V/4), one
# per pooled level-1 value of each level-2 window and cell (V/64) and one per level-2 value (V/256)
POW_REF_PER_VOXEL = 1.0 + 1.0 / 16 + 1.0 / 256
POW_POOLED_PER_VOXEL = 1.0 / 4 + 1.0 / 64 + 1.0 / 256
FMA_F64_PER_POW = 7    # pow14_zf / pow14_core_r: five series steps, fma(Phi, q, Plo), fma(Phi, G, s)


def level_work(pmc, T, tile):
    """roofline.work: the work the level kernel EXECUTES against the work
    the algorithm needs, from the PMC work pass of the same ISA (profiles/pmc_level1*.json,
    tools/pmc_r03.sh 'work'), so that a change which removes redundant work shows as less work
    and not only as a different issue-slot fraction.
      mac_slots_vs_algorithmic: i8 MFMA multiply-adds executed (SQ_INSTS_VALU_MFMA_MOPS_I8 x 512
        math ops / 2) over ws^2 = 25 per level-0 voxel (each voxel's correlation once); sweep 1
        (min / max) and sweep 2 (pooling) each compute every voxel, and K = 32 holds 25 or 30 taps.
      pow_evals_per_voxel: float64 FMAs executed (SQ_INSTS_VALU_FMA_F64 wave instructions x 64
        lanes) / 7 per pow evaluation, over V; beside it the reference's count (every value of
        levels 0-2) and the pool-before-rectify count (pow14 is monotone: only pooled values).
    None without a work pass made on this ISA (the caller drops it with the PMC pass)."""
    w = pmc.get('work_counters_per_launch') if pmc else None
    if not w or not w.get('SQ_INSTS_VALU_MFMA_MOPS_I8'):
        return None
    V = T * float(tile) ** 4
    macs = w['SQ_INSTS_VALU_MFMA_MOPS_I8'] * 512 / 2.0
    pows = w.get('SQ_INSTS_VALU_FMA_F64', 0.0) * 64 / FMA_F64_PER_POW
    return {'voxels_per_launch': V,
            'mac_slots_per_launch': macs, 'macs_algorithmic_per_launch': WS * WS * V,
            'mac_slots_vs_algorithmic': round(macs / (WS * WS * V), 4),
            'pow_evals_per_launch': pows, 'pow_evals_per_voxel': round(pows / V, 5),
            'pow_evals_reference_per_voxel': round(POW_REF_PER_VOXEL, 5),
            'pow_evals_pool_before_rectify_per_voxel': round(POW_POOLED_PER_VOXEL, 5),
            'pow_evals_vs_reference': round(pows / V / POW_REF_PER_VOXEL, 4),
            'f64_insts_per_launch': {k: w.get(k) for k in ('SQ_INSTS_VALU_FMA_F64', 'SQ_INSTS_VALU_MUL_F64',
                                                           'SQ_INSTS_VALU_ADD_F64')},
            'source': 'profile: PMC work pass (tools/pmc_r03.sh work) of this ISA; MACs = MOPS_I8 x 512 / 2, '
                      'pows = FMA_F64 x 64 lanes / %d' % FMA_F64_PER_POW}


def volume_equivalent(solver, tile, l1_ms):
    """NOT a roofline: the rate at which the fused level kernel consumes level-0 voxels,
    expressed as the HBM bandwidth a kernel that wrote the float32 volume (4 B
    per voxel) would need.  It can exceed the 8 TB/s peak because this kernel never writes
    the volume."""
    vox = solver.batch.T * float(tile) ** 4
    gbs = 4.0 * vox / (l1_ms * 1e-3) / 1e9
    return {'gb_s': round(gbs, 1), 'vs_hbm_peak': round(gbs / HBM_PEAK_GBS, 4),
            'voxels_per_launch': int(vox),
            'note': 'level-0 voxels per launch x 4 B / live kernel time; the volume is never written'}


def split_breakdown(solver, rank, world, dev):
    """c5 split: one more (untimed) solve, instrumented per rank -- compute (this rank's band of
    tiles, chunk by chunk: pyramid + matching, each chunk's gather to rank 0 issued behind it),
    the wait for the gathers still in flight when the compute ends, stitch (rank 0) -- in ms,
    for every rank."""
    import torch.distributed as tdist
    torch.cuda.synchronize()
    tdist.barrier()
    t0 = time.perf_counter()
    g = solver.start_split()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    full = g.result()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    if full is not None:
        engine.stitch(full, solver.n, solver.tile, solver.tile, [solver.tile, solver.tile], ['elevation'])
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    mine = torch.tensor([t1 - t0, t2 - t1, t3 - t2, float(len(solver.origins)), float(g.chunks)],
                        dtype=torch.float64, device=dev if tdist.get_backend() == 'nccl' else 'cpu')
    parts = [torch.empty_like(mine) for _ in range(world)]
    tdist.all_gather(parts, mine)
    return [{'rank': r, 'tiles': int(p[3]), 'chunks': int(p[4]), 'compute_ms': round(float(p[0]) * 1e3, 3),
             'gather_wait_ms': round(float(p[1]) * 1e3, 3), 'stitch_ms': round(float(p[2]) * 1e3, 3)}
            for r, p in enumerate(parts)]


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


class Pipeline:
    """Consecutive pair solves over `nstreams` HIP streams, round-robin and pipelined: each
    solve's level kernel waits for the previous solve's level kernel (chain_levels), so level
    kernels never share the GPU with each other and each one's event time stays its own,
    while the previous pair's latency-bound tail (levels >= 3, matching on demand, stitch:
    ~5 % of a solve) runs beside it.  Each solve still solves its pair completely.  The c5
    split's gather to rank 0 is issued from whichever stream the solve runs on: one process
    group's collectives run in issue order on its own communication stream, each waiting for
    the issuing stream, so solves on two streams gather in order."""

    def __init__(self, solvers, dev, dist, nstreams=2, chain_levels=True, level_stream=False,
                 stats_stream=False, priority=0):
        self.solvers, self.dist, self.dev = solvers, dist, dev
        self.chain = bool(chain_levels)
        # level_stream: every solve's level kernel goes to one more stream (serialised there,
        # no cross-pair event), so a pair's stats never wait behind the previous pair's tail.
        # HIP maps streams onto GPU_MAX_HW_QUEUES (4) hardware queues in order: a stream
        # sharing a queue with another waits behind that stream's work, so the pipeline keeps
        # to 3 streams (1 pair stream + level + stats) or 4.
        self.lstream = torch.cuda.Stream(device=dev) if level_stream else None
        self.streams = ([torch.cuda.Stream(device=dev, priority=priority) for _ in range(nstreams)]
                        if (nstreams > 1 or self.lstream is not None) else [None])
        # stats_stream: every solve's stats + window operands on one more stream, ahead of it
        self.sstream = (torch.cuda.Stream(device=dev) if (stats_stream and self.lstream is not None)
                        else None)
        self.nsolve = 0
        self.prev_end = None

    def step(self, timed=False, hold=None):
        """One step: every solver's pair once.  hold: list that receives (solver index,
        stitched (d_map, out_map)) of each solve, so its outputs can be checked after the
        timed region (the tensors stay alive; nothing is copied inside it)."""
        for i, s in enumerate(self.solvers):
            st = self.streams[self.nsolve % len(self.streams)]
            self.nsolve += 1
            wait = self.prev_end if (st is not None and self.lstream is None and self.chain) else None
            res = s.step(timed=timed, stream=st, wait=wait, level_stream=self.lstream,
                         stats_stream=self.sstream)
            self.prev_end = s.last_end
            if hold is not None and res is not None:
                hold.append((i, res))

    def run(self, steps, warmup, timed=True, hold=None):
        """warmup untimed steps, then `steps` timed ones bracketed by barrier + synchronize;
        seconds, max over ranks"""
        import torch.distributed as tdist
        for _ in range(warmup):
            self.step()
        torch.cuda.synchronize()
        if self.dist:
            tdist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            self.step(timed=timed, hold=hold)
        torch.cuda.synchronize()
        if self.dist:
            tdist.barrier()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        if self.dist:
            t = torch.tensor([el], dtype=torch.float64, device=self.dev)
            tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
            el = float(t.item())
        return el


def _bits(t):
    """The raw bits of a float64 map (NaN-safe bitwise comparison: uncovered cells are NaN)."""
    return t.contiguous().view(torch.int64)


def _sha256(maps):
    import hashlib
    h = hashlib.sha256()
    for t in maps:
        h.update(t.cpu().numpy().tobytes())
    return h.hexdigest()


def check_step_outputs(held, solvers, dist, steps):
    """Output check of the timed path.  Every solve of the timed steps -- pipelined over the
    streams, level kernels event-chained or overlapped, buffers shared across streams through
    record_stream -- left its stitched maps in `held`; each is compared bit for bit with the
    same pair solved once more after timing, on one stream, un-pipelined (the path
    tests/test_c3_batch.py pins tile by tile to the oracle).  The comparison runs on the
    device; sha256 of pair 0's maps is taken for every step and for the re-solve.  With
    ranks, `identical` is the AND over ranks (every rank takes part in the re-solve: the c5
    split gathers)."""
    torch.cuda.synchronize()
    ref = [s.step() for s in solvers]            # current stream, no wait, no overlap
    torch.cuda.synchronize()
    bad = 0
    for i, res in held:
        if ref[i] is None or not all(torch.equal(_bits(a), _bits(b)) for a, b in zip(res, ref[i])):
            bad += 1
    step_hashes = [_sha256(res)[:16] for i, res in held if i == 0]
    ref_hash = _sha256(ref[0]) if (ref and ref[0] is not None) else None
    # a rank of the c5 split other than 0 receives no maps (held and ref empty): nothing to check
    ok = int(bad == 0 and (len(held) > 0 or all(r is None for r in ref)))
    if dist:
        import torch.distributed as tdist
        t = torch.tensor([ok], dtype=torch.int64, device=torch.cuda.current_device())
        tdist.all_reduce(t, op=tdist.ReduceOp.MIN)
        ok = int(t.item())
    return {'identical': bool(ok), 'solves_checked': len(held), 'mismatched': bad,
            'steps': steps, 'sha256': ref_hash, 'step_sha256_16': step_hashes,
            'against': 'each timed solve\'s stitched (d_map, out_map) bit for bit vs the same pair '
                       're-solved after timing on one stream, un-pipelined (rank 0\'s figures; '
                       'identical = AND over ranks)'}


def c5_split(args, rank, world, dev, dist):
    """BASELINE configs[4] / north_star's "tiled 4096^2 pairs" line: one 4096^2 pair (16 x 16
    tiles of S = 256, the reference's ImageCutSolver loop, image_cut_solver.py:144-179) per
    step with its 256 tiles split over the ranks (shard.BandSolver: rank r solves one
    contiguous band of tiles in chunks, each chunk gathered to rank 0 over RCCL / xGMI behind
    the compute), and rank 0 stitches.  Timed like the main line (warmup, barrier +
    synchronize, max over ranks), outputs checked like it.  With N > 1, rank 0 then solves the
    whole pair alone on its GPU (the other ranks wait at a barrier): the N = 1 reference of
    the same run, so speedup = its ms_per_pair / the split's."""
    import torch.distributed as tdist
    tile, grid = CONFIGS['c5']
    side = (grid + 1) * tile + WS - 1
    # the pair is made (read, for a real input) on rank 0 only and sent to every rank once
    # (shard.broadcast_pair: 2 x 19 MB of uint8, before the timed region)
    from deepmatching_stereo_matching_amd import shard
    a = b = None
    if rank == 0 or not shard._group():
        a, b = stereo_pair(side, side, seed=1000, dx=2, max_disp=tile // 4, sinusoidal=True)
    img1, img2 = shard.broadcast_pair(a, b, src=0, device=dev)
    del a, b
    voxels = grid * grid * float(tile) ** 4
    steps, warmup = args.c5_steps, 1
    # with a process group (N > 1, or the one-rank RCCL group main() starts at N = 1) the tiles
    # go through the split path: shard.BandSolver, the product path of ImageCutSolver's tile
    # sharding (bands, chunked gathers to rank 0)
    split = world > 1 or shard.world()[1] == 1 and shard._group()
    solver = PairSolver(img1, img2, tile, grid, split=split)
    pipe = Pipeline([solver], dev, dist, nstreams=max(1, args.streams), chain_levels=args.chain_levels)
    held = [] if not args.no_step_check else None
    el = pipe.run(steps, warmup, hold=held)
    ms = el / steps * 1e3
    out = {'workload': 'C5: one %dx%d pair per step, %dx%d tiles of S=%d, ws=%d, full pyramid + '
                       'sub-pixel + cal_map + stitch; tiles split %d-way in contiguous bands, each '
                       'band in %d chunks gathered to rank 0 behind the compute%s'
                       % (grid * tile, grid * tile, grid, grid, tile, WS, world,
                          len(solver.chunk_idx), ' (RCCL process group of one rank)' if world == 1 and split else ''),
           'n_gpus': world, 'steps': steps, 'warmup': warmup, 'ms_per_pair': round(ms, 3),
           'value': round(voxels / (ms * 1e-3) / 1e9, 3), 'unit': 'Gvox/s',
           'level_kernel_ms': round(solver.level1_ms(), 3) if solver.ev else None}
    if held is not None:
        out['step_outputs'] = check_step_outputs(held, [solver], dist, steps)
        del held
    if split:
        out['split_breakdown'] = split_breakdown(solver, rank, world, dev)
    del pipe, solver
    torch.cuda.empty_cache()
    ref_ms = ms
    if world > 1:
        if rank == 0:
            alone = PairSolver(img1, img2, tile, grid, split=False)
            p1 = Pipeline([alone], dev, False, nstreams=max(1, args.streams), chain_levels=args.chain_levels)
            ref_ms = p1.run(steps, warmup) / steps * 1e3
            del p1, alone
            torch.cuda.empty_cache()
        t = torch.tensor([ref_ms], dtype=torch.float64, device=dev)
        tdist.broadcast(t, 0)
        ref_ms = float(t.item())
    out['reference_n1_ms_per_pair'] = round(ref_ms, 3)
    out['speedup_vs_n1'] = round(ref_ms / ms, 3)
    out['reference_n1'] = ('the same pair solved whole on rank 0\'s GPU alone in this run (same '
                           'pipelining, steps and timing)' if world > 1 else 'this line (N = 1)')
    return out


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
    # scaling, results gathered to rank 0); c4: a fixed batch of pairs split over the ranks
    # (strong scaling); c2/c3: one pair per rank per step (weak scaling)
    split = args.config == 'c5' and world > 1
    host_pairs, pair_idx, job_pairs = make_pairs(args, tile, grid, rank, world)
    solvers = []
    for a, b in host_pairs:
        img1, img2 = torch.from_numpy(a).to(dev), torch.from_numpy(b).to(dev)
        solvers.append(PairSolver(img1, img2, tile, grid, split=split, levels=args.levels))
    del host_pairs
    solver = solvers[0] if solvers else None
    voxels = grid * grid * float(tile) ** 4      # per pair

    nstreams = max(1, args.streams)
    pipe = Pipeline(solvers, dev, dist, nstreams=nstreams, chain_levels=args.chain_levels,
                    level_stream=args.level_stream, stats_stream=args.stats_stream,
                    priority=-1 if args.pair_priority == 'high' else 0)
    held = [] if not args.no_step_check else None
    elapsed = pipe.run(args.steps, args.warmup, hold=held)
    ms_step = elapsed / args.steps * 1e3
    value = job_pairs * args.steps * voxels / elapsed / 1e9
    l1_ms = solver.level1_ms() if solver else None
    if rank == 0 and solver is None:
        raise SystemExit('rank 0 has no pairs (--pairs < --gpus)')
    # the timed solves' outputs, checked after the timed region
    step_check = check_step_outputs(held, solvers, dist, args.steps) if held is not None else None
    del held

    # BASELINE.json states C2 / C3 (/ C4) on a 3- / 4-level pyramid: the same timed run with
    # the pyramid cut to k levels (levels 0..k-1 built, matching starts at level k-1), next to
    # the full pyramid Correlation_map always builds
    k_level = None
    k = BASELINE_LEVELS.get(args.config)
    if args.levels is None and k and not args.no_k_level and not split:
        for s_ in solvers:
            s_.levels = k
        el_k = pipe.run(args.steps, 1, timed=False)
        for s_ in solvers:
            s_.levels = None
        k_level = {'levels': k, 'ms_per_step': round(el_k / args.steps * 1e3, 3),
                   'ms_per_pair': round(el_k / args.steps * 1e3 / job_pairs, 3),
                   'value': round(job_pairs * args.steps * voxels / el_k / 1e9, 3), 'unit': 'Gvox/s',
                   'note': 'same workload and timing, pyramid cut to %d levels (co_map_list[:%d], '
                           'N_map = %d)' % (k, k, 2 ** (k - 1))}

    breakdown = split_breakdown(solver, rank, world, dev) if split else None
    # (every rank decides alike: the re-solve below is collective for the c5 split)
    out_hash = step_check['sha256'] if step_check else None
    if args.output_hash and step_check is None:
        res = solvers[0].step() if solvers else None    # split: every rank takes part
        torch.cuda.synchronize()
        if res is not None:
            out_hash = _sha256(res)

    if rank == 0:
        roof = level_roofline(solver, tile, l1_ms)
        lv = ('%d-level pyramid' % args.levels) if args.levels else 'full pyramid'
        if args.config == 'c4':
            workload = ('C4: batch of %d independent %dx%d pairs per step (%dx%d tiles of S=%d each), '
                        'ws=%d, %s + sub-pixel + cal_map + stitch'
                        % (job_pairs, grid * tile, grid * tile, grid, grid, tile, WS, lv))
            per_gpu, par = job_pairs / float(world), 'pairs of the batch sharded %d-way' % world
        else:
            workload = ('%s: %dx%d pair, %dx%d tiles of S=%d, ws=%d, %s '
                        '+ sub-pixel + cal_map + stitch'
                        % (args.config.upper(), grid * tile, grid * tile, grid, grid, tile, WS, lv))
            per_gpu = (1.0 / world) if split else 1
            par = ('tiles of one pair sharded %d-way, gathered to rank 0' if split
                   else 'pairs sharded %d-way') % world
        rec = {'metric': 'correlation-volume G-voxels/sec + ms/stereo-pair @1/8 GPU, 1024^2 d=128',
               'value': round(value, 3), 'unit': 'Gvox/s', 'n_gpus': joined, 'steps': args.steps,
               'warmup': args.warmup, 'ms_per_step': round(ms_step, 3),
               # wall time per pair of the whole job, and GPU time per pair (ms_step x GPUs / pairs)
               'ms_per_pair': round(ms_step / job_pairs, 3),
               'gpu_ms_per_pair': round(ms_step / job_pairs * world, 3),
               'higher_is_better': True,
               'scaling': 'strong' if (split or args.config == 'c4') else 'weak',
               'vs_baseline': None, 'dtype': 'u8->i32/f32/f64',
               'data': 'synthetic (Gaussian-smoothed uniform texture, sinusoidal shift)',
               'config': {'workload': workload, 'tile': tile, 'tiles_per_pair': grid * grid,
                          'window_size': WS, 'pyramid_levels': args.levels or 'full',
                          'pairs_per_step': job_pairs,
                          'pairs_per_gpu_per_step': per_gpu, 'parallelism': par,
                          'streams': nstreams, 'level_stream': bool(args.level_stream),
                          'stats_stream': bool(args.stats_stream and args.level_stream),
                          'pair_priority': args.pair_priority, 'chain_levels': bool(args.chain_levels)},
               'roofline': roof,
               'level_kernel_volume_equivalent': volume_equivalent(solver, tile, l1_ms)}
        if step_check is not None:
            rec['step_outputs_identical'] = step_check['identical']
            rec['step_outputs'] = step_check
        if os.environ.get('DM_BENCH_DIAG'):   # tools/run_r03dg.sh: skipped work, never a bench line
            rec['metric'] = 'DIAGNOSTIC (not the metric): ' + rec['metric']
            rec['diagnostic'] = ('DM_BENCH_DIAG=%s: matching (and, l12only, levels >= 3) skipped inside '
                                 'the timed steps' % os.environ['DM_BENCH_DIAG'])
        if k_level:
            rec['k_level'] = k_level
        if out_hash:
            rec['output_sha256'] = out_hash
        if breakdown:
            rec['split_breakdown'] = breakdown
        if not args.no_volume:
            rec['volume_kernel_roofline'] = volume_roofline(solver)
            rec['volume_f16_kernel_roofline'] = volume_roofline(solver, f16=True)
            if world == 1:
                rec['fp16_flip_rate'] = fp16_flip_rate(solver)
        if world == 1 and not args.no_cpu_baseline and tile <= 128:   # S=256: 17 GB level 0 per tile on the host
            rec['cpu_baseline'] = cpu_baseline(args.cpu_sample_tiles, tile)

    # north_star's "tiled 4096^2 pairs, 8 GPUs" line, carried by the default (c3) run, so the
    # driver's `bench.py --gpus N` measures it at every N (all ranks take part)
    if args.config == 'c3' and not args.no_c5_split and args.tile is None and args.grid is None:
        del pipe
        torch.cuda.empty_cache()
        own_group = False
        if not dist and not args.c5_no_group:
            # N = 1: a one-rank process group (RCCL with the default backend), so the c5 split's
            # band / chunked-gather path and its split_breakdown run at N = 1 too
            import socket
            import torch.distributed as tdist
            with socket.socket() as sk:
                sk.bind(('127.0.0.1', 0))
                port = sk.getsockname()[1]
            kw = {'device_id': dev} if BACKEND == 'nccl' else {}
            tdist.init_process_group(BACKEND, init_method='tcp://127.0.0.1:%d' % port, rank=0, world_size=1, **kw)
            own_group = True
        c5 = c5_split(args, rank, world, dev, dist)
        if own_group:
            tdist.destroy_process_group()
        if rank == 0:
            rec['c5_split'] = c5
    if rank == 0:
        print(json.dumps(rec))
    if dist:
        tdist.barrier()
        tdist.destroy_process_group()


if __name__ == '__main__':
    main()

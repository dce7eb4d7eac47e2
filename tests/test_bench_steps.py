"""The bench's TIMED path, output-checked (VERDICT r3 "Next" 1, 2, 8).

bench.py times pair solves pipelined over 2 (or 3) HIP streams, each solve's level kernel
event-chained to the previous one's (or, with --chain-levels 0, overlapping it), buffers
crossing streams through record_stream.  bench.py keeps every timed solve's stitched maps on
the device and, after the timed region, compares each bit for bit with the same pair solved
again on one stream, un-pipelined (`step_outputs`).  These tests run bench.py itself (a
subprocess, the driver's command line) and check that:

  * every timed solve is identical to the un-pipelined solve (`step_outputs_identical`);
  * that solve's sha256 equals the single-stream engine path of tests/test_c3_batch.py --
    TileBatch -> DevicePyramid.build -> match -> stitch, in this process -- which that test
    pins tile by tile to the oracle (so each timed step is oracle-pinned transitively);
  * for C4, one rank's full-size share (8 pairs of 1024^2, seeds 1000-1007) through the
    pipelined path matches each pair solved alone;
  * the default line's c5_split sub-line (one 4096^2 pair, tiles split over the ranks) runs
    and is output-checked the same way.

Reference: /root/reference/misc/image_cut_solver.py:144-179 (the per-tile solve + stitch
loop the bench's step is).
"""
import hashlib
import json
import os
import subprocess
import sys

import pytest
import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WS, GRID = 5, 8

pytestmark = pytest.mark.gpu


def _bench(*args, timeout=170):
    env = {k: v for k, v in os.environ.items()
           if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_ADDR', 'MASTER_PORT')}
    out = subprocess.run([sys.executable, os.path.join(REPO, 'bench.py'), '--no-volume',
                          '--no-cpu-baseline', '--no-k-level'] + list(args),
                         cwd=REPO, env=env, capture_output=True, text=True, timeout=timeout)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, out.stdout[-2000:]
    return json.loads(lines[0])


def _single_stream_sha(S, seed=1000, grid=GRID):
    """sha256 of (d_map, out_map) of the pair solved as tests/test_c3_batch.py solves it."""
    from deepmatching_stereo_matching_amd import _lib as L
    from deepmatching_stereo_matching_amd import engine
    from deepmatching_stereo_matching_amd.synthetic import stereo_pair
    side = (grid + 1) * S + WS - 1
    a, b = stereo_pair(side, side, seed=seed, dx=2, max_disp=S // 4, sinusoidal=True)
    dev = torch.device('cuda', 0)
    n, org = engine.cut_grid(a.shape, [S, S], [S, S], WS)
    batch = engine.TileBatch(torch.from_numpy(a).to(dev), torch.from_numpy(b).to(dev), org, S, S, WS,
                             L.DM_TM_CCOEFF_NORMED, dev)
    pyr = engine.DevicePyramid(batch, build=False)
    pyr.build()
    match = pyr.match(sub_pix=True)
    maps = engine.stitch(match, n, S, S, [S, S], ['elevation'])
    h = hashlib.sha256()
    for t in maps:
        h.update(t.cpu().numpy().tobytes())
    del pyr, batch, match, maps
    torch.cuda.empty_cache()
    return h.hexdigest()


def _check(rec, solves, sha=None):
    so = rec['step_outputs']
    assert rec['step_outputs_identical'] is True, so
    assert so['identical'] and so['mismatched'] == 0 and so['solves_checked'] == solves, so
    assert len(set(so['step_sha256_16'])) == 1, so['step_sha256_16']
    assert so['step_sha256_16'][0] == so['sha256'][:16]
    if sha is not None:
        assert so['sha256'] == sha


@pytest.mark.parametrize('config,S', [('c3', 128), ('c2', 64)])
@pytest.mark.parametrize('streams,chain', [(2, 1), (3, 0), (1, 1)])
def test_timed_steps_match_single_stream(config, S, streams, chain):
    rec = _bench('--config', config, '--steps', '6', '--warmup', '1', '--streams', str(streams),
                 '--chain-levels', str(chain), '--no-c5-split')
    assert rec['config']['streams'] == streams and rec['config']['chain_levels'] == bool(chain)
    _check(rec, 6, _single_stream_sha(S))


def test_c4_full_size_share():
    # one rank's C4 share at full size: 8 pairs of 1024^2 (seeds 1000-1007) per step, pipelined;
    # every solve equals that pair solved alone, and pair 0 the oracle-pinned single-stream map
    rec = _bench('--config', 'c4', '--pairs', '8', '--steps', '2', '--warmup', '1')
    assert rec['config']['pairs_per_step'] == 8
    _check(rec, 16)
    so = rec['step_outputs']
    assert so['sha256'] == _single_stream_sha(128, seed=1000)


def test_default_line_carries_c5_split():
    rec = _bench('--steps', '2', '--warmup', '1', '--c5-steps', '2')
    _check(rec, 2, _single_stream_sha(128))
    c5 = rec['c5_split']
    assert c5['n_gpus'] == 1 and c5['steps'] == 2 and c5['ms_per_pair'] > 0
    assert c5['speedup_vs_n1'] == 1.0
    so = c5['step_outputs']
    assert so['identical'] and so['solves_checked'] == 2 and len(set(so['step_sha256_16'])) == 1


def test_rccl_world_one_gather_and_breakdown():
    """The RCCL ("nccl") backend initialised at world size 1 on cuda:0: gather_units_to,
    _gather_units and bench.split_breakdown's all_gather run the real collectives (a process
    group disables the size-1 shortcut), and the split solve equals the unsplit one."""
    import socket
    import torch.distributed as tdist
    sys.path.insert(0, REPO)
    import bench
    from deepmatching_stereo_matching_amd import shard
    from deepmatching_stereo_matching_amd.synthetic import stereo_pair
    assert bench.BACKEND == 'nccl'
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    tdist.init_process_group('nccl', init_method='tcp://127.0.0.1:%d' % port, rank=0, world_size=1,
                             device_id=dev)
    try:
        assert tdist.get_backend() == 'nccl' and shard.world() == (0, 1)
        x = torch.arange(5 * 3 * 4, dtype=torch.float64, device=dev).reshape(5, 3, 4)
        g = shard.gather_units_to(x, 5, 0, 1, 0)
        assert g.is_cuda and torch.equal(g, x)
        g2 = shard._gather_units(x, 5, 0, 1, (3, 4), torch.float64)
        assert g2.is_cuda and torch.equal(g2, x)
        S, grid = 64, 2
        side = (grid + 1) * S + WS - 1
        a, b = stereo_pair(side, side, seed=1000, dx=2, max_disp=S // 4, sinusoidal=True)
        i1, i2 = torch.from_numpy(a).to(dev), torch.from_numpy(b).to(dev)
        split = bench.PairSolver(i1, i2, S, grid, split=True)
        whole = bench.PairSolver(i1, i2, S, grid, split=False)
        assert split.world == 1
        r_split, r_whole = split.step(), whole.step()
        torch.cuda.synchronize()
        for p, q in zip(r_split, r_whole):
            assert torch.equal(bench._bits(p), bench._bits(q))
        bd = bench.split_breakdown(split, 0, 1, dev)
        assert len(bd) == 1 and bd[0]['rank'] == 0 and bd[0]['tiles'] == grid * grid
        assert bd[0]['compute_ms'] > 0 and bd[0]['gather_wait_ms'] >= 0 and bd[0]['chunks'] >= 1
        # round 6: the product path through RCCL -- the pair sent by broadcast_pair, the mirror
        # ImageCutSolver with tile sharding (shard.BandSolver, chunked gathers) -- equals the
        # bench's split solve (the same BandSolver) and the unsharded mirror
        from deepmatching_stereo_matching_amd.misc.image_cut_solver import ImageCutSolver
        p1, p2 = shard.broadcast_pair(a, b, src=0, device=dev)
        assert p1.is_cuda and torch.equal(p1.cpu(), torch.from_numpy(a)) and torch.equal(p2.cpu(), torch.from_numpy(b))
        plain = ImageCutSolver(a, b, image_size=[S, S], stride=[S, S], window_size=WS)()
        with shard.tile_sharding():
            assert not shard.tile_sharding_enabled()      # one rank: the mirror solves it whole
        d_band, o_band = shard.solve_image_sharded(a, b, [S, S], [S, S], WS, 5, ('elevation',), sub_pix=True,
                                                   filtering_mode='median', result='all', chunks=2)
        assert np.array_equal(d_band.cpu().numpy(), plain[0], equal_nan=True)
        assert np.array_equal(o_band.cpu().numpy(), plain[1], equal_nan=True)
        assert torch.equal(bench._bits(d_band), bench._bits(r_whole[0]))
    finally:
        tdist.destroy_process_group()

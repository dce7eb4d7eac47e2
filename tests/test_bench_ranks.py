"""The multi-rank bench path end to end on one GPU: `bench.py --gpus N` starts N ranks itself
(torch.distributed.run as a child), the ranks join, time with barrier + max-over-ranks, and
rank 0 prints the JSON line.  The driver's scaling runs use one GPU per rank over RCCL; here
DM_BENCH_BACKEND=gloo and DM_BENCH_ONE_DEVICE=1 put every rank on cuda:0 (RCCL refuses two
ranks on one device), which exercises the same launcher, rendezvous, sharding, C5 gather-to-rank-0
and reporting code; every multi-rank run's stitched output (sha256 of rank 0's maps) must
equal a one-rank run of the same pair."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, timeout=150):
    env = {k: v for k, v in os.environ.items()
           if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_ADDR', 'MASTER_PORT')}
    env.update(DM_BENCH_BACKEND='gloo', DM_BENCH_ONE_DEVICE='1', OMP_NUM_THREADS='4')
    out = subprocess.run([sys.executable, os.path.join(REPO, 'bench.py'), '--steps', '1', '--warmup', '1',
                          '--no-volume', '--no-cpu-baseline'] + list(args),
                         cwd=REPO, env=env, capture_output=True, text=True, timeout=timeout)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, out.stdout[-2000:]   # rank 0 only
    return json.loads(lines[0])


@pytest.mark.gpu
def test_bench_two_ranks_weak():
    rec = _bench('--gpus', '2', '--config', 'c2', '--output-hash')
    assert rec['n_gpus'] == 2 and rec['scaling'] == 'weak'
    assert rec['config']['pairs_per_step'] == 2 and rec['config']['parallelism'] == 'pairs sharded 2-way'
    assert rec['value'] > 0 and rec['ms_per_step'] > 0
    assert rec['k_level']['levels'] == 3 and rec['k_level']['value'] > 0
    # rank 0 solves pair 0 (seed 1000) in both runs: its stitched maps must be identical
    one = _bench('--gpus', '1', '--config', 'c2', '--output-hash', '--no-k-level')
    assert rec['output_sha256'] == one['output_sha256']


@pytest.mark.gpu
def test_bench_two_ranks_c5_split():
    # one pair, its 2x2 tiles of S=256 split over the ranks, gathered to rank 0 and stitched
    rec = _bench('--gpus', '2', '--config', 'c5', '--grid', '2', '--output-hash')
    assert rec['n_gpus'] == 2 and rec['scaling'] == 'strong'
    assert rec['config']['tiles_per_pair'] == 4
    assert rec['config']['parallelism'] == 'tiles of one pair sharded 2-way, gathered to rank 0'
    assert rec['value'] > 0
    bd = rec['split_breakdown']
    assert [b['rank'] for b in bd] == [0, 1] and [b['tiles'] for b in bd] == [2, 2]
    assert all(b['compute_ms'] > 0 for b in bd)
    one = _bench('--gpus', '1', '--config', 'c5', '--grid', '2', '--output-hash')
    assert rec['output_sha256'] == one['output_sha256']


@pytest.mark.gpu
def test_bench_three_ranks_c4():
    rec = _bench('--gpus', '3', '--config', 'c4', '--pairs', '6', '--grid', '2', '--output-hash')
    assert rec['n_gpus'] == 3 and rec['scaling'] == 'strong'
    assert rec['config']['pairs_per_step'] == 6
    assert rec['value'] > 0
    one = _bench('--gpus', '1', '--config', 'c4', '--pairs', '6', '--grid', '2', '--output-hash')
    assert rec['output_sha256'] == one['output_sha256']


@pytest.mark.gpu
def test_bench_levels_option():
    rec = _bench('--gpus', '1', '--config', 'c2', '--levels', '3', '--no-k-level')
    assert rec['config']['pyramid_levels'] == 3 and '3-level pyramid' in rec['config']['workload']
    assert rec['value'] > 0

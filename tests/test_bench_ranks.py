"""The multi-rank bench path end to end on one GPU: `bench.py --gpus N` starts N ranks itself
(torch.distributed.run as a child), the ranks join, time with barrier + max-over-ranks, and
rank 0 prints the JSON line.  The driver's scaling runs use one GPU per rank over RCCL; here
DM_BENCH_BACKEND=gloo and DM_BENCH_ONE_DEVICE=1 put every rank on cuda:0 (RCCL refuses two
ranks on one device), which exercises the same launcher, rendezvous, sharding, C5 all-gather
and reporting code."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, timeout=300):
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
    rec = _bench('--gpus', '2', '--config', 'c2')
    assert rec['n_gpus'] == 2 and rec['scaling'] == 'weak'
    assert rec['config']['pairs_per_step'] == 2 and rec['config']['parallelism'] == 'pairs sharded 2-way'
    assert rec['value'] > 0 and rec['ms_per_step'] > 0


@pytest.mark.gpu
def test_bench_two_ranks_c5_split():
    # one pair, its 2x2 tiles of S=256 split over the ranks and all-gathered before stitching
    rec = _bench('--gpus', '2', '--config', 'c5', '--grid', '2')
    assert rec['n_gpus'] == 2 and rec['scaling'] == 'strong'
    assert rec['config']['tiles_per_pair'] == 4 and rec['config']['parallelism'] == 'tiles of one pair sharded 2-way'
    assert rec['value'] > 0


@pytest.mark.gpu
def test_bench_three_ranks_c4():
    rec = _bench('--gpus', '3', '--config', 'c4', '--pairs', '6', '--grid', '2')
    assert rec['n_gpus'] == 3 and rec['scaling'] == 'strong'
    assert rec['config']['pairs_per_step'] == 6
    assert rec['value'] > 0

"""Multi-rank sharding with the REAL engine on the GPU: world size 2 (and 3) on the one GPU
of the test box, gloo process group (RCCL refuses two ranks on one device; the per-tile
results are gathered through host copies, shard._gather_units).

Every rank receives the pair from rank 0 (shard.broadcast_pair) and runs
shard.solve_image_sharded -> shard.BandSolver (its contiguous band of tiles, chunk by chunk,
each chunk gathered to rank 0) -> engine.stitch on rank 0 -> the maps broadcast, and the mirror
ImageCutSolver()() with the process group initialised (it dispatches to shard; with
tile_sharding(result='root') only rank 0 gets the maps).  Both must equal a single-process solve byte for
byte, and the oracle's ImageCutSolver (misc/image_cut_solver.py:144-179) bit for bit.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

S, STRIDE, WS = 32, [24, 32], 5
MODES = ('elevation', 'distance')


def _case():
    from deepmatching_stereo_matching_amd.synthetic import stereo_pair
    return stereo_pair(137, 103, seed=77, dx=2, sinusoidal=True)   # 4 x 2 tiles, rows overlap


def _worker(rank, size, port, q):
    try:
        os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
        dist.init_process_group('gloo', rank=rank, world_size=size)
        torch.cuda.set_device(0)
        from deepmatching_stereo_matching_amd import shard
        from deepmatching_stereo_matching_amd.misc.image_cut_solver import ImageCutSolver
        a, b = _case() if rank == 0 else (None, None)
        a, b = (t.cpu().numpy() for t in shard.broadcast_pair(a, b, src=0))   # only rank 0 has the pair
        d, s = shard.solve_image_sharded(a, b, [S, S], STRIDE, WS, 5, MODES)
        cut = ImageCutSolver(a, b, image_size=[S, S], stride=STRIDE, window_size=WS,
                             degree_map_mode=list(MODES))
        with shard.tile_sharding():      # opt-in: every rank solves this same pair together
            d2, s2 = cut()
        with shard.tile_sharding(result='root'):   # the maps on rank 0 only (no broadcast)
            d3, s3 = ImageCutSolver(a, b, image_size=[S, S], stride=STRIDE, window_size=WS,
                                    degree_map_mode=list(MODES))()
        assert (d3 is None and s3 is None) == (rank != 0)
        if rank == 0:
            assert np.array_equal(d3, d2, equal_nan=True) and np.array_equal(s3, s2, equal_nan=True)
        dist.barrier()
        q.put((rank, d.cpu().numpy(), s.cpu().numpy(), d2, s2))
    except BaseException as e:   # report, do not hang the parent
        q.put((rank, repr(e), None, None, None))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


@pytest.fixture(scope='module')
def single():
    from deepmatching_stereo_matching_amd import engine
    from oracle import oracle as O
    a, b = _case()
    n, org = engine.cut_grid(a.shape, [S, S], STRIDE, WS)
    m = engine.solve_tiles(a, b, org, S, S, WS, 5)
    d, s = engine.stitch(m, n, S, S, STRIDE, list(MODES))
    O.set_pow_mode('pinned')
    try:
        od, os_ = O.cut_solve(a, b, image_size=[S, S], stride=STRIDE, window_size=WS,
                              degree_map_mode=MODES)
    finally:
        O.set_pow_mode('libm')
    return d.cpu().numpy(), s.cpu().numpy(), od, os_


@pytest.mark.parametrize('size', [2, 3])
def test_sharded_engine_equals_single_process(size, single):
    d1, s1, od, os_ = single
    assert np.array_equal(d1, od, equal_nan=True) and np.array_equal(s1, os_, equal_nan=True)
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, size, port, q)) for r in range(size)]
    for p in procs:
        p.start()
    try:
        res = [q.get(timeout=100) for _ in range(size)]
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for rank, d, s, d2, s2 in res:
        assert not isinstance(d, str), 'rank %d failed: %s' % (rank, d)
        for got in ((d, s), (d2, s2)):
            assert np.array_equal(got[0], d1, equal_nan=True), rank
            assert np.array_equal(got[1], s1, equal_nan=True), rank
    for p in procs:
        assert p.exitcode == 0

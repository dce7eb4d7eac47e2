"""Multi-rank sharding on CPU: gloo, world_size 2 (and 3), the oracle as the per-rank tile
solver.  The gathered / stitched result must equal the single-process one exactly."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from deepmatching_stereo_matching_amd import engine, shard


def _oracle_tiles(img1, img2, origins, h0, w0, ws, method, sub_pix, filtering, fws, fnum, fmode,
                  device=None):
    from oracle import oracle as O
    feat = 'cv2.TM_CCOEFF_NORMED' if method == 5 else 'cv2.TM_CCOEFF'
    out = []
    for r, c in np.asarray(origins).reshape(-1, 2):
        a = img1[r:r + h0 + ws - 1, c:c + w0 + ws - 1]
        b = img2[r:r + h0 + ws - 1, c:c + w0 + ws - 1]
        m, _, _ = O.solve_pair(a, b, ws, feat, sub_pix)
        out.append(m)
    return torch.from_numpy(np.stack(out))


def _host_stitch(match, n, h0, w0, stride, modes):
    """Stitching on the host (ImageCutSolver._execute_matching order, last writer wins)."""
    from oracle import oracle as O
    m = match.numpy()
    H, W = stride[0] * (n[0] - 1) + h0, stride[1] * (n[1] - 1) + w0
    dmap = np.full((len(modes), H, W), np.nan)
    score = np.full((H, W), np.nan)
    for t in range(len(m)):
        i, j = t % n[0], t // n[0]
        r, c = stride[0] * i, stride[1] * j
        for k, mode in enumerate(modes):
            dmap[k, r:r + h0, c:c + w0] = O.cal_map(m[t], mode)
        score[r:r + h0, c:c + w0] = m[t][2]
    return dmap, score


def _case():
    from deepmatching_stereo_matching_amd.synthetic import stereo_pair
    return stereo_pair(16 * 3 + 4 + 8, 16 * 4 + 4 + 8, seed=11, dx=2)


def _worker(rank, size, port, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=size)
    try:
        a, b = _case()
        d, s = shard.solve_image_sharded(a, b, [16, 16], [12, 16], 5, 5, ('elevation', 'distance'),
                                         solver=_oracle_tiles, stitcher=_host_stitch)
        q.put((rank, d, s))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def test_rank_units_partition():
    for n in (0, 1, 7, 64):
        for size in (1, 2, 3, 8):
            got = sorted(i for r in range(size) for i in shard.rank_units(n, r, size))
            assert got == list(range(n))
            counts = [len(shard.rank_units(n, r, size)) for r in range(size)]
            assert max(counts) - min(counts) <= 1


@pytest.mark.parametrize('size', [2, 3])
def test_sharded_image_equals_serial(size):
    a, b = _case()
    ref = shard.solve_image_sharded(a, b, [16, 16], [12, 16], 5, 5, ('elevation', 'distance'),
                                    solver=_oracle_tiles, stitcher=_host_stitch)
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, size, port, q)) for r in range(size)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(size)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, d, s in res:
        assert np.array_equal(d, ref[0], equal_nan=True), rank
        assert np.array_equal(s, ref[1], equal_nan=True), rank


def test_pairs_sharded_single_process():
    got = shard.solve_pairs_sharded(list(range(5)), lambda x: x * x)
    assert got == {i: i * i for i in range(5)}


def _pairs_worker(rank, size, port, q):
    """solve_pairs_sharded with the mirror ImageCutSolver inside fn and unequal pair counts
    per rank (5 pairs over 3 ranks: 2/2/1), DM_SHARD_TILES=1 set: tile sharding must stay
    off inside fn, so no rank enters a collective its peers do not (it used to
    mix tiles of different pairs, or hang)."""
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), DM_SHARD_TILES='1')
    dist.init_process_group('gloo', rank=rank, world_size=size)
    try:
        _patch_engine()
        from deepmatching_stereo_matching_amd.misc.image_cut_solver import ImageCutSolver
        pairs = _pairs()
        got = shard.solve_pairs_sharded(
            pairs, lambda p: ImageCutSolver(p[0], p[1], image_size=[16, 16], stride=[16, 16],
                                            window_size=5)())
        # and opted in explicitly with the SAME pair on every rank: tiles sharded, all-gathered
        with shard.tile_sharding():
            one = ImageCutSolver(pairs[0][0], pairs[0][1], image_size=[16, 16], stride=[16, 16],
                                 window_size=5)()
        q.put((rank, sorted(got), [got[i] for i in sorted(got)], one))
    finally:
        dist.destroy_process_group()


def _pairs():
    from deepmatching_stereo_matching_amd.synthetic import stereo_pair
    return [stereo_pair(16 * 2 + 4 + 16, 16 * 2 + 4 + 16, seed=30 + i, dx=1 + i % 2) for i in range(5)]


def _patch_engine():
    """The CPU stand-ins for the GPU solver and stitcher, returning torch tensors."""
    def stitch(match, n, h0, w0, stride, modes):
        d, s = _host_stitch(match, n, h0, w0, stride, modes)
        return torch.from_numpy(d), torch.from_numpy(s)
    engine.solve_tiles = _oracle_tiles
    engine.stitch = stitch
    shard.TILE_SOLVER = _oracle_tiles     # BandSolver's chunks (the sharded ImageCutSolver)


def test_pairs_sharded_with_image_cut_solver_unequal_counts():
    ref_engine = (engine.solve_tiles, engine.stitch)
    try:
        _patch_engine()
        from deepmatching_stereo_matching_amd.misc.image_cut_solver import ImageCutSolver
        ref = [ImageCutSolver(a, b, image_size=[16, 16], stride=[16, 16], window_size=5)()
               for a, b in _pairs()]
    finally:
        engine.solve_tiles, engine.stitch = ref_engine
        shard.TILE_SOLVER = None
    size = 3
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pairs_worker, args=(r, size, port, q)) for r in range(size)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(size)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    seen = []
    for rank, idx, outs, one in res:
        assert idx == shard.rank_units(5, rank, size)
        seen += idx
        for i, (d, s) in zip(idx, outs):
            assert np.array_equal(d, ref[i][0], equal_nan=True) and np.array_equal(s, ref[i][1], equal_nan=True)
        assert np.array_equal(one[0], ref[0][0], equal_nan=True)
        assert np.array_equal(one[1], ref[0][1], equal_nan=True)
    assert sorted(seen) == list(range(5))


def test_tile_sharding_is_opt_in(monkeypatch):
    monkeypatch.delenv('DM_SHARD_TILES', raising=False)
    assert not shard.tile_sharding_enabled()          # no process group, not opted in
    with shard.tile_sharding():
        assert not shard.tile_sharding_enabled()      # opted in, but a single process
        with shard.tile_sharding(False):
            assert shard._TILE_SHARDING is False
        assert shard._TILE_SHARDING is True
    assert shard._TILE_SHARDING is None


def test_rank_band_partition():
    """Contiguous bands: every unit once, in order, balanced to within one unit."""
    for n in (0, 1, 7, 64, 256):
        for size in (1, 2, 3, 8):
            bands = [shard.rank_band(n, r, size) for r in range(size)]
            assert sum(bands, []) == list(range(n))
            assert all(b == list(range(b[0], b[-1] + 1)) for b in bands if b)
            counts = [len(b) for b in bands]
            assert max(counts) - min(counts) <= 1


def _chunk_worker(rank, size, port, n, chunks, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=size)
    try:
        g = shard.ChunkGather(n, rank, size, (2, 3), torch.float64, 'cpu', dst=0, chunks=chunks)
        for c in range(g.chunks):
            idx = g.chunk_units(c)
            local = torch.tensor([[[float(i)] * 3] * 2 for i in idx], dtype=torch.float64).reshape(len(idx), 2, 3)
            g.put(c, local)
        out = g.result()
        band = shard.rank_band(n, rank, size)
        local = torch.tensor([[[float(i)] * 3] * 2 for i in band], dtype=torch.float64).reshape(len(band), 2, 3)
        once = shard.gather_units_to(local, n, rank, size, 0, units=shard.rank_band)
        bad = None
        try:
            shard.gather_units_to(local, n, rank, 1, 0)      # a size that is not the group's
        except ValueError as e:
            bad = str(e)
        q.put((rank, None if out is None else out.numpy(), None if once is None else once.numpy(), g.chunks, bad))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('size,n,chunks', [(2, 256, 4), (3, 256, 4), (3, 10, 4), (2, 3, 2), (8, 256, 4), (4, 3, 4)])
def test_chunk_gather_bands(size, n, chunks):
    """ChunkGather (bands cut into chunks, one asynchronous gather per chunk) and the one-shot
    band gather deliver every unit to rank 0 in unit order; a gather over a size other than
    the process group's raises instead of entering a mismatched collective."""
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_chunk_worker, args=(r, size, port, n, chunks, q)) for r in range(size)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(size))
    for p in procs:
        p.join(60)
    want = np.repeat(np.arange(n, dtype=np.float64), 6).reshape(n, 2, 3)
    for rank, out, once, nch, bad in res:
        assert bad is not None and 'group' in bad
        if rank == 0:
            assert np.array_equal(out, want) and np.array_equal(once, want)
        else:
            assert out is None and once is None
    assert len({r[3] for r in res}) == 1


def test_chunk_gather_without_group():
    g = shard.ChunkGather(5, 0, 1, (1,), torch.float64, 'cpu', chunks=2)
    for c in range(g.chunks):
        idx = g.chunk_units(c)
        g.put(c, torch.tensor(idx, dtype=torch.float64).reshape(-1, 1))
    assert torch.equal(g.result(), torch.arange(5, dtype=torch.float64).reshape(5, 1))
    with pytest.raises(ValueError):
        shard.gather_units_to(torch.zeros((2, 1)), 4, 0, 2)


def _band_worker(rank, size, port, q):
    """The product path of a tiled pair on every rank: the pair sent from rank
    0 (broadcast_pair), ImageCutSolver with tile sharding -> shard.BandSolver (bands, chunked
    gathers to rank 0, rank 0 stitches) with the maps returned on every rank ('all') or on rank
    0 only ('root'), and BandSolver itself (the object bench.py's c5_split drives)."""
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=size)
    try:
        _patch_engine()
        from deepmatching_stereo_matching_amd.misc.image_cut_solver import ImageCutSolver
        a, b = _case() if rank == 0 else (None, None)
        i1, i2 = shard.broadcast_pair(a, b, src=0, device='cpu')
        a, b = i1.numpy(), i2.numpy()
        with shard.tile_sharding():
            all_ = ImageCutSolver(a, b, image_size=[16, 16], stride=[12, 16], window_size=5,
                                  degree_map_mode=['elevation', 'distance'])()
        with shard.tile_sharding(result='root'):
            root = ImageCutSolver(a, b, image_size=[16, 16], stride=[12, 16], window_size=5,
                                  degree_map_mode=['elevation', 'distance'])()
        n, org = engine.cut_grid(a.shape, [16, 16], [12, 16], 5)
        band = shard.BandSolver(a, b, org, 16, 16, 5, 5, chunks=2)
        m = band.solve()
        q.put((rank, (a, b), all_, root, None if m is None else m.numpy(), band.tiles(),
               len(band.chunk_idx)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('size', [2, 3])
def test_band_solver_through_image_cut_solver(size):
    ref_engine = (engine.solve_tiles, engine.stitch)
    try:
        _patch_engine()
        from deepmatching_stereo_matching_amd.misc.image_cut_solver import ImageCutSolver
        a, b = _case()
        ref = ImageCutSolver(a, b, image_size=[16, 16], stride=[12, 16], window_size=5,
                             degree_map_mode=['elevation', 'distance'])()
        n, org = engine.cut_grid(a.shape, [16, 16], [12, 16], 5)
        ref_m = _oracle_tiles(a, b, org, 16, 16, 5, 5, True, False, 3, 3, 'median').numpy()
    finally:
        engine.solve_tiles, engine.stitch = ref_engine
        shard.TILE_SOLVER = None
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_band_worker, args=(r, size, port, q)) for r in range(size)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=240) for _ in range(size)), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    T = len(org)
    tiles = []
    for rank, pair, all_, root, m, mine, nch in res:
        assert np.array_equal(pair[0], a) and np.array_equal(pair[1], b)   # broadcast_pair
        assert np.array_equal(all_[0], ref[0], equal_nan=True) and np.array_equal(all_[1], ref[1], equal_nan=True)
        if rank == 0:
            assert np.array_equal(root[0], ref[0], equal_nan=True) and np.array_equal(root[1], ref[1], equal_nan=True)
            assert np.array_equal(m, ref_m, equal_nan=True)
        else:
            assert root == (None, None) and m is None
        assert mine == shard.rank_band(T, rank, size)
        tiles += mine
        assert nch == res[0][6]          # every rank issues the same number of gathers
    assert tiles == list(range(T))


def test_band_solver_single_process_and_result_setting(monkeypatch):
    """Without a process group BandSolver solves every tile (the chunks only bound memory), and a
    memory budget below one chunk's pyramid raises the chunk count; shard_result() follows
    tile_sharding(result=) and DM_SHARD_RESULT."""
    a, b = _case()
    n, org = engine.cut_grid(a.shape, [16, 16], [12, 16], 5)
    band = shard.BandSolver(a, b, org, 16, 16, 5, 5, chunks=2, solver=_oracle_tiles)
    assert band.tiles() == list(range(len(org))) and len(band.chunk_idx) == 2
    m = band.solve()
    assert np.array_equal(m.numpy(), _oracle_tiles(a, b, org, 16, 16, 5, 5, True, False, 3, 3, 'median').numpy(),
                          equal_nan=True)
    small = shard.BandSolver(a, b, org, 16, 16, 5, 5, chunks=1, solver=_oracle_tiles,
                             mem_budget=engine.tile_bytes(16, 16) * 3)
    assert len(small.chunk_idx) == -(-len(org) // 3)
    monkeypatch.delenv('DM_SHARD_RESULT', raising=False)
    assert shard.shard_result() == 'all'
    with shard.tile_sharding(result='root'):
        assert shard.shard_result() == 'root'
        with shard.tile_sharding():
            assert shard.shard_result() == 'root'
    monkeypatch.setenv('DM_SHARD_RESULT', 'root')
    assert shard.shard_result() == 'root'
    with pytest.raises(ValueError):
        with shard.tile_sharding(result='some'):
            pass
    i1, i2 = shard.broadcast_pair(a, b, device='cpu')
    assert np.array_equal(i1.numpy(), a) and np.array_equal(i2.numpy(), b)

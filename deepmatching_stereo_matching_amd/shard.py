"""Sharding of independent units over ranks (one process per GPU, torch.distributed).

SURVEY.md 8(e): tiles of one pair and whole pairs are independent (each tile depends only
on its (S + 2e)^2 crop, image_cut_solver.py:105-127), so the data path has no collective.
The tiles of ONE pair (ImageCutSolver with tile sharding, solve_image_sharded, and bench.py's
c5_split line -- the same code, BandSolver) go in contiguous bands: rank r solves tiles
[T r / N, T (r + 1) / N), chunk by chunk, and each chunk's (3, h0, w0) results travel to rank 0
by an asynchronous RCCL gather over xGMI while the rank computes its next chunk; rank 0
stitches.  Whole pairs (solve_pairs_sharded) go round robin, no collective at all.  Every
rank holds the whole input pair -- read from disk by rank 0 and sent once by broadcast_pair
(19 MB at C5) -- so a tiled pair needs no halo exchange.
"""

import contextlib
import os

import numpy as np
import torch
import torch.distributed as dist

from . import engine

# Tile sharding of the mirror ImageCutSolver is OPT-IN: a process group alone does not turn it
# on (ranks that each solve their own pairs, solve_pairs_sharded, must not enter one
# collective per pair).  None: the DM_SHARD_TILES environment variable decides (1 = on).
_TILE_SHARDING = None


def world():
    """(rank, world_size) of the default process group, (0, 1) without one."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


# Test hook: a callable with engine.solve_tiles' signature that BandSolver uses per chunk instead
# of the device batches when no `solver` is passed (the CPU multi-rank tests set it to the oracle).
TILE_SOLVER = None

# Which ranks ImageCutSolver's sharded solve returns the stitched maps on: 'all' (rank 0
# broadcasts them once, so every rank gets what a one-process ImageCutSolver()() returns; the
# default, and what DM_SHARD_RESULT=all selects) or 'root' (rank 0 only, the others get None:
# no broadcast of the (modes + 1) x H x W float64 maps, 268 MB at C5).
_SHARD_RESULT = None


@contextlib.contextmanager
def tile_sharding(enabled=True, result=None):
    """Inside this block, ImageCutSolver()() (misc/image_cut_solver.py) shards its tiles over
    the process group: every rank must then call it with the SAME pair, and collectively
    (BandSolver: rank r solves one contiguous band of tiles, rank 0 gathers and stitches).
    ``result``: 'all' (every rank returns the stitched maps: one broadcast from rank 0) or
    'root' (rank 0 returns them, the others (None, None)); None keeps the enclosing setting
    (default 'all', or DM_SHARD_RESULT).  tile_sharding(False) turns sharding off whatever
    DM_SHARD_TILES says."""
    global _TILE_SHARDING, _SHARD_RESULT
    if result not in (None, 'all', 'root'):
        raise ValueError("result must be 'all' or 'root'")
    prev, prev_r = _TILE_SHARDING, _SHARD_RESULT
    _TILE_SHARDING = bool(enabled)
    if result is not None:
        _SHARD_RESULT = result
    try:
        yield
    finally:
        _TILE_SHARDING, _SHARD_RESULT = prev, prev_r


def shard_result():
    """'all' or 'root': where the sharded ImageCutSolver returns its maps (tile_sharding)."""
    r = _SHARD_RESULT or os.environ.get('DM_SHARD_RESULT', 'all')
    if r not in ('all', 'root'):
        raise ValueError("DM_SHARD_RESULT must be 'all' or 'root'")
    return r


def tile_sharding_enabled():
    """True when ImageCutSolver should shard its tiles: opted in (tile_sharding() or
    DM_SHARD_TILES=1) and a process group of more than one rank is initialised."""
    on = _TILE_SHARDING if _TILE_SHARDING is not None else os.environ.get('DM_SHARD_TILES') == '1'
    return bool(on) and world()[1] > 1


def _group():
    """True when a process group is initialised: the gathers then always run the collective,
    at world size 1 too (a one-rank RCCL group is still exercised end to end)."""
    return dist.is_available() and dist.is_initialized()


def rank_units(n, rank, size):
    """Units of this rank: round robin (balanced to within one unit)."""
    return list(range(rank, n, size))


def rank_band(n, rank, size):
    """Units of this rank: one contiguous band [n r / N, n (r + 1) / N) (balanced to within one
    unit).  For the tiles of one pair, a band is a run of whole tile columns (ImageCutSolver's
    tile order), so a rank's image reads are one contiguous region instead of N-strided tiles."""
    return list(range(n * rank // size, n * (rank + 1) // size))


def _collective(size):
    """Run the collective?  Only with a process group, and only when `size` is that group's
    size: a caller passing another size while a group of N ranks is initialised would enter a
    collective whose parts list does not match the group."""
    if not _group():
        if size != 1:
            raise ValueError('no process group for a %d-rank gather' % size)
        return False
    if size != dist.get_world_size():
        raise ValueError('gather over %d ranks inside a process group of %d' % (size, dist.get_world_size()))
    return True


def _gather_units(local, n, rank, size, shape, dtype):
    """All-gather per-rank unit results ([k_r][*shape]) back into unit order [n][*shape].
    With the nccl (RCCL) backend the gather runs device to device over xGMI; a gloo group
    (CPU tests, or ranks sharing one GPU) gathers host copies and the result goes back to
    ``local``'s device."""
    per = (n + size - 1) // size
    group = _collective(size)
    host = group and local.is_cuda and dist.get_backend() == 'gloo'
    dev = local.device
    buf = torch.zeros((per,) + tuple(shape), dtype=dtype, device='cpu' if host else dev)
    if len(local):
        buf[:len(local)] = local
    if not group:
        return buf[:n]
    parts = [torch.empty_like(buf) for _ in range(size)]
    dist.all_gather(parts, buf)
    out = torch.empty((n,) + tuple(shape), dtype=dtype, device=buf.device)
    for r in range(size):
        idx = rank_units(n, r, size)
        if idx:
            out[idx] = parts[r][:len(idx)]
    return out.to(dev) if host else out


def gather_units_to(local, n, rank, size, dst=0, units=rank_units):
    """Gather per-rank unit results ([k_r][*shape], the units ``units(n, r, size)`` of rank r:
    round robin by default, rank_band for bands) to rank ``dst`` only, in unit order
    [n][*shape]; the other ranks get None.  Only the rank that stitches receives the tiles:
    with nccl (RCCL over xGMI) each peer sends its k_r units device to device, one link per
    peer, instead of every rank receiving every unit (all-gather).  gloo gathers host copies;
    the result goes back to ``local``'s device."""
    shape, dtype = tuple(local.shape[1:]), local.dtype
    per = max(len(units(n, r, size)) for r in range(size))
    group = _collective(size)
    host = group and local.is_cuda and dist.get_backend() == 'gloo'
    dev = local.device
    if len(local) == per and not host:
        buf = local.contiguous()
    else:
        buf = torch.zeros((per,) + shape, dtype=dtype, device='cpu' if host else dev)
        if len(local):
            buf[:len(local)] = local
    if not group:
        return buf[:n]
    parts = [torch.empty_like(buf) for _ in range(size)] if rank == dst else None
    dist.gather(buf, parts, dst=dst)
    if rank != dst:
        return None
    out = torch.empty((n,) + shape, dtype=dtype, device=buf.device)
    for r in range(size):
        idx = units(n, r, size)
        if idx:
            out[idx] = parts[r][:len(idx)]
    return out.to(dev) if host else out


class ChunkGather:
    """The units of every rank gathered to rank ``dst`` chunk by chunk, each chunk's gather
    issued (asynchronously) as soon as the rank has computed it, so it travels over xGMI while
    the rank computes its next chunk; only the last chunk's transfer is left when the rank's
    compute ends.  Rank r's units are ``units(n, r, size)`` (contiguous bands by default), cut
    into ``chunks`` chunks of equal count (every rank issues the same number of collectives,
    shorter ones padded).  put(c, local) for c = 0 .. chunks - 1 in order on every rank, then
    result() -> [n][*shape] on dst, None elsewhere.  Without a process group (size 1) the
    chunks are assembled locally."""

    def __init__(self, n, rank, size, shape, dtype, device, dst=0, chunks=1, units=rank_band):
        self.n, self.rank, self.size, self.dst = n, rank, size, dst
        self.shape, self.dtype = tuple(shape), dtype
        self.units = units
        self.per = max(len(units(n, r, size)) for r in range(size))
        self.chunks = max(1, min(int(chunks), self.per)) if self.per else 1
        self.csz = (self.per + self.chunks - 1) // self.chunks if self.per else 0
        self.group = _collective(size)
        self.host = self.group and torch.device(device).type == 'cuda' and dist.get_backend() == 'gloo'
        self.device = torch.device(device)
        self.work, self.parts, self.bufs = [], [], []

    def chunk_units(self, c, r=None):
        """Unit indices of chunk c of rank r (default: this rank)."""
        idx = self.units(self.n, self.rank if r is None else r, self.size)
        return idx[c * self.csz:(c + 1) * self.csz]

    def put(self, c, local):
        k = len(self.chunk_units(c))
        assert local.shape[0] == k, (local.shape, k)
        if not self.group:
            self.parts.append([local])
            return
        dev = 'cpu' if self.host else self.device
        if k == self.csz and not self.host:
            buf = local.contiguous()
        else:
            buf = torch.zeros((self.csz,) + self.shape, dtype=self.dtype, device=dev)
            if k:
                buf[:k] = local
        parts = [torch.empty_like(buf) for _ in range(self.size)] if self.rank == self.dst else None
        self.bufs.append(buf)               # kept alive until the collective has completed
        self.parts.append(parts)
        self.work.append(dist.gather(buf, parts, dst=self.dst, async_op=True))

    def result(self):
        for w in self.work:
            w.wait()
        self.work, self.bufs = [], []
        if self.rank != self.dst:
            self.parts = []
            return None
        out = torch.empty((self.n,) + self.shape, dtype=self.dtype,
                          device='cpu' if self.host else self.device)
        for c, parts in enumerate(self.parts):
            for r in range(self.size if self.group else 1):
                idx = self.chunk_units(c, r if self.group else self.rank)
                if idx:
                    out[idx] = parts[r][:len(idx)]
        self.parts = []
        return out.to(self.device) if self.host else out


def _bcast(t, src=0):
    """dist.broadcast of one tensor in place; a gloo group broadcasts a host copy of a device
    tensor (gloo has no device transport) and copies the result back."""
    if t.is_cuda and dist.get_backend() == 'gloo':
        h = t.cpu()
        dist.broadcast(h, src)
        t.copy_(h)
    else:
        dist.broadcast(t, src)
    return t


def broadcast_pair(img1=None, img2=None, src=0, device=None):
    """The input pair of a tiled solve, sent once from rank ``src`` (which passes it: host arrays
    or tensors, uint8 (H, W)) to every rank (the others pass None) -> (img1, img2) uint8 tensors
    on ``device`` on every rank.  SURVEY.md 8(e): the one-time broadcast (19 MB at C5) replaces
    a halo exchange -- every rank then holds the whole pair and crops its own band's tiles
    (image_cut_solver.py:105-112), and only rank ``src`` reads the file
    (ex_deepmatching_rawinput.py:50-55 loads both bands in one process).  Without a process group
    the pair is just moved to ``device``."""
    device = torch.device(device) if device is not None else engine.default_device()
    if not _group():
        return engine.to_device_u8(img1, device), engine.to_device_u8(img2, device)
    rank = dist.get_rank()
    host = dist.get_backend() == 'gloo'
    meta = torch.zeros(4, dtype=torch.int64, device='cpu' if host else device)
    if rank == src:
        a, b = np.asarray(img1) if not torch.is_tensor(img1) else img1, np.asarray(img2) if not torch.is_tensor(img2) else img2
        if tuple(a.shape) != tuple(b.shape) or len(a.shape) != 2:
            raise ValueError('broadcast_pair: two uint8 images of one (H, W) shape')
        meta[0], meta[1] = int(a.shape[0]), int(a.shape[1])
    _bcast(meta, src)
    H, W = int(meta[0]), int(meta[1])
    buf = torch.empty((2, H, W), dtype=torch.uint8, device=device)
    if rank == src:
        buf[0] = engine.to_device_u8(img1, device)
        buf[1] = engine.to_device_u8(img2, device)
    _bcast(buf, src)
    return buf[0], buf[1]


class BandSolver:
    """The tiles of ONE pair solved over the process group -- the multi-GPU product path that
    ImageCutSolver's tile sharding (solve_image_sharded) and bench.py's c5_split both run.

    Rank r takes one contiguous band of the pair's tile order (rank_band: whole tile columns,
    image_cut_solver.py:103-113, so its image reads are one region), cut into ``chunks`` chunks
    of equal count on every rank.  Each chunk is one engine batch (TileBatch -> DevicePyramid ->
    match: the pyramid, matching and sub-pixel of Correlation_map / Matching, solved per tile as
    image_cut_solver.py:115-142 does), and its [k][3][h0][w0] float64 results go to rank ``dst``
    by an asynchronous gather issued as soon as the chunk is enqueued (ChunkGather): the
    transfer of chunk c runs over xGMI while the rank computes chunk c + 1, so only the last
    chunk's gather is left when its compute ends.  Without a process group the one rank solves
    every tile, and the chunks only bound memory (``mem_budget``, engine.solve_tiles' rule).
    The per-chunk TileBatches (images on the device, tile origins) are built once and reused by
    every solve.  ``solver`` (engine.solve_tiles' signature) replaces the device solve per chunk
    (CPU tests)."""

    def __init__(self, img1, img2, origins, h0, w0, ws, method, device=None, chunks=4, dst=0,
                 mem_budget=None, solver=None):
        self.rank, self.size = world()
        solver = solver or TILE_SOLVER
        self.origins = np.asarray(origins, dtype=np.int64).reshape(-1, 2)
        self.T, self.h0, self.w0, self.ws, self.method, self.dst = len(self.origins), h0, w0, ws, method, dst
        self.solver = solver
        if solver is None:
            self.device = torch.device(device) if device is not None else engine.default_device()
            self.img1 = engine.to_device_u8(img1, self.device)
            self.img2 = engine.to_device_u8(img2, self.device)
        else:
            self.device = torch.device(device) if device is not None else torch.device('cpu')
            self.img1, self.img2 = img1, img2
        # chunks: at least `chunks` per band (overlap of gather and compute) and enough that one
        # chunk's pyramid fits the memory budget; the same count on every rank (the longest band)
        per = max(len(rank_band(self.T, r, self.size)) for r in range(self.size))
        budget = int(mem_budget if mem_budget is not None else os.environ.get('DM_MEM_BUDGET', 64 << 30))
        # (the fused level kernel keeps level 1 on chip at the MFMA shapes the band sizes take:
        # w0 a multiple of 64 and ws <= 5; otherwise the pyramid stores it and the estimate keeps it)
        fused = not engine.level1_stored() and w0 % 64 == 0 and h0 % 4 == 0 and ws <= 5
        fit = max(1, budget // max(engine.tile_bytes(h0, w0, level1=not fused), 1))
        self.chunks = max(1, int(chunks or 1), -(-per // fit))
        g = self._gather()
        self.chunk_idx = [g.chunk_units(c) for c in range(g.chunks)]
        if solver is None:
            self.batches = [engine.TileBatch(self.img1, self.img2, self.origins[idx], h0, w0, ws, method,
                                             self.device) if idx else None for idx in self.chunk_idx]
        else:
            self.batches = [None] * len(self.chunk_idx)

    def _gather(self):
        return ChunkGather(self.T, self.rank, self.size, (3, self.h0, self.w0), torch.float64, self.device,
                           dst=self.dst, chunks=self.chunks, units=rank_band)

    def tiles(self):
        """This rank's tile indices (its band, in order)."""
        return sum(self.chunk_idx, [])

    def start(self, sub_pix=True, filtering=False, filter_window_size=3, filtering_num=3,
              filtering_mode='median', nlev=None, events=None, wait=None, level_stream=None,
              stats_stream=None):
        """Enqueue this rank's band, chunk by chunk on the current stream, each chunk's gather
        to rank dst issued behind it -> the ChunkGather (result() waits and assembles).
        ``events``: a list that gets each chunk's (start, end) events around its level kernel;
        ``wait``: an event the first chunk's level kernel waits for; ``level_stream`` /
        ``stats_stream``: DevicePyramid's (pipelined solves)."""
        g = self._gather()
        for c, (idx, b) in enumerate(zip(self.chunk_idx, self.batches)):
            if not idx:      # a rank with fewer tiles than the longest band: an empty chunk
                out = torch.empty((0, 3, self.h0, self.w0), dtype=torch.float64, device=self.device)
            elif self.solver is not None:
                out = self.solver(self.img1, self.img2, self.origins[idx], self.h0, self.w0, self.ws,
                                  self.method, sub_pix, filtering, filter_window_size, filtering_num,
                                  filtering_mode, device=self.device)
            else:
                pyr = engine.DevicePyramid(b, build=False, stats_stream=stats_stream)
                ev = None
                if events is not None:
                    ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                    events.append(ev)
                pyr.build(events=ev, wait=wait if c == 0 else None, nlev=nlev, level_stream=level_stream)
                out = pyr.match(sub_pix, filtering, filter_window_size, filtering_num, filtering_mode, nlev=nlev)
                del pyr
            g.put(c, out)
        return g

    def solve(self, **kw):
        """start(**kw).result(): [T][3][h0][w0] float64 on rank dst, None elsewhere."""
        return self.start(**kw).result()


def solve_tiles_sharded(img1, img2, origins, h0, w0, ws, method, sub_pix=True, filtering=False,
                        filter_window_size=3, filtering_num=3, filtering_mode='median',
                        device=None, solver=None, dst=0, chunks=4):
    """engine.solve_tiles over all ranks (BandSolver: contiguous bands, chunked gathers) ->
    [T][3][h0][w0] float64 in tile order on rank ``dst``, None on the others; ``dst=None``: on
    every rank (rank 0 broadcasts the gathered results).  ``solver`` (same signature as
    engine.solve_tiles) replaces the GPU solver in tests."""
    band = BandSolver(img1, img2, origins, h0, w0, ws, method, device=device, chunks=chunks,
                      dst=0 if dst is None else dst, solver=solver)
    out = band.solve(sub_pix=sub_pix, filtering=filtering, filter_window_size=filter_window_size,
                     filtering_num=filtering_num, filtering_mode=filtering_mode)
    if dst is None and _group():
        if out is None:
            out = torch.empty((band.T, 3, h0, w0), dtype=torch.float64, device=band.device)
        _bcast(out, 0)
    return out


def solve_image_sharded(img1, img2, image_size, stride, window_size, method, modes=('elevation',),
                        sub_pix=True, filtering=False, filter_window_size=3, filtering_num=3,
                        filtering_mode='average', device=None, solver=None, stitcher=None,
                        result='all', chunks=4, grid=None):
    """ImageCutSolver()() for one (large) pair with its tiles sharded over the ranks
    (BandSolver), stitched on rank 0 -> (d_map [len(modes)][H][W], out_map [H][W]) on every rank
    (``result='all'``: one broadcast of the stitched maps from rank 0) or on rank 0 only
    (``'root'``: the others get (None, None)).  ``grid``: (tile counts, origins) when the caller
    counted them itself (ImageCutSolver counts on the shape before _padding, :46,58-62)."""
    if result not in ('all', 'root'):
        raise ValueError("result must be 'all' or 'root'")
    n, origins = grid if grid is not None else engine.cut_grid(np.shape(img1), image_size, stride, window_size)
    band = BandSolver(img1, img2, origins, image_size[0], image_size[1], window_size, method, device=device,
                      chunks=chunks, dst=0, solver=solver)
    match = band.solve(sub_pix=sub_pix, filtering=filtering, filter_window_size=filter_window_size,
                       filtering_num=filtering_num, filtering_mode=filtering_mode)
    stitch = stitcher or engine.stitch
    maps = stitch(match, n, image_size[0], image_size[1], stride, list(modes)) if match is not None else None
    if not _group() or world()[1] == 1:
        return maps
    if result == 'root':
        return maps if maps is not None else (None, None)
    H = stride[0] * (n[0] - 1) + image_size[0]
    W = stride[1] * (n[1] - 1) + image_size[1]
    dev = band.device
    if maps is None:
        d = torch.empty((len(modes), H, W), dtype=torch.float64, device=dev)
        o = torch.empty((H, W), dtype=torch.float64, device=dev)
    else:
        d, o = (torch.as_tensor(m) for m in maps)
    _bcast(d, 0)
    _bcast(o, 0)
    return d, o


def solve_pairs_sharded(pairs, fn):
    """Independent pairs (BASELINE configs[3]): rank r runs fn(pair) for pairs r::N and
    returns {pair index: result} for its own pairs (per-rank outputs, no collective).  Ranks
    hold different pairs (and different counts of them), so tile sharding is off inside fn:
    an ImageCutSolver there solves its whole pair on this rank."""
    rank, size = world()
    with tile_sharding(False):
        return {i: fn(pairs[i]) for i in rank_units(len(pairs), rank, size)}

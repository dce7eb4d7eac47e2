"""Sharding of independent units over ranks (one process per GPU, torch.distributed).

SURVEY.md 8(e): tiles of one pair and whole pairs are independent (each tile depends only
on its (S + 2e)^2 crop, image_cut_solver.py:105-127), so the data path has no collective:
rank r solves units r, r + N, r + 2N, ... on its own GPU.  The only exchange is the final
gather of the (3, h0, w0) per-tile results (RCCL over xGMI with the "nccl" backend; gloo on
CPU in the tests).  Every rank holds the whole input image (read from disk or broadcast
once), so a tiled pair needs no halo exchange.
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


@contextlib.contextmanager
def tile_sharding(enabled=True):
    """Inside this block, ImageCutSolver()() (misc/image_cut_solver.py) shards its tiles over
    the process group: every rank must then call it with the SAME pair, and collectively
    (rank r solves tiles r::N, results gathered to every rank).  tile_sharding(False) turns it
    off whatever DM_SHARD_TILES says."""
    global _TILE_SHARDING
    prev = _TILE_SHARDING
    _TILE_SHARDING = bool(enabled)
    try:
        yield
    finally:
        _TILE_SHARDING = prev


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


def solve_tiles_sharded(img1, img2, origins, h0, w0, ws, method, sub_pix=True, filtering=False,
                        filter_window_size=3, filtering_num=3, filtering_mode='median',
                        device=None, solver=None):
    """engine.solve_tiles over all ranks: rank r solves tiles r::N, results are gathered
    to every rank in the original tile order -> [T][3][h0][w0] float64.
    ``solver`` (same signature as engine.solve_tiles) replaces the GPU solver in tests."""
    rank, size = world()
    origins = np.asarray(origins, dtype=np.int64).reshape(-1, 2)
    mine = rank_units(len(origins), rank, size)
    solve = solver or engine.solve_tiles
    if mine:
        local = solve(img1, img2, origins[mine], h0, w0, ws, method, sub_pix, filtering,
                      filter_window_size, filtering_num, filtering_mode, device=device)
    else:
        dev = device or (engine.default_device() if solver is None else torch.device('cpu'))
        local = torch.empty((0, 3, h0, w0), dtype=torch.float64, device=dev)
    return _gather_units(local, len(origins), rank, size, (3, h0, w0), torch.float64)


def solve_image_sharded(img1, img2, image_size, stride, window_size, method, modes=('elevation',),
                        sub_pix=True, filtering=False, filter_window_size=3, filtering_num=3,
                        filtering_mode='average', device=None, solver=None, stitcher=None):
    """ImageCutSolver()() for one (large) pair with its tiles sharded over the ranks; every
    rank returns the stitched (d_map [len(modes)][H][W], out_map [H][W])."""
    n, origins = engine.cut_grid(np.shape(img1), image_size, stride, window_size)
    match = solve_tiles_sharded(img1, img2, origins, image_size[0], image_size[1], window_size,
                                method, sub_pix, filtering, filter_window_size, filtering_num,
                                filtering_mode, device=device, solver=solver)
    stitch = stitcher or engine.stitch
    return stitch(match, n, image_size[0], image_size[1], stride, list(modes))


def solve_pairs_sharded(pairs, fn):
    """Independent pairs (BASELINE configs[3]): rank r runs fn(pair) for pairs r::N and
    returns {pair index: result} for its own pairs (per-rank outputs, no collective).  Ranks
    hold different pairs (and different counts of them), so tile sharding is off inside fn:
    an ImageCutSolver there solves its whole pair on this rank."""
    rank, size = world()
    with tile_sharding(False):
        return {i: fn(pairs[i]) for i in rank_units(len(pairs), rank, size)}

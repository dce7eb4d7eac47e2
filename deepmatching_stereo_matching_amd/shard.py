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


def _gather_units(local, n, rank, size, shape, dtype):
    """All-gather per-rank unit results ([k_r][*shape]) back into unit order [n][*shape].
    With the nccl (RCCL) backend the gather runs device to device over xGMI; a gloo group
    (CPU tests, or ranks sharing one GPU) gathers host copies and the result goes back to
    ``local``'s device."""
    per = (n + size - 1) // size
    group = _group()
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


def gather_units_to(local, n, rank, size, dst=0):
    """Gather per-rank unit results ([k_r][*shape], units r::N) to rank ``dst`` only, in unit
    order [n][*shape]; the other ranks get None.  Only the rank that stitches receives the
    tiles: with nccl (RCCL over xGMI) each peer sends its k_r units device to device, one link
    per peer, instead of every rank receiving every unit (all-gather).  gloo gathers host
    copies; the result goes back to ``local``'s device."""
    shape, dtype = tuple(local.shape[1:]), local.dtype
    per = (n + size - 1) // size
    group = _group()
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
        k = len(rank_units(n, r, size))
        if k:
            out[r::size] = parts[r][:k]
    return out.to(dev) if host else out


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

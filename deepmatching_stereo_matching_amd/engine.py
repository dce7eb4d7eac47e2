"""Device-resident correlation engine: batches of equally sized tiles -> pyramid -> matches.

This is the layer the reference-surface mirror (``misc/``) and the tile scheduler sit on.
Everything stays in HBM as torch tensors; the HIP library (``_lib``) is called with raw
device pointers on the current torch stream.  Reference call stack it replaces:
``Correlation_map.__call__`` (misc/Correlation_map.py:161-173) ->
``Matching.__call__`` (misc/Matching.py:211-222) -> ``Calc_difference.cal_map``
(misc/Calc_difference.py:26-49), per tile of ``ImageCutSolver`` (misc/image_cut_solver.py).
"""

import contextlib
import ctypes
import os

import numpy as np
import torch

from . import _lib as L

LAM = 1.4
FUSE_DEFAULT = 2   # DevicePyramid level-1/level-2 mode (see its docstring); 2 is fastest on C3


def default_device():
    if not torch.cuda.is_available():
        raise L.DmUnavailable('no HIP device visible: the engine runs on MI355X only')
    return torch.device('cuda', torch.cuda.current_device())


def pyramid_plan(h0, w0):
    """Level count and N_map of Correlation_map._multi_level_correlation_pyramid
    (misc/Correlation_map.py:143-156).  Raises where its _aggregation would (:96-103)."""
    N, it, h, w = 1, 1, h0, w0
    while N < min(h0, w0):
        if h % 2 or w % 2:
            raise ValueError('could not broadcast input array from shape (%d,%d) into shape '
                             '(%d,%d)' % ((h + 1) // 2, (w + 1) // 2, h // 2, w // 2))
        h, w, N, it = h // 2, w // 2, N * 2, it + 1
    return it, N


def to_device_u8(img, device):
    if isinstance(img, torch.Tensor):
        t = img
    else:
        t = torch.from_numpy(np.ascontiguousarray(np.asarray(img, dtype=np.uint8)))
    if t.dtype != torch.uint8 or t.dim() != 2:
        raise ValueError('images must be 2-D uint8')
    return t.to(device).contiguous()


class TileBatch:
    """T tiles of one image pair: tile t is the (h0+ws-1) x (w0+ws-1) crop at origins[t]."""

    def __init__(self, img1, img2, origins, h0, w0, ws, method, device=None):
        self.device = device or default_device()
        self.img1 = to_device_u8(img1, self.device)
        self.img2 = to_device_u8(img2, self.device)
        if self.img1.shape != self.img2.shape:
            raise ValueError('img1 and img2 must have the same shape')
        org = np.asarray(origins, dtype=np.int64).reshape(-1, 2)
        H, W = self.img1.shape
        if ws < 1 or ws % 2 == 0:
            raise ValueError('could not broadcast: window_size must be odd (got %d)' % ws)
        if len(org) == 0 or h0 < 1 or w0 < 1:
            raise ValueError('empty tile batch')
        # the kernels trust these bounds: check them here, on the host
        if org.min() < 0 or (org[:, 0] + h0 + ws - 1).max() > H or (org[:, 1] + w0 + ws - 1).max() > W:
            raise ValueError('tile crop outside the image')
        self.origins_host = org
        self.origins = torch.from_numpy(org.astype(np.int32)).to(self.device).contiguous()
        self.T, self.h0, self.w0, self.ws, self.method = len(org), int(h0), int(w0), int(ws), int(method)
        self.struct = L.DmTiles(self.img1.data_ptr(), self.img2.data_ptr(),
                                self.img1.stride(0), self.img2.stride(0),
                                self.origins.data_ptr(), self.T, self.h0, self.w0,
                                self.ws, self.method)

    @property
    def P(self):
        return self.h0 * self.w0

    def ref(self):
        return ctypes.byref(self.struct)


class DevicePyramid:
    """co_map_list of a TileBatch, resident on the device.

    levels[0] is never stored (the fused kernels do not write level 0; matching evaluates
    it on demand).  ``fuse_level2`` (env DM_FUSE_L2) selects how levels 1-2 are built, on
    shapes the fused level-1/level-2 kernel supports:
      0  dm_corr_level1 writes level 1, dm_aggregate pools it into level 2;
      1  dm_corr_level12 writes levels 1 and 2 in one pass (no level-1 re-read);
      2  dm_corr_level12 writes level 2 only: level 1 stays on chip (levels[1] is None
         until ``level(1)`` asks for it) and matching evaluates it on demand.
    levels[l] for the others are float64 [T][Pl][Pl] tensors."""

    def __init__(self, batch, stream=None, build=True, fuse_level2=None, stats_stream=None):
        """stats_stream: optional stream the per-patch stats and window operands
        (dm_corr_stats) are computed on, ahead of this pyramid's own stream -- a caller
        pipelining pairs keeps them off the pair streams, where they would queue behind the
        previous pair's matching."""
        self.b = batch
        self.lib = L.load()
        try:   # a shape the pyramid rejects can still give its level-0 volume (bad_matching.py)
            self._plan = pyramid_plan(batch.h0, batch.w0)
        except ValueError as e:
            self._plan = e
        self.stream = stream
        self._stats_stream = stats_stream
        self._stats_ready = None
        nbytes = self.lib.dm_stats_bytes(batch.ref())
        if stats_stream is None:
            self.stats = torch.empty(nbytes, dtype=torch.uint8, device=batch.device)
        else:
            # from the stats stream's pool; every other stream that touches it is recorded, so
            # the caching allocator reuses it only after their work on it has finished
            with torch.cuda.stream(stats_stream):
                self.stats = torch.empty(nbytes, dtype=torch.uint8, device=batch.device)
            self.stats.record_stream(stream if stream is not None else torch.cuda.current_stream())
        if fuse_level2 is None:
            fuse_level2 = int(os.environ.get('DM_FUSE_L2', str(FUSE_DEFAULT)))
        self.fuse_level2 = int(fuse_level2)
        self.levels = [None]
        self._volume = None
        self._have_minmax = False
        self._have_stats = False
        if build:
            self.build()

    def _s(self):
        return L.stream_handle(self.stream)

    @property
    def nlev(self):
        """Level count (Correlation_map.iteration); raises the reference's aggregation
        error for shapes whose sides do not halve down to the top level."""
        if isinstance(self._plan, Exception):
            raise self._plan
        return self._plan[0]

    @property
    def N_map(self):
        if isinstance(self._plan, Exception):
            raise self._plan
        return self._plan[1]

    def compute_stats(self):
        if not self._have_stats:
            ss = self._stats_stream
            if ss is not None:
                # forward order: the images / origins may have been written on this pyramid's
                # own stream (a conversion, a non-blocking upload); the stats read them
                ready = torch.cuda.Event()
                ready.record(self.stream if self.stream is not None else torch.cuda.current_stream())
                ss.wait_event(ready)
            L.check(self.lib.dm_corr_stats(self.b.ref(), L.ptr(self.stats),
                                           L.stream_handle(ss) if ss is not None else self._s()),
                    'dm_corr_stats')
            if ss is not None:
                self._stats_ready = torch.cuda.Event()
                self._stats_ready.record(ss)
                (self.stream if self.stream is not None else torch.cuda.current_stream()).wait_event(
                    self._stats_ready)
            self._have_stats = True
        return self

    def _empty_level(self, k):
        b = self.b
        Pk = (b.h0 >> k) * (b.w0 >> k)
        return torch.empty((b.T, Pk, Pk), dtype=torch.float64, device=b.device)

    def _level1(self, stream=None, l1=None):
        if l1 is None:
            l1 = self._empty_level(1)
        sh = L.stream_handle(stream) if stream is not None else self._s()
        L.check(self.lib.dm_corr_level1(self.b.ref(), L.ptr(self.stats), L.ptr(l1), sh),
                'dm_corr_level1')
        self._have_minmax = True
        return l1

    def build(self, events=None, wait=None, nlev=None, level_stream=None):
        """Levels >= 1 up to level ``nlev`` - 1 (default: the full pyramid, as
        Correlation_map always builds it; a smaller ``nlev`` is the k-level pyramid of
        BASELINE configs C2/C3, whose levels above k - 1 Matching never reads).  ``events``:
        optional (start, end) torch.cuda.Event pair recorded around the level-1 (or fused
        level-1/level-2) kernel on this pyramid's stream.  ``wait``: optional event the level
        kernel waits for (the stats run before it) -- a caller pipelining pairs over streams
        passes the previous pair's level-kernel end, so the level kernels run one after
        another while each pair's latency-bound tail (levels >= 3, matching, stitch) overlaps
        the next pair's level kernel.  ``level_stream``: optional stream the level kernel runs
        on (it waits for this pyramid's stats, and this pyramid's stream waits for it): a
        caller that sends every pair's level kernel to one such stream serialises them without
        events, and a pair's stats no longer queue behind the previous pair's tail on a shared
        pair stream.  Building more levels later extends the pyramid."""
        b, lib = self.b, self.lib
        self.compute_stats()
        top = self.nlev if nlev is None else max(1, min(int(nlev), self.nlev))
        if top > 1 and len(self.levels) == 1:
            fused = False
            st = self.stream if self.stream is not None else torch.cuda.current_stream()
            ls = st
            if level_stream is not None and level_stream != st:
                ls = level_stream
                if self._stats_ready is not None:   # stats on their own stream: wait for them only
                    ls.wait_event(self._stats_ready)
                else:
                    ready = torch.cuda.Event()
                    ready.record(st)
                    ls.wait_event(ready)
                self.stats.record_stream(ls)
            if wait is not None:
                ls.wait_event(wait)
            if events:
                events[0].record(ls)
            # level buffers come from the level stream's pool (st's too when they are one):
            # st's later use of them is recorded, so the caching allocator reuses them only
            # after both streams' work on them
            with torch.cuda.stream(ls):
                l2 = self._empty_level(2) if (self.fuse_level2 and top >= 3) else None
                l1 = self._empty_level(1) if (self.fuse_level2 == 1 or l2 is None) else None
            if ls is not st:
                for t in (l1, l2):
                    if t is not None:
                        t.record_stream(st)
            if l2 is not None:
                rc = lib.dm_corr_level12(b.ref(), L.ptr(self.stats), L.ptr(l1), L.ptr(l2),
                                         L.stream_handle(ls))
                if rc == L.DM_OK:
                    self.levels += [l1, l2]
                    self._have_minmax = True
                    fused = True
                elif rc != L.DM_ERR_UNSUPPORTED:
                    L.check(rc, 'dm_corr_level12')
            if not fused:
                if l1 is None:
                    with torch.cuda.stream(ls):
                        l1 = self._empty_level(1)
                    if ls is not st:
                        l1.record_stream(st)
                self.levels.append(self._level1(ls, l1))
            if events:
                events[1].record(ls)
            if ls is not st:
                done = torch.cuda.Event()
                done.record(ls)
                st.wait_event(done)
        while len(self.levels) < top:
            k = len(self.levels)               # build level k from level k - 1
            h, w = b.h0 >> (k - 1), b.w0 >> (k - 1)
            nxt = self._empty_level(k)
            L.check(lib.dm_aggregate(L.ptr(self.levels[k - 1]), b.T, h, w, 1, L.ptr(nxt),
                                     self._s()), 'dm_aggregate')
            self.levels.append(nxt)
        return self

    def level_shape(self, k):
        h, w = self.b.h0 >> k, self.b.w0 >> k
        return (h, w, h, w)

    def _volume_into(self, v, f16):
        """dm_corr_volume_ex into v; once the level kernel (or an earlier volume call) has left
        the per-patch min/max in the stats workspace, the volume kernel reuses them
        (DM_VOLUME_MINMAX_KNOWN) instead of sweeping every window a second time."""
        self.compute_stats()
        flags = (L.DM_VOLUME_F16 if f16 else 0) | (L.DM_VOLUME_MINMAX_KNOWN if self._have_minmax else 0)
        L.check(self.lib.dm_corr_volume_ex(self.b.ref(), L.ptr(self.stats), flags, L.ptr(v), self._s()),
                'dm_corr_volume_ex')
        self._have_minmax = True
        return v

    def volume(self):
        """Level-0 min-max volume (co_map before rectification), float32 [T][P][P]."""
        if self._volume is None:
            b = self.b
            self._volume = self._volume_into(torch.empty((b.T, b.P, b.P), dtype=torch.float32,
                                                         device=b.device), False)
        return self._volume

    def volume_f16(self):
        """The level-0 min-max volume as binary16 (dm_corr_volume_f16, BASELINE config C5's
        fp16 correlation): float16 [T][P][P], each value np.float16 of volume()'s."""
        b = self.b
        return self._volume_into(torch.empty((b.T, b.P, b.P), dtype=torch.float16, device=b.device),
                                 True)

    def materialized_levels(self, l0_dtype='f32'):
        """co_map_list built the reference's way (misc/Correlation_map.py:132-156): level 0
        stored (float32 ``co_map`` or its fp16 rounding), rectified to float64
        (_rectification, :158-159), then every level by dm_aggregate (_aggregation,
        :89-130).  With 'f32' the levels equal the fused path's bit for bit; 'f16' is the
        C5 fp16-volume variant whose argmax flip rate the tests and bench report.
        Needs T * P^2 * (8 + 2|4) bytes of HBM."""
        b, lib = self.b, self.lib
        v = self.volume_f16() if l0_dtype == 'f16' else self.volume()
        l0 = torch.empty(v.shape, dtype=torch.float64, device=v.device)
        fn = lib.dm_rectify_f16 if l0_dtype == 'f16' else lib.dm_rectify
        L.check(fn(L.ptr(v), v.numel(), L.ptr(l0), self._s()), 'dm_rectify')
        if l0_dtype == 'f16':
            del v
        levels, h, w = [l0], b.h0, b.w0
        for _ in range(1, self.nlev):
            P2 = (h // 2) * (w // 2)
            nxt = torch.empty((b.T, P2, P2), dtype=torch.float64, device=b.device)
            L.check(lib.dm_aggregate(L.ptr(levels[-1]), b.T, h, w, 1, L.ptr(nxt), self._s()),
                    'dm_aggregate')
            levels.append(nxt)
            h, w = h // 2, w // 2
        return levels

    def level(self, k):
        """co_map_list[k] as a float64 device tensor [T][Pk][Pk]."""
        if k < 0:
            k += self.nlev
        if not 0 <= k < self.nlev:
            raise IndexError('list index out of range')
        if k > 0:
            if k >= len(self.levels):          # a k-level build: extend it
                self.build(nlev=k + 1)
            if self.levels[k] is None:   # level 1 kept on chip by dm_corr_level12
                self.levels[k] = self._level1()
            return self.levels[k]
        v = self.volume()
        out = torch.empty(v.shape, dtype=torch.float64, device=v.device)
        L.check(self.lib.dm_rectify(L.ptr(v), v.numel(), L.ptr(out), self._s()), 'dm_rectify')
        return out

    def match(self, sub_pix=True, filtering=False, filter_window_size=3, filtering_num=3,
              filtering_mode='median', levels=None, nlev=None):
        """Matching()() for every tile: float64 [T][3][h0][w0] (row, col, score).
        ``levels``: an explicit co_map_list (e.g. materialized_levels()) to match on
        instead of this pyramid's (level 0 then read from memory, not re-derived).
        ``nlev``: match on the first ``nlev`` levels only, the reference's Matching on a
        co_map_list cut to k levels with N_map = 2^(k-1): the descent
        starts at level nlev - 1, one start per cell of that level (Matching.py:80-96)."""
        b = self.b
        n = self.nlev if nlev is None else int(nlev)
        if not 1 <= n <= self.nlev:
            raise IndexError('list index out of range')
        if levels is None:
            if not self._have_minmax:
                self.volume()
            for k in range(len(self.levels), n):
                self.level(k)
            if n == 2 and self.levels[1] is None:   # the top level must be stored
                self.level(1)
        out = torch.empty((b.T, 3, b.h0, b.w0), dtype=torch.float64, device=b.device)
        scratch = torch.empty_like(out)
        if levels is not None:
            ptrs = (ctypes.c_void_p * n)(*[t.data_ptr() for t in levels[:n]])
        else:
            ptrs = (ctypes.c_void_p * n)(*([None] + [None if t is None else t.data_ptr()
                                                      for t in self.levels[1:n]]))
        fnum = int(filtering_num) if filtering else 0
        L.check(self.lib.dm_match(b.ref(), L.ptr(self.stats), ptrs, n, b.T, b.h0, b.w0,
                                  int(bool(sub_pix)), int(filter_window_size), fnum,
                                  1 if filtering_mode == 'median' else 0,
                                  L.ptr(scratch), L.ptr(out), self._s()), 'dm_match')
        return out


def match_levels(levels, sub_pix=True, filtering=False, filter_window_size=3, filtering_num=3,
                 filtering_mode='median', device=None):
    """Matching on an arbitrary (host or device) co_map_list, level 0 materialised."""
    device = device or default_device()
    lib = L.load()
    lv = [torch.as_tensor(np.ascontiguousarray(x) if not isinstance(x, torch.Tensor) else x,
                          dtype=torch.float64).to(device).contiguous() for x in levels]
    h0, w0 = lv[0].shape[:2]
    out = torch.empty((1, 3, h0, w0), dtype=torch.float64, device=device)
    scratch = torch.empty_like(out)
    ptrs = (ctypes.c_void_p * len(lv))(*[t.data_ptr() for t in lv])
    fnum = int(filtering_num) if filtering else 0
    L.check(lib.dm_match(None, None, ptrs, len(lv), 1, h0, w0, int(bool(sub_pix)),
                         int(filter_window_size), fnum, 1 if filtering_mode == 'median' else 0,
                         L.ptr(scratch), L.ptr(out), L.stream_handle()), 'dm_match')
    return out[0]


def subpix_map(level0, match):
    """Matching._sub_pix_cal (Matching.py:177-209) in place on a map that a descent left at a
    level above 0: `match` float64 [3][hm][wm] (device), refined against co_map_list[0]
    (`level0`: [h0][w0][h0][w0], host or device) at patch (i, j) and window (row, col) of each
    entry, as the reference does (dm_subpix_map).  Any entry is accepted and indexed the way
    numpy indexes co_map_list[0] (negative indices wrap, out-of-range ones take the
    reference's except branch)."""
    lib = L.load()
    if not isinstance(match, torch.Tensor) or not match.is_cuda:
        raise ValueError('match must be a device (cuda) tensor: the kernel refines it in place')
    if not match.is_contiguous() or match.dtype != torch.float64 or match.dim() != 3 or match.shape[0] != 3:
        raise ValueError('match must be a contiguous float64 [3][h][w] tensor')
    dev = match.device
    l0 = torch.as_tensor(level0, dtype=torch.float64).to(dev).contiguous()
    if l0.dim() != 4:
        raise ValueError('level 0 must be [h0][w0][h0][w0]')
    h0, w0 = l0.shape[:2]
    _, hm, wm = match.shape
    L.check(lib.dm_subpix_map(L.ptr(l0), 1, h0, w0, hm, wm, L.ptr(match), L.stream_handle()),
            'dm_subpix_map')
    return match


def subpix_map_tiles(pyr, match, stream=None):
    """subpix_map with level 0 on demand (dm_subpix_map_tiles): the five level-0 values an entry
    reads are recomputed from the pyramid's images and statistics, so co_map_list[0] is never
    materialised.  `match`: contiguous float64 device tensor [T][3][hm][wm] (or [3][hm][wm]
    when the batch holds one tile), refined in place."""
    if not isinstance(match, torch.Tensor) or not match.is_cuda:
        raise ValueError('match must be a device (cuda) tensor: the kernel refines it in place')
    m = match if match.dim() == 4 else match[None]
    b = pyr.b
    if not m.is_contiguous() or m.dtype != torch.float64 or m.shape[0] != b.T or m.shape[1] != 3:
        raise ValueError('match must be a contiguous float64 [T][3][h][w] tensor (T = %d)' % b.T)
    if not pyr._have_minmax:   # the per-patch min / max a level kernel or volume leaves in the stats
        pyr.build(nlev=2)
    if stream is not None and pyr.stream is not None and stream != pyr.stream:
        stream.wait_stream(pyr.stream)   # the stats the pyramid's stream wrote
    _, _, hm, wm = m.shape
    L.check(pyr.lib.dm_subpix_map_tiles(b.ref(), L.ptr(pyr.stats), hm, wm, L.ptr(m),
                                        L.stream_handle(stream) if stream is not None else pyr._s()),
            'dm_subpix_map_tiles')
    return match


def cal_map(match, mode, stream=None):
    """Calc_difference.cal_map on a [T][3][h][w] (or [3][h][w]) device tensor."""
    if mode not in L.CAL_MODES:
        raise ValueError(mode)
    m = match if match.dim() == 4 else match[None]
    m = m.contiguous()
    T, _, h, w = m.shape
    out = torch.empty((T, h, w), dtype=torch.float64, device=m.device)
    L.check(L.load().dm_cal_map(L.ptr(m), T, h, w, L.CAL_MODES[mode], L.ptr(out),
                                L.stream_handle(stream)), 'dm_cal_map')
    return out if match.dim() == 4 else out[0]


# ----------------------------------------------------------------------------------------
# tile scheduler (ImageCutSolver semantics, misc/image_cut_solver.py:58-179)
# ----------------------------------------------------------------------------------------
def cut_grid(shape, image_size, stride, window_size):
    """Tile counts and origins in the reference order (j outer, i inner; :62, :103-113)."""
    ex = int((window_size - 1) / 2)
    trimmed = [image_size[i] + 2 * ex for i in range(2)]
    n = [int(np.floor((shape[i] - trimmed[i]) / stride[i])) for i in range(2)]
    if n[0] < 1 or n[1] < 1:
        raise IndexError('list index out of range (no tile fits: image_cut_solver.py:150)')
    org = [(stride[0] * i, stride[1] * j) for j in range(n[1]) for i in range(n[0])]
    return n, np.array(org, dtype=np.int64)


def tile_bytes(h0, w0, level1=True):
    """Device bytes one tile needs inside DevicePyramid + match (levels >= 1, stats, maps).
    ``level1=False``: without the float64 level 1, which the fused level kernel never stores
    (DM_FUSE_L2=2, the default: matching re-derives it) -- 2.1 GB of the 2.3 GB of an S = 256
    tile."""
    nlev, _ = pyramid_plan(h0, w0)
    P = h0 * w0
    total = 6 * 4 * P + 2 * 3 * 8 * P
    h, w = h0, w0
    for k in range(1, nlev):
        h, w = h // 2, w // 2
        if k > 1 or level1:
            total += 8 * (h * w) ** 2
    return total


def level1_stored():
    """Does a DevicePyramid of the current configuration store level 1 (DM_FUSE_L2 != 2)?  The
    fused level kernel (mode 2) keeps it on chip; a shape it does not take stores it anyway, so
    callers sizing memory for such shapes keep tile_bytes' default."""
    return int(os.environ.get('DM_FUSE_L2', str(FUSE_DEFAULT))) != 2


def _on(stream):
    """Run a block with ``stream`` as torch's current stream, so that the library calls
    (launched on the current stream), the copies and the caching allocator's frees are all
    ordered on it."""
    return torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext()


def solve_tiles(img1, img2, origins, h0, w0, ws, method, sub_pix=True, filtering=False,
                filter_window_size=3, filtering_num=3, filtering_mode='median',
                device=None, mem_budget=None, stream=None):
    """Correlation_map + Matching for every tile; float64 [T][3][h0][w0] device tensor.
    Tiles are processed in chunks that fit ``mem_budget`` bytes of HBM.  Everything,
    allocations included, is ordered on ``stream`` (default: the current stream)."""
    device = device or default_device()
    with _on(stream):
        img1 = to_device_u8(img1, device)
        img2 = to_device_u8(img2, device)
        origins = np.asarray(origins, dtype=np.int64).reshape(-1, 2)
        if mem_budget is None:
            mem_budget = int(os.environ.get('DM_MEM_BUDGET', 64 << 30))
        per = tile_bytes(h0, w0)
        chunk = max(1, min(len(origins), mem_budget // max(per, 1)))
        out = torch.empty((len(origins), 3, h0, w0), dtype=torch.float64, device=device)
        for s in range(0, len(origins), chunk):
            b = TileBatch(img1, img2, origins[s:s + chunk], h0, w0, ws, method, device)
            pyr = DevicePyramid(b)
            out[s:s + len(b.origins_host)] = pyr.match(sub_pix, filtering, filter_window_size,
                                                       filtering_num, filtering_mode)
            del pyr, b
    return out


def stitch(match, n, h0, w0, stride, modes, stream=None):
    """ImageCutSolver._execute_matching stitching on the device -> (d_map, out_map)."""
    mode_ids = [L.CAL_MODES[m] for m in modes]
    Hout, Wout = stride[0] * (n[0] - 1) + h0, stride[1] * (n[1] - 1) + w0
    with _on(stream):
        m = match.contiguous()
        dmap = torch.empty((len(modes), Hout, Wout), dtype=torch.float64, device=match.device)
        score = torch.empty((Hout, Wout), dtype=torch.float64, device=match.device)
        arr = (ctypes.c_int32 * max(1, len(mode_ids)))(*mode_ids)
        L.check(L.load().dm_stitch(L.ptr(m), n[0], n[1], h0, w0, stride[0], stride[1], arr,
                                   len(mode_ids), L.ptr(dmap), L.ptr(score), L.stream_handle()),
                'dm_stitch')
    return dmap, score

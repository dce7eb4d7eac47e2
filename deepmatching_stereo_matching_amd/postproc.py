"""Device side of the Gauss-Seidel post-processing.

Reference: misc/optimize_loop.py (optimize_loop :15-37, image_threshold :40-44) and
misc/opt_loop.py (optimize_loop_bilateral_horizon :16-35, _vertical :39-58, make_weight
:60-85).  The mirrors in ``misc/`` keep the reference's signatures and numpy in/out
semantics; this module holds the float64 device maps, the dependency-level schedules
(``dm_gs_schedule``, cached per sweep shape and device) and the launches
(``dm_optimize_loop``, ``dm_make_weight``, ``dm_opt_loop_bilateral``).

Arrays may be numpy (copied in and out, like the reference's return values) or float64
torch tensors on the GPU (used in place where the reference works in place, no copies).
"""

import ctypes

import numpy as np
import torch

from . import _lib as L
from . import engine

_SCHED = {}


def schedule(kind, h, w, s0, s1, e, device):
    """(order, level_off, n_levels) of one sweep on `device` (dm_gs_schedule, host C++)."""
    key = (kind, h, w, s0, s1, e, str(device))
    hit = _SCHED.get(key)
    if hit is not None:
        return hit
    n = max(0, s0 - 2 * e - 1) * max(0, s1 - 2 * e - 1)
    order = np.empty(max(n, 1), dtype=np.int32)
    off = np.empty(n + 1, dtype=np.int32)
    nl = ctypes.c_int32(0)
    L.check(L.load().dm_gs_schedule(kind, h, w, s0, s1, e, order.ctypes.data_as(ctypes.c_void_p),
                                    off.ctypes.data_as(ctypes.c_void_p), ctypes.byref(nl)),
            'dm_gs_schedule')
    res = (torch.from_numpy(order).to(device), torch.from_numpy(off[:nl.value + 1].copy()).to(device),
           nl.value, n)
    _SCHED[key] = res
    return res


def host_schedule(kind, h, w, s0, s1, e):
    """numpy (order, level_off) of dm_gs_schedule (no device needed: host-only entry)."""
    n = max(0, s0 - 2 * e - 1) * max(0, s1 - 2 * e - 1)
    order = np.empty(max(n, 1), dtype=np.int32)
    off = np.empty(n + 1, dtype=np.int32)
    nl = ctypes.c_int32(0)
    L.check(L.load().dm_gs_schedule(kind, h, w, s0, s1, e, order.ctypes.data_as(ctypes.c_void_p),
                                    off.ctypes.data_as(ctypes.c_void_p), ctypes.byref(nl)),
            'dm_gs_schedule')
    return order[:n], off[:nl.value + 1]


def as_device(a, device):
    """(float64 contiguous device tensor, was_numpy)."""
    if isinstance(a, torch.Tensor):
        t = a
        if t.device != device or t.dtype != torch.float64 or not t.is_contiguous():
            t = t.to(device=device, dtype=torch.float64).contiguous()
        return t, False
    return torch.from_numpy(np.ascontiguousarray(np.asarray(a, dtype=np.float64))).to(device), True


def _size(size, shape, e):
    s0, s1 = int(size[0]), int(size[1])
    if e < 0:
        raise ValueError('exclusion must be >= 0')
    if s0 > shape[0] or s1 > shape[1]:
        raise IndexError('size (%d, %d) exceeds the map (%d, %d)' % (s0, s1, shape[0], shape[1]))
    return s0, s1


def threshold(t, lo, hi):
    out = torch.empty_like(t)
    L.check(L.load().dm_image_threshold(L.ptr(t), t.numel(), float(lo), float(hi), L.ptr(out),
                                        L.stream_handle()), 'dm_image_threshold')
    return out


def optimize_loop(img, coef, alpha, e, size):
    """img: thresholded float64 device map, swept in place; returns the error (device scalar)."""
    h, w = img.shape
    s0, s1 = _size(size, img.shape, e)
    hc, wc = coef.shape
    n = max(0, s0 - 2 * e - 1) * max(0, s1 - 2 * e - 1)
    err = torch.zeros((), dtype=torch.float64, device=img.device)
    if n == 0:
        return err
    if hc < s0 - e or wc < s1 - e:
        raise IndexError('index %d is out of bounds for axis 0 with size %d' % (s0 - e - 1, hc))
    if s0 - e >= h or s1 - e >= w:
        raise IndexError('index %d is out of bounds for axis 0 with size %d' % (s0 - e, h))
    fo, ff, fl, _ = schedule(L.DM_GS_FWD4, h, w, s0, s1, e, img.device)
    bo, bf, bl, _ = schedule(L.DM_GS_BWD4, h, w, s0, s1, e, img.device)
    diff = torch.empty(n, dtype=torch.float64, device=img.device)
    L.check(L.load().dm_optimize_loop(L.ptr(img), L.ptr(coef), hc, wc, h, w, s0, s1, e, float(alpha),
                                      L.ptr(fo), L.ptr(ff), fl, L.ptr(bo), L.ptr(bf), bl, L.ptr(diff),
                                      L.ptr(err), L.stream_handle()), 'dm_optimize_loop')
    return err


def make_weight(guide, e, size, den_c, den_s):
    """(gauss (W, W), color (s0-e, s1-e, W, W)) float64 device tensors."""
    h, w = guide.shape
    s0, s1 = _size(size, guide.shape, e)
    W = 2 * e + 1
    gauss = torch.empty((W, W), dtype=torch.float64, device=guide.device)
    color = torch.empty((max(s0 - e, 0), max(s1 - e, 0), W, W), dtype=torch.float64, device=guide.device)
    if s0 - e < 0 or s1 - e < 0:
        raise ValueError('negative dimensions are not allowed')
    L.check(L.load().dm_make_weight(L.ptr(guide), h, w, s0, s1, e, float(den_c), float(den_s), L.ptr(gauss),
                                    L.ptr(color), L.stream_handle()), 'dm_make_weight')
    return gauss, color


def bilateral(img, color, gauss, coef, e, size, vertical):
    """One sweep in place on img (float64 device map); returns the error (device scalar)."""
    h, w = img.shape
    s0, s1 = _size(size, img.shape, e)
    n = max(0, s0 - 2 * e - 1) * max(0, s1 - 2 * e - 1)
    err = torch.zeros((), dtype=torch.float64, device=img.device)
    if n == 0:
        return err
    W = 2 * e + 1
    if tuple(gauss.shape) != (W, W):
        raise ValueError('gausian_weight must be (%d, %d)' % (W, W))
    if color.dim() != 4 or tuple(color.shape[2:]) != (W, W) or color.shape[0] < s0 - 2 * e - 1 or \
            color.shape[1] != s1 - e:
        raise ValueError('color_weight_matrix must be (size[0]-e, size[1]-e, %d, %d) as make_weight makes it'
                         % (W, W))
    hc, wc = coef.shape
    if e >= hc or e >= wc or (e + 1 >= hc if vertical else e + 1 >= wc):
        raise IndexError('index %d is out of bounds for axis %d with size %d'
                         % (e + 1, 0 if vertical else 1, hc if vertical else wc))
    o, f, nl, _ = schedule(L.DM_GS_BILAT, h, w, s0, s1, e, img.device)
    diff = torch.empty(n, dtype=torch.float64, device=img.device)
    L.check(L.load().dm_opt_loop_bilateral(L.ptr(img), L.ptr(color), L.ptr(gauss), L.ptr(coef), hc, wc, h, w, s0,
                                           s1, e, int(bool(vertical)), L.ptr(o), L.ptr(f), nl, L.ptr(diff),
                                           L.ptr(err), L.stream_handle()), 'dm_opt_loop_bilateral')
    return err


def device_for(*arrays):
    for a in arrays:
        if isinstance(a, torch.Tensor) and a.is_cuda:
            return a.device
    return engine.default_device()

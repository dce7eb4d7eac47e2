"""Correlation_map mirror (reference: misc/Correlation_map.py:29-184) on gfx950 kernels.

Same constructor, attributes and methods.  ``__call__`` builds the pyramid on the GPU:
dm_corr_level12 evaluates levels 0 -> 1 -> 2 in one pass (level 2 written; levels 0 and 1
stay on chip and are re-derived on request) and dm_aggregate builds the levels above.
``co_map_list`` is a lazy sequence whose items are materialised to numpy float64
(h, w, h, w) only when indexed, and ``co_map`` (the min-max level-0 volume) only when read.
``Matching`` recognises the device pyramid (also cut to its first k levels) and matches
without copying.
"""

import operator
import sys
from collections.abc import Sequence

import numpy as np
import torch
import torch.nn as nn

from deepmatching_stereo_matching_amd import _lib as L
from deepmatching_stereo_matching_amd import engine

from deepmatching_stereo_matching_amd.misc.Feature_value import Feature_value


class LevelList(Sequence):
    """co_map_list backed by a DevicePyramid (one tile).

    Behaves like the reference's plain list where callers touch it: indexing materialises a
    level to numpy; a prefix slice (``co_map_list[:k]``, the SURVEY.md section 0 way of asking
    for a k-level pyramid) stays a device-backed LevelList of the first k levels, and so do
    ``del co_map_list[k:]`` and ``pop()``; any other slice is a plain list of arrays."""

    def __init__(self, pyr, n=None):
        self._pyr = pyr
        self._n = pyr.nlev if n is None else int(n)
        self._cache = {}

    @property
    def pyramid(self):
        return self._pyr

    def __len__(self):
        return self._n

    def _index(self, k):
        k = operator.index(k)
        if k < 0:
            k += len(self)
        if not 0 <= k < len(self):
            raise IndexError('list index out of range')
        return k

    def __getitem__(self, k):
        if isinstance(k, slice):
            start, stop, step = k.indices(len(self))
            if start == 0 and step == 1:
                view = LevelList(self._pyr, max(stop, 0))
                view._cache = self._cache
                return view
            return [self[i] for i in range(start, stop, step)]
        k = self._index(k)
        if k not in self._cache:
            t = self._pyr.level(k)[0]
            self._cache[k] = t.reshape(self._pyr.level_shape(k)).cpu().numpy()
        return self._cache[k]

    def __delitem__(self, k):
        if isinstance(k, slice):
            idx = sorted(range(*k.indices(len(self))))
            if not idx:                      # an empty cut deletes nothing, as on a list
                return
            if idx == list(range(idx[0], len(self))):   # a top suffix, in either direction
                self._n = idx[0]
                return
        elif self._index(k) == len(self) - 1:
            self._n -= 1
            return
        raise TypeError('co_map_list backed by the device pyramid can only drop its top levels')

    def pop(self, k=-1):
        if self._index(k) != len(self) - 1:
            raise TypeError('co_map_list backed by the device pyramid can only drop its top levels')
        top = self[len(self) - 1]
        self._n -= 1
        return top

    def device(self, k):
        """Level k as a float64 device tensor [Pk][Pk] (no host copy)."""
        return self._pyr.level(self._index(k))[0]


class Correlation_map():
    '''
    deepmatchingみたいにピラミッド状の特徴マップを作成する
    (builds the DeepMatching-style multi-level correlation pyramid)
    '''

    def __init__(self, img, template, window_size=3, feature_name='cv2.TM_CCOEFF_NORMED'):
        if img.shape != template.shape:
            print('use same size images!(サイズが違うと悲しい気持ちになるので(そのうち対応したいですね))')
            sys.exit()
        self.img = img
        self.template = template
        self.window_size = window_size
        self.lam = 1.4  # rectification

        self.exclusive_pix = int((window_size - 1) / 2)
        self.image_size = [x for x in img.shape]

        self.Feature = Feature_value(feature_name=feature_name)

        self.Maxpool = Maxpool()
        self.Maxpool.eval()

        self._pyr = None
        self._co_map = None

    # -- device plumbing -----------------------------------------------------------------
    def _map_sides(self):
        return (self.image_size[0] - 2 * self.exclusive_pix,
                self.image_size[1] - 2 * self.exclusive_pix)

    def _device_pyramid(self, build):
        if self._pyr is None:
            h0, w0 = self._map_sides()
            if self.window_size % 2 == 0:
                ws = self.window_size
                raise ValueError('could not broadcast input array from shape ({0},{0}) into '
                                 'shape ({1},{1})'.format(ws - 1, ws))
            b = engine.TileBatch(self.img, self.template, [(0, 0)], h0, w0, self.window_size,
                                 self.Feature.method)
            self._pyr = engine.DevicePyramid(b, build=False).compute_stats()
        if build:
            self._pyr.build()
        return self._pyr

    # -- reference methods -----------------------------------------------------------------
    def _create_atomic_patch(self):
        '''
        重なりありのatomic patchを作成する (overlapping ws x ws patches, uint8)
        '''
        h0, w0 = self._map_sides()
        ws = self.window_size
        img = np.asarray(self.img)
        if ws % 2 == 0:
            raise ValueError('could not broadcast input array from shape ({0},{0}) into shape '
                             '({1},{1})'.format(ws - 1, ws))
        win = np.lib.stride_tricks.sliding_window_view(img, (ws, ws))[:h0, :w0]
        self.atomic_patch = np.ascontiguousarray(win).astype(np.uint8)

    def _create_simple_initial_co_map(self):
        '''
        初めの相関マップを計算する (level-0 min-max volume, materialised on request)
        '''
        pyr = self._device_pyramid(build=False)
        h0, w0 = self._map_sides()
        self.co_map = pyr.volume()[0].to(torch.float64).reshape(h0, w0, h0, w0).cpu().numpy()

    @property
    def co_map(self):
        if self._co_map is None:
            if self._pyr is None:
                raise AttributeError("'Correlation_map' object has no attribute 'co_map'")
            self._create_simple_initial_co_map()
        return self._co_map

    @co_map.setter
    def co_map(self, value):
        self._co_map = value

    def _aggregation(self, map):
        '''
        aggregation to make upper class co_map: MaxPool(3,2,1) per p-map, then the
        4-children average (no rectification), on the GPU.
        '''
        m = np.ascontiguousarray(map, dtype=np.float64)
        h, w = m.shape[:2]
        dev = engine.default_device()
        src = torch.from_numpy(m.reshape(1, h * w, h * w)).to(dev)
        if h % 2 or w % 2:
            raise ValueError('could not broadcast input array from shape ({},{}) into shape '
                             '({},{})'.format((m.shape[2] + 1) // 2, (m.shape[3] + 1) // 2,
                                              m.shape[2] // 2, m.shape[3] // 2))
        out = torch.empty((1, (h // 2) * (w // 2), (h // 2) * (w // 2)), dtype=torch.float64,
                          device=dev)
        L.check(L.load().dm_aggregate(L.ptr(src), 1, h, w, 0, L.ptr(out), L.stream_handle()),
                'dm_aggregate')
        return out.reshape(h // 2, w // 2, h // 2, w // 2).cpu().numpy()

    def _multi_level_correlation_pyramid(self):
        '''
        aggregationを繰り返し、multi-level correlation pyramidを計算する
        '''
        pyr = self._device_pyramid(build=True)
        self.co_map_list = LevelList(pyr)
        self.iteration = pyr.nlev
        self.N_map = pyr.N_map

    def _rectification(self, map):
        m = np.asarray(map)
        dev = engine.default_device()
        if m.dtype == np.float32:
            src = torch.from_numpy(np.ascontiguousarray(m)).to(dev)
            fn = L.load().dm_rectify
        else:
            src = torch.from_numpy(np.ascontiguousarray(m, dtype=np.float64)).to(dev)
            fn = L.load().dm_rectify64
        out = torch.empty(src.shape, dtype=torch.float64, device=dev)
        L.check(fn(L.ptr(src), src.numel(), L.ptr(out), L.stream_handle()), 'dm_rectify')
        return out.cpu().numpy()

    def __call__(self):
        '''
        特徴マップの計算までを行う
        '''
        self._create_atomic_patch()
        self._multi_level_correlation_pyramid()
        return self.co_map_list


class Maxpool(nn.Module):
    """Kept for API compatibility (misc/Correlation_map.py:176-184); the pyramid kernels
    implement this pooling themselves."""

    def __init__(self, window=3, stride=2, padding=1):
        super(Maxpool, self).__init__()
        self.pool = nn.MaxPool2d(window, stride, padding=padding)

    def forward(self, x):
        return self.pool(x)

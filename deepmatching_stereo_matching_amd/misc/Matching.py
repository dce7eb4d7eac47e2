"""Matching mirror (reference: misc/Matching.py:20-268), backtracking on gfx950 kernels.

``__call__`` runs the whole coarse-to-fine descent (_initial_move_map, _B / _calc_match,
optional _filter, _sub_pix_cal) in dm_match.  It reads ``co_map_list`` and ``N_map`` the
way the reference does (Matching.py:85,96,105-106,127,133-134,182): the descent starts at
``co_map_list[-1]`` and takes one step per halving of ``N_map``, so a list cut to k levels
with N_map = 2^(k-1) is a k-level pyramid.  On a GPU-backed ``Correlation_map`` level 0
(and level 1) is re-evaluated on demand from the images (never materialised); for any
other object with a ``co_map_list`` the levels are uploaded and matched as given.
"""

import sys

import numpy as np
import torch
import torch.nn as nn

from deepmatching_stereo_matching_amd import engine


class Matching():
    '''
    multi-level correlation pyramidからマッチングを行う
    原著の14式に従って計算していく
    '''

    def __init__(
        self,
        Co_obj=None,
        filter_window_size=3,
        filtering=False,
        filtering_num=3,
        filtering_mode='median',
        sub_pix=True
    ):
        try:
            Co_obj.co_map_list
        except AttributeError as e:
            print('Error!: {}'.format(e))
            print('please run \'obj=Correlation_map()\' and \'obj()\' first.')
            sys.exit()

        MODES = ['average', 'median']
        assert filtering_mode in MODES, 'invalid filtering mode is input!: {}'.format(filtering_mode)

        self.obj = Co_obj
        self.Padding = Zero_padding()
        self.Padding.eval()

        self.filtering_num = filtering_num
        self.filter_window_size = filter_window_size
        self.filtering = filtering
        self.filtering_mode = filtering_mode
        self.sub_pix = sub_pix

    @classmethod
    def _sub_pix_compute(self, r0, r1, r_):
        '''
        二次関数近似の計算 (vertex of the parabola through r_, r0, r1; 0 if r0 is not a
        strict maximum).  Scalar helper; the kernel k_subpix evaluates the same expression.
        '''
        if r0 > r1 and r0 > r_:
            diff = - (r1 - r_) / (2 * (r1 + r_ - 2 * r0))
        else:
            diff = 0
        return diff

    def _descent(self):
        """(co_map_list, bottom, steps) of the reference's loop: _initial_move_map on
        co_map_list[-1] with N = N_map (:85-96), then one _B per halving of N until N == 1,
        _B number s reading co_map_list[-1 - s] (:105-106, :127, :133-134, :146-149).  A list
        cut to k levels with N_map = 2^(k-1) descends to level 0; a
        N_map that needs more levels than the list holds raises the reference's IndexError."""
        lst = self.obj.co_map_list
        n = len(lst)
        N = self.obj.N_map
        steps = 0
        while True:
            steps += 1
            if steps > n - 1:
                raise IndexError('list index out of range')
            N = int(N / 2)
            if N == 1:
                return lst, n - 1 - steps, steps

    def _device_match(self):
        lst, bottom, steps = self._descent()
        n = len(lst)
        fnum = self.filtering_num if self.filtering else 0
        # a descent that stops above level 0 is refined against co_map_list[0] all the same,
        # at the coarse map's (i, j, row, col) (:182-186): match without sub-pixel, then
        # dm_subpix_map_tiles (level 0 on demand from the images, never materialised) or, for
        # a plain co_map_list, dm_subpix_map on the given level 0
        sub_here = self.sub_pix and bottom == 0
        pyr = getattr(lst, 'pyramid', None)
        if isinstance(pyr, engine.DevicePyramid) and bottom == 0:
            out = pyr.match(self.sub_pix, self.filtering, self.filter_window_size, fnum,
                            self.filtering_mode, nlev=n)[0]
        elif isinstance(pyr, engine.DevicePyramid):
            levels = [lst.device(k).reshape(pyr.level_shape(k)) for k in range(bottom, n)]
            # match_levels runs on the current stream: it reads levels the pyramid wrote on its own
            if pyr.stream is not None:
                torch.cuda.current_stream().wait_stream(pyr.stream)
            out = engine.match_levels(levels, sub_here, self.filtering, self.filter_window_size,
                                      fnum, self.filtering_mode)
        else:
            out = engine.match_levels([lst[k] for k in range(bottom, n)], sub_here, self.filtering,
                                      self.filter_window_size, fnum, self.filtering_mode)
        if self.sub_pix and bottom > 0:
            if isinstance(pyr, engine.DevicePyramid):
                # the stream match_levels wrote `out` on (the pyramid's own stream
                # would refine the map before dm_match has written it)
                engine.subpix_map_tiles(pyr, out, stream=torch.cuda.current_stream())
            else:
                engine.subpix_map(lst[0], out)
        if self.filtering:  # _initial_move_map / _B decrement it once per level (:91-93, :136-138)
            self.filtering_num = max(0, self.filtering_num - (steps + 1))
        return out

    def __call__(self):
        '''
        multi-level correlation pyramidからマッチング計算を行う
        -> float64 (3, H', W'): matched row, matched col (sub-pixel if sub_pix), score
        '''
        self.map = self._device_match().cpu().numpy()
        return self.map


class Zero_padding(nn.Module):
    '''
    原著の14式の計算のため、ゼロパディングしておく (API compatibility; the matching kernel
    reads out-of-range window cells as 0 instead of padding each map)
    '''

    def __init__(self):
        super(Zero_padding, self).__init__()
        self.m = nn.ZeroPad2d(1)

    def forward(self, x):
        return self.m(x)

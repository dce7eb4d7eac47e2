"""Calc_difference mirror (reference: misc/Calc_difference.py:17-49), cal_map on the GPU."""

import sys

import numpy as np
import torch

from deepmatching_stereo_matching_amd import engine


class Calc_difference():
    '''
    Matchingクラスで計算したマップから視差マップを計算する
    '''

    def __init__(self):
        pass

    @staticmethod
    def cal_map(map, mode='elevation'):
        '''
        視差画像を計算する: elevation = j - map[1], elevation2 = i - map[0],
        distance = ||(i, j) - map[:2]||  (float64, shape map.shape[1:])
        '''
        MODES = ['elevation', 'elevation2', 'distance']
        if mode not in MODES:
            print('please input valid mode! {} are ok. yours is \'{}\''.format(MODES, mode))
            sys.exit()
        if isinstance(map, torch.Tensor) and map.is_cuda:
            return engine.cal_map(map.to(torch.float64), mode)
        dev = engine.default_device()
        m = torch.from_numpy(np.ascontiguousarray(map, dtype=np.float64)).to(dev)
        return engine.cal_map(m, mode).cpu().numpy()

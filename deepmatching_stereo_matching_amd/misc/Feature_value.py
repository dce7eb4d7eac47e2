"""Feature_value mirror (reference: misc/Feature_value.py:18-43).

The similarity primitive is fused into the level-0 kernels (csrc/dm_kernels.hip); this
class keeps the reference's validation, ``min_max`` helper and per-patch call surface.
"""

import sys

import numpy as np
import torch

from deepmatching_stereo_matching_amd import _lib as L
from deepmatching_stereo_matching_amd import engine


class Feature_value():
    '''
    特徴マップを計算する (computes one patch's min-max normalised similarity map)
    '''

    def __init__(self, feature_name='cv2.TM_CCOEFF_NORMED'):
        FEATURE_NAME_LIST = ['cv2.TM_CCOEFF_NORMED', 'cv2.TM_CCOEFF']
        if feature_name not in FEATURE_NAME_LIST:
            print('invalid feature_name \'{}\' is inputed!'.format(feature_name))
            sys.exit()
        self.feature_name = feature_name
        self.method = L.METHODS[feature_name]   # the reference eval()s the cv2 constant

    @staticmethod
    def min_max(x, axis=None):
        """Feature_value.min_max (:32-37), kept for API compatibility (host arrays)."""
        min = x.min(axis=axis, keepdims=True)
        max = x.max(axis=axis, keepdims=True)
        result = (x - min) / (max - min)
        return result

    def __call__(self, img, template):
        """matchTemplate(patch, template) + min_max for ONE ws x ws patch, on the GPU.

        Runs the level-0 volume kernel on a 1-tile batch whose first patch is ``img``;
        the pipeline itself never calls this (level 0 is fused into dm_corr_level1)."""
        patch = np.asarray(img, dtype=np.uint8)
        tmpl = np.asarray(template, dtype=np.uint8)
        ws = patch.shape[0]
        if patch.shape != (ws, ws) or tmpl.shape[0] < ws or tmpl.shape[1] < ws:
            raise ValueError('patch must be square and not larger than the template')
        canvas = np.zeros_like(tmpl)
        canvas[:ws, :ws] = patch
        h0, w0 = tmpl.shape[0] - ws + 1, tmpl.shape[1] - ws + 1
        b = engine.TileBatch(canvas, tmpl, [(0, 0)], h0, w0, ws, self.method)
        vol = engine.DevicePyramid(b, build=False).volume()
        return vol[0, 0].reshape(h0, w0).cpu().numpy()

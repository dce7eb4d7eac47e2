"""Loader mirror (reference: misc/loader.py:15-48) without OpenCV.

cv2.imread is replaced by Pillow.  Integrated mode keeps the reference's BGR channel
meaning (channel 1 = before, 2 = after, 0 = change map; cv2 loads B,G,R): with Pillow's
RGB order that is G, R, B.  Grayscale mode converts with ITU-R 601-2 luma (Pillow 'L'),
which can differ from cv2's fixed-point conversion by 1 for colour sources.
Documented deviation: the reference's ``assert type(path) == 'str'`` is always false
(loader.py:30,40) and would reject every call; this mirror checks isinstance instead.
"""

import numpy as np

from deepmatching_stereo_matching_amd.imageio import imread_bgr as _imread_bgr
from deepmatching_stereo_matching_amd.imageio import imread_gray as _imread_gray


class Loader():
    '''
    class to load images
    '''

    def __init__(self, path, start=[3500, 1760], size=[68, 260], integrated=True):
        self.img_list = []
        if integrated:
            assert isinstance(path, str), 'path must be string when integrated mode'
            img_loaded = _imread_bgr(path)
            img1_raw = img_loaded[:, :, 1]  # 地震前 (before)
            img2_raw = img_loaded[:, :, 2]  # 地震後 (after)
            img3_raw = img_loaded[:, :, 0]  # 変化マップ (change map)
            for im in (img1_raw, img2_raw, img3_raw):
                self.img_list.append(np.ascontiguousarray(im[start[0]:start[0] + size[0], start[1]:start[1] + size[1]]))
        else:
            assert isinstance(path, (list, tuple)), 'path must be list when not integrated mode'
            img1_raw = _imread_gray(path[0])
            img2_raw = _imread_gray(path[1])
            for im in (img1_raw, img2_raw):
                self.img_list.append(np.ascontiguousarray(im[start[0]:start[0] + size[0], start[1]:start[1] + size[1]]))

    def __call__(self):
        return self.img_list

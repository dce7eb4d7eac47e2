"""optimize_loop mirror (reference: misc/optimize_loop.py), evaluated by dm_optimize_loop.

Same signatures and results as the reference: ``optimize_loop`` thresholds a copy of the
map to [0, 10] and runs one forward and one backward Gauss-Seidel sweep of the 4-neighbour
update over it, returning (map, error); ``image_threshold`` clamps with two np.where.
numpy in -> numpy out; a float64 GPU tensor in -> tensor out (error stays a device scalar).
"""

import numpy as np
import torch

from deepmatching_stereo_matching_amd import postproc


def image_threshold(arr, threshold=[0, 10]):
    """misc/optimize_loop.py:40-44 (dm_image_threshold)."""
    dev = postproc.device_for(arr)
    t, was_np = postproc.as_device(arr, dev)
    out = postproc.threshold(t, threshold[0], threshold[1])
    return out.cpu().numpy() if was_np else out


def optimize_loop(img_dis, coefficient, alpha, exclusion, size):
    """misc/optimize_loop.py:15-37 -> (img_dis, error)."""
    dev = postproc.device_for(img_dis, coefficient)
    t, was_np = postproc.as_device(img_dis, dev)
    if t.dim() != 2:
        raise ValueError('img_dis must be a 2-D map')
    img = postproc.threshold(t, 0, 10)  # a new array, as image_threshold's np.where
    coef, _ = postproc.as_device(coefficient, dev)
    err = postproc.optimize_loop(img, coef, alpha, int(exclusion), size)
    if was_np:
        return img.cpu().numpy(), np.float64(err.item())
    return img, err

"""opt_loop mirror (reference: misc/opt_loop.py), evaluated by dm_make_weight and
dm_opt_loop_bilateral.

Same signatures and side effects as the reference: the two bilateral sweeps update
``img_dis`` in place and return (img_dis, error); ``make_weight`` returns
(gausian_weight, color_weight_matrix) with the matrix shaped (size[0]-e, size[1]-e, 2e+1,
2e+1) and zero outside the cells it fills.  exp is the pinned dm_exp (<= 1 ulp from
numpy's np.exp).  numpy in -> numpy out; float64 GPU tensors in ->
tensors out, swept in place with no copies.
"""

import numpy as np
import torch

from deepmatching_stereo_matching_amd import postproc


def _sweep(img_dis, color_weight_matrix, gausian_weight, coefficient, exclusion, size, vertical):
    dev = postproc.device_for(img_dis, color_weight_matrix, gausian_weight, coefficient)
    img, was_np = postproc.as_device(img_dis, dev)
    if img.dim() != 2:
        raise ValueError('img_dis must be a 2-D map')
    cw, _ = postproc.as_device(color_weight_matrix, dev)
    gw, _ = postproc.as_device(gausian_weight, dev)
    coef, _ = postproc.as_device(coefficient, dev)
    err = postproc.bilateral(img, cw, gw, coef, int(exclusion), size, vertical)
    if was_np:
        img_dis[...] = img.cpu().numpy()  # the reference updates img_dis in place
        return img_dis, np.float64(err.item())
    if img is not img_dis:
        img_dis.copy_(img)
    return img_dis, err


def optimize_loop_bilateral_horizon(img_dis, color_weight_matrix, gausian_weight, coefficient, alpha,
                                    exclusion, size):
    """misc/opt_loop.py:16-35 (coefficient[e, e +- 1]); alpha is unused, as in the reference."""
    return _sweep(img_dis, color_weight_matrix, gausian_weight, coefficient, exclusion, size, False)


def optimize_loop_bilateral_vertical(img_dis, color_weight_matrix, gausian_weight, coefficient, alpha,
                                     exclusion, size):
    """misc/opt_loop.py:39-58 (coefficient[e +- 1, e]); alpha is unused, as in the reference."""
    return _sweep(img_dis, color_weight_matrix, gausian_weight, coefficient, exclusion, size, True)


def make_weight(guide_img, exclusion, size, sigma):
    """misc/opt_loop.py:60-85.  The denominators are evaluated here exactly as the reference
    writes them (2.0 * sigma[k]**2 on the caller's sigma object)."""
    dev = postproc.device_for(guide_img)
    g, was_np = postproc.as_device(guide_img, dev)
    if g.dim() != 2:
        raise ValueError('guide_img must be a 2-D map')
    den_c = 2.0 * sigma[0] ** 2
    den_s = 2.0 * sigma[1] ** 2
    gauss, color = postproc.make_weight(g, int(exclusion), size, den_c, den_s)
    if was_np:
        return gauss.cpu().numpy(), color.cpu().numpy()
    return gauss, color

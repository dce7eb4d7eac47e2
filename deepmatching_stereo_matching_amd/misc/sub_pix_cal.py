"""sub_pix_cal mirror (reference: misc/sub_pix_cal.py:22-53), evaluated by dm_sub_pix_cal."""

import numpy as np
import torch

from deepmatching_stereo_matching_amd import _lib as L
from deepmatching_stereo_matching_amd import engine
from deepmatching_stereo_matching_amd.misc.optimize_loop import image_threshold  # noqa: F401  (as the reference imports it, :19)



def sub_pix_cal(arr, co_map, direction=0, ratio=100.):
    """Clamp the disparity map to [-3, 3], refine interior pixels with the quadratic vertex
    of the (score * ratio) map along ``direction`` (0 rows, 1 cols), reject |delta| > 1,
    clamp again.  float64 (h, w)."""
    dev = engine.default_device()
    a = torch.from_numpy(np.ascontiguousarray(arr, dtype=np.float64)).to(dev)
    c = torch.from_numpy(np.ascontiguousarray(co_map, dtype=np.float64)).to(dev)
    if a.shape != c.shape or a.dim() != 2:
        raise IndexError('arr and co_map must be 2-D arrays of the same shape')
    out = torch.empty_like(a)
    L.check(L.load().dm_sub_pix_cal(L.ptr(a), L.ptr(c), a.shape[0], a.shape[1], int(direction),
                                    float(ratio), L.ptr(out), L.stream_handle()), 'dm_sub_pix_cal')
    return out.cpu().numpy()

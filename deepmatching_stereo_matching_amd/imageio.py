"""Image I/O without OpenCV (cv2 is not part of this stack): Pillow readers with cv2's
channel order, and a cv2.imwrite-compatible writer for the float maps the reference saves.

cv2.imwrite on a float64 array converts each value with saturate_cast<uchar>: round half
to even (cvRound), clamp to [0, 255]; NaN becomes 0.  ``to_u8`` reproduces that.
"""

import numpy as np
from PIL import Image


def imread_bgr(path):
    """cv2.imread(path) (IMREAD_COLOR): uint8 (H, W, 3) in B, G, R order."""
    a = np.asarray(Image.open(path).convert('RGB'))
    return np.ascontiguousarray(a[:, :, ::-1])


def imread_gray(path):
    """cv2.imread(path, cv2.IMREAD_GRAYSCALE).  Single-band sources are returned as
    stored; colour sources use ITU-R 601-2 luma (Pillow 'L'), which can differ from
    cv2's fixed-point conversion by 1 (documented deviation)."""
    return np.ascontiguousarray(np.asarray(Image.open(path).convert('L')))


def to_u8(a):
    """saturate_cast<uchar> of cv2.imwrite for float / integer arrays."""
    a = np.asarray(a)
    if a.dtype == np.uint8:
        return a
    f = np.asarray(a, dtype=np.float64)
    f = np.where(np.isnan(f), 0.0, f)
    return np.clip(np.rint(f), 0, 255).astype(np.uint8)


def imwrite(path, a):
    """cv2.imwrite for a 2-D (grayscale) or (H, W, 3) B,G,R array."""
    u = to_u8(a)
    if u.ndim == 3:
        u = u[:, :, ::-1]
    Image.fromarray(np.ascontiguousarray(u)).save(path)
    return True

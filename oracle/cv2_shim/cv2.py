"""Repo-owned stand-in for the one OpenCV primitive the hot path calls.

TEST INFRASTRUCTURE ONLY.  This module is put on ``sys.path`` by
``tests/golden/make_golden.py`` so that the reference's own Python
(``misc/Feature_value.py:41`` calls ``cv2.matchTemplate``) can be imported and run
unchanged in this container, where OpenCV is not installed.  It is never imported by
the product package.

It implements ``matchTemplate`` for ``TM_CCOEFF`` / ``TM_CCOEFF_NORMED`` with OpenCV's
argument-swap rule and with the *pinned* arithmetic that the C oracle
(``oracle/dm_oracle.c``) and the HIP kernels share (DESIGN.md "Pinned ZNCC"):

    n    = ws*ws
    num  = n*sum(T*I) - sum(T)*sum(I)                    exact integer
    dT   = n*sum(T*T) - sum(T)**2 ; dI likewise           exact integer
    NORMED:  dT == 0           -> r = 1.0 for every window (OpenCV: templNorm < eps)
             a = f32(1/sqrt(f64 dT)),  b = 0 if dI == 0 else f32(1/sqrt(f64 dI))
             y = f32(num) * b ;  r = clamp(y * a, -1, 1)   products rounded to float32
             (b first, a last: r is then a monotone function of y for a fixed patch, which
             the kernels use to pool and min/max on y -- see DESIGN.md)
    CCOEFF:  r = f32(num) * f32(1/n)

OpenCV 3.4.1 itself (``environment.yml:15``) correlates in float32 via DFT/IPP and is
not bit-reproducible against any exact formula, so this boundary is pinned by the
build, not by OpenCV.
"""

import numpy as np

TM_CCOEFF = 4
TM_CCOEFF_NORMED = 5
IMREAD_GRAYSCALE = 0


def _windows(img, th, tw):
    return np.lib.stride_tricks.sliding_window_view(img, (th, tw))


def matchTemplate(image, templ, method):
    image = np.asarray(image)
    templ = np.asarray(templ)
    if image.dtype != np.uint8 or templ.dtype != np.uint8:
        raise TypeError("shim supports uint8 inputs only")
    if image.shape[0] < templ.shape[0] or image.shape[1] < templ.shape[1]:
        image, templ = templ, image  # OpenCV's needswap rule
    th, tw = templ.shape
    n = th * tw
    T = templ.astype(np.int64)
    W = _windows(image.astype(np.int64), th, tw)           # (H', W', th, tw)
    sTI = np.einsum('abij,ij->ab', W, T)
    sI = W.sum(axis=(2, 3))
    sI2 = np.einsum('abij,abij->ab', W, W)
    sT = int(T.sum())
    sT2 = int((T * T).sum())
    num = n * sTI - sT * sI
    numf = num.astype(np.float32)
    if method == TM_CCOEFF:
        c = np.float32(1.0 / n)
        return (numf * c).astype(np.float32)
    if method != TM_CCOEFF_NORMED:
        raise ValueError("shim supports TM_CCOEFF and TM_CCOEFF_NORMED only")
    dT = n * sT2 - sT * sT
    if dT == 0:
        return np.ones(num.shape, dtype=np.float32)
    dI = n * sI2 - sI * sI
    a = np.float32(1.0 / np.sqrt(np.float64(dT)))
    with np.errstate(divide='ignore'):
        b = (1.0 / np.sqrt(dI.astype(np.float64))).astype(np.float32)
    b[dI == 0] = np.float32(0.0)
    y = (numf * b).astype(np.float32)
    r = (y * a).astype(np.float32)
    return np.clip(r, np.float32(-1.0), np.float32(1.0)).astype(np.float32)

"""Python face of the CPU oracle.  TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module, as the checker (or the timed CPU baseline) -- never the product
path.  Heavy loops are in ``dm_oracle.c`` (built by ``oracle/Makefile`` into
``oracle/build/libdm_oracle.so``); the small pure-Python parts restate:

  * ``filter_map``   Matching._filter         (misc/Matching.py:224-255)
  * ``match``        Matching.__call__ with _filter hooks (misc/Matching.py:80-149, 211-222)
  * ``cut_solve``    ImageCutSolver            (misc/image_cut_solver.py:26-184)
  * ``atomic_patch`` Correlation_map._create_atomic_patch (misc/Correlation_map.py:51-67)
  * ``pyramid_stream`` / ``match_stream`` / ``corr_l0_rows``: the same pipeline without
    storing level 0 (C5 tiles, S = 256, whose float64 level 0 is 34 GB; dm_oracle.c)
  * ``bad_matching`` the row argmax of bad_matching.py:66-70
  * ``sub_pix_cal``  sub_pix_cal               (misc/sub_pix_cal.py:22-53)
  * ``optimize_loop``, ``make_weight``, ``opt_loop_bilateral``: the Gauss-Seidel loops of
    misc/optimize_loop.py:15-44 and misc/opt_loop.py:16-85 (loops in dm_oracle.c)

Parity of this oracle is pinned against ``tests/golden/*.npz`` (generated from the
reference itself by ``tests/golden/make_golden.py``) in ``tests/test_oracle_golden.py``.
"""

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, 'build', 'libdm_oracle.so')
LAM = 1.4
METHODS = {'cv2.TM_CCOEFF_NORMED': 5, 'cv2.TM_CCOEFF': 4}
CAL_MODES = {'elevation': 0, 'elevation2': 1, 'distance': 2}

_lib = None


def build():
    subprocess.run(['make', '-s', '-C', HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        L.dmo_corr_l0.argtypes = [P, P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, P]
        L.dmo_corr_l0_rows.argtypes = [P, P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                       P, ctypes.c_long, P]
        L.dmo_corr_level1_stream.argtypes = [P, P, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                             ctypes.c_int, ctypes.c_double, P]
        L.dmo_match_stream.argtypes = [P, P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_double, P, ctypes.c_int, ctypes.c_int, P]
        L.dmo_rectify_f32.argtypes = [P, ctypes.c_long, ctypes.c_double, P]
        L.dmo_rectify_f64.argtypes = [P, ctypes.c_long, ctypes.c_double]
        L.dmo_aggregate.argtypes = [P, ctypes.c_int, ctypes.c_int, P]
        L.dmo_match.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, P]
        L.dmo_cal_map.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, P]
        L.dmo_set_pow_mode.argtypes = [ctypes.c_int]
        L.dmo_set_zncc_formula.argtypes = [ctypes.c_int]
        L.dmo_zncc_formula_diff.argtypes = [P, P, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                            ctypes.c_int, P, P]
        L.dmo_pow14.argtypes = [ctypes.c_double]
        I, D = ctypes.c_int, ctypes.c_double
        L.dmo_optimize_loop.argtypes = [P, P, I, I, I, I, I, I, D]
        L.dmo_optimize_loop.restype = D
        L.dmo_make_weight.argtypes = [P, I, I, I, I, D, D, P, P]
        L.dmo_opt_loop_bilateral.argtypes = [P, P, P, P, I, I, I, I, I, I, I]
        L.dmo_opt_loop_bilateral.restype = D
        L.dmo_exp.argtypes = [D]
        L.dmo_exp.restype = D
        L.dmo_pow14.restype = ctypes.c_double
        _lib = L
    return _lib


def set_pow_mode(mode):
    """'libm' (numpy-like, default) or 'pinned' (dm_pow.h, what the GPU computes)."""
    lib().dmo_set_pow_mode({'libm': 0, 'pinned': 1}[mode])


def set_zncc_formula(name):
    """'pinned' (default: the kernels' two-multiply formula) or 'f64div'
    (f32(clamp(num / sqrt(f64 dT * f64 dI)))).  For tools/zncc_pin.py only."""
    lib().dmo_set_zncc_formula({'pinned': 0, 'f64div': 1}[name])


def zncc_formula_diff(img1, img2, ws, feature='cv2.TM_CCOEFF_NORMED'):
    """Level-0 difference between the two formulas: dict(values, max_ulp, nan_mismatch, rows,
    max_abs)."""
    img1 = np.ascontiguousarray(img1, dtype=np.uint8)
    img2 = np.ascontiguousarray(img2, dtype=np.uint8)
    H, W = img1.shape
    st = np.zeros(4, dtype=np.int64)
    ma = np.zeros(1, dtype=np.float64)
    with np.errstate(all='ignore'):
        rc = lib().dmo_zncc_formula_diff(_p(img1), _p(img2), H, W, ws, METHODS[feature], _p(st), _p(ma))
    if rc != 0:
        raise ValueError('dmo_zncc_formula_diff failed: %d' % rc)
    d = dict(zip(('values', 'max_ulp', 'nan_mismatch', 'rows'), (int(x) for x in st)))
    d['max_abs'] = float(ma[0])
    return d


def pow14(x):
    return lib().dmo_pow14(float(x))


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def corr_l0(img1, img2, ws, feature='cv2.TM_CCOEFF_NORMED'):
    """Level-0 min-max ZNCC volume (h0, w0, h0, w0) float32 (== co_map, pre-pow)."""
    img1 = np.ascontiguousarray(img1, dtype=np.uint8)
    img2 = np.ascontiguousarray(img2, dtype=np.uint8)
    H, W = img1.shape
    h0, w0 = H - ws + 1, W - ws + 1
    out = np.empty((h0, w0, h0, w0), dtype=np.float32)
    with np.errstate(all='ignore'):
        rc = lib().dmo_corr_l0(_p(img1), _p(img2), H, W, ws, METHODS[feature], _p(out))
    if rc != 0:
        raise ValueError('dmo_corr_l0 failed: %d' % rc)
    return out


def corr_l0_rows(img1, img2, ws, patches, feature='cv2.TM_CCOEFF_NORMED'):
    """Rows ``patches`` (flat p indices) of the level-0 volume: [n][h0*w0] float32, equal to
    corr_l0(...).reshape(P, P)[patches] without materialising the volume."""
    img1 = np.ascontiguousarray(img1, dtype=np.uint8)
    img2 = np.ascontiguousarray(img2, dtype=np.uint8)
    H, W = img1.shape
    P = (H - ws + 1) * (W - ws + 1)
    idx = np.ascontiguousarray(patches, dtype=np.int64).ravel()
    out = np.empty((len(idx), P), dtype=np.float32)
    with np.errstate(all='ignore'):
        rc = lib().dmo_corr_l0_rows(_p(img1), _p(img2), H, W, ws, METHODS[feature], _p(idx),
                                    len(idx), _p(out))
    if rc != 0:
        raise ValueError('dmo_corr_l0_rows failed: %d' % rc)
    return out


def pyramid_stream(img1, img2, ws, feature='cv2.TM_CCOEFF_NORMED'):
    """Levels >= 1 of Correlation_map()() without storing level 0 (dmo_corr_level1_stream,
    then the same aggregation as pyramid()): for tiles whose float64 level 0 does not fit
    the host (C5: S = 256 is 34 GB).  Returns ([None, level1, ...], iteration, N_map);
    bit-identical to pyramid(corr_l0(...)) levels >= 1."""
    img1 = np.ascontiguousarray(img1, dtype=np.uint8)
    img2 = np.ascontiguousarray(img2, dtype=np.uint8)
    H, W = img1.shape
    h0, w0 = H - ws + 1, W - ws + 1
    if min(h0, w0) == 1:          # no aggregation at all (:145)
        return [None], 1, 1
    if h0 % 2 or w0 % 2:
        raise ValueError('could not broadcast input array: map sides must halve '
                         '(misc/Correlation_map.py:96-103)')
    L = lib()
    cur = np.empty((h0 // 2, w0 // 2, h0 // 2, w0 // 2), dtype=np.float64)
    with np.errstate(all='ignore'):
        rc = L.dmo_corr_level1_stream(_p(img1), _p(img2), H, W, ws, METHODS[feature], LAM, _p(cur))
    if rc != 0:
        raise ValueError('dmo_corr_level1_stream failed: %d' % rc)
    levels, N, it = [None, cur], 2, 2
    while N < min(h0, w0):
        h, w = cur.shape[:2]
        if h % 2 or w % 2:
            raise ValueError('could not broadcast input array: map sides must halve '
                             '(misc/Correlation_map.py:96-103)')
        nxt = np.empty((h // 2, w // 2, h // 2, w // 2), dtype=np.float64)
        L.dmo_aggregate(_p(cur), h, w, _p(nxt))
        L.dmo_rectify_f64(_p(nxt), nxt.size, LAM)
        levels.append(nxt)
        cur = nxt
        N *= 2
        it += 1
    return levels, it, N


def match_stream(img1, img2, ws, levels, sub_pix=True, feature='cv2.TM_CCOEFF_NORMED'):
    """Matching()() with level 0 recomputed per pixel (dmo_match_stream); levels[0] unused.
    Bit-identical to match(pyramid(corr_l0(...))[0], sub_pix)."""
    img1 = np.ascontiguousarray(img1, dtype=np.uint8)
    img2 = np.ascontiguousarray(img2, dtype=np.uint8)
    H, W = img1.shape
    h0, w0 = H - ws + 1, W - ws + 1
    ptrs = (ctypes.c_void_p * len(levels))(*[None if lv is None else lv.ctypes.data for lv in levels])
    out = np.empty((3, h0, w0), dtype=np.float64)
    with np.errstate(all='ignore'):
        rc = lib().dmo_match_stream(_p(img1), _p(img2), H, W, ws, METHODS[feature], LAM, ptrs,
                                    len(levels), int(bool(sub_pix)), _p(out))
    if rc != 0:
        raise IndexError('list index out of range (Matching._B needs >= 2 levels)')
    return out


def atomic_patch(img, ws):
    """Correlation_map._create_atomic_patch (misc/Correlation_map.py:51-67): the overlapping
    ws x ws patch at every pixel of the trimmed image, (h0, w0, ws, ws) uint8."""
    img = np.asarray(img)
    e = (ws - 1) // 2
    H, W = img.shape
    out = np.empty((H - 2 * e, W - 2 * e, ws, ws))
    for i in range(e, H - e):
        for j in range(e, W - e):
            out[i - e, j - e] = img[i - e:i + e + 1, j - e:j + e + 1]
    return out.astype(np.uint8)


def bad_matching(l0):
    """bad_matching.py:66-70: dis[i, j] = j - argmax(co_map[i, j, i, :]) on the level-0
    min-max volume (pre-rectification); np.argmax takes the first maximum (first NaN)."""
    h0, w0 = l0.shape[:2]
    dis = np.zeros((h0, w0))
    for i in range(h0):
        for j in range(w0):
            dis[i, j] = j - np.argmax(l0[i, j, i, :])
    return dis


def pyramid(l0):
    """Correlation_map._multi_level_correlation_pyramid (misc/Correlation_map.py:132-156).
    Returns (co_map_list, iteration, N_map)."""
    h0, w0 = l0.shape[:2]
    L = lib()
    cur = np.empty(l0.shape, dtype=np.float64)
    L.dmo_rectify_f32(_p(np.ascontiguousarray(l0)), l0.size, LAM, _p(cur))
    levels = [cur]
    N, it = 1, 1
    while N < min(h0, w0):
        h, w = cur.shape[:2]
        if h % 2 or w % 2:
            raise ValueError('could not broadcast input array: map sides must halve '
                             '(misc/Correlation_map.py:96-103)')
        nxt = np.empty((h // 2, w // 2, h // 2, w // 2), dtype=np.float64)
        L.dmo_aggregate(_p(cur), h, w, _p(nxt))
        L.dmo_rectify_f64(_p(nxt), nxt.size, LAM)
        levels.append(nxt)
        cur = nxt
        N *= 2
        it += 1
    return levels, it, N


def filter_map(map_here, window, mode):
    """Matching._filter (misc/Matching.py:224-255), including its square-only d_map."""
    shp = map_here.shape
    if shp[1] >= window and shp[2] >= window:
        ex = int((window - 1) / 2)
        d_map = np.empty((shp[1], shp[1]), dtype=np.int64)
        d_map2 = np.empty((shp[1], shp[1]), dtype=np.int64)
        for i in range(d_map.shape[0]):
            for j in range(d_map.shape[1]):
                d_map[i, j] = map_here[1, i, j] - j
                d_map2[i, j] = map_here[0, i, j] - i
        red = np.mean if mode == 'average' else np.median
        for i in range(ex, shp[1] - ex):
            for j in range(ex, shp[2] - ex):
                map_here[1, i, j] = round(red(d_map[i - ex:i + ex + 1, j - ex:j + ex + 1])) + j
                map_here[0, i, j] = round(red(d_map2[i - ex:i + ex + 1, j - ex:j + ex + 1])) + i
    return map_here


def match(levels, sub_pix=True, filtering=False, filter_window_size=3, filtering_num=3,
          filtering_mode='median'):
    """Matching()() on a level list.  Without filtering the whole descent is in C; with
    filtering the per-level descent is driven from here so _filter can run between levels."""
    h0, w0 = levels[0].shape[:2]
    L = lib()
    if not filtering:
        ptrs = (ctypes.c_void_p * len(levels))(*[lv.ctypes.data for lv in levels])
        out = np.empty((3, h0, w0), dtype=np.float64)
        if L.dmo_match(ptrs, len(levels), h0, w0, int(bool(sub_pix)), _p(out)) != 0:
            raise IndexError('list index out of range (Matching._B needs >= 2 levels)')
        return out
    return _match_filtered(levels, sub_pix, filter_window_size, filtering_num, filtering_mode)


def match_from(levels, bottom, sub_pix=True, filtering=False, filter_window_size=3, filtering_num=3,
               filtering_mode='median'):
    """Matching()() with an N_map that stops the descent at level `bottom` (Matching.py:85-96,
    :133-134): the descent on levels[bottom:], then (sub_pix) _sub_pix_cal of that coarse map
    against levels[0] (Matching.py:177-209)."""
    mp = match(levels[bottom:], sub_pix=False, filtering=filtering, filter_window_size=filter_window_size,
               filtering_num=filtering_num, filtering_mode=filtering_mode)
    return _sub_pix(mp, levels[0]) if sub_pix else mp


def _near(M, pd0, pd1):
    h, w = M.shape
    win = np.zeros((3, 3))
    for a in range(3):
        for b in range(3):
            r, c = pd0 - 1 + a, pd1 - 1 + b
            if 0 <= r < h and 0 <= c < w:
                win[a, b] = M[r, c]
    m = np.unravel_index(np.argmax(win), win.shape)
    if np.max(win) < 0.0001:
        m = (1, 1)
    return pd0 + m[0] - 1, pd1 + m[1] - 1, win[m[0], m[1]] + M[pd0, pd1]


def _match_filtered(levels, sub_pix, fw, fnum, fmode):
    top = levels[-1]
    h, w = top.shape[:2]
    mp = np.zeros((3, h, w))
    for i in range(h):
        for j in range(w):
            mp[:, i, j] = _near(top[i, j], i, j)
    if fnum > 0:
        mp = filter_map(mp, fw, fmode)
        fnum -= 1
    offs = [(1, 1), (0, 1), (1, 0), (0, 0)]
    for lv in reversed(levels[:-1]):
        h, w = mp.shape[1:]
        nx = np.empty((3, 2 * h, 2 * w))
        for i in range(h):
            for j in range(w):
                b0, b1 = int(mp[0, i, j] * 2), int(mp[1, i, j] * 2)
                for o0, o1 in offs:
                    nx[:, 2 * i + o0, 2 * j + o1] = _near(lv[2 * i + o0, 2 * j + o1],
                                                         b0 + o0, b1 + o1)
        if fnum > 0:
            nx = filter_map(nx, fw, fmode)
            fnum -= 1
        mp = nx
    if sub_pix:
        mp = _sub_pix(mp, levels[0])
    return mp


def _py_index(v):
    """int(v) as the reference's list comprehension takes it (Matching.py:183); None where int()
    would raise (NaN) or the index cannot be in range."""
    if v != v or abs(v) >= 2 ** 30:
        return None
    return int(v)


def _sub_pix(mp, L0):
    """Matching._sub_pix_cal (Matching.py:177-209): the map may be a coarser level's (a
    descent that stops above level 0); co_map_list[0] is read at (i, j, row, col) of each
    entry and the bounds are level 0's window sides.  Indices behave as numpy's on
    co_map_list[0][i, j] (wrap in [-N, 0), IndexError outside [-N, N) -> the bare except)."""
    def comp(r0, r1, r_):
        return -(r1 - r_) / (2 * (r1 + r_ - 2 * r0)) if (r0 > r1 and r0 > r_) else 0

    def ok(k, n):
        return k is not None and -n <= k < n
    h0, w0 = L0.shape[2:]
    for i in range(mp.shape[1]):
        for j in range(mp.shape[2]):
            c0, c1 = _py_index(mp[0, i, j]), _py_index(mp[1, i, j])
            d_x = i - mp[0, i, j]
            if ok(c0, h0) and ok(c0 + 1, h0) and ok(c0 - 1, h0) and ok(c1, w0):
                mp[0, i, j] = i - d_x + comp(L0[i, j, c0, c1], L0[i, j, c0 + 1, c1], L0[i, j, c0 - 1, c1])
            else:
                mp[0, i, j] = i - d_x
            d_y = j - mp[1, i, j]
            if ok(c0, h0) and ok(c1, w0) and ok(c1 + 1, w0) and ok(c1 - 1, w0):
                mp[1, i, j] = j - d_y + comp(L0[i, j, c0, c1], L0[i, j, c0, c1 + 1], L0[i, j, c0, c1 - 1])
            else:
                mp[1, i, j] = j - d_y
    return mp


def cal_map(mp, mode='elevation'):
    mp = np.ascontiguousarray(mp, dtype=np.float64)
    out = np.empty(mp.shape[1:], dtype=np.float64)
    lib().dmo_cal_map(_p(mp), mp.shape[1], mp.shape[2], CAL_MODES[mode], _p(out))
    return out


def solve_pair(img1, img2, ws=5, feature='cv2.TM_CCOEFF_NORMED', sub_pix=True, **filt):
    """Correlation_map()() + Matching()() on one pair; returns (match, levels, l0)."""
    l0 = corr_l0(img1, img2, ws, feature)
    levels, _, _ = pyramid(l0)
    return match(levels, sub_pix=sub_pix, **filt), levels, l0


def cut_solve(img1, img2, image_size=(32, 32), stride=(32, 32), window_size=5,
              feature_name='cv2.TM_CCOEFF_NORMED', degree_map_mode=('elevation',),
              padding=False, sub_pix=True, filtering=False, filtering_window_size=3,
              filtering_num=3, filtering_mode='average'):
    """ImageCutSolver(...)() (misc/image_cut_solver.py:31-184).  Uncovered output cells
    (np.empty in the reference) are NaN here."""
    ex = int((window_size - 1) / 2)
    trimmed = [image_size[i] + 2 * ex for i in range(2)]
    shape = img1.shape   # self.img_shape, recorded before _padding (:46) and used by :62
    if padding:  # _padding (:73-93): img1 copied twice, img2 left zero
        a = np.zeros((img1.shape[0] + 2 * ex, img1.shape[1] + 2 * ex))
        a[ex:-ex, ex:-ex] = img1
        img1, img2 = a.astype(np.uint8), np.zeros(a.shape, dtype=np.uint8)
    n = [int(np.floor((shape[i] - trimmed[i]) / stride[i])) for i in range(2)]
    tiles = [(i, j) for j in range(n[1]) for i in range(n[0])]
    size = [stride[i] * tiles[-1][i] + image_size[i] for i in range(2)]
    d_map = np.full([len(degree_map_mode)] + size, np.nan)
    out_map = np.full(size, np.nan)
    for i, j in tiles:
        r0, c0 = stride[0] * i, stride[1] * j
        a = img1[r0:r0 + trimmed[0], c0:c0 + trimmed[1]]
        b = img2[r0:r0 + trimmed[0], c0:c0 + trimmed[1]]
        mp, _, _ = solve_pair(a, b, window_size, feature_name, sub_pix, filtering=filtering,
                              filter_window_size=filtering_window_size,
                              filtering_num=filtering_num, filtering_mode=filtering_mode)
        d_map[:, r0:r0 + image_size[0], c0:c0 + image_size[1]] = \
            np.array([cal_map(mp, m) for m in degree_map_mode])
        out_map[r0:r0 + image_size[0], c0:c0 + image_size[1]] = mp[2]
    return d_map, out_map


def image_threshold(arr, threshold=(0, 10)):
    """misc/optimize_loop.py:40-44"""
    arr = np.where(arr > threshold[1], threshold[1], arr)
    return np.where(arr < threshold[0], threshold[0], arr)


def sub_pix_cal(arr, co_map, direction=0, ratio=100.):
    """misc/sub_pix_cal.py:22-53 (disparity-domain quadratic refinement on a score map)."""
    arr = image_threshold(arr, threshold=[-3, 3]).astype(float)
    with np.errstate(all='ignore'):
        for i in range(1, arr.shape[0] - 1):
            for j in range(1, arr.shape[1] - 1):
                pl = [i + 1, j] if direction == 0 else [i, j + 1]
                mi = [i - 1, j] if direction == 0 else [i, j - 1]
                d = arr[i, j]
                r0 = co_map[i, j] * ratio
                r1 = co_map[pl[0], pl[1]] * ratio
                r_ = co_map[mi[0], mi[1]] * ratio
                dis = d - (r1 - r_) / (2 * (r1 + r_ - 2 * r0))
                if abs(d - dis) > 1:
                    dis = d
                arr[i, j] = dis
    return image_threshold(arr, threshold=[-3, 3])


# ---- Gauss-Seidel post-processing -------------------------------

def exp(x):
    """The pinned float64 exp (csrc/dm_exp.h) the post-processing kernels use."""
    return lib().dmo_exp(float(x))


def optimize_loop(img_dis, coefficient, alpha, exclusion, size):
    """misc/optimize_loop.py:15-37 -> (thresholded + swept copy, error)."""
    img = np.ascontiguousarray(image_threshold(np.asarray(img_dis, dtype=np.float64)), dtype=np.float64).copy()
    coef = np.ascontiguousarray(coefficient, dtype=np.float64)
    err = lib().dmo_optimize_loop(_p(img), _p(coef), coef.shape[1], img.shape[0], img.shape[1],
                                  int(size[0]), int(size[1]), int(exclusion), float(alpha))
    return img, np.float64(err)


def make_weight(guide_img, exclusion, size, sigma):
    """misc/opt_loop.py:60-85 -> (gausian_weight, color_weight_matrix)."""
    g = np.ascontiguousarray(guide_img, dtype=np.float64)
    e = int(exclusion)
    W = 2 * e + 1
    gauss = np.zeros((W, W))
    color = np.zeros((size[0] - e, size[1] - e, W, W))
    lib().dmo_make_weight(_p(g), g.shape[1], int(size[0]), int(size[1]), e,
                          float(2.0 * sigma[0] ** 2), float(2.0 * sigma[1] ** 2), _p(gauss), _p(color))
    return gauss, color


def opt_loop_bilateral(img_dis, color_weight_matrix, gausian_weight, coefficient, exclusion, size,
                       vertical=False):
    """misc/opt_loop.py:16-58 on a float64 copy -> (map, error)."""
    img = np.array(img_dis, dtype=np.float64, copy=True, order='C')
    cw = np.ascontiguousarray(color_weight_matrix, dtype=np.float64)
    gw = np.ascontiguousarray(gausian_weight, dtype=np.float64)
    coef = np.ascontiguousarray(coefficient, dtype=np.float64)
    err = lib().dmo_opt_loop_bilateral(_p(img), _p(cw), _p(gw), _p(coef), coef.shape[0], coef.shape[1],
                                       img.shape[1], int(size[0]), int(size[1]), int(exclusion),
                                       int(bool(vertical)))
    return img, np.float64(err)

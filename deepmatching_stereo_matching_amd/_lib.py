"""ctypes binding of libdmstereo.so (C ABI: include/dmstereo.h).

``import torch`` happens before the library is loaded so that its ``libamdhip64.so.7``
dependency resolves to the HIP runtime torch already loaded (one runtime per process:
torch's device pointers and streams are then valid in the library).

There is no fallback: if the library is missing or cannot be loaded, every entry point
raises ``DmUnavailable`` (build it with ``python -m deepmatching_stereo_matching_amd.build_ext``).
"""

import ctypes
import os
import re

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('DM_LIB_PATH') or os.path.join(HERE, 'libdmstereo.so')
HEADER = os.path.join(os.path.dirname(HERE), 'include', 'dmstereo.h')

DM_OK, DM_ERR_ARG, DM_ERR_SHAPE, DM_ERR_UNSUPPORTED, DM_ERR_HIP = 0, -1, -2, -3, -4
DM_VOLUME_F16, DM_VOLUME_MINMAX_KNOWN = 1, 2   # dm_corr_volume_ex flags
DM_POW_F32, DM_POW_Q4, DM_POW_K, DM_POW_FULL, DM_POW_Q4G, DM_POW_KG = 0, 1, 2, 3, 4, 5   # dm_pow14_variant forms
DM_TM_CCOEFF, DM_TM_CCOEFF_NORMED = 4, 5
METHODS = {'cv2.TM_CCOEFF_NORMED': DM_TM_CCOEFF_NORMED, 'cv2.TM_CCOEFF': DM_TM_CCOEFF}
CAL_MODES = {'elevation': 0, 'elevation2': 1, 'distance': 2}
DM_GS_FWD4, DM_GS_BWD4, DM_GS_BILAT = 0, 1, 2


class DmUnavailable(ImportError):
    pass


class DmError(RuntimeError):
    pass


class DmTiles(ctypes.Structure):
    _fields_ = [('d_img1', ctypes.c_void_p), ('d_img2', ctypes.c_void_p),
                ('pitch1', ctypes.c_int32), ('pitch2', ctypes.c_int32),
                ('d_origins', ctypes.c_void_p), ('T', ctypes.c_int32),
                ('h0', ctypes.c_int32), ('w0', ctypes.c_int32),
                ('ws', ctypes.c_int32), ('method', ctypes.c_int32)]


_P = ctypes.c_void_p
_I = ctypes.c_int32
_TP = ctypes.POINTER(DmTiles)
SIGNATURES = {
    'dm_abi_version': ([], ctypes.c_int),
    'dm_last_error': ([], ctypes.c_char_p),
    'dm_build_config': ([], ctypes.c_char_p),
    'dm_stats_bytes': ([_TP], ctypes.c_size_t),
    'dm_corr_stats': ([_TP, _P, _P], ctypes.c_int),
    'dm_corr_level1': ([_TP, _P, _P, _P], ctypes.c_int),
    'dm_corr_level12': ([_TP, _P, _P, _P, _P], ctypes.c_int),
    'dm_corr_volume': ([_TP, _P, _P, _P], ctypes.c_int),
    'dm_corr_volume_f16': ([_TP, _P, _P, _P], ctypes.c_int),
    'dm_corr_volume_ex': ([_TP, _P, _I, _P, _P], ctypes.c_int),
    'dm_rectify_f16': ([_P, ctypes.c_size_t, _P, _P], ctypes.c_int),
    'dm_rectify': ([_P, ctypes.c_size_t, _P, _P], ctypes.c_int),
    'dm_rectify64': ([_P, ctypes.c_size_t, _P, _P], ctypes.c_int),
    'dm_pow14_variant': ([_I, _P, ctypes.c_size_t, _P, _P], ctypes.c_int),
    'dm_aggregate': ([_P, _I, _I, _I, _I, _P, _P], ctypes.c_int),
    'dm_match': ([_TP, _P, ctypes.POINTER(ctypes.c_void_p), _I, _I, _I, _I, _I, _I, _I, _I,
                  _P, _P, _P], ctypes.c_int),
    'dm_subpix_map': ([_P, _I, _I, _I, _I, _I, _P, _P], ctypes.c_int),
    'dm_subpix_map_tiles': ([_TP, _P, _I, _I, _P, _P], ctypes.c_int),
    'dm_sub_pix_cal': ([_P, _P, _I, _I, _I, ctypes.c_double, _P, _P], ctypes.c_int),
    'dm_cal_map': ([_P, _I, _I, _I, _I, _P, _P], ctypes.c_int),
    'dm_gs_schedule': ([_I, _I, _I, _I, _I, _I, _P, _P, ctypes.POINTER(ctypes.c_int32)], ctypes.c_int),
    'dm_image_threshold': ([_P, ctypes.c_size_t, ctypes.c_double, ctypes.c_double, _P, _P], ctypes.c_int),
    'dm_optimize_loop': ([_P, _P, _I, _I, _I, _I, _I, _I, _I, ctypes.c_double, _P, _P, _I, _P, _P, _I,
                          _P, _P, _P], ctypes.c_int),
    'dm_make_weight': ([_P, _I, _I, _I, _I, _I, ctypes.c_double, ctypes.c_double, _P, _P, _P], ctypes.c_int),
    'dm_opt_loop_bilateral': ([_P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _P, _P, _I, _P, _P, _P],
                              ctypes.c_int),
    'dm_stitch': ([_P, _I, _I, _I, _I, _I, _I, ctypes.POINTER(ctypes.c_int32), _I, _P, _P, _P],
                  ctypes.c_int),
    'dm_seq_sum': ([_P, ctypes.c_int64, _P, _P], ctypes.c_int),
}

_lib = None


def header_symbols():
    """Function names declared in include/dmstereo.h."""
    txt = open(HEADER).read()
    txt = re.sub(r'/\*.*?\*/', '', txt, flags=re.S)
    return sorted(set(re.findall(r'\b(dm_[a-z0-9_]+)\s*\(', txt)))


def load(path=LIB_PATH):
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise DmUnavailable('HIP library %s is not built; run '
                            '`python -m deepmatching_stereo_matching_amd.build_ext`' % path)
    try:
        L = ctypes.CDLL(path)
    except OSError as e:
        raise DmUnavailable('cannot load %s: %s' % (path, e)) from e
    for name, (args, res) in SIGNATURES.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    _lib = L
    return L


def last_error():
    msg = load().dm_last_error()
    return msg.decode() if msg else ''


def check(rc, what=''):
    if rc == DM_OK:
        return
    msg = '%s: %s' % (what, last_error()) if what else last_error()
    if rc == DM_ERR_SHAPE:
        if 'list index out of range' in msg:
            raise IndexError(msg)
        raise ValueError(msg)
    if rc == DM_ERR_ARG:
        raise ValueError(msg)
    if rc == DM_ERR_UNSUPPORTED:
        raise NotImplementedError(msg)
    raise DmError(msg)


def stream_handle(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)

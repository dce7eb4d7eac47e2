"""The C-ABI library (include/dmstereo.h) loads and exports every declared symbol.

CPU only: no call here launches a kernel (argument validation returns before any HIP
call), so these run in the build container without a GPU.
"""
import ctypes

import pytest

from deepmatching_stereo_matching_amd import _lib as L


@pytest.fixture(scope='module')
def lib():
    return L.load()


def test_exports_every_header_symbol(lib):
    syms = L.header_symbols()
    assert len(syms) >= 13
    for s in syms:
        assert hasattr(lib, s), s
        assert s in L.SIGNATURES, 'ctypes signature missing for ' + s


def test_abi_version(lib):
    assert lib.dm_abi_version() == 110


def test_stats_bytes(lib):
    t = L.DmTiles(1, 1, 20, 20, 1, 3, 16, 16, 5, 5)
    assert lib.dm_stats_bytes(ctypes.byref(t)) == 6 * 4 * 3 * 256
    assert lib.dm_stats_bytes(None) == 0


@pytest.mark.parametrize('ws,rc,needle', [(4, L.DM_ERR_SHAPE, 'odd'), (17, L.DM_ERR_UNSUPPORTED, '15')])
def test_window_validation(lib, ws, rc, needle):
    t = L.DmTiles(1, 1, 20, 20, 1, 1, 16, 16, ws, 5)
    assert lib.dm_corr_stats(ctypes.byref(t), ctypes.c_void_p(1), None) == rc
    assert needle in L.last_error()


def test_null_and_method_validation(lib):
    assert lib.dm_corr_stats(None, None, None) == L.DM_ERR_ARG
    t = L.DmTiles(1, 1, 20, 20, 1, 1, 16, 16, 5, 3)
    assert lib.dm_corr_stats(ctypes.byref(t), ctypes.c_void_p(1), None) == L.DM_ERR_ARG
    assert 'method' in L.last_error()


def test_aggregate_odd_side_is_shape_error(lib):
    assert lib.dm_aggregate(ctypes.c_void_p(8), 1, 6, 3, 1, ctypes.c_void_p(8), None) == L.DM_ERR_SHAPE
    assert 'broadcast' in L.last_error()
    with pytest.raises(ValueError):
        L.check(L.DM_ERR_SHAPE)


def test_match_needs_two_levels(lib):
    ptrs = (ctypes.c_void_p * 1)(8)
    rc = lib.dm_match(None, None, ptrs, 1, 1, 4, 4, 1, 3, 0, 1, ctypes.c_void_p(8),
                      ctypes.c_void_p(8), None)
    assert rc == L.DM_ERR_SHAPE
    with pytest.raises(IndexError):
        L.check(rc)


def test_cal_map_and_stitch_validation(lib):
    assert lib.dm_cal_map(ctypes.c_void_p(8), 1, 4, 4, 7, ctypes.c_void_p(8), None) == L.DM_ERR_ARG
    modes = (ctypes.c_int32 * 1)(9)
    assert lib.dm_stitch(ctypes.c_void_p(8), 2, 2, 4, 4, 4, 4, modes, 1, ctypes.c_void_p(8),
                         ctypes.c_void_p(8), None) == L.DM_ERR_ARG
    assert lib.dm_sub_pix_cal(ctypes.c_void_p(8), ctypes.c_void_p(8), 4, 4, 2, 1.0,
                              ctypes.c_void_p(8), None) == L.DM_ERR_ARG

"""MI355X-native DeepMatching stereo correlation engine.

Drop-in for the hot path of Yuki-Kumon/deepmatching_stereo_matching:
``misc.Correlation_map`` / ``misc.Matching`` / ``misc.Calc_difference`` /
``misc.image_cut_solver`` / ``misc.loader`` and the ``deep_dem_mathing.py`` driver,
re-provided under ``deepmatching_stereo_matching_amd.misc`` on hand-written gfx950 HIP
kernels (``csrc/``, C ABI in ``include/dmstereo.h``).
"""

__version__ = '0.1.0'


def lib():
    """Load the HIP library (raises DmUnavailable if it is not built)."""
    from . import _lib
    return _lib.load()

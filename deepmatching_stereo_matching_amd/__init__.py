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


def alias_misc():
    """Make ``import misc.Correlation_map`` (the reference's import style,
    deep_dem_mathing.py:11-13) resolve to this package's mirror, so reference-side
    scripts run unchanged on the MI355X engine."""
    import importlib
    import sys
    pkg = importlib.import_module(__name__ + '.misc')
    sys.modules.setdefault('misc', pkg)
    for sub in ('Correlation_map', 'Matching', 'Calc_difference', 'Feature_value', 'image_cut_solver',
                'loader', 'raw_read', 'sub_pix_cal', 'optimize_loop', 'opt_loop'):
        mod = importlib.import_module('%s.misc.%s' % (__name__, sub))
        sys.modules.setdefault('misc.' + sub, mod)
    return pkg

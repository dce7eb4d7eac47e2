"""Driver mirror of the reference's deep_dem_mathing.py (stereo matching with
DeepMatching): same flags and defaults (:22-34), same steps (:37-78) and outputs
(result PNG d_map*30+100, correlation PNG score*70, the two input crops, response.npy).

    python -m deepmatching_stereo_matching_amd.deep_dem_mathing \\
        --original_image_path=a.tif --template_image_path=b.tif --image_cut_size=68,260

absl is not part of this stack: flags are parsed in absl's syntax (``--name=value``,
``--name value``, ``--flag`` / ``--noflag`` for booleans, comma lists).  Images are read
and written through Pillow (imageio.py) instead of cv2.  The correlation pyramid and the
matching run on the MI355X through the ``misc`` mirror.
"""

import argparse
import logging
import os
import sys

import numpy as np

from . import alias_misc
from .imageio import imread_bgr, imread_gray, imwrite

FLAG_DEFAULTS = [  # (name, default, kind, help): deep_dem_mathing.py:22-34
    ('original_image_path', './data/band3s.tif', 'string', 'image path of original image'),
    ('template_image_path', './data/band3bs.tif', 'string', 'image path of template image'),
    ('integrated_image_path', './data/after-before-crossdis.tif', 'string', 'image path to integrated image'),
    ('two_images_input', True, 'bool', '2 images are inputed or not'),
    ('save_name', './output/result.png', 'string', 'save name'),
    ('origin_save_name', './output/here.png', 'string', 'save name of original one'),
    ('correlation_save_name', './output/correlation.png', 'string', 'save name of correlation'),
    ('GT_save_name', './output/gt.png', 'string', 'save name of grand truth'),
    ('array_save_name', './output/response.npy', 'string', 'save name of deepmathing result'),
    ('feature_name', 'cv2.TM_CCOEFF_NORMED', 'string', 'feature name used to calculate feature map'),
    ('degree_map_mode', 'elevation', 'string', 'mode to calculate degree map'),
    ('image_cut_size', '68, 260', 'list', 'image size cut from start point'),
    ('image_cut_start', '100, 100', 'list', 'point to cut image from'),
]


def _parse_bool(v):
    s = str(v).strip().lower()
    if s in ('1', 'true', 't', 'yes', 'y'):
        return True
    if s in ('0', 'false', 'f', 'no', 'n'):
        return False
    raise argparse.ArgumentTypeError('bool flag value %r' % v)


def _parse_list(v):
    return [x.strip() for x in str(v).split(',') if x.strip()]


def parse_flags(argv):
    """absl-style flag parsing -> argparse.Namespace (lists as lists of strings)."""
    ap = argparse.ArgumentParser(prog='deep_dem_mathing', allow_abbrev=False)
    for name, default, kind, hlp in FLAG_DEFAULTS:
        if kind == 'bool':
            ap.add_argument('--' + name, nargs='?', const=True, default=default, type=_parse_bool, help=hlp)
            ap.add_argument('--no' + name, dest=name, action='store_false')
        elif kind == 'list':
            ap.add_argument('--' + name, default=_parse_list(default), type=_parse_list, help=hlp)
        else:
            ap.add_argument('--' + name, default=default, help=hlp)
    return ap.parse_args(argv)


def run(FLAGS):
    alias_misc()
    from misc.Calc_difference import Calc_difference
    from misc.Correlation_map import Correlation_map
    from misc.Matching import Matching

    size = [int(x) for x in FLAGS.image_cut_size]
    start = [int(x) for x in FLAGS.image_cut_start]
    img3 = None
    if not FLAGS.two_images_input:
        img_loaded = imread_bgr(FLAGS.integrated_image_path)
        img1_raw = img_loaded[:, :, 1]  # before
        img2_raw = img_loaded[:, :, 2]  # after
        img3_raw = img_loaded[:, :, 0]  # change map
        img3 = img3_raw[start[0]:start[0] + size[0], start[1]:start[1] + size[1]]
    else:
        img1_raw = imread_gray(FLAGS.original_image_path)
        img2_raw = imread_gray(FLAGS.template_image_path)
    img1 = np.ascontiguousarray(img1_raw[start[0]:start[0] + size[0], start[1]:start[1] + size[1]])
    img2 = np.ascontiguousarray(img2_raw[start[0]:start[0] + size[0], start[1]:start[1] + size[1]])
    logging.info('complete to load images')

    logging.info('start deepmathing')
    co_cls = Correlation_map(img1, img2, window_size=5, feature_name=FLAGS.feature_name)
    co_cls()
    cls = Matching(co_cls)
    out = cls()
    d_map = Calc_difference.cal_map(out, mode=FLAGS.degree_map_mode)

    for p in (FLAGS.save_name, FLAGS.correlation_save_name, FLAGS.origin_save_name, FLAGS.array_save_name):
        d = os.path.dirname(p)
        if d:
            os.makedirs(d, exist_ok=True)
    imwrite(FLAGS.save_name, d_map * 30 + 100)
    imwrite(FLAGS.correlation_save_name, out[2, :, :] * 70)
    imwrite(FLAGS.origin_save_name, img1)
    if os.path.isdir('./output'):  # hard-coded in the reference (:74); cv2.imwrite fails silently
        imwrite('./output/here2.png', img2)
    np.save(FLAGS.array_save_name, out)
    if img3 is not None:
        imwrite(FLAGS.GT_save_name, img3)
    logging.info('complete to save results')
    return out, d_map


def main(argv=None):
    logging.basicConfig(level=logging.INFO)
    run(parse_flags(sys.argv[1:] if argv is None else argv))


if __name__ == '__main__':
    main()

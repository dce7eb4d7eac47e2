"""deep_dem_mathing.py driver mirror: absl-style flags, cv2.imwrite conversion, the misc
import alias (CPU), and one end-to-end run against the oracle (GPU)."""
import os

import numpy as np
import pytest
from PIL import Image

from deepmatching_stereo_matching_amd import deep_dem_mathing as D
from deepmatching_stereo_matching_amd.imageio import imread_gray, to_u8


def test_flag_defaults_match_reference():
    f = D.parse_flags([])
    assert f.original_image_path == './data/band3s.tif'
    assert f.two_images_input is True
    assert f.image_cut_size == ['68', '260'] and f.image_cut_start == ['100', '100']
    assert f.feature_name == 'cv2.TM_CCOEFF_NORMED' and f.degree_map_mode == 'elevation'


def test_flag_syntax():
    f = D.parse_flags(['--image_cut_size=36,36', '--notwo_images_input', '--feature_name', 'cv2.TM_CCOEFF'])
    assert f.image_cut_size == ['36', '36'] and f.two_images_input is False
    assert f.feature_name == 'cv2.TM_CCOEFF'
    assert D.parse_flags(['--two_images_input=false']).two_images_input is False
    assert D.parse_flags(['--two_images_input']).two_images_input is True


def test_imwrite_saturate_cast():
    a = np.array([-3.0, 0.5, 1.5, 2.5, 254.5, 255.4, 300.0, np.nan, 100.49])
    assert to_u8(a).tolist() == [0, 0, 2, 2, 254, 255, 255, 0, 100]   # cvRound: half to even


def test_misc_alias_imports():
    from deepmatching_stereo_matching_amd import alias_misc
    alias_misc()
    import misc.Correlation_map
    import misc.Matching
    from misc.Calc_difference import Calc_difference
    assert misc.Correlation_map.Correlation_map.__module__.startswith('deepmatching_stereo_matching_amd')
    assert callable(Calc_difference.cal_map)


@pytest.mark.gpu
def test_driver_end_to_end(tmp_path):
    from oracle import oracle as O
    from deepmatching_stereo_matching_amd.synthetic import stereo_pair
    a, b = stereo_pair(60, 70, seed=5, dx=2)
    pa, pb = str(tmp_path / 'a.png'), str(tmp_path / 'b.png')
    Image.fromarray(a).save(pa)
    Image.fromarray(b).save(pb)
    out_dir = tmp_path / 'output'
    flags = D.parse_flags(['--original_image_path=' + pa, '--template_image_path=' + pb,
                           '--image_cut_size=36,36', '--image_cut_start=10,20',
                           '--save_name=%s/result.png' % out_dir,
                           '--correlation_save_name=%s/correlation.png' % out_dir,
                           '--origin_save_name=%s/here.png' % out_dir,
                           '--array_save_name=%s/response.npy' % out_dir])
    out, d_map = D.run(flags)
    resp = np.load(str(out_dir / 'response.npy'))
    O.set_pow_mode('pinned')
    try:
        ref, _, _ = O.solve_pair(a[10:46, 20:56], b[10:46, 20:56], 5)
    finally:
        O.set_pow_mode('libm')
    assert np.array_equal(resp, ref, equal_nan=True)
    assert np.array_equal(imread_gray(str(out_dir / 'result.png')), to_u8(d_map * 30 + 100))
    assert np.array_equal(imread_gray(str(out_dir / 'here.png')), a[10:46, 20:56])

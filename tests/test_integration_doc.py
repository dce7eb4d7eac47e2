"""The ctypes stub printed in INTEGRATION.md section 3 is executed as written (library path
substituted) and must reproduce Matching(Correlation_map(...)())() of the oracle."""
import os
import re

import numpy as np
import pytest

from deepmatching_stereo_matching_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _stub_source():
    txt = open(os.path.join(ROOT, 'INTEGRATION.md')).read()
    sec = txt[txt.index('## 3.'):txt.index('## 4.')]
    code = re.search(r'```python\n(.*?)```', sec, re.S).group(1)
    return code.replace('/path/to/deepmatching_stereo_matching_amd/libdmstereo.so', _lib.LIB_PATH)


def test_stub_compiles():
    compile(_stub_source(), 'INTEGRATION.md', 'exec')


@pytest.mark.gpu
def test_stub_matches_oracle():
    from oracle import oracle as O
    from deepmatching_stereo_matching_amd.synthetic import stereo_pair
    ns = {}
    exec(compile(_stub_source(), 'INTEGRATION.md', 'exec'), ns)
    a, b = stereo_pair(36, 36, seed=9, dx=2)
    got = ns['deepmatching_tile'](a, b, 5, 5, True)
    O.set_pow_mode('pinned')
    try:
        ref, _, _ = O.solve_pair(a, b, 5)
    finally:
        O.set_pow_mode('libm')
    assert np.array_equal(got, ref, equal_nan=True)

"""Build the gfx950 HIP library in-tree: deepmatching_stereo_matching_amd/libdmstereo.so.

    python -m deepmatching_stereo_matching_amd.build_ext

hipcc cross-compiles for gfx950 without a GPU.  The .so is git-ignored but travels to the
GPU box with the gpurun snapshot.  Floating point: -ffp-contract=off and no fast-math,
because the kernels reproduce float32/float64 rounding of the reference bit for bit.
"""

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CSRC = os.path.join(HERE, 'csrc')
LIB = os.path.join(HERE, 'libdmstereo.so')
SOURCES = [os.path.join(CSRC, 'dm_kernels.hip'), os.path.join(CSRC, 'dm_postproc.hip')]
DEPS = SOURCES + sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith('.h')) + \
    [os.path.join(REPO, 'include', 'dmstereo.h')]
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
ARCH = os.environ.get('PYTORCH_ROCM_ARCH', 'gfx950')
FLAGS = ['-O3', '-std=c++17', '-ffp-contract=off', '-fPIC', '-shared', '-Wno-pass-failed',
         '-mllvm', '-amdgpu-mfma-vgpr-form',  # MFMA C/D in VGPRs: no v_accvgpr copies per tile
         '--offload-arch=%s' % ARCH, '-I', os.path.join(REPO, 'include')]


def up_to_date():
    if not os.path.exists(LIB):
        return False
    t = os.path.getmtime(LIB)
    return all(os.path.getmtime(d) <= t for d in DEPS)


def build(force=False, verbose=False):
    if not force and up_to_date():
        return LIB
    cmd = [HIPCC] + FLAGS + SOURCES + ['-o', LIB + '.tmp']
    if verbose:
        print(' '.join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(LIB + '.tmp', LIB)
    return LIB


if __name__ == '__main__':
    build(force='--force' in sys.argv, verbose=True)
    print(LIB)

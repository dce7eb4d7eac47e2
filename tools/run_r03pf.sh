#!/bin/bash
# A/B: the level kernel with the child pows' table reads issued one pow ahead (DM_POW_PREFETCH)
R=$GRAFT_REPO_ROOT
cd $R
for pass in 1 2; do
  for lib in deepmatching_stereo_matching_amd/libdmstereo.so deepmatching_stereo_matching_amd/ab/libdm_pf.so; do
    echo "== pass $pass $lib"
    DM_LIB_PATH=$R/$lib timeout -k 10 120 python3 tools/kbench.py --variants l12 --rounds 5 2>&1 | grep -v amdgpu.ids || exit 1
    DM_LIB_PATH=$R/$lib timeout -k 10 120 python3 tools/kbench.py --variants l12 --rounds 3 --tile 256 --grid 2 2>&1 | grep -v amdgpu.ids || exit 1
  done
done

#!/bin/bash
# Round 6: the price of the C3 level kernel's L2 read traffic (ablations bwrow0 / strow0: the same
# load instructions served from the CU's vector cache; results wrong) against the in-tree kernel
# (head), same box, interleaved, 3 passes.
set -uo pipefail
R=$GRAFT_REPO_ROOT
cd $R
for pass in 1 2 3; do
  for lib in abx/libdm_head.so abx/libdm_bwrow0.so abx/libdm_strow0.so; do
    echo "== pass $pass $(basename $lib)"
    DM_LIB_PATH=$R/$lib timeout -k 10 120 python3 tools/kbench.py --variants l12 --rounds 10 --tile 128 2>&1 | grep -v amdgpu.ids || exit 1
  done
done > gpurun_out/r06m_l2traffic_ab.txt 2>&1

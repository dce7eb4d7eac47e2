#!/bin/bash
# Round 6: the strip kernel's pow-table fill priced by ablation (nofill, results wrong) against
# the in-tree kernel (head), C2 and C5-size tiles, same box, interleaved.
set -uo pipefail
R=$GRAFT_REPO_ROOT
cd $R
for pass in 1 2 3; do
  for lib in abx/libdm_head.so abx/libdm_nofill.so; do
    echo "== pass $pass $(basename $lib)"
    DM_LIB_PATH=$R/$lib timeout -k 10 120 python3 tools/kbench.py --variants l12 --rounds 8 --tile 64 2>&1 | grep -v amdgpu.ids || exit 1
    DM_LIB_PATH=$R/$lib timeout -k 10 120 python3 tools/kbench.py --variants l12 --rounds 3 --tile 256 --grid 4 2>&1 | grep -v amdgpu.ids || exit 1
  done
done > gpurun_out/r06i_nofill_ab.txt 2>&1

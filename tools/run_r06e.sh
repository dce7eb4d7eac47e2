#!/bin/bash
# Round 6: the persistent C2 level-kernel grid (DM_C2_ITERS=4) against the round-5 grid (head),
# C2 and C5-size tiles, same box, interleaved, level-2 sha256 printed for each.
set -uo pipefail
R=$GRAFT_REPO_ROOT
cd $R
for pass in 1 2 3; do
  for lib in ab6/libdm_head.so ab6/libdm_pers4.so; do
    echo "== pass $pass $(basename $lib)"
    DM_LIB_PATH=$R/$lib timeout -k 10 120 python3 tools/kbench.py --variants l12 --rounds 8 --tile 64 --sha 2>&1 | grep -v amdgpu.ids || exit 1
    DM_LIB_PATH=$R/$lib timeout -k 10 120 python3 tools/kbench.py --variants l12 --rounds 3 --tile 256 --grid 4 --sha 2>&1 | grep -v amdgpu.ids || exit 1
  done
done > gpurun_out/r06e_c2pers_ab.txt 2>&1

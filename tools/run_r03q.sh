#!/bin/bash
# L1S = false level-kernel instances (no runtime level-1 branch in the row-pair body) vs r03p
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_c3_golden.py tests/test_c3_batch.py tests/test_c5_tile.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03q_gputest.log 2>&1 || exit 1
DM_LIB_PATH=$R/abl/lib_yb.so timeout -k 10 600 python -u -m pytest tests/test_c3_batch.py tests/test_c5_tile.py tests/test_c3_golden.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03q_gputest_yb.log 2>&1 || exit 1
for pass in 1 2; do
  for lib in abl/lib_seg.so abl/lib_l1s.so abl/lib_yb.so; do
    echo "== pass $pass $lib C3"
    DM_LIB_PATH=$R/$lib timeout -k 10 120 python3 tools/kbench.py --variants l12 --rounds 3 2>&1 | grep -v amdgpu.ids || exit 1
  done
done > gpurun_out/r03q_ab.txt
for lib in abl/lib_seg.so abl/lib_l1s.so abl/lib_yb.so; do
  echo "== $lib C5"
  DM_LIB_PATH=$R/$lib timeout -k 10 200 python3 tools/kbench.py --variants l12 --rounds 2 --tile 256 --grid 16 2>&1 | grep -v amdgpu.ids || exit 1
done >> gpurun_out/r03q_ab.txt

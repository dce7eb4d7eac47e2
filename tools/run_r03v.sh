#!/bin/bash
# two cell blocks per workgroup at S = 64 (C2, GW = 4) vs the r03p build: parity, then A/B
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03v_gputest.log 2>&1 || exit 1
for pass in 1 2; do
  for lib in abl/lib_seg.so abl/lib_nb.so; do
    echo "== pass $pass $lib C2"
    DM_LIB_PATH=$R/$lib timeout -k 10 120 python3 tools/kbench.py --variants l12 --rounds 5 --tile 64 --grid 8 2>&1 | grep -v amdgpu.ids || exit 1
    echo "== pass $pass $lib C3"
    DM_LIB_PATH=$R/$lib timeout -k 10 120 python3 tools/kbench.py --variants l12 --rounds 3 2>&1 | grep -v amdgpu.ids || exit 1
  done
done > gpurun_out/r03v_ab.txt
for lib in abl/lib_seg.so abl/lib_nb.so; do
  DM_LIB_PATH=$R/$lib timeout -k 10 200 python3 bench.py --config c2 --no-cpu-baseline > gpurun_out/r03v_bench_c2_$(basename $lib .so).json 2>/dev/null || exit 1
done

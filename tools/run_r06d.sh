#!/bin/bash
# Round 6: the pruned C3 level kernel (k_level12_prune) against k_level1_mfq, same box,
# interleaved, the level-2 sha256 of each printed (must be equal), and the pow forms' GPU test.
set -uo pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 120 python -u -m pytest -x -q --timeout 100 --timeout-method thread -m gpu tests/test_pow_gpu.py > gpurun_out/r06d_powtest.log 2>&1 || exit 1
for pass in 1 2; do
  for lib in ab6/libdm_prune0.so ab6/libdm_prune1.so; do
    echo "== pass $pass $(basename $lib) C3"
    DM_LIB_PATH=$R/$lib timeout -k 10 120 python3 tools/kbench.py --variants l12 --rounds 6 --sha 2>&1 | grep -v amdgpu.ids || exit 1
  done
done > gpurun_out/r06d_prune_ab.txt 2>&1

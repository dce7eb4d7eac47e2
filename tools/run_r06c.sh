#!/bin/bash
# Round 6, first GPU pass: the level kernel's PMC work pass (C3), the pruning price (papprox /
# papprox2 ablations against the in-tree build, C3), the C2 strip kernel with wave-level block
# syncs against round 5's workgroup barriers (ssync), the C5 forecast, the shard GPU test.
set -uo pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_MFMA_MOPS_I8 SQ_INSTS_MFMA SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_TRANS_F32 --output-format csv -d $R/gpurun_out/r06c_work/l12_c3_work -o run -- python3 $R/tools/kbench.py --variants l12 --rounds 1 --tile 128 --grid 8 > $R/gpurun_out/r06c_work.log 2>&1 || exit 1
cd $R
for pass in 1 2; do
  for lib in deepmatching_stereo_matching_amd/libdmstereo.so ab6/libdm_papprox.so ab6/libdm_papprox2.so; do
    echo "== pass $pass $(basename $lib) C3"
    DM_LIB_PATH=$R/$lib timeout -k 10 120 python3 tools/kbench.py --variants l12 --rounds 6 --sha 2>&1 | grep -v amdgpu.ids || exit 1
  done
  for lib in deepmatching_stereo_matching_amd/libdmstereo.so ab6/libdm_ssync.so; do
    echo "== pass $pass $(basename $lib) C2"
    DM_LIB_PATH=$R/$lib timeout -k 10 120 python3 tools/kbench.py --variants l12 --rounds 8 --tile 64 --sha 2>&1 | grep -v amdgpu.ids || exit 1
  done
done > gpurun_out/r06c_ab.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/c5_share.py --steps 4 --warmup 2 > gpurun_out/r06c_c5_share.json 2> gpurun_out/r06c_c5_share.err || exit 1
timeout -k 10 200 python -u -m pytest -x -q --timeout 180 --timeout-method thread -m gpu tests/test_shard_gpu.py > gpurun_out/r06c_gputest.log 2>&1

#!/bin/bash
# Round 6 final tree: the bench lines (default C3 with c5_split, C2, C5), the rocprofv3 kernel trace
# of the default bench (tools/run_prof.sh), and the PMC work pass of the three level-kernel shapes.
set -uo pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/r06g_bench.json 2> gpurun_out/r06g_bench.err || exit 1
echo "bench done"
timeout -k 10 300 python -u bench.py --config c2 --no-cpu-baseline > gpurun_out/r06g_bench_c2.json 2> gpurun_out/r06g_bench_c2.err || exit 1
echo "c2 done"
timeout -k 10 400 python -u bench.py --config c5 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r06g_bench_c5.json 2> gpurun_out/r06g_bench_c5.err || exit 1
echo "c5 done"
timeout -k 10 500 bash tools/run_prof.sh r06g > gpurun_out/r06g_prof.log 2>&1 || exit 1
echo "prof done"
cd /tmp && export TMPDIR=/tmp
WORK="SQ_INSTS_VALU_MFMA_MOPS_I8 SQ_INSTS_MFMA SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_TRANS_F32"
for s in "128 8 l12_c3" "64 8 l12_c2" "256 16 l12_c5"; do
  set -- $s
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $WORK --output-format csv -d $R/gpurun_out/r06g_work/${3}_work -o run -- python3 $R/tools/kbench.py --variants l12 --rounds 1 --tile $1 --grid $2 > $R/gpurun_out/r06g_work_$3.log 2>&1 || exit 1
  echo "work $3 done"
done

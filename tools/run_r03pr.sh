#!/bin/bash
# A/B: tail kernels at raised wave priority (DM_TAIL_PRIO build) vs default, pipelined C3 bench
R=$GRAFT_REPO_ROOT
cd $R
B="python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-volume --no-k-level"
for pass in 1 2; do
  for lib in deepmatching_stereo_matching_amd/libdmstereo.so deepmatching_stereo_matching_amd/ab/libdm_prio.so; do
    echo "== pass $pass $lib"
    DM_LIB_PATH=$R/$lib timeout -k 10 120 $B 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('ms/pair %.3f  level kernel %.3f' % (d['ms_per_pair'], d['roofline']['ms']))" || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp && \
DM_LIB_PATH=$R/deepmatching_stereo_matching_amd/ab/libdm_prio.so timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r03pr_prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-volume --no-k-level > $R/gpurun_out/r03pr_bench_traced.json 2> $R/gpurun_out/r03pr_bench_traced.err && \
cd $R && python3 tools/gap_trace.py gpurun_out/r03pr_prof > gpurun_out/r03pr_gaps.txt 2>&1

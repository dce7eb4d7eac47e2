#!/bin/bash
# packed window statistics {sum(I'), b_q} (one 8-B load) + dword template loads in the on-demand
# matching kernels: GPU parity suite, then same-box A/B of the pipelined C3 bench
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03sq_gputest.log 2>&1 || exit 1
B="python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-volume --no-k-level"
for pass in 1 2 3; do
  for lib in deepmatching_stereo_matching_amd/ab/libdm_base.so deepmatching_stereo_matching_amd/libdmstereo.so; do
    echo "== pass $pass $lib"
    DM_LIB_PATH=$R/$lib timeout -k 10 120 $B 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('ms/pair %.3f  level kernel %.3f' % (d['ms_per_pair'], d['roofline']['ms']))" || exit 1
    DM_BENCH_DIAG=nomatch DM_LIB_PATH=$R/$lib timeout -k 10 120 $B 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('  nomatch ms/pair %.3f  level kernel %.3f' % (d['ms_per_pair'], d['roofline']['ms']))" || exit 1
  done
done

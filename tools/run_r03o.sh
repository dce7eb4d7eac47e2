#!/bin/bash
# round-3 build with the 20 KB level kernel: GPU suite, PMC passes, bench lines, trace
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03o_gputest.log 2>&1 && \
timeout -k 10 400 bash tools/pmc_r03.sh r03o l12_c3 l12_c5 > gpurun_out/r03o_pmc.log 2>&1 && \
timeout -k 10 200 python3 bench.py > gpurun_out/r03o_bench.json 2> gpurun_out/r03o_bench.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r03o_prof -o run -- python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/r03o_bench_profiled.json 2> $R/gpurun_out/r03o_bench_profiled.err && \
cd $R && timeout -k 10 300 python3 bench.py --config c5 > gpurun_out/r03o_bench_c5.json 2> gpurun_out/r03o_bench_c5.err && \
timeout -k 10 200 python3 bench.py --config c2 > gpurun_out/r03o_bench_c2.json 2> gpurun_out/r03o_bench_c2.err && \
timeout -k 10 300 python3 bench.py --config c4 --no-cpu-baseline > gpurun_out/r03o_bench_c4.json 2> gpurun_out/r03o_bench_c4.err

#!/bin/bash
# round-3 build after the C2 workgroup change: GPU suite, smoke, PMC passes, bench lines, trace
R=$GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03w_gputest.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r03w_smoke.log 2>&1 && \
timeout -k 10 500 bash tools/pmc_r03.sh r03w l12_c3 l12_c5 l12_c2 > gpurun_out/r03w_pmc.log 2>&1 && \
timeout -k 10 200 python3 bench.py > gpurun_out/r03w_bench.json 2> gpurun_out/r03w_bench.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r03w_prof -o run -- python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/r03w_bench_profiled.json 2> $R/gpurun_out/r03w_bench_profiled.err && \
cd $R && timeout -k 10 300 python3 bench.py --config c5 > gpurun_out/r03w_bench_c5.json 2> gpurun_out/r03w_bench_c5.err && \
timeout -k 10 200 python3 bench.py --config c2 > gpurun_out/r03w_bench_c2.json 2> gpurun_out/r03w_bench_c2.err && \
timeout -k 10 300 python3 bench.py --config c4 --no-cpu-baseline > gpurun_out/r03w_bench_c4.json 2> gpurun_out/r03w_bench_c4.err && \
timeout -k 10 300 python3 tools/postbench.py > gpurun_out/r03w_postbench.json 2> gpurun_out/r03w_postbench.err

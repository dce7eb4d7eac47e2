R=$GRAFT_REPO_ROOT
timeout -k 10 900 bash tools/pmc_r03.sh r03g > gpurun_out/r03g_pmc.log 2>&1 && \
timeout -k 10 200 python3 bench.py > gpurun_out/r03g_bench.json 2> gpurun_out/r03g_bench.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r03g_prof -o run -- python3 $R/bench.py > $R/gpurun_out/r03g_bench_profiled.json 2> $R/gpurun_out/r03g_bench_profiled.err && \
cd $R && timeout -k 10 300 python3 bench.py --config c5 > gpurun_out/r03g_bench_c5.json 2> gpurun_out/r03g_bench_c5.err

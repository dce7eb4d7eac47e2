R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_pow_gpu.py tests/test_abi.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03m_powtest.log 2>&1 && \
timeout -k 10 600 bash tools/pmc_r03.sh r03m l12_c3 l12_c5 > gpurun_out/r03m_pmc.log 2>&1 && \
timeout -k 10 200 python3 bench.py > gpurun_out/r03m_bench.json 2> gpurun_out/r03m_bench.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r03m_prof -o run -- python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/r03m_bench_profiled.json 2> $R/gpurun_out/r03m_bench_profiled.err && \
cd $R && timeout -k 10 300 python3 bench.py --config c5 > gpurun_out/r03m_bench_c5.json 2> gpurun_out/r03m_bench_c5.err && \
cd $R && timeout -k 10 700 bash tools/tail_ab.sh > gpurun_out/r03m_tail_ab.txt 2>&1

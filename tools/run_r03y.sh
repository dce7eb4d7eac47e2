#!/bin/bash
# timeline of the pipelined C3 bench (tools/gap_trace.py) + the extended flat-patch test
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k flat_patches > gpurun_out/r03y_flat.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r03y_prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-volume --no-k-level > $R/gpurun_out/r03y_bench_traced.json 2> $R/gpurun_out/r03y_bench_traced.err && \
cd $R && python3 tools/gap_trace.py gpurun_out/r03y_prof > gpurun_out/r03y_gaps.txt 2>&1 && \
timeout -k 10 200 python3 bench.py --streams 1 --no-cpu-baseline --no-volume --no-k-level > gpurun_out/r03y_bench_s1.json 2> gpurun_out/r03y_bench_s1.err

#!/bin/bash
# round-3 final build (clamp-bit normalisation, one-wave tail workgroups): GPU suite, smoke, PMC
# passes of the level kernel (C3, C5, C2), bench lines (C3 default, profiled, C5, C2, C4), trace,
# post-processing bench
R=$GRAFT_REPO_ROOT
T=${1:-r03fin}
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gputest.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1 && \
timeout -k 10 500 bash tools/pmc_r03.sh $T l12_c3 l12_c5 l12_c2 > gpurun_out/${T}_pmc.log 2>&1 && \
timeout -k 10 200 python3 bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_prof -o run -- python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/${T}_bench_profiled.json 2> $R/gpurun_out/${T}_bench_profiled.err && \
cd $R && python3 tools/gap_trace.py gpurun_out/${T}_prof > gpurun_out/${T}_gaps.txt 2>&1 && \
timeout -k 10 300 python3 bench.py --config c5 > gpurun_out/${T}_bench_c5.json 2> gpurun_out/${T}_bench_c5.err && \
timeout -k 10 200 python3 bench.py --config c2 > gpurun_out/${T}_bench_c2.json 2> gpurun_out/${T}_bench_c2.err && \
timeout -k 10 300 python3 bench.py --config c4 --no-cpu-baseline > gpurun_out/${T}_bench_c4.json 2> gpurun_out/${T}_bench_c4.err && \
timeout -k 10 300 python3 tools/postbench.py > gpurun_out/${T}_postbench.json 2> gpurun_out/${T}_postbench.err

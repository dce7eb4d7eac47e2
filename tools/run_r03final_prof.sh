#!/bin/bash
# rocprofv3 kernel trace + stats of the final tree's default bench command, the by-grid split
# and the bench-vs-trace cross-check of the level kernel's launch times.
#   usage (GPU box): bash tools/run_r03final_prof.sh
set -euo pipefail
R=$GRAFT_REPO_ROOT
T=r03final
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_prof -o run -- python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/${T}_bench_profiled.json 2> $R/gpurun_out/${T}_bench_profiled.err
cd $R
python3 tools/kstats.py gpurun_out/${T}_prof > gpurun_out/${T}_kernel_stats_by_grid.csv
python3 tools/level_launches.py gpurun_out/${T}_prof gpurun_out/${T}_bench_profiled.json "$T" > gpurun_out/${T}_level_kernel_launches.txt
python3 tools/gap_trace.py gpurun_out/${T}_prof > gpurun_out/${T}_gaps.txt
cp $(find gpurun_out/${T}_prof -name '*kernel_stats.csv' | head -1) gpurun_out/${T}_kernel_stats.csv

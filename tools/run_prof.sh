#!/bin/bash
# rocprofv3 kernel trace + stats of the default bench command, the by-grid split, the
# bench-vs-trace cross-check of the level kernel's launch times and the gap timeline, then
# (optionally) the PMC passes of tools/pmc_r03.sh for the roofline fields.
#   usage (GPU box): bash tools/run_prof.sh <tag> [pmc shapes...]     -> gpurun_out/<tag>_*
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
T=$1; shift
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_prof -o run -- python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/${T}_bench_profiled.json 2> $R/gpurun_out/${T}_bench_profiled.err
cd $R
python3 tools/kstats.py gpurun_out/${T}_prof > gpurun_out/${T}_kernel_stats_by_grid.csv
python3 tools/level_launches.py gpurun_out/${T}_prof gpurun_out/${T}_bench_profiled.json "$T" > gpurun_out/${T}_level_kernel_launches.txt
python3 tools/gap_trace.py gpurun_out/${T}_prof > gpurun_out/${T}_gaps.txt
cp $(find gpurun_out/${T}_prof -name '*kernel_stats.csv' | head -1) gpurun_out/${T}_kernel_stats.csv
rm -rf gpurun_out/${T}_prof
if [ $# -gt 0 ]; then bash tools/pmc_r03.sh $T "$@"; fi

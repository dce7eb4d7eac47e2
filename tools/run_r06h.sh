#!/bin/bash
# C2 pipeline study: kernel trace + gap timeline of the C2 bench line, and the C2 line at 1 / 2 / 3
# streams (same box, interleaved twice).
set -uo pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for rep in 1 2; do
  for s in 2 3 1; do
    timeout -k 10 200 python -u bench.py --config c2 --no-cpu-baseline --streams $s > gpurun_out/r06h_c2_s${s}_${rep}.json 2> gpurun_out/r06h_c2_s${s}_${rep}.err || exit 1
    echo "c2 streams $s rep $rep done"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r06h_c2_prof -o run -- python3 $R/bench.py --config c2 --no-cpu-baseline > $R/gpurun_out/r06h_c2_profiled.json 2> $R/gpurun_out/r06h_c2_profiled.err || exit 1
cd $R
python3 tools/gap_trace.py gpurun_out/r06h_c2_prof > gpurun_out/r06h_c2_gaps.txt || exit 1
python3 tools/kstats.py gpurun_out/r06h_c2_prof > gpurun_out/r06h_c2_kernel_stats_by_grid.csv || exit 1
rm -rf gpurun_out/r06h_c2_prof
echo done

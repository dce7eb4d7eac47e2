# round 5: rocprofv3 kernel trace + stats of the C2 and C5 bench lines (the strip level kernel),
# with the level-kernel launch cross-check -> gpurun_out/r05s_{c2,c5}_*
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for c in c2 c5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r05s_${c}_prof -o run -- \
      python3 $R/bench.py --config $c --no-cpu-baseline --no-volume > $R/gpurun_out/r05s_${c}_bench_profiled.json 2> $R/gpurun_out/r05s_${c}_bench_profiled.err || exit 1
  (cd $R && python3 tools/kstats.py gpurun_out/r05s_${c}_prof > gpurun_out/r05s_${c}_kernel_stats_by_grid.csv &&
   python3 tools/level_launches.py gpurun_out/r05s_${c}_prof gpurun_out/r05s_${c}_bench_profiled.json r05s_$c > gpurun_out/r05s_${c}_level_kernel_launches.txt &&
   cp $(find gpurun_out/r05s_${c}_prof -name '*kernel_stats.csv' | head -1) gpurun_out/r05s_${c}_kernel_stats.csv &&
   rm -rf gpurun_out/r05s_${c}_prof) || exit 1
done
echo done

# round 4: kernel trace of the C2 line (the tail's composition in the gaps between level kernels)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r04x_prof -o run -- python3 $R/bench.py --config c2 --no-cpu-baseline --no-volume > $R/gpurun_out/r04x_bench_c2.json 2> $R/gpurun_out/r04x.err || exit 1
cd $R
python3 tools/gap_trace.py gpurun_out/r04x_prof > gpurun_out/r04x_c2_gaps.txt || exit 1
python3 tools/kstats.py gpurun_out/r04x_prof > gpurun_out/r04x_c2_kernel_stats_by_grid.csv || exit 1
rm -rf gpurun_out/r04x_prof
echo done

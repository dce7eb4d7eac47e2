R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 200 rocprofv3 --kernel-trace --hip-trace --output-format csv -d $R/gpurun_out/r03j_prof -o run -- python3 $R/bench.py --streams 3 --level-stream 1 --stats-stream 1 --steps 10 --warmup 3 --no-cpu-baseline --no-volume --no-k-level > $R/gpurun_out/r03j_bench_prof.json 2>/dev/null

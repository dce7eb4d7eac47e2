R=$GRAFT_REPO_ROOT
timeout -k 10 700 bash tools/pipe_ab.sh > gpurun_out/r03i_pipe_ab.txt 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r03i_prof -o run -- python3 $R/bench.py --streams 3 --level-stream 1 --stats-stream 1 --steps 10 --warmup 3 --no-cpu-baseline --no-volume --no-k-level > $R/gpurun_out/r03i_bench_prof.json 2>/dev/null && \
cd $R && timeout -k 10 200 python3 tools/kbench.py --variants l12 --rounds 2 --tile 256 --grid 16 > gpurun_out/r03i_c5_nw8.txt 2>&1 && \
DM_MFQ_NWMAX=4 timeout -k 10 200 python3 tools/kbench.py --variants l12 --rounds 2 --tile 256 --grid 16 > gpurun_out/r03i_c5_nw4.txt 2>&1

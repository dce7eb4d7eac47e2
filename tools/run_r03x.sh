#!/bin/bash
# round-3 re-entry: GPU suite + smoke on the rebuilt tree (clamp-bit normalisation, norm_clamp),
# same-box A/B of DM_MFQ_CLAMP, power/clock samples over a sustained C3 bench, default bench
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03x_gputest.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r03x_smoke.log 2>&1 && \
timeout -k 10 200 python3 tools/kbench.py --variants l12,l12+DM_MFQ_CLAMP=0 --rounds 6 > gpurun_out/r03x_clamp_ab.txt 2>&1 && \
timeout -k 10 200 python3 tools/kbench.py --variants l12,l12+DM_MFQ_CLAMP=0 --rounds 4 --tile 256 --grid 2 >> gpurun_out/r03x_clamp_ab.txt 2>&1 && \
rocm-smi --showpower --showclocks --showtemp --showmaxpower --json > gpurun_out/r03x_smi_idle.json 2>&1; \
timeout -k 10 200 python3 tools/power_watch.py gpurun_out/r03x_power_c3.jsonl -- python3 bench.py --steps 2500 --warmup 5 --no-volume --no-cpu-baseline --no-k-level > gpurun_out/r03x_bench_long.json 2> gpurun_out/r03x_bench_long.err && \
timeout -k 10 200 python3 bench.py > gpurun_out/r03x_bench.json 2> gpurun_out/r03x_bench.err

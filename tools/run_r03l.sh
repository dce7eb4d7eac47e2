R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03l_gputest.log 2>&1 && \
timeout -k 10 200 python3 tools/kbench.py --variants l12,l12+DM_MFQ_GW=2 --rounds 3 > gpurun_out/r03l_c3_gw.txt 2>&1 && \
timeout -k 10 600 bash tools/pipe_ab.sh > gpurun_out/r03l_pipe_ab.txt 2>&1 && \
timeout -k 10 200 python3 bench.py > gpurun_out/r03l_bench.json 2> gpurun_out/r03l_bench.err

#!/bin/bash
# binade-segmented sequence sum: parity, then the post-processing timer with both sums
timeout -k 10 400 python -u -m pytest tests/test_seq_sum_gpu.py tests/test_postproc.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03p_gputest.log 2>&1 || exit 1
DM_SEQ_SUM=chain timeout -k 10 300 python3 tools/postbench.py > gpurun_out/r03p_postbench_chain.json 2> gpurun_out/r03p_postbench_chain.err || exit 1
timeout -k 10 300 python3 tools/postbench.py > gpurun_out/r03p_postbench.json 2> gpurun_out/r03p_postbench.err

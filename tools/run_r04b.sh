# round 4: the pruned library + the timed-path output checks, then the full GPU suite and bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest tests/test_bench_steps.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r04b_steps.log 2>&1 &&
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread --deselect tests/test_bench_steps.py > gpurun_out/r04b_gputest.log 2>&1 &&
timeout -k 10 300 python3 bench.py > gpurun_out/r04b_bench.json 2> gpurun_out/r04b_bench.err

set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r04a_bench.json 2> gpurun_out/r04a_bench.err &&
timeout -k 10 120 python3 tools/kbench.py --variants l12 --rounds 5 > gpurun_out/r04a_kbench.txt 2>&1

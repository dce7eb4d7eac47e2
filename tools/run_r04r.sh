# round 4: PMC passes of the binary16 min/max-known C3 volume (4-wave workgroups), then the
# default bench line and C2 lines (chained / overlapped level kernels) on the final build
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
bash tools/pmc_r03.sh r04r v16mm_c3 || exit 1
timeout -k 10 300 python3 bench.py > gpurun_out/r04r_bench.json 2> gpurun_out/r04r_bench.err || exit 1
timeout -k 10 300 python3 bench.py --config c2 --no-cpu-baseline > gpurun_out/r04r_bench_c2.json 2> gpurun_out/r04r_bench_c2.err || exit 1
timeout -k 10 300 python3 bench.py --config c2 --no-cpu-baseline --no-volume --chain-levels 0 > gpurun_out/r04r_bench_c2_ov2.json 2>> gpurun_out/r04r_bench_c2.err || exit 1
timeout -k 10 300 python3 bench.py --config c2 --no-cpu-baseline --no-volume --chain-levels 0 --streams 3 > gpurun_out/r04r_bench_c2_ov3.json 2>> gpurun_out/r04r_bench_c2.err || exit 1
echo done

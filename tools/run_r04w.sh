# round 4 final check on the final tree: the GPU suite, then the default bench line (its
# roofline fields must come out non-null: profiles made on these kernels)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r04w_gputest.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py > gpurun_out/r04w_bench.json 2> gpurun_out/r04w_bench.err || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04w_smoke.log 2>&1 || exit 1
echo done

# round 4 final (frozen build): the full GPU suite, then the rocprofv3 trace + stats of the
# default bench, the level-kernel launch cross-check, the gap timeline, and the PMC passes of
# the level kernel (C3, C2, C5) and the C3 volumes -> gpurun_out/r04p_*, gpurun_out/pmc3_r04p/
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r04p_gputest.log 2>&1 || exit 1
bash tools/run_prof.sh r04p l12_c3 l12_c2 l12_c5 v16_c3 v32_c3 v16mm_c3 v32mm_c3 || exit 1
echo done

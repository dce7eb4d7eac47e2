# round 5 final (frozen build): the rocprofv3 trace + stats of the default bench, the level-kernel
# launch cross-check, the gap timeline, and the PMC passes of the level kernel (C3, C2, C5) and
# of the C3 and C5 volumes -> gpurun_out/r05p_*, gpurun_out/pmc3_r05p/
set -o pipefail
mkdir -p gpurun_out
bash tools/run_prof.sh r05p l12_c3 l12_c2 l12_c5 v16_c3 v32_c3 v16mm_c3 v32mm_c3 v16_c5 v32_c5 v16mm_c5 v32mm_c5 || exit 1
echo done

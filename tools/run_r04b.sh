# round 4: full GPU suite (the timed-path output checks first), then the bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r04b_gputest.log 2>&1 &&
timeout -k 10 300 python3 bench.py > gpurun_out/r04b_bench.json 2> gpurun_out/r04b_bench.err &&
# level-kernel ablation upper bounds (tools/abl_build.sh; their results are wrong by design)
L=deepmatching_stereo_matching_amd/libdmstereo.so
for pass in 1 2; do
  for lib in $L ab/libdm_nobar.so ab/libdm_nopow.so ab/libdm_nosw1.so; do
    echo "== pass $pass $lib" >> gpurun_out/r04b_abl.txt
    DM_LIB_PATH=$PWD/$lib timeout -k 10 120 python3 tools/kbench.py --variants l12 --rounds 3 >> gpurun_out/r04b_abl.txt 2>&1 || exit 1
  done
done

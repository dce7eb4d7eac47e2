# round 4: the full GPU suite on the working tree, then the on-demand level-1 step with 3
# sum-pows per wave (working tree) against the last commit (ab/libdm_head.so): C2 and C3 lines
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r04t_gputest.log 2>&1 || exit 1
for pass in 1 2; do
  for lib in deepmatching_stereo_matching_amd/libdmstereo.so ab/libdm_head.so; do
    for c in c2 c3; do
      echo "== pass $pass $lib $c" >> gpurun_out/r04t_l1.txt
      DM_LIB_PATH=$PWD/$lib timeout -k 10 200 python3 bench.py --config $c --no-cpu-baseline --no-volume --no-c5-split >> gpurun_out/r04t_l1.txt 2>> gpurun_out/r04t.err || exit 1
    done
  done
done
echo done

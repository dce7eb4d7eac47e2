# round 4: the S = 256 level kernel with two cell blocks per workgroup (ab/libdm_c5nb2.so):
# parity, then same-box A/B on the C5 shape
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
DM_LIB_PATH=$PWD/ab/libdm_c5nb2.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_c5_tile.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r04u_c5nb2_test.log 2>&1 || exit 1
for pass in 1 2 3; do
  for lib in deepmatching_stereo_matching_amd/libdmstereo.so ab/libdm_c5nb2.so; do
    echo "== pass $pass $lib" >> gpurun_out/r04u_c5nb.txt
    DM_LIB_PATH=$PWD/$lib timeout -k 10 200 python3 tools/kbench.py --variants l12 --rounds 3 --tile 256 --grid 16 >> gpurun_out/r04u_c5nb.txt 2>&1 || exit 1
  done
done
echo done

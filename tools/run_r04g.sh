# round 4: k_volume_ls transposed-store builds (ab/libdm_vtr*.so) and the S = 64 level kernel
# with 4 cell blocks per workgroup (ab/libdm_c2nb4.so): parity, then same-box A/B
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r04g
L=deepmatching_stereo_matching_amd/libdmstereo.so
timeout -k 10 120 ./tools/store_probe.bin c3_f16 c3_f32 c5_f16 > ${O}_store.jsonl 2>&1 || exit 1
for v in vtr vtr2 vtr2m; do
  DM_LIB_PATH=$PWD/ab/libdm_$v.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_c5_tile.py tests/test_c3_golden.py -m gpu -x -v -k "volume" --timeout 120 --timeout-method thread > ${O}_${v}_test.log 2>&1 || exit 1
done
DM_LIB_PATH=$PWD/ab/libdm_c2nb4.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "level" --timeout 120 --timeout-method thread > ${O}_c2nb4_test.log 2>&1 || exit 1
for pass in 1 2; do
  for lib in $L ab/libdm_pnoread.so ab/libdm_prow.so; do
    echo "== pass $pass $lib" >> ${O}_abl.txt
    DM_LIB_PATH=$PWD/$lib timeout -k 10 120 python3 tools/kbench.py --variants l12 --rounds 3 >> ${O}_abl.txt 2>&1 || exit 1
  done
  for lib in $L ab/libdm_c2nb4.so; do
    echo "== pass $pass $lib" >> ${O}_c2nb4.txt
    DM_LIB_PATH=$PWD/$lib timeout -k 10 120 python3 tools/kbench.py --variants l12 --rounds 3 --tile 64 --grid 8 >> ${O}_c2nb4.txt 2>&1 || exit 1
  done
  for lib in $L ab/libdm_vtr.so ab/libdm_vtr2.so ab/libdm_vtr2m.so; do
    for a in "--f16" "--f16 --mm" "--tiles 64" "--f16 --tile 256 --tiles 8"; do
      echo "== pass $pass $lib $a" >> ${O}_vtr.txt
      DM_LIB_PATH=$PWD/$lib timeout -k 10 120 python3 tools/vbench.py --tiles 64 $a --rounds 3 >> ${O}_vtr.txt 2>&1 || exit 1
    done
  done
done
echo done

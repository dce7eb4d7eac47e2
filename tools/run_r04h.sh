# round 4: level-kernel cell blocks per workgroup at S = 64 (DM_C2_NB) and S = 128 (DM_C3_NB),
# w0 = 128 volume instances (store runs / register budget / nontemporal), same-box A/B with
# output checksums; the new GPU tests
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r04h
L=deepmatching_stereo_matching_amd/libdmstereo.so
timeout -k 10 200 python3 -u -m pytest tests/test_stop_above_l0.py -m gpu -x -v --timeout 120 --timeout-method thread > ${O}_stop_test.log 2>&1 || exit 1
for v in c3nb2 c3nb4; do
  DM_LIB_PATH=$PWD/ab/libdm_$v.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "level" --timeout 120 --timeout-method thread > ${O}_${v}_test.log 2>&1 || exit 1
done
for pass in 1 2; do
  ck=""; [ $pass = 1 ] && ck="--checksum"
  for lib in $L ab/libdm_c3nb2.so ab/libdm_c3nb4.so; do
    echo "== pass $pass $lib" >> ${O}_c3nb.txt
    DM_LIB_PATH=$PWD/$lib timeout -k 10 120 python3 tools/kbench.py --variants l12 --rounds 3 >> ${O}_c3nb.txt 2>&1 || exit 1
  done
  for lib in $L ab/libdm_c2nb2.so ab/libdm_c2nb8.so; do
    echo "== pass $pass $lib" >> ${O}_c2nb.txt
    DM_LIB_PATH=$PWD/$lib timeout -k 10 120 python3 tools/kbench.py --variants l12 --rounds 3 --tile 64 --grid 8 >> ${O}_c2nb.txt 2>&1 || exit 1
  done
  for lib in $L ab/libdm_h2n.so ab/libdm_h2p.so ab/libdm_h4p.so ab/libdm_h0p.so; do
    echo "== pass $pass $lib --f16 --mm" >> ${O}_vol.txt
    DM_LIB_PATH=$PWD/$lib timeout -k 10 120 python3 tools/vbench.py --tiles 64 --f16 --mm --rounds 3 $ck >> ${O}_vol.txt 2>&1 || exit 1
  done
  for lib in $L ab/libdm_f4m.so ab/libdm_f4mp.so ab/libdm_f2mp.so ab/libdm_f4p.so ab/libdm_f0p.so; do
    for a in "" "--mm"; do
      echo "== pass $pass $lib f32 $a" >> ${O}_vol.txt
      DM_LIB_PATH=$PWD/$lib timeout -k 10 120 python3 tools/vbench.py --tiles 64 $a --rounds 3 $ck >> ${O}_vol.txt 2>&1 || exit 1
    done
  done
done
echo done

# round 4: full GPU suite on the final matching code, then pow-table LDS ablations (same box)
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r04f
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > ${O}_gputest.log 2>&1 || exit 1
L=deepmatching_stereo_matching_amd/libdmstereo.so
for pass in 1 2; do
  for lib in $L ab/libdm_pconst.so ab/libdm_pnoread.so ab/libdm_prow.so; do
    echo "== pass $pass $lib" >> ${O}_abl.txt
    DM_LIB_PATH=$PWD/$lib timeout -k 10 120 python3 tools/kbench.py --variants l12 --rounds 3 >> ${O}_abl.txt 2>&1 || exit 1
  done
done
timeout -k 10 120 ./tools/store_probe.bin c3_f16 c3_f32 c5_f16 > ${O}_store.jsonl 2>&1 || exit 1

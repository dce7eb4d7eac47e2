# round 4: the w0 = 256 (C5) volume instances with transposed store runs: parity, store probe,
# same-box A/B with checksums
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
for v in; do
  DM_LIB_PATH=$PWD/ab/libdm_$v.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_c5_tile.py -m gpu -x -v -k "volume" --timeout 200 --timeout-method thread > gpurun_out/r04v_${v}_test.log 2>&1 || exit 1
done
true
for pass in 1 2; do
  ck=""; [ $pass = 1 ] && ck="--checksum"
  for lib in deepmatching_stereo_matching_amd/libdmstereo.so ab/libdm_c5h2w4.so ab/libdm_c5f4m.so; do
    for a in "--f16 --mm --tiles 8" "--tiles 4" "--mm --tiles 4"; do
      echo "== pass $pass $lib $a" >> gpurun_out/r04v_vol.txt
      DM_LIB_PATH=$PWD/$lib timeout -k 10 120 python3 tools/vbench.py --tile 256 $a --rounds 3 $ck >> gpurun_out/r04v_vol.txt 2>&1 || exit 1
    done
  done
done
echo done

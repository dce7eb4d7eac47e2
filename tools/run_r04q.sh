# round 4 final: the C5 volumes' PMC passes, then one bench line per BASELINE config
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
bash tools/pmc_r03.sh r04q v16_c5 v32_c5 v16mm_c5 v32mm_c5 || exit 1
for c in c2 c4 c5; do
  timeout -k 10 300 python3 bench.py --config $c > gpurun_out/r04q_bench_$c.json 2> gpurun_out/r04q_bench_$c.err || exit 1
done
timeout -k 10 300 python3 bench.py > gpurun_out/r04q_bench.json 2> gpurun_out/r04q_bench.err || exit 1
for pass in 1 2; do
  ck=""; [ $pass = 1 ] && ck="--checksum"
  for lib in deepmatching_stereo_matching_amd/libdmstereo.so ab/libdm_h2w4.so ab/libdm_h2w2.so; do
    echo "== pass $pass $lib --f16 --mm" >> gpurun_out/r04q_vol.txt
    DM_LIB_PATH=$PWD/$lib timeout -k 10 120 python3 tools/vbench.py --tiles 64 --f16 --mm --rounds 3 $ck >> gpurun_out/r04q_vol.txt 2>&1 || exit 1
  done
done
echo done

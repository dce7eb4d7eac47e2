# round 4: the per-tile matching chain -- parity, then same-box A/B against the per-level schedule
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r04d
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -k "schedules or per_tile or upper" -x -v --timeout 240 --timeout-method thread > ${O}_tests.log 2>&1 || exit 1
timeout -k 10 600 python3 -u -m pytest tests/test_c3_batch.py tests/test_bench_steps.py -x -v --timeout 240 --timeout-method thread >> ${O}_tests.log 2>&1 || exit 1
for pass in 1 2; do
  for cfg in c3 c2; do
    for sch in tile level; do
      echo "== pass $pass $cfg $sch" >> ${O}_ab.txt
      timeout -k 10 200 python3 bench.py --config $cfg --match-schedule $sch --steps 30 --no-volume --no-cpu-baseline --no-c5-split --no-k-level >> ${O}_ab.txt 2>> ${O}_ab.err || exit 1
    done
  done
done
timeout -k 10 60 ab/mfma44_probe > ${O}_mfma44.txt 2>&1

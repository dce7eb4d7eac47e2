# round 4: per-tile chain with / without the aggregation folded in, against per level (same box)
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r04e
for pass in 1 2; do
  for cfg in c3 c2; do
    for sch in level tile tileagg; do
      echo "== pass $pass $cfg $sch" >> ${O}_ab.txt
      timeout -k 10 200 python3 bench.py --config $cfg --match-schedule $sch --steps 30 --no-volume --no-cpu-baseline --no-c5-split --no-k-level >> ${O}_ab.txt 2>> ${O}_ab.err || exit 1
    done
  done
done
timeout -k 10 60 ab/mfma44_probe > ${O}_mfma44.txt 2>&1

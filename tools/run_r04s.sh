# round 4: C2 with level 1 stored by the level kernel (DM_FUSE_L2=1) against kept on chip (2)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
for pass in 1 2; do
  for f in 2 1; do
    for a in "" "--streams 3" "--level-stream 1" "--chain-levels 0 --streams 3"; do
      echo "== pass $pass DM_FUSE_L2=$f $a" >> gpurun_out/r04s_c2_fuse.txt
      DM_FUSE_L2=$f timeout -k 10 200 python3 bench.py --config c2 --no-cpu-baseline --no-volume $a >> gpurun_out/r04s_c2_fuse.txt 2>> gpurun_out/r04s.err || exit 1
    done
  done
done
echo done

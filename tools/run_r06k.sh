#!/bin/bash
# Round 6: the driver's default bench command rehearsed with 4 and 6 ranks on the one GPU of the
# box (gloo, every rank on cuda:0 -- a mechanical check of the launcher, the per-rank pair
# sharding of the C3 line and the c5_split's bands / chunked gathers / N = 1 re-solve at more
# ranks than the tests use; the times mean nothing, the ranks share one GPU), and one rank for
# the output hashes to compare.
set -uo pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
export DM_BENCH_BACKEND=gloo DM_BENCH_ONE_DEVICE=1 OMP_NUM_THREADS=2
for n in 1 4 6; do
  timeout -k 10 400 python -u bench.py --gpus $n --steps 3 --warmup 1 --no-volume --no-cpu-baseline --output-hash > gpurun_out/r06k_n$n.json 2> gpurun_out/r06k_n$n.err || exit 1
  echo "n=$n done"
done

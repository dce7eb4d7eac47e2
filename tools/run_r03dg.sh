#!/bin/bash
# bounds on the tail's cost per C3 pair: the pipelined bench as is, without matching, and with
# only the stats + fused level kernel (DM_BENCH_DIAG; diagnostic lines, not bench results)
R=$GRAFT_REPO_ROOT
cd $R
B="python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-volume --no-k-level"
for pass in 1 2; do
  for d in "" nomatch l12only; do
    echo "== pass $pass diag [$d]"
    DM_BENCH_DIAG=$d timeout -k 10 120 $B 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('ms/pair %.3f  level kernel %.3f' % (d['ms_per_pair'], d['roofline']['ms']))" || exit 1
  done
  echo "== pass $pass kbench (level kernel alone)"
  timeout -k 10 120 python3 tools/kbench.py --variants l12 --rounds 5 2>&1 | grep -v amdgpu.ids || exit 1
done

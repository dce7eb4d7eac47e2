#!/bin/bash
# tail kernels (on-demand matching, ws = 5): workgroup size / register budget, same box, 2 passes
R=$GRAFT_REPO_ROOT
cd $R
B="python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-volume --no-k-level"
for pass in 1 2; do
  for env in "DM_TAIL_WG=256" "X=0" "DM_TAIL_WG=256 DM_TAIL_MINW=4" "DM_TAIL_MINW=4"; do
    echo "== pass $pass env [$env]"
    env $env timeout -k 10 120 $B 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('ms/pair %.3f  level kernel %.3f' % (d['ms_per_pair'], d['roofline']['ms']))" || exit 1
  done
done

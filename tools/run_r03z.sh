#!/bin/bash
# stream / priority configurations of the pipelined C3 bench, same box, two passes
R=$GRAFT_REPO_ROOT
cd $R
B="python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-volume --no-k-level"
for pass in 1 2; do
  for cfg in "" "--pair-priority high" "--level-stream 1 --pair-priority high" "--level-stream 1 --stats-stream 1 --pair-priority high" "--streams 3" "--streams 3 --pair-priority high"; do
    echo "== pass $pass cfg [$cfg]"
    timeout -k 10 120 $B $cfg 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('ms/pair %.3f  level kernel %.3f' % (d['ms_per_pair'], d['roofline']['ms']))" || exit 1
  done
done

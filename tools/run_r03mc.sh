#!/bin/bash
# fused coarse descent (k_match_coarse): GPU parity suite, then same-box A/B vs one launch per level
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03mc_gputest.log 2>&1 || exit 1
B="python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-volume --no-k-level"
for pass in 1 2 3; do
  for e in DM_MATCH_COARSE=0 DM_MATCH_COARSE=1; do
    echo "== pass $pass $e"
    env $e timeout -k 10 120 $B 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('ms/pair %.3f  level kernel %.3f' % (d['ms_per_pair'], d['roofline']['ms']))" || exit 1
    env $e timeout -k 10 120 $B --config c2 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('  c2 ms/pair %.4f  level kernel %.4f' % (d['ms_per_pair'], d['roofline']['ms']))" || exit 1
  done
done

#!/bin/bash
# A/B: consecutive pairs' level kernels chained by an event (--chain-levels 1, so no two level
# kernels share the GPU) vs free to overlap (--chain-levels 0: the next pair's workgroups fill
# the CUs the draining one leaves), 2 and 3 pair streams; bench.py C3 and C2, interleaved.
#   usage (GPU box): bash tools/overlap_ab.sh [passes]
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
line() {
  python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('ms/pair %.4f  level kernel %.4f' % (d['ms_per_pair'], d['roofline']['ms']))"
}
for pass in $(seq 1 ${1:-2}); do
  for cfg in c3 c2; do
    for v in "1 2" "0 2" "0 3"; do
      set -- $v
      echo "== pass $pass $cfg chain-levels $1 streams $2"
      timeout -k 10 120 python3 "$REPO/bench.py" --config $cfg --chain-levels $1 --streams $2 --no-cpu-baseline --no-volume --no-k-level 2>/dev/null | line || exit 1
    done
  done
done

#!/bin/bash
# Same-box A/B: bench.py (C3) with the ws=5 on-demand matching kernels at their default
# register budget vs DM_TAIL_MINW=6 (<= 80 VGPRs: they fit beside a running level kernel).
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
for pass in 1 2; do
  for v in "0 --streams 2" "6 --streams 2" "6 --streams 3" "6 --streams 1 --level-stream 1 --stats-stream 1"; do
    set -- $v; m=$1; shift
    out=$(DM_TAIL_MINW=$m timeout -k 10 150 python3 "$REPO/bench.py" "$@" --steps 30 --no-cpu-baseline --no-volume --no-k-level --output-hash 2>/dev/null) || exit 1
    echo "$out" | python3 -c "
import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1])
print('pass $pass DM_TAIL_MINW=%s %-50s ms/pair %.3f  level %.3f  sha %s' % ('$m', '$*', d['ms_per_pair'], d['roofline']['ms'], d.get('output_sha256','')[:12]))"
  done
done

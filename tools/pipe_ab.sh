#!/bin/bash
# Same-box A/B of bench.py's pair pipelining options (C3 defaults otherwise), two passes.
#   usage (GPU box): bash tools/pipe_ab.sh > gpurun_out/<tag>_pipe_ab.txt
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
V=("--streams 2" "--streams 1 --level-stream 1 --stats-stream 1" "--streams 2 --level-stream 1 --stats-stream 1"
   "--streams 1 --level-stream 1" "--streams 2 --level-stream 1")
for pass in 1 2; do
  for v in "${V[@]}"; do
    out=$(timeout -k 10 150 python3 "$REPO/bench.py" $v --steps 30 --no-cpu-baseline --no-volume --no-k-level --output-hash 2>/dev/null) || exit 1
    echo "$out" | python3 -c "
import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1])
print('pass $pass %-66s ms/pair %.3f  level %.3f  sha %s' % ('$v', d['ms_per_pair'], d['roofline']['ms'], d.get('output_sha256','')[:12]))"
  done
done

#!/bin/bash
# Same-box A/B of the C5 pair (bench.py --config c5: one 4096^2 pair of 256 S=256 tiles per step)
# for library builds, alternating, two passes; prints ms per pair, level-kernel ms, output hash.
#   usage (GPU box): bash tools/c5ab.sh lib1.so lib2.so ...
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
for pass in 1 2; do
  for lib in "$@"; do
    DM_LIB_PATH=$lib timeout -k 10 200 python3 "$REPO/bench.py" --config c5 --steps 3 --warmup 1 --no-cpu-baseline \
        --no-volume --no-k-level > /tmp/c5ab.json 2> /tmp/c5ab.err || { echo "$lib failed"; tail -3 /tmp/c5ab.err; exit 1; }
    python3 - "$lib" "$pass" <<'PY'
import json, sys
d = json.loads(open('/tmp/c5ab.json').read().strip().splitlines()[-1])
print('pass %s %-40s ms/pair %.3f  level %.3f  sha %s' % (sys.argv[2], sys.argv[1], d['ms_per_step'],
      (d.get('roofline') or {}).get('ms') or -1, (d.get('step_outputs') or {}).get('sha256', '')[:16]))
PY
  done
done

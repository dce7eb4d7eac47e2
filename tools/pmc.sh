#!/bin/bash
# PMC passes (one rocprofv3 run per counter group) of tools/kbench.py variants.
#   usage (GPU box): bash tools/pmc.sh <tag> <kbench variants> "<counters pass 1>" ["<pass 2>" ...]
set -euo pipefail
TAG=$1; VAR=$2; shift 2
REPO=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$REPO/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
k=0
for grp in "$@"; do
    k=$((k + 1))
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$OUT/p$k" -o run -- \
        python3 "$REPO/tools/${BENCH:-kbench}.py" --variants "$VAR" --rounds 1 > "$OUT/p$k.log" 2>&1
done
python3 "$REPO/tools/pmc_summary.py" "$OUT" > "$OUT/summary.txt"
cat "$OUT/summary.txt"

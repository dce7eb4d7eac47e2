#!/bin/bash
# rocprofv3 evidence for profiles/: kernel-trace stats of bench.py, then separate PMC passes
# (HBM FETCH_SIZE / WRITE_SIZE each alone, SQ counters) of the dominant kernel via kbench.
#   usage (on the GPU box): bash tools/profile.sh <tag>
set -euo pipefail
TAG=${1:-r01}
REPO=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$REPO/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- \
    python3 "$REPO/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/stats.err"
KB="$REPO/tools/kbench.py --variants ${KVAR:-l12} --rounds 2"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
    python3 $KB > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- \
    python3 $KB > "$OUT/write.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS \
    SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES --output-format csv -d "$OUT/sq" -o run -- \
    python3 $KB > "$OUT/sq.log" 2>&1
echo done

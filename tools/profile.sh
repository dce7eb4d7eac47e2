#!/bin/bash
# rocprofv3 evidence for profiles/ (round 2): kernel-trace stats of bench.py (C3) with a
# per-grid-size split, HBM PMC passes (FETCH_SIZE and WRITE_SIZE each alone), the VALU and
# vector-memory passes of the dominant kernels, and the per-launch summaries.
#   usage (on the GPU box): bash tools/profile.sh <tag>
set -euo pipefail
TAG=${1:-r02}
REPO=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$REPO/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BENCH="$REPO/bench.py --steps 5 --warmup 2 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- \
    python3 $BENCH > "$OUT/bench.json" 2> "$OUT/stats.err"
python3 "$REPO/tools/kstats.py" "$OUT/stats" > "$OUT/kernel_stats_by_grid.csv"
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
    python3 $BENCH > "$OUT/fetch.log" 2>&1
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- \
    python3 $BENCH > "$OUT/write.log" 2>&1
python3 "$REPO/tools/traffic.py" "$OUT" 128
bash "$REPO/tools/pmc_valu.sh" "$TAG"
bash "$REPO/tools/pmc_mem.sh" "$TAG"
echo done

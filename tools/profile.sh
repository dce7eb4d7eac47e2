#!/bin/bash
# rocprofv3 evidence for profiles/: kernel-trace stats of bench.py, HBM PMC passes
# (FETCH_SIZE and WRITE_SIZE each alone) of the same command, and an SQ pass of the
# dominant kernel via kbench; then per-launch HBM bytes of the level-1 and volume kernels.
#   usage (on the GPU box): bash tools/profile.sh <tag>
set -euo pipefail
TAG=${1:-r01}
REPO=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$REPO/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BENCH="$REPO/bench.py --steps 5 --warmup 2 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- \
    python3 $BENCH > "$OUT/bench.json" 2> "$OUT/stats.err"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
    python3 $BENCH > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- \
    python3 $BENCH > "$OUT/write.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
    SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES --output-format csv -d "$OUT/sq" -o run -- \
    python3 "$REPO/tools/kbench.py" --variants l12 --rounds 2 > "$OUT/sq.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
    SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES --output-format csv -d "$OUT/sqv16" -o run -- \
    python3 "$REPO/tools/vbench.py" --f16 --rounds 1 --tiles 32 > "$OUT/sqv16.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$OUT/l2v16" -o run -- \
    python3 "$REPO/tools/vbench.py" --f16 --rounds 1 --tiles 32 > "$OUT/l2v16.log" 2>&1
python3 "$REPO/tools/traffic.py" "$OUT" 128
echo done

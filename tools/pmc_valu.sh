#!/bin/bash
# VALU-busy and clock passes for the roofline of the dominant kernel (k_level1_mfq via kbench
# l12, the C3 batch) and of the binary16 volume kernel (vbench --f16): one rocprofv3 --pmc run
# per pass (<= 8 SQ + 2 GRBM counters), each under its own kill timeout.
#   usage (GPU box): bash tools/pmc_valu.sh <tag>      -> gpurun_out/pmc_<tag>/...
set -euo pipefail
TAG=${1:-valu}
REPO=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$REPO/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
SQ="SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $SQ GRBM_GUI_ACTIVE --output-format csv -d "$OUT/l12" -o run -- \
    python3 "$REPO/tools/kbench.py" --variants l12 --rounds 2 > "$OUT/l12.log" 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $SQ GRBM_GUI_ACTIVE --output-format csv -d "$OUT/v16" -o run -- \
    python3 "$REPO/tools/vbench.py" --f16 --rounds 1 --tiles 64 > "$OUT/v16.log" 2>&1
python3 "$REPO/tools/valu_summary.py" "$OUT" > "$OUT/summary.txt"
echo done

#!/bin/bash
# One SQ pass (VALU / MFMA / SALU activity) over the dominant level kernel (kbench l12) and
# the binary16 volume kernel (vbench --f16).   usage (GPU box): bash tools/pmc_valu.sh <tag>
set -euo pipefail
TAG=${1:-valu}
REPO=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$REPO/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
CTR="SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_THREAD_CYCLES_VALU"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc $CTR --output-format csv -d "$OUT/l12" -o run -- \
    python3 "$REPO/tools/kbench.py" --variants l12 --rounds 1 > "$OUT/l12.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc $CTR --output-format csv -d "$OUT/v16" -o run -- \
    python3 "$REPO/tools/vbench.py" --f16 --rounds 1 --tiles 32 > "$OUT/v16.log" 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d "$OUT/clk" -o run -- \
    python3 "$REPO/tools/kbench.py" --variants l12 --rounds 1 > "$OUT/clk.log" 2>&1
echo done

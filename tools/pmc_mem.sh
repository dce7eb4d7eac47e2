#!/bin/bash
# Vector-memory pipe (TA/TD/TCP) and VALU-type passes over the binary16 volume kernel and the
# fused level kernel: is the per-CU load path (fragment-shaped B loads) or the VALU the limit?
#   usage (GPU box): bash tools/pmc_mem.sh <tag>     -> gpurun_out/pmcm_<tag>/...
set -euo pipefail
TAG=${1:-mem}
REPO=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$REPO/gpurun_out/pmcm_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
MEM="TA_TA_BUSY_sum TA_BUFFER_TOTAL_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE"
MIX="SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU SQ_INSTS_MFMA"
for k in v16 l12; do
  if [ $k = v16 ]; then CMD="$REPO/tools/vbench.py --f16 --rounds 1 --tiles 64"; else CMD="$REPO/tools/kbench.py --variants l12 --rounds 1"; fi
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $MEM --output-format csv -d "$OUT/mem_$k" -o run -- python3 $CMD > "$OUT/mem_$k.log" 2>&1
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $MIX --output-format csv -d "$OUT/mix_$k" -o run -- python3 $CMD > "$OUT/mix_$k.log" 2>&1
done
python3 "$REPO/tools/pmc_table.py" "$OUT" > "$OUT/summary.txt"
echo done

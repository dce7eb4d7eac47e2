#!/bin/bash
# Same-box VALU/LDS PMC pass of the fused level kernel for several library builds
# (DM_LIB_PATH), alternating, so instruction counts and busy fractions compare like with like.
#   usage (GPU box): bash tools/pmc_ab.sh <tag> lib1.so lib2.so ...   -> gpurun_out/pmcab_<tag>/
set -euo pipefail
TAG=$1; shift
REPO=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$REPO/gpurun_out/pmcab_$TAG
mkdir -p "$OUT"
LIBS=(); for l in "$@"; do LIBS+=("$(cd "$(dirname "$l")" && pwd)/$(basename "$l")"); done
cd /tmp && export TMPDIR=/tmp
SQ="SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_ANY"
for pass in 1 2; do
  for lib in "${LIBS[@]}"; do
    b=$(basename "$lib" .so)
    DM_LIB_PATH=$lib timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $SQ GRBM_GUI_ACTIVE --output-format csv \
        -d "$OUT/${b}_$pass/l12" -o run -- python3 "$REPO/tools/kbench.py" --variants l12 --rounds 2 > "$OUT/${b}_$pass.log" 2>&1
    python3 "$REPO/tools/valu_summary.py" "$OUT/${b}_$pass" | python3 -c "import sys; print('$b pass $pass', ' '.join(l.strip() for l in sys.stdin if 'valu' in l or 'clock' in l or 'INSTS' in l or 'ms' in l))"
  done
done

#!/bin/bash
# Same-box LDS / VALU PMC pass of the level kernel (C3 batch, tools/kbench.py) for several
# library builds, alternating: LDS instruction / active / wait cycles and bank conflicts next to
# the VALU figures, per launch (round 5: k_level12_strip against k_level1_mfq).
#   usage (GPU box): bash tools/pmc_lds5.sh <tag> lib1.so lib2.so ...   -> gpurun_out/pmclds_<tag>/
set -euo pipefail
TAG=$1; shift
REPO=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$REPO/gpurun_out/pmclds_$TAG
mkdir -p "$OUT"
LIBS=(); for l in "$@"; do LIBS+=("$(cd "$(dirname "$l")" && pwd)/$(basename "$l")"); done
cd /tmp && export TMPDIR=/tmp
SQ="SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
for pass in 1 2; do
  for lib in "${LIBS[@]}"; do
    b=$(basename "$lib" .so)
    DM_LIB_PATH=$lib timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $SQ GRBM_GUI_ACTIVE --output-format csv \
        -d "$OUT/${b}_$pass" -o run -- python3 "$REPO/tools/kbench.py" --variants l12 --rounds 2 > "$OUT/${b}_$pass.log" 2>&1
    python3 - "$OUT/${b}_$pass" "$b pass $pass" <<'PY'
import collections, csv, glob, os, sys
d, tag = sys.argv[1], sys.argv[2]
cc = glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True)
kt = glob.glob(os.path.join(d, '**', '*kernel_trace.csv'), recursive=True)
dur = {}
for r in csv.DictReader(open(kt[0])):
    if 'k_level1' in r['Kernel_Name']:
        dur[r['Dispatch_Id']] = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) * 1e-6
big = max(dur.values())
keep = {k for k, v in dur.items() if v >= 0.5 * big}
acc = collections.defaultdict(float)
for r in csv.DictReader(open(cc[0])):
    if r['Dispatch_Id'] in keep:
        acc[r['Counter_Name']] += float(r['Counter_Value'])
n = len(keep)
ms = sum(dur[k] for k in keep) / n
print(tag, 'launches', n, 'ms %.3f' % ms, ' '.join('%s=%.4g' % (k, v / n) for k, v in sorted(acc.items())))
PY
  done
done

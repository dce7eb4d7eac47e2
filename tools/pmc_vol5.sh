#!/bin/bash
# PMC pass (VALU / LDS / wave cycles) over the C3 binary16 standalone volume (tools/vbench.py,
# 64 tiles of S = 128) for library builds: per launch of the volume kernel (k_volume_*).
#   usage (GPU box): bash tools/pmc_vol5.sh <tag> "<vbench args>" lib1.so lib2.so ...  -> gpurun_out/pmcvol_<tag>/
set -euo pipefail
TAG=$1; ARGS=$2; shift 2
REPO=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$REPO/gpurun_out/pmcvol_$TAG
mkdir -p "$OUT"
LIBS=(); for l in "$@"; do LIBS+=("$(cd "$(dirname "$l")" && pwd)/$(basename "$l")"); done
cd /tmp && export TMPDIR=/tmp
SQ="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
for lib in "${LIBS[@]}"; do
  b=$(basename "$lib" .so)
  DM_LIB_PATH=$lib timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $SQ GRBM_GUI_ACTIVE --output-format csv \
      -d "$OUT/$b" -o run -- python3 "$REPO/tools/vbench.py" --rounds 2 $ARGS > "$OUT/$b.log" 2>&1
  python3 - "$OUT/$b" "$b" <<'PY'
import collections, csv, glob, os, sys
d, tag = sys.argv[1], sys.argv[2]
cc = glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True)
kt = glob.glob(os.path.join(d, '**', '*kernel_trace.csv'), recursive=True)
dur = {}
for r in csv.DictReader(open(kt[0])):
    if 'k_volume' in r['Kernel_Name']:
        dur[r['Dispatch_Id']] = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) * 1e-6
acc = collections.defaultdict(float)
for r in csv.DictReader(open(cc[0])):
    if r['Dispatch_Id'] in dur:
        acc[r['Counter_Name']] += float(r['Counter_Value'])
n = len(dur)
ms = sum(dur.values()) / n
print(tag, 'launches', n, 'ms %.3f' % ms, ' '.join('%s=%.4g' % (k, v / n) for k, v in sorted(acc.items())))
PY
done

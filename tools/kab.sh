#!/bin/bash
# Same-box per-kernel A/B of library builds: rocprofv3 kernel-trace stats of bench.py (C3) for
# each build (DM_LIB_PATH), alternating, then the per-step averages of the named kernels.
#   usage (GPU box): bash tools/kab.sh <tag> lib1.so lib2.so ...   -> gpurun_out/kab_<tag>/
set -euo pipefail
TAG=$1; shift
REPO=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$REPO/gpurun_out/kab_$TAG
mkdir -p "$OUT"
# an entry may carry environment settings: lib.so+DM_AGG_BR=8+...
LIBS=(); for l in "$@"; do f=${l%%+*}; e=${l#"$f"}; LIBS+=("$(cd "$(dirname "$f")" && pwd)/$(basename "$f")$e"); done
cd /tmp && export TMPDIR=/tmp
for pass in 1 2; do
  for ent in "${LIBS[@]}"; do
    lib=${ent%%+*}; envs=${ent#"$lib"}; envs=${envs//+/ }
    b=$(basename "$lib" .so)$(echo "$envs" | tr ' =' '_-')
    env $envs DM_LIB_PATH=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${b}_$pass" -o run -- \
        python3 "$REPO/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-volume > "$OUT/${b}_$pass.json" 2> "$OUT/${b}_$pass.err"
    python3 - "$OUT/${b}_$pass" "$b pass $pass" <<'PY'
import csv, glob, json, sys
d, tag = sys.argv[1], sys.argv[2]
rows = list(csv.DictReader(open(glob.glob(d + '/**/*kernel_stats.csv', recursive=True)[0])))
keep = ('k_match_step_l1', 'k_match_step_l0', 'k_subpix_t', 'k_aggregate_rows', 'k_level1_mfq', 'k_prep_windows16')
out = {}
for r in rows:
    for k in keep:
        if k in r['Name']:
            out[k] = out.get(k, 0) + float(r['TotalDurationNs']) / 1e3
print(tag, json.dumps({k: round(v / 7, 1) for k, v in out.items()}), 'us/step;',
      'ms_per_step', json.load(open(d + '.json'))['ms_per_step'])
PY
  done
done

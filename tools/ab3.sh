#!/bin/bash
# A/B/C of library builds on one box, two passes: kbench l12 and vbench (fp16, float32).
#   usage (GPU box): bash tools/ab3.sh lib1.so lib2.so [lib3.so ...]
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
for pass in 1 2; do
  for lib in "$@"; do
    echo "== pass $pass $(basename $lib)"
    DM_LIB_PATH=$lib timeout -k 10 120 python3 "$REPO/tools/kbench.py" --variants l12 --rounds 3 2>&1 | grep -v amdgpu.ids || exit 1
    DM_LIB_PATH=$lib timeout -k 10 120 python3 "$REPO/tools/vbench.py" --tiles 64 --rounds 3 --f16 2>&1 | grep -v amdgpu.ids || exit 1
    DM_LIB_PATH=$lib timeout -k 10 120 python3 "$REPO/tools/vbench.py" --tiles 59 --rounds 3 2>&1 | grep -v amdgpu.ids || exit 1
  done
done

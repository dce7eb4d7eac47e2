#!/bin/bash
# Level-kernel A/B of library builds on one box (round 5): C3 (S = 128, 64 tiles), C2 (S = 64,
# 64 tiles) and C5-size tiles (S = 256, 16 tiles), two interleaved passes; every run prints the
# sha256 of its whole level-2 output, so the builds' bit-identity is checked on the same data.
#   usage (GPU box): bash tools/kab5.sh lib1.so lib2.so [...]
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
for pass in 1 2; do
  for lib in "$@"; do
    echo "== pass $pass $(basename $lib)"
    DM_LIB_PATH=$lib timeout -k 10 120 python3 "$REPO/tools/kbench.py" --variants l12 --rounds 4 --sha 2>&1 | grep -v amdgpu.ids || exit 1
    DM_LIB_PATH=$lib timeout -k 10 120 python3 "$REPO/tools/kbench.py" --variants l12 --rounds 6 --tile 64 --sha 2>&1 | grep -v amdgpu.ids || exit 1
    DM_LIB_PATH=$lib timeout -k 10 120 python3 "$REPO/tools/kbench.py" --variants l12 --rounds 3 --tile 256 --grid 4 --sha 2>&1 | grep -v amdgpu.ids || exit 1
  done
done

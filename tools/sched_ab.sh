#!/bin/bash
# A/B of library builds that differ only in the AMDGPU machine scheduler strategy
# (-mllvm -amdgpu-sched-strategy=...): kbench l12 at C3 (S=128), C5 shape (S=256, 64 tiles)
# and C2 (S=64), three interleaved passes.   usage (GPU box): bash tools/sched_ab.sh lib1.so lib2.so ...
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
for pass in 1 2 3; do
  for lib in "$@"; do
    echo "== pass $pass $(basename $lib)"
    DM_LIB_PATH=$lib timeout -k 10 120 python3 "$REPO/tools/kbench.py" --variants l12 --rounds 3 2>&1 | grep -v amdgpu.ids || exit 1
    DM_LIB_PATH=$lib timeout -k 10 120 python3 "$REPO/tools/kbench.py" --variants l12 --rounds 2 --tile 256 --grid 8 2>&1 | grep -v amdgpu.ids || exit 1
    DM_LIB_PATH=$lib timeout -k 10 120 python3 "$REPO/tools/kbench.py" --variants l12 --rounds 3 --tile 64 2>&1 | grep -v amdgpu.ids || exit 1
  done
done

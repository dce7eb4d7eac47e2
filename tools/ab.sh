#!/bin/bash
# Same-box A/B of two library builds (DM_LIB_PATH): the volume kernels (vbench, float32 and
# binary16, 64 C3 tiles) and the fused level kernel (kbench l12), old then new then old.
#   usage (GPU box): bash tools/ab.sh <old.so> [new.so] > gpurun_out/ab.log
set -uo pipefail
OLD=$1
NEW=${2:-}
REPO=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
run() {
    local tag=$1 lib=$2
    echo "== $tag"
    DM_LIB_PATH=$lib timeout -k 10 120 python3 "$REPO/tools/vbench.py" --tiles 64 --rounds 3 --f16 || exit 1
    DM_LIB_PATH=$lib timeout -k 10 120 python3 "$REPO/tools/vbench.py" --tiles 59 --rounds 3 || exit 1
    DM_LIB_PATH=$lib timeout -k 10 120 python3 "$REPO/tools/kbench.py" --variants l12 --rounds 3 || exit 1
}
run old "$OLD"
run new "$NEW"
run old "$OLD"

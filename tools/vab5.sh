#!/bin/bash
# Same-box A/B of the volume kernels for library builds (round 5: the min/max sweep on the
# row-pair strips, DM_VS1), two interleaved passes, each run printing the volume checksum:
# C3 (64 tiles of S = 128) float32 / binary16 standalone and min/max known, C5-size (4 / 8
# tiles of S = 256) float32 / binary16 standalone.
#   usage (GPU box): bash tools/vab5.sh lib1.so lib2.so ...
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
for pass in 1 2; do
  for lib in "$@"; do
    for cfg in "--tiles 64" "--tiles 64 --f16" "--tiles 64 --mm" "--tiles 64 --f16 --mm" "--tiles 4 --tile 256" "--tiles 8 --tile 256 --f16"; do
      echo "== pass $pass $(basename $lib) $cfg"
      DM_LIB_PATH=$lib timeout -k 10 120 python3 "$REPO/tools/vbench.py" --rounds 3 --checksum $cfg 2>&1 | grep -v amdgpu.ids || exit 1
    done
  done
done

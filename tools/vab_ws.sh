#!/bin/bash
# Same-box A/B of the standalone w0 = 128 volumes (C3: 64 tiles of S = 128, binary16 and float32)
# for library builds, two interleaved passes, each run printing the volume checksum (round 5:
# k_volume_ws against k_volume_ls and its ablations; the binary16 volume with the min/max known
# as the store-sweep floor).
#   usage (GPU box): bash tools/vab_ws.sh lib1.so lib2.so ...
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
for pass in 1 2; do
  for lib in "$@"; do
    for cfg in "--tiles 64 --f16" "--tiles 64" "--tiles 64 --f16 --mm"; do
      echo "== pass $pass $(basename $lib) $cfg"
      DM_LIB_PATH=$lib timeout -k 10 120 python3 "$REPO/tools/vbench.py" --rounds 3 --checksum $cfg 2>&1 | grep -v amdgpu.ids || exit 1
    done
  done
done

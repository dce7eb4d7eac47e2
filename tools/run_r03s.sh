#!/bin/bash
# volume kernels: nontemporal (default) vs plain stores, same box, interleaved rounds
for args in "--f16" "--f16 --mm" "" "--mm"; do
  echo "== vbench $args"
  timeout -k 10 200 python3 tools/vbench.py $args --tiles 64 --rounds 5 --variants ls,ls+DM_VOLUME_NT=0,ls2,ls2+DM_VOLUME_NT=0 2>&1 | grep -v amdgpu.ids || exit 1
done

#!/bin/bash
# Round 6: the level kernels' in-kernel clock under a sustained load (tools/clock_probe.py on the
# DM_CLOCK_STAMP=1 build), C3, C2 and a C5-size batch, each after 3 s of back-to-back launches;
# then the in-tree library's C3 kernel timed the same way for comparison (no stamps).
set -uo pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for s in "128 8" "64 8" "256 4" "128 8"; do
  set -- $s
  DM_LIB_PATH=$R/abx/libdm_clk.so timeout -k 10 120 python3 tools/clock_probe.py --tile $1 --grid $2 --seconds 3 2>&1 | grep -v amdgpu.ids || exit 1
done > gpurun_out/r06l_clock.jsonl
timeout -k 10 120 python3 tools/kbench.py --variants l12 --rounds 8 --tile 128 >> gpurun_out/r06l_clock.jsonl 2>&1 || exit 1

#!/bin/bash
# C5 volume rooflines: store-pattern probe for the float32 S=256 volume, PMC passes (HBM bytes)
# of the C5 line's float32 / min-max-known volumes, then the C5 bench line that reads them.
#   usage (GPU box): bash tools/run_r03c5v.sh   (tools/store_probe.bin built beforehand)
set -euo pipefail
R=$GRAFT_REPO_ROOT
T=r03c5v
cd $R
timeout -k 10 120 ./tools/store_probe.bin c5_f32 > gpurun_out/${T}_store_probe.jsonl
cat gpurun_out/${T}_store_probe.jsonl >> profiles/store_probe.jsonl
timeout -k 10 600 bash tools/pmc_r03.sh $T v32_c5 v16mm_c5 v32mm_c5 > gpurun_out/${T}_pmc.log 2>&1
cp gpurun_out/pmc3_$T/pmc_volume_s256.json gpurun_out/pmc3_$T/pmc_volume_f16_mm_s256.json gpurun_out/pmc3_$T/pmc_volume_mm_s256.json profiles/
timeout -k 10 300 python3 bench.py --config c5 > gpurun_out/${T}_bench_c5.json 2> gpurun_out/${T}_bench_c5.err

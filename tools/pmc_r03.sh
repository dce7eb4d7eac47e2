#!/bin/bash
# Round-3 PMC passes (rocprofv3, one --pmc run per pass, each under its own kill timeout) for
# the roofline fields of bench.py: per launch SQ instruction / cycle counters + the clock,
# FETCH_SIZE and WRITE_SIZE (separate passes: TCC slots), for the level kernel a fourth pass of
# its work counters (MFMA math ops, float64 instruction mix), for
#   l12_c3   dm_corr_level12, C3 batch (64 tiles of S=128)          tools/kbench.py
#   l12_c5   dm_corr_level12, C5 pair (256 tiles of S=256)          tools/kbench.py
#   l12_c2   dm_corr_level12, C2 pair (64 tiles of S=64)            tools/kbench.py
#   v16_c3   dm_corr_volume_f16, 64 tiles of S=128                  tools/vbench.py
#   v16_c5   dm_corr_volume_f16, 8 tiles of S=256
#   v32_c3   dm_corr_volume (float32), 64 tiles of S=128
#   v16mm_c3, v32mm_c3   the same with the min/max known (dm_corr_volume_ex MINMAX_KNOWN)
#   v32_c5, v16mm_c5, v32mm_c5   the C5 line's volumes (4 float32 / 8 binary16 tiles of S=256)
# then tools/pmc_r03.py writes profiles/pmc_<kernel>[_s256].json.
#   usage (GPU box): bash tools/pmc_r03.sh <tag> [shapes...]     -> gpurun_out/pmc3_<tag>/
set -euo pipefail
TAG=${1:-r03}; shift || true
SHAPES=${*:-l12_c3 l12_c5 v16_c3 v16_c5 v32_c3 v16mm_c3 v32mm_c3}
REPO=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$REPO/gpurun_out/pmc3_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
SQ="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
# the level kernel's work pass (round 6, bench.py roofline.work): i8 MFMA math ops / 512 and the
# float64 VALU instruction mix (wave instructions), one pass of 7 SQ counters
WORK="SQ_INSTS_VALU_MFMA_MOPS_I8 SQ_INSTS_MFMA SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_TRANS_F32"
for s in $SHAPES; do
  case $s in
    l12_c3) CMD="$REPO/tools/kbench.py --variants l12 --rounds 1 --tile 128 --grid 8" ;;
    l12_c5) CMD="$REPO/tools/kbench.py --variants l12 --rounds 1 --tile 256 --grid 16" ;;
    l12_c2) CMD="$REPO/tools/kbench.py --variants l12 --rounds 1 --tile 64 --grid 8" ;;
    v16_c3) CMD="$REPO/tools/vbench.py --f16 --rounds 1 --tiles 64 --tile 128" ;;
    v16_c5) CMD="$REPO/tools/vbench.py --f16 --rounds 1 --tiles 8 --tile 256" ;;
    v32_c3) CMD="$REPO/tools/vbench.py --rounds 1 --tiles 64 --tile 128" ;;
    v16mm_c3) CMD="$REPO/tools/vbench.py --f16 --mm --rounds 1 --tiles 64 --tile 128" ;;
    v32_c5) CMD="$REPO/tools/vbench.py --rounds 1 --tiles 4 --tile 256" ;;
    v16mm_c5) CMD="$REPO/tools/vbench.py --f16 --mm --rounds 1 --tiles 8 --tile 256" ;;
    v32mm_c5) CMD="$REPO/tools/vbench.py --mm --rounds 1 --tiles 4 --tile 256" ;;
    v32mm_c3) CMD="$REPO/tools/vbench.py --mm --rounds 1 --tiles 64 --tile 128" ;;
    *) echo "unknown shape $s"; exit 2 ;;
  esac
  PASSES="sq fetch write"
  case $s in l12_*) PASSES="sq fetch write work" ;; esac
  for pass in $PASSES; do
    case $pass in sq) P="$SQ" ;; fetch) P="FETCH_SIZE" ;; write) P="WRITE_SIZE" ;; work) P="$WORK" ;; esac
    timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $P --output-format csv -d "$OUT/${s}_$pass" -o run -- \
        python3 $CMD > "$OUT/${s}_$pass.log" 2>&1
    echo "$s $pass done"
  done
done
python3 "$REPO/tools/pmc_r03.py" "$OUT" > "$OUT/summary.json"
echo done

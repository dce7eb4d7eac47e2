#!/bin/bash
# Ablation builds of the level kernel (timing upper bounds only; their results are WRONG):
#   nobar   no barrier between the two waves of a workgroup in sweep 2 (dm_mfma.h:628)
#   nopow   pow14_zf replaced by a widening multiply (the eight child pows per row pair)
#   papprox  (round 6) the child pows replaced by the bin-centre approximation (1/c_i)^y 2^(yE):
#           the floor of any pruning of the child pows (C3 k_level1_mfq only)
#   papprox2 the same with 2 of a lane's 8 child pows per row exact: the ideal pruned count (one
#           exact level-1 value per level-2 window), without the candidate bookkeeping
#   ssync   (round 6) the strip kernel's one-wave cell blocks (C2) synchronised by workgroup
#           barriers between the sweeps, as in round 5 (DM_STRIP_WAVESYNC=0; results exact)
#   prune0, prune1  (round 6) the C3 level kernel without / with the child-pow pruning
#           (k_level1_mfq / k_level12_prune, DM_PRUNE; results exact)
#   nosw1   sweep 1 (per-patch min / max) skipped
#   pconst  pow14_zf's three LDS table reads at fixed rows (broadcast: no bank conflicts)
#   pnoread pow14_zf without its LDS table reads (values from the index bits, no LDS)
#   prow    c_i and a float32 (1/c_i)^y lo packed into the fp row: one b128 read instead of
#           b128 + b32 (a layout probe: the row's contents are not rebuilt)
#   h2n, h2p, h4p, h0p   the w0 = 128 binary16 volume with the min/max known: runs of 2 / 4
#           256-B chunks per store (transposed across lane groups) or none, nontemporal (n) or
#           plain (p) stores (DM_VL_H_*; results exact); h2w8 / h2w2: 8 / 2 waves per workgroup (4 in-tree)
#   f4m, f4mp, f2mp, f4p, f0p   the w0 = 128 float32 volume: runs of 4 / 2 / none, m = compiled
#           for 4 waves per SIMD, p = plain stores (DM_VL_F_*; results exact)
#   s0      sweep 1 on the 16 x 16 tiles instead of the row-pair strips (DM_S1=0; results exact)
#   x0      the level kernel's workgroups in dispatch order, not XCD-grouped (DM_XCD_MAP=0; exact)
#   s2off   sweep 2 on the 16 x 16 tiles (k_level1_mfq) for every shape (DM_S2=0; results exact)
#   s2all   the strip kernel (k_level12_strip) for C3 as well (DM_S2=7; results exact)
#   vs0     the standalone volumes' min/max sweep on the 16 x 16 tiles, not the strips (DM_VS1=0; exact)
#   c3mw3   the S = 128 strip kernel compiled for 3 waves per SIMD (A, patch sums in registers,
#           two row pairs per loop trip; DM_C3_MW=3; results exact)
#   head    the last commit's sources (an A/B of the working tree against it)
#   hsw4, fw4   the w0 = 128 binary16 standalone / float32 volumes in 4-wave workgroups
#   smilp, smclause, strack   every kernel scheduled by the AMDGPU machine scheduler's max-ilp /
#           max-memory-clause strategy, or with the AMDGPU register-pressure trackers (-mllvm
#           -amdgpu-sched-strategy=..., -amdgpu-use-amdgpu-trackers; results exact: scheduling only)
#   vs1l2   the standalone volumes' strip min/max sweep with every wave reading the units from
#           L2 instead of each unit staged in LDS once per workgroup (DM_VS1_LDS=0; exact)
#   hs4t2, hs8t2   the binary16 standalone volume in 4- / 8-wave workgroups with 2 x 512-B runs per
#           store (DM_VL_HS_NW, DM_VL_HS_TR; results exact)
#   c5h2w4, c5f4m   the w0 = 256 volumes: binary16 min/max known with 2 x 512-B runs in
#           4-wave workgroups; float32 with 1-KB runs at 4 waves/SIMD (DM_VL_H2_*, DM_VL_F2_*)
#   c2nb2, c2nb8   the S = 64 level kernel with 2 / 8 one-wave cell blocks per workgroup
#           instead of 4 (DM_C2_NB; results exact)
#   c3nb1, c3nb4   the S = 128 level kernel with 1 / 4 two-wave cell blocks per workgroup instead of 2
#   c5nb2   the S = 256 level kernel with 2 four-wave cell blocks per workgroup instead of 1
#           (DM_C3_NB / DM_C5_NB; results exact)
#   nofill  (round 6) the strip kernel (C2 / C5) without its pow-table fill: the price of the
#           workgroup prologue's table copy (results wrong)
#   bwrow0, strow0  (round 6) C3 k_level1_mfq with every sweep-2 window-operand load (bwrow0) or
#           every sweep-1 strip load (strow0) at row 0: the same instructions, served from the
#           CU's vector cache instead of L2 (row index masked by a run-time zero, so the loads stay in
#           the loop) -- the price of the L2 read traffic (results wrong)
#   clk     (round 6) the level kernels with per-workgroup clock stamps (DM_CLOCK_STAMP=1;
#           results exact, tools/clock_probe.py reads them)
# Each is the in-tree source with one sed patch, built to ab/libdm_<name>.so (git-ignored,
# travels to the GPU box); tools/ab3.sh / kbench A/B them with DM_LIB_PATH.
set -euo pipefail
REPO=$(cd "$(dirname "$0")/.." && pwd)
FLAGS="-O3 -std=c++17 -ffp-contract=off -fPIC -shared -Wno-pass-failed -mllvm -amdgpu-mfma-vgpr-form --offload-arch=gfx950"
for v in "$@"; do
  EXTRA=""; r=/tmp/abl_$v; rm -rf $r; d=$r/pkg; mkdir -p $d; cp -r $REPO/deepmatching_stereo_matching_amd/csrc $d/; cp -r $REPO/include $r/
  case $v in
    nobar) sed -i '628s/__syncthreads();/__builtin_amdgcn_wave_barrier();/' $d/csrc/dm_mfma.h ;;
    nopow) python3 - $d/csrc/dm_kernels.hip <<'PY'
import sys
p = sys.argv[1]; s = open(p).read()
a = s.index('__device__ __forceinline__ double pow14_zf(float x, const T &t, unsigned mant = 0x7FFFFFu)\n{')
b = s.index('\n}\n', a)
s = s[:a] + '__device__ __forceinline__ double pow14_zf(float x, const T &t, unsigned mant = 0x7FFFFFu)\n{\n    return (double)x * 1.25;' + s[b:]
open(p, 'w').write(s)
PY
    ;;
    papprox) EXTRA="-DDM_ABL_PAPPROX=1" ;;
    ssync) EXTRA="-DDM_STRIP_WAVESYNC=0" ;;
    prune0) EXTRA="-DDM_PRUNE=0" ;;
    prune1) EXTRA="-DDM_PRUNE=1" ;;
    papprox2) EXTRA="-DDM_ABL_PAPPROX=2" ;;
    clk) EXTRA="-DDM_CLOCK_STAMP=1" ;;
    bwrow0) sed -i 's/^            const unsigned ti = (unsigned)q0 \* G + tw;$/            const unsigned ti = (unsigned)(q0 \& (g.h0 >> 16)) * G + tw;/' $d/csrc/dm_mfma.h
            grep -q "(unsigned)(q0 & (g.h0 >> 16)) \* G + tw;" $d/csrc/dm_mfma.h || { echo "bwrow0 patch failed"; exit 1; } ;;
    strow0) sed -i 's/^                f.b\[j\] = __builtin_amdgcn_raw_buffer_load_b128(rS1, voS, (unsigned)(rp \* NT32 + j) \* 1024u, 0);$/                f.b[j] = __builtin_amdgcn_raw_buffer_load_b128(rS1, voS, (unsigned)((rp \& (g.h0 >> 16)) * NT32 + j) * 1024u, 0);/' $d/csrc/dm_mfma.h
            grep -q "(unsigned)((rp & (g.h0 >> 16)) \* NT32 + j) \* 1024u" $d/csrc/dm_mfma.h || { echo "strow0 patch failed"; exit 1; } ;;
    nofill) sed -i 's/^    pow_lds_fill(plds, tid, 64 \* NW, false);$/    (void)plds;/' $d/csrc/dm_strip.h
            grep -q "^    (void)plds;" $d/csrc/dm_strip.h || { echo "nofill patch failed"; exit 1; } ;;
    nosw1) sed -i '457s/q0 < h0; q0 += 2) {/q0 < 0; q0 += 2) {/' $d/csrc/dm_mfma.h ;;
    pconst) sed -i 's/    const unsigned ofp = (u >> 10) \& 0x1FF0u, og = (u >> 19) \& 0xFF0u;/    const unsigned ofp = (u \& 0u), og = (u \& 0u) + 16u;/' $d/csrc/dm_kernels.hip
            grep -q "ofp = (u & 0u)" $d/csrc/dm_kernels.hip || { echo "pconst patch failed"; exit 1; } ;;
    pnoread) python3 - $d/csrc/dm_kernels.hip <<'PY'
import sys
p = sys.argv[1]; s = open(p).read()
old = """    const float ci = *(const float *)((const char *)t.fc32 + (ofp >> 2));
    const dm_d2 G = *(const dm_d2 *)((const char *)t.g32 + og);
    const dm_d2 Pr = *(const dm_d2 *)((const char *)t.fp + ofp);"""
new = """    const float ci = __uint_as_float(0x3F800000u | (ofp & 0x70u));
    const dm_d2 G = dm_d2{1.0 + (double)(og & 0x30u), 1e-17};
    const dm_d2 Pr = dm_d2{1.0 + (double)(ofp & 0x30u), 1e-17};"""
assert s.count(old) == 1
s = s.replace(old, new)
open(p, 'w').write(s)
PY
    ;;
    prow) python3 - $d/csrc/dm_kernels.hip <<'PY'
import sys
p = sys.argv[1]; s = open(p).read()
old = """    const float ci = *(const float *)((const char *)t.fc32 + (ofp >> 2));
    const dm_d2 G = *(const dm_d2 *)((const char *)t.g32 + og);
    const dm_d2 Pr = *(const dm_d2 *)((const char *)t.fp + ofp);"""
new = """    const dm_d2 G = *(const dm_d2 *)((const char *)t.g32 + og);
    const dm_d2 P0 = *(const dm_d2 *)((const char *)t.fp + ofp);
    const unsigned long long lo_ = (unsigned long long)__double_as_longlong(P0.y);
    const float ci = __uint_as_float((unsigned)lo_);
    const dm_d2 Pr = dm_d2{P0.x, (double)__uint_as_float((unsigned)(lo_ >> 32))};"""
assert s.count(old) == 1
s = s.replace(old, new)
open(p, 'w').write(s)
PY
    ;;
    smilp) EXTRA="-mllvm -amdgpu-sched-strategy=max-ilp" ;;
    smclause) EXTRA="-mllvm -amdgpu-sched-strategy=max-memory-clause" ;;
    strack) EXTRA="-mllvm -amdgpu-use-amdgpu-trackers" ;;
    vs1l2) EXTRA="-DDM_VS1_LDS=0" ;;
    hs4t2) EXTRA="-DDM_VL_HS_NW=4 -DDM_VL_HS_TR=2" ;;
    hs8t2) EXTRA="-DDM_VL_HS_NW=8 -DDM_VL_HS_TR=2" ;;
    h2n) EXTRA="-DDM_VL_H_TR=2" ;;
    h2p) EXTRA="-DDM_VL_H_TR=2 -DDM_VL_H_NT=0" ;;
    h4p) EXTRA="-DDM_VL_H_TR=4 -DDM_VL_H_NT=0" ;;
    h0p) EXTRA="-DDM_VL_H_NT=0" ;;
    h2w8) EXTRA="-DDM_VL_H_NW=8" ;;
    h2w2) EXTRA="-DDM_VL_H_NW=2" ;;
    f4m) EXTRA="-DDM_VL_F_TR=4 -DDM_VL_F_MW=4" ;;
    f4mp) EXTRA="-DDM_VL_F_TR=4 -DDM_VL_F_MW=4 -DDM_VL_F_NT=0" ;;
    f2mp) EXTRA="-DDM_VL_F_TR=2 -DDM_VL_F_MW=4 -DDM_VL_F_NT=0" ;;
    f4p) EXTRA="-DDM_VL_F_TR=4 -DDM_VL_F_NT=0" ;;
    f0p) EXTRA="-DDM_VL_F_NT=0" ;;
    hsw4) EXTRA="-DDM_VL_HS_NW=4" ;;
    fw4) EXTRA="-DDM_VL_F_NW=4" ;;
    c5h2w4) EXTRA="-DDM_VL_H2_TR=2 -DDM_VL_H2_NW=4" ;;
    c5f4m) EXTRA="-DDM_VL_F2_TR=4 -DDM_VL_F2_MW=4" ;;
    c2nb2) EXTRA="-DDM_C2_NB=2" ;;
    c3nb1) EXTRA="-DDM_C3_NB=1" ;;
    c3nb4) EXTRA="-DDM_C3_NB=4" ;;
    c5nb2) EXTRA="-DDM_C5_NB=2" ;;
    c2nb8) EXTRA="-DDM_C2_NB=8" ;;
    s0) EXTRA="-DDM_S1=0" ;;
    x0) EXTRA="-DDM_XCD_MAP=0" ;;
    s2off) EXTRA="-DDM_S2=0" ;;
    s2all) EXTRA="-DDM_S2=7" ;;
    c3mw3) EXTRA="-DDM_S2=7 -DDM_C3_MW=3" ;;
    vs0) EXTRA="-DDM_VS1=0" ;;
    head) rm -rf $d/csrc $r/include; mkdir -p $d/csrc $r/include
          (cd $REPO && for f in $(git ls-files deepmatching_stereo_matching_amd/csrc include); do
             case $f in include/*) git show HEAD:$f > $r/$f ;; *) git show HEAD:$f > $d/csrc/$(basename $f) ;; esac; done) ;;
    base) ;;
    *) echo "unknown $v"; exit 2 ;;
  esac
  (cd $d && /opt/rocm/bin/hipcc $FLAGS $EXTRA -I $r/include csrc/dm_kernels.hip csrc/dm_postproc.hip -o $REPO/ab/libdm_$v.so) &
done
wait
ls -la $REPO/ab

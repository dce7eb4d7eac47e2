"""Issue-cycle model of the fused level kernel (k_level1_mfq) for bench.py's roofline, merged
into profiles/pmc_level1.json (C3) and profiles/pmc_level1_s256.json (C5).

The kernel's ISA (hipcc -S of dm_kernels.hip, the same flags as the library) is split into
basic blocks and priced by tools/isa_cost.py (per-instruction issue cycles measured on
gfx950 by tools/valu_probe.hip, profiles/r03_valu_probe.txt); each block is weighted by how
often one wave runs it (profiles/issue_model_level1_{c3,c5}_weights.json, read off the loop
structure: sweep 1 h0/2 iterations, sweep 2 h0/2 - 2 plus two peeled, level 2 on every
second level-1 row, the level-2 stash rectified every 4th level-2 row).  The weighted instruction count is checked against the
PMC SQ_INSTS_VALU of the same build (both count MFMAs); the modelled cycles x waves per
launch is 'issue_cycles_per_launch'.

    python tools/issue_model.py [--asm /tmp/dm.s]     (compiles the asm when not given)
"""
import argparse
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'tools'))
import isa_cost  # noqa: E402
import kernel_hash  # noqa: E402

KERNELS = {  # shape -> (kernel symbol substring, weights file, pmc file, waves per launch)
    'c3': (kernel_hash.symbol('level', 128), 'issue_model_level1_c3_weights.json',
           'pmc_level1.json', 64 * (128 // 4) * (128 // 4) * 2),
    'c2': (kernel_hash.symbol('level', 64), 'issue_model_level1_c2_weights.json',
           'pmc_level1_s64.json', 64 * (64 // 4) * (64 // 4)),
    'c5': (kernel_hash.symbol('level', 256), 'issue_model_level1_c5_weights.json',
           'pmc_level1_s256.json', 256 * (256 // 4) * (256 // 4) * 4),
}


def compile_asm(out):
    src = os.path.join(REPO, 'deepmatching_stereo_matching_amd', 'csrc', 'dm_kernels.hip')
    subprocess.run(['/opt/rocm/bin/hipcc', '-O3', '-std=c++17', '-ffp-contract=off', '-Wno-pass-failed',
                    '-mllvm', '-amdgpu-mfma-vgpr-form', '--offload-arch=gfx950', '--cuda-device-only', '-S',
                    '-I', os.path.join(REPO, 'include'), src, '-o', out], check=True, cwd='/tmp')


def model(asm, kernel, weights):
    bl = isa_cost.blocks(isa_cost.kernel_lines(asm, kernel))
    w = json.load(open(weights))
    insts = cyc = 0.0
    for k, b in bl:
        n = w.get(k, w.get('_default', 1))
        insts += n * (b['valu'] + b['mfma'])
        cyc += n * b['cycles']
    return insts, cyc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--asm')
    args = ap.parse_args()
    asm = args.asm or '/tmp/dm_issue_model.s'
    if not args.asm:
        compile_asm(asm)
    for shape, (kern, wname, pname, waves) in KERNELS.items():
        insts, cyc = model(asm, kern, os.path.join(REPO, 'profiles', wname))
        path = os.path.join(REPO, 'profiles', pname)
        d = json.load(open(path)) if os.path.exists(path) else {}
        d['issue_model_insts_per_wave'] = insts
        d['issue_model_cycles_per_wave'] = round(cyc, 1)
        d['waves_per_launch'] = waves
        d['issue_cycles_per_launch'] = cyc * waves
        # the in-tree library built from the same source the asm was compiled from: bench.py
        # prices a launch with this model only while it loads the same kernel bytes
        d['issue_model_isa_sha16'] = kernel_hash.kernel_hash(kern)
        pmc = d.get('valu_insts_per_launch')
        check = ''
        if pmc:
            d['issue_model_insts_vs_pmc'] = round(insts * waves / pmc, 4)
            check = '; its instruction count is %.2f %% of the PMC SQ_INSTS_VALU' % (100.0 * insts * waves / pmc)
        d['issue_model_note'] = ('tools/issue_model.py: the ISA of this build priced per instruction by '
                                 'the probe-measured issue cycles (tools/isa_cost.py), blocks weighted by '
                                 'their executions per wave (profiles/%s)%s' % (wname, check))
        with open(path, 'w') as f:
            json.dump(d, f, indent=1)
        print(shape, json.dumps({k: d[k] for k in d if k.startswith('issue') or k == 'waves_per_launch'}))


if __name__ == '__main__':
    main()

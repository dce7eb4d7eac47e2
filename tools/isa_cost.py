"""Static VALU issue-cost model of one kernel in a hipcc device assembly listing.

Splits the kernel into basic blocks, classifies every vector instruction by the issue cost
tools/valu_probe.hip measured on gfx950 (profiles/r02_valu_probe.txt: wave64 cycles per
instruction on one SIMD, many waves):

  2.2  v_fma_f32 / v_fmac_f32, v_mul_f32, v_add_f32 / v_sub_f32, v_and_b32, v_or_b32, v_xor_b32,
       v_lshrrev_b32 / v_lshlrev_b32 / v_ashrrev_i32, v_mov_b32 (not DPP), v_add_u32 / v_sub_u32,
       v_bitop3_b32 (VOP2 / VOP1 encodings of simple 32-bit ops, VGPR / constant operands)
  4    float64 ops, packed float32, v_max/min/med3, v_max_f32 / v_min_f32, integer max / min,
       v_mul_i32_i24, DPP forms, converts, frexp / ldexp, VOP3 integer forms (bfe, and_or,
       lshl_add, mad_u32_u24, mul_lo), the cheap ops above with an SGPR operand, all else
  8    transcendental, v_permlane32_swap
  14   v_mfma_i32_16x16x64_i8 and 11.2 v_mfma_i32_16x16x32_i8: what one MFMA adds to a stream of
       independent VALU work on its SIMD (profiles/r03_valu_probe.txt: one MFMA + N v_fma_f32 per
       step takes ~13.4 + 2.4 N cycles for K=64 and ~11.2 + 2.2 N for K=32, N = 4..12; both take
       16 cycles alone)
  22   v_mfma_i32_32x32x32_i8 (the row-pair strips of sweep 1, round 5): 41.6 cycles with 8
       v_fma_f32 and 56.1 with 16 in the same probe, i.e. 24.0 / 20.9 besides their 2.2 each
       (35.9 alone)

and, given per-block execution counts per wave (--weights file: {"block": count}), the
modelled issue cycles per wave.  Without weights it prints the per-block table, which is
what the weights are read from.

    python tools/isa_cost.py dm_kernels.s KERNEL_SUBSTRING [--weights w.json] [--waves N]
"""
import argparse
import json
import re
import sys

CHEAP = re.compile(r'^v_(fma_f32|fmac_f32|mul_f32|add_f32|sub_f32|subrev_f32|and_b32|or_b32|xor_b32|'
                   r'lshrrev_b32|lshlrev_b32|ashrrev_i32|mov_b32|add_u32|sub_u32|subrev_u32|bitop3_b32)(_e32)?$')
SGPR = re.compile(r'[ ,]s(\d+|\[)')
TRANS = re.compile(r'^v_(exp|log|rcp|rsq|sqrt|sin|cos)_f32|^v_permlane32_swap')


def cost(op, line):
    if op.startswith('v_mfma'):
        if '32x32x32' in op:
            return 22.0
        return 11.2 if '16x16x32' in op else 14.0
    if TRANS.match(op):
        return 8.0
    if CHEAP.match(op) and 'dpp' not in line and '_e64' not in op and not SGPR.search(line.split(None, 1)[-1]):
        # VOP3 (_e64) forms, DPP and SGPR-operand forms measured at 4 cycles
        return 2.2
    return 4.0


def blocks(lines):
    cur, out = 'entry', {}
    order = ['entry']
    for ln in lines:
        s = ln.strip()
        m = re.match(r'^(\.LBB\d+_\d+):', s) or re.match(r'^; %(bb\.\d+):', s)
        if m:
            cur = m.group(1)
            order.append(cur)
            continue
        if not s or s.startswith(';') or s.startswith('.'):
            continue
        op = s.split()[0]
        b = out.setdefault(cur, {'valu': 0, 'cycles': 0.0, 'mfma': 0, 'lds': 0, 'vmem': 0, 'ops': {}})
        if op.startswith('v_'):
            c = cost(op, s)
            if op.startswith('v_mfma'):
                b['mfma'] += 1
            else:
                b['valu'] += 1
            b['cycles'] += c
            b['ops'][op] = b['ops'].get(op, 0) + 1
        elif op.startswith('ds_'):
            b['lds'] += 1
        elif op.startswith(('buffer_', 'global_')):
            b['vmem'] += 1
    return [(k, out[k]) for k in order if k in out]


def kernel_lines(path, name):
    lines = open(path).read().splitlines()
    start = next(i for i, ln in enumerate(lines) if ln.startswith('_Z') and name in ln and ln.rstrip().endswith(':')
                 or (name in ln and ln.split(';')[0].rstrip().endswith(':') and ln.startswith('_Z')))
    end = next(i for i in range(start, len(lines)) if lines[i].strip().startswith('.Lfunc_end'))
    return lines[start + 1:end]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('asm')
    ap.add_argument('kernel')
    ap.add_argument('--weights', help='JSON {"block": executions per wave}; unlisted blocks count '
                                      '"_default" (1 if absent)')
    ap.add_argument('--waves', type=float, default=1.0, help='waves per launch (to scale the totals)')
    args = ap.parse_args()
    bl = blocks(kernel_lines(args.asm, args.kernel))
    w = json.load(open(args.weights)) if args.weights else None
    tot_i = tot_c = 0.0
    for k, b in bl:
        n = (w or {}).get(k, (w or {}).get('_default', 1))
        tot_i += n * (b['valu'] + b['mfma'])
        tot_c += n * b['cycles']
        top = sorted(b['ops'].items(), key=lambda kv: -kv[1])[:6]
        print('%-12s x%-6g valu %4d mfma %2d lds %3d vmem %2d  cycles %7.1f  %s'
              % (k, n, b['valu'], b['mfma'], b['lds'], b['vmem'], b['cycles'],
                 ' '.join('%s:%d' % kv for kv in top)))
    if w:
        print(json.dumps({'vector_insts_per_wave': tot_i, 'issue_cycles_per_wave': round(tot_c, 1),
                          'vector_insts_per_launch': tot_i * args.waves,
                          'issue_cycles_per_launch': tot_c * args.waves}))


if __name__ == '__main__':
    sys.exit(main())

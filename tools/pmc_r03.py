"""Summarise tools/pmc_r03.sh's rocprofv3 passes into per-launch figures, one JSON per
(kernel, shape): <dir>/pmc_level1.json (C3), pmc_level1_s256.json (C5), pmc_volume_f16.json,
pmc_volume_f16_s256.json, pmc_volume.json -- the files bench.py's roofline fields read from
profiles/ (copied there after review).

Per launch, over the full-size launches (>= half the longest) of the kernel:
  hbm_bytes_per_launch = 2 x FETCH_SIZE + WRITE_SIZE (KiB x 1024; gfx950 tallies a 128-B
                         streaming read at 64 B, MI355X_MICROARCH.md HBM section)
  clock_ghz            = GRBM_GUI_ACTIVE / 8 XCDs / kernel time (DVFS note of the same guide)
  valu_busy_frac       = 4 x SQ_ACTIVE_INST_VALU / (1024 SIMDs x cycles) -- prices every VALU
                         instruction at 4 cycles (round-2 figure, an upper bound)

    python tools/pmc_r03.py gpurun_out/pmc3_<tag>
"""
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import kernel_hash  # noqa: E402

SHAPES = {  # shape -> (kernel prefix, f16 instantiation?, json name, tile, tiles)
    'l12_c3': ('k_level1_mfq', None, 'pmc_level1.json', 128, 64),
    'l12_c5': ('k_level1_mfq', None, 'pmc_level1_s256.json', 256, 256),
    'l12_c2': ('k_level1_mfq', None, 'pmc_level1_s64.json', 64, 64),
    'v16_c3': ('k_volume_ls', True, 'pmc_volume_f16.json', 128, 64),
    'v16_c5': ('k_volume_ls', True, 'pmc_volume_f16_s256.json', 256, 8),
    'v32_c3': ('k_volume_ls', False, 'pmc_volume.json', 128, 64),
    'v16mm_c3': ('k_volume_ls', True, 'pmc_volume_f16_mm.json', 128, 64),
    'v32mm_c3': ('k_volume_ls', False, 'pmc_volume_mm.json', 128, 64),
    'v32_c5': ('k_volume_ls', False, 'pmc_volume_s256.json', 256, 4),
    'v16mm_c5': ('k_volume_ls', True, 'pmc_volume_f16_mm_s256.json', 256, 8),
    'v32mm_c5': ('k_volume_ls', False, 'pmc_volume_mm_s256.json', 256, 4),
}


def _is(name, prefix):
    if prefix == 'k_level1_mfq':   # the level kernel: k_level1_mfq or (round 5) k_level12_strip
        return _is(name, 'k_level1_mfq_') or _is(name, 'k_level12_strip')
    prefix = prefix.rstrip('_')
    if name.startswith('_Z'):
        return ('%d%sI' % (len(prefix), prefix)) in name[:len(prefix) + 8]
    return name.split('<')[0].split('(')[0].strip().split()[-1] == prefix


def _f16(name):
    return '_Float16' in name or 'DF16_' in name


def _match(name, prefix, f16):
    return _is(name, prefix) and (f16 is None or _f16(name) == f16)


def launches(d, prefix, f16, skip_first=False):
    """{dispatch id: (seconds, {counter: value})} of the full-size launches in pass dir d
    (skip_first: drop the kernel's first launch -- vbench --mm's untimed standalone one)"""
    cc = glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True)
    kt = glob.glob(os.path.join(d, '**', '*kernel_trace.csv'), recursive=True)
    if not cc or not kt:
        return {}
    dur = {}
    with open(kt[0]) as f:
        for r in csv.DictReader(f):
            if _match(r['Kernel_Name'], prefix, f16):
                dur[r['Dispatch_Id']] = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) * 1e-9
    cnt = collections.defaultdict(dict)
    with open(cc[0]) as f:
        for r in csv.DictReader(f):
            if _match(r['Kernel_Name'], prefix, f16):
                c = cnt[r['Dispatch_Id']]
                c[r['Counter_Name']] = c.get(r['Counter_Name'], 0.0) + float(r['Counter_Value'])
    if skip_first and dur:
        dur.pop(min(dur, key=int))
    if not dur:
        return {}
    big = max(dur.values())
    return {k: (t, cnt[k]) for k, t in dur.items() if t >= 0.5 * big and k in cnt}


def kernel_label(sym):
    """The kernel's name (the template prefix of its mangled-name fragment), e.g.
    'k_level12_stripILi1E...' -> 'k_level12_strip'."""
    return sym.split('I', 1)[0] if 'I' in sym else sym


def mean(ls, counter):
    v = [c[counter] for _, c in ls.values() if counter in c]
    return sum(v) / len(v) if v else None


def main(root):
    out = {}
    for shape, (prefix, f16, name, tile, tiles) in SHAPES.items():
        mm = 'mm' in shape
        sq = launches(os.path.join(root, shape + '_sq'), prefix, f16, mm)
        fe = launches(os.path.join(root, shape + '_fetch'), prefix, f16, mm)
        wr = launches(os.path.join(root, shape + '_write'), prefix, f16, mm)
        if not sq and not fe:
            continue
        sym = (kernel_hash.symbol('level', tile) if prefix == 'k_level1_mfq'
               else kernel_hash.symbol('volume', tile, 2 if f16 else 4, mm))
        # the label names the instance the pass profiled (k_level1_mfq or k_level12_strip)
        label = kernel_label(sym) if sym else prefix
        d = {'kernel': label + (' (binary16)' if f16 else ''), 'tile': tile, 'tiles': tiles,
             'source': 'tools/pmc_r03.sh %s (rocprofv3 --kernel-trace --pmc, separate passes)' % shape}
        # the ISA these counters were taken on (the library the passes loaded): bench.py uses
        # the figures only while its loaded library holds the same kernel bytes
        d['isa_symbol'] = sym
        d['isa_sha16'] = kernel_hash.kernel_hash(sym) if sym else None
        if sq:
            t = sum(v[0] for v in sq.values()) / len(sq)
            grbm = mean(sq, 'GRBM_GUI_ACTIVE')
            d['launches'] = len(sq)
            d['kernel_ms_profiled'] = round(t * 1e3, 4)
            d['sq_counters_per_launch'] = {c: mean(sq, c) for c in next(iter(sq.values()))[1]}
            if grbm:
                d['gpu_cycles_per_launch'] = grbm / 8.0
                d['clock_ghz'] = round(grbm / 8.0 / t / 1e9, 4)
            v = mean(sq, 'SQ_INSTS_VALU')
            if v:
                d['valu_insts_per_launch'] = v
            m = mean(sq, 'SQ_INSTS_MFMA')
            if m:
                d['mfma_insts_per_launch'] = m
            a = mean(sq, 'SQ_ACTIVE_INST_VALU')
            if a and grbm:
                d['valu_active_cycles_per_launch'] = 4.0 * a
                d['valu_busy_frac'] = round(4.0 * a / (1024 * grbm / 8.0), 4)
        wk = launches(os.path.join(root, shape + '_work'), prefix, f16, mm)
        if wk:
            # bench.py roofline.work: per launch, the same ISA (one library for all passes)
            d['work_counters_per_launch'] = {c: mean(wk, c) for c in next(iter(wk.values()))[1]}
        f, w = mean(fe, 'FETCH_SIZE'), mean(wr, 'WRITE_SIZE')
        if f is not None and w is not None:
            d['fetch_kib'], d['write_kib'] = f, w
            d['hbm_bytes_per_launch'] = int(2 * f * 1024 + w * 1024)
            d['hbm_note'] = 'FETCH_SIZE x2 (gfx950) + WRITE_SIZE, KiB x 1024, per full-size launch'
        with open(os.path.join(root, name), 'w') as fh:
            json.dump(d, fh, indent=1)
        out[shape] = d
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main(sys.argv[1])

"""Per-launch VALU-busy cycles and effective clock of the dominant kernels from
tools/pmc_valu.sh's passes (rocprofv3 csv).

    valu_active_cycles = 4 x SQ_ACTIVE_INST_VALU   (quad-cycles summed over every wave: the
                         rocprofv3 VALUBusy numerator; / 1024 SIMDs / cycles = VALUBusy)
    clock_ghz          = GRBM_GUI_ACTIVE / 8 XCDs / kernel duration (MI355X_MICROARCH.md,
                         DVFS note; within 3 % of the in-kernel clock on >= 10 ms dispatches)

Only full-size launches count (>= half the largest duration).  Merges the figures into
profiles/pmc_level1.json and profiles/pmc_volume_f16.json when --commit is given."""
import collections
import csv
import glob
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PASSES = {'l12': ('k_level1_mfq', None, 'level1'), 'v16': ('k_volume_ls', True, 'volume_f16')}


def _is(name, prefix):
    if name.startswith('_Z'):
        return ('%d%sI' % (len(prefix), prefix)) in name[:len(prefix) + 8]
    return name.split('<')[0].split('(')[0].strip().split()[-1] == prefix


def _f16(name):
    return '_Float16' in name or 'DF16_' in name


def _rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def summarize(d, prefix, f16):
    cc = glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True)
    kt = glob.glob(os.path.join(d, '**', '*kernel_trace.csv'), recursive=True)
    if not cc or not kt:
        return None
    dur = {}
    for r in _rows(kt[0]):
        if _is(r['Kernel_Name'], prefix) and (f16 is None or _f16(r['Kernel_Name']) == f16):
            dur[r.get('Dispatch_Id')] = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) * 1e-9
    by = collections.defaultdict(dict)
    for r in _rows(cc[0]):
        if _is(r['Kernel_Name'], prefix) and (f16 is None or _f16(r['Kernel_Name']) == f16):
            by[r.get('Dispatch_Id')][r['Counter_Name']] = \
                by[r.get('Dispatch_Id')].get(r['Counter_Name'], 0.0) + float(r['Counter_Value'])
    if not dur:
        return None
    big = max(dur.values())
    keep = [k for k, t in dur.items() if t >= 0.5 * big and k in by]
    if not keep:
        return None
    mean = {c: sum(by[k].get(c, 0.0) for k in keep) / len(keep) for c in by[keep[0]]}
    t = sum(dur[k] for k in keep) / len(keep)
    out = {'launches': len(keep), 'kernel_ms_profiled': round(t * 1e3, 4), 'counters': mean}
    if 'SQ_ACTIVE_INST_VALU' in mean:
        out['valu_active_cycles_per_launch'] = 4.0 * mean['SQ_ACTIVE_INST_VALU']
    if 'GRBM_GUI_ACTIVE' in mean:
        out['gpu_cycles_per_launch'] = mean['GRBM_GUI_ACTIVE'] / 8.0
        out['clock_ghz'] = round(mean['GRBM_GUI_ACTIVE'] / 8.0 / t / 1e9, 4)
        if 'SQ_ACTIVE_INST_VALU' in mean:
            out['valu_busy_frac'] = round(out['valu_active_cycles_per_launch'] /
                                          (1024 * mean['GRBM_GUI_ACTIVE'] / 8.0), 4)
    if 'SQ_INSTS_VALU' in mean:
        out['valu_insts_per_launch'] = mean['SQ_INSTS_VALU']
    return out


def main(root, commit=False):
    for sub, (prefix, f16, key) in PASSES.items():
        s = summarize(os.path.join(root, sub), prefix, f16)
        print(sub, json.dumps(s, indent=1))
        if commit and s:
            path = os.path.join(REPO, 'profiles', 'pmc_%s.json' % key)
            d = json.load(open(path)) if os.path.exists(path) else {}
            for k in ('valu_active_cycles_per_launch', 'gpu_cycles_per_launch', 'clock_ghz', 'valu_busy_frac',
                      'valu_insts_per_launch', 'kernel_ms_profiled'):
                if k in s:
                    d[k] = s[k]
            d['sq_counters_per_launch'] = s['counters']
            d['valu_note'] = ('tools/pmc_valu.sh: SQ_ACTIVE_INST_VALU x4 = VALU-busy SIMD-cycles; '
                              'clock = GRBM_GUI_ACTIVE/8/t; full-size launches only')
            with open(path, 'w') as fh:
                json.dump(d, fh, indent=1)


if __name__ == '__main__':
    main(sys.argv[1], '--commit' in sys.argv)

"""Mean per-launch counters of the full-size launches of each kernel under a pmc_mem.sh
output directory, plus derived per-CU busy fractions (TA/TD busy sums over 256 CUs /
(GRBM_GUI_ACTIVE / 8 XCDs))."""
import collections
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from valu_summary import _rows  # noqa: E402


COMMIT = {'mem_l12': 'level1', 'mem_v16': 'volume_f16'}


def main(root, commit=False):
    for d in sorted(glob.glob(os.path.join(root, '*_*'))):
        if not os.path.isdir(d):
            continue
        cc = glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True)
        kt = glob.glob(os.path.join(d, '**', '*kernel_trace.csv'), recursive=True)
        if not cc or not kt:
            continue
        dur = {}
        names = {}
        for r in _rows(kt[0]):
            dur[r['Dispatch_Id']] = int(r['End_Timestamp']) - int(r['Start_Timestamp'])
            names[r['Dispatch_Id']] = r['Kernel_Name']
        by = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in _rows(cc[0]):
            by[r['Dispatch_Id']][r['Counter_Name']] += float(r['Counter_Value'])
        longest = max(dur, key=dur.get)
        name = names[longest].split('(')[0][:70]
        keep = [k for k in by if names.get(k) == names[longest] and dur[k] >= 0.5 * dur[longest]]
        mean = {c: sum(by[k][c] for k in keep) / len(keep) for c in by[keep[0]]}
        t = sum(dur[k] for k in keep) / len(keep) * 1e-9
        print('%s  %s  launches=%d  t=%.3f ms' % (os.path.basename(d), name, len(keep), t * 1e3))
        cyc = mean.get('GRBM_GUI_ACTIVE', 0) / 8.0
        for c, v in sorted(mean.items()):
            extra = ''
            if cyc and c in ('TA_TA_BUSY_sum', 'TD_TD_BUSY_sum', 'TA_BUFFER_TOTAL_CYCLES_sum', 'TD_TC_STALL_sum'):
                extra = '   per-CU busy frac %.3f' % (v / 256.0 / cyc)
            print('    %-32s %16.6g%s' % (c, v, extra))
        key = COMMIT.get(os.path.basename(d))
        if commit and key and cyc:
            path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'profiles',
                                'pmc_%s.json' % key)
            rec = json.load(open(path)) if os.path.exists(path) else {}
            rec['ta_busy_frac'] = round(mean['TA_TA_BUSY_sum'] / 256.0 / cyc, 4)
            rec['td_busy_frac'] = round(mean['TD_TD_BUSY_sum'] / 256.0 / cyc, 4)
            rec['tcp_accesses_per_launch'] = mean.get('TCP_TOTAL_CACHE_ACCESSES_sum')
            rec['mem_note'] = ('tools/pmc_mem.sh: TA_TA_BUSY_sum, TD_TD_BUSY_sum over 256 CUs / '
                               '(GRBM_GUI_ACTIVE / 8); vector-memory pipe occupancy')
            with open(path, 'w') as fh:
                json.dump(rec, fh, indent=1)


if __name__ == '__main__':
    main(sys.argv[1], '--commit' in sys.argv)

"""Cross-check of bench.py's HIP-event timing against a rocprofv3 kernel trace of the same
command: the level kernel's launch durations in order, and the mean over the timed launches.

    python tools/level_launches.py <rocprofv3 -d dir> <bench json> <tag text> > profiles/<tag>_level_kernel_launches.txt
"""
import csv
import glob
import json
import os
import sys


def main(root, bench, label):
    kt = glob.glob(os.path.join(root, '**', '*kernel_trace.csv'), recursive=True)
    rows = []
    for path in kt:
        with open(path) as f:
            for r in csv.DictReader(f):
                if r['Kernel_Name'].lstrip('void ').startswith(('k_level1_mfq', 'k_level12_strip')):
                    rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'].split('(')[0]))
    rows.sort()
    d = json.loads(open(bench).read().strip().splitlines()[-1])
    warm, steps = d['warmup'], d['steps']
    ms = [(e - s) * 1e-6 for s, e, _ in rows]
    timed = ms[warm:warm + steps]
    print('%s, full C3 grid, rocprofv3 --kernel-trace --stats -- python3 bench.py --no-cpu-baseline (%s)'
          % (rows[0][2] if rows else '?', label))
    print('launch durations (ms), in order (%d warm-up, %d timed, then the k_level line and the volume checks): %s'
          % (warm, steps, ', '.join('%.3f' % m for m in ms)))
    print('mean of the %d timed launches (%d..%d): %.3f ms; bench.py HIP events on the same run: %.3f ms'
          % (steps, warm, warm + steps - 1, sum(timed) / len(timed), d['roofline']['ms']))


if __name__ == '__main__':
    main(*sys.argv[1:4])

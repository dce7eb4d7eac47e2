"""Timeline of the pipelined bench from a rocprofv3 kernel trace: where the time per pair goes
besides the level kernel.

For the timed launches of k_level1_mfq (bench.py's warm-up skipped) it reports the mean
duration, the mean start-to-start period, the idle gap between one level kernel's end and
the next one's start, and for every other kernel the GPU time it spent overlapping a level
kernel vs inside the gaps (per pair).

    python tools/gap_trace.py <rocprofv3 -d dir> [--warmup 5] [--steps 20]
"""
import argparse
import collections
import csv
import glob
import os

LEVEL = ('k_level1_mfq', 'k_level12_strip')   # the level kernel (round 5: the strip form for S = 64, 256)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('root')
    ap.add_argument('--warmup', type=int, default=5)
    ap.add_argument('--steps', type=int, default=20)
    args = ap.parse_args()
    rows = []
    for path in glob.glob(os.path.join(args.root, '**', '*kernel_trace.csv'), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                name = r['Kernel_Name'].replace('void ', '').split('(')[0].split('<')[0]
                rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), name))
    rows.sort()
    lv = [r for r in rows if r[2] in LEVEL]
    timed = lv[args.warmup:args.warmup + args.steps + 1]
    t0, t1 = timed[0][0], timed[-1][0]          # steps periods, start to start
    n = len(timed) - 1
    dur = sum(e - s for s, e, _ in timed[:-1]) / n
    per = (t1 - t0) / n
    busy = [(s, e) for s, e, _ in timed]
    inside = collections.Counter()
    outside = collections.Counter()
    calls = collections.Counter()
    for s, e, name in rows:
        if name in LEVEL or e <= t0 or s >= t1:
            continue
        s, e = max(s, t0), min(e, t1)
        ov = sum(max(0, min(e, b1) - max(s, b0)) for b0, b1 in busy)
        inside[name] += ov
        outside[name] += (e - s) - ov
        calls[name] += 1
    print('timed level kernels: %d periods; mean duration %.3f ms, mean period %.3f ms, mean gap %.3f ms'
          % (n, dur * 1e-6, per * 1e-6, (per - dur) * 1e-6))
    print('%-28s %6s %14s %14s' % ('kernel', 'calls', 'ms/pair beside', 'ms/pair in gap'))
    for name in sorted(calls, key=lambda k: -(inside[k] + outside[k])):
        print('%-28s %6.1f %14.4f %14.4f' % (name, calls[name] / n, inside[name] * 1e-6 / n, outside[name] * 1e-6 / n))


if __name__ == '__main__':
    main()

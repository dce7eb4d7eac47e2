"""Average each PMC counter per kernel over the dispatches of every pass under a directory
written by tools/pmc.sh (rocprofv3 csv output)."""
import collections
import csv
import glob
import os
import sys


def main(root):
    acc = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(root, 'p*', 'run_counter_collection.csv'))):
        for r in csv.DictReader(open(f)):
            name = r['Kernel_Name'].split('(')[0][:60]
            acc[(name, r['Counter_Name'])].append(float(r['Counter_Value']))
    for (k, cn), v in sorted(acc.items()):
        if k.startswith('__amd'):
            continue
        print('%-60s %-28s n=%-3d mean=%.6g' % (k, cn, len(v), sum(v) / len(v)))


if __name__ == '__main__':
    main(sys.argv[1])

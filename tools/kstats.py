"""Per-kernel launch statistics from a rocprofv3 kernel trace, split by grid size, so the
full-size bench launches are not averaged with the small test-size ones.

    python tools/kstats.py <rocprofv3 -d dir> > profiles/<tag>_kernel_stats_by_grid.csv
"""
import collections
import csv
import glob
import os
import sys


def main(root):
    kt = glob.glob(os.path.join(root, '**', '*kernel_trace.csv'), recursive=True)
    acc = collections.defaultdict(list)
    for path in kt:
        with open(path) as f:
            for r in csv.DictReader(f):
                name = r['Kernel_Name'].split('(')[0].replace(',', ';')[:90]
                grid = r.get('Grid_Size') or 'x'.join(r[k] for k in ('Grid_Size_X', 'Grid_Size_Y', 'Grid_Size_Z'))
                wg = r.get('Workgroup_Size') or 'x'.join(r[k] for k in ('Workgroup_Size_X', 'Workgroup_Size_Y',
                                                                         'Workgroup_Size_Z'))
                acc[(name, grid, wg)].append(
                    int(r['End_Timestamp']) - int(r['Start_Timestamp']))
    w = csv.writer(sys.stdout)
    w.writerow(['Kernel_Name', 'Grid_Size', 'Workgroup_Size', 'Calls', 'TotalNs', 'AverageNs', 'MinNs', 'MaxNs'])
    for (name, grid, wg), v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
        w.writerow([name, grid, wg, len(v), sum(v), round(sum(v) / len(v), 1), min(v), max(v)])


if __name__ == '__main__':
    main(sys.argv[1])

"""Per-launch HBM bytes of the level-1 and volume kernels from tools/profile.sh's PMC
passes: FETCH_SIZE (KiB, x2: gfx950 tallies 128-B reads at 64 B, MI355X_MICROARCH.md HBM
section) + WRITE_SIZE (KiB).  Writes <dir>/pmc_level1.json, <dir>/pmc_volume.json and
<dir>/pmc_volume_f16.json (the binary16 instantiation of the volume kernel)."""
import csv
import json
import os
import sys

# key: (kernel name prefixes, f16 instantiation?)
KERNELS = {'level1': (('k_level1_mfq', 'k_level12_strip'), None), 'volume': (('k_volume_ls', 'k_volume_cs', 'k_volume_mfq'), False),
           'volume_f16': (('k_volume_ls', 'k_volume_cs'), True)}


def _is(name, prefix):
    """demangled ('void k_volume_cs<...>(...)') or mangled ('_Z11k_volume_csI...') name"""
    if name.startswith('_Z'):
        return ('%d%sI' % (len(prefix), prefix)) in name[:len(prefix) + 8]
    return name.split('<')[0].split('(')[0].strip().split()[-1] == prefix


def _f16(name):
    return '_Float16' in name or 'DF16_' in name


def per_launch(path, counter, prefix, f16=None):
    """mean over the full-size launches (>= half the largest: bench.py's one-tile flip-rate
    batches use the same kernel on far fewer tiles)"""
    vals = [float(r['Counter_Value']) for r in csv.DictReader(open(path))
            if r['Counter_Name'] == counter and _is(r['Kernel_Name'], prefix)
            and (f16 is None or _f16(r['Kernel_Name']) == f16)]
    if not vals:
        return None
    big = [v for v in vals if v >= 0.5 * max(vals)]
    return sum(big) / len(big)


def main(root, tile):
    for key, (prefixes, f16) in KERNELS.items():
        for prefix in prefixes:
            f = per_launch(os.path.join(root, 'fetch', 'run_counter_collection.csv'), 'FETCH_SIZE', prefix, f16)
            w = per_launch(os.path.join(root, 'write', 'run_counter_collection.csv'), 'WRITE_SIZE', prefix, f16)
            if f is not None and w is not None:
                break
        if f is None or w is None:
            continue
        d = {'kernel': prefix, 'tile': tile, 'fetch_kib': f, 'write_kib': w,
             'hbm_bytes_per_launch': int(2 * f * 1024 + w * 1024),
             'note': 'FETCH_SIZE x2 (gfx950) + WRITE_SIZE, mean over the launches of bench.py'}
        sq = os.path.join(root, 'sq', 'run_counter_collection.csv')
        if key == 'level1' and os.path.exists(sq):
            v = per_launch(sq, 'SQ_INSTS_VALU', prefix)
            if v is not None:
                d['valu_insts_per_launch'] = v
        with open(os.path.join(root, 'pmc_%s.json' % key), 'w') as fh:
            json.dump(d, fh, indent=1)
        print(json.dumps(d))


if __name__ == '__main__':
    main(sys.argv[1], int(sys.argv[2]))

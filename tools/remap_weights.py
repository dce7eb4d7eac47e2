"""Carry an issue-model weights file (tools/issue_model.py) over to a new build of the same
kernel: the basic blocks of the old and new ISA are aligned by their instruction multisets
(difflib over per-block signatures) and each new block takes the weight of the old block it
matches; unmatched blocks take the weight of the nearest matched block before them.  The
result is checked the usual way: its instruction count against the PMC SQ_INSTS_VALU of a
run of the new build.

    python tools/remap_weights.py old.s OLD_KERNEL old_weights.json new.s NEW_KERNEL [LABEL=N ...] > new.json

LABEL=N arguments set a block's weight by hand (a block the alignment cannot match: new code,
or a loop whose trip count changed).
"""
import difflib
import json
import sys

import isa_cost


def sig(b):
    return tuple(sorted(b['ops'].items())) + (b['lds'], b['vmem'])


def main(old_s, old_k, old_w, new_s, new_k, *sets):
    ob = isa_cost.blocks(isa_cost.kernel_lines(old_s, old_k))
    nb = isa_cost.blocks(isa_cost.kernel_lines(new_s, new_k))
    w = json.load(open(old_w))
    dflt = w.get('_default', 1)
    ow = [w.get(k, dflt) for k, _ in ob]
    sm = difflib.SequenceMatcher(None, [sig(b) for _, b in ob], [sig(b) for _, b in nb], autojunk=False)
    nw = [None] * len(nb)
    for i, j, n in sm.get_matching_blocks():
        for d in range(n):
            nw[j + d] = ow[i + d]
    # near-matches (same position in a replaced run of equal length)
    for tag, i1, i2, j1, j2 in sm.get_opcodes():
        if tag == 'replace' and i2 - i1 == j2 - j1:
            for d in range(i2 - i1):
                nw[j1 + d] = ow[i1 + d]
    last = dflt
    out = {'_default': dflt}
    for (k, _), v in zip(nb, nw):
        if v is None:
            v = last
        out[k] = v
        last = v
    for kv in sets:
        k, v = kv.split('=')
        assert k in out, 'no block ' + k
        out[k] = float(v) if '.' in v else int(v)
    if '_build' in w:
        out['_build'] = w['_build']
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == '__main__':
    main(*sys.argv[1:])

"""ISA identity of one kernel in a built library: sha256 of its machine code and its kernel
descriptor, read from the gfx950 code objects embedded in libdmstereo.so.

bench.py's level-kernel roofline prices the live launch time with an issue-cycle model of
ONE build's ISA (profiles/pmc_level1*.json, tools/issue_model.py).  The profile records this
hash of the kernel it modelled; bench.py recomputes it from the library it actually loaded
and reports frac: null (with the reason) when they differ, so a kernel change without a
refreshed profile can no longer print a confident, wrong fraction.

    python tools/kernel_hash.py [--lib path/to/libdmstereo.so] SYMBOL_SUBSTRING...
"""
import argparse
import hashlib
import os
import struct
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EM_AMDGPU = 224

# the kernel instance each profiled shape launches (mangled-name substrings, unique in the
# library): (kind, tile, bytes per voxel or None) -> symbol
LEVEL = {64: 'k_level1_mfqILi1ELi4ELi4ELi4ELb1ELb1ELi4ELb1EE',      # C2: 4 one-wave blocks per workgroup
         128: 'k_level1_mfqILi1ELi4ELi4ELi4ELb1ELb1ELi2ELb1EE',     # C3: GW = 4, 2 two-wave blocks
         256: 'k_level1_mfqILi1ELi4ELi4ELi4ELb1ELb1ELi1ELb1EE'}     # C5: GW = 4, 4 waves
# k_volume_ls<G, NW, NT, OT, TR, MW>: (tile, bytes per voxel, min/max known) -> instance
# (dm_kernels.hip launch_volume_ls: DM_VL_H_* / DM_VL_F_* at w0 = 128, TR 0 elsewhere)
VOLUME = {(128, 4, False): 'k_volume_lsILi8ELi8ELb1EfLi4ELi4E', (128, 4, True): 'k_volume_lsILi8ELi8ELb1EfLi4ELi4E',
          (128, 2, False): 'k_volume_lsILi8ELi8ELb1EDF16_Li0ELi1E',
          (128, 2, True): 'k_volume_lsILi8ELi4ELb1EDF16_Li2ELi1E',
          (256, 4, False): 'k_volume_lsILi16ELi8ELb1EfLi0ELi1E', (256, 4, True): 'k_volume_lsILi16ELi8ELb1EfLi0ELi1E',
          (256, 2, False): 'k_volume_lsILi16ELi8ELb1EDF16_Li0ELi1E',
          (256, 2, True): 'k_volume_lsILi16ELi8ELb1EDF16_Li0ELi1E'}


def symbol(kind, tile, esz=None, mm=False):
    """The symbol substring of the level kernel ('level') or a volume kernel ('volume', esz
    bytes per voxel, min/max known or not) that a tile of side `tile` launches; None if not
    profiled."""
    return LEVEL.get(tile) if kind == 'level' else VOLUME.get((tile, esz, bool(mm)))


def _elfs(data):
    """(offset, bytes view) of every embedded little-endian ELF64 for EM_AMDGPU."""
    i = data.find(b'\x7fELF')
    while i >= 0:
        if data[i + 4] == 2 and data[i + 5] == 1 and struct.unpack_from('<H', data, i + 18)[0] == EM_AMDGPU:
            yield i
        i = data.find(b'\x7fELF', i + 4)


def _symbols(data, base):
    """name -> (file offset of the symbol's bytes, size) for one embedded ELF64 at `base`."""
    shoff, = struct.unpack_from('<Q', data, base + 0x28)
    shentsize, shnum = struct.unpack_from('<HH', data, base + 0x3A)
    secs = []
    for k in range(shnum):
        o = base + shoff + k * shentsize
        name, typ, flags, addr, off, size, link, info, align, entsize = struct.unpack_from('<IIQQQQIIQQ', data, o)
        secs.append((typ, addr, off, size, link, entsize))
    out = {}
    for typ, addr, off, size, link, entsize in secs:
        if typ != 2:     # SHT_SYMTAB
            continue
        stroff = secs[link][2]
        for j in range(size // entsize):
            o = base + off + j * entsize
            st_name, st_info, st_other, st_shndx, st_value, st_size = struct.unpack_from('<IBBHQQ', data, o)
            if not st_name or st_shndx == 0 or st_shndx >= len(secs):
                continue
            end = data.index(b'\0', base + stroff + st_name)
            nm = data[base + stroff + st_name:end].decode()
            s_addr, s_off = secs[st_shndx][1], secs[st_shndx][2]
            out[nm] = (base + s_off + (st_value - s_addr), st_size)
    return out


def kernel_hash(symbol_substring, lib=None):
    """sha256 (hex, 16 chars) of the machine code + kernel descriptor (less its code offset) of
    the ONE kernel whose mangled name contains `symbol_substring`; None if the library or the
    kernel is absent."""
    lib = lib or os.environ.get('DM_LIB_PATH') or os.path.join(
        REPO, 'deepmatching_stereo_matching_amd', 'libdmstereo.so')
    try:
        data = open(lib, 'rb').read()
    except OSError:
        return None
    found = []
    for base in _elfs(data):
        syms = _symbols(data, base)
        for nm, (off, size) in syms.items():
            if symbol_substring in nm and not nm.endswith('.kd') and size:
                kd = syms.get(nm + '.kd')
                h = hashlib.sha256(data[off:off + size])
                if kd:
                    # the descriptor without kernel_code_entry_byte_offset (bytes 16-23): that
                    # field is where the linker put the code relative to the descriptor, which
                    # moves whenever another kernel of the library is added or grows
                    d = bytearray(data[kd[0]:kd[0] + kd[1]])
                    d[16:24] = bytes(8)
                    h.update(bytes(d))
                found.append((nm, h.hexdigest()[:16]))
    if len(found) != 1:
        return None
    return found[0][1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--lib')
    ap.add_argument('symbols', nargs='+')
    args = ap.parse_args()
    for s in args.symbols:
        print(s, kernel_hash(s, args.lib))


if __name__ == '__main__':
    sys.exit(main())

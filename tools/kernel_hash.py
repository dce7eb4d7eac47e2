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

# The kernel instance each profiled shape launches depends on the library's compile-time
# switches (dm_kernels.hip: DM_S1, DM_S2, DM_C*_NB, DM_VL_*), which the library reports through
# dm_build_config(); the symbols below are derived from it, so an A/B build made with -D
# overrides (tools/abl_build.sh) is looked up under its own instances.  A library without
# dm_build_config (before round 5) uses the round-4 instances (LEGACY).
LEVEL = (64, 128, 256)       # profiled level-kernel tiles: C2, C3, C5
VOLUME = ((128, 4, False), (128, 4, True), (128, 2, False), (128, 2, True),
          (256, 4, False), (256, 4, True), (256, 2, False), (256, 2, True))
# DEFAULTS mirror the C defaults of dm_kernels.hip (every key dm_build_config reports); they
# only fill keys a library's config string lacks -- a library that cannot be loaded at all is
# an error (symbol() raises), never a guess.
DEFAULTS = {'S1': 1, 'S2': 5, 'PRUNE': 0, 'STRIP_WAVESYNC': 0, 'VS1': 1, 'VS1_LDS': 1, 'XCD_MAP': 1, 'C2_NB': 4, 'C3_NB': 2, 'C3_MW': 4,
            'C3_MINW': 4, 'C5_NB': 1, 'VL_H_TR': 2, 'VL_H_NT': 1, 'VL_H_NW': 4,
            'VL_H2_TR': 0, 'VL_H2_NW': 8, 'VL_F2_TR': 0, 'VL_F2_MW': 1, 'VL_HS_NW': 8, 'VL_HS_TR': 0,
            'VL_F_NW': 8, 'VL_F_TR': 4, 'VL_F_MW': 4, 'VL_F_NT': 1}
LEGACY = {('level', 64): 'k_level1_mfqILi1ELi4ELi4ELi4ELb1ELb1ELi4ELb1EE',
          ('level', 128): 'k_level1_mfqILi1ELi4ELi4ELi4ELb1ELb1ELi2ELb1EE',
          ('level', 256): 'k_level1_mfqILi1ELi4ELi4ELi4ELb1ELb1ELi1ELb1EE'}
_CONFIG = {}


def _lib_path(lib=None):
    return lib or os.environ.get('DM_LIB_PATH') or os.path.join(
        REPO, 'deepmatching_stereo_matching_amd', 'libdmstereo.so')


def build_config(lib=None):
    """The library's compile-time switches as a dict (dm_build_config()); None if the library
    cannot be loaded, {} if it predates dm_build_config."""
    path = _lib_path(lib)
    if path not in _CONFIG:
        try:
            import ctypes
            h = ctypes.CDLL(path)
        except OSError:
            return None
        try:
            fn = h.dm_build_config
        except AttributeError:
            _CONFIG[path] = {}
        else:
            fn.restype = ctypes.c_char_p
            _CONFIG[path] = {k: int(v) for k, v in (kv.split('=') for kv in fn().decode().split())}
    return _CONFIG[path]


def symbol(kind, tile, esz=None, mm=False, lib=None):
    """The symbol substring of the level kernel ('level') or a volume kernel ('volume', esz
    bytes per voxel, min/max known or not) that a tile of side `tile` launches in `lib` (the
    loaded one by default); None if not profiled."""
    cfg = build_config(lib)
    if cfg is None:
        raise RuntimeError('kernel_hash.symbol: cannot load %s to read its build config' % _lib_path(lib))
    if cfg == {} and kind == 'level':
        return LEGACY.get((kind, tile))
    c = dict(DEFAULTS, **cfg)
    if kind == 'level':
        if tile not in LEVEL:
            return None
        nb = c['C2_NB'] if tile == 64 else c['C3_NB'] if tile == 128 else c['C5_NB']
        nwc = 1 if tile == 64 else 2 if tile == 128 else 4
        if (c['S2'] >> {64: 0, 128: 1, 256: 2}[tile]) & 1:   # both sweeps on the strips (dm_strip.h)
            return 'k_level12_stripILi%dELi%dELb1ELb1ELi%dEE' % (nwc, nb, c['C3_MW'] if tile == 128 else 4)
        if tile == 128 and c['PRUNE']:   # round 6: the pruned C3 kernel (dm_prune.h), when built in
            return 'k_level12_pruneILi2ELi%dELi%dEE' % (nb, c['C3_MINW'])
        minw = c['C3_MINW'] if tile == 128 else 4
        return 'k_level1_mfqILi1ELi4ELi%dELi%dELb1ELb1ELi%dELb1ELb%dEE' % (nb * nwc, minw, nb, c['S1'])
    if (tile, esz, bool(mm)) not in VOLUME:
        return None
    if tile == 128 and esz == 4:
        return 'k_volume_lsILi8ELi%dELb%dEfLi%dELi%dE' % (c['VL_F_NW'], c['VL_F_NT'], c['VL_F_TR'], c['VL_F_MW'])
    if tile == 128:
        if mm:
            return 'k_volume_lsILi8ELi%dELb%dEDF16_Li%dELi1E' % (c['VL_H_NW'], c['VL_H_NT'], c['VL_H_TR'])
        return 'k_volume_lsILi8ELi%dELb1EDF16_Li%dELi1E' % (c['VL_HS_NW'], c['VL_HS_TR'])
    if esz == 4:
        return 'k_volume_lsILi16ELi8ELb1EfLi%dELi%dE' % (c['VL_F2_TR'], c['VL_F2_MW'])
    if mm:
        return 'k_volume_lsILi16ELi%dELb1EDF16_Li%dELi1E' % (c['VL_H2_NW'], c['VL_H2_TR'])
    return 'k_volume_lsILi16ELi8ELb1EDF16_Li0ELi1E'


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


def _mask_pc_literals(code):
    """The code with the 32-bit literals of `s_getpc_b64` + `s_add_u32` / `s_addc_u32` zeroed:
    those are the PC-relative offsets of the constant tables (the pow tables' rel32 relocations),
    which move whenever another kernel of the library grows -- not part of this kernel's ISA.
    gfx9 encodings: s_getpc_b64 = SOP1 0xBE80_1C00 | sdst << 16; the adds are SOP2 (bits 31:30 =
    0b10) with ssrc1 = 0xFF, the literal in the next word."""
    n = len(code) // 4
    w = list(struct.unpack_from('<%dI' % n, code))
    for i in range(n):
        if (w[i] & 0xFF80FF00) != 0xBE801C00:
            continue
        j = i + 1
        for _ in range(2):
            if j + 1 < n and (w[j] >> 30) == 2 and ((w[j] >> 8) & 0xFF) == 0xFF:
                w[j + 1] = 0
                j += 2
    return struct.pack('<%dI' % n, *w) + code[4 * n:]


def kernel_hash(symbol_substring, lib=None):
    """sha256 (hex, 16 chars) of the machine code (PC-relative table offsets masked,
    _mask_pc_literals) + kernel descriptor (less its code offset) of the ONE kernel whose
    mangled name contains `symbol_substring`; None if the library or the kernel is absent."""
    lib = _lib_path(lib)
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
                h = hashlib.sha256(_mask_pc_literals(data[off:off + size]))
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

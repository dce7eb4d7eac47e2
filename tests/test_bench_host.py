"""bench.py's host logic on CPU: the roofline fraction is tied to the build it describes
(VERDICT r3 "Next" 5).  The committed profiles carry the sha256 of the profiled kernel's
machine code + descriptor (tools/kernel_hash.py, read from the gfx950 code objects inside
libdmstereo.so); bench.py reports frac: null with the reason when the loaded library's kernel
differs."""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'tools'))


@pytest.fixture(scope='module')
def bench():
    import bench as b
    return b


def test_every_profiled_kernel_is_in_the_library():
    import kernel_hash as K
    hashes = {}
    for tile in K.LEVEL:
        hashes[('level', tile)] = K.kernel_hash(K.symbol('level', tile))
    for tile, esz, mm in K.VOLUME:
        hashes[('volume', tile, esz, mm)] = K.kernel_hash(K.symbol('volume', tile, esz, mm))
    assert all(h and len(h) == 16 for h in hashes.values()), hashes
    syms = {K.symbol(*k) for k in hashes}
    assert len(set(hashes.values())) == len(syms)            # one hash per distinct instance
    assert K.kernel_hash('no_such_kernel') is None
    assert K.kernel_hash('k_level1_mfq') is None             # ambiguous: many instances


class _Batch:
    T = 64


class _Solver:
    batch = _Batch()


def test_frac_null_for_a_stale_profile(bench, monkeypatch):
    import kernel_hash as K
    cur = K.kernel_hash(K.symbol('level', 128))
    good = {'tile': 128, 'tiles': 64, 'issue_cycles_per_launch': 13.0e9, 'gpu_cycles_per_launch': 14.0e6,
            'clock_ghz': 1.7, 'kernel_ms_profiled': 8.0, 'hbm_bytes_per_launch': 1.2e9,
            'issue_model_isa_sha16': cur, 'isa_sha16': cur}
    monkeypatch.setattr(bench, 'load_pmc', lambda *a, **k: dict(good))
    r = bench.level_roofline(_Solver(), 128, 7.5)
    assert r['frac'] == pytest.approx(13.0e9 / 7.5e-3 / 1e9 / (1024 * 2.4), abs=1e-4)
    assert r['traffic'] == 1.2e9 and 'issue_occupancy_profiled' in r

    stale = dict(good, issue_model_isa_sha16='0123456789abcdef')
    monkeypatch.setattr(bench, 'load_pmc', lambda *a, **k: dict(stale))
    r = bench.level_roofline(_Solver(), 128, 7.5)
    assert r['frac'] is None and r['achieved'] is None
    assert 'stale profile' in r['source']['issue_cycles_per_launch']
    assert r['traffic'] == 1.2e9                            # the PMC pass itself is current

    stale_pmc = dict(good, isa_sha16=None)
    monkeypatch.setattr(bench, 'load_pmc', lambda *a, **k: dict(stale_pmc))
    r = bench.level_roofline(_Solver(), 128, 7.5)
    assert r['frac'] is not None                            # model current
    assert r['traffic'] is None and 'issue_occupancy_profiled' not in r
    assert 'stale profile' in r['isa_check']['pmc']


def test_volume_traffic_needs_a_current_profile(bench, monkeypatch):
    import kernel_hash as K
    cur = K.kernel_hash(K.symbol('volume', 128, 2))
    monkeypatch.setattr(bench, 'load_pmc', lambda *a, **k: {'hbm_bytes_per_launch': 35e9, 'isa_sha16': cur})
    assert bench.load_traffic(128, 'volume_f16', 64) == 35e9
    assert bench.load_traffic(128, 'volume', 64) is None     # float32 instance: other bytes
    assert bench.load_traffic(128, 'volume_f16_mm', 64) is None   # min/max-known instance
    monkeypatch.setattr(bench, 'load_pmc', lambda *a, **k: {'hbm_bytes_per_launch': 35e9})
    assert bench.load_traffic(128, 'volume_f16', 64) is None


def test_store_ceiling_follows_the_instance_pattern(bench):
    # the w0 = 128 instances store 2 x 512 B (binary16, min/max known) or 1 KB (float32) per
    # instruction; the others 4 x 256 B -- each line is priced against its own pattern
    h_mm = bench.store_ceiling(128, 64, 2, 5000.0, mm=True)
    h = bench.store_ceiling(128, 64, 2, 5000.0)
    f = bench.store_ceiling(128, 64, 4, 5000.0)
    c5 = bench.store_ceiling(256, 8, 2, 5000.0, mm=True)
    assert '"volh_nt"' in h_mm['source'] and '"vol_nt"' in h['source']
    assert '"volx_nt"' in f['source'] and '"vol_nt"' in c5['source']
    assert h_mm['frac'] == round(5000.0 / h_mm['gb_s'], 4)
    assert bench.store_ceiling(64, 64, 2, 5000.0) is None


def test_roofline_work_derivation(bench, monkeypatch):
    """roofline.work: MAC slots from the PMC MFMA math-op counter and pow
    evaluations from the float64 FMA count, each against the algorithmic count; present only
    with a work pass made on the loaded ISA."""
    import kernel_hash as K
    cur = K.kernel_hash(K.symbol('level', 128))
    V = 64 * 128.0 ** 4
    # round 5's C3 launch: 16.8 M 32x32x32 + 67.1 M 16x16x32 i8 MFMAs = 1.0995 T multiply-adds;
    # 4 child pows per level-1 value (V/4) + V/64 + V/256 pooled ones, 7 float64 FMAs each
    macs = 16777216 * 32768 + 67108864 * 8192
    pows = V * (0.25 + 1 / 64.0 + 1 / 256.0)
    work = {'SQ_INSTS_VALU_MFMA_MOPS_I8': macs * 2 / 512.0, 'SQ_INSTS_VALU_FMA_F64': pows * 7 / 64.0,
            'SQ_INSTS_VALU_MUL_F64': 1.0, 'SQ_INSTS_VALU_ADD_F64': 2.0}
    good = {'tile': 128, 'tiles': 64, 'issue_cycles_per_launch': 12.25e9, 'gpu_cycles_per_launch': 13.5e6,
            'issue_model_isa_sha16': cur, 'isa_sha16': cur, 'work_counters_per_launch': work}
    monkeypatch.setattr(bench, 'load_pmc', lambda *a, **k: dict(good))
    w = bench.level_roofline(_Solver(), 128, 7.0)['work']
    assert w['mac_slots_per_launch'] == pytest.approx(macs)
    assert w['mac_slots_vs_algorithmic'] == pytest.approx(macs / (25 * V), abs=1e-4)
    assert w['mac_slots_vs_algorithmic'] == pytest.approx(2.56, abs=0.01)
    assert w['pow_evals_per_voxel'] == pytest.approx(0.25 + 1 / 64.0 + 1 / 256.0, abs=1e-5)
    assert w['pow_evals_vs_reference'] == pytest.approx(w['pow_evals_per_voxel'] / (1 + 1 / 16.0 + 1 / 256.0), abs=1e-4)
    # no work pass, or a work pass of other kernel bytes: no work object
    monkeypatch.setattr(bench, 'load_pmc', lambda *a, **k: {k_: v for k_, v in good.items()
                                                             if k_ != 'work_counters_per_launch'})
    assert 'work' not in bench.level_roofline(_Solver(), 128, 7.0)
    monkeypatch.setattr(bench, 'load_pmc', lambda *a, **k: dict(good, isa_sha16='0123456789abcdef'))
    assert 'work' not in bench.level_roofline(_Solver(), 128, 7.0)

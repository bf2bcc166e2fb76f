"""The C-ABI library builds for gfx950, loads, and exports every symbol include/kad_sched.h declares.

No compute call here (CPU container, no GPU): the -m gpu suite exercises them.
"""
import ctypes
import os

from kubeadmiral_amd import build, runtime


def test_library_exports_every_declared_symbol():
    build.build()
    lib = ctypes.CDLL(runtime.LIB_PATH)
    names = runtime.declared_functions()
    assert len(names) >= 15
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_abi_version():
    lib = runtime.load_library()
    assert lib.kad_abi_version() == 2


def test_library_is_gfx950_code_object():
    with open(runtime.LIB_PATH, "rb") as f:
        data = f.read()
    assert b"gfx950" in data


def test_header_layout_matches_packer():
    """ctypes mirrors of the blob headers have the C sizes/offsets documented in the header."""
    from kubeadmiral_amd import pack
    assert ctypes.sizeof(pack.SnapshotHeader) == 48 + 8 * pack.S_NARRAYS
    assert pack.BatchHeader.n_out_slots.offset == 24
    assert pack.BatchHeader.flags.offset == 48
    assert pack.BatchHeader.total_bytes.offset == 56
    assert pack.BatchHeader.off.offset == 72


def test_batch_split_host_only():
    """kad_batch_split (no device): the contiguous unit ranges a kad_group of n members takes and their first
    output slots — unit_lo[i] = W*i/n, slot_lo[i] = OUT_OFF[unit_lo[i]] — for every n, including n > W."""
    import numpy as np
    import pytest

    from kubeadmiral_amd import pack, synth
    clusters, units = synth.gen_fuzz(5, W=37, C=20)
    fwk = synth.fuzz_framework(1)
    snap = pack.Snapshot(clusters)
    batch = pack.Batch(snap, fwk, units)
    oo = np.asarray(batch.out_off, np.int64)
    for n in (1, 2, 3, 4, 8, 37, 50):
        ulo, slo = runtime.batch_split(batch, n)
        assert ulo[0] == 0 and ulo[-1] == batch.W and (np.diff(ulo) >= 0).all()
        assert ulo.tolist() == [batch.W * i // n for i in range(n + 1)]
        assert (slo == oo[ulo]).all() and slo[-1] == batch.n_out_slots
    with pytest.raises(runtime.KadError):
        runtime.batch_split(batch, 0)
    bad = pack.Batch(snap, fwk, units)
    bad.blob = bad.blob.copy()
    bad.blob[0] ^= 0xFF  # magic
    with pytest.raises(runtime.KadError):
        runtime.batch_split(bad, 2)

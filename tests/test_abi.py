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

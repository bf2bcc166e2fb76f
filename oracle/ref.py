"""ctypes wrapper of oracle/build/libkad_ref.so (TEST INFRASTRUCTURE ONLY).

Loads the C restatement of the reference path (oracle/kad_ref.c) and runs it
on packed blobs. Used by tests/ as the large-size parity checker and by
bench.py's ``cpu_baseline`` leg as the timed CPU baseline ("port").
"""

from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libkad_ref.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        L.kad_ref_schedule.argtypes = [P, P, P, ctypes.c_int, ctypes.c_int, ctypes.c_int, P, P, P, P, P, P, P]
        L.kad_ref_schedule.restype = ctypes.c_int
        L.kad_ref_select_row.argtypes = [ctypes.c_int, P, ctypes.c_int64, ctypes.c_int, ctypes.c_uint32, P]
        L.kad_ref_select_row.restype = ctypes.c_int
        L.kad_ref_trigger_hashes.argtypes = [ctypes.c_int, P, P, P, ctypes.c_int64, P, ctypes.c_int]
        L.kad_ref_trigger_hashes.restype = ctypes.c_int
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def schedule(snap, batch, fwk, begin=0, end=None, n_threads=1, debug=False):
    """Run the C oracle on (snapshot, batch) → kubeadmiral_amd.results.BatchResult (+ debug arrays)."""
    from kubeadmiral_amd.results import BatchResult

    res = BatchResult.empty(batch)
    end = batch.W if end is None else end
    prof = fwk.to_c()
    feas = tot = None
    if debug:
        feas = np.zeros(batch.W * snap.C, np.uint8)
        tot = np.zeros(batch.W * snap.C, np.int64)
    rc = lib().kad_ref_schedule(_p(snap.blob), _p(batch.blob), ctypes.addressof(prof), begin, end, n_threads,
                                _p(res.status), _p(res.count), _p(res.flags), _p(res.cluster), _p(res.replicas),
                                _p(feas), _p(tot))
    if rc != 0:
        raise RuntimeError(f"kad_ref_schedule failed: {rc}")
    if debug:
        return res, feas.reshape(batch.W, snap.C), tot.reshape(batch.W, snap.C)
    return res


def select_row(scores, max_clusters=None, flags=0):
    s = np.ascontiguousarray(scores, dtype=np.int64)
    out = np.zeros(len(s) + 1, np.int32)
    k = lib().kad_ref_select_row(len(s), _p(s), 0 if max_clusters is None else max_clusters,
                                 0 if max_clusters is None else 1, flags, _p(out))
    if k < 0:
        return None
    return out[:k].tolist()


def trigger_hashes(prefixes, suffix: bytes, n_threads=1):
    """FNV-1 32 of prefix_i ‖ suffix per object, each end to end (schedulingtriggers.go:141-145)."""
    off = np.zeros(len(prefixes) + 1, np.int64)
    off[1:] = np.cumsum([len(p) for p in prefixes])
    pre = np.frombuffer(b"".join(prefixes) or b"\0", np.uint8)
    suf = np.frombuffer(suffix or b"\0", np.uint8)
    out = np.zeros(max(1, len(prefixes)), np.uint32)
    rc = lib().kad_ref_trigger_hashes(len(prefixes), _p(off), _p(pre), _p(suf), len(suffix), _p(out), n_threads)
    if rc != 0:
        raise RuntimeError(f"kad_ref_trigger_hashes failed: {rc}")
    return out[:len(prefixes)]

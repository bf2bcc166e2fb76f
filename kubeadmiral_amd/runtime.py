"""ctypes binding of libkad.so and the ScheduleAlgorithm-shaped host API.

``BatchScheduler.schedule(fwk, units, clusters)`` is the batch counterpart of
``core.ScheduleAlgorithm.Schedule(ctx, fwk, su, clusters)``
(pkg/controllers/scheduler/core/generic_scheduler.go:37-44): same inputs (a
framework, scheduling units, the cluster list), same per-unit output
(``ScheduleResult`` or the error class). There is no CPU fallback: if the HIP
library or a GPU is missing this raises.
"""

from __future__ import annotations

import ctypes
import os
import re
from typing import List, Optional, Sequence, Union

import numpy as np

from . import types as T
from .framework import Framework
from .pack import Batch, Snapshot, SnapshotDelta
from .results import BatchResult, to_schedule_result

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libkad.so")
HEADER = os.path.join(os.path.dirname(HERE), "include", "kad_sched.h")

KAD_ERRORS = {-1: "KAD_EINVAL", -2: "KAD_EHIP", -3: "KAD_ENOMEM", -4: "KAD_ESTATE", -5: "KAD_EUNSUPPORTED",
              -6: "KAD_EHOST"}


class KadError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{KAD_ERRORS.get(code, code)}: {msg}")
        self.code = code


class ResultView(ctypes.Structure):
    _fields_ = [("status", ctypes.c_void_p), ("count", ctypes.c_void_p), ("flags", ctypes.c_void_p),
                ("cluster", ctypes.c_void_p), ("replicas", ctypes.c_void_p)]


class ResultState(ctypes.Structure):  # kad_result_state
    _fields_ = [("n_units", ctypes.c_int32), ("place_off", ctypes.c_void_p), ("place_cluster", ctypes.c_void_p),
                ("place_has", ctypes.c_void_p), ("ovr_off", ctypes.c_void_p), ("ovr_cluster", ctypes.c_void_p),
                ("ovr_value", ctypes.c_void_p), ("ovr_kind", ctypes.c_void_p)]


_lib = None


def declared_functions() -> List[str]:
    """Names of the functions include/*.h declare (kad_sched.h, kad_pack.h, kad_objects.h)."""
    import glob

    names = set()
    for h in sorted(glob.glob(os.path.join(os.path.dirname(HEADER), "*.h"))):
        with open(h) as f:
            names |= set(re.findall(r"^\s*(?:int|void|const char\*)\s+(kad_\w+)\s*\(", f.read(), re.M))
    return sorted(names)


def load_library(path: str = LIB_PATH):
    """Load libkad.so (fails loudly: the product path has no CPU fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(f"libkad.so not built at {path}: run `python -m kubeadmiral_amd.build`")
    L = ctypes.CDLL(path)
    P, I, U32, SZ = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint32, ctypes.c_size_t
    L.kad_abi_version.restype = I
    L.kad_ctx_create.argtypes = [I, ctypes.POINTER(P)]
    L.kad_ctx_destroy.argtypes = [P]
    L.kad_last_error.argtypes = [P]
    L.kad_last_error.restype = ctypes.c_char_p
    L.kad_snapshot_upload.argtypes = [P, P, SZ]
    L.kad_snapshot_upload_device.argtypes = [P, P, SZ]
    L.kad_snapshot_update.argtypes = [P, P, SZ]
    L.kad_batch_upload.argtypes = [P, P, SZ]
    L.kad_schedule.argtypes = [P, P]
    L.kad_sync.argtypes = [P]
    L.kad_last_timing.argtypes = [P, P]
    L.kad_set_timing.argtypes = [P, I]
    L.kad_results_download.argtypes = [P, P]
    L.kad_results_copy_device.argtypes = [P, P]
    L.kad_stage_timing.argtypes = [P, P, I]
    L.kad_path_counts.argtypes = [P, P]
    if hasattr(L, "kad_snapshot_paths"):  # (absent from libraries of older revisions: A/B runs)
        L.kad_snapshot_paths.argtypes = [P, P]
    L.kad_result_diff.argtypes = [P, P, P]
    L.kad_schedule_batch.argtypes = [P, P, P, SZ, P]
    L.kad_select_rows.argtypes = [P, I, P, P, P, U32, P, P, P]
    L.kad_plan_rows.argtypes = [P, I, P, P, P, P, P, P, P, P, P, P, P, P]
    L.kad_debug_scores.argtypes = [P, P, P, P]
    L.kad_debug_inject_fault.argtypes = [P, I]
    L.kad_debug_plan_force_workspace.argtypes = [P, I]
    L.kad_trigger_suffix_upload.argtypes = [P, P, SZ]
    L.kad_trigger_prefixes_upload.argtypes = [P, I, P, P]
    L.kad_trigger_run.argtypes = [P]
    L.kad_trigger_timing.argtypes = [P, P]
    L.kad_trigger_download.argtypes = [P, P]
    L.kad_trigger_hashes.argtypes = [P, I, P, P, P, SZ, P]
    L.kad_host_alloc.argtypes = [SZ, ctypes.POINTER(P)]
    L.kad_host_free.argtypes = [P]
    _bind_group(L, P, I, SZ)
    _lib = L
    return L


def _bind_group(L, P, I, SZ):
    """The kad_group_* entry points (ABI 3). A library built from an older revision for a same-box A/B run
    (scripts/build_old.sh) may lack them: its Context still works, GroupContext raises on first use.
    tests/test_abi.py checks that the product library exports every declared symbol."""
    if not hasattr(L, "kad_group_create"):
        return
    L.kad_group_create.argtypes = [P, I, ctypes.POINTER(P)]
    L.kad_group_destroy.argtypes = [P]
    L.kad_group_last_error.argtypes = [P]
    L.kad_group_last_error.restype = ctypes.c_char_p
    L.kad_group_size.argtypes = [P]
    L.kad_group_snapshot_upload.argtypes = [P, P, SZ]
    L.kad_group_snapshot_update.argtypes = [P, P, SZ]
    L.kad_group_batch_upload.argtypes = [P, P, SZ]
    L.kad_group_schedule.argtypes = [P, P]
    L.kad_group_sync.argtypes = [P]
    L.kad_group_results_download.argtypes = [P, P]
    L.kad_group_schedule_batch.argtypes = [P, P, P, SZ, P]
    L.kad_group_ranges.argtypes = [P, P, P]
    L.kad_group_path_counts.argtypes = [P, P]
    L.kad_group_set_timing.argtypes = [P, I]
    L.kad_group_member.argtypes = [P, I, ctypes.POINTER(P)]
    L.kad_batch_split.argtypes = [P, SZ, I, P, P]


class _HostBlock:
    """One kad_host_alloc block; freed when the last array viewing it goes away."""

    def __init__(self, nbytes: int):
        self.L = load_library()
        p = ctypes.c_void_p()
        rc = self.L.kad_host_alloc(nbytes, ctypes.byref(p))
        if rc != 0 or not p.value:
            raise KadError(rc, f"kad_host_alloc({nbytes}) failed")
        self.p = p.value

    def __del__(self):
        if getattr(self, "p", None):
            self.L.kad_host_free(self.p)
            self.p = None


def host_array(n: int, dtype) -> np.ndarray:
    """A page-locked numpy array of n elements (kad_host_alloc): D2H / H2D copies DMA straight into it."""
    dt = np.dtype(dtype)
    nbytes = max(1, n) * dt.itemsize
    blk = _HostBlock(nbytes)
    buf = (ctypes.c_uint8 * nbytes).from_address(blk.p)
    buf._owner = blk  # the array's base chain keeps the block alive
    return np.frombuffer(buf, dtype=dt, count=max(1, n))


def _p(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


class Context:
    """A kad_ctx: one HIP device, one stream, resident snapshot + batch."""

    def __init__(self, device: int = 0):
        self.device = device
        self.L = load_library()
        h = ctypes.c_void_p()
        rc = self.L.kad_ctx_create(device, ctypes.byref(h))
        if rc != 0:
            raise KadError(rc, f"kad_ctx_create(device={device}) failed (no GPU?)")
        self.h = h
        self.snap: Optional[Snapshot] = None
        self.batch: Optional[Batch] = None

    def close(self):
        if self.h:
            self.L.kad_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, rc):
        if rc != 0:
            raise KadError(rc, self.L.kad_last_error(self.h).decode())

    def upload_snapshot(self, snap: Snapshot):
        self._chk(self.L.kad_snapshot_upload(self.h, _p(snap.blob), snap.blob.nbytes))
        self.snap = snap

    def upload_snapshot_blob(self, blob: np.ndarray, snap: Optional[Snapshot] = None):
        """kad_snapshot_upload of a packed snapshot blob (e.g. received from the packing rank)."""
        blob = np.ascontiguousarray(blob, np.uint8)
        self._chk(self.L.kad_snapshot_upload(self.h, _p(blob), blob.nbytes))
        self.snap = snap

    def upload_snapshot_device(self, dev_ptr: int, nbytes: int, snap: Optional[Snapshot] = None):
        self._chk(self.L.kad_snapshot_upload_device(self.h, ctypes.c_void_p(dev_ptr), nbytes))
        self.snap = snap

    def inject_fault(self, where: int):
        """kad_debug_inject_fault (tests): 1 = the next snapshot upload / update fails in its derived-state
        rebuild."""
        self._chk(self.L.kad_debug_inject_fault(self.h, where))

    def plan_force_workspace(self, on):
        """kad_debug_plan_force_workspace (tests): plan_rows through the LDS-workspace planner (True / 1), the
        half-wave pair planner (2), or the default choice by row length (False / 0)."""
        self._chk(self.L.kad_debug_plan_force_workspace(self.h, int(on)))

    def update_snapshot(self, delta: SnapshotDelta):
        """kad_snapshot_update: patch the resident snapshot; the resident batch stays valid."""
        self._chk(self.L.kad_snapshot_update(self.h, _p(delta.blob), delta.blob.nbytes))

    def upload_batch(self, batch: Batch):
        chk = getattr(batch, "check_current", None)
        if chk is not None:
            chk()
        self._chk(self.L.kad_batch_upload(self.h, _p(batch.blob), batch.blob.nbytes))
        self.batch = batch

    def schedule(self, fwk: Framework):
        prof = fwk.to_c()
        self._chk(self.L.kad_schedule(self.h, ctypes.byref(prof)))

    def sync(self):
        self._chk(self.L.kad_sync(self.h))

    def set_timing(self, on: bool):
        """kad_set_timing: HIP event records around the stages of later schedule() calls."""
        self._chk(self.L.kad_set_timing(self.h, 1 if on else 0))

    def timing(self):
        ms = (ctypes.c_float * 3)()
        self._chk(self.L.kad_last_timing(self.h, ms))
        return float(ms[0]), float(ms[1]), float(ms[2])

    STAGES = ("req_mask", "prep", "main", "defer", "planner", "total", "rows")

    def stage_timing(self) -> dict:
        """kad_stage_timing: device ms per stage of the last timed schedule() (rows = schedule_row_kernel,
        defer = schedule_kernel over the defer list)."""
        ms = (ctypes.c_float * 7)()
        self._chk(self.L.kad_stage_timing(self.h, ms, 7))
        return {k: float(v) for k, v in zip(self.STAGES, ms)}

    DIFF_PLACEMENT, DIFF_OVERRIDES, DIFF_SKIP, DIFF_STICKY = 1, 2, 4, 8

    def result_diff(self, state: dict) -> np.ndarray:
        """kad_result_diff: per unit of the last schedule(), which parts of applySchedulingResult would change
        its object (KAD_DIFF_* flags). ``state``: objects.result_states(...) arrays."""
        W = len(state["place_has"])
        keep = {k: np.ascontiguousarray(v) for k, v in state.items() if isinstance(v, np.ndarray)}
        st = ResultState(W, *(_p(keep[k]) for k in ("place_off", "place_cluster", "place_has", "ovr_off", "ovr_cluster",
                                                    "ovr_value", "ovr_kind")))
        out = np.zeros(max(1, W), np.uint32)
        self._chk(self.L.kad_result_diff(self.h, ctypes.byref(st), _p(out)))
        return out[:W]

    def path_counts(self) -> dict:
        """kad_path_counts: units per kernel path of the last schedule()."""
        out = (ctypes.c_int32 * 4)()
        self._chk(self.L.kad_path_counts(self.h, out))
        return {"units": out[0], "full_kernel": out[1], "row_kernel": out[2], "planner_rows": out[3]}

    def snapshot_paths(self) -> dict:
        """kad_snapshot_paths: the resident snapshot's resource class and the kernel path it takes."""
        out = (ctypes.c_int32 * 5)()
        self._chk(self.L.kad_snapshot_paths(self.h, out))
        return {"resource_class": {2: "strict", 1: "relaxed", 0: "generic"}[out[0]], "exact_f64": bool(out[1]),
                "wide": bool(out[2]), "fold": bool(out[3]), "fitfold": bool(out[4])}

    def copy_results_device(self, status_ptr: int, count_ptr: int, flags_ptr: int, cluster_ptr: int,
                            replicas_ptr: int):
        """kad_results_copy_device: results D2D into caller device buffers (e.g. torch tensors)."""
        v = ResultView(status_ptr, count_ptr, flags_ptr, cluster_ptr, replicas_ptr)
        self._chk(self.L.kad_results_copy_device(self.h, ctypes.byref(v)))

    def download(self, out: Optional[BatchResult] = None) -> BatchResult:
        """kad_results_download into fresh arrays, or into ``out`` (e.g. page-locked arrays reused across
        batches: BatchResult.pinned), which must be sized for the uploaded batch."""
        if out is None:
            res = BatchResult.empty(self.batch)
        else:  # views of the batch's sizes
            W, n = self.batch.W, max(1, self.batch.n_out_slots)
            arrs = ((out.status, W), (out.count, W), (out.flags, W), (out.cluster, n), (out.replicas, n))
            for (a, m), dt in zip(arrs, (np.int32, np.int32, np.uint32, np.int32, np.int64)):
                if a.dtype != dt:  # kad_results_download copies 4 or 8 bytes per element
                    raise ValueError(f"download buffer dtype {a.dtype}, kad_results_download writes {np.dtype(dt)}")
                if len(a) < m or not a.flags.c_contiguous:
                    raise ValueError("download buffers smaller than the uploaded batch")
            res = BatchResult(*(a[:m] for a, m in arrs), self.batch.out_off)
        v = ResultView(res.status.ctypes.data, res.count.ctypes.data, res.flags.ctypes.data, res.cluster.ctypes.data,
                       res.replicas.ctypes.data)
        self._chk(self.L.kad_results_download(self.h, ctypes.byref(v)))
        return res

    def schedule_batch(self, fwk: Framework, batch: Batch) -> BatchResult:
        """kad_schedule_batch: upload, schedule and download under one hold of the context lock."""
        chk = getattr(batch, "check_current", None)
        if chk is not None:
            chk()
        res = BatchResult.empty(batch)
        v = ResultView(res.status.ctypes.data, res.count.ctypes.data, res.flags.ctypes.data, res.cluster.ctypes.data,
                       res.replicas.ctypes.data)
        prof = fwk.to_c()
        self._chk(self.L.kad_schedule_batch(self.h, ctypes.byref(prof), _p(batch.blob), batch.blob.nbytes,
                                            ctypes.byref(v)))
        self.batch = batch
        return res

    def run(self, fwk: Framework, batch: Batch) -> BatchResult:
        self.upload_batch(batch)
        self.schedule(fwk)
        return self.download()

    def debug_scores(self, fwk: Framework):
        W, C = self.batch.W, self.snap.C
        feas = np.zeros(max(1, W * C), np.uint8)
        tot = np.zeros(max(1, W * C), np.int64)
        prof = fwk.to_c()
        self._chk(self.L.kad_debug_scores(self.h, ctypes.byref(prof), _p(feas), _p(tot)))
        return feas[:W * C].reshape(W, C), tot[:W * C].reshape(W, C)

    def select_rows(self, rows: Sequence[Sequence[int]], max_clusters: Sequence[Optional[int]], flags: int = 0):
        """MaxCluster on explicit score rows → per row (status, sorted selected positions)."""
        off = np.zeros(len(rows) + 1, np.int32)
        off[1:] = np.cumsum([len(r) for r in rows])
        scores = np.array([x for r in rows for x in r] or [0], np.int64)
        mc = np.array([(np.iinfo(np.int64).max if m is None else m) for m in max_clusters], np.int64)
        cnt = np.zeros(len(rows), np.int32)
        st = np.zeros(len(rows), np.int32)
        sel = np.zeros(max(1, int(off[-1])), np.int32)
        self._chk(self.L.kad_select_rows(self.h, len(rows), _p(off), _p(scores), _p(mc), flags, _p(cnt), _p(sel),
                                         _p(st)))
        return [(int(st[r]), sel[off[r]:off[r] + cnt[r]].tolist()) for r in range(len(rows))]

    def plan_rows(self, rows):
        """planner.Plan on explicit rows.

        rows: list of dicts with ``elems`` (list of dicts hash, weight, min, max(None), cap(None), current),
        ``total``, ``avoid``, ``keep``. Returns per row (plan list, overflow list with None for absent).
        """
        n = len(rows)
        off = np.zeros(n + 1, np.int32)
        off[1:] = np.cumsum([len(r["elems"]) for r in rows])
        tot = max(1, int(off[-1]))
        hsh = np.zeros(tot, np.uint32)
        wt, mn, mx, cp, cur = (np.zeros(tot, np.int64) for _ in range(5))
        ef = np.zeros(tot, np.uint32)
        i = 0
        for r in rows:
            for e in r["elems"]:
                hsh[i], wt[i], mn[i], cur[i] = e["hash"], e["weight"], e["min"], e["current"]
                if e.get("max") is not None:
                    mx[i] = e["max"]
                    ef[i] |= 2
                if e.get("cap") is not None:
                    cp[i] = e["cap"]
                    ef[i] |= 4
                i += 1
        total = np.array([r["total"] for r in rows] or [0], np.int64)
        rf = np.array([(1 if r["avoid"] else 0) | (2 if r["keep"] else 0) for r in rows] or [0], np.uint32)
        plan = np.zeros(tot, np.int64)
        over = np.zeros(tot, np.int64)
        self._chk(self.L.kad_plan_rows(self.h, n, _p(off), _p(hsh), _p(wt), _p(mn), _p(mx), _p(cp), _p(cur), _p(ef),
                                       _p(total), _p(rf), _p(plan), _p(over)))
        out = []
        for r in range(n):
            a, b = off[r], off[r + 1]
            out.append((plan[a:b].tolist(), [None if o < 0 else int(o) for o in over[a:b].tolist()]))
        return out


    # ------------------------------------------------ scheduling-trigger hashes
    def trigger_suffix_upload(self, suffix: bytes):
        buf = np.frombuffer(suffix, np.uint8) if suffix else np.zeros(1, np.uint8)
        self._chk(self.L.kad_trigger_suffix_upload(self.h, _p(buf), len(suffix)))

    def trigger_prefixes_upload(self, prefixes: Sequence[bytes]):
        off = np.zeros(len(prefixes) + 1, np.int64)
        off[1:] = np.cumsum([len(p) for p in prefixes])
        data = np.frombuffer(b"".join(prefixes) or b"\0", np.uint8)
        self._chk(self.L.kad_trigger_prefixes_upload(self.h, len(prefixes), _p(off), _p(data)))
        self._trig_n = len(prefixes)

    def trigger_run(self):
        self._chk(self.L.kad_trigger_run(self.h))

    def trigger_timing(self):
        ms = (ctypes.c_float * 2)()
        self._chk(self.L.kad_trigger_timing(self.h, ms))
        return float(ms[0]), float(ms[1])

    def trigger_download(self) -> np.ndarray:
        out = np.zeros(max(1, self._trig_n), np.uint32)
        self._chk(self.L.kad_trigger_download(self.h, _p(out)))
        return out[:self._trig_n]


def batch_split(batch, n: int):
    """kad_batch_split (host only): the contiguous unit ranges a kad_group of n members gives its members,
    and their first output slots: (unit_lo[n+1], slot_lo[n+1])."""
    L = load_library()
    ulo = np.zeros(n + 1, np.int64)
    slo = np.zeros(n + 1, np.int64)
    rc = L.kad_batch_split(_p(batch.blob), batch.blob.nbytes, n, _p(ulo), _p(slo))
    if rc != 0:
        raise KadError(rc, "kad_batch_split: malformed batch blob or n < 1")
    return ulo, slo


class _MemberContext(Context):
    """A kad_group member's kad_ctx, owned by the group (GroupContext.member)."""

    def close(self):
        self.h = None


class GroupContext:
    """A kad_group: one process scheduling each batch over several GPUs (contiguous unit ranges, one
    kad_ctx per device), results in one view as from a single Context. Same interface as :class:`Context`
    for what :class:`BatchScheduler` uses (upload_snapshot, update_snapshot, upload_batch, schedule, sync,
    download, run, path_counts), so a BatchScheduler / CoalescingScheduler drives N GPUs unchanged."""

    def __init__(self, devices: Sequence[int]):
        self.devices = list(devices)
        self.L = load_library()
        h = ctypes.c_void_p()
        arr = (ctypes.c_int * len(self.devices))(*self.devices)
        rc = self.L.kad_group_create(arr, len(self.devices), ctypes.byref(h))
        if rc != 0:
            raise KadError(rc, f"kad_group_create(devices={self.devices}) failed (no GPU?)")
        self.h = h
        self.snap: Optional[Snapshot] = None
        self.batch: Optional[Batch] = None

    @property
    def device(self):
        return self.devices[0]

    def close(self):
        if self.h:
            self.L.kad_group_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, rc):
        if rc != 0:
            raise KadError(rc, self.L.kad_group_last_error(self.h).decode())

    def upload_snapshot(self, snap: Snapshot):
        self._chk(self.L.kad_group_snapshot_upload(self.h, _p(snap.blob), snap.blob.nbytes))
        self.snap = snap

    def member(self, i: int) -> "Context":
        """kad_group_member: member i's kad_ctx (its shard of the resident batch) as a Context that the group
        owns (closing it does nothing). Its per-ctx calls — copy_results_device, result_diff, path_counts,
        stage_timing — cover the member's units."""
        c = ctypes.c_void_p()
        self._chk(self.L.kad_group_member(self.h, i, ctypes.byref(c)))
        m = _MemberContext.__new__(_MemberContext)
        m.device, m.L, m.h, m.snap, m.batch = self.devices[i], self.L, c, self.snap, None
        return m

    def update_snapshot(self, delta: SnapshotDelta):
        self._chk(self.L.kad_group_snapshot_update(self.h, _p(delta.blob), delta.blob.nbytes))

    def upload_batch(self, batch: Batch):
        chk = getattr(batch, "check_current", None)
        if chk is not None:
            chk()
        self._chk(self.L.kad_group_batch_upload(self.h, _p(batch.blob), batch.blob.nbytes))
        self.batch = batch

    def schedule(self, fwk: Framework):
        prof = fwk.to_c()
        self._chk(self.L.kad_group_schedule(self.h, ctypes.byref(prof)))

    def sync(self):
        self._chk(self.L.kad_group_sync(self.h))

    def set_timing(self, on: bool):
        self._chk(self.L.kad_group_set_timing(self.h, 1 if on else 0))

    def ranges(self):
        n = len(self.devices)
        ulo = np.zeros(n + 1, np.int64)
        slo = np.zeros(n + 1, np.int64)
        self._chk(self.L.kad_group_ranges(self.h, _p(ulo), _p(slo)))
        return ulo, slo

    def path_counts(self) -> dict:
        out = (ctypes.c_int32 * 4)()
        self._chk(self.L.kad_group_path_counts(self.h, out))
        return {"units": out[0], "full_kernel": out[1], "row_kernel": out[2], "planner_rows": out[3]}

    def member_stage_timing(self, i: int) -> dict:
        """kad_stage_timing of member i (timing on)."""
        c = ctypes.c_void_p()
        self._chk(self.L.kad_group_member(self.h, i, ctypes.byref(c)))
        ms = (ctypes.c_float * 7)()
        rc = self.L.kad_stage_timing(c, ms, 7)
        if rc != 0:
            raise KadError(rc, self.L.kad_last_error(c).decode())
        return {k: float(v) for k, v in zip(Context.STAGES, ms)}

    def download(self, out: Optional[BatchResult] = None) -> BatchResult:
        res = BatchResult.empty(self.batch) if out is None else out
        v = ResultView(res.status.ctypes.data, res.count.ctypes.data, res.flags.ctypes.data, res.cluster.ctypes.data,
                       res.replicas.ctypes.data)
        self._chk(self.L.kad_group_results_download(self.h, ctypes.byref(v)))
        return res

    def schedule_batch(self, fwk: Framework, batch: Batch) -> BatchResult:
        res = BatchResult.empty(batch)
        v = ResultView(res.status.ctypes.data, res.count.ctypes.data, res.flags.ctypes.data, res.cluster.ctypes.data,
                       res.replicas.ctypes.data)
        prof = fwk.to_c()
        self._chk(self.L.kad_group_schedule_batch(self.h, ctypes.byref(prof), _p(batch.blob), batch.blob.nbytes,
                                                  ctypes.byref(v)))
        self.batch = batch
        return res

    def run(self, fwk: Framework, batch: Batch) -> BatchResult:
        self.upload_batch(batch)
        self.schedule(fwk)
        return self.download()


class TriggerHasher:
    """Scheduler.computeSchedulingTriggerHash for a batch of objects (schedulingtriggers.go:106-147).

    The cluster part of the trigger JSON is built once per cluster list
    (:meth:`set_clusters`), each object's part on the host, and the FNV-1 over
    object part ‖ cluster part runs on the GPU (``kad_trigger_*``). Returns the
    decimal strings the reference writes to the
    ``kubeadmiral.io/scheduling-trigger-hash`` annotation.
    """

    def __init__(self, ctx: Optional[Context] = None, device: int = 0):
        self.ctx = ctx if ctx is not None else Context(device)
        self.suffix: Optional[bytes] = None

    def set_clusters(self, clusters: List[T.FederatedCluster]) -> bytes:
        from .objects import trigger_suffix

        self.suffix = trigger_suffix(clusters)
        self.ctx.trigger_suffix_upload(self.suffix)
        return self.suffix

    def hashes(self, type_config, objs: Sequence[dict], policies: Sequence) -> List[str]:
        from .objects import format_trigger_hash, trigger_prefix

        if self.suffix is None:
            raise RuntimeError("set_clusters first")
        self.ctx.trigger_prefixes_upload([trigger_prefix(type_config, o, p) for o, p in zip(objs, policies)])
        self.ctx.trigger_run()
        h = self.ctx.trigger_download()
        return [format_trigger_hash(x) for x in h.tolist()]


class BatchScheduler:
    """Batch ScheduleAlgorithm on the GPU (generic_scheduler.go:37-44 semantics per unit).

    The resident snapshot follows the cluster list of every call: each call
    diffs the list against it by content (``types.cluster_key``), so a new
    list, replaced elements or elements edited in place are all picked up —
    the library keeps no caller pointers. Host columns are committed only
    after the device accepted the delta; a failed device update forces a full
    re-upload on the next call.
    """

    def __init__(self, ctx: Optional[Context] = None, device: int = 0, devices: Optional[Sequence[int]] = None):
        """``devices``: schedule every batch over these GPUs (a :class:`GroupContext`, one process), else one
        Context on ``device``."""
        if ctx is None:
            ctx = GroupContext(devices) if devices is not None else Context(device)
        self.ctx = ctx
        self.full_uploads = 0   # snapshot (re)packs + uploads
        self.delta_updates = 0  # in-place kad_snapshot_update calls

    def set_clusters(self, clusters: List[T.FederatedCluster]) -> Snapshot:
        """Make ``clusters`` the resident snapshot: an in-place delta when only existing clusters changed
        within the interned vocabulary (cluster status / label / taint events, scheduler.go:157-177), else a
        repack and full upload (join, leave, new label value / taint / API resource)."""
        snap = self.ctx.snap
        if snap is not None:
            delta = snap.diff(clusters)
            if delta is not None:
                if delta.changed:
                    try:
                        self.ctx.update_snapshot(delta)
                    except BaseException:
                        self.ctx.snap = None  # device state unknown: the next call re-uploads in full
                        raise
                    self.delta_updates += 1
                snap.commit(delta)
                return snap
        snap = Snapshot(clusters)
        self.ctx.upload_snapshot(snap)
        self.full_uploads += 1
        return snap

    def schedule(self, fwk: Framework, units: List[T.SchedulingUnit], clusters: List[T.FederatedCluster]
                 ) -> List[Union[T.ScheduleResult, T.ScheduleError]]:
        snap = self.set_clusters(clusters)
        batch = Batch(snap, fwk, units)
        res = self.ctx.run(fwk, batch)
        return [to_schedule_result(res, w, su, snap.names) for w, su in enumerate(units)]

    def schedule_columns(self, fwk: Framework, cols, clusters: List[T.FederatedCluster]):
        """The same for units already in columns (``columns.SUColumns``, e.g. from ``columns.units_from_objects``):
        the native packer, one GPU batch. Returns (BatchResult, snapshot)."""
        from .columns import NativePacker

        snap = self.set_clusters(clusters)
        pk = getattr(self, "_packer", None)
        if pk is None or pk.snap is not snap or getattr(self, "_packer_fp", None) != snap.fingerprint:
            pk = self._packer = NativePacker(snap)  # the packer interns against the snapshot's vocabulary
            self._packer_fp = snap.fingerprint
        batch = pk.pack(fwk, cols)
        return self.ctx.run(fwk, batch), snap

"""Columnar SchedulingUnits and the native packer (include/kad_pack.h).

``SUColumns`` is the batch a cgo shim hands to ``kad_pack_batch``: every field
of ``framework.SchedulingUnit`` (``pkg/controllers/scheduler/framework/
types.go:33-69``) as flat arrays, maps and lists as CSR ranges, strings as ids
into one string table. ``NativePacker(snap).pack(fwk, cols)`` runs the C++
packer in libkad.so and returns a :class:`NativeBatch`, which the runtime
uploads like a ``pack.Batch`` — its blob is byte-identical to the Python
packer's for the same units (``tests/test_native_pack.py``).

``from_units`` converts ``types.SchedulingUnit`` objects (the Python mirror of
the reference's type) into columns; ``to_units`` converts back (tests use it to
run the object-level oracle on natively packed batches). ``gen_units_c2_columns``
(in ``synth``) generates the C2/C3 workload directly as columns.
"""

from __future__ import annotations

import ctypes
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import types as T
from .framework import Framework

# include/kad_pack.h KAD_SU_*
SU_DUPLICATE = 1 << 0
SU_STICKY = 1 << 1
SU_AVOID_DISRUPTION = 1 << 2
SU_HAS_DESIRED = 1 << 3
SU_HAS_MAX_CLUSTERS = 1 << 4
SU_HAS_AUTO_MIGRATION = 1 << 5
SU_KEEP_UNSCHED = 1 << 6
SU_HAS_CLUSTER_AFFINITY = 1 << 7
SU_HAS_REQUIRED = 1 << 8

I32, I64, U8, U32 = np.int32, np.int64, np.uint8, np.uint32

# kad_su_columns fields after (n_units, str) in declaration order; n_reqs sits before rq_key
FIELDS = [("group", I32), ("version", I32), ("kind", I32), ("namespace_", I32), ("name", I32), ("flags", U32),
          ("desired", I64), ("max_clusters", I64), ("req_cpu", I64), ("req_mem", I64), ("req_eph", I64),
          ("scalar_off", I32), ("scalar_name", I32), ("scalar_val", I64),
          ("tol_off", I32), ("tol_key", I32), ("tol_op", I32), ("tol_value", I32), ("tol_effect", I32),
          ("sel_off", I32), ("sel_key", I32), ("sel_value", I32),
          ("rq_key", I32), ("rq_op", I32), ("rq_val_off", I32), ("rq_val", I32),
          ("rterm_off", I32), ("rt_req", I32), ("rt_n_expr", I32), ("rt_n_field", I32),
          ("pterm_off", I32), ("pt_weight", I32), ("pt_req", I32), ("pt_n_expr", I32),
          ("place_off", I32), ("place_name", I32),
          ("cur_off", I32), ("cur_name", I32), ("cur_rep", I64), ("cur_has_rep", U8),
          ("wt_off", I32), ("wt_name", I32), ("wt_val", I64),
          ("min_off", I32), ("min_name", I32), ("min_val", I64),
          ("max_off", I32), ("max_name", I32), ("max_val", I64),
          ("cap_off", I32), ("cap_name", I32), ("cap_val", I64)]
DTYPES = dict(FIELDS)
CSR_GROUPS = ["scalar", "tol", "sel", "rterm", "pterm", "place", "cur", "wt", "min", "max", "cap"]


class StringTable:
    """Strings by id: ``bytes[off[i]:off[i+1]]``. ``id()`` interns (dedup)."""

    def __init__(self):
        self._ids: Dict[str, int] = {}
        self._parts: List[bytes] = []

    def id(self, s: str) -> int:
        i = self._ids.get(s)
        if i is None:
            i = self._ids[s] = len(self._parts)
            self._parts.append(s.encode())
        return i

    def arrays(self):
        off = np.zeros(len(self._parts) + 1, I64)
        if self._parts:
            off[1:] = np.cumsum([len(p) for p in self._parts])
        data = np.frombuffer(b"".join(self._parts) or b"\0", U8).copy()
        return off, data


class SUColumns:
    """A batch of SchedulingUnits as columns (kad_su_columns); arrays are contiguous numpy."""

    def __init__(self, n_units: int, str_off: np.ndarray, str_data: np.ndarray, cols: Dict[str, np.ndarray]):
        self.n_units = n_units
        self.str_off = np.ascontiguousarray(str_off, I64)
        self.str_data = np.ascontiguousarray(str_data, U8)
        self.cols = {k: np.ascontiguousarray(cols[k], dt) for k, dt in FIELDS}

    def __getitem__(self, k) -> np.ndarray:
        return self.cols[k]

    @property
    def n_reqs(self) -> int:
        return len(self.cols["rq_key"])

    def slice(self, lo: int, hi: int) -> "SUColumns":
        """Units [lo, hi) as their own columns (CSR offsets rebased; the requirement table cut to the range its
        terms reference; the string table shared) — e.g. the chunks of a pipelined pack."""
        c = self.cols
        out = {}
        for k in ("group", "version", "kind", "namespace_", "name", "flags", "desired", "max_clusters", "req_cpu",
                  "req_mem", "req_eph"):
            out[k] = c[k][lo:hi]

        def cut(grp, fields):
            off = c[grp + "_off"]
            a, b = int(off[lo]), int(off[hi])
            out[grp + "_off"] = (off[lo:hi + 1] - a).astype(I32)
            for f in fields:
                out[f] = c[f][a:b]

        cut("scalar", ("scalar_name", "scalar_val"))
        cut("tol", ("tol_key", "tol_op", "tol_value", "tol_effect"))
        cut("sel", ("sel_key", "sel_value"))
        cut("rterm", ("rt_req", "rt_n_expr", "rt_n_field"))
        cut("pterm", ("pt_weight", "pt_req", "pt_n_expr"))
        cut("place", ("place_name",))
        cut("cur", ("cur_name", "cur_rep", "cur_has_rep"))
        cut("wt", ("wt_name", "wt_val"))
        cut("min", ("min_name", "min_val"))
        cut("max", ("max_name", "max_val"))
        cut("cap", ("cap_name", "cap_val"))
        # requirement entries the range's terms reference: [r0, r1)
        starts = np.concatenate([out["rt_req"], out["pt_req"]]).astype(np.int64)
        ends = np.concatenate([out["rt_req"] + out["rt_n_expr"] + out["rt_n_field"],
                               out["pt_req"] + out["pt_n_expr"]]).astype(np.int64)
        r0, r1 = (int(starts.min()), int(ends.max())) if len(starts) else (0, 0)
        out["rt_req"] = (out["rt_req"] - r0).astype(I32)
        out["pt_req"] = (out["pt_req"] - r0).astype(I32)
        vo = c["rq_val_off"]
        out["rq_key"], out["rq_op"] = c["rq_key"][r0:r1], c["rq_op"][r0:r1]
        out["rq_val_off"] = (vo[r0:r1 + 1] - vo[r0]).astype(I32)
        out["rq_val"] = c["rq_val"][int(vo[r0]):int(vo[r1])]
        return SUColumns(hi - lo, self.str_off, self.str_data, out)

    def strings(self) -> List[str]:
        b = self.str_data.tobytes()
        o = self.str_off
        return [b[o[i]:o[i + 1]].decode() for i in range(len(o) - 1)]


def _csr_off(lengths) -> np.ndarray:
    off = np.zeros(len(lengths) + 1, I32)
    if len(lengths):
        off[1:] = np.cumsum(lengths)
    return off


# ------------------------------------------------------------------ objects → columns
def from_units(units: Sequence[T.SchedulingUnit], st: Optional[StringTable] = None) -> SUColumns:
    """SchedulingUnit objects → columns (what a Go shim fills from []SchedulingUnit)."""
    st = st or StringTable()
    c: Dict[str, list] = {k: [] for k, _ in FIELDS}
    lens: Dict[str, list] = {k: [] for k in CSR_GROUPS}
    rq_val_off = [0]
    sid = st.id

    def add_req(r: T.ClusterSelectorRequirement) -> None:
        c["rq_key"].append(sid(r.key))
        c["rq_op"].append(sid(r.operator))
        for v in r.values or []:
            c["rq_val"].append(sid(v))
        rq_val_off.append(len(c["rq_val"]))

    for su in units:
        f = 0
        if su.scheduling_mode == T.SCHEDULING_MODE_DUPLICATE:
            f |= SU_DUPLICATE
        if su.sticky_cluster:
            f |= SU_STICKY
        if su.avoid_disruption:
            f |= SU_AVOID_DISRUPTION
        if su.desired_replicas is not None:
            f |= SU_HAS_DESIRED
        c["desired"].append(su.desired_replicas if su.desired_replicas is not None else 0)
        mc = 0
        if su.max_clusters is not None:
            f |= SU_HAS_MAX_CLUSTERS
            mc = max(min(su.max_clusters, (1 << 63) - 1), -(1 << 63))
        c["max_clusters"].append(mc)
        am = su.auto_migration
        if am is not None:
            f |= SU_HAS_AUTO_MIGRATION
            if am.keep_unschedulable_replicas:
                f |= SU_KEEP_UNSCHED
        ca = su.affinity.cluster_affinity if su.affinity is not None else None
        if ca is not None:
            f |= SU_HAS_CLUSTER_AFFINITY
            if ca.required is not None:
                f |= SU_HAS_REQUIRED
        c["flags"].append(f)
        for k, v in (("group", su.group), ("version", su.version), ("kind", su.kind),
                     ("namespace_", su.namespace), ("name", su.name)):
            c[k].append(sid(v))
        rr = su.resource_request
        c["req_cpu"].append(rr.milli_cpu)
        c["req_mem"].append(rr.memory)
        c["req_eph"].append(rr.ephemeral_storage)
        sc = rr.scalar_resources or {}
        lens["scalar"].append(len(sc))
        for n, v in sc.items():
            c["scalar_name"].append(sid(n))
            c["scalar_val"].append(v)
        tols = su.tolerations or []
        lens["tol"].append(len(tols))
        for t in tols:
            c["tol_key"].append(sid(t.key))
            c["tol_op"].append(sid(t.operator))
            c["tol_value"].append(sid(t.value))
            c["tol_effect"].append(sid(t.effect))
        sel = su.cluster_selector or {}
        lens["sel"].append(len(sel))
        for k, v in sel.items():
            c["sel_key"].append(sid(k))
            c["sel_value"].append(sid(v))
        terms = (ca.required.cluster_selector_terms or []) if (ca is not None and ca.required is not None) else []
        lens["rterm"].append(len(terms))
        for t in terms:
            c["rt_req"].append(len(c["rq_key"]))
            exprs, fields = t.match_expressions or [], t.match_fields or []
            c["rt_n_expr"].append(len(exprs))
            c["rt_n_field"].append(len(fields))
            for r in exprs:
                add_req(r)
            for r in fields:
                add_req(r)
        prefs = (ca.preferred or []) if ca is not None else []
        lens["pterm"].append(len(prefs))
        for p in prefs:
            exprs = p.preference.match_expressions or []
            c["pt_weight"].append(p.weight)
            c["pt_req"].append(len(c["rq_key"]))
            c["pt_n_expr"].append(len(exprs))
            for r in exprs:
                add_req(r)
        names = su.cluster_names or set()
        lens["place"].append(len(names))
        for n in sorted(names):
            c["place_name"].append(sid(n))
        cur = su.current_clusters or {}
        lens["cur"].append(len(cur))
        for n, r in cur.items():
            c["cur_name"].append(sid(n))
            c["cur_rep"].append(r if r is not None else 0)
            c["cur_has_rep"].append(0 if r is None else 1)
        for key, m in (("wt", su.weights), ("min", su.min_replicas), ("max", su.max_replicas),
                       ("cap", am.estimated_capacity if am is not None else None)):
            m = m or {}
            lens[key].append(len(m))
            for n, v in m.items():
                c[key + "_name"].append(sid(n))
                c[key + "_val"].append(v)

    cols = {k: (np.asarray(c[k], dtype=dt) if c[k] else np.zeros(0, dt)) for k, dt in FIELDS}
    for k in CSR_GROUPS:
        cols[k + "_off"] = _csr_off(lens[k])
    cols["rq_val_off"] = np.asarray(rq_val_off, I32)
    off, data = st.arrays()
    return SUColumns(len(units), off, data, cols)


# ------------------------------------------------------------------ columns → objects
def to_units(cols: SUColumns) -> List[T.SchedulingUnit]:
    """Columns → SchedulingUnit objects (for the object-level oracle in tests)."""
    S = cols.strings()
    C = cols.cols
    out = []

    def rng(k, w):
        o = C[k + "_off"]
        return range(int(o[w]), int(o[w + 1]))

    def req(i):
        a, b = int(C["rq_val_off"][i]), int(C["rq_val_off"][i + 1])
        return T.ClusterSelectorRequirement(S[C["rq_key"][i]], S[C["rq_op"][i]], [S[v] for v in C["rq_val"][a:b]])

    for w in range(cols.n_units):
        f = int(C["flags"][w])
        ca = None
        if f & SU_HAS_CLUSTER_AFFINITY:
            required = None
            if f & SU_HAS_REQUIRED:
                terms = []
                for t in rng("rterm", w):
                    r0, ne, nf = int(C["rt_req"][t]), int(C["rt_n_expr"][t]), int(C["rt_n_field"][t])
                    terms.append(T.ClusterSelectorTerm([req(i) for i in range(r0, r0 + ne)] or None,
                                                       [req(i) for i in range(r0 + ne, r0 + ne + nf)] or None))
                required = T.ClusterSelector(terms)
            prefs = [T.PreferredSchedulingTerm(int(C["pt_weight"][t]), T.ClusterSelectorTerm(
                [req(i) for i in range(int(C["pt_req"][t]), int(C["pt_req"][t]) + int(C["pt_n_expr"][t]))] or None))
                for t in rng("pterm", w)]
            ca = T.ClusterAffinity(required, prefs or None)
        am = None
        if f & SU_HAS_AUTO_MIGRATION:
            cap = {S[C["cap_name"][i]]: int(C["cap_val"][i]) for i in rng("cap", w)}
            am = T.AutoMigrationSpec(cap or None, bool(f & SU_KEEP_UNSCHED))
        out.append(T.SchedulingUnit(
            group=S[C["group"][w]], version=S[C["version"][w]], kind=S[C["kind"][w]],
            namespace=S[C["namespace_"][w]], name=S[C["name"][w]],
            desired_replicas=int(C["desired"][w]) if f & SU_HAS_DESIRED else None,
            resource_request=T.Resource(int(C["req_cpu"][w]), int(C["req_mem"][w]), int(C["req_eph"][w]),
                                        {S[C["scalar_name"][i]]: int(C["scalar_val"][i]) for i in rng("scalar", w)}
                                        or None),
            current_clusters={S[C["cur_name"][i]]: (int(C["cur_rep"][i]) if C["cur_has_rep"][i] else None)
                              for i in rng("cur", w)} or None,
            auto_migration=am,
            scheduling_mode=T.SCHEDULING_MODE_DUPLICATE if f & SU_DUPLICATE else T.SCHEDULING_MODE_DIVIDE,
            sticky_cluster=bool(f & SU_STICKY), avoid_disruption=bool(f & SU_AVOID_DISRUPTION),
            cluster_selector={S[C["sel_key"][i]]: S[C["sel_value"][i]] for i in rng("sel", w)} or None,
            cluster_names={S[C["place_name"][i]] for i in rng("place", w)} or None,
            affinity=T.Affinity(ca) if ca is not None else None,
            tolerations=[T.Toleration(S[C["tol_key"][i]], S[C["tol_op"][i]], S[C["tol_value"][i]],
                                      S[C["tol_effect"][i]]) for i in rng("tol", w)] or None,
            max_clusters=int(C["max_clusters"][w]) if f & SU_HAS_MAX_CLUSTERS else None,
            min_replicas={S[C["min_name"][i]]: int(C["min_val"][i]) for i in rng("min", w)} or None,
            max_replicas={S[C["max_name"][i]]: int(C["max_val"][i]) for i in rng("max", w)} or None,
            weights={S[C["wt_name"][i]]: int(C["wt_val"][i]) for i in rng("wt", w)} or None))
    return out


# ------------------------------------------------------------------ ctypes mirror of kad_pack.h
class KadStrs(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int32), ("off", ctypes.c_void_p), ("bytes", ctypes.c_void_p)]


class KadPackVocab(ctypes.Structure):
    _fields_ = [("cluster_names", KadStrs), ("scalar_names", KadStrs), ("gvk_group", KadStrs),
                ("gvk_version", KadStrs), ("gvk_kind", KadStrs), ("label_keys", KadStrs),
                ("label_val_off", ctypes.c_void_p), ("label_vals", KadStrs), ("taint_key", KadStrs),
                ("taint_value", KadStrs), ("taint_effect", KadStrs), ("n_taint_words", ctypes.c_int32),
                ("fingerprint", ctypes.c_uint64)]


def _su_fields():
    f = [("n_units", ctypes.c_int32), ("str", KadStrs)]
    for k, _ in FIELDS:
        if k == "rq_key":
            f.append(("n_reqs", ctypes.c_int32))
        f.append((k, ctypes.c_void_p))
    return f


class KadSUColumns(ctypes.Structure):
    _fields_ = _su_fields()


class KadPackStats(ctypes.Structure):
    _fields_ = [("n_reqs", ctypes.c_void_p), ("n_tols", ctypes.c_void_p), ("n_distinct_reqs", ctypes.c_int32),
                ("n_tolsets", ctypes.c_int32)]


def _strs(strings: Sequence[str], keep: list) -> KadStrs:
    parts = [s.encode() for s in strings]
    off = np.zeros(len(parts) + 1, I64)
    if parts:
        off[1:] = np.cumsum([len(p) for p in parts])
    data = np.frombuffer(b"".join(parts) or b"\0", U8).copy()
    keep += [off, data]
    return KadStrs(len(parts), off.ctypes.data, data.ctypes.data)


class NativeBatch:
    """A batch blob from the native packer; duck-types ``pack.Batch`` for the runtime and bench."""

    def __init__(self, snap, fwk: Framework, blob: np.ndarray, n_reqs: np.ndarray, n_tols: np.ndarray,
                 n_distinct_reqs: int, n_tolsets: int):
        from .pack import B_FLAGS, B_OUT_OFF, BatchHeader, array_of, header_of

        self.snap, self.fwk, self.blob = snap, fwk, blob
        h = header_of(blob, BatchHeader)
        self.W = int(h.n_units)
        self.n_out_slots = int(h.n_out_slots)
        self.out_off = array_of(blob, h, B_OUT_OFF, np.int64, self.W + 1)
        self.flags = array_of(blob, h, B_FLAGS, np.uint32, self.W)
        self.n_reqs, self.n_tols = n_reqs, n_tols
        self.n_distinct_reqs, self.n_tolsets = n_distinct_reqs, n_tolsets
        self.units = None
        self.in_place = None  # (packer, generation) for a blob that lives in the packer's buffer

    def check_current(self):
        """An in-place blob (pack(take=False)) is the packer's buffer, which its next pack rewrites and its
        close() frees: refuse to hand a stale or freed one to the device."""
        if self.in_place is not None:
            packer, gen = self.in_place
            if not getattr(packer, "h", None):
                raise ValueError("in-place batch: its NativePacker was closed")
            if packer.gen != gen:
                raise ValueError("in-place batch: its NativePacker has packed another batch since (pack with "
                                 "take=True to keep a batch)")


def _from_blob(blob: np.ndarray, fwk: Framework) -> "NativeBatch":
    """A received batch blob (e.g. sent by the packing rank) as a NativeBatch without pack statistics."""
    return NativeBatch(None, fwk, blob, np.zeros(0, np.int64), np.zeros(0, np.int64), -1, -1)


NativeBatch.from_blob = staticmethod(_from_blob)


def default_threads() -> int:
    """Packer threads: the process's CPU share — OMP_NUM_THREADS when set (16 on the GPU boxes), else the CPU
    count — at most 16 (beyond that the interning merge and memory bandwidth stop scaling)."""
    import os

    try:
        n = int(os.environ.get("OMP_NUM_THREADS", "0"))
    except ValueError:
        n = 0
    if n <= 0:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def vocab_of(snap, keep: list) -> KadPackVocab:
    """kad_pack_vocab of a pack.Snapshot (the arrays it points into are appended to ``keep``)."""
    gvks = sorted(snap.gvk_id, key=snap.gvk_id.get)
    keys = sorted(snap.label_key_id, key=snap.label_key_id.get)
    vals, voff = [], [0]
    for k in keys:
        d = snap.label_vals[snap.label_key_id[k]]
        vals += sorted(d, key=d.get)
        voff.append(len(vals))
    voff_a = np.asarray(voff, I32)
    keep.append(voff_a)
    v = KadPackVocab()
    v.cluster_names = _strs(snap.names, keep)
    v.scalar_names = _strs(sorted(snap.scalar_id, key=snap.scalar_id.get), keep)
    v.gvk_group = _strs([g[0] for g in gvks], keep)
    v.gvk_version = _strs([g[1] for g in gvks], keep)
    v.gvk_kind = _strs([g[2] for g in gvks], keep)
    v.label_keys = _strs(keys, keep)
    v.label_val_off = voff_a.ctypes.data
    v.label_vals = _strs(vals, keep)
    v.taint_key = _strs([t.key for t in snap.taint_defs], keep)
    v.taint_value = _strs([t.value for t in snap.taint_defs], keep)
    v.taint_effect = _strs([t.effect for t in snap.taint_defs], keep)
    v.n_taint_words = snap.TW
    v.fingerprint = snap.fingerprint
    return v


class NativePacker:
    """kad_packer for one pack.Snapshot's vocabulary."""

    def __init__(self, snap):
        from .runtime import load_library

        self.L = L = load_library()
        P = ctypes.c_void_p
        L.kad_packer_create.argtypes = [P, ctypes.POINTER(P)]
        L.kad_packer_destroy.argtypes = [P]
        L.kad_packer_error.argtypes = [P]
        L.kad_packer_error.restype = ctypes.c_char_p
        L.kad_pack_batch.argtypes = [P, P, P, ctypes.c_int, ctypes.POINTER(ctypes.c_size_t), P]
        L.kad_packer_take.argtypes = [P, P, ctypes.c_size_t]
        L.kad_packer_blob.argtypes = [P, ctypes.POINTER(P), ctypes.POINTER(ctypes.c_size_t)]
        self.snap = snap
        self._keep: list = []
        v = vocab_of(snap, self._keep)
        h = ctypes.c_void_p()
        rc = L.kad_packer_create(ctypes.byref(v), ctypes.byref(h))
        if rc != 0:
            raise RuntimeError(f"kad_packer_create failed ({rc}): {L.kad_packer_error(None).decode()}")
        self.h = h
        self.gen = 0  # packs so far: an in-place batch is valid only while it is the latest

    def close(self):
        if getattr(self, "h", None):
            self.L.kad_packer_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def pack(self, fwk: Framework, cols: SUColumns, threads: int = 0, take: bool = True) -> NativeBatch:
        """kad_pack_batch. ``threads`` 0: the process's CPU share (OMP_NUM_THREADS, else the CPU count, at most
        16). ``take=False`` returns the blob in place (kad_packer_blob: page-locked, no copy), valid until this
        packer's next pack."""
        if threads <= 0:
            threads = default_threads()
        su = KadSUColumns()
        su.n_units = cols.n_units
        su.str = KadStrs(len(cols.str_off) - 1, cols.str_off.ctypes.data, cols.str_data.ctypes.data)
        for k, _ in FIELDS:
            setattr(su, k, cols.cols[k].ctypes.data)
        su.n_reqs = cols.n_reqs
        W = cols.n_units
        nr = np.zeros(max(1, W), I32)
        nt = np.zeros(max(1, W), I32)
        st = KadPackStats(nr.ctypes.data, nt.ctypes.data, 0, 0)
        prof = fwk.to_c()
        n = ctypes.c_size_t()
        if not self.h:
            raise RuntimeError("NativePacker is closed")
        self.gen += 1
        rc = self.L.kad_pack_batch(self.h, ctypes.byref(prof), ctypes.byref(su), threads, ctypes.byref(n),
                                   ctypes.byref(st))
        if rc != 0:
            raise RuntimeError(f"kad_pack_batch: {self.L.kad_packer_error(self.h).decode()}")
        if take:
            blob = np.empty(n.value, U8)
            rc = self.L.kad_packer_take(self.h, blob.ctypes.data, blob.nbytes)
            if rc != 0:
                raise RuntimeError(f"kad_packer_take: {self.L.kad_packer_error(self.h).decode()}")
        else:
            ptr, nb = ctypes.c_void_p(), ctypes.c_size_t()
            rc = self.L.kad_packer_blob(self.h, ctypes.byref(ptr), ctypes.byref(nb))
            if rc != 0:
                raise RuntimeError(f"kad_packer_blob: {self.L.kad_packer_error(self.h).decode()}")
            buf = (ctypes.c_uint8 * nb.value).from_address(ptr.value)
            buf._owner = self  # the array's base chain keeps the packer (and its page-locked buffer) alive
            blob = np.frombuffer(buf, dtype=U8)
        nbatch = NativeBatch(self.snap, fwk, blob, nr[:W].astype(np.int64), nt[:W].astype(np.int64),
                             int(st.n_distinct_reqs), int(st.n_tolsets))
        if not take:
            nbatch.in_place = (self, self.gen)
        return nbatch


# ------------------------------------------------------------------ federated objects → columns (native)
class KadTypeConfig(ctypes.Structure):
    _fields_ = [("group", ctypes.c_char_p), ("version", ctypes.c_char_p), ("kind", ctypes.c_char_p),
                ("plural_name", ctypes.c_char_p), ("namespaced", ctypes.c_int32), ("replicas_spec", ctypes.c_char_p)]


# include/kad_objects.h KAD_OBJ_*
OBJ_OK, OBJ_NO_POLICY, OBJ_POLICY_NOT_FOUND, OBJ_UNIT_ERROR, OBJ_UNIT_PANIC, OBJ_BAD_JSON, OBJ_POLICY_ERROR = range(7)

_PER_UNIT = ("group", "version", "kind", "namespace_", "name", "flags", "desired", "max_clusters", "req_cpu", "req_mem",
             "req_eph")
_CSR_PAYLOAD = {"scalar": ("scalar_name", "scalar_val"), "tol": ("tol_key", "tol_op", "tol_value", "tol_effect"),
                "sel": ("sel_key", "sel_value"), "rterm": ("rt_req", "rt_n_expr", "rt_n_field"),
                "pterm": ("pt_weight", "pt_req", "pt_n_expr"), "place": ("place_name",),
                "cur": ("cur_name", "cur_rep", "cur_has_rep"), "wt": ("wt_name", "wt_val"),
                "min": ("min_name", "min_val"), "max": ("max_name", "max_val"), "cap": ("cap_name", "cap_val")}


class ObjectUnits:
    """kad_units_from_objects: the SchedulingUnits of a batch of federated objects as columns, plus per
    object its status (``OBJ_*``), its row in the columns (-1 unless OK) and the matched policy's index."""

    def __init__(self, cols: SUColumns, status: np.ndarray, unit_index: np.ndarray, policy_index: np.ndarray,
                 messages: List[str]):
        self.cols, self.status, self.unit_index, self.policy_index = cols, status, unit_index, policy_index
        self.messages = messages


def _texts(items) -> List[bytes]:
    import json

    out = []
    for x in items:
        if isinstance(x, (bytes, bytearray)):
            out.append(bytes(x))
        elif isinstance(x, str):
            out.append(x.encode())
        else:
            out.append(json.dumps(x, separators=(",", ":")).encode())
    return out


def units_from_objects(type_config, objects: Sequence, policies: Sequence, policy_of: Optional[Sequence[int]] = None,
                       threads: int = 0) -> ObjectUnits:
    """Federated objects and (Cluster)PropagationPolicies — JSON texts (str / bytes) or decoded dicts — through
    the native builder (include/kad_objects.h): MatchedPolicyKey, the policy lookup and
    schedulingUnitForFedObject for every object, on the library's worker threads. ``policy_of``: each object's
    policy index (-1 none) when the caller did the lookup, else the objects' labels choose."""
    from .runtime import load_library

    L = load_library()
    P = ctypes.c_void_p
    L.kad_units_from_objects.argtypes = [P, P, P, P, ctypes.c_int, ctypes.POINTER(P)]
    L.kad_units_view.argtypes = [P, P, P, P, P]
    L.kad_units_message.argtypes = [P, ctypes.c_int32]
    L.kad_units_message.restype = ctypes.c_char_p
    L.kad_units_free.argtypes = [P]
    L.kad_units_free.restype = None
    keep: list = []
    ot, pt = _texts(objects), _texts(policies)

    def strs(parts):
        off = np.zeros(len(parts) + 1, I64)
        if parts:
            off[1:] = np.cumsum([len(p) for p in parts])
        data = np.frombuffer(b"".join(parts) or b"\0", U8).copy()
        keep.extend([off, data])
        return KadStrs(len(parts), off.ctypes.data, data.ctypes.data)

    so, sp = strs(ot), strs(pt)
    tc = KadTypeConfig(type_config.group.encode(), type_config.version.encode(), type_config.kind.encode(),
                       type_config.plural_name.encode(), 1 if type_config.namespaced else 0,
                       type_config.replicas_spec.encode())
    h = P()
    po = None
    if policy_of is not None:
        po = np.ascontiguousarray(policy_of, I32)
        if len(po) != len(ot):
            raise ValueError("policy_of: one entry per object")
        keep.append(po)
    rc = L.kad_units_from_objects(ctypes.byref(tc), ctypes.byref(so), ctypes.byref(sp),
                                  None if po is None else po.ctypes.data, threads if threads > 0 else default_threads(),
                                  ctypes.byref(h))
    if rc != 0:
        raise RuntimeError(f"kad_units_from_objects failed ({rc})")
    try:
        v = KadSUColumns()
        st, ui, pi = P(), P(), P()
        rc = L.kad_units_view(h, ctypes.byref(v), ctypes.byref(st), ctypes.byref(ui), ctypes.byref(pi))
        if rc != 0:
            raise RuntimeError(f"kad_units_view failed ({rc})")
        n = len(ot)

        def arr(ptr, dt, cnt):
            if cnt == 0:
                return np.zeros(0, dt)
            return np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(np.ctypeslib.as_ctypes_type(dt))),
                                         (cnt,)).copy()

        W = int(v.n_units)
        cols = {}
        for k in _PER_UNIT:
            cols[k] = arr(getattr(v, k), DTYPES[k], W)
        for g, payload in _CSR_PAYLOAD.items():
            off = arr(getattr(v, g + "_off"), I32, W + 1)
            cols[g + "_off"] = off
            for k in payload:
                cols[k] = arr(getattr(v, k), DTYPES[k], int(off[-1]))
        R = int(v.n_reqs)
        cols["rq_key"], cols["rq_op"] = arr(v.rq_key, I32, R), arr(v.rq_op, I32, R)
        cols["rq_val_off"] = arr(v.rq_val_off, I32, R + 1)
        cols["rq_val"] = arr(v.rq_val, I32, int(cols["rq_val_off"][-1]))
        ns = int(v.str.n)
        soff = arr(v.str.off, I64, ns + 1)
        sdata = arr(v.str.bytes, U8, int(soff[-1])) if soff[-1] else np.zeros(1, U8)
        status = arr(st, I32, n)
        out = ObjectUnits(SUColumns(W, soff, sdata, cols), status, arr(ui, I32, n), arr(pi, I32, n),
                          [L.kad_units_message(h, i).decode(errors="replace") if status[i] else "" for i in range(n)])
        return out
    finally:
        L.kad_units_free(h)


# include/kad_objects.h KAD_APPLY_*
APPLY_OK, APPLY_ERROR, APPLY_PANIC, APPLY_BAD_JSON = range(4)


APPLY_FIELDS = (("spec", "placements"), ("spec", "overrides"), ("metadata", "annotations"))


class Applied:
    """kad_apply_results' outputs: per object the status (``APPLY_*``), applySchedulingResult's "modified",
    whether the text changed at all (modified, or the added trigger annotation), the new texts (bytes), the
    failure messages and, per object, the new JSON of each of ``APPLY_FIELDS`` it wrote (None where not)."""

    def __init__(self, status, modified, changed, texts, messages, fields):
        self.status, self.modified, self.changed = status, modified, changed
        self.texts, self.messages, self.fields = texts, messages, fields


def apply_results_ex(type_config, objects: Sequence, cluster_names: Sequence[str], res_off, res_cluster, res_replicas,
                     follower=None, threshold_ns=None, trigger: Optional[Sequence[Optional[str]]] = None,
                     ann_only=None, threads: int = 0, with_fields: bool = True) -> Applied:
    """kad_apply_results: applySchedulingResult for a batch of objects (JSON texts or dicts) with results in
    kad_results_download's form (CSR of snapshot cluster ids, replicas -1 = nil). ``follower``: per object
    !DisableFollowerScheduling (default all True); ``threshold_ns``: per object the pod-unschedulable threshold
    or None; ``trigger``: per object the scheduling-trigger-hash annotation to add first (None: none);
    ``ann_only``: per object True = only that annotation (no result)."""
    from .runtime import load_library

    L = load_library()
    P = ctypes.c_void_p
    L.kad_apply_results.argtypes = [P, P, P, P, P, P, P, P, P, P, ctypes.c_int, ctypes.POINTER(P)]
    L.kad_applied_view.argtypes = [P, P, P, P, P]
    L.kad_applied_fields.argtypes = [P, P]
    L.kad_applied_message.argtypes = [P, ctypes.c_int32]
    L.kad_applied_message.restype = ctypes.c_char_p
    L.kad_applied_free.argtypes = [P]
    L.kad_applied_free.restype = None
    ot = _texts(objects)
    n = len(ot)
    keep: list = []

    def strs(parts):
        off = np.zeros(len(parts) + 1, I64)
        if parts:
            off[1:] = np.cumsum([len(p) for p in parts])
        data = np.frombuffer(b"".join(parts) or b"\0", U8).copy()
        keep.extend([off, data])
        return KadStrs(len(parts), off.ctypes.data, data.ctypes.data)

    so, sc = strs(ot), strs([c.encode() for c in cluster_names])
    st_trig = strs([(t or "").encode() for t in trigger]) if trigger is not None else None
    ao = np.ascontiguousarray(np.asarray(ann_only, U8)) if ann_only is not None else None
    ro = np.ascontiguousarray(res_off, I32)
    rc_ = np.ascontiguousarray(res_cluster, I32) if len(res_cluster) else np.zeros(1, I32)
    rr = np.ascontiguousarray(res_replicas, I64) if len(res_replicas) else np.zeros(1, I64)
    fo = np.ascontiguousarray(np.ones(n, U8) if follower is None else np.asarray(follower, U8))
    th = np.full(max(1, n), np.iinfo(np.int64).min, I64)
    if threshold_ns is not None:
        for i, t in enumerate(threshold_ns):
            if t is not None:
                th[i] = t
    if len(ro) != n + 1:
        raise ValueError("res_off: n_objects + 1 entries")
    h = P()
    rc = L.kad_apply_results(ctypes.byref(KadTypeConfig(
        type_config.group.encode(), type_config.version.encode(), type_config.kind.encode(),
        type_config.plural_name.encode(), 1 if type_config.namespaced else 0, type_config.replicas_spec.encode())),
        ctypes.byref(so), ctypes.byref(sc), ro.ctypes.data, rc_.ctypes.data, rr.ctypes.data, fo.ctypes.data,
        th.ctypes.data, None if st_trig is None else ctypes.byref(st_trig), None if ao is None else ao.ctypes.data,
        threads if threads > 0 else default_threads(), ctypes.byref(h))
    if rc != 0:
        raise RuntimeError(f"kad_apply_results failed ({rc})")
    try:
        st, md, ch = P(), P(), P()
        tx = KadStrs()
        L.kad_applied_view(h, ctypes.byref(st), ctypes.byref(md), ctypes.byref(ch), ctypes.byref(tx))

        def arr(ptr, ct, dt):
            return np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ct)), (n,)).astype(dt) if n else np.zeros(0, dt)

        status = arr(st, ctypes.c_int32, I32)
        modified = arr(md, ctypes.c_uint8, bool)
        changed = arr(ch, ctypes.c_uint8, bool)
        texts = []
        if n:
            off = np.ctypeslib.as_array(ctypes.cast(tx.off, ctypes.POINTER(ctypes.c_int64)), (n + 1,))
            data = ctypes.string_at(tx.bytes, int(off[-1])) if off[-1] else b""
            texts = [data[int(off[i]):int(off[i + 1])] for i in range(n)]
        msgs = [L.kad_applied_message(h, i).decode(errors="replace") if status[i] else "" for i in range(n)]
        fs = KadStrs()
        L.kad_applied_fields(h, ctypes.byref(fs))
        fields = []
        if n and with_fields:
            m = len(APPLY_FIELDS)
            foff = np.ctypeslib.as_array(ctypes.cast(fs.off, ctypes.POINTER(ctypes.c_int64)), (m * n + 1,))
            fdata = ctypes.string_at(fs.bytes, int(foff[-1])) if foff[-1] else b""
            for i in range(n):
                fields.append(tuple(fdata[int(foff[m * i + q]):int(foff[m * i + q + 1])] or None for q in range(m)))
        return Applied(status, modified, changed, texts, msgs, fields)
    finally:
        L.kad_applied_free(h)


def apply_results(type_config, objects: Sequence, cluster_names: Sequence[str], res_off, res_cluster, res_replicas,
                  follower=None, threshold_ns=None, threads: int = 0, with_fields: bool = False):
    """:func:`apply_results_ex` as (status, modified, texts, messages[, fields])."""
    a = apply_results_ex(type_config, objects, cluster_names, res_off, res_cluster, res_replicas, follower,
                         threshold_ns, threads=threads, with_fields=with_fields)
    if with_fields:
        return a.status, a.modified, a.texts, a.messages, a.fields
    return a.status, a.modified, a.texts, a.messages


# include/kad_objects.h KAD_TRIG_*
TRIG_HAS_HASH, TRIG_NO_SCHEDULING, TRIG_ANN_NOT_MAP = 1, 2, 4


class TriggerObjects:
    """kad_trigger_prefixes: per object the status (``OBJ_*``), the matched policy index (-1 none), the flags
    (``TRIG_*``), the trigger JSON's object part (bytes), the current trigger-hash annotation and messages."""

    def __init__(self, status, policy_index, flags, prefixes, current_hash, messages):
        self.status, self.policy_index, self.flags = status, policy_index, flags
        self.prefixes, self.current_hash, self.messages = prefixes, current_hash, messages


def trigger_prefixes(type_config, objects: Sequence, policies: Sequence, policy_of: Optional[Sequence[int]] = None,
                     threads: int = 0) -> TriggerObjects:
    """The object part of every object's scheduling-trigger JSON (objects.trigger_prefix) from the objects' texts,
    natively, with the policy lookup of kad_units_from_objects."""
    from .runtime import load_library

    L = load_library()
    P = ctypes.c_void_p
    L.kad_trigger_prefixes.argtypes = [P, P, P, P, ctypes.c_int, ctypes.POINTER(P)]
    L.kad_trigger_objs_view.argtypes = [P, P, P, P, P, P]
    L.kad_trigger_objs_message.argtypes = [P, ctypes.c_int32]
    L.kad_trigger_objs_message.restype = ctypes.c_char_p
    L.kad_trigger_objs_free.argtypes = [P]
    L.kad_trigger_objs_free.restype = None
    keep: list = []
    ot, pt = _texts(objects), _texts(policies)
    n = len(ot)

    def strs(parts):
        off = np.zeros(len(parts) + 1, I64)
        if parts:
            off[1:] = np.cumsum([len(p) for p in parts])
        data = np.frombuffer(b"".join(parts) or b"\0", U8).copy()
        keep.extend([off, data])
        return KadStrs(len(parts), off.ctypes.data, data.ctypes.data)

    so, sp = strs(ot), strs(pt)
    po = None
    if policy_of is not None:
        po = np.ascontiguousarray(policy_of, I32)
        if len(po) != n:
            raise ValueError("policy_of: one entry per object")
        keep.append(po)
    h = P()
    rc = L.kad_trigger_prefixes(ctypes.byref(KadTypeConfig(
        type_config.group.encode(), type_config.version.encode(), type_config.kind.encode(),
        type_config.plural_name.encode(), 1 if type_config.namespaced else 0, type_config.replicas_spec.encode())),
        ctypes.byref(so), ctypes.byref(sp), None if po is None else po.ctypes.data,
        threads if threads > 0 else default_threads(), ctypes.byref(h))
    if rc != 0:
        raise RuntimeError(f"kad_trigger_prefixes failed ({rc})")
    try:
        st, pi, fl = P(), P(), P()
        pf, ch = KadStrs(), KadStrs()
        L.kad_trigger_objs_view(h, ctypes.byref(st), ctypes.byref(pi), ctypes.byref(fl), ctypes.byref(pf),
                                ctypes.byref(ch))

        def arr(ptr, ct, dt):
            return np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ct)), (n,)).astype(dt) if n else np.zeros(0, dt)

        def split(s):
            if not n:
                return []
            off = np.ctypeslib.as_array(ctypes.cast(s.off, ctypes.POINTER(ctypes.c_int64)), (n + 1,))
            data = ctypes.string_at(s.bytes, int(off[-1])) if off[-1] else b""
            return [data[int(off[i]):int(off[i + 1])] for i in range(n)]

        status = arr(st, ctypes.c_int32, I32)
        msgs = [L.kad_trigger_objs_message(h, i).decode(errors="replace") if status[i] else "" for i in range(n)]
        return TriggerObjects(status, arr(pi, ctypes.c_int32, I32), arr(fl, ctypes.c_uint8, U8), split(pf),
                              [x.decode(errors="surrogateescape") for x in split(ch)], msgs)
    finally:
        L.kad_trigger_objs_free(h)

"""Host packer: FederatedCluster snapshot / SchedulingUnit batch → device blobs.

Layouts are defined in ``include/kad_sched.h``. Everything the reference
re-derives per (SchedulingUnit, cluster) pair — ResourceList → Resource
conversion (``clusterresources/fit.go:136-147``), label-selector construction
and validation (``util/clusterselector/util.go:31-93``), toleration matching
(``framework/util.go:406-450``), the FNV-1 prefix of each cluster name
(``util/planner/planner.go:185-195``) — is resolved here once, so the device
only compares interned ids and integers.

Interning is snapshot-wide: every label key/value, taint, GVK and scalar
resource present on any cluster gets an id; a SchedulingUnit term that names
something no cluster has is constant-folded (``KAD_OP_TRUE`` / ``FALSE``).
"""

from __future__ import annotations

import ctypes
import hashlib
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import k8s
from . import types as T
from .framework import ClusterAffinity, ClusterResourcesFit, Framework, PlacementFilter

ABI_VERSION = 2
ALIGN = 256

# ---------------------------------------------------------------- header mirrors
S_ALLOC_CPU, S_ALLOC_MEM, S_USED_CPU, S_USED_MEM, S_ALLOC_SCALAR, S_USED_SCALAR, S_ALLOC_CORES, \
    S_AVAIL_CORES, S_GVK, S_TAINT_NSNE, S_TAINT_NE, S_TAINT_PNS, S_LABEL_VAL, S_LABEL_INT, S_LABEL_INT_OK, \
    S_NAME_FNV, S_CFLAGS, S_NARRAYS = range(18)

(B_FLAGS, B_GVK, B_REQ_CPU, B_REQ_MEM, B_DESIRED, B_MAX_CLUSTERS, B_TOLSET, B_TOL_ALL, B_TOL_PNS, B_SREQ_OFF,
 B_SREQ_ID, B_SREQ_VAL, B_FPROG_OFF, B_FPROG, B_SPROG_OFF, B_SPROG, B_PLACE_OFF, B_PLACE, B_CUR_OFF, B_CUR_ID,
 B_CUR_REP, B_PREF_OFF, B_PREF_ID, B_PREF_W, B_PREF_MIN, B_PREF_MAX, B_PREF_CAP, B_PREF_FLAGS, B_KEY_OFF, B_KEY,
 B_OUT_OFF, B_REQ_OFF, B_REQ, B_NARRAYS) = range(34)

SNAPSHOT_MAGIC = 0x5344414B
BATCH_MAGIC = 0x4241444B
BATCH_NARROW_PREFS = 1  # kad_batch_header.flags KAD_BATCH_NARROW_PREFS

W_DUPLICATE = 1 << 0
W_STICKY = 1 << 1
W_AVOID_DISRUPTION = 1 << 2
W_KEEP_UNSCHED = 1 << 3
W_HAS_DESIRED = 1 << 4
W_HAS_MAX_CLUSTERS = 1 << 5
W_FIT_NONZERO = 1 << 6
W_HAS_PLACEMENT = 1 << 7
W_SCORE_ERROR = 1 << 8
W_DYNAMIC_WEIGHTS = 1 << 9
W_HAS_CURRENT = 1 << 10
W_WIDE_SCORES = 1 << 11

PREF_HAS_WEIGHT, PREF_HAS_MAX, PREF_HAS_CAP = 1, 2, 4

OP_IN, OP_NOTIN, OP_EXISTS, OP_DNE, OP_GT, OP_LT, OP_EQ, OP_TRUE, OP_FALSE, OP_NAME_EQ, OP_NAME_NE = range(1, 12)
TERM_HAS_EXPR, TERM_EXPR_VALID, TERM_HAS_FIELD, TERM_FIELD_VALID = 1, 2, 4, 8

ST_OK, ST_STICKY, ST_NO_FEASIBLE, ST_ERR_SCORE, ST_ERR_SELECT, ST_ERR_REPLICAS = range(6)
RF_TIE_STRADDLE, RF_REMAINDER_TIE, RF_HASH_TIE = 1, 2, 4


class SnapshotHeader(ctypes.Structure):
    _fields_ = [("magic", ctypes.c_uint32), ("abi_version", ctypes.c_uint32), ("n_clusters", ctypes.c_int32),
                ("n_gvk_words", ctypes.c_int32), ("n_taint_words", ctypes.c_int32),
                ("n_label_keys", ctypes.c_int32), ("n_scalar", ctypes.c_int32), ("reserved0", ctypes.c_int32),
                ("total_bytes", ctypes.c_uint64), ("fingerprint", ctypes.c_uint64),
                ("off", ctypes.c_uint64 * S_NARRAYS)]


class BatchHeader(ctypes.Structure):
    _fields_ = [("magic", ctypes.c_uint32), ("abi_version", ctypes.c_uint32), ("n_units", ctypes.c_int32),
                ("n_clusters", ctypes.c_int32), ("n_taint_words", ctypes.c_int32), ("n_tolsets", ctypes.c_int32),
                ("n_out_slots", ctypes.c_int64), ("max_row_slots", ctypes.c_int32),
                ("packed_filter_mask", ctypes.c_uint32), ("packed_select_plugin", ctypes.c_int32),
                ("n_reqs", ctypes.c_int32), ("flags", ctypes.c_uint32), ("reserved", ctypes.c_uint32),
                ("total_bytes", ctypes.c_uint64),
                ("snapshot_fingerprint", ctypes.c_uint64), ("off", ctypes.c_uint64 * B_NARRAYS)]


def _assemble(header, arrays: Sequence[np.ndarray]) -> np.ndarray:
    """Header + 256-B aligned arrays → one uint8 blob; fills header.off / total_bytes."""
    pos = (ctypes.sizeof(header) + ALIGN - 1) // ALIGN * ALIGN
    offs = []
    for a in arrays:
        offs.append(pos)
        pos += (a.nbytes + ALIGN - 1) // ALIGN * ALIGN
    blob = np.zeros(max(pos, ALIGN), dtype=np.uint8)
    for o, a in zip(offs, arrays):
        if a.nbytes:
            blob[o:o + a.nbytes] = np.ascontiguousarray(a).view(np.uint8).reshape(-1)
    for i, o in enumerate(offs):
        header.off[i] = o
    header.total_bytes = len(blob)
    hb = bytes(header)
    blob[:len(hb)] = np.frombuffer(hb, dtype=np.uint8)
    return blob


def _words(n_bits: int) -> int:
    return max(1, (n_bits + 63) // 64)


def _csr(rows: List[list], dtype) -> tuple:
    off = np.zeros(len(rows) + 1, dtype=np.int64)
    if rows:
        off[1:] = np.cumsum([len(r) for r in rows])
    if off[-1] >= (1 << 31):
        raise ValueError("CSR array exceeds 2^31 entries; split the batch")
    flat = np.fromiter((x for r in rows for x in r), dtype=dtype, count=int(off[-1]))
    return off.astype(np.int32), flat


# ===================================================================== snapshot
class Snapshot:
    """A packed cluster snapshot plus the host-side vocabularies the batch packer needs.

    Two passes over the clusters: :meth:`_intern` assigns vocabulary ids (label
    keys / values, taints by occurrence, API resources, scalar resource names,
    in cluster order), :meth:`_columns` computes one cluster's column of every
    snapshot array against that vocabulary. :meth:`update` reuses the second
    pass for cluster update events that fit the existing vocabulary.
    """

    # snapshot arrays in enum kad_snapshot_array order: (dtype, rows attribute or None = 1 row)
    ARRAYS = [(np.int64, None), (np.int64, None), (np.int64, None), (np.int64, None), (np.int64, "S"),
              (np.int64, "S"), (np.int64, None), (np.int64, None), (np.uint64, "GW"), (np.uint64, "TW"),
              (np.uint64, "TW"), (np.uint64, "TW"), (np.int32, "K"), (np.int64, "K"), (np.uint8, "K"),
              (np.uint32, None), (np.uint32, None)]

    def __init__(self, clusters: List[T.FederatedCluster]):
        C = len(clusters)
        self.clusters = list(clusters)
        self.keys = [T.cluster_key(c) for c in clusters]  # content identity per cluster (diff)
        self.names = [c.name for c in clusters]
        self.name_id: Dict[str, int] = {}
        for i, n in enumerate(self.names):
            if n in self.name_id:
                raise ValueError(f"duplicate cluster name {n!r} in snapshot")
            self.name_id[n] = i
        self.C = C
        self.scalar_id: Dict[str, int] = {}
        self.gvk_id: Dict[tuple, int] = {}
        self.taint_id: Dict[tuple, int] = {}
        self.taint_defs: List[T.Taint] = []
        self.label_key_id: Dict[str, int] = {}
        self.label_vals: List[Dict[str, int]] = []
        for c in clusters:
            self._intern(c)
        self.S = len(self.scalar_id)
        self.GW = _words(len(self.gvk_id))
        self.TW = _words(len(self.taint_defs))
        self.K = len(self.label_vals)
        arrays = [np.zeros((self._rows(r), C) if r else C, dt) for dt, r in self.ARRAYS]
        for i, c in enumerate(clusters):
            for a, col in zip(arrays, self._columns(c)):
                a[..., i] = col
        self.fingerprint = self._vocab_fingerprint()
        hdr = SnapshotHeader()
        hdr.magic, hdr.abi_version = SNAPSHOT_MAGIC, ABI_VERSION
        hdr.n_clusters, hdr.n_gvk_words, hdr.n_taint_words, hdr.n_label_keys, hdr.n_scalar = \
            C, self.GW, self.TW, self.K, self.S
        hdr.fingerprint = self.fingerprint
        self.blob = _assemble(hdr, arrays)
        self.offsets = list(hdr.off)
        # the arrays live inside the blob from here on: update() writes through these views
        self.arrays = [self.blob[o:o + a.nbytes].view(a.dtype).reshape(a.shape) for o, a in zip(self.offsets, arrays)]

    def _rows(self, attr: Optional[str]) -> int:
        return 1 if attr is None else getattr(self, attr)

    def _intern(self, c: T.FederatedCluster) -> None:
        a = _Resource.new(c.allocatable)
        u = _Resource.new(c.allocatable)
        u.sub(c.available)
        for n in list(a.scalar or {}) + list(u.scalar or {}):
            self.scalar_id.setdefault(n, len(self.scalar_id))
        for r in c.api_resource_types:
            self.gvk_id.setdefault((r.group, r.version, r.kind), len(self.gvk_id))
        seen: Dict[tuple, int] = {}
        for t in c.taints:
            base = (t.key, t.value, t.effect)
            occ = seen.get(base, 0)
            seen[base] = occ + 1
            key = base + (occ,)
            if key not in self.taint_id:
                self.taint_id[key] = len(self.taint_defs)
                self.taint_defs.append(t)
        for k, v in (c.labels or {}).items():
            kid = self.label_key_id.get(k)
            if kid is None:
                kid = self.label_key_id[k] = len(self.label_vals)
                self.label_vals.append({})
            self.label_vals[kid].setdefault(v, len(self.label_vals[kid]))

    def _columns(self, c: T.FederatedCluster) -> Optional[list]:
        """Cluster ``c``'s column of every snapshot array, or None if it needs a vocabulary entry not interned."""
        a = _Resource.new(c.allocatable)
        u = _Resource.new(c.allocatable)
        cflags = 1 if u.sub(c.available) else 0
        S, GW, TW, K = self.S, self.GW, self.TW, self.K
        alloc_s, used_s = np.zeros(S, np.int64), np.zeros(S, np.int64)
        for m, dst in ((a.scalar or {}, alloc_s), (u.scalar or {}, used_s)):
            for n, v in m.items():
                sid = self.scalar_id.get(n)
                if sid is None:
                    return None
                dst[sid] = v
        # rsp.go:286-325: cpu defaults to "0" and is summed with the listed quantity
        alloc_cores = k8s.value(k8s.quantity("0") + k8s.quantity(c.allocatable["cpu"])) \
            if c.allocatable and "cpu" in c.allocatable else 0
        avail_cores = k8s.value(k8s.quantity("0") + k8s.quantity(c.available["cpu"])) \
            if c.available and "cpu" in c.available else 0
        gvk = np.zeros(GW, np.uint64)
        for r in c.api_resource_types:
            g = self.gvk_id.get((r.group, r.version, r.kind))
            if g is None:
                return None
            gvk[g // 64] |= np.uint64(1 << (g % 64))
        nsne, ne, pns = np.zeros(TW, np.uint64), np.zeros(TW, np.uint64), np.zeros(TW, np.uint64)
        seen: Dict[tuple, int] = {}
        for t in c.taints:
            base = (t.key, t.value, t.effect)
            occ = seen.get(base, 0)
            seen[base] = occ + 1
            tid = self.taint_id.get(base + (occ,))
            if tid is None:
                return None
            bit = np.uint64(1 << (tid % 64))
            if t.effect in (T.TAINT_NO_SCHEDULE, T.TAINT_NO_EXECUTE):
                nsne[tid // 64] |= bit
            if t.effect == T.TAINT_NO_EXECUTE:
                ne[tid // 64] |= bit
            if t.effect == T.TAINT_PREFER_NO_SCHEDULE:
                pns[tid // 64] |= bit
        lval, lint, lok = np.full(K, -1, np.int32), np.zeros(K, np.int64), np.zeros(K, np.uint8)
        for k, v in (c.labels or {}).items():
            kid = self.label_key_id.get(k)
            if kid is None or v not in self.label_vals[kid]:
                return None
            lval[kid] = self.label_vals[kid][v]
            iv, ok = k8s.parse_int64(v)
            if ok:
                lint[kid] = iv
                lok[kid] = 1
        return [a.milli_cpu, a.memory, u.milli_cpu, u.memory, alloc_s, used_s, alloc_cores, avail_cores, gvk, nsne,
                ne, pns, lval, lint, lok, k8s.fnv1_32(c.name.encode()), cflags]

    def _vocab_fingerprint(self) -> int:
        h = hashlib.blake2b(digest_size=8)
        h.update(repr((self.C, self.names, list(self.scalar_id), list(self.gvk_id), list(self.taint_id),
                       list(self.label_key_id), [list(v) for v in self.label_vals])).encode())
        return int.from_bytes(h.digest(), "little")

    def diff(self, clusters: List[T.FederatedCluster]) -> Optional["SnapshotDelta"]:
        """The delta from this snapshot to ``clusters`` (cluster update events), without applying it.

        Returns None — the caller repacks (``Snapshot(clusters)``) and re-uploads
        — when the names or their order changed (join / leave) or a changed
        cluster needs a vocabulary entry that is not interned yet. Otherwise a
        delta blob of the changed clusters' columns (compared by
        :func:`types.cluster_key`: resourceVersion, else content) for
        ``kad_snapshot_update``; the vocabulary (and with it every packed
        batch) stays valid. :meth:`commit` writes it into this snapshot once
        the device has taken it.
        """
        if len(clusters) != self.C or any(c.name != n for c, n in zip(clusters, self.names)):
            return None
        changed, cols, keys = [], [], []
        for i, new in enumerate(clusters):
            k = T.cluster_key(new)
            if k == self.keys[i]:
                continue
            col = self._columns(new)
            if col is None:
                return None
            changed.append(i)
            cols.append(col)
            keys.append(k)
        d = SnapshotDelta(self, changed, cols)
        d.clusters, d.keys = list(clusters), keys
        return d

    def commit(self, delta: "SnapshotDelta") -> None:
        """Apply a delta from :meth:`diff` to the host copy (blob columns, cluster list, keys)."""
        for i, col, k in zip(delta.changed, delta.cols, delta.keys):
            for a, v in zip(self.arrays, col):
                a[..., i] = v
            self.keys[i] = k
        self.clusters = delta.clusters

    def update(self, clusters: List[T.FederatedCluster]) -> Optional["SnapshotDelta"]:
        """:meth:`diff` + :meth:`commit` on the host copy; returns the delta (None: repack)."""
        d = self.diff(clusters)
        if d is not None:
            self.commit(d)
        return d


DELTA_MAGIC = 0x4441444B


class SnapshotDeltaHeader(ctypes.Structure):
    _fields_ = [("magic", ctypes.c_uint32), ("abi_version", ctypes.c_uint32), ("n_clusters", ctypes.c_int32),
                ("n_changed", ctypes.c_int32), ("total_bytes", ctypes.c_uint64), ("fingerprint", ctypes.c_uint64),
                ("idx_off", ctypes.c_uint64), ("off", ctypes.c_uint64 * S_NARRAYS)]


class SnapshotDelta:
    """A kad_snapshot_delta blob: the changed clusters' columns of every snapshot array ([rows][n_changed])."""

    def __init__(self, snap: Snapshot, changed: List[int], cols: List[list]):
        n = len(changed)
        self.changed = changed
        self.cols = cols
        self.clusters: List[T.FederatedCluster] = []
        self.keys: list = []
        arrays = [np.array(changed, np.int32)]
        for k, (dt, r) in enumerate(Snapshot.ARRAYS):
            rows = snap._rows(r)
            m = np.zeros((rows, n) if r else n, dt)
            for j, col in enumerate(cols):
                m[..., j] = col[k]
            arrays.append(m)
        hdr = SnapshotDeltaHeader()
        hdr.magic, hdr.abi_version, hdr.n_clusters, hdr.n_changed = DELTA_MAGIC, ABI_VERSION, snap.C, n
        hdr.fingerprint = snap.fingerprint
        # _assemble fills a header's `off` array; lay the index array out first, then the snapshot arrays
        pos = (ctypes.sizeof(hdr) + ALIGN - 1) // ALIGN * ALIGN
        offs = []
        for a in arrays:
            offs.append(pos)
            pos += (a.nbytes + ALIGN - 1) // ALIGN * ALIGN
        blob = np.zeros(max(pos, ALIGN), np.uint8)
        for o, a in zip(offs, arrays):
            if a.nbytes:
                blob[o:o + a.nbytes] = np.ascontiguousarray(a).view(np.uint8).reshape(-1)
        hdr.idx_off = offs[0]
        for k, o in enumerate(offs[1:]):
            hdr.off[k] = o
        hdr.total_bytes = len(blob)
        hb = bytes(hdr)
        blob[:len(hb)] = np.frombuffer(hb, np.uint8)
        self.blob = blob


class _Resource:
    """framework.Resource Add/Sub (framework/util.go:98-168) over quantity strings."""

    __slots__ = ("milli_cpu", "memory", "eph", "scalar")

    def __init__(self):
        self.milli_cpu = self.memory = self.eph = 0
        self.scalar = None

    @staticmethod
    def new(rl):
        r = _Resource()
        for n, q in (rl or {}).items():
            if n == "cpu":
                r.milli_cpu = k8s.wrap64(r.milli_cpu + k8s.milli_value(q))
            elif n == "memory":
                r.memory = k8s.wrap64(r.memory + k8s.value(q))
            elif n == "ephemeral-storage":
                r.eph = k8s.wrap64(r.eph + k8s.value(q))
            elif k8s.is_scalar_resource_name(n):
                if r.scalar is None:
                    r.scalar = {}
                r.scalar[n] = k8s.wrap64(r.scalar.get(n, 0) + k8s.value(q))
        return r

    def sub(self, rl) -> bool:
        """Returns True on error (early return, like the reference)."""
        for n, q in (rl or {}).items():
            if n == "cpu":
                v = k8s.milli_value(q)
                if self.milli_cpu < v:
                    return True
                self.milli_cpu -= v
            elif n == "memory":
                v = k8s.value(q)
                if self.memory < v:
                    return True
                self.memory -= v
            elif n == "ephemeral-storage":
                v = k8s.value(q)
                if self.eph < v:
                    return True
                self.eph -= v
            elif k8s.is_scalar_resource_name(n):
                sc = self.scalar or {}
                v = k8s.value(q)
                if n not in sc and v > 0:
                    return True
                rv = sc.get(n, 0)
                if rv < v:
                    return True
                if self.scalar is None:
                    self.scalar = {}
                self.scalar[n] = rv - v
        return False


# ===================================================================== programs
_OPS = {T.OP_IN: OP_IN, T.OP_NOT_IN: OP_NOTIN, T.OP_EXISTS: OP_EXISTS, T.OP_DOES_NOT_EXIST: OP_DNE,
        T.OP_GT: OP_GT, T.OP_LT: OP_LT}


def _valid_requirement(r: T.ClusterSelectorRequirement) -> bool:
    """labels.NewRequirement validation (apimachinery v0.26.6 labels/selector.go)."""
    op = _OPS.get(r.operator)
    if op is None:
        return False
    vals = r.values or []
    if not k8s.is_qualified_name(r.key):
        return False
    if op in (OP_IN, OP_NOTIN) and len(vals) == 0:
        return False
    if op in (OP_EXISTS, OP_DNE) and len(vals) != 0:
        return False
    if op in (OP_GT, OP_LT):
        if len(vals) != 1:
            return False
        if not k8s.parse_int64(vals[0])[1]:
            return False
    return all(k8s.is_valid_label_value(v) for v in vals)


def _i64_words(v: int):
    u = v & ((1 << 64) - 1)
    lo, hi = u & 0xFFFFFFFF, u >> 32
    return [lo - (1 << 32) if lo >= (1 << 31) else lo, hi - (1 << 32) if hi >= (1 << 31) else hi]


class _Compiler:
    def __init__(self, snap: Snapshot):
        self.snap = snap
        self.req_id: Dict[tuple, int] = {}
        self.reqs: List[list] = []

    def intern(self, words: list) -> int:
        key = tuple(words)
        rid = self.req_id.get(key)
        if rid is None:
            rid = self.req_id[key] = len(self.reqs)
            self.reqs.append(list(words))
        return rid

    def label_req(self, r: T.ClusterSelectorRequirement) -> list:
        op = _OPS[r.operator]
        kid = self.snap.label_key_id.get(r.key)
        vals = r.values or []
        if kid is None:
            return [OP_TRUE if op in (OP_NOTIN, OP_DNE) else OP_FALSE, -1]
        if op in (OP_IN, OP_NOTIN):
            vocab = self.snap.label_vals[kid]
            ids = sorted({vocab[v] for v in vals if v in vocab})
            if not ids:
                return [OP_FALSE if op == OP_IN else OP_TRUE, -1]
            return [op | (len(ids) << 8), kid] + ids
        if op in (OP_EXISTS, OP_DNE):
            return [op, kid]
        thr, _ = k8s.parse_int64(vals[0])
        return [op | (2 << 8), kid] + _i64_words(thr)

    def eq_req(self, key: str, value: str) -> list:
        kid = self.snap.label_key_id.get(key)
        if kid is None or value not in self.snap.label_vals[kid]:
            return [OP_FALSE, -1]
        return [OP_EQ | (1 << 8), kid, self.snap.label_vals[kid][value]]

    def field_req(self, r: T.ClusterSelectorRequirement) -> list:
        v = (r.values or [""])[0]
        eq = r.operator == T.OP_IN
        if r.key == "metadata.name":
            return [OP_NAME_EQ if eq else OP_NAME_NE, self.snap.name_id.get(v, -1)]
        hit = (v == "")  # fields.Set.Get of a missing key reads as ""
        return [OP_TRUE if hit == eq else OP_FALSE, -1]

    @staticmethod
    def _valid_fields(reqs) -> bool:
        for r in reqs:
            if r.operator not in (T.OP_IN, T.OP_NOT_IN) or len(r.values or []) != 1:
                return False
        return True

    def filter_program(self, su: T.SchedulingUnit) -> list:
        prog = []
        sel = su.cluster_selector or {}
        prog.append(len(sel))
        for k, v in sel.items():
            prog.append(self.intern(self.eq_req(k, v)))
        ca = su.affinity.cluster_affinity if su.affinity is not None else None
        if ca is None or ca.required is None:
            prog.append(0)
            return prog
        prog.append(1)
        terms = ca.required.cluster_selector_terms or []
        prog.append(len(terms))
        for t in terms:
            exprs = t.match_expressions or []
            fields = t.match_fields or []
            flags = 0
            body_e, body_f = [], []
            n_e = n_f = 0
            if exprs:
                flags |= T_HAS_EXPR
                if all(_valid_requirement(r) for r in exprs):
                    flags |= T_EXPR_VALID
                    for r in exprs:
                        body_e.append(self.intern(self.label_req(r)))
                    n_e = len(exprs)
            if fields:
                flags |= T_HAS_FIELD
                if self._valid_fields(fields):
                    flags |= T_FIELD_VALID
                    for r in fields:
                        body_f.append(self.intern(self.field_req(r)))
                    n_f = len(fields)
            prog += [flags, n_e, n_f] + body_e + body_f
        return prog

    def score_program(self, su: T.SchedulingUnit):
        """→ (program, score_error, sum |weights|)."""
        ca = su.affinity.cluster_affinity if su.affinity is not None else None
        if ca is None or ca.preferred is None:
            return [0], False, 0
        body, n, err, wsum = [], 0, False, 0
        for p in ca.preferred:
            if p.weight == 0:
                continue
            exprs = p.preference.match_expressions or []
            if not exprs:
                continue  # labels.Nothing(): never matches
            if not all(_valid_requirement(r) for r in exprs):
                err = True
                continue
            n += 1
            wsum += abs(p.weight)
            body += [int(p.weight), len(exprs)]
            for r in exprs:
                body.append(self.intern(self.label_req(r)))
        return [n] + body, err, wsum


T_HAS_EXPR, T_EXPR_VALID, T_HAS_FIELD, T_FIELD_VALID = TERM_HAS_EXPR, TERM_EXPR_VALID, TERM_HAS_FIELD, TERM_FIELD_VALID


def _count_reqs(fp, sp) -> int:
    """Label/field requirements a unit evaluates per cluster (SURVEY.md §8(d) R_w)."""
    n, pc = fp[0], 1 + fp[0]
    present = fp[pc]
    pc += 1
    if present:
        n_terms = fp[pc]
        pc += 1
        for _ in range(n_terms):
            ne, nf = fp[pc + 1], fp[pc + 2]
            pc += 3 + ne + nf
            n += ne + nf
    pc = 1
    for _ in range(sp[0]):
        ne = sp[pc + 1]
        pc += 2 + ne
        n += ne
    return n


# ===================================================================== batch
class Batch:
    """A packed batch of SchedulingUnits (against one Snapshot, for one Framework)."""

    def __init__(self, snap: Snapshot, fwk: Framework, units: List[T.SchedulingUnit]):
        W = len(units)
        C = snap.C
        comp = _Compiler(snap)
        flags = np.zeros(W, np.uint32)
        gvk = np.full(W, -1, np.int32)
        req_cpu = np.zeros(W, np.int64)
        req_mem = np.zeros(W, np.int64)
        desired = np.zeros(W, np.int64)
        maxc = np.zeros(W, np.int64)
        tolset = np.zeros(W, np.int32)
        tol_key: Dict[tuple, int] = {}
        tol_rows: List[tuple] = []
        sreq, fprog, sprog, place, cur_id, cur_rep, keys = [], [], [], [], [], [], []
        pref_id, pref_w, pref_min, pref_max, pref_cap, pref_fl = [], [], [], [], [], []
        out_len = np.zeros(W, np.int64)
        narrow = True  # KAD_BATCH_NARROW_PREFS: every preference map value fits int32
        n_reqs = np.zeros(W, np.int64)
        n_tols = np.zeros(W, np.int64)
        select_max = fwk.select_plugin == 8
        place_on = fwk.has_filter(PlacementFilter)

        for w, su in enumerate(units):
            f = 0
            if su.scheduling_mode == T.SCHEDULING_MODE_DUPLICATE:
                f |= W_DUPLICATE
            cur = su.current_clusters or {}
            if su.sticky_cluster and len(cur) > 0:
                f |= W_STICKY
            if len(cur) > 0:
                f |= W_HAS_CURRENT
            if su.avoid_disruption:
                f |= W_AVOID_DISRUPTION
            am = su.auto_migration
            if am is not None and am.keep_unschedulable_replicas:
                f |= W_KEEP_UNSCHED
            if su.desired_replicas is not None:
                f |= W_HAS_DESIRED
                desired[w] = su.desired_replicas
            if su.max_clusters is not None:
                f |= W_HAS_MAX_CLUSTERS
                maxc[w] = max(min(su.max_clusters, k8s.INT64_MAX), k8s.INT64_MIN)
            rr = su.resource_request
            if not (rr.milli_cpu == 0 and rr.memory == 0 and rr.ephemeral_storage == 0
                    and len(rr.scalar_resources or {}) == 0):
                f |= W_FIT_NONZERO
            req_cpu[w], req_mem[w] = rr.milli_cpu, rr.memory
            sreq.append([(snap.scalar_id.get(n, -1), v) for n, v in (rr.scalar_resources or {}).items() if v > 0])
            gvk[w] = snap.gvk_id.get((su.group, su.version, su.kind), -1)
            # tolerations → tolerated-taint masks (one row per distinct toleration list)
            tk = tuple((t.key, t.operator, t.value, t.effect) for t in (su.tolerations or []))
            tid = tol_key.get(tk)
            if tid is None:
                tid = tol_key[tk] = len(tol_rows)
                tol_rows.append(su.tolerations or [])
            tolset[w] = tid
            fp_ = comp.filter_program(su)
            fprog.append(fp_)
            sp, serr, wsum = comp.score_program(su)
            sprog.append(sp)
            n_reqs[w] = _count_reqs(fp_, sp)
            n_tols[w] = len(su.tolerations or [])
            if serr:
                f |= W_SCORE_ERROR
            if wsum > (1 << 20):
                f |= W_WIDE_SCORES
            names = su.cluster_names or set()
            if len(names) > 0:
                f |= W_HAS_PLACEMENT
            place.append(sorted({snap.name_id[n] for n in names if n in snap.name_id}))
            total = su.desired_replicas if su.desired_replicas is not None else 0
            cl = sorted((snap.name_id[n], (r if r is not None else total)) for n, r in cur.items()
                        if n in snap.name_id)
            cur_id.append([c for c, _ in cl])
            cur_rep.append([r for _, r in cl])
            if len(su.weights or {}) == 0:
                f |= W_DYNAMIC_WEIGHTS
            ec = {}
            if am is not None:
                ec = {n: v for n, v in (am.estimated_capacity or {}).items() if v >= 0}
            for m in (su.weights, su.min_replicas, su.max_replicas, am.estimated_capacity if am is not None else None):
                narrow = narrow and all(k8s.INT32_MIN <= v <= k8s.INT32_MAX for v in (m or {}).values())
            pn = set(su.weights or {}) | set(su.min_replicas or {}) | set(su.max_replicas or {}) | set(ec)
            prefs = sorted((snap.name_id[n], n) for n in pn if n in snap.name_id)
            pid, pw, pmin, pmax, pcap, pfl = [], [], [], [], [], []
            for cid, n in prefs:
                fl = 0
                wv = (su.weights or {}).get(n)
                if wv is not None:
                    fl |= PREF_HAS_WEIGHT
                mx = (su.max_replicas or {}).get(n)
                if mx is not None:
                    fl |= PREF_HAS_MAX
                cp = ec.get(n)
                if cp is not None:
                    fl |= PREF_HAS_CAP
                pid.append(cid)
                pw.append(wv or 0)
                pmin.append((su.min_replicas or {}).get(n, 0))
                pmax.append(mx or 0)
                pcap.append(cp or 0)
                pfl.append(fl)
            pref_id.append(pid)
            pref_w.append(pw)
            pref_min.append(pmin)
            pref_max.append(pmax)
            pref_cap.append(pcap)
            pref_fl.append(pfl)
            keys.append(list(su.key().encode()))
            bound = C
            if select_max and su.max_clusters is not None and su.max_clusters >= 0:
                bound = min(bound, su.max_clusters)
            if place_on and (f & W_HAS_PLACEMENT):
                bound = min(bound, len(place[-1]))
            if f & W_STICKY:
                bound = 0
            out_len[w] = bound
            flags[w] = f

        TW = snap.TW
        NT = max(1, len(tol_rows))
        tol_all = np.zeros((NT, TW), np.uint64)
        tol_pns = np.zeros((NT, TW), np.uint64)
        for r, tols in enumerate(tol_rows):
            pns_tols = [t for t in tols if t.effect in ("", T.TAINT_PREFER_NO_SCHEDULE)]
            for tid_, taint in enumerate(snap.taint_defs):
                bit = np.uint64(1 << (tid_ % 64))
                if any(k8s.tolerates_taint(t, taint) for t in tols):
                    tol_all[r, tid_ // 64] |= bit
                if any(k8s.tolerates_taint(t, taint) for t in pns_tols):
                    tol_pns[r, tid_ // 64] |= bit

        sreq_off, sreq_id = _csr([[a for a, _ in r] for r in sreq], np.int32)
        _, sreq_val = _csr([[b for _, b in r] for r in sreq], np.int64)
        fprog_off, fprog_a = _csr(fprog, np.int32)
        sprog_off, sprog_a = _csr(sprog, np.int32)
        place_off, place_a = _csr(place, np.int32)
        cur_off, cur_id_a = _csr(cur_id, np.int32)
        _, cur_rep_a = _csr(cur_rep, np.int64)
        pref_off, pref_id_a = _csr(pref_id, np.int32)
        pdt = np.int32 if narrow else np.int64
        _, pref_w_a = _csr(pref_w, pdt)
        _, pref_min_a = _csr(pref_min, pdt)
        _, pref_max_a = _csr(pref_max, pdt)
        _, pref_cap_a = _csr(pref_cap, pdt)
        _, pref_fl_a = _csr(pref_fl, np.uint32)
        key_off, key_a = _csr(keys, np.uint8)
        req_off, req_a = _csr(comp.reqs, np.int32)
        out_off = np.zeros(W + 1, np.int64)
        out_off[1:] = np.cumsum(out_len)

        arrays = [flags, gvk, req_cpu, req_mem, desired, maxc, tolset, tol_all, tol_pns, sreq_off, sreq_id,
                  sreq_val, fprog_off, fprog_a, sprog_off, sprog_a, place_off, place_a, cur_off, cur_id_a, cur_rep_a,
                  pref_off, pref_id_a, pref_w_a, pref_min_a, pref_max_a, pref_cap_a, pref_fl_a, key_off, key_a,
                  out_off, req_off, req_a]
        hdr = BatchHeader()
        hdr.magic, hdr.abi_version = BATCH_MAGIC, ABI_VERSION
        hdr.n_units, hdr.n_clusters, hdr.n_taint_words, hdr.n_tolsets = W, C, TW, NT
        hdr.n_out_slots = int(out_off[-1])
        hdr.max_row_slots = int(out_len.max()) if W else 0
        hdr.packed_filter_mask = fwk.filter_mask
        hdr.packed_select_plugin = fwk.select_plugin
        hdr.n_reqs = len(comp.reqs)
        hdr.flags = BATCH_NARROW_PREFS if narrow else 0
        hdr.snapshot_fingerprint = snap.fingerprint
        self.blob = _assemble(hdr, arrays)
        self.n_reqs = n_reqs
        self.n_distinct_reqs = len(comp.reqs)
        self.n_tols = n_tols
        self.W = W
        self.n_out_slots = int(out_off[-1])
        self.out_off = out_off
        self.units = units
        self.snap = snap
        self.fwk = fwk
        self.arrays = arrays


def pack_snapshot(clusters: List[T.FederatedCluster]) -> Snapshot:
    return Snapshot(clusters)


def pack_batch(snap: Snapshot, fwk: Framework, units: List[T.SchedulingUnit]) -> Batch:
    return Batch(snap, fwk, units)


def header_of(blob: np.ndarray, cls):
    return cls.from_buffer_copy(blob[:ctypes.sizeof(cls)].tobytes())


def array_of(blob: np.ndarray, hdr, idx: int, dtype, count: Optional[int] = None) -> np.ndarray:
    start = hdr.off[idx]
    end = hdr.off[idx + 1] if idx + 1 < len(hdr.off) else hdr.total_bytes
    a = blob[start:end].view(dtype)
    return a if count is None else a[:count]

"""TEST INFRASTRUCTURE ONLY — restatement of Scheduler.computeSchedulingTriggerHash.

``pkg/controllers/scheduler/schedulingtriggers.go:69-262``: build the
``schedulingTriggers`` struct, ``json.Marshal`` it, FNV-1 32 the bytes,
format the sum as a decimal. Written independently of the product's
split-and-concatenate builder (kubeadmiral_amd/objects.py): here the whole
struct is assembled as nested ordered values and serialised by Python's json
encoder, then the output is corrected to Go 1.19's ``encodeState.string``
rules (HTML-safe escapes, ``\\u0008``/``\\u000c`` instead of ``\\b``/``\\f``,
U+2028/2029 escaped, unpaired surrogates → U+FFFD).

Parity status: the FNV-1 function is pinned by planner_test.go's vectors
(tests/golden); the JSON layout is restated from the struct tags and has no
reference fixture (the reference has no test for this function) — parity
unpinned beyond that.
"""

from __future__ import annotations

import json
import re

from .gosem import fnv1_32, go_sort_slice

KNOWN = {
    "kubeadmiral.io/scheduling-mode", "kubeadmiral.io/sticky-cluster", "kubeadmiral.io/tolerations",
    "kubeadmiral.io/placements", "kubeadmiral.io/clusterSelector", "kubeadmiral.io/affinity",
    "kubeadmiral.io/maxClusters", "kubeadmiral.io/follows-object",
}  # schedulingtriggers.go:150-159 via constants.go:31-43
AUTO_MIGRATION_INFO = "kubeadmiral.io/auto-migration-info"

_ESC = re.compile(r"\\(u[0-9a-fA-F]{4}|.)")


def _go_string(s: str) -> str:
    s = "".join("�" if 0xD800 <= ord(c) <= 0xDFFF else c for c in s)
    out = json.dumps(s, ensure_ascii=False)

    def fix(m):
        e = m.group(1)
        return {"b": "\\u0008", "f": "\\u000c"}.get(e, "\\" + e)

    out = _ESC.sub(fix, out)
    for a, b in (("<", "\\u003c"), (">", "\\u003e"), ("&", "\\u0026"), ("\u2028", "\\u2028"),
                 ("\u2029", "\\u2029")):
        out = out.replace(a, b)
    return out


class _Obj(list):
    """A struct: ordered (json name, value) members."""


def _marshal(v) -> str:
    if v is None:
        return "null"
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, int):
        return str(v)
    if isinstance(v, str):
        return _go_string(v)
    if isinstance(v, _Obj):
        return "{" + ",".join(_go_string(k) + ":" + _marshal(x) for k, x in v) + "}"
    return "[" + ",".join(_marshal(x) for x in v) + "]"


def _sort_map(m):
    # sortMap: collect then sort.Slice by key (keys unique)
    kv = [(k, v) for k, v in (m or {}).items()]
    go_sort_slice(kv, lambda a, b: a[0].encode() < b[0].encode())
    return [_Obj([("key", k), ("value", v)]) for k, v in kv]


def _taint_less(l, r):  # :215-227 — the effect branch compares values
    if l.key != r.key:
        return l.key.encode() < r.key.encode()
    if l.value != r.value:
        return l.value.encode() < r.value.encode()
    if l.effect != r.effect:
        return l.value.encode() < r.value.encode()
    return False


def _api_less(l, r):  # :241-257 — the kind branch returns Kind != Kind
    if l.group != r.group:
        return l.group.encode() < r.group.encode()
    if l.version != r.version:
        return l.version.encode() < r.version.encode()
    if l.kind != r.kind:
        return l.kind != r.kind
    if l.plural_name != r.plural_name:
        return l.plural_name.encode() < r.plural_name.encode()
    if l.scope != r.scope:
        return l.scope.encode() < r.scope.encode()
    return False


def trigger_json(annotations, replica_count: int, policy, clusters) -> bytes:
    """json.Marshal(schedulingTriggers) — policy: None or (name, generation, auto_migration_enabled)."""
    ann = dict(annotations or {})
    sched = {k: v for k, v in ann.items() if k in KNOWN}
    fields = [
        ("schedulingAnnotations", _sort_map(sched)),
        ("replicaCount", replica_count),
        ("resourceRequest", _Obj([("millicpu", 0), ("memory", 0), ("ephemeralStorage", 0),
                                  ("scalarResources", None)])),
    ]
    name, gen = "", 0
    if policy is not None:
        name, gen, auto = policy
        if auto and AUTO_MIGRATION_INFO in ann:
            fields.append(("autoMigrationInfo", ann[AUTO_MIGRATION_INFO]))
    fields += [("policyName", name), ("policyGeneration", gen)]
    labels, taints, apis = {}, {}, {}
    for c in clusters:
        labels[c.name] = _sort_map(c.labels)
        tl = list(c.taints or [])
        go_sort_slice(tl, _taint_less)
        taints[c.name] = [_Obj([("key", t.key)] + ([("value", t.value)] if t.value else []) + [("effect", t.effect)])
                          for t in tl]
        al = list(c.api_resource_types or [])
        go_sort_slice(al, _api_less)
        apis[c.name] = [_Obj(([("group", a.group)] if a.group else []) + [
            ("version", a.version), ("kind", a.kind), ("pluralName", a.plural_name), ("scope", a.scope)]) for a in al]
    fields += [("clusterLabels", _sort_map(labels)), ("clusterTaints", _sort_map(taints)),
               ("clusterAPIResourceTypes", _sort_map(apis))]
    return _marshal(_Obj(fields)).encode("utf-8")


def trigger_hash(annotations, replica_count, policy, clusters) -> str:
    """strconv.FormatInt(int64(fnv.New32 over the JSON)), as written to the trigger-hash annotation."""
    return str(fnv1_32(trigger_json(annotations, replica_count, policy, clusters)))

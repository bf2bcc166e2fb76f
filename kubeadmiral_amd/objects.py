"""Federated objects and policies on either side of the batch scheduler.

Host-side restatement of the scheduler controller's object handling — the
data formats that feed ``genericScheduler.Schedule`` and the step that writes
its result back:

* :func:`scheduling_unit_for_fed_object` — ``schedulingunit.go:38-163``: a
  federated object (unstructured, i.e. decoded JSON) + its propagation policy
  (+ the object's annotation overrides, ``:224-668``) → ``SchedulingUnit``.
* :func:`matched_policy_key` — ``scheduler/util.go:37-49``.
* :func:`apply_scheduling_result` — ``scheduler.go:632-695`` with
  ``util/placement.go:44-59``, ``scheduler/util.go:71-185`` and
  ``util/overrides.go:68-180``: placements + replica overrides + annotations,
  reporting whether the object changed.
* :class:`TriggerHasher` — the bytes of ``computeSchedulingTriggerHash``
  (``schedulingtriggers.go:106-262``); the FNV-1 over them runs on the GPU
  (``kad_trigger_hashes``), see :mod:`kubeadmiral_amd.runtime`.

Unstructured objects are plain ``dict``/``list`` trees as ``json.loads``
returns them: ints stand for Go int64, floats for float64. Go ``nil`` is
``None`` where the reference distinguishes it from empty. Where the reference
panics (a type assertion on a non-float override value, a nil spec) this
module raises :class:`GoPanic`; where it returns an error, :class:`ObjectError`.
"""

from __future__ import annotations

import copy
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Set, Tuple

from . import gojson as J
from . import types as T
from .gosort import sort_slice

# pkg/controllers/common/constants.go:27-29,56,79-81,97-132
DEFAULT_PREFIX = "kubeadmiral.io/"
INTERNAL_PREFIX = "internal." + DEFAULT_PREFIX
TEMPLATE_PATH = ("spec", "template")
PLACEMENTS_PATH = ("spec", "placements")
OVERRIDES_PATH = ("spec", "overrides")
ANNOTATION_VALUE_TRUE, ANNOTATION_VALUE_FALSE = "true", "false"
NO_SCHEDULING_ANNOTATION = DEFAULT_PREFIX + "no-scheduling"
AUTO_MIGRATION_INFO_ANNOTATION = DEFAULT_PREFIX + "auto-migration-info"
ENABLE_FOLLOWER_SCHEDULING_ANNOTATION = INTERNAL_PREFIX + "enable-follower-scheduling"
POD_UNSCHEDULABLE_THRESHOLD_ANNOTATION = INTERNAL_PREFIX + "pod-unschedulable-threshold"

# pkg/controllers/scheduler/constants.go:24-52
GLOBAL_SCHEDULER_NAME = "global-scheduler"
PREFIXED_GLOBAL_SCHEDULER_NAME = DEFAULT_PREFIX + "global-scheduler"
PROPAGATION_POLICY_NAME_LABEL = DEFAULT_PREFIX + "propagation-policy-name"
CLUSTER_PROPAGATION_POLICY_NAME_LABEL = DEFAULT_PREFIX + "cluster-propagation-policy-name"
FOLLOWS_OBJECT_ANNOTATION = DEFAULT_PREFIX + "follows-object"
SCHEDULING_MODE_ANNOTATION = DEFAULT_PREFIX + "scheduling-mode"
STICKY_CLUSTER_ANNOTATION = DEFAULT_PREFIX + "sticky-cluster"
TOLERATIONS_ANNOTATIONS = DEFAULT_PREFIX + "tolerations"
PLACEMENTS_ANNOTATIONS = DEFAULT_PREFIX + "placements"
CLUSTER_SELECTOR_ANNOTATIONS = DEFAULT_PREFIX + "clusterSelector"
AFFINITY_ANNOTATIONS = DEFAULT_PREFIX + "affinity"
MAX_CLUSTERS_ANNOTATIONS = DEFAULT_PREFIX + "maxClusters"
SCHEDULING_TRIGGER_HASH_ANNOTATION = DEFAULT_PREFIX + "scheduling-trigger-hash"
DEFAULT_SCHEDULING_MODE = T.SCHEDULING_MODE_DUPLICATE
OPERATION_REPLACE = "replace"  # scheduler/util.go:33-35

# util/overrides.go:43-48
INVALID_OVERRIDE_PATHS = frozenset({"/metadata/namespace", "/metadata/name", "/metadata/generateName", "/kind"})


class ObjectError(ValueError):
    """The reference returns a non-nil error for this object."""


class GoPanic(RuntimeError):
    """The reference panics on this input (e.g. a failed type assertion)."""


# ------------------------------------------------------------ policy / type config
@dataclass
class Preferences:  # pkg/apis/core/v1alpha1/types_propagationpolicy.go:138-154
    min_replicas: int = 0
    max_replicas: Optional[int] = None
    weight: Optional[int] = None


@dataclass
class Placement:  # types_propagationpolicy.go:128-134
    cluster: str = ""
    preferences: Preferences = field(default_factory=Preferences)


@dataclass
class AutoMigrationTrigger:  # types_propagationpolicy.go:172-178
    pod_unschedulable_for: Optional[str] = None   # metav1.Duration text, e.g. "1m30s"


@dataclass
class AutoMigration:  # types_propagationpolicy.go:157-168
    when: AutoMigrationTrigger = field(default_factory=AutoMigrationTrigger)
    keep_unschedulable_replicas: bool = False


@dataclass
class ReplicaRescheduling:  # types_propagationpolicy.go:181-189
    avoid_disruption: bool = False


@dataclass
class PropagationPolicySpec:  # types_propagationpolicy.go:62-110
    scheduling_profile: str = ""
    scheduling_mode: str = ""
    sticky_cluster: bool = False
    cluster_selector: Optional[Dict[str, str]] = None
    cluster_affinity: Optional[List[T.ClusterSelectorTerm]] = None
    tolerations: Optional[List[T.Toleration]] = None
    max_clusters: Optional[int] = None
    placements: Optional[List[Placement]] = None
    disable_follower_scheduling: bool = False
    auto_migration: Optional[AutoMigration] = None
    replica_rescheduling: Optional[ReplicaRescheduling] = None


@dataclass
class PropagationPolicy:
    """(Cluster)PropagationPolicy: the metadata the scheduler reads + the spec."""

    name: str = ""
    namespace: str = ""          # "" for a ClusterPropagationPolicy
    generation: int = 0
    spec: PropagationPolicySpec = field(default_factory=PropagationPolicySpec)

    @staticmethod
    def from_json(d: dict) -> "PropagationPolicy":
        meta = d.get("metadata") or {}
        spec = J.decode(POLICY_SPEC, J.from_unstructured(d.get("spec") or {}))
        return PropagationPolicy(meta.get("name", ""), meta.get("namespace", ""), int(meta.get("generation", 0)), spec)


def policy_to_json(pol: "PropagationPolicy") -> dict:
    """The (Cluster)PropagationPolicy as the API object the informer holds (metadata + spec JSON): the inverse of
    :meth:`PropagationPolicy.from_json` (``from_json(policy_to_json(p)) == p``), for the native object path
    (include/kad_objects.h), which reads policies as JSON."""
    sp = pol.spec
    spec: dict = {}
    if sp.scheduling_profile:
        spec["schedulingProfile"] = sp.scheduling_profile
    if sp.scheduling_mode:
        spec["schedulingMode"] = sp.scheduling_mode
    if sp.sticky_cluster:
        spec["stickyCluster"] = True
    if sp.cluster_selector is not None:
        spec["clusterSelector"] = dict(sp.cluster_selector)
    if sp.cluster_affinity is not None:
        spec["clusterAffinity"] = [t.to_json() for t in sp.cluster_affinity]
    if sp.tolerations is not None:
        spec["tolerations"] = [t.to_json() for t in sp.tolerations]
    if sp.max_clusters is not None:
        spec["maxClusters"] = sp.max_clusters
    if sp.placements is not None:
        pls = []
        for p in sp.placements:
            pr = {"minReplicas": p.preferences.min_replicas}
            if p.preferences.max_replicas is not None:
                pr["maxReplicas"] = p.preferences.max_replicas
            if p.preferences.weight is not None:
                pr["weight"] = p.preferences.weight
            pls.append({"cluster": p.cluster, "preferences": pr})
        spec["placement"] = pls
    if sp.disable_follower_scheduling:
        spec["disableFollowerScheduling"] = True
    if sp.auto_migration is not None:
        when = {}
        if sp.auto_migration.when.pod_unschedulable_for is not None:
            when["podUnschedulableFor"] = sp.auto_migration.when.pod_unschedulable_for
        spec["autoMigration"] = {"when": when,
                                 "keepUnschedulableReplicas": sp.auto_migration.keep_unschedulable_replicas}
    if sp.replica_rescheduling is not None:
        spec["replicaRescheduling"] = {"avoidDisruption": sp.replica_rescheduling.avoid_disruption}
    meta = {"name": pol.name, "generation": pol.generation}
    if pol.namespace:
        meta["namespace"] = pol.namespace
    return {"metadata": meta, "spec": spec}


@dataclass
class FederatedTypeConfig:
    """The FederatedTypeConfig fields the scheduler reads (types_federatedtypeconfig.go)."""

    group: str = ""
    version: str = ""
    kind: str = ""
    plural_name: str = ""
    scope: str = "Namespaced"
    replicas_spec: str = ""      # Spec.PathDefinition.ReplicasSpec, dot path under the template

    @property
    def namespaced(self) -> bool:
        return self.scope == "Namespaced"


# --------------------------------------------------------------- Go decoders
_REQ = J.struct(T.ClusterSelectorRequirement, [
    ("key", "key", J.STRING), ("operator", "operator", J.STRING), ("values", "values", J.slice_of(J.STRING))])
_TERM = J.struct(T.ClusterSelectorTerm, [
    ("matchExpressions", "match_expressions", J.slice_of(_REQ)), ("matchFields", "match_fields", J.slice_of(_REQ))])
_SELECTOR = J.struct(T.ClusterSelector, [("clusterSelectorTerms", "cluster_selector_terms", J.slice_of(_TERM))])
_PREF_TERM = J.struct(T.PreferredSchedulingTerm, [("weight", "weight", J.INT32), ("preference", "preference", _TERM)])
_CLUSTER_AFFINITY = J.struct(T.ClusterAffinity, [
    ("requiredDuringSchedulingIgnoredDuringExecution", "required", J.ptr_to(_SELECTOR)),
    ("preferredDuringSchedulingIgnoredDuringExecution", "preferred", J.slice_of(_PREF_TERM))])
AFFINITY = J.struct(T.Affinity, [("clusterAffinity", "cluster_affinity", J.ptr_to(_CLUSTER_AFFINITY))])
TOLERATION = J.struct(T.Toleration, [
    ("key", "key", J.STRING), ("operator", "operator", J.STRING), ("value", "value", J.STRING),
    ("effect", "effect", J.STRING), ("tolerationSeconds", "toleration_seconds", J.ptr_to(J.INT64))])
_PREFERENCES = J.struct(Preferences, [
    ("minReplicas", "min_replicas", J.INT64), ("maxReplicas", "max_replicas", J.ptr_to(J.INT64)),
    ("weight", "weight", J.ptr_to(J.INT64))])
PLACEMENT = J.struct(Placement, [("cluster", "cluster", J.STRING), ("preferences", "preferences", _PREFERENCES)])
_AUTO_MIGRATION = J.struct(AutoMigration, [
    ("when", "when", J.struct(AutoMigrationTrigger, [("podUnschedulableFor", "pod_unschedulable_for",
                                                      J.ptr_to(J.STRING))])),
    ("keepUnschedulableReplicas", "keep_unschedulable_replicas", J.BOOL)])
_REPLICA_RESCHEDULING = J.struct(ReplicaRescheduling, [("avoidDisruption", "avoid_disruption", J.BOOL)])

POLICY_SPEC = J.struct(PropagationPolicySpec, [
    ("schedulingProfile", "scheduling_profile", J.STRING),
    ("schedulingMode", "scheduling_mode", J.STRING),
    ("stickyCluster", "sticky_cluster", J.BOOL),
    ("clusterSelector", "cluster_selector", J.map_of(J.STRING)),
    ("clusterAffinity", "cluster_affinity", J.slice_of(_TERM)),
    ("tolerations", "tolerations", J.slice_of(TOLERATION)),
    ("maxClusters", "max_clusters", J.ptr_to(J.INT64)),
    ("placement", "placements", J.slice_of(PLACEMENT)),
    ("disableFollowerScheduling", "disable_follower_scheduling", J.BOOL),
    ("autoMigration", "auto_migration", J.ptr_to(_AUTO_MIGRATION)),
    ("replicaRescheduling", "replica_rescheduling", J.ptr_to(_REPLICA_RESCHEDULING)),
])


# federated object views (pkg/apis/types/v1alpha1/types_placements.go, types_overrides.go)
@dataclass
class _ClusterRef:
    name: str = ""


@dataclass
class _PlacementSet:
    clusters: Optional[List[_ClusterRef]] = None


@dataclass
class _PlacementWithController:
    controller: str = ""
    placement: _PlacementSet = field(default_factory=_PlacementSet)


@dataclass
class _SpecWithPlacements:
    placements: Optional[List[_PlacementWithController]] = None


@dataclass
class _ObjectMeta:
    name: str = ""
    namespace: str = ""
    generate_name: str = ""
    uid: str = ""
    resource_version: str = ""
    generation: int = 0
    labels: Optional[Dict[str, str]] = None
    annotations: Optional[Dict[str, str]] = None


@dataclass
class _ObjectWithPlacements:
    api_version: str = ""
    kind: str = ""
    metadata: _ObjectMeta = field(default_factory=_ObjectMeta)
    spec: _SpecWithPlacements = field(default_factory=_SpecWithPlacements)


@dataclass
class _OverridePatch:
    op: str = ""
    path: str = ""
    value: object = None


@dataclass
class _ClusterOverride:
    cluster_name: str = ""
    patches: Optional[List[_OverridePatch]] = None


@dataclass
class _ControllerOverride:
    controller: str = ""
    clusters: Optional[List[_ClusterOverride]] = None


@dataclass
class _SpecWithOverrides:
    overrides: Optional[List[_ControllerOverride]] = None


@dataclass
class _ObjectWithOverrides:
    spec: Optional[_SpecWithOverrides] = None


# metav1.ObjectMeta: the fields whose type is checked here (others are skipped — the
# scheduler's objects come from the API server, where they are well-typed)
_OBJECT_META = J.struct(_ObjectMeta, [
    ("name", "name", J.STRING), ("namespace", "namespace", J.STRING), ("generateName", "generate_name", J.STRING),
    ("uid", "uid", J.STRING), ("resourceVersion", "resource_version", J.STRING),
    ("generation", "generation", J.INT64), ("labels", "labels", J.map_of(J.STRING)),
    ("annotations", "annotations", J.map_of(J.STRING))])
_OBJ_PLACEMENTS = J.struct(_ObjectWithPlacements, [
    ("apiVersion", "api_version", J.STRING), ("kind", "kind", J.STRING), ("metadata", "metadata", _OBJECT_META),
    ("spec", "spec", J.struct(_SpecWithPlacements, [
        ("placements", "placements", J.slice_of(J.struct(_PlacementWithController, [
            ("controller", "controller", J.STRING),
            ("placement", "placement", J.struct(_PlacementSet, [
                ("clusters", "clusters", J.slice_of(J.struct(_ClusterRef, [("name", "name", J.STRING)])))]))])))]))])
_OVERRIDE_PATCH = J.struct(_OverridePatch, [("op", "op", J.STRING), ("path", "path", J.STRING), ("value", "value", J.ANY)])
_OBJ_OVERRIDES = J.struct(_ObjectWithOverrides, [
    ("spec", "spec", J.ptr_to(J.struct(_SpecWithOverrides, [
        ("overrides", "overrides", J.slice_of(J.struct(_ControllerOverride, [
            ("controller", "controller", J.STRING),
            ("clusters", "clusters", J.slice_of(J.struct(_ClusterOverride, [
                ("clusterName", "cluster_name", J.STRING),
                ("paths", "patches", J.slice_of(_OVERRIDE_PATCH))])))])))])))])


# ------------------------------------------------------------ unstructured access
def _nested(obj, *fields):
    """unstructured.NestedFieldNoCopy: (value, found); error if an intermediate is not a map."""
    v = obj
    for i, f in enumerate(fields):
        if not isinstance(v, dict):
            raise ObjectError(f"{'.'.join(fields[:i])} accessor error: {v!r} is of the type {type(v).__name__}, "
                              f"expected map[string]interface{{}}")
        if f not in v:
            return None, False
        v = v[f]
    return v, True


def _nested_string_map(obj, *fields) -> Optional[Dict[str, str]]:
    """GetAnnotations / GetLabels: NestedStringMap with every error read as nil."""
    try:
        m, found = _nested(obj, *fields)
    except ObjectError:
        return None
    if not found or not isinstance(m, dict) or not all(isinstance(x, str) for x in m.values()):
        return None
    return dict(m)


def get_annotations(obj) -> Optional[Dict[str, str]]:
    return _nested_string_map(obj, "metadata", "annotations")


def get_labels(obj) -> Optional[Dict[str, str]]:
    return _nested_string_map(obj, "metadata", "labels")


def _nested_string(obj, *fields) -> str:
    try:
        v, found = _nested(obj, *fields)
    except ObjectError:
        return ""
    return v if found and isinstance(v, str) else ""


def get_namespace(obj) -> str:
    return _nested_string(obj, "metadata", "namespace")


def get_name(obj) -> str:
    return _nested_string(obj, "metadata", "name")


def set_annotations(obj, annotations: Optional[Dict[str, str]]) -> None:
    """Unstructured.SetAnnotations."""
    if annotations is None:
        meta = obj.get("metadata")
        if isinstance(meta, dict):
            meta.pop("annotations", None)
        return
    _set_nested(obj, dict(annotations), "metadata", "annotations")


def _set_nested(obj, value, *fields) -> None:
    """unstructured.SetNestedField (creates missing intermediate maps)."""
    m = obj
    for i, f in enumerate(fields[:-1]):
        if f in m:
            if not isinstance(m[f], dict):
                raise ObjectError(f"value cannot be set because {'.'.join(fields[:i + 1])} is not a map[string]interface{{}}")
        else:
            m[f] = {}
        m = m[f]
    m[fields[-1]] = value


def split_dot_path(path: str, prefix=()) -> List[str]:
    """utilunstructured.SplitDotPath (unstructured.go:87-95)."""
    return list(prefix) + [p for p in path.split(".") if p != ""]


def to_slash_path(path: str) -> str:
    """utilunstructured.ToSlashPath (unstructured.go:97-99)."""
    return "/" + "/".join(split_dot_path(path))


def get_int64_from_path(obj, path: str, prefix=TEMPLATE_PATH) -> Optional[int]:
    """utilunstructured.GetInt64FromPath (unstructured.go:61-70): NestedInt64 under prefix."""
    fields = split_dot_path(path, prefix)
    try:
        v, found = _nested(obj, *fields)
    except ObjectError as e:
        raise ObjectError(f"cannot access {list(prefix)}: {e}") from None
    if not found:
        return None
    if isinstance(v, bool) or not isinstance(v, int) or not J.INT64_MIN <= v <= J.INT64_MAX:
        raise ObjectError(f"cannot access {list(prefix)}: {'.'.join(fields)} accessor error: {v!r} is of the type "
                          f"{type(v).__name__}, expected int64")
    return v


def f64_to_i64(x: float) -> int:
    """Go ``int64(f)`` on amd64 (CVTTSD2SI): truncation, out-of-range → MinInt64."""
    if x != x or not (-9.223372036854776e18 <= x < 9.223372036854776e18):
        return J.INT64_MIN
    return int(x)


# ------------------------------------------------------------ f2: SchedulingUnit packer
def matched_policy_key(obj, namespaced: bool) -> Optional[Tuple[str, str]]:
    """MatchedPolicyKey (scheduler/util.go:37-49) → (namespace, name) or None."""
    labels = get_labels(obj) or {}
    if PROPAGATION_POLICY_NAME_LABEL in labels and namespaced:
        return get_namespace(obj), labels[PROPAGATION_POLICY_NAME_LABEL]
    if CLUSTER_PROPAGATION_POLICY_NAME_LABEL in labels:
        return "", labels[CLUSTER_PROPAGATION_POLICY_NAME_LABEL]
    return None


def _get_template(obj):
    """getTemplate (schedulingunit.go:165-179): the template's PartialObjectMetadata."""
    tmpl, found = _nested(obj, *TEMPLATE_PATH)
    if found and not isinstance(tmpl, dict):
        raise ObjectError("error retrieving template: .spec.template accessor error: not a map")
    if not found:
        raise ObjectError("template not found")
    for k in ("apiVersion", "kind"):
        if k in tmpl and tmpl[k] is not None and not isinstance(tmpl[k], str):
            raise ObjectError("template cannot be converted from unstructured")
    meta = tmpl.get("metadata")
    if meta is None:
        return _ObjectMeta()
    if not isinstance(meta, dict):
        raise ObjectError("template cannot be converted from unstructured")
    out = _ObjectMeta()
    for k, attr in (("name", "name"), ("namespace", "namespace"), ("generateName", "generate_name")):
        v = meta.get(k)
        if v is not None and not isinstance(v, str):
            raise ObjectError("template cannot be converted from unstructured")
        setattr(out, attr, v or "")
    for k in ("labels", "annotations"):
        v = meta.get(k)
        if v is None:
            continue
        if not isinstance(v, dict) or not all(isinstance(x, str) for x in v.values()):
            raise ObjectError("template cannot be converted from unstructured")
        setattr(out, k, dict(v))
    return out


def _unmarshal_placements(obj) -> _ObjectWithPlacements:
    try:
        return J.decode(_OBJ_PLACEMENTS, J.from_unstructured(obj))
    except J.GoJSONError as e:
        raise ObjectError(str(e)) from None


def get_overrides(obj, controller: str) -> Dict[str, List[_OverridePatch]]:
    """util.GetOverrides (util/overrides.go:68-112)."""
    if obj is None:
        return {}
    try:
        o = J.decode(_OBJ_OVERRIDES, J.from_unstructured(obj))
    except J.GoJSONError as e:
        raise ObjectError(str(e)) from None
    if o.spec is None or o.spec.overrides is None:
        return {}
    clusters = None
    for co in o.spec.overrides:
        if co.controller == controller:
            clusters = co.clusters
            break
    if clusters is None:
        return {}
    out: Dict[str, List[_OverridePatch]] = {}
    for item in clusters:
        if item.cluster_name in out:
            raise ObjectError(f'cluster "{item.cluster_name}" appears more than once')
        for i, p in enumerate(item.patches or []):
            if p.path in INVALID_OVERRIDE_PATHS:
                raise ObjectError(f'override[{i}] for cluster "{item.cluster_name}" has an invalid path: {p.path}')
        out[item.cluster_name] = item.patches
    return out


def get_current_replicas(type_config: FederatedTypeConfig, obj) -> Dict[str, Optional[int]]:
    """getCurrentReplicasFromObject (schedulingunit.go:181-222)."""
    placements = _unmarshal_placements(obj)
    names: Set[str] = set()
    for p in placements.spec.placements or []:
        if p.controller == PREFIXED_GLOBAL_SCHEDULER_NAME:
            names = {c.name for c in (p.placement.clusters or [])}
            break
    overrides = get_overrides(obj, PREFIXED_GLOBAL_SCHEDULER_NAME)
    path = to_slash_path(type_config.replicas_spec)
    res: Dict[str, Optional[int]] = {}
    for cluster in names:
        res[cluster] = None
        for p in overrides.get(cluster) or []:
            if p.path == path and p.op in (OPERATION_REPLACE, ""):
                if not isinstance(p.value, float):
                    raise GoPanic(f"interface conversion: interface {{}} is {type(p.value).__name__}, not float64")
                res[cluster] = f64_to_i64(p.value)
                break
    return res


def _annotation(obj, key) -> Optional[str]:
    return (get_annotations(obj) or {}).get(key)


def _mode_from_object(obj) -> Optional[str]:  # schedulingunit.go:234-259
    v = _annotation(obj, SCHEDULING_MODE_ANNOTATION)
    return v if v in (T.SCHEDULING_MODE_DUPLICATE, T.SCHEDULING_MODE_DIVIDE) else None


def _sticky_from_object(obj) -> Optional[bool]:  # :278-304
    v = _annotation(obj, STICKY_CLUSTER_ANNOTATION)
    return {"true": True, "false": False}.get(v) if v is not None else None


def _json_annotation(obj, key, t):
    v = _annotation(obj, key)
    if v is None:
        return False, None
    try:
        return True, J.unmarshal(v, t)
    except J.GoJSONError:
        return False, None


def _placements_from_object(obj):  # the shared part of :465-668
    v = _annotation(obj, PLACEMENTS_ANNOTATIONS)
    if v is None:
        return None
    try:
        return J.unmarshal(v, J.slice_of(PLACEMENT)) or []
    except J.GoJSONError:
        return None


def scheduling_unit_for_fed_object(type_config: FederatedTypeConfig, obj: dict,
                                   policy: PropagationPolicy) -> T.SchedulingUnit:
    """schedulingUnitForFedObject (schedulingunit.go:38-163)."""
    template = _get_template(obj)
    spec = policy.spec

    # :224-232 policy mode, :48-58 annotation override and the Divide→Duplicate fallback
    mode = spec.scheduling_mode if spec.scheduling_mode in (T.SCHEDULING_MODE_DUPLICATE,
                                                            T.SCHEDULING_MODE_DIVIDE) else DEFAULT_SCHEDULING_MODE
    override = _mode_from_object(obj)
    if override is not None:
        mode = override
    desired = None
    if mode == T.SCHEDULING_MODE_DIVIDE and type_config.replicas_spec == "":
        mode = T.SCHEDULING_MODE_DUPLICATE
    if mode == T.SCHEDULING_MODE_DIVIDE:
        desired = get_int64_from_path(obj, type_config.replicas_spec, TEMPLATE_PATH)

    current = get_current_replicas(type_config, obj)
    su = T.SchedulingUnit(
        group=type_config.group, version=type_config.version, kind=type_config.kind,
        resource=type_config.plural_name, namespace=template.namespace, name=template.name,
        labels=template.labels, annotations=template.annotations, desired_replicas=desired,
        current_clusters=current, avoid_disruption=True)

    if spec.auto_migration is not None:  # :91-100, getAutoMigrationInfo :261-272
        info = None
        v = _annotation(obj, AUTO_MIGRATION_INFO_ANNOTATION)
        if v is not None:
            try:
                decoded = J.unmarshal(v, J.struct(_Capacity, [("estimatedCapacity", "ec", J.map_of(J.INT64))]))
            except J.GoJSONError as e:
                raise ObjectError(str(e)) from None
            info = decoded.ec if decoded.ec is not None else {}
        su.auto_migration = T.AutoMigrationSpec(info, spec.auto_migration.keep_unschedulable_replicas)
    if spec.replica_rescheduling is not None:
        su.avoid_disruption = spec.replica_rescheduling.avoid_disruption
    su.scheduling_mode = mode

    su.sticky_cluster = spec.sticky_cluster
    s = _sticky_from_object(obj)
    if s is not None:
        su.sticky_cluster = s

    su.cluster_selector = spec.cluster_selector
    ok, sel = _json_annotation(obj, CLUSTER_SELECTOR_ANNOTATIONS, J.map_of(J.STRING))
    if ok:
        su.cluster_selector = sel

    pols = spec.placements
    ann_pl = _placements_from_object(obj)
    # :626-668 ClusterNames
    su.cluster_names = None if pols is None else {p.cluster for p in pols}
    if ann_pl is not None:
        su.cluster_names = {p.cluster for p in ann_pl}
    # :510-564 MinReplicas (negative values invalidate the override)
    su.min_replicas = None if pols is None else {p.cluster: p.preferences.min_replicas for p in pols}
    if ann_pl is not None:
        m = {p.cluster: p.preferences.min_replicas for p in ann_pl}
        if all(x >= 0 for x in m.values()):
            su.min_replicas = m
    # :566-624 MaxReplicas
    su.max_replicas = None if pols is None else {p.cluster: p.preferences.max_replicas for p in pols
                                                 if p.preferences.max_replicas is not None}
    if ann_pl is not None:
        m = {p.cluster: p.preferences.max_replicas for p in ann_pl if p.preferences.max_replicas is not None}
        if all(x >= 0 for x in m.values()):
            su.max_replicas = m
    # :450-508 Weights
    su.weights = None if pols is None else {p.cluster: p.preferences.weight for p in pols
                                            if p.preferences.weight is not None}
    if ann_pl is not None:
        m = {p.cluster: p.preferences.weight for p in ann_pl if p.preferences.weight is not None}
        if all(x >= 0 for x in m.values()):
            su.weights = m

    # :336-377 Affinity
    su.affinity = None
    if spec.cluster_affinity:
        su.affinity = T.Affinity(T.ClusterAffinity(required=T.ClusterSelector(list(spec.cluster_affinity))))
    ok, aff = _json_annotation(obj, AFFINITY_ANNOTATIONS, AFFINITY)
    if ok:
        su.affinity = aff
    # :379-407 Tolerations ("null" decodes to a nil slice)
    su.tolerations = spec.tolerations
    v = _annotation(obj, TOLERATIONS_ANNOTATIONS)
    if v is not None:
        try:
            su.tolerations = J.unmarshal(v, J.slice_of(TOLERATION))
        except J.GoJSONError:
            pass
    # :409-448 MaxClusters
    su.max_clusters = spec.max_clusters
    v = _annotation(obj, MAX_CLUSTERS_ANNOTATIONS)
    if v is not None:
        n = J.atoi(v)
        if n is not None and n >= 0:
            su.max_clusters = n
    return su


@dataclass
class _Capacity:
    ec: Optional[Dict[str, int]] = None


# ------------------------------------------------------------ f3: result application
def _placement_list_json(pls: List[_PlacementWithController]):
    out = []
    for p in pls:
        pl = {}
        if p.placement.clusters:
            pl["clusters"] = [{"name": c.name} for c in p.placement.clusters]
        out.append({"controller": p.controller, "placement": pl})
    return out


def set_placement_cluster_names(obj, controller: str, clusters: Set[str]) -> bool:
    """util.SetPlacementClusterNames (util/placement.go:44-59) + SetPlacementNames (extensions_placements.go:81-103)."""
    po = _unmarshal_placements(obj)
    pls = list(po.spec.placements or [])
    idx = next((i for i, p in enumerate(pls) if p.controller == controller), -1)
    if len(clusters) == 0:
        if idx == -1:
            return False
        del pls[idx]
    else:
        if idx == -1:
            pls.append(_PlacementWithController(controller))
            idx = len(pls) - 1
        old = {c.name for c in (pls[idx].placement.clusters or [])}
        if old == set(clusters):
            return False
        pls[idx].placement.clusters = [_ClusterRef(n) for n in sorted(clusters, key=lambda s: s.encode())]
    # SetGenericPlacements: InterfaceToUnstructured of the typed list (nil → null)
    _set_nested(obj, _placement_list_json(pls) if po.spec.placements is not None or pls else None, *PLACEMENTS_PATH)
    return True


def override_update_needed(type_config: FederatedTypeConfig, overrides: Dict[str, List[_OverridePatch]],
                           result: Dict[str, int]) -> bool:
    """OverrideUpdateNeeded (scheduler/util.go:154-185)."""
    path = to_slash_path(type_config.replicas_spec)
    checked = 0
    for cluster, patches in overrides.items():
        for p in patches or []:
            if p.path != path:
                continue
            if not isinstance(p.value, float):
                return True
            if cluster not in result or f64_to_i64(p.value) != result[cluster]:
                return True
            checked += 1
    return checked != len(result)


def _update_overrides_map(type_config, overrides, replicas: Dict[str, int]) -> None:
    """updateOverridesMap (scheduler/util.go:109-152)."""
    path = to_slash_path(type_config.replicas_spec)
    for cluster in list(overrides):
        if cluster in replicas:
            continue
        patches = overrides[cluster] or []
        for i, p in enumerate(patches):
            if p.path == path:
                patches = patches[:i] + patches[i + 1:]
                if not patches:
                    del overrides[cluster]
                else:
                    overrides[cluster] = patches
                break
    for cluster, n in replicas.items():
        found = False
        for p in overrides.get(cluster) or []:
            if p.path == path:
                p.value = n
                found = True
                break
        if not found:
            overrides[cluster] = list(overrides.get(cluster) or []) + [_OverridePatch("", path, n)]


def _patch_json(p: _OverridePatch):
    d = {}
    if p.op:
        d["op"] = p.op
    d["path"] = p.path
    if p.value is not None:
        d["value"] = _roundtrip(p.value)
    return d


def _roundtrip(v):
    """json.Marshal → json.Unmarshal into interface{}: numbers become float64."""
    if isinstance(v, bool) or isinstance(v, str) or v is None:
        return v
    if isinstance(v, (int, float)):
        return float(v)
    if isinstance(v, dict):
        return {k: _roundtrip(x) for k, x in v.items()}
    return [_roundtrip(x) for x in v]


def set_overrides(obj, controller: str, overrides: Dict[str, List[_OverridePatch]]) -> None:
    """util.SetOverrides (util/overrides.go:114-169)."""
    for c in [c for c, p in overrides.items() if not p]:
        del overrides[c]
    try:
        o = J.decode(_OBJ_OVERRIDES, J.from_unstructured(obj))
    except J.GoJSONError as e:
        raise ObjectError(str(e)) from None
    if o.spec is None:
        raise GoPanic("invalid memory address or nil pointer dereference")
    cos = o.spec.overrides
    idx = next((i for i, co in enumerate(cos or []) if co.controller == controller), -1)
    if not overrides:
        if idx != -1:
            cos = cos[:idx] + cos[idx + 1:]
    else:
        if idx == -1:
            cos = list(cos or []) + [_ControllerOverride(controller)]
            idx = len(cos) - 1
        cos[idx].clusters = [_ClusterOverride(c, overrides[c]) for c in sorted(overrides, key=lambda s: s.encode())]
    if cos is None:
        value = None
    else:
        value = []
        for co in cos:
            clusters = None if co.clusters is None else [
                dict([("clusterName", c.cluster_name)] + ([("paths", [_patch_json(p) for p in c.patches])]
                                                         if c.patches else [])) for c in co.clusters]
            value.append({"controller": co.controller, "clusters": clusters})
    _set_nested(obj, value, *OVERRIDES_PATH)


def update_replicas_override(type_config: FederatedTypeConfig, obj, result: Dict[str, int]) -> bool:
    """UpdateReplicasOverride (scheduler/util.go:71-94)."""
    try:
        overrides = get_overrides(obj, PREFIXED_GLOBAL_SCHEDULER_NAME)
    except ObjectError as e:
        raise ObjectError(f"Error reading cluster overrides for {get_namespace(obj)}/{get_name(obj)}: {e}") from None
    if override_update_needed(type_config, overrides, result):
        _update_overrides_map(type_config, overrides, result)
        set_overrides(obj, PREFIXED_GLOBAL_SCHEDULER_NAME, overrides)
        return True
    return False


def result_state_of(type_config: FederatedTypeConfig, obj, index: Dict[str, int]):
    """One object's current state for kad_result_diff (include/kad_sched.h kad_result_state): whether the
    scheduler's placement exists and its clusters (the first placement of the controller, as
    GetOrCreatePlacement / DeletePlacement find it, extensions_placements.go:38-76), and its replicas-path
    override patches (util.GetOverrides, util/overrides.go:68-112) as (cluster position, int64(value), kind) —
    kind 1 for a value that is not a JSON number. Positions come from ``index`` (snapshot cluster name →
    position; -1 for other names). Raises ObjectError where applySchedulingResult would fail on the object."""
    po = _unmarshal_placements(obj)
    has, ids = False, []
    for p in po.spec.placements or []:
        if p.controller == PREFIXED_GLOBAL_SCHEDULER_NAME:
            has = True
            ids = [index.get(c.name, -1) for c in (p.placement.clusters or [])]
            break
    path = to_slash_path(type_config.replicas_spec)
    ov = []
    for cluster, patches in get_overrides(obj, PREFIXED_GLOBAL_SCHEDULER_NAME).items():
        for p in patches or []:
            if p.path != path:
                continue
            if isinstance(p.value, float):
                ov.append((index.get(cluster, -1), f64_to_i64(p.value), 0))
            else:
                ov.append((index.get(cluster, -1), 0, 1))
    return has, ids, ov


def result_states(type_config: FederatedTypeConfig, objs, names: List[str]) -> dict:
    """kad_result_state arrays for a batch of objects (their units in the same order); objects whose state
    cannot be read (ObjectError) get an empty state and are listed under ``errors``."""
    import numpy as np

    index = {n: i for i, n in enumerate(names)}
    has, p_off, p_id, o_off, o_id, o_val, o_kind, errors = [], [0], [], [0], [], [], [], []
    for w, obj in enumerate(objs):
        try:
            h, ids, ov = result_state_of(type_config, obj, index)
        except ObjectError:
            h, ids, ov = False, [], []
            errors.append(w)
        has.append(1 if h else 0)
        p_id += ids
        p_off.append(len(p_id))
        for cid, val, kind in ov:
            o_id.append(cid)
            o_val.append(val)
            o_kind.append(kind)
        o_off.append(len(o_id))
    return {"place_off": np.asarray(p_off, np.int32), "place_cluster": np.asarray(p_id, np.int32),
            "place_has": np.asarray(has, np.uint8), "ovr_off": np.asarray(o_off, np.int32),
            "ovr_cluster": np.asarray(o_id, np.int32), "ovr_value": np.asarray(o_val, np.int64),
            "ovr_kind": np.asarray(o_kind, np.uint8), "errors": errors}


def apply_scheduling_result(type_config: FederatedTypeConfig, obj: dict, result: T.ScheduleResult,
                            enable_follower_scheduling: bool, unschedulable_threshold_ns: Optional[int]) -> bool:
    """applySchedulingResult (scheduler.go:632-695): mutates ``obj``; True if anything changed."""
    modified = set_placement_cluster_names(obj, PREFIXED_GLOBAL_SCHEDULER_NAME, result.cluster_set())
    desired = {c: n for c, n in (result.suggested_clusters or {}).items() if n is not None}
    modified = update_replicas_override(type_config, obj, desired) or modified

    ann = get_annotations(obj)
    if ann is None:
        ann = {}
    changed = False
    val = ANNOTATION_VALUE_TRUE if enable_follower_scheduling else ANNOTATION_VALUE_FALSE
    if ann.get(ENABLE_FOLLOWER_SCHEDULING_ANNOTATION, "") != val:
        ann[ENABLE_FOLLOWER_SCHEDULING_ANNOTATION] = val
        changed = True
    if unschedulable_threshold_ns is None:
        if POD_UNSCHEDULABLE_THRESHOLD_ANNOTATION in ann:
            del ann[POD_UNSCHEDULABLE_THRESHOLD_ANNOTATION]
            changed = True
    else:
        s = duration_string(unschedulable_threshold_ns)
        if ann.get(POD_UNSCHEDULABLE_THRESHOLD_ANNOTATION, "") != s:
            ann[POD_UNSCHEDULABLE_THRESHOLD_ANNOTATION] = s
            changed = True
    if changed:
        set_annotations(obj, ann)
        modified = True
    return modified


def add_annotation(obj, key: str, value: str) -> bool:
    """annotation.AddAnnotation (util/annotation/annotation.go:70-97): True if the value changed."""
    if key == "":
        raise ObjectError("key is a empty string.")
    ann = get_annotations(obj)
    if ann is not None and ann.get(key) == value and key in ann:
        return False
    ann = ann if ann is not None else {}
    ann[key] = value
    set_annotations(obj, ann)
    return True


# ------------------------------------------------------------ time.Duration
_UNITS = (("h", 3600 * 10**9), ("m", 60 * 10**9), ("s", 10**9), ("ms", 10**6), ("us", 10**3), ("µs", 10**3),
          ("μs", 10**3), ("ns", 1))


def parse_duration(s: str) -> int:
    """time.ParseDuration → nanoseconds (ObjectError where Go returns an error)."""
    orig = s
    neg = False
    if s[:1] in ("-", "+"):
        neg = s[0] == "-"
        s = s[1:]
    if s == "0":
        return 0
    if s == "":
        raise ObjectError(f'time: invalid duration "{orig}"')
    total = 0
    while s:
        i = 0
        while i < len(s) and s[i].isdigit():
            i += 1
        ip, s = s[:i], s[i:]
        fp = ""
        if s[:1] == ".":
            j = 1
            while j < len(s) and s[j].isdigit():
                j += 1
            fp, s = s[1:j], s[j:]
        if ip == "" and fp == "":
            raise ObjectError(f'time: invalid duration "{orig}"')
        j = 0
        while j < len(s) and s[j] not in ".0123456789":
            j += 1
        u, s = s[:j], s[j:]
        unit = dict(_UNITS).get(u)
        if unit is None:
            raise ObjectError(f'time: {"missing" if u == "" else "unknown"} unit in duration "{orig}"')
        v = int(ip or "0") * unit
        if fp:
            # Go accumulates the fraction with float64 scale and truncates
            f, scale = 0, 1
            for ch in fp:
                if f > (1 << 63) // 10:
                    break
                f = f * 10 + int(ch)
                scale *= 10
            v += int(f * (unit / scale))
        total += v
        if total > (1 << 63) - 1:
            raise ObjectError(f'time: invalid duration "{orig}"')
    return -total if neg else total


def _fmt_frac(v: int, prec: int) -> Tuple[str, int]:
    digits = []
    printed = False
    for _ in range(prec):
        d = v % 10
        printed = printed or d != 0
        if printed:
            digits.append(str(d))
        v //= 10
    s = ("." + "".join(reversed(digits))) if printed else ""
    return s, v


def duration_string(d: int) -> str:
    """time.Duration.String."""
    if d == 0:
        return "0s"
    neg = d < 0
    u = -d if neg else d
    if u < 10**9:
        if u < 10**3:
            s = f"{u}ns"
        elif u < 10**6:
            f, w = _fmt_frac(u, 3)
            s = f"{w}{f}µs"
        else:
            f, w = _fmt_frac(u, 6)
            s = f"{w}{f}ms"
    else:
        f, w = _fmt_frac(u, 9)
        secs = w % 60
        w //= 60
        s = f"{secs}{f}s"
        if w > 0:
            mins = w % 60
            w //= 60
            s = f"{mins}m" + s
            if w > 0:
                s = f"{w}h" + s
    return ("-" + s) if neg else s


# ------------------------------------------------------------ f4: scheduling-trigger bytes
_KNOWN_SCHEDULING_ANNOTATIONS = frozenset({
    SCHEDULING_MODE_ANNOTATION, STICKY_CLUSTER_ANNOTATION, TOLERATIONS_ANNOTATIONS, PLACEMENTS_ANNOTATIONS,
    CLUSTER_SELECTOR_ANNOTATIONS, AFFINITY_ANNOTATIONS, MAX_CLUSTERS_ANNOTATIONS, FOLLOWS_OBJECT_ANNOTATION})

_RESOURCE_REQUEST_JSON = '{"millicpu":0,"memory":0,"ephemeralStorage":0,"scalarResources":null}'


def _kv_list(d: Optional[Dict[str, str]]) -> str:
    """sortMap of a string map, encoded: [{"key":k,"value":v},...] (keys unique ⇒ a total order)."""
    es = J.encode_string
    return "[" + ",".join('{"key":' + es(k) + ',"value":' + es(d[k]) + "}"
                          for k in sorted(d or {}, key=lambda s: s.encode("utf-8", "surrogatepass"))) + "]"


def get_replica_count(type_config: FederatedTypeConfig, obj) -> int:
    """getReplicaCount (schedulingtriggers.go:171-186)."""
    if len(type_config.replicas_spec) == 0:
        return 0
    v = get_int64_from_path(obj, type_config.replicas_spec, TEMPLATE_PATH)
    return 0 if v is None else v


def _taint_less(l: T.Taint, r: T.Taint) -> bool:  # schedulingtriggers.go:215-227 (effect branch compares values)
    if l.key != r.key:
        return l.key.encode() < r.key.encode()
    if l.value != r.value:
        return l.value.encode() < r.value.encode()
    if l.effect != r.effect:
        return l.value.encode() < r.value.encode()
    return False


def _api_less(l: T.APIResource, r: T.APIResource) -> bool:  # schedulingtriggers.go:241-257 (Kind branch is !=)
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


def _taint_json(t: T.Taint) -> str:
    es = J.encode_string
    return '{"key":' + es(t.key) + (',"value":' + es(t.value) if t.value else "") + ',"effect":' + es(t.effect) + "}"


def _api_json(a: T.APIResource) -> str:
    es = J.encode_string
    return ("{" + ('"group":' + es(a.group) + "," if a.group else "") + '"version":' + es(a.version) + ',"kind":'
            + es(a.kind) + ',"pluralName":' + es(a.plural_name) + ',"scope":' + es(a.scope) + "}")


def trigger_suffix(clusters: List[T.FederatedCluster]) -> bytes:
    """The cluster part of the trigger JSON, shared by every object of one pass.

    ``getClusterLabels`` / ``getClusterTaints`` / ``getClusterAPIResourceTypes``
    (schedulingtriggers.go:193-262) encoded as json.Marshal would, from the
    ``clusterLabels`` value to the closing brace. Later clusters with a
    duplicate name replace earlier ones (the reference builds maps by name).
    """
    by_name: Dict[str, T.FederatedCluster] = {}
    for c in clusters:
        by_name[c.name] = c
    names = sorted(by_name, key=lambda s: s.encode("utf-8", "surrogatepass"))
    es = J.encode_string
    labels = ",".join('{"key":' + es(n) + ',"value":' + _kv_list(by_name[n].labels) + "}" for n in names)
    taint_parts = []
    api_parts = []
    for n in names:
        c = by_name[n]
        taints = [T.Taint(t.key, t.value, t.effect) for t in (c.taints or [])]
        sort_slice(taints, _taint_less)
        taint_parts.append('{"key":' + es(n) + ',"value":[' + ",".join(_taint_json(t) for t in taints) + "]}")
        apis = list(c.api_resource_types or [])
        sort_slice(apis, _api_less)
        api_parts.append('{"key":' + es(n) + ',"value":[' + ",".join(_api_json(a) for a in apis) + "]}")
    s = ("[" + labels + '],"clusterTaints":[' + ",".join(taint_parts) + '],"clusterAPIResourceTypes":['
         + ",".join(api_parts) + "]}")
    return s.encode("utf-8")  # encode_string already turned unpaired surrogates into \ufffd


def trigger_prefix(type_config: FederatedTypeConfig, obj: dict, policy: Optional[PropagationPolicy]) -> bytes:
    """The per-object part of the trigger JSON, up to and including ``"clusterLabels":``.

    ``computeSchedulingTriggerHash`` (schedulingtriggers.go:106-134): scheduling
    annotations (sorted), replica count, the (always empty) resource request,
    the auto-migration annotation when the policy enables auto migration, and
    the policy's name and generation.
    """
    ann = get_annotations(obj) or {}
    sched = {k: v for k, v in ann.items() if k in _KNOWN_SCHEDULING_ANNOTATIONS}
    replicas = get_replica_count(type_config, obj)
    parts = ['{"schedulingAnnotations":', _kv_list(sched), ',"replicaCount":', str(replicas),
             ',"resourceRequest":', _RESOURCE_REQUEST_JSON]
    name, gen = "", 0
    if policy is not None:
        name, gen = policy.name, policy.generation
        if policy.spec.auto_migration is not None and AUTO_MIGRATION_INFO_ANNOTATION in ann:
            parts += [',"autoMigrationInfo":', J.encode_string(ann[AUTO_MIGRATION_INFO_ANNOTATION])]
    parts += [',"policyName":', J.encode_string(name), ',"policyGeneration":', str(gen), ',"clusterLabels":']
    return "".join(parts).encode("utf-8")


def format_trigger_hash(h: int) -> str:
    """strconv.FormatInt(int64(hash.Sum32()), 10)."""
    return str(int(h) & 0xFFFFFFFF)

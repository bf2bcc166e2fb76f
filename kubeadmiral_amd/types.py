"""Object model of the scheduling hot path, mirroring the reference Go types.

This is the `SchedulingUnit`-in / `ScheduleResult`-out data contract of
KubeAdmiral's scheduler framework, restated as Python dataclasses so that the
host side (packer + batch scheduler) and the tests speak the reference's
vocabulary:

* ``SchedulingUnit``      ← ``pkg/controllers/scheduler/framework/types.go:33-69``
* ``Resource``            ← ``pkg/controllers/scheduler/framework/util.go:71-77``
* ``AutoMigrationSpec``   ← ``framework/types.go:71-80``
* ``Affinity`` & co.      ← ``framework/types.go:82-121``
* ``FederatedCluster``    ← ``pkg/apis/core/v1alpha1/types_federatedcluster.go:40-143``
  (only the fields the scheduling path reads: name, labels, taints,
  APIResourceTypes, Resources.{Allocatable,Available})
* ``APIResource``         ← ``pkg/apis/core/v1alpha1/types_federatedtypeconfig.go:165-182``
* ``ClusterSelectorTerm`` ← ``pkg/apis/core/v1alpha1/types_common.go:50-77``
* ``Taint``/``Toleration``← ``k8s.io/api/core/v1`` v0.26.6
* ``ScheduleResult``      ← ``pkg/controllers/scheduler/core/generic_scheduler.go:48-53``

Go ``nil`` is represented by ``None`` wherever the reference distinguishes nil
from empty (pointers, nil slices / maps whose nil-ness changes behaviour, e.g.
``RequiredDuringSchedulingIgnoredDuringExecution`` or
``ClusterSelectorTerm.MatchExpressions``).

JSON: ``FederatedCluster`` and the affinity / toleration types use the
reference's JSON tags; ``SchedulingUnit`` (an in-memory struct without JSON tags
in the reference) uses its Go field names.
"""

from __future__ import annotations

import hashlib
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Set, Tuple

# pkg/apis/core/v1alpha1/types_propagationpolicy.go (SchedulingMode constants)
SCHEDULING_MODE_DUPLICATE = "Duplicate"
SCHEDULING_MODE_DIVIDE = "Divide"

# k8s.io/api/core/v1 taint effects / toleration operators
TAINT_NO_SCHEDULE = "NoSchedule"
TAINT_PREFER_NO_SCHEDULE = "PreferNoSchedule"
TAINT_NO_EXECUTE = "NoExecute"
TOLERATION_OP_EQUAL = "Equal"
TOLERATION_OP_EXISTS = "Exists"

# pkg/apis/core/v1alpha1/types_common.go:66-77
OP_IN = "In"
OP_NOT_IN = "NotIn"
OP_EXISTS = "Exists"
OP_DOES_NOT_EXIST = "DoesNotExist"
OP_GT = "Gt"
OP_LT = "Lt"


@dataclass
class Taint:
    key: str = ""
    value: str = ""
    effect: str = ""

    def to_json(self):
        d = {"key": self.key, "effect": self.effect}
        if self.value:
            d["value"] = self.value
        return d

    @staticmethod
    def from_json(d):
        return Taint(d.get("key", ""), d.get("value", ""), d.get("effect", ""))


@dataclass
class Toleration:
    key: str = ""
    operator: str = ""
    value: str = ""
    effect: str = ""
    toleration_seconds: Optional[int] = None  # not read by the scheduling path

    def to_json(self):
        d = {}
        for k in ("key", "operator", "value", "effect"):
            v = getattr(self, k)
            if v:
                d[k] = v
        if self.toleration_seconds is not None:
            d["tolerationSeconds"] = self.toleration_seconds
        return d

    @staticmethod
    def from_json(d):
        return Toleration(d.get("key", ""), d.get("operator", ""), d.get("value", ""), d.get("effect", ""),
                          d.get("tolerationSeconds"))


@dataclass
class APIResource:
    group: str = ""
    version: str = ""
    kind: str = ""
    plural_name: str = ""   # read by the scheduling-trigger hash only
    scope: str = ""

    def to_json(self):
        d = {"group": self.group, "version": self.version, "kind": self.kind}
        if self.plural_name:
            d["pluralName"] = self.plural_name
        if self.scope:
            d["scope"] = self.scope
        return d

    @staticmethod
    def from_json(d):
        return APIResource(d.get("group", ""), d.get("version", ""), d.get("kind", ""), d.get("pluralName", ""),
                           d.get("scope", ""))


@dataclass
class FederatedCluster:
    """The parts of ``FederatedCluster`` read by the scheduling path.

    ``allocatable`` / ``available`` are ``corev1.ResourceList`` values: maps of
    resource name → Kubernetes quantity string (e.g. ``"1500m"``, ``"16Gi"``).
    Dict order stands in for Go map order where the reference is map-order
    dependent (only on inconsistent input).
    """

    name: str = ""
    labels: Optional[Dict[str, str]] = None
    taints: List[Taint] = field(default_factory=list)
    api_resource_types: List[APIResource] = field(default_factory=list)
    allocatable: Optional[Dict[str, str]] = None
    available: Optional[Dict[str, str]] = None
    resource_version: str = ""  # metadata.resourceVersion ("" = unknown: content is compared instead)

    def to_json(self):
        meta = {"name": self.name}
        if self.resource_version:
            meta["resourceVersion"] = self.resource_version
        if self.labels is not None:
            meta["labels"] = dict(self.labels)
        spec = {}
        if self.taints:
            spec["taints"] = [t.to_json() for t in self.taints]
        status = {}
        res = {}
        if self.allocatable is not None:
            res["allocatable"] = dict(self.allocatable)
        if self.available is not None:
            res["available"] = dict(self.available)
        if res:
            status["resources"] = res
        if self.api_resource_types:
            status["apiResourceTypes"] = [r.to_json() for r in self.api_resource_types]
        return {"metadata": meta, "spec": spec, "status": status}

    @staticmethod
    def from_json(d):
        meta = d.get("metadata", {}) or {}
        spec = d.get("spec", {}) or {}
        status = d.get("status", {}) or {}
        res = status.get("resources", {}) or {}
        return FederatedCluster(
            name=meta.get("name", ""),
            labels=meta.get("labels"),
            taints=[Taint.from_json(t) for t in (spec.get("taints") or [])],
            api_resource_types=[APIResource.from_json(r) for r in (status.get("apiResourceTypes") or [])],
            allocatable=res.get("allocatable"),
            available=res.get("available"),
            resource_version=meta.get("resourceVersion", "") or "",
        )


def cluster_key(c: FederatedCluster):
    """What identifies a cluster object's content: (name, resourceVersion) when it carries one — the API
    server bumps resourceVersion on every change, and informer-cache objects are never mutated in place —
    else the whole content (so a list whose elements were replaced or edited in place is still seen)."""
    return ("rv", c.name, c.resource_version) if c.resource_version else repr(c)


def clusters_fingerprint(clusters: Sequence[FederatedCluster]) -> bytes:
    """Content fingerprint of a cluster list, in order (the order is part of the snapshot)."""
    h = hashlib.blake2b(digest_size=16)
    for c in clusters:
        h.update(repr(cluster_key(c)).encode())
        h.update(b"\0")
    return h.digest()


@dataclass
class ClusterSelectorRequirement:
    key: str = ""
    operator: str = ""
    values: Optional[List[str]] = None

    def to_json(self):
        d = {"key": self.key, "operator": self.operator}
        if self.values is not None:
            d["values"] = list(self.values)
        return d

    @staticmethod
    def from_json(d):
        return ClusterSelectorRequirement(d.get("key", ""), d.get("operator", ""), d.get("values"))


def _reqs_to_json(reqs):
    return None if reqs is None else [r.to_json() for r in reqs]


def _reqs_from_json(v):
    return None if v is None else [ClusterSelectorRequirement.from_json(r) for r in v]


@dataclass
class ClusterSelectorTerm:
    match_expressions: Optional[List[ClusterSelectorRequirement]] = None
    match_fields: Optional[List[ClusterSelectorRequirement]] = None

    def to_json(self):
        d = {}
        if self.match_expressions is not None:
            d["matchExpressions"] = _reqs_to_json(self.match_expressions)
        if self.match_fields is not None:
            d["matchFields"] = _reqs_to_json(self.match_fields)
        return d

    @staticmethod
    def from_json(d):
        return ClusterSelectorTerm(_reqs_from_json(d.get("matchExpressions")), _reqs_from_json(d.get("matchFields")))


@dataclass
class ClusterSelector:
    cluster_selector_terms: Optional[List[ClusterSelectorTerm]] = None

    def to_json(self):
        return {"clusterSelectorTerms": None if self.cluster_selector_terms is None
                else [t.to_json() for t in self.cluster_selector_terms]}

    @staticmethod
    def from_json(d):
        terms = d.get("clusterSelectorTerms")
        return ClusterSelector(None if terms is None else [ClusterSelectorTerm.from_json(t) for t in terms])


@dataclass
class PreferredSchedulingTerm:
    weight: int = 0
    preference: ClusterSelectorTerm = field(default_factory=ClusterSelectorTerm)

    def to_json(self):
        return {"weight": self.weight, "preference": self.preference.to_json()}

    @staticmethod
    def from_json(d):
        return PreferredSchedulingTerm(int(d.get("weight", 0)), ClusterSelectorTerm.from_json(d.get("preference", {}) or {}))


@dataclass
class ClusterAffinity:
    required: Optional[ClusterSelector] = None
    preferred: Optional[List[PreferredSchedulingTerm]] = None

    def to_json(self):
        d = {}
        if self.required is not None:
            d["requiredDuringSchedulingIgnoredDuringExecution"] = self.required.to_json()
        if self.preferred is not None:
            d["preferredDuringSchedulingIgnoredDuringExecution"] = [p.to_json() for p in self.preferred]
        return d

    @staticmethod
    def from_json(d):
        req = d.get("requiredDuringSchedulingIgnoredDuringExecution")
        pref = d.get("preferredDuringSchedulingIgnoredDuringExecution")
        return ClusterAffinity(
            None if req is None else ClusterSelector.from_json(req),
            None if pref is None else [PreferredSchedulingTerm.from_json(p) for p in pref],
        )


@dataclass
class Affinity:
    cluster_affinity: Optional[ClusterAffinity] = None

    def to_json(self):
        d = {}
        if self.cluster_affinity is not None:
            d["clusterAffinity"] = self.cluster_affinity.to_json()
        return d

    @staticmethod
    def from_json(d):
        ca = d.get("clusterAffinity")
        return Affinity(None if ca is None else ClusterAffinity.from_json(ca))


@dataclass
class Resource:
    """framework.Resource (util.go:71-77): integer milli-CPU / bytes / scalars."""

    milli_cpu: int = 0
    memory: int = 0
    ephemeral_storage: int = 0
    scalar_resources: Optional[Dict[str, int]] = None

    def to_json(self):
        d = {"millicpu": self.milli_cpu, "memory": self.memory, "ephemeralStorage": self.ephemeral_storage}
        if self.scalar_resources is not None:
            d["scalarResources"] = dict(self.scalar_resources)
        return d

    @staticmethod
    def from_json(d):
        d = d or {}
        return Resource(int(d.get("millicpu", 0)), int(d.get("memory", 0)), int(d.get("ephemeralStorage", 0)),
                        d.get("scalarResources"))


@dataclass
class AutoMigrationSpec:
    estimated_capacity: Optional[Dict[str, int]] = None  # Info.EstimatedCapacity; None ⇔ Info == nil
    keep_unschedulable_replicas: bool = False

    def to_json(self):
        d = {"KeepUnschedulableReplicas": self.keep_unschedulable_replicas}
        if self.estimated_capacity is not None:
            d["Info"] = {"estimatedCapacity": dict(self.estimated_capacity)}
        return d

    @staticmethod
    def from_json(d):
        info = d.get("Info")
        ec = None if info is None else dict(info.get("estimatedCapacity") or {})
        return AutoMigrationSpec(ec, bool(d.get("KeepUnschedulableReplicas", False)))


@dataclass
class SchedulingUnit:
    """framework.SchedulingUnit (types.go:33-69)."""

    group: str = ""
    version: str = ""
    kind: str = ""
    resource: str = ""
    namespace: str = ""
    name: str = ""
    labels: Optional[Dict[str, str]] = None
    annotations: Optional[Dict[str, str]] = None
    desired_replicas: Optional[int] = None
    resource_request: Resource = field(default_factory=Resource)
    current_clusters: Optional[Dict[str, Optional[int]]] = None
    auto_migration: Optional[AutoMigrationSpec] = None
    scheduling_mode: str = ""
    sticky_cluster: bool = False
    avoid_disruption: bool = False
    cluster_selector: Optional[Dict[str, str]] = None
    cluster_names: Optional[Set[str]] = None
    affinity: Optional[Affinity] = None
    tolerations: Optional[List[Toleration]] = None
    max_clusters: Optional[int] = None
    min_replicas: Optional[Dict[str, int]] = None
    max_replicas: Optional[Dict[str, int]] = None
    weights: Optional[Dict[str, int]] = None

    def key(self) -> str:
        """SchedulingUnit.Key() (types.go:123-128)."""
        if len(self.namespace) > 0:
            return self.namespace + "/" + self.name
        return self.name

    def to_json(self):
        d = {
            "GroupVersion": {"Group": self.group, "Version": self.version},
            "Kind": self.kind,
            "Resource": self.resource,
            "Namespace": self.namespace,
            "Name": self.name,
            "ResourceRequest": self.resource_request.to_json(),
            "SchedulingMode": self.scheduling_mode,
            "StickyCluster": self.sticky_cluster,
            "AvoidDisruption": self.avoid_disruption,
        }
        opt = {
            "Labels": self.labels, "Annotations": self.annotations, "DesiredReplicas": self.desired_replicas,
            "CurrentClusters": self.current_clusters, "ClusterSelector": self.cluster_selector,
            "MaxClusters": self.max_clusters, "MinReplicas": self.min_replicas,
            "MaxReplicas": self.max_replicas, "Weights": self.weights,
        }
        for k, v in opt.items():
            if v is not None:
                d[k] = v
        if self.cluster_names is not None:
            d["ClusterNames"] = sorted(self.cluster_names)
        if self.auto_migration is not None:
            d["AutoMigration"] = self.auto_migration.to_json()
        if self.affinity is not None:
            d["Affinity"] = self.affinity.to_json()
        if self.tolerations is not None:
            d["Tolerations"] = [t.to_json() for t in self.tolerations]
        return d

    @staticmethod
    def from_json(d):
        gv = d.get("GroupVersion", {}) or {}
        am = d.get("AutoMigration")
        aff = d.get("Affinity")
        tols = d.get("Tolerations")
        cn = d.get("ClusterNames")
        return SchedulingUnit(
            group=gv.get("Group", ""), version=gv.get("Version", ""), kind=d.get("Kind", ""),
            resource=d.get("Resource", ""), namespace=d.get("Namespace", ""), name=d.get("Name", ""),
            labels=d.get("Labels"), annotations=d.get("Annotations"),
            desired_replicas=d.get("DesiredReplicas"),
            resource_request=Resource.from_json(d.get("ResourceRequest")),
            current_clusters=d.get("CurrentClusters"),
            auto_migration=None if am is None else AutoMigrationSpec.from_json(am),
            scheduling_mode=d.get("SchedulingMode", ""),
            sticky_cluster=bool(d.get("StickyCluster", False)),
            avoid_disruption=bool(d.get("AvoidDisruption", False)),
            cluster_selector=d.get("ClusterSelector"),
            cluster_names=None if cn is None else set(cn),
            affinity=None if aff is None else Affinity.from_json(aff),
            tolerations=None if tols is None else [Toleration.from_json(t) for t in tols],
            max_clusters=d.get("MaxClusters"),
            min_replicas=d.get("MinReplicas"), max_replicas=d.get("MaxReplicas"), weights=d.get("Weights"),
        )


@dataclass
class ScheduleResult:
    """core.ScheduleResult (generic_scheduler.go:48-53).

    ``suggested_clusters`` is ``None`` for the Go nil map (no feasible cluster),
    otherwise a dict cluster-name → replicas (``None`` = Go nil pointer, i.e.
    Duplicate mode).
    """

    suggested_clusters: Optional[Dict[str, Optional[int]]] = None

    def cluster_set(self) -> Set[str]:
        return set(self.suggested_clusters or {})


class ScheduleError(Exception):
    """Error returned by Schedule (generic_scheduler.go:108,118,125,141).

    ``stage`` is one of ``"score"``, ``"select"``, ``"replicas"`` — parity is
    on the error class per workload, not on message text.
    """

    def __init__(self, stage: str, msg: str = ""):
        super().__init__(f"failed to {stage}: {msg}")
        self.stage = stage


GroupVersionKind = Tuple[str, str, str]

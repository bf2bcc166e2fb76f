"""Deterministic synthetic workloads (BASELINE.json configs).

There is no cluster or dataset here, so every benchmark and parity run uses
seeded synthetic FederatedCluster snapshots and SchedulingUnit batches with the
shapes and distributions of SURVEY.md §8(d):

* ``c1`` 1k Deployment units × 16 clusters, default plugins, Divide (seed 0xC1)
* ``c2`` 100k × 256: Fit + Taint + Affinity filters, LeastAllocated, MaxCluster, Duplicate (0xC2)
* ``c3`` 1M × 1k, same generator as c2 (0xC3)
* ``c4`` 1M Divide units × 512 clusters: weights, min/max, capacity caps (0xC4)
* ``c5`` 100k × 10k adversarial filters (0xC5)
* ``fuzz`` small batches exercising every branch and edge case of the path

``scale`` shrinks W (and C for c5) so tests can run the same generators on CPU.
"""

from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import json

import numpy as np

from . import framework as F
from . import k8s
from . import types as T

GI = 1 << 30
TI = 1 << 40
EFFECTS = [T.TAINT_NO_SCHEDULE, T.TAINT_PREFER_NO_SCHEDULE, T.TAINT_NO_EXECUTE]
GVKS = [("apps", "v1", "Deployment"), ("apps", "v1", "StatefulSet"), ("apps", "v1", "DaemonSet"),
        ("batch", "v1", "Job"), ("", "v1", "ConfigMap"), ("", "v1", "Service"), ("batch", "v1", "CronJob"),
        ("networking.k8s.io", "v1", "Ingress")]

SEEDS = {"c1": 0xC1, "c2": 0xC2, "c3": 0xC3, "c4": 0xC4, "c5": 0xC5, "c3r": 0xC3, "c3p": 0xC3}
SIZES = {"c1": (1000, 16), "c2": (100_000, 256), "c3": (1_000_000, 1000), "c4": (1_000_000, 512),
         "c5": (100_000, 10_000), "c3r": (1_000_000, 1000), "c3p": (1_000_000, 1000)}


def production_resources(clusters, rng: np.random.Generator, p_over: float = 0.015, p_empty: float = 0.005):
    """``clusters`` (in place) with the resource shapes aggregateResources
    (pkg/controllers/federatedcluster/util.go:178-214) reports for real member clusters: nodes that are
    Unschedulable, NotReady or carry a NoSchedule / NoExecute taint (isNodeSchedulable, :114-131) are left out
    of allocatable, while every non-terminal pod's requests are still subtracted from available (:199-210) —
    * a fraction ``p_over`` of clusters whose pods on left-out nodes push cpu and / or memory available
      below 0 (used = allocatable - available above allocatable by up to 30 %);
    * a fraction ``p_empty`` whose every node is left out: empty Allocatable and Available lists
      (allocatable 0, used 0 — pods subtract only from resources present, :203-207).
    Returns the indices of the two groups."""
    C = len(clusters)
    u = rng.random(C)
    over = np.nonzero(u < p_over)[0]
    empty = np.nonzero((u >= p_over) & (u < p_over + p_empty))[0]
    for c in over:
        cl = clusters[int(c)]
        which = int(rng.integers(1, 4))  # 1 cpu, 2 memory, 3 both
        if which & 1 and "cpu" in (cl.allocatable or {}):
            ac = k8s.milli_value(k8s.quantity(cl.allocatable["cpu"]))
            cl.available = dict(cl.available or {}, cpu=f"{-int(ac * rng.uniform(0.001, 0.3))}m")
        if which & 2 and "memory" in (cl.allocatable or {}):
            am = k8s.value(k8s.quantity(cl.allocatable["memory"]))
            cl.available = dict(cl.available or {}, memory=str(-int(am * rng.uniform(0.001, 0.3))))
    for c in empty:
        clusters[int(c)].allocatable = {}
        clusters[int(c)].available = {}
    return over, empty

# ------------------------------------------------------- production-shaped API-resource lists
# What a member cluster's discovery returns (kube 1.26 built-ins and commonly installed operators' CRDs), as
# FederatedCluster.Status.APIResourceTypes holds it: updateClusterAPIResources
# (pkg/controllers/federatedcluster/clusterstatus.go:204-268) keeps every resource of every group version
# whose name has no "/" (subresources skipped, :239-241) and sorts the list by Kind (:262-264). The same Kind
# appears under several group versions (autoscaling/v1 and v2 HorizontalPodAutoscaler, core and events.k8s.io
# Event, ...). Go's sort.Slice is unstable, so the order among equal Kinds is pdqsort's; here it is discovery
# order (a stable sort) — the order only decides the snapshot's GVK ids, never a scheduling result.
_BUILTIN_API = [
    ("", "v1", ["Binding", "ComponentStatus", "ConfigMap", "Endpoints", "Event", "LimitRange", "Namespace", "Node",
                "PersistentVolumeClaim", "PersistentVolume", "Pod", "PodTemplate", "ReplicationController",
                "ResourceQuota", "Secret", "ServiceAccount", "Service"]),
    ("admissionregistration.k8s.io", "v1", ["MutatingWebhookConfiguration", "ValidatingWebhookConfiguration"]),
    ("apiextensions.k8s.io", "v1", ["CustomResourceDefinition"]),
    ("apiregistration.k8s.io", "v1", ["APIService"]),
    ("apps", "v1", ["ControllerRevision", "DaemonSet", "Deployment", "ReplicaSet", "StatefulSet"]),
    ("authentication.k8s.io", "v1", ["TokenReview"]),
    ("authorization.k8s.io", "v1", ["LocalSubjectAccessReview", "SelfSubjectAccessReview", "SelfSubjectRulesReview",
                                    "SubjectAccessReview"]),
    ("autoscaling", "v1", ["HorizontalPodAutoscaler"]),
    ("autoscaling", "v2", ["HorizontalPodAutoscaler"]),
    ("batch", "v1", ["CronJob", "Job"]),
    ("certificates.k8s.io", "v1", ["CertificateSigningRequest"]),
    ("coordination.k8s.io", "v1", ["Lease"]),
    ("discovery.k8s.io", "v1", ["EndpointSlice"]),
    ("events.k8s.io", "v1", ["Event"]),
    ("flowcontrol.apiserver.k8s.io", "v1beta2", ["FlowSchema", "PriorityLevelConfiguration"]),
    ("flowcontrol.apiserver.k8s.io", "v1beta3", ["FlowSchema", "PriorityLevelConfiguration"]),
    ("networking.k8s.io", "v1", ["IngressClass", "Ingress", "NetworkPolicy"]),
    ("node.k8s.io", "v1", ["RuntimeClass"]),
    ("policy", "v1", ["PodDisruptionBudget"]),
    ("rbac.authorization.k8s.io", "v1", ["ClusterRoleBinding", "ClusterRole", "RoleBinding", "Role"]),
    ("scheduling.k8s.io", "v1", ["PriorityClass"]),
    ("storage.k8s.io", "v1", ["CSIDriver", "CSINode", "CSIStorageCapacity", "StorageClass", "VolumeAttachment"]),
    ("metrics.k8s.io", "v1beta1", ["NodeMetrics", "PodMetrics"]),
]
# operators: a cluster has each one's whole group (p = 0.9), so some clusters lack a kind (API-resource gaps)
_OPERATOR_API = [
    ("cert-manager.io", "v1", ["Certificate", "CertificateRequest", "ClusterIssuer", "Issuer"]),
    ("acme.cert-manager.io", "v1", ["Challenge", "Order"]),
    ("monitoring.coreos.com", "v1", ["Alertmanager", "PodMonitor", "Probe", "Prometheus", "PrometheusRule",
                                     "ServiceMonitor", "ThanosRuler"]),
    ("monitoring.coreos.com", "v1alpha1", ["AlertmanagerConfig"]),
    ("argoproj.io", "v1alpha1", ["AnalysisRun", "AnalysisTemplate", "ClusterAnalysisTemplate", "Experiment",
                                 "Rollout"]),
    ("apps.kruise.io", "v1alpha1", ["AdvancedCronJob", "BroadcastJob", "CloneSet", "DaemonSet", "ImagePullJob",
                                    "NodeImage", "ResourceDistribution", "SidecarSet", "UnitedDeployment",
                                    "WorkloadSpread"]),
    ("apps.kruise.io", "v1beta1", ["StatefulSet"]),
    ("snapshot.storage.k8s.io", "v1", ["VolumeSnapshotClass", "VolumeSnapshotContent", "VolumeSnapshot"]),
    ("networking.istio.io", "v1beta1", ["DestinationRule", "Gateway", "ServiceEntry", "Sidecar", "VirtualService",
                                        "WorkloadEntry", "WorkloadGroup"]),
    ("security.istio.io", "v1beta1", ["AuthorizationPolicy", "PeerAuthentication", "RequestAuthentication"]),
    ("keda.sh", "v1alpha1", ["ClusterTriggerAuthentication", "ScaledJob", "ScaledObject", "TriggerAuthentication"]),
    ("velero.io", "v1", ["Backup", "BackupStorageLocation", "DeleteBackupRequest", "DownloadRequest",
                         "PodVolumeBackup", "PodVolumeRestore", "Restore", "Schedule", "ServerStatusRequest",
                         "VolumeSnapshotLocation"]),
]
# workload kinds a federation schedules (FederatedTypeConfig targets): the c3r units' GVKs and their shares
C3R_WORKLOADS = [(("apps", "v1", "Deployment"), 0.40), (("apps", "v1", "StatefulSet"), 0.15),
                 (("apps", "v1", "DaemonSet"), 0.10), (("batch", "v1", "Job"), 0.10),
                 (("batch", "v1", "CronJob"), 0.05), (("", "v1", "Service"), 0.10),
                 (("argoproj.io", "v1alpha1", "Rollout"), 0.05), (("apps.kruise.io", "v1alpha1", "CloneSet"), 0.05)]


def discovery_api_resources(rng: np.random.Generator, C: int, n_extra_crds: int = 40, p_operator: float = 0.9,
                            p_builtin: float = 1.0):
    """C clusters' ``APIResourceTypes`` shaped like updateClusterAPIResources' output (module comment above):
    the ~60 built-in resources (each with probability ``p_builtin``: 1 on real clusters), each operator's
    group with probability ``p_operator``, and ``n_extra_crds`` single-kind CRDs with probability
    ``p_operator`` each; Kind-sorted. About 150 entries per cluster (3 GVK words)."""
    def res(groups):
        out = []
        for g, v, kinds in groups:
            for k in kinds:
                out.append(T.APIResource(g, v, k, k.lower() + "s", "Namespaced"))
        return out

    builtin = res(_BUILTIN_API)
    ops = [res([grp]) for grp in _OPERATOR_API]
    extra = [T.APIResource(f"crd{i // 4}.example.com", "v1", f"Custom{i:02d}", f"custom{i:02d}s", "Namespaced")
             for i in range(n_extra_crds)]
    lists = []
    for _ in range(C):
        lst = list(builtin) if p_builtin >= 1.0 else [r for r, k in zip(builtin, rng.random(len(builtin)) < p_builtin) if k]
        for grp, keep in zip(ops, rng.random(len(ops)) < p_operator):
            if keep:
                lst.extend(grp)
        lst.extend(r for r, keep in zip(extra, rng.random(len(extra)) < p_operator) if keep)
        lst.sort(key=lambda r: r.kind)  # clusterstatus.go:262-264 (stable here, see module comment)
        lists.append(lst)
    return lists


def profile_for(config: str) -> F.Framework:
    """The plugin set each config is quoted on (BASELINE.json configs)."""
    if config in ("c2", "c3", "c3r", "c3p"):
        return F.Framework(F.EnabledPlugins(
            [F.APIResources, F.TaintToleration, F.ClusterResourcesFit, F.ClusterAffinity],
            [F.ClusterResourcesLeastAllocated], [F.MaxCluster], [F.ClusterCapacityWeight]))
    return F.Framework(F.default_enabled_plugins())


# ----------------------------------------------------------------- clusters
def gen_clusters(rng: np.random.Generator, C: int, n_keys=8, n_vals=8, n_int_keys=0, n_taints=16,
                 taints_per=(0, 3), p_gvk=1.0, gvks=GVKS[:1], scalars=False) -> List[T.FederatedCluster]:
    alloc_cpu = rng.integers(8_000, 4_000_001, C)
    alloc_mem = rng.integers(32 * GI, 16 * TI + 1, C, dtype=np.int64)
    fa = rng.random(C)
    fm = rng.random(C)
    taint_pool = [T.Taint(f"taint-{i % max(1, n_taints // 3)}", f"v{i}", EFFECTS[i % 3]) for i in range(n_taints)]
    out = []
    for c in range(C):
        labels = {}
        for k in range(n_keys):
            if rng.random() < 0.9:
                labels[f"key{k}"] = f"val{int(rng.integers(0, n_vals))}"
        for k in range(n_int_keys):
            if rng.random() < 0.9:
                labels[f"num{k}"] = str(int(rng.integers(0, 1000)))
        nt = int(rng.integers(taints_per[0], taints_per[1] + 1)) if n_taints else 0
        taints = [taint_pool[int(i)] for i in rng.choice(n_taints, size=min(nt, n_taints), replace=False)] if nt else []
        api = [T.APIResource(*g) for g in gvks if rng.random() < p_gvk]
        ac, am = int(alloc_cpu[c]), int(alloc_mem[c])
        vc, vm = int(ac * fa[c]), int(am * fm[c])
        alloc = {"cpu": f"{ac}m", "memory": str(am)}
        avail = {"cpu": f"{vc}m", "memory": str(vm)}
        if scalars:
            g = int(rng.integers(0, 9))
            alloc["example.com/gpu"] = str(g)
            avail["example.com/gpu"] = str(int(rng.integers(0, g + 1)))
        out.append(T.FederatedCluster(name=f"cluster-{c:05d}", labels=labels, taints=taints,
                                      api_resource_types=api, allocatable=alloc, available=avail))
    return out


def _tolerations(rng, n_taints, lo, hi, allow_wild=False):
    tols = []
    for _ in range(int(rng.integers(lo, hi + 1))):
        i = int(rng.integers(0, max(1, n_taints)))
        r = rng.random()
        if allow_wild and r < 0.05:
            tols.append(T.Toleration("", T.TOLERATION_OP_EXISTS, "", ""))
        elif r < 0.5:
            tols.append(T.Toleration(f"taint-{i % max(1, n_taints // 3)}", T.TOLERATION_OP_EQUAL, f"v{i}",
                                     EFFECTS[i % 3] if rng.random() < 0.7 else ""))
        else:
            tols.append(T.Toleration(f"taint-{i % max(1, n_taints // 3)}", T.TOLERATION_OP_EXISTS, "",
                                     EFFECTS[int(rng.integers(0, 3))] if rng.random() < 0.7 else ""))
    return tols


def _expr(rng, n_keys, n_vals, n_int_keys=0, all_ops=False, p_invalid=0.0):
    if p_invalid and rng.random() < p_invalid:
        bad = int(rng.integers(0, 4))
        if bad == 0:
            return T.ClusterSelectorRequirement("key0", T.OP_IN, ["invalid value: ___@#$%^"])
        if bad == 1:
            return T.ClusterSelectorRequirement("bad key/with/slashes", T.OP_EXISTS, None)
        if bad == 2:
            return T.ClusterSelectorRequirement("key1", "Bogus", ["val1"])
        return T.ClusterSelectorRequirement("key2", T.OP_IN, [])
    ops = [T.OP_IN, T.OP_NOT_IN, T.OP_EXISTS] + ([T.OP_DOES_NOT_EXIST, T.OP_GT, T.OP_LT] if all_ops else [])
    op = ops[int(rng.integers(0, len(ops)))]
    if op in (T.OP_GT, T.OP_LT) and n_int_keys:
        return T.ClusterSelectorRequirement(f"num{int(rng.integers(0, n_int_keys))}", op,
                                            [str(int(rng.integers(0, 1000)))])
    if op in (T.OP_GT, T.OP_LT):
        op = T.OP_IN
    key = f"key{int(rng.integers(0, n_keys))}"
    if op in (T.OP_EXISTS, T.OP_DOES_NOT_EXIST):
        return T.ClusterSelectorRequirement(key, op, None)
    nv = int(rng.integers(1, 4))
    return T.ClusterSelectorRequirement(key, op, [f"val{int(v)}" for v in rng.integers(0, n_vals, nv)])


# ------------------------------------------------------------------- units
def gen_units_c2(rng, W: int, n_keys=8, n_vals=8, n_taints=16, mode=T.SCHEDULING_MODE_DUPLICATE,
                 prefix="su") -> List[T.SchedulingUnit]:
    cpu = rng.integers(0, 64_001, W)
    mem = rng.integers(0, 256 * GI + 1, W, dtype=np.int64)
    maxc = rng.integers(1, 17, W)
    out = []
    for w in range(W):
        sel = None
        if rng.random() < 0.5:
            sel = {f"key{int(rng.integers(0, n_keys))}": f"val{int(rng.integers(0, n_vals))}"}
        exprs = [_expr(rng, n_keys, n_vals) for _ in range(int(rng.integers(1, 3)))]
        aff = T.Affinity(T.ClusterAffinity(required=T.ClusterSelector([T.ClusterSelectorTerm(exprs)])))
        out.append(T.SchedulingUnit(
            group="apps", version="v1", kind="Deployment", resource="deployments", namespace="default",
            name=f"{prefix}-{w}", desired_replicas=int(rng.integers(1, 101)),
            resource_request=T.Resource(int(cpu[w]), int(mem[w])), scheduling_mode=mode,
            cluster_selector=sel, affinity=aff, tolerations=_tolerations(rng, n_taints, 0, 3),
            max_clusters=int(maxc[w])))
    return out


def gen_units_c1(rng, W: int, clusters) -> List[T.SchedulingUnit]:
    names = [c.name for c in clusters]
    out = []
    for w in range(W):
        weights = None
        if w % 2 == 0:
            weights = {n: int(rng.integers(0, 11)) for n in names}
        out.append(T.SchedulingUnit(
            group="apps", version="v1", kind="Deployment", namespace="default", name=f"dep-{w}",
            desired_replicas=int(rng.integers(1, 101)), scheduling_mode=T.SCHEDULING_MODE_DIVIDE,
            avoid_disruption=True, weights=weights, tolerations=_tolerations(rng, 16, 0, 3),
            resource_request=T.Resource(int(rng.integers(0, 4001)), int(rng.integers(0, 8 * GI)))))
    return out


def gen_units_c4(rng, W: int, clusters) -> List[T.SchedulingUnit]:
    names = [c.name for c in clusters]
    C = len(names)
    out = []
    for w in range(W):
        k = int(rng.integers(8, 65))
        place = [names[int(i)] for i in rng.choice(C, size=min(k, C), replace=False)]
        weights = {n: int(rng.integers(0, 101)) for n in place} if rng.random() < 0.5 else None
        mins = {n: int(rng.integers(0, 6)) for n in place if rng.random() < 0.3}
        maxs = {n: int(rng.integers(0, 200)) for n in place if rng.random() < 0.3}
        caps = {n: int(rng.integers(0, 500)) for n in place if rng.random() < 0.2}
        cur = None
        if rng.random() < 0.25:
            cur = {n: (int(rng.integers(0, 300)) if rng.random() < 0.9 else None)
                   for n in place if rng.random() < 0.5}
        out.append(T.SchedulingUnit(
            group="apps", version="v1", kind="Deployment", namespace=f"ns{w % 7}", name=f"c4-{w}",
            desired_replicas=int(rng.integers(1, 10_001)), scheduling_mode=T.SCHEDULING_MODE_DIVIDE,
            avoid_disruption=bool(rng.random() < 0.5), cluster_names=set(place), weights=weights,
            min_replicas=mins or None, max_replicas=maxs or None, current_clusters=cur,
            auto_migration=T.AutoMigrationSpec(caps, bool(rng.random() < 0.5)) if caps else None,
            tolerations=_tolerations(rng, 16, 0, 3)))
    return out


def gen_units_c5(rng, W: int, clusters, n_keys=64, n_vals=16, n_int_keys=4, n_taints=256):
    names = [c.name for c in clusters]
    out = []
    for w in range(W):
        terms = []
        for _ in range(int(rng.integers(2, 9))):
            exprs = [_expr(rng, n_keys, n_vals, n_int_keys, all_ops=True, p_invalid=0.01)
                     for _ in range(int(rng.integers(2, 7)))]
            fields = None
            if rng.random() < 0.3:
                fields = [T.ClusterSelectorRequirement("metadata.name", T.OP_NOT_IN,
                                                       [names[int(rng.integers(0, len(names)))]])]
            terms.append(T.ClusterSelectorTerm(exprs, fields))
        prefs = [T.PreferredSchedulingTerm(int(rng.integers(1, 101)), T.ClusterSelectorTerm(
            [_expr(rng, n_keys, n_vals, n_int_keys, all_ops=True) for _ in range(int(rng.integers(1, 4)))]))
            for _ in range(int(rng.integers(2, 5)))]
        out.append(T.SchedulingUnit(
            group=GVKS[w % 8][0], version="v1", kind=GVKS[w % 8][2], namespace="default", name=f"c5-{w}",
            desired_replicas=int(rng.integers(1, 101)), scheduling_mode=T.SCHEDULING_MODE_DIVIDE
            if rng.random() < 0.5 else T.SCHEDULING_MODE_DUPLICATE,
            affinity=T.Affinity(T.ClusterAffinity(T.ClusterSelector(terms), prefs)),
            tolerations=_tolerations(rng, n_taints, 1, 8, allow_wild=True), max_clusters=int(rng.integers(1, 17)),
            resource_request=T.Resource(int(rng.integers(0, 64_001)), int(rng.integers(0, 256 * GI)))))
    return out


def make_config(config: str, scale: float = 1.0, seed: Optional[int] = None, W: Optional[int] = None,
                C: Optional[int] = None) -> Tuple[List[T.FederatedCluster], List[T.SchedulingUnit], F.Framework]:
    W0, C0 = SIZES[config]
    W = W if W is not None else max(1, int(W0 * scale))
    if C is None:
        C = C0 if config != "c5" else max(16, int(C0 * min(1.0, scale * 10)))
    rng = np.random.default_rng(SEEDS[config] if seed is None else seed)
    if config == "c1":
        cl = gen_clusters(rng, C, p_gvk=1.0)
        return cl, gen_units_c1(rng, W, cl), profile_for(config)
    if config in ("c2", "c3"):
        cl = gen_clusters(rng, C)
        return cl, gen_units_c2(rng, W), profile_for(config)
    if config in ("c3r", "c3p"):
        cl = gen_clusters(rng, C)
        for c, api in zip(cl, discovery_api_resources(np.random.default_rng([SEEDS[config], 0xA91]), C)):
            c.api_resource_types = api
        units = gen_units_c2(rng, W)
        if config == "c3p":  # over-committed / cordoned clusters, no ResourceRequest (bench.make_clusters)
            production_resources(cl, np.random.default_rng([SEEDS[config], 0x9E5]))
            for su in units:
                su.resource_request = T.Resource()
        r2 = np.random.default_rng([SEEDS[config], 0x6E7])
        gv = [g for g, _ in C3R_WORKLOADS]
        share = np.array([p for _, p in C3R_WORKLOADS])
        for su, i in zip(units, r2.choice(len(gv), size=W, p=share / share.sum())):
            su.group, su.version, su.kind = gv[i]
        return cl, units, profile_for(config)
    if config == "c4":
        cl = gen_clusters(rng, C)
        return cl, gen_units_c4(rng, W, cl), profile_for(config)
    if config == "c5":
        cl = gen_clusters(rng, C, n_keys=64, n_vals=16, n_int_keys=4, n_taints=256, taints_per=(4, 16), p_gvk=0.9,
                          gvks=GVKS)
        return cl, gen_units_c5(rng, W, cl), profile_for(config)
    raise KeyError(config)


# ------------------------------------------------------------------- fuzz
def widen_prefs(units, seed: int, share: float = 0.3):
    """Push some preference-map values of ``units`` (in place) past int32 — weights, min / max replicas,
    estimated capacities of 2^31 … 2^40 — so the packers choose the wide (i64) preference columns
    (KAD_BATCH_NARROW_PREFS off). Returns the units."""
    rng = np.random.default_rng(seed)
    for su in units:
        if rng.random() >= share:
            continue
        maps = [m for m in (su.weights, su.min_replicas, su.max_replicas,
                            su.auto_migration.estimated_capacity if su.auto_migration is not None else None) if m]
        for m in maps:
            for k in list(m):
                if rng.random() < 0.5 and m[k] is not None and m[k] >= 0:
                    m[k] = int(m[k]) + int(rng.integers(1 << 31, 1 << 40))
    return units


def gen_fuzz(seed: int, W: int = 60, C: Optional[int] = None, n_taints: int = 9):
    """Small batch hitting every branch: all operators, invalid requirements, nil/empty terms, fields,
    sticky, current clusters, scalars, NoExecute on scheduled clusters, ties, weights/min/max/caps.
    n_taints > 64 spreads the taint ids over several 64-bit words (SnapDev::TW > 1)."""
    rng = np.random.default_rng(seed)
    C = C if C is not None else int(rng.integers(1, 40))
    cl = gen_clusters(rng, C, n_keys=4, n_vals=3, n_int_keys=2, n_taints=n_taints,
                      taints_per=(0, 3) if n_taints <= 9 else (1, 12), p_gvk=0.8, gvks=GVKS[:3], scalars=True)
    # make scores tie-heavy: quantise resources on some clusters
    for c in cl:
        if rng.random() < 0.5:
            c.allocatable["cpu"] = "8"
            c.available["cpu"] = "4"
            c.allocatable["memory"] = "16Gi"
            c.available["memory"] = "8Gi"
        if rng.random() < 0.1:
            c.taints = c.taints + c.taints[:1]  # duplicate taint: PNS counts with multiplicity
        if rng.random() < 0.05:
            c.labels = None
    names = [c.name for c in cl] + ["ghost-cluster"]
    units = []
    for w in range(W):
        r = rng.random
        mode = T.SCHEDULING_MODE_DUPLICATE if r() < 0.4 else T.SCHEDULING_MODE_DIVIDE
        aff = None
        if r() < 0.8:
            req = None
            if r() < 0.7:
                terms = []
                for _ in range(int(rng.integers(0, 4))):
                    exprs = [_expr(rng, 5, 4, 3, all_ops=True, p_invalid=0.08) for _ in range(int(rng.integers(0, 3)))]
                    fields = None
                    if r() < 0.3:
                        fk = "metadata.name" if r() < 0.8 else "metadata.namespace"
                        op = [T.OP_IN, T.OP_NOT_IN, T.OP_EXISTS][int(rng.integers(0, 3))] if r() < 0.9 else T.OP_IN
                        vals = [names[int(rng.integers(0, len(names)))]] if r() < 0.9 else ["a", "b"]
                        fields = [T.ClusterSelectorRequirement(fk, op, vals)]
                    terms.append(T.ClusterSelectorTerm(exprs if (exprs or r() < 0.5) else None, fields))
                req = T.ClusterSelector(terms if (terms or r() < 0.5) else None)
            prefs = None
            if r() < 0.6:
                prefs = []
                for _ in range(int(rng.integers(0, 4))):
                    exprs = [_expr(rng, 5, 4, 3, all_ops=True, p_invalid=0.05) for _ in range(int(rng.integers(0, 3)))]
                    wgt = int(rng.integers(-20, 101)) if r() < 0.9 else 0
                    prefs.append(T.PreferredSchedulingTerm(wgt, T.ClusterSelectorTerm(exprs)))
            aff = T.Affinity(T.ClusterAffinity(req, prefs) if r() < 0.95 else None)
        sel = None
        if r() < 0.3:
            sel = {f"key{int(rng.integers(0, 5))}": f"val{int(rng.integers(0, 4))}" for _ in range(int(rng.integers(0, 3)))}
        place = None
        if r() < 0.3:
            place = {names[int(i)] for i in rng.integers(0, len(names), int(rng.integers(0, 6)))}
        cur = None
        if r() < 0.3:
            cur = {names[int(i)]: (int(rng.integers(0, 30)) if r() < 0.8 else None)
                   for i in rng.integers(0, len(names), int(rng.integers(0, 4)))}
        weights = None
        if r() < 0.4:
            weights = {names[int(i)]: int(rng.integers(0, 10)) for i in rng.integers(0, len(names), int(rng.integers(0, 6)))}
        mins = {names[int(i)]: int(rng.integers(0, 5)) for i in rng.integers(0, len(names), 2)} if r() < 0.3 else None
        maxs = {names[int(i)]: int(rng.integers(0, 8)) for i in rng.integers(0, len(names), 2)} if r() < 0.3 else None
        am = None
        if r() < 0.3:
            am = T.AutoMigrationSpec({names[int(i)]: int(rng.integers(-2, 6)) for i in rng.integers(0, len(names), 3)}
                                     if r() < 0.8 else None, bool(r() < 0.5))
        scal = None
        if r() < 0.2:
            scal = {"example.com/gpu": int(rng.integers(0, 4))}
            if r() < 0.3:
                scal["example.com/missing"] = int(rng.integers(0, 2))
        g = GVKS[int(rng.integers(0, 4))]
        units.append(T.SchedulingUnit(
            group=g[0], version=g[1], kind=g[2], namespace="ns" if r() < 0.7 else "", name=f"fz-{seed}-{w}",
            desired_replicas=(int(rng.integers(-1, 40)) if r() < 0.9 else None),
            resource_request=T.Resource(int(rng.integers(0, 5000)) if r() < 0.7 else 0,
                                        int(rng.integers(0, 20 * GI)) if r() < 0.7 else 0,
                                        int(rng.integers(0, 2)) if r() < 0.1 else 0, scal),
            current_clusters=cur, auto_migration=am, scheduling_mode=mode, sticky_cluster=bool(r() < 0.1),
            avoid_disruption=bool(r() < 0.5), cluster_selector=sel, cluster_names=place, affinity=aff,
            tolerations=(_tolerations(rng, n_taints, 0, 3 if n_taints <= 9 else 10, allow_wild=True)
                         if r() < 0.8 else None),
            max_clusters=(int(rng.integers(-1, 8)) if r() < 0.8 else None), min_replicas=mins, max_replicas=maxs,
            weights=weights))
    return cl, units


def with_discovery(clusters, units, seed: int, p_operator: float = 0.7, p_builtin: float = 0.9):
    """``clusters`` (in place) with discovery-shaped API-resource lists (:func:`discovery_api_resources`, with
    gaps in the built-ins too) and ``units`` (in place) over :data:`C3R_WORKLOADS`' kinds plus one kind no
    cluster serves: GVK ids past the first 64 (the snapshot interns ~150). Returns (clusters, units)."""
    rng = np.random.default_rng([seed, 0xD15C])
    for c, api in zip(clusters, discovery_api_resources(rng, len(clusters), p_operator=p_operator,
                                                        p_builtin=p_builtin)):
        c.api_resource_types = api
    kinds = [g for g, _ in C3R_WORKLOADS] + [("example.com", "v1", "NowhereServed")]
    for su, i in zip(units, rng.integers(0, len(kinds), len(units))):
        su.group, su.version, su.kind = kinds[int(i)]
    return clusters, units


FUZZ_PROFILES = [
    F.EnabledPlugins(),  # nothing: all clusters feasible, all selected
    None,  # default
    F.EnabledPlugins([F.ClusterAffinity, F.TaintToleration], [F.ClusterAffinity, F.TaintToleration],
                     [F.MaxCluster], [F.ClusterCapacityWeight]),
    F.EnabledPlugins([F.ClusterResourcesFit, F.APIResources, F.PlacementFilter],
                     [F.ClusterResourcesMostAllocated, F.ClusterResourcesBalancedAllocation],
                     [F.MaxCluster], [F.ClusterCapacityWeight]),
    F.EnabledPlugins([F.PlacementFilter], [F.ClusterResourcesLeastAllocated], [], [F.ClusterCapacityWeight]),
    F.EnabledPlugins([F.TaintToleration, F.ClusterResourcesFit], [F.TaintToleration,
                                                                  F.ClusterResourcesLeastAllocated,
                                                                  F.ClusterResourcesMostAllocated],
                     [F.MaxCluster], []),
]


def fuzz_framework(i: int) -> F.Framework:
    ep = FUZZ_PROFILES[i % len(FUZZ_PROFILES)]
    return F.Framework(ep if ep is not None else F.default_enabled_plugins())


# ------------------------------------------------------------ scheduling-trigger workload (§8(f) f4)
TRIGGER_SIZES = {"t1": (1000, 16), "t2": (100_000, 256)}


def _api_pool(n: int):
    base = [("apps", "v1", "Deployment", "deployments"), ("apps", "v1", "StatefulSet", "statefulsets"),
            ("apps", "v1", "DaemonSet", "daemonsets"), ("batch", "v1", "Job", "jobs"),
            ("batch", "v1", "CronJob", "cronjobs"), ("", "v1", "ConfigMap", "configmaps"),
            ("", "v1", "Secret", "secrets"), ("", "v1", "Service", "services"),
            ("networking.k8s.io", "v1", "Ingress", "ingresses")]
    out = [T.APIResource(g, v, k, p, "Namespaced") for g, v, k, p in base]
    i = 0
    while len(out) < n:
        out.append(T.APIResource(f"crd{i // 4}.example.com", f"v{1 + i % 2}", f"Kind{i}", f"kind{i}s",
                                 "Cluster" if i % 5 == 0 else "Namespaced"))
        i += 1
    return out[:n]


def gen_trigger_workload(rng: np.random.Generator, W: int, C: int, n_policies: int = 64, n_api: int = 64):
    """Joined clusters as the trigger hash sees them (labels, taints, ~n_api API resources each) and W
    federated Deployments: a policy out of ``n_policies`` (some with auto migration), replicas 1-100,
    10 % with scheduling annotations. Returns (type_config, clusters, objects, policies)."""
    from . import objects as O

    clusters = gen_clusters(rng, C)
    pool = _api_pool(n_api)
    for c in clusters:
        keep = rng.random(len(pool)) < 0.9
        api = [pool[i] for i in np.nonzero(keep)[0]]
        rng.shuffle(api)
        c.api_resource_types = api
    pols = [O.PropagationPolicy(f"policy-{i}", "default", int(rng.integers(1, 20)), O.PropagationPolicySpec(
        scheduling_mode=T.SCHEDULING_MODE_DIVIDE,
        auto_migration=O.AutoMigration() if i % 4 == 0 else None)) for i in range(n_policies)]
    ftc = O.FederatedTypeConfig("apps", "v1", "Deployment", "deployments", "Namespaced", "spec.replicas")
    objs, opols = [], []
    for w in range(W):
        p = pols[int(rng.integers(0, n_policies))]
        ann = {O.PROPAGATION_POLICY_NAME_LABEL: p.name}
        annotations = {"kubectl.kubernetes.io/last-applied-configuration": "{}"}
        r = rng.random()
        if r < 0.05:
            annotations[O.MAX_CLUSTERS_ANNOTATIONS] = str(int(rng.integers(1, 8)))
        elif r < 0.10:
            annotations[O.PLACEMENTS_ANNOTATIONS] = json.dumps(
                [{"cluster": clusters[int(rng.integers(0, C))].name, "preferences": {"weight": int(rng.integers(1, 9))}}])
        if p.spec.auto_migration is not None and rng.random() < 0.5:
            annotations[O.AUTO_MIGRATION_INFO_ANNOTATION] = json.dumps(
                {"estimatedCapacity": {clusters[int(rng.integers(0, C))].name: int(rng.integers(0, 50))}})
        objs.append({"apiVersion": "types.kubeadmiral.io/v1alpha1", "kind": "FederatedDeployment",
                     "metadata": {"name": f"app-{w}", "namespace": "default", "labels": ann,
                                  "annotations": annotations},
                     "spec": {"template": {"apiVersion": "apps/v1", "kind": "Deployment",
                                           "metadata": {"name": f"app-{w}", "namespace": "default"},
                                           "spec": {"replicas": int(rng.integers(1, 101))}}}})
        opols.append(p)
    return ftc, clusters, objs, opols


# ------------------------------------------------------- cluster update events
def mutate_clusters(rng: np.random.Generator, clusters: List[T.FederatedCluster], n_changed: int,
                    structural: bool = True) -> Tuple[List[T.FederatedCluster], List[int]]:
    """A cluster informer update: ``n_changed`` clusters get new status resources (the periodic status
    collection) and, with ``structural``, label values / taints / API resources drawn from what the other
    clusters already carry (so the snapshot vocabulary does not grow). Returns (new list, changed positions)."""
    import copy

    vals: Dict[str, list] = {}
    taints, apis = {}, {}
    for c in clusters:
        for k, v in (c.labels or {}).items():
            vals.setdefault(k, []).append(v)
        for t in c.taints:
            taints[(t.key, t.value, t.effect)] = t
        for r in c.api_resource_types:
            apis[(r.group, r.version, r.kind)] = r
    taint_pool, api_pool = list(taints.values()), list(apis.values())
    idx = sorted(int(i) for i in rng.choice(len(clusters), size=min(n_changed, len(clusters)), replace=False))
    out = list(clusters)
    for i in idx:
        c = copy.deepcopy(clusters[i])
        if c.allocatable and "cpu" in c.allocatable:
            ac = k8s.milli_value(k8s.quantity(c.allocatable["cpu"]))
            am = k8s.value(k8s.quantity(c.allocatable["memory"])) if "memory" in c.allocatable else 0
            c.available = dict(c.available or {}, cpu=f"{int(ac * rng.random())}m", memory=str(int(am * rng.random())))
            if "example.com/gpu" in c.allocatable:
                c.available["example.com/gpu"] = str(int(rng.integers(0, int(c.allocatable["example.com/gpu"]) + 1)))
        if structural:
            if c.labels and rng.random() < 0.5:
                k = sorted(c.labels)[int(rng.integers(0, len(c.labels)))]
                c.labels = dict(c.labels)
                c.labels[k] = vals[k][int(rng.integers(0, len(vals[k])))]
            if taint_pool and rng.random() < 0.4:
                nt = int(rng.integers(0, min(4, len(taint_pool)) + 1))
                c.taints = [taint_pool[int(j)] for j in rng.choice(len(taint_pool), size=nt, replace=False)]
            if api_pool and rng.random() < 0.3:
                c.api_resource_types = [r for r in api_pool if rng.random() < 0.8]
        out[i] = c
    return out, idx


# ------------------------------------------------------------ columnar generator (native packer input)
def gen_units_c2_columns(rng: np.random.Generator, W: int, n_keys=8, n_vals=8, n_taints=16,
                         mode=T.SCHEDULING_MODE_DUPLICATE, prefix="su", workloads=None):
    """The C2/C3 workload of :func:`gen_units_c2` (same distributions, its own random stream) generated
    directly as ``columns.SUColumns`` with numpy — the packer input a Go shim would hand over — so 1M-unit
    batches (C3) are generated in about a second instead of minutes of Python objects.

    ``workloads``: [((group, version, kind), share), ...] — each unit's GVK drawn with these shares (c3r:
    :data:`C3R_WORKLOADS`) after every other column, so the rest of the batch equals the one without it;
    default: every unit an apps/v1 Deployment."""
    from . import columns as CO

    st = CO.StringTable()
    sid = st.id
    key_ids = np.array([sid(f"key{k}") for k in range(n_keys)], np.int32)
    val_ids = np.array([sid(f"val{v}") for v in range(n_vals)], np.int32)
    op_ids = np.array([sid(o) for o in (T.OP_IN, T.OP_NOT_IN, T.OP_EXISTS)], np.int32)
    nt5 = max(1, n_taints // 3)
    tkey_ids = np.array([sid(f"taint-{i % nt5}") for i in range(max(1, n_taints))], np.int32)
    tval_ids = np.array([sid(f"v{i}") for i in range(max(1, n_taints))], np.int32)
    empty = sid("")
    eff_ids = np.array([sid(e) for e in EFFECTS], np.int32)
    equal_id, exists_id = sid(T.TOLERATION_OP_EQUAL), sid(T.TOLERATION_OP_EXISTS)
    g, v, k, ns = sid("apps"), sid("v1"), sid("Deployment"), sid("default")
    name0 = len(st._parts)
    for w in range(W):
        st._parts.append(f"{prefix}-{w}".encode())
    str_off, str_data = st.arrays()

    cols = {}
    cols["group"] = np.full(W, g, np.int32)
    cols["version"] = np.full(W, v, np.int32)
    cols["kind"] = np.full(W, k, np.int32)
    cols["namespace_"] = np.full(W, ns, np.int32)
    cols["name"] = np.arange(name0, name0 + W, dtype=np.int32)
    f = CO.SU_HAS_DESIRED | CO.SU_HAS_MAX_CLUSTERS | CO.SU_HAS_CLUSTER_AFFINITY | CO.SU_HAS_REQUIRED
    if mode == T.SCHEDULING_MODE_DUPLICATE:
        f |= CO.SU_DUPLICATE
    cols["flags"] = np.full(W, f, np.uint32)
    cols["req_cpu"] = rng.integers(0, 64_001, W).astype(np.int64)
    cols["req_mem"] = rng.integers(0, 256 * GI + 1, W, dtype=np.int64)
    cols["req_eph"] = np.zeros(W, np.int64)
    cols["max_clusters"] = rng.integers(1, 17, W).astype(np.int64)
    cols["desired"] = rng.integers(1, 101, W).astype(np.int64)
    # ClusterSelector: half the units, one entry
    has_sel = rng.random(W) < 0.5
    ns_ = int(has_sel.sum())
    cols["sel_off"] = CO._csr_off(has_sel.astype(np.int32))
    cols["sel_key"] = key_ids[rng.integers(0, n_keys, ns_)]
    cols["sel_value"] = val_ids[rng.integers(0, n_vals, ns_)]
    # one required term of 1-2 In / NotIn / Exists expressions
    n_expr = rng.integers(1, 3, W).astype(np.int32)
    R = int(n_expr.sum())
    cols["rterm_off"] = np.arange(W + 1, dtype=np.int32)
    rt_req = np.zeros(W, np.int32)
    rt_req[1:] = np.cumsum(n_expr)[:-1]
    cols["rt_req"] = rt_req
    cols["rt_n_expr"] = n_expr
    cols["rt_n_field"] = np.zeros(W, np.int32)
    op = rng.integers(0, 3, R)
    cols["rq_key"] = key_ids[rng.integers(0, n_keys, R)]
    cols["rq_op"] = op_ids[op]
    nv = np.where(op == 2, 0, rng.integers(1, 4, R)).astype(np.int32)
    cols["rq_val_off"] = CO._csr_off(nv)
    cols["rq_val"] = val_ids[rng.integers(0, n_vals, int(nv.sum()))]
    # tolerations: 0-3, half Equal (effect 70 %), half Exists (random effect 70 %)
    n_tol = rng.integers(0, 4, W).astype(np.int32)
    TT = int(n_tol.sum())
    cols["tol_off"] = CO._csr_off(n_tol)
    i = rng.integers(0, max(1, n_taints), TT)
    r = rng.random(TT)
    with_eff = rng.random(TT) < 0.7
    eq = r < 0.5
    cols["tol_key"] = tkey_ids[i]
    cols["tol_op"] = np.where(eq, equal_id, exists_id).astype(np.int32)
    cols["tol_value"] = np.where(eq, tval_ids[i], empty).astype(np.int32)
    eff = np.where(eq, eff_ids[i % 3], eff_ids[rng.integers(0, 3, TT)])
    cols["tol_effect"] = np.where(with_eff, eff, empty).astype(np.int32)
    zero_off = np.zeros(W + 1, np.int32)
    for grp in ("scalar", "pterm", "place", "cur", "wt", "min", "max", "cap"):
        cols[grp + "_off"] = zero_off
    for kname, dt in CO.FIELDS:
        if kname not in cols:
            cols[kname] = np.zeros(0, dt)
    if workloads:
        gvks = [wk for wk, _ in workloads]
        share = np.array([p for _, p in workloads], np.float64)
        pick = rng.choice(len(gvks), size=W, p=share / share.sum())
        # the string table already holds every unit name: new strings go after them
        ids = np.array([[st.id(x) for x in g] for g in gvks], np.int32)
        str_off, str_data = st.arrays()
        cols["group"], cols["version"], cols["kind"] = ids[pick, 0], ids[pick, 1], ids[pick, 2]
    return CO.SUColumns(W, str_off, str_data, cols)


def _tol_columns(rng, st, W: int, n_taints: int, lo: int, hi: int, allow_wild: bool = False):
    """Columns of :func:`_tolerations` (same distribution, vectorised): lo..hi tolerations per unit; 5 %
    wildcard (empty key, Exists) with ``allow_wild``; else half Equal (key/value of a pool taint, its effect
    70 %), half Exists (a pool key, a random effect 70 %)."""
    from . import columns as CO

    sid = st.id
    nt = max(1, n_taints)
    nt3 = max(1, n_taints // 3)
    tkey = np.array([sid(f"taint-{i % nt3}") for i in range(nt)], np.int32)
    tval = np.array([sid(f"v{i}") for i in range(nt)], np.int32)
    eff = np.array([sid(e) for e in EFFECTS], np.int32)
    empty, equal_id, exists_id = sid(""), sid(T.TOLERATION_OP_EQUAL), sid(T.TOLERATION_OP_EXISTS)
    n = rng.integers(lo, hi + 1, W).astype(np.int32)
    TT = int(n.sum())
    i = rng.integers(0, nt, TT)
    r = rng.random(TT)
    with_eff = rng.random(TT) < 0.7
    wild = (r < 0.05) if allow_wild else np.zeros(TT, bool)
    eq = ~wild & (r < 0.5)
    e = np.where(eq, eff[i % 3], eff[rng.integers(0, 3, TT)])
    return {"tol_off": CO._csr_off(n),
            "tol_key": np.where(wild, empty, tkey[i]).astype(np.int32),
            "tol_op": np.where(eq, equal_id, exists_id).astype(np.int32),
            "tol_value": np.where(eq, tval[i], empty).astype(np.int32),
            "tol_effect": np.where(wild | ~with_eff, empty, e).astype(np.int32)}


def _fill_columns(W: int, st, cols):
    from . import columns as CO

    zero_off = np.zeros(W + 1, np.int32)
    for grp in CO.CSR_GROUPS:
        cols.setdefault(grp + "_off", zero_off)
    cols.setdefault("rq_val_off", np.zeros(1, np.int32))  # no requirements: one offset
    for kname, dt in CO.FIELDS:
        if kname not in cols:
            cols[kname] = np.zeros(W if kname in ("desired", "max_clusters", "req_cpu", "req_mem", "req_eph")
                                   else 0, dt)
    str_off, str_data = st.arrays()
    return CO.SUColumns(W, str_off, str_data, cols)


def _names(st, W: int, prefix: str) -> np.ndarray:
    name0 = len(st._parts)
    for w in range(W):
        st._parts.append(f"{prefix}-{w}".encode())
    return np.arange(name0, name0 + W, dtype=np.int32)


def gen_units_c4_columns(rng: np.random.Generator, W: int, cluster_names, prefix="c4"):
    """The C4 replica-planner stress workload of :func:`gen_units_c4` (same distributions, its own random
    stream) as ``columns.SUColumns``: Divide units with ClusterNames of 8-64 distinct clusters (a random
    start and odd stride over the snapshot, distinct for C a power of two — else rejected and redrawn),
    static weights U{0..100} on half the units, MinReplicas U{0..5} / MaxReplicas U{0..199} on 30 % and
    EstimatedCapacity U{0..499} on 20 % of the entries (AutoMigration when any, KeepUnschedulable 50 %),
    CurrentClusters on 25 % of the units (half the entries, 10 % nil replicas), DesiredReplicas
    U{1..10 000}, AvoidDisruption 50 %, 0-3 tolerations."""
    from . import columns as CO

    C = len(cluster_names)
    st = CO.StringTable()
    sid = st.id
    cid = np.array([sid(n) for n in cluster_names], np.int32)
    g, v, k = sid("apps"), sid("v1"), sid("Deployment")
    nss = np.array([sid(f"ns{i}") for i in range(7)], np.int32)
    cols = {"group": np.full(W, g, np.int32), "version": np.full(W, v, np.int32), "kind": np.full(W, k, np.int32),
            "namespace_": nss[np.arange(W) % 7], "name": _names(st, W, prefix)}
    kk = np.minimum(rng.integers(8, 65, W), C).astype(np.int32)
    P = int(kk.sum())
    place_off = CO._csr_off(kk)
    unit_of = np.repeat(np.arange(W), kk)
    j = np.arange(P) - place_off[:-1][unit_of]
    start = rng.integers(0, C, W)
    if C & (C - 1) == 0:
        stride = (2 * rng.integers(0, max(1, C // 2), W) + 1) % C if C > 1 else np.zeros(W, np.int64)
        pos = (start[unit_of] + stride[unit_of] * j) % max(C, 1)
    else:  # consecutive clusters from a random start (distinct for k <= C)
        pos = (start[unit_of] + j) % C
    cols["place_off"] = place_off
    cols["place_name"] = cid[pos]
    has_w = rng.random(W) < 0.5
    wl = np.where(has_w, kk, 0).astype(np.int32)
    cols["wt_off"] = CO._csr_off(wl)
    sel_w = has_w[unit_of]
    cols["wt_name"] = cid[pos[sel_w]]
    cols["wt_val"] = rng.integers(0, 101, int(sel_w.sum())).astype(np.int64)

    def sub_map(p, lo, hi, grp):
        m = rng.random(P) < p
        cols[grp + "_off"] = CO._csr_off(np.bincount(unit_of[m], minlength=W).astype(np.int32))
        cols[grp + "_name"] = cid[pos[m]]
        cols[grp + "_val"] = rng.integers(lo, hi + 1, int(m.sum())).astype(np.int64)
        return m

    sub_map(0.3, 0, 5, "min")
    sub_map(0.3, 0, 199, "max")
    mc = sub_map(0.2, 0, 499, "cap")
    has_am = np.bincount(unit_of[mc], minlength=W) > 0
    has_cur = rng.random(W) < 0.25
    mcur = has_cur[unit_of] & (rng.random(P) < 0.5)
    cols["cur_off"] = CO._csr_off(np.bincount(unit_of[mcur], minlength=W).astype(np.int32))
    cols["cur_name"] = cid[pos[mcur]]
    ncur = int(mcur.sum())
    hr = rng.random(ncur) < 0.9
    cols["cur_rep"] = np.where(hr, rng.integers(0, 300, ncur), 0).astype(np.int64)
    cols["cur_has_rep"] = hr.astype(np.uint8)
    f = np.full(W, CO.SU_HAS_DESIRED, np.uint32)
    f |= np.where(rng.random(W) < 0.5, CO.SU_AVOID_DISRUPTION, 0).astype(np.uint32)
    f |= np.where(has_am, CO.SU_HAS_AUTO_MIGRATION, 0).astype(np.uint32)
    f |= np.where(has_am & (rng.random(W) < 0.5), CO.SU_KEEP_UNSCHED, 0).astype(np.uint32)
    cols["flags"] = f
    cols["desired"] = rng.integers(1, 10_001, W).astype(np.int64)
    cols.update(_tol_columns(rng, st, W, 16, 0, 3))
    return _fill_columns(W, st, cols)


def _expr_columns(rng, st, R: int, n_keys: int, n_vals: int, n_int_keys: int, p_invalid: float):
    """R requirements of :func:`_expr` (all_ops=True, vectorised): (rq_key, rq_op, per-requirement value
    counts, flat value ids)."""
    sid = st.id
    keys = np.array([sid(f"key{k}") for k in range(n_keys)], np.int32)
    ikeys = np.array([sid(f"num{k}") for k in range(max(1, n_int_keys))], np.int32)
    vals = np.array([sid(f"val{v}") for v in range(n_vals)], np.int32)
    nums = np.array([sid(str(i)) for i in range(1000)], np.int32)
    ops = np.array([sid(o) for o in (T.OP_IN, T.OP_NOT_IN, T.OP_EXISTS, T.OP_DOES_NOT_EXIST, T.OP_GT, T.OP_LT)],
                   np.int32)
    # the invalid forms of _expr: an invalid label value, an invalid key, an unknown operator, In with no value
    bad_key = np.array([sid("key0"), sid("bad key/with/slashes"), sid("key1"), sid("key2")], np.int32)
    bad_op = np.array([ops[0], ops[2], sid("Bogus"), ops[0]], np.int32)
    bad_nv = np.array([1, 0, 1, 0], np.int32)
    bad_v = np.array([sid("invalid value: ___@#$%^"), -1, sid("val1"), -1], np.int32)
    op = rng.integers(0, 6, R)
    if not n_int_keys:
        op = np.where(op >= 4, 0, op)
    rk = np.where(op >= 4, ikeys[rng.integers(0, max(1, n_int_keys), R)], keys[rng.integers(0, n_keys, R)])
    nv = np.where(op >= 4, 1, np.where(op >= 2, 0, rng.integers(1, 4, R)))
    rop = ops[op]
    inv = (rng.random(R) < p_invalid) if p_invalid else np.zeros(R, bool)
    bad = rng.integers(0, 4, R)
    rk = np.where(inv, bad_key[bad], rk).astype(np.int32)
    rop = np.where(inv, bad_op[bad], rop).astype(np.int32)
    nv = np.where(inv, bad_nv[bad], nv).astype(np.int32)
    owner = np.repeat(np.arange(R), nv)
    V = len(owner)
    rv = np.where(op[owner] >= 4, nums[rng.integers(0, 1000, V)], vals[rng.integers(0, n_vals, V)])
    rv = np.where(inv[owner], bad_v[bad[owner]], rv).astype(np.int32)
    return rk, rop, nv, rv


def _excl_in_group(lengths, group_first):
    """Offset of each item within its group: exclusive prefix of ``lengths`` minus that of the group's first
    item (``group_first[i]`` = index of item i's group's first item)."""
    excl = np.cumsum(lengths) - lengths
    return excl - excl[group_first]


def gen_units_c5_columns(rng: np.random.Generator, W: int, cluster_names, n_keys=64, n_vals=16, n_int_keys=4,
                         n_taints=256, prefix="c5"):
    """The C5 adversarial-filtering workload of :func:`gen_units_c5` (same distributions, its own random
    stream) as ``columns.SUColumns``: 2-8 required terms of 2-6 expressions over every operator (1 %
    invalid) with a metadata.name NotIn field on 30 % of the terms, 2-4 preferred terms of 1-3 expressions
    (weights U{1..100}), GVK = GVKS[w % 8], Divide / Duplicate 50/50, 1-8 tolerations over 256 taints
    (5 % wildcard), MaxClusters U{1..16}, requests cpu U[0, 64 000] milli, memory U[0, 256 GiB)."""
    from . import columns as CO

    C = len(cluster_names)
    st = CO.StringTable()
    sid = st.id
    cid = np.array([sid(n) for n in cluster_names], np.int32)
    gv = [(sid(g[0]), sid("v1"), sid(g[2])) for g in GVKS]
    gw = np.arange(W) % 8
    cols = {"group": np.array([gv[i][0] for i in range(8)], np.int32)[gw],
            "version": np.array([gv[i][1] for i in range(8)], np.int32)[gw],
            "kind": np.array([gv[i][2] for i in range(8)], np.int32)[gw],
            "namespace_": np.full(W, sid("default"), np.int32), "name": _names(st, W, prefix)}
    md_name, notin = sid("metadata.name"), sid(T.OP_NOT_IN)
    # required terms: 2-8 per unit, 2-6 expressions, 30 % with one metadata.name field
    nrt = rng.integers(2, 9, W).astype(np.int32)
    NT = int(nrt.sum())
    ne = rng.integers(2, 7, NT).astype(np.int32)
    nf = (rng.random(NT) < 0.3).astype(np.int32)
    # preferred terms: 2-4 per unit, 1-3 expressions
    npt = rng.integers(2, 5, W).astype(np.int32)
    NP = int(npt.sum())
    pne = rng.integers(1, 4, NP).astype(np.int32)
    # requirement table: unit by unit, its required terms (exprs then fields), then its preferred terms
    rt_unit = np.repeat(np.arange(W), nrt)
    pt_unit = np.repeat(np.arange(W), npt)
    per_rt = ne + nf
    req_per_unit = np.bincount(rt_unit, weights=per_rt, minlength=W).astype(np.int64) + \
        np.bincount(pt_unit, weights=pne, minlength=W).astype(np.int64)
    unit_base = np.zeros(W + 1, np.int64)
    unit_base[1:] = np.cumsum(req_per_unit)
    R = int(unit_base[-1])
    rterm_off, pterm_off = CO._csr_off(nrt), CO._csr_off(npt)
    rt_total = np.bincount(rt_unit, weights=per_rt, minlength=W).astype(np.int64)
    rt_req = (unit_base[:-1][rt_unit] + _excl_in_group(per_rt, rterm_off[:-1][rt_unit])).astype(np.int32)
    pt_req = (unit_base[:-1][pt_unit] + rt_total[pt_unit] +
              _excl_in_group(pne, pterm_off[:-1][pt_unit])).astype(np.int32)
    # which requirement slots are fields (one per term with nf, after its expressions)
    is_field = np.zeros(R, bool)
    is_field[(rt_req + ne)[nf == 1]] = True
    is_pref = np.zeros(R, bool)
    pref_slots = np.repeat(pt_req.astype(np.int64), pne) + _excl_in_group(
        np.ones(int(pne.sum()), np.int64), np.repeat(np.cumsum(pne) - pne, pne))
    is_pref[pref_slots] = True
    # expressions: required ones with 1 % invalid, preferred ones all valid
    rk = np.zeros(R, np.int32)
    rop = np.zeros(R, np.int32)
    nv = np.zeros(R, np.int32)
    out_v = []
    for mask, p_inv in ((~is_field & ~is_pref, 0.01), (is_pref, 0.0)):
        idx = np.nonzero(mask)[0]
        k_, o_, n_, v_ = _expr_columns(rng, st, len(idx), n_keys, n_vals, n_int_keys, p_inv)
        rk[idx], rop[idx], nv[idx] = k_, o_, n_
        out_v.append((idx, n_, v_))
    fidx = np.nonzero(is_field)[0]
    rk[fidx], rop[fidx], nv[fidx] = md_name, notin, 1
    out_v.append((fidx, np.ones(len(fidx), np.int32), cid[rng.integers(0, C, len(fidx))]))
    val_off = CO._csr_off(nv)
    rq_val = np.zeros(int(val_off[-1]), np.int32)
    for idx, n_, v_ in out_v:
        if len(v_):
            dst = np.repeat(val_off[:-1][idx].astype(np.int64), n_) + _excl_in_group(
                np.ones(int(n_.sum()), np.int64), np.repeat(np.cumsum(n_) - n_, n_))
            rq_val[dst] = v_
    cols.update({"rq_key": rk, "rq_op": rop, "rq_val_off": val_off, "rq_val": rq_val,
                 "rterm_off": rterm_off, "rt_req": rt_req, "rt_n_expr": ne, "rt_n_field": nf,
                 "pterm_off": pterm_off, "pt_weight": rng.integers(1, 101, NP).astype(np.int32),
                 "pt_req": pt_req, "pt_n_expr": pne})
    f = np.full(W, CO.SU_HAS_DESIRED | CO.SU_HAS_MAX_CLUSTERS | CO.SU_HAS_CLUSTER_AFFINITY | CO.SU_HAS_REQUIRED,
                np.uint32)
    f |= np.where(rng.random(W) < 0.5, 0, CO.SU_DUPLICATE).astype(np.uint32)
    cols["flags"] = f
    cols["desired"] = rng.integers(1, 101, W).astype(np.int64)
    cols["max_clusters"] = rng.integers(1, 17, W).astype(np.int64)
    cols["req_cpu"] = rng.integers(0, 64_001, W).astype(np.int64)
    cols["req_mem"] = rng.integers(0, 256 * GI, W, dtype=np.int64)
    cols.update(_tol_columns(rng, st, W, n_taints, 1, 8, allow_wild=True))
    return _fill_columns(W, st, cols)


# ------------------------------------------------------- result application (§8 f3)
def gen_result_objects(rng: np.random.Generator, W: int, names: List[str], replicas_path: str = "/spec/replicas"):
    """W federated objects whose placements / overrides exercise every branch of applySchedulingResult's
    result-dependent half: the scheduler's placement present or not (other controllers' placements beside
    it, a second scheduler entry after the first), clusters from the snapshot, unknown names and duplicates,
    an empty cluster list; replicas-path override patches with integral, fractional and non-numeric values,
    other paths, other controllers, clusters outside the snapshot."""
    from . import objects as O

    sched = O.PREFIXED_GLOBAL_SCHEDULER_NAME
    pool = list(names) + ["ghost-a", "ghost-b"]
    out = []
    for w in range(W):
        r = rng.random
        pls = []
        if r() < 0.3:
            pls.append({"controller": "other-controller", "placement": {"clusters": [{"name": pool[0]}]}})
        if r() < 0.75:
            k = int(rng.integers(0, 6))
            cl = [{"name": pool[int(i)]} for i in rng.integers(0, len(pool) if r() < 0.3 else len(names), k)]
            pls.append({"controller": sched, "placement": {"clusters": cl} if (cl or r() < 0.5) else {}})
            if r() < 0.1:
                pls.append({"controller": sched, "placement": {"clusters": [{"name": pool[1]}]}})
        ovs = []
        if r() < 0.6:
            clusters = []
            for c in sorted({pool[int(i)] for i in rng.integers(0, len(pool) if r() < 0.2 else len(names),
                                                                 int(rng.integers(0, 6)))}):
                paths = []
                if r() < 0.2:
                    paths.append({"path": "/spec/template/spec/containers/0/image", "value": "nginx"})
                if r() < 0.85:
                    v = r()
                    val = float(rng.integers(0, 40)) if v < 0.8 else (float(rng.integers(0, 40)) + 0.5 if v < 0.9
                                                                      else str(int(rng.integers(0, 40))))
                    paths.append({"path": replicas_path, "value": val})
                clusters.append({"clusterName": c, "paths": paths})
            ovs.append({"controller": sched, "clusters": clusters})
        if r() < 0.2:
            ovs.append({"controller": "other-controller", "clusters": [{"clusterName": pool[0], "paths": [
                {"path": replicas_path, "value": 7.0}]}]})
        obj = {"apiVersion": "types.kubeadmiral.io/v1alpha1", "kind": "FederatedDeployment",
               "metadata": {"name": f"obj-{w}", "namespace": "default"}, "spec": {"template": {}}}
        if pls or r() < 0.5:
            obj["spec"]["placements"] = pls
        if ovs:
            obj["spec"]["overrides"] = ovs
        out.append(obj)
    return out

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

SEEDS = {"c1": 0xC1, "c2": 0xC2, "c3": 0xC3, "c4": 0xC4, "c5": 0xC5}
SIZES = {"c1": (1000, 16), "c2": (100_000, 256), "c3": (1_000_000, 1000), "c4": (1_000_000, 512),
         "c5": (100_000, 10_000)}


def profile_for(config: str) -> F.Framework:
    """The plugin set each config is quoted on (BASELINE.json configs)."""
    if config in ("c2", "c3"):
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
    if config == "c4":
        cl = gen_clusters(rng, C)
        return cl, gen_units_c4(rng, W, cl), profile_for(config)
    if config == "c5":
        cl = gen_clusters(rng, C, n_keys=64, n_vals=16, n_int_keys=4, n_taints=256, taints_per=(4, 16), p_gvk=0.9,
                          gvks=GVKS)
        return cl, gen_units_c5(rng, W, cl), profile_for(config)
    raise KeyError(config)


# ------------------------------------------------------------------- fuzz
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
                         mode=T.SCHEDULING_MODE_DUPLICATE, prefix="su"):
    """The C2/C3 workload of :func:`gen_units_c2` (same distributions, its own random stream) generated
    directly as ``columns.SUColumns`` with numpy — the packer input a Go shim would hand over — so 1M-unit
    batches (C3) are generated in about a second instead of minutes of Python objects."""
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
    return CO.SUColumns(W, str_off, str_data, cols)

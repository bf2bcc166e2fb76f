"""CPU restatement of KubeAdmiral's scheduling hot path (TEST INFRASTRUCTURE ONLY).

ORACLE HEADER — this module is the parity checker, never the product:
only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import it. It restates, in the reference's own
structure (one function per reference function, each citing file:line under
``/root/reference``), the Go path

  genericScheduler.Schedule → RunFilterPlugins → RunScorePlugins (+Normalize)
  → RunSelectClustersPlugin (MaxCluster) → RunReplicasPlugin (rsp + planner).

Parity pin: ``tests/golden/*.json`` — every table-driven case of the
reference's unit tests on this path, extracted by
``tests/golden/extract_golden.py`` — is replayed
against this module by ``tests/test_oracle_golden.py``.

Reference non-determinism is made explicit:
``AvailableToPercentage``'s remainder recipient among tied maxima is chosen by a
``tie_rule`` (default: lowest snapshot index, the product's rule); callers can
enumerate all admissible recipients.
"""

from __future__ import annotations

from typing import Dict, List, Optional

from kubeadmiral_amd import types as T
from oracle.gosem import (GoSort, LabelSelector, Requirement, XorShiftVariant, fnv1_32, go_div, go_f64_to_i64,
                          go_round, go_sort_slice, go_sort_sort, qty_milli_value, qty_value, selector_from_set,
                          tolerates_taint, wrap64, parse_quantity)

SUCCESS, UNSCHEDULABLE, ERROR = 0, 1, 2  # framework/types.go:156-164

# plugins/names/names.go:19-30
APIResources = "APIResources"
TaintToleration = "TaintToleration"
ClusterResourcesFit = "ClusterResourcesFit"
PlacementFilter = "PlacementFilter"
ClusterAffinity = "ClusterAffinity"
ClusterResourcesBalancedAllocation = "ClusterResourcesBalancedAllocation"
ClusterResourcesLeastAllocated = "ClusterResourcesLeastAllocated"
ClusterResourcesMostAllocated = "ClusterResourcesMostAllocated"
MaxCluster = "MaxCluster"
ClusterCapacityWeight = "ClusterCapacityWeight"

MAX_CLUSTER_SCORE = 100  # framework/util.go:53


class Result:
    def __init__(self, code=SUCCESS, reasons=()):
        self.code = code
        self.reasons = list(reasons)

    def is_success(self):
        return self is None or self.code == SUCCESS


def _ok(r):
    return r is None or r.code == SUCCESS


# ================================================================ resources
def is_native_resource(name):  # framework/util.go:390-393
    return "/" not in name or "kubernetes.io/" in name


def is_extended_resource_name(name):  # framework/util.go:369-379
    from oracle.gosem import is_qualified_name
    if is_native_resource(name) or name.startswith("requests."):
        return False
    return is_qualified_name("requests." + name)


def is_scalar_resource_name(name):  # framework/util.go:359-362
    return (is_extended_resource_name(name) or name.startswith("hugepages-") or "kubernetes.io/" in name
            or name.startswith("attachable-volumes-"))


class Resource:
    """framework.Resource with Add / Sub (framework/util.go:71-168)."""

    def __init__(self):
        self.milli_cpu = 0
        self.memory = 0
        self.ephemeral_storage = 0
        self.scalar = None  # map; None ⇔ nil

    @staticmethod
    def new(rl):  # framework/util.go:91-95
        r = Resource()
        r.add(rl)
        return r

    def add(self, rl):  # framework/util.go:98-119
        for name, q in (rl or {}).items():
            if name == "cpu":
                self.milli_cpu = wrap64(self.milli_cpu + qty_milli_value(q))
            elif name == "memory":
                self.memory = wrap64(self.memory + qty_value(q))
            elif name == "ephemeral-storage":
                self.ephemeral_storage = wrap64(self.ephemeral_storage + qty_value(q))
            elif is_scalar_resource_name(name):
                if self.scalar is None:
                    self.scalar = {}
                self.scalar[name] = wrap64(self.scalar.get(name, 0) + qty_value(q))

    def sub(self, rl):  # framework/util.go:123-168 (early return on first error, map order = dict order)
        for name, q in (rl or {}).items():
            if name == "cpu":
                v = qty_milli_value(q)
                if self.milli_cpu < v:
                    return "cpu"
                self.milli_cpu -= v
            elif name == "memory":
                v = qty_value(q)
                if self.memory < v:
                    return "memory"
                self.memory -= v
            elif name == "ephemeral-storage":
                v = qty_value(q)
                if self.ephemeral_storage < v:
                    return "ephemeral-storage"
                self.ephemeral_storage -= v
            elif is_scalar_resource_name(name):
                sc = self.scalar or {}
                v = qty_value(q)
                if name not in sc and v > 0:
                    return name
                rv = sc.get(name, 0)
                if rv < v:
                    return name
                if self.scalar is None:  # Go would panic writing a nil map; only reachable with v <= 0
                    self.scalar = {}
                self.scalar[name] = rv - v
        return None


def cluster_allocatable(c):  # fit.go:140 (getFederatedClusterAllocatableResource)
    return Resource.new(c.allocatable)


def cluster_request(c):  # fit.go:140-147 (getFederatedClusterRequestResource)
    r = Resource.new(c.allocatable)
    r.sub(c.available)
    return r


# ==================================================================== filters
def filter_api_resources(su, c):  # plugins/apiresources/apiresources.go:25-43
    gvk = (su.group, su.version, su.kind)
    for r in c.api_resource_types:
        if (r.group, r.version, r.kind) == gvk:
            return Result(SUCCESS)
    return Result(UNSCHEDULABLE, ["No matched group version kind."])


def find_matching_untolerated_taint(taints, tolerations, pred):  # framework/util.go:421-450
    for t in taints:
        if pred is not None and not pred(t):
            continue
        if not any(tolerates_taint(tol, t) for tol in (tolerations or [])):
            return t, True
    return None, False


def filter_taint_toleration(su, c):  # plugins/tainttoleration/taint_toleration.go:44-89
    scheduled = c.name in (su.current_clusters or {})

    def pred(t):
        if scheduled:
            return t.effect == T.TAINT_NO_EXECUTE
        return t.effect in (T.TAINT_NO_SCHEDULE, T.TAINT_NO_EXECUTE)

    _, untolerated = find_matching_untolerated_taint(c.taints, su.tolerations, pred)
    if not untolerated:
        return Result(SUCCESS)
    return Result(UNSCHEDULABLE, ["taint"])


def fits_request(su, c):  # plugins/clusterresources/fit.go:73-134
    insufficient = []
    req = su.resource_request
    alloc = cluster_allocatable(c)
    used = cluster_request(c)
    if req.milli_cpu == 0 and req.memory == 0 and req.ephemeral_storage == 0 and len(req.scalar_resources or {}) == 0:
        return insufficient
    if alloc.milli_cpu < wrap64(req.milli_cpu + used.milli_cpu):
        insufficient.append("Insufficient cpu")
    if alloc.memory < wrap64(req.memory + used.memory):
        insufficient.append("Insufficient memory")
    for name, q in (req.scalar_resources or {}).items():
        if q <= 0:
            continue
        if (alloc.scalar or {}).get(name, 0) < wrap64(q + (used.scalar or {}).get(name, 0)):
            insufficient.append(f"Insufficient {name}")
    return insufficient


def filter_fit(su, c):  # plugins/clusterresources/fit.go:47-71
    ins = fits_request(su, c)
    if ins:
        return Result(UNSCHEDULABLE, ins)
    return Result(SUCCESS)


def filter_placement(su, c):  # plugins/placement/filter.go:37-57
    if len(su.cluster_names or ()) == 0:
        return Result(SUCCESS)
    if c.name not in su.cluster_names:
        return Result(UNSCHEDULABLE, ["cluster is not in placement list"])
    return Result(SUCCESS)


_OPS = {T.OP_IN: Requirement.IN, T.OP_NOT_IN: Requirement.NOT_IN, T.OP_EXISTS: Requirement.EXISTS,
        T.OP_DOES_NOT_EXIST: Requirement.DNE, T.OP_GT: Requirement.GT, T.OP_LT: Requirement.LT}


def requirements_as_selector(csm):  # util/clusterselector/util.go:31-61 → (selector, err)
    if len(csm or []) == 0:
        return LabelSelector([], nothing=True), False
    reqs = []
    for e in csm:
        op = _OPS.get(e.operator)
        if op is None:
            return None, True
        r, err = Requirement.new(e.key, op, e.values)
        if err:
            return None, True
        reqs.append(r)
    return LabelSelector(reqs), False


def requirements_as_field_selector(csm):  # util/clusterselector/util.go:65-93 → (terms, err)
    if len(csm or []) == 0:
        return ("nothing",), False
    terms = []
    for e in csm:
        if e.operator == T.OP_IN:
            if len(e.values or []) != 1:
                return None, True
            terms.append((e.key, True, e.values[0]))
        elif e.operator == T.OP_NOT_IN:
            if len(e.values or []) != 1:
                return None, True
            terms.append((e.key, False, e.values[0]))
        else:
            return None, True
    return terms, False


def _field_matches(sel, fields):
    if sel == ("nothing",):
        return False
    for key, eq, val in sel:
        got = fields.get(key, "")
        if (got == val) != eq:
            return False
    return True


def match_cluster_selector_terms(terms, c):  # util/clusterselector/util.go:97-132 → (matched, err)
    labels = c.labels
    fields = {"metadata.name": c.name}
    for t in terms or []:
        if len(t.match_expressions or []) == 0 and len(t.match_fields or []) == 0:
            continue
        if len(t.match_expressions or []) != 0:
            sel, err = requirements_as_selector(t.match_expressions)
            if err:
                return False, True
            if not sel.matches(labels):
                continue
        if len(t.match_fields or []) != 0:
            fsel, err = requirements_as_field_selector(t.match_fields)
            if err:
                return False, True
            if not _field_matches(fsel, fields):
                continue
        return True, False
    return False, False


def filter_cluster_affinity(su, c):  # plugins/clusteraffinity/cluster_affinity.go:50-94
    if len(su.cluster_selector or {}) > 0:
        if not selector_from_set(su.cluster_selector).matches(c.labels):
            return Result(UNSCHEDULABLE, ["cluster(s) didn't match cluster selector"])
    aff = su.affinity
    if aff is not None and aff.cluster_affinity is not None:
        ca = aff.cluster_affinity
        if ca.required is None:
            return Result(SUCCESS)
        matched, err = match_cluster_selector_terms(ca.required.cluster_selector_terms, c)
        if err or not matched:
            return Result(UNSCHEDULABLE, ["cluster(s) didn't match cluster selector"])
    return Result(SUCCESS)


# ===================================================================== scores
def default_normalize_score(max_priority, reverse, scores):  # framework/util.go:455-483
    max_count = 0
    for s in scores:
        if s > max_count:
            max_count = s
    if max_count == 0:
        if reverse:
            for i in range(len(scores)):
                scores[i] = max_priority
        return
    for i in range(len(scores)):
        score = go_div(wrap64(max_priority * scores[i]), max_count)
        if reverse:
            score = max_priority - score
        scores[i] = score


def score_taint_toleration(su, c):  # taint_toleration.go:91-113,133-159
    tols = [t for t in (su.tolerations or []) if t.effect in ("", T.TAINT_PREFER_NO_SCHEDULE)]
    n = 0
    for t in c.taints:
        if t.effect != T.TAINT_PREFER_NO_SCHEDULE:
            continue
        if not any(tolerates_taint(tol, t) for tol in tols):
            n += 1
    return n, None


def calculate_resource_allocatable_request(su, c, resource):  # fit.go:153-177
    req = su.resource_request
    alloc = cluster_allocatable(c)
    used = cluster_request(c)
    if resource == "cpu":
        return alloc.milli_cpu, wrap64(used.milli_cpu + req.milli_cpu)
    if resource == "memory":
        return alloc.memory, wrap64(used.memory + req.memory)
    raise AssertionError(resource)


def least_requested_score(requested, capacity):  # least_allocated.go:88-94
    if capacity == 0:
        return 0
    if requested > capacity:
        return 0
    return go_div(wrap64(wrap64(capacity - requested) * MAX_CLUSTER_SCORE), capacity)


def most_requested_score(requested, capacity):  # most_allocated.go:90-97
    if capacity == 0:
        return 0
    if requested > capacity:
        return 0
    return go_div(wrap64(requested * MAX_CLUSTER_SCORE), capacity)


def score_least_allocated(su, c):  # least_allocated.go:42-75 (weights cpu=1, memory=1, util.go:62)
    score, wsum = 0, 0
    for res in ("memory", "cpu"):
        cap, req = calculate_resource_allocatable_request(su, c, res)
        score = wrap64(score + least_requested_score(req, cap))
        wsum += 1
    return go_div(score, wsum), None


def score_most_allocated(su, c):  # most_allocated.go:42-74
    score, wsum = 0, 0
    for res in ("memory", "cpu"):
        cap, req = calculate_resource_allocatable_request(su, c, res)
        score = wrap64(score + most_requested_score(req, cap))
        wsum += 1
    return go_div(score, wsum), None


def fraction_of_capacity(requested, capacity):  # balanced_allocation.go:83-88
    if capacity == 0:
        return 1.0
    return float(requested) / float(capacity)


def score_balanced_allocation(su, c):  # balanced_allocation.go:45-76
    cap_c, req_c = calculate_resource_allocatable_request(su, c, "cpu")
    cap_m, req_m = calculate_resource_allocatable_request(su, c, "memory")
    cf = fraction_of_capacity(req_c, cap_c)
    mf = fraction_of_capacity(req_m, cap_m)
    if cf >= 1 or mf >= 1:
        return 0, None
    diff = abs(cf - mf)
    return go_f64_to_i64((1 - diff) * float(MAX_CLUSTER_SCORE)), None


def score_cluster_affinity(su, c):  # cluster_affinity.go:96-135 → (score, err)
    score = 0
    aff = su.affinity
    if aff is not None and aff.cluster_affinity is not None and aff.cluster_affinity.preferred is not None:
        for term in aff.cluster_affinity.preferred:
            if term.weight == 0:
                continue
            sel, err = requirements_as_selector(term.preference.match_expressions)
            if err:
                return 0, Result(ERROR, ["invalid preferred term"])
            if sel.matches(c.labels):
                score = wrap64(score + term.weight)
    return score, None


# plugin table: name → (filter, score, normalize(max_priority, reverse) or None)
FILTERS = {
    APIResources: filter_api_resources,
    TaintToleration: filter_taint_toleration,
    ClusterResourcesFit: filter_fit,
    PlacementFilter: filter_placement,
    ClusterAffinity: filter_cluster_affinity,
}
SCORES = {
    TaintToleration: (score_taint_toleration, (MAX_CLUSTER_SCORE, True)),
    ClusterResourcesLeastAllocated: (score_least_allocated, None),
    ClusterResourcesMostAllocated: (score_most_allocated, None),
    ClusterResourcesBalancedAllocation: (score_balanced_allocation, None),
    ClusterAffinity: (score_cluster_affinity, (MAX_CLUSTER_SCORE, False)),
}
SELECTS = {MaxCluster}
REPLICAS = {ClusterCapacityWeight}
IN_TREE = set(FILTERS) | set(SCORES) | SELECTS | REPLICAS  # scheduler/profile.go:39-50


# ===================================================================== select
def select_max_cluster(su, cluster_scores, triple=XorShiftVariant.GO119):
    """plugins/maxcluster/max_cluster.go:42-66; cluster_scores: list of [cluster, score]."""
    if su.max_clusters is not None and su.max_clusters < 0:
        return [], Result(UNSCHEDULABLE, ["max cluster is less than 0"])
    go_sort_slice(cluster_scores, lambda x, y: x[1] > y[1], triple)
    length = len(cluster_scores)
    if su.max_clusters is not None and su.max_clusters < length:
        length = su.max_clusters
    return [cluster_scores[i][0] for i in range(length)], Result(SUCCESS)


# ==================================================================== planner
class ClusterPreferences:  # util/planner/planner.go:30-41
    def __init__(self, min_replicas=0, max_replicas=None, weight=0):
        self.min_replicas = min_replicas
        self.max_replicas = max_replicas
        self.weight = weight


class _Named:
    __slots__ = ("name", "hash", "min_replicas", "max_replicas", "weight")


def get_named_preferences(prefs: Dict[str, ClusterPreferences], key: str, triple=XorShiftVariant.GO119):
    """planner.go:179-209: FNV-1 32 of name ‖ key; sort by weight desc, hash asc."""
    out = []
    for name, p in prefs.items():
        n = _Named()
        n.name = name
        n.hash = fnv1_32(name.encode() + key.encode())
        n.min_replicas, n.max_replicas, n.weight = p.min_replicas, p.max_replicas, p.weight
        out.append(n)
    go_sort_sort(out, lambda a, b: (a.weight > b.weight) or (a.weight == b.weight and a.hash < b.hash), triple)
    return out


def get_desired_plan(preferences, estimated_capacity, total_replicas, keep_unschedulable):  # planner.go:211-304
    remaining = total_replicas
    plan = {}
    overflow = {}
    for p in preferences:
        mn = min(p.min_replicas, remaining)
        if estimated_capacity is not None and p.name in estimated_capacity and estimated_capacity[p.name] < mn:
            overflow[p.name] = mn - estimated_capacity[p.name]
            mn = estimated_capacity[p.name]
        remaining = wrap64(remaining - mn)
        plan[p.name] = mn
    modified = True
    while modified and remaining > 0:
        modified = False
        weight_sum = 0
        for p in preferences:
            weight_sum = wrap64(weight_sum + p.weight)
        if weight_sum <= 0:
            break
        new_prefs = []
        distribute = remaining
        for p in preferences:
            start = plan[p.name]
            extra = go_div(wrap64(wrap64(distribute * p.weight) + weight_sum - 1), weight_sum)
            extra = min(extra, remaining)
            total = wrap64(start + extra)
            full = False
            if p.max_replicas is not None and total > p.max_replicas:
                total = p.max_replicas
                full = True
            if estimated_capacity is not None and p.name in estimated_capacity and total > estimated_capacity[p.name]:
                overflow[p.name] = overflow.get(p.name, 0) + total - estimated_capacity[p.name]
                total = estimated_capacity[p.name]
                full = True
            if not full:
                new_prefs.append(p)
            remaining = wrap64(remaining - (total - start))
            plan[p.name] = total
            if total > start:
                modified = True
        preferences = new_prefs
    if keep_unschedulable:
        return plan, overflow
    new_overflow = {}
    for k, v in overflow.items():
        v = min(v, remaining)
        if v > 0:
            new_overflow[k] = v
    return plan, new_overflow


def scale_up(rsp_clusters, current, desired, count, key, triple):  # planner.go:306-338
    prefs = {}
    for cluster, d in desired.items():
        cur = current.get(cluster, 0)
        if d > cur:
            p = ClusterPreferences(weight=d - cur)
            rp = rsp_clusters.get(cluster)
            if rp is not None and rp.max_replicas is not None:
                p.max_replicas = rp.max_replicas - cur
            prefs[cluster] = p
    named = get_named_preferences(prefs, key, triple)
    up, _ = get_desired_plan(named, None, count, False)
    for cluster, n in up.items():
        current[cluster] = current.get(cluster, 0) + n
    return current


def scale_down(current, desired, count, key, triple):  # planner.go:340-366
    prefs = {}
    for cluster, d in desired.items():
        cur = current.get(cluster, 0)
        if d < cur:
            prefs[cluster] = ClusterPreferences(weight=cur - d, max_replicas=cur)
    named = get_named_preferences(prefs, key, triple)
    down, _ = get_desired_plan(named, None, count, False)
    for cluster, n in down.items():
        current[cluster] = current.get(cluster, 0) - n
    return current


def plan(rsp_clusters: Dict[str, ClusterPreferences], total_replicas, available_clusters, current_replica_count,
         estimated_capacity, key, avoid_disruption, keep_unschedulable, triple=XorShiftVariant.GO119):
    """planner.Plan (planner.go:83-177) → (plan, overflow)."""
    prefs = {}
    for c in available_clusters:
        if c in rsp_clusters:
            prefs[c] = rsp_clusters[c]
        elif "*" in rsp_clusters:
            prefs[c] = rsp_clusters["*"]
    named = get_named_preferences(prefs, key, triple)
    if not avoid_disruption:
        keep_unschedulable = True
    desired, desired_overflow = get_desired_plan(named, estimated_capacity, total_replicas, keep_unschedulable)
    if not avoid_disruption:
        return desired, desired_overflow
    current_total = 0
    current_plan = {}
    for p in named:
        r = (current_replica_count or {}).get(p.name, 0)
        if estimated_capacity is not None and p.name in estimated_capacity and estimated_capacity[p.name] < r:
            r = estimated_capacity[p.name]
        current_plan[p.name] = r
        current_total = wrap64(current_total + r)
    desired_total = 0
    for r in desired.values():
        desired_total = wrap64(desired_total + r)
    if current_total == desired_total:
        return current_plan, desired_overflow
    if current_total > desired_total:
        return scale_down(current_plan, desired, current_total - desired_total, key, triple), desired_overflow
    return scale_up(rsp_clusters, current_plan, desired, desired_total - current_total, key, triple), desired_overflow


# ======================================================================== rsp
SUPPLY_LIMIT_PROPORTION = 1.4  # rsp.go:42
SUM_WEIGHT = 1000.0  # rsp.go:43


def _query_cpu(clusters, which):  # rsp.go:286-325 (QueryAvailable / QueryAllocatable), cpu only
    out = {}
    for c in clusters:
        rl = c.available if which == "available" else c.allocatable
        q = parse_quantity("0")
        if rl is not None and "cpu" in rl:
            q = q + parse_quantity(rl["cpu"])
        out[c.name] = q
    return out


def _value(q):
    from oracle.gosem import _ceil_away
    return _ceil_away(q)


def calc_weight_limit(clusters, supply_limit_ratio):  # rsp.go:183-213 → (map, err)
    alloc = _query_cpu(clusters, "allocatable")
    if len(alloc) != len(clusters):
        return None, "allocatables are incomplete"
    s = 0.0
    for q in alloc.values():
        s += float(_value(q))
    wl = {}
    if s == 0:
        for m in alloc:
            wl[m] = go_f64_to_i64(go_round(SUM_WEIGHT / float(len(alloc))))
        return wl, None
    for m, q in alloc.items():
        wl[m] = go_f64_to_i64(go_round(float(_value(q)) / s * SUM_WEIGHT * supply_limit_ratio))
    return wl, None


def available_to_percentage(avail_cpu: Dict[str, object], weight_limit, tie_pick=None):
    """rsp.go:215-272 → (weights, tied_max_candidates).

    ``avail_cpu``: member → cpu Quantity (Fraction). The remainder
    ``1000 - Σ`` goes to the first strictly-max member in Go map order; the
    reference is non-deterministic when several members tie. ``tie_pick``
    picks among the tied candidates (default: first in ``avail_cpu`` order).
    """
    sum_avail = 0.0
    for q in avail_cpu.values():
        v = _value(q)
        if v > 0.0:
            sum_avail += float(v)
    weights = {}
    if sum_avail == 0:
        for m in avail_cpu:
            weights[m] = go_f64_to_i64(go_round(SUM_WEIGHT / float(len(avail_cpu))))
        return weights, []
    tmp = {}
    sum_tmp = 0
    for m, q in avail_cpu.items():
        v = float(_value(q))
        if v < 0.0:
            v = 0.0
        w = go_f64_to_i64(go_round(v / sum_avail * SUM_WEIGHT))
        if w > weight_limit.get(m, 0):
            w = weight_limit.get(m, 0)
        tmp[m] = w
        sum_tmp = wrap64(sum_tmp + w)
    other_sum = 0
    max_w = 0
    cands = []
    for m, tw in tmp.items():
        if sum_tmp == 0:
            w = go_f64_to_i64(float("nan"))
        else:
            w = go_f64_to_i64(go_round(float(tw) / float(sum_tmp) * SUM_WEIGHT))
        if w > max_w:
            max_w = w
            cands = [m]
        elif w == max_w and max_w > 0:
            cands.append(m)
        weights[m] = w
        other_sum = wrap64(other_sum + w)
    if not cands:
        cands = [""]
    pick = cands[0] if tie_pick is None else tie_pick(cands)
    weights[pick] = wrap64(weights.get(pick, 0) + int(SUM_WEIGHT) - other_sum)
    return weights, cands


def replica_scheduling(su, clusters, triple=XorShiftVariant.GO119, tie_pick=None, info=None):
    """ClusterCapacityWeight.ReplicaScheduling (rsp.go:65-181) → (list[(cluster, replicas)], Result)."""
    dynamic = len(su.weights or {}) == 0
    if dynamic:
        avail = _query_cpu(clusters, "available")
        if len(clusters) != len(avail):
            return [], Result(ERROR)
        wl, err = calc_weight_limit(clusters, SUPPLY_LIMIT_PROPORTION)
        if err:
            return [], Result(ERROR)
        weights, cands = available_to_percentage(avail, wl, tie_pick)
        if info is not None:
            info["remainder_candidates"] = cands
    else:
        weights = su.weights
    prefs = {}
    for c in clusters:
        p = ClusterPreferences(weight=weights.get(c.name, 0), min_replicas=(su.min_replicas or {}).get(c.name, 0))
        if su.max_replicas is not None and c.name in su.max_replicas:
            p.max_replicas = su.max_replicas[c.name]
        prefs[c.name] = p
    total = su.desired_replicas if su.desired_replicas is not None else 0
    current = {}
    for name, r in (su.current_clusters or {}).items():
        current[name] = r if r is not None else total
    est = {}
    keep = False
    if su.auto_migration is not None:
        keep = su.auto_migration.keep_unschedulable_replicas
        for name, ec in (su.auto_migration.estimated_capacity or {}).items():
            if ec >= 0:
                est[name] = ec
    pl, ov = plan(prefs, total, [c.name for c in clusters], current, est, su.key(), su.avoid_disruption, keep, triple)
    result = dict(pl)
    for name, r in ov.items():
        result[name] = result.get(name, 0) + r
    out = []
    for c in clusters:
        r = result.get(c.name)
        if r is None or r == 0:
            continue
        out.append((c, r))
    return out, Result(SUCCESS)


# ============================================================== framework
class FrameworkError(Exception):
    pass


class EnabledPlugins:  # pkg/apis/core/types.go:21-43
    def __init__(self, filter=(), score=(), select=(), replicas=()):
        self.filter_plugins = list(filter)
        self.score_plugins = list(score)
        self.select_plugins = list(select)
        self.replicas_plugins = list(replicas)


def default_enabled_plugins():  # apis/core/v1alpha1/extensions_schedulingprofile.go:24-49
    return EnabledPlugins(
        [APIResources, TaintToleration, ClusterResourcesFit, PlacementFilter, ClusterAffinity],
        [TaintToleration, ClusterResourcesBalancedAllocation, ClusterResourcesLeastAllocated, ClusterAffinity],
        [MaxCluster], [ClusterCapacityWeight])


class Framework:
    """runtime.frameworkImpl (framework/runtime/framework.go:36-68) over in-tree plugins."""

    def __init__(self, enabled: EnabledPlugins, registry=None):
        registry = set(IN_TREE if registry is None else registry)
        for point, names, impl in (("FilterPlugin", enabled.filter_plugins, FILTERS),
                                   ("ScorePlugin", enabled.score_plugins, SCORES),
                                   ("SelectPlugin", enabled.select_plugins, SELECTS),
                                   ("ReplicasPlugin", enabled.replicas_plugins, REPLICAS)):
            seen = set()
            for n in names:  # framework.go:70-95 (addPlugins)
                if n not in registry:
                    raise FrameworkError(f"{point} {n} does not exist")
                if n not in impl:
                    raise FrameworkError(f"plugin {n} does not implement {point}")
                if n in seen:
                    raise FrameworkError(f"plugin {n} already registered as {point}")
                seen.add(n)
        self.filters = list(enabled.filter_plugins)
        self.scores = list(enabled.score_plugins)
        self.selects = list(enabled.select_plugins)
        self.replicas = list(enabled.replicas_plugins)

    def run_filter_plugins(self, su, c):  # framework.go:114-126
        for n in self.filters:
            r = FILTERS[n](su, c)
            if not _ok(r):
                return r
        return Result(SUCCESS)

    def run_score_plugins(self, su, clusters):  # framework.go:139-181
        out = {}
        for n in self.scores:
            fn, norm = SCORES[n]
            lst = []
            for c in clusters:
                s, res = fn(su, c)
                if res is not None and not _ok(res):
                    return None, Result(ERROR, [n])
                lst.append(s)
            if norm is not None:
                default_normalize_score(norm[0], norm[1], lst)
            out[n] = lst
        return out, None

    def run_select_plugin(self, su, scored, triple):  # framework.go:183-209
        if not self.selects:
            return [c for c, _ in scored], Result(SUCCESS)
        for n in self.selects:
            clusters, res = select_max_cluster(su, scored, triple)
            if not _ok(res):
                return clusters, Result(ERROR, [n])
            return clusters, res

    def run_replicas_plugin(self, su, clusters, triple, tie_pick, info):  # framework.go:211-249
        if len(clusters) == 0:
            return [], Result(SUCCESS)
        if su.desired_replicas is None or su.desired_replicas <= 0:
            return [], Result(SUCCESS)
        if not self.replicas:
            return [], Result(SUCCESS)
        for n in self.replicas:
            lst, res = replica_scheduling(su, clusters, triple, tie_pick, info)
            if not _ok(res):
                return lst, Result(ERROR, [n])
            return lst, res


def reconcile_ext_point(enabled, enabled_names, disabled_names):  # scheduler/profile.go:62-82
    disabled = set(disabled_names)
    result = []
    if "*" not in disabled:
        result = [e for e in enabled if e not in disabled]
    result.extend(enabled_names)
    return result


def apply_profile(base: EnabledPlugins, profile_plugins):  # scheduler/profile.go:52-60
    """profile_plugins: None or {"filter": {"enabled": [...], "disabled": [...]}, "score": ..., "select": ...}."""
    if profile_plugins is None:
        return base
    for point, attr in (("filter", "filter_plugins"), ("score", "score_plugins"), ("select", "select_plugins")):
        ps = profile_plugins.get(point) or {}
        setattr(base, attr, reconcile_ext_point(getattr(base, attr), ps.get("enabled") or [], ps.get("disabled") or []))
    return base


# ============================================================== scheduler
def schedule(fwk: Framework, su: T.SchedulingUnit, clusters: List[T.FederatedCluster],
             triple=XorShiftVariant.GO119, tie_pick=None, info=None) -> T.ScheduleResult:
    """genericScheduler.Schedule (core/generic_scheduler.go:92-150).

    Raises ``T.ScheduleError`` for the error returns. ``tie_pick`` picks the
    AvailableToPercentage remainder recipient among tied maxima (default:
    the candidate with the lowest index in ``clusters`` — the product's rule).
    """
    if tie_pick is None:
        order = {c.name: i for i, c in enumerate(clusters)}
        tie_pick = lambda cands: min(cands, key=lambda n: order.get(n, 1 << 62))  # noqa: E731
    if su.sticky_cluster and len(su.current_clusters or {}) > 0:
        return T.ScheduleResult(su.current_clusters)
    feasible = [c for c in clusters if _ok(fwk.run_filter_plugins(su, c))]  # :152-169
    if info is not None:
        info["feasible"] = [c.name for c in feasible]
    if len(feasible) == 0:
        return T.ScheduleResult(None)
    scores, res = fwk.run_score_plugins(su, feasible)  # :171-192
    if res is not None and not _ok(res):
        raise T.ScheduleError("scoreClusters")
    totals = [0] * len(feasible)
    for lst in scores.values():
        for i, s in enumerate(lst):
            totals[i] = wrap64(totals[i] + s)
    if info is not None:
        info["scores"] = {k: list(v) for k, v in scores.items()}
        info["totals"] = list(totals)
    selected, res = fwk.run_select_plugin(su, [[c, s] for c, s in zip(feasible, totals)], triple)  # :194-205
    if not _ok(res):
        raise T.ScheduleError("selectClusters")
    if info is not None:
        info["selected"] = [c.name for c in selected]
    if su.scheduling_mode == T.SCHEDULING_MODE_DUPLICATE:  # :130-137
        return T.ScheduleResult({c.name: None for c in selected})
    lst, res = fwk.run_replicas_plugin(su, selected, triple, tie_pick, info)  # :207-218
    if not _ok(res):
        raise T.ScheduleError("replicaScheduling")
    return T.ScheduleResult({c.name: r for c, r in lst})


def schedule_or_error(fwk, su, clusters, **kw):
    """Schedule → ("ok", ScheduleResult) | ("error", stage)."""
    try:
        return "ok", schedule(fwk, su, clusters, **kw)
    except T.ScheduleError as e:
        return "error", e.stage

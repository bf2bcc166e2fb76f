"""Federated object ↔ SchedulingUnit, result application, trigger bytes (CPU).

The reference's own test tables (scheduler_test.go TestGetSchedulingUnit*, TestSchedulingMode,
util_test.go TestMatchedPolicyKey) run from extracted fixtures in ``tests/test_objects_golden.py``;
this file holds edge cases read from ``schedulingunit.go`` / ``util.go`` /
``util/overrides.go`` (marked with the lines they follow), and the trigger
JSON against the independent restatement in oracle/triggers.py.
"""

import json
import random

import pytest

from kubeadmiral_amd import gojson as J
from kubeadmiral_amd import objects as O
from kubeadmiral_amd import types as T
from kubeadmiral_amd.gosort import sort_slice
from oracle import triggers as OT
from oracle.gosem import GoSort, fnv1_32

P = O.DEFAULT_PREFIX
DEPLOY_FTC = O.FederatedTypeConfig("apps", "v1", "Deployment", "deployments", "Namespaced", "spec.replicas")


def _policy(**spec):
    return O.PropagationPolicy("pp", "default", 1, O.PropagationPolicySpec(**spec))


def _bare_obj(annotations=None):
    # scheduler_test.go:398-402: empty object with annotations and an empty template
    obj = {"spec": {"template": {}}}
    if annotations is not None:
        obj["metadata"] = {"annotations": annotations}
    return obj


# ------------------------------------------------------------ edge cases read from schedulingunit.go
def _su(ann=None, ftc=DEPLOY_FTC, obj=None, **spec):
    return O.scheduling_unit_for_fed_object(ftc, obj if obj is not None else _bare_obj(ann), _policy(**spec))


def test_invalid_annotations_fall_back_to_policy():
    # :245-258, :290-303, :322-331, :365-374, :395-404, :424-444 — bad values log and keep the policy's
    su = _su({O.SCHEDULING_MODE_ANNOTATION: "Spread", O.STICKY_CLUSTER_ANNOTATION: "yes",
              O.CLUSTER_SELECTOR_ANNOTATIONS: '{"a": 1}', O.AFFINITY_ANNOTATIONS: "{",
              O.TOLERATIONS_ANNOTATIONS: '{"key": "x"}', O.MAX_CLUSTERS_ANNOTATIONS: "ten"},
             scheduling_mode="Divide", sticky_cluster=True, cluster_selector={"x": "y"}, max_clusters=3,
             tolerations=[T.Toleration("t", "Exists")])
    assert su.scheduling_mode == "Divide" and su.sticky_cluster is True
    assert su.cluster_selector == {"x": "y"} and su.max_clusters == 3 and su.affinity is None
    assert su.tolerations == [T.Toleration("t", "Exists")]


@pytest.mark.parametrize("v,want", [("10", 10), ("+7", 7), ("007", 7), ("0", 0), ("-1", 3), (" 5", 3), ("5.0", 3),
                                    ("", 3), ("9223372036854775807", 9223372036854775807),
                                    ("9223372036854775808", 3), ("1_000", 3)])
def test_max_clusters_annotation_atoi(v, want):  # :424-447 strconv.Atoi, negative rejected
    assert _su({O.MAX_CLUSTERS_ANNOTATIONS: v}, max_clusters=3).max_clusters == want


def test_placements_annotation_negative_values_rejected_per_field():
    # :495-505, :551-561, :611-621: a negative weight drops only the weights override, and so on
    ann = {O.PLACEMENTS_ANNOTATIONS: json.dumps([
        {"cluster": "a", "preferences": {"minReplicas": 1, "maxReplicas": -2, "weight": -1}},
        {"cluster": "b"}])}
    su = _su(ann, placements=[O.Placement("p", O.Preferences(3, 4, 5))])
    assert su.cluster_names == {"a", "b"}
    assert su.min_replicas == {"a": 1, "b": 0}
    assert su.max_replicas == {"p": 4}          # annotation rejected (negative maxReplicas)
    assert su.weights == {"p": 5}               # annotation rejected (negative weight)


def test_json_null_and_case_insensitive_keys():
    # json.Unmarshal: "null" into a map/slice gives nil; struct fields match keys case-insensitively
    ann = {O.CLUSTER_SELECTOR_ANNOTATIONS: "null", O.TOLERATIONS_ANNOTATIONS: "null",
           O.PLACEMENTS_ANNOTATIONS: '[{"CLUSTER": "x", "Preferences": {"WEIGHT": 4, "minreplicas": 2}}]',
           O.AFFINITY_ANNOTATIONS: '{"ClusterAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": '
                                   '{"clusterSelectorTerms": []}}}'}
    su = _su(ann, cluster_selector={"a": "b"}, tolerations=[T.Toleration("t")])
    assert su.cluster_selector is None and su.tolerations is None
    assert su.weights == {"x": 4} and su.min_replicas == {"x": 2} and su.cluster_names == {"x"}
    assert su.affinity == T.Affinity(T.ClusterAffinity(required=T.ClusterSelector([])))
    # "null" placements: an empty (non-nil) list → empty maps
    su = _su({O.PLACEMENTS_ANNOTATIONS: "null"}, placements=[O.Placement("p")])
    assert su.cluster_names == set() and su.min_replicas == {} and su.weights == {}


def test_int_fields_reject_floats_and_overflow():
    for bad in ('[{"cluster": "a", "preferences": {"weight": 1.0}}]',
                '[{"cluster": "a", "preferences": {"weight": 9223372036854775808}}]',
                '[{"cluster": "a", "preferences": {"minReplicas": "1"}}]'):
        su = _su({O.PLACEMENTS_ANNOTATIONS: bad}, placements=[O.Placement("p")])
        assert su.cluster_names == {"p"}
    # PreferredSchedulingTerm.Weight is int32
    aff = '{"clusterAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [{"weight": 2147483648}]}}'
    assert _su({O.AFFINITY_ANNOTATIONS: aff}).affinity is None


def test_affinity_from_policy_and_divide_replicas():
    terms = [T.ClusterSelectorTerm([T.ClusterSelectorRequirement("k", "Exists")])]
    obj = _bare_obj()
    obj["spec"]["template"] = {"metadata": {"name": "n", "namespace": "ns"}, "spec": {"replicas": 7}}
    su = _su(obj=obj, scheduling_mode="Divide", cluster_affinity=terms)
    assert su.desired_replicas == 7 and su.scheduling_mode == "Divide" and su.key() == "ns/n"
    assert su.affinity == T.Affinity(T.ClusterAffinity(required=T.ClusterSelector(terms)))
    assert _su(cluster_affinity=[]).affinity is None  # :338 len == 0 → nil
    # Divide without replicas in the template: DesiredReplicas nil
    assert _su(scheduling_mode="Divide").desired_replicas is None
    obj["spec"]["template"]["spec"]["replicas"] = "7"
    with pytest.raises(O.ObjectError):
        _su(obj=obj, scheduling_mode="Divide")


def test_template_required():
    with pytest.raises(O.ObjectError):
        O.scheduling_unit_for_fed_object(DEPLOY_FTC, {"spec": {}}, _policy())


def test_current_clusters_from_placements_and_overrides():
    # getCurrentReplicasFromObject :181-222
    obj = _bare_obj()
    obj["spec"]["placements"] = [
        {"controller": "other", "placement": {"clusters": [{"name": "z"}]}},
        {"controller": O.PREFIXED_GLOBAL_SCHEDULER_NAME,
         "placement": {"clusters": [{"name": "a"}, {"name": "b"}, {"name": "c"}, {"name": "d"}]}}]
    obj["spec"]["overrides"] = [{"controller": O.PREFIXED_GLOBAL_SCHEDULER_NAME, "clusters": [
        {"clusterName": "a", "paths": [{"path": "/spec/replicas", "value": 3}]},
        {"clusterName": "b", "paths": [{"op": "add", "path": "/spec/replicas", "value": 4},
                                       {"op": "replace", "path": "/spec/replicas", "value": 5.9}]},
        {"clusterName": "c", "paths": [{"path": "/spec/paused", "value": True}]},
        {"clusterName": "x", "paths": [{"path": "/spec/replicas", "value": 9}]}]}]
    su = _su(obj=obj)
    assert su.current_clusters == {"a": 3, "b": 5, "c": None, "d": None}
    obj["spec"]["overrides"][0]["clusters"][0]["paths"][0]["value"] = "3"
    with pytest.raises(O.GoPanic):  # override.Value.(float64) on a string
        _su(obj=obj)
    obj["spec"]["overrides"][0]["clusters"][0]["paths"][0] = {"path": "/metadata/name", "value": "x"}
    with pytest.raises(O.ObjectError):  # util/overrides.go:102-106
        _su(obj=obj)
    obj["spec"]["overrides"][0]["clusters"][0] = {"clusterName": "b"}
    with pytest.raises(O.ObjectError):  # duplicate cluster, :96-99
        _su(obj=obj)


def test_auto_migration_info():
    am = O.AutoMigration(keep_unschedulable_replicas=True)
    su = _su({O.AUTO_MIGRATION_INFO_ANNOTATION: '{"estimatedCapacity": {"a": 3, "b": -1}}'}, auto_migration=am)
    assert su.auto_migration == T.AutoMigrationSpec({"a": 3, "b": -1}, True)
    with pytest.raises(O.ObjectError):  # :268-270 the error propagates
        _su({O.AUTO_MIGRATION_INFO_ANNOTATION: '{"estimatedCapacity": {"a": "3"}}'}, auto_migration=am)
    # without auto migration in the policy the annotation is not read
    assert _su({O.AUTO_MIGRATION_INFO_ANNOTATION: "{"}).auto_migration is None


def test_policy_from_json_and_replica_rescheduling():
    pol = O.PropagationPolicy.from_json({
        "metadata": {"name": "p", "namespace": "ns", "generation": 4},
        "spec": {"schedulingMode": "Divide", "stickyCluster": True, "maxClusters": 2,
                 "placement": [{"cluster": "a", "preferences": {"weight": 3}}],
                 "autoMigration": {"when": {"podUnschedulableFor": "1m"}, "keepUnschedulableReplicas": True},
                 "replicaRescheduling": {"avoidDisruption": True}}})
    assert pol.generation == 4 and pol.spec.auto_migration.when.pod_unschedulable_for == "1m"
    su = O.scheduling_unit_for_fed_object(DEPLOY_FTC, _bare_obj(), pol)
    assert su.avoid_disruption is True and su.sticky_cluster and su.max_clusters == 2 and su.weights == {"a": 3}
    assert su.min_replicas == {"a": 0} and su.max_replicas == {} and su.cluster_names == {"a"}


# ------------------------------------------------------------ f3: result application
def test_apply_scheduling_result_round_trip():
    obj = _bare_obj()
    obj["metadata"] = {"name": "o", "namespace": "ns"}
    res = T.ScheduleResult({"b": 2, "a": 3})
    assert O.apply_scheduling_result(DEPLOY_FTC, obj, res, True, None)
    assert obj["spec"]["placements"] == [{"controller": O.PREFIXED_GLOBAL_SCHEDULER_NAME,
                                          "placement": {"clusters": [{"name": "a"}, {"name": "b"}]}}]
    assert obj["spec"]["overrides"] == [{"controller": O.PREFIXED_GLOBAL_SCHEDULER_NAME, "clusters": [
        {"clusterName": "a", "paths": [{"path": "/spec/replicas", "value": 3.0}]},
        {"clusterName": "b", "paths": [{"path": "/spec/replicas", "value": 2.0}]}]}]
    assert obj["metadata"]["annotations"] == {O.ENABLE_FOLLOWER_SCHEDULING_ANNOTATION: "true"}
    # the unit the next reconcile builds sees the result as its current clusters
    assert O.get_current_replicas(DEPLOY_FTC, obj) == {"a": 3, "b": 2}
    # same result again: nothing changes
    assert not O.apply_scheduling_result(DEPLOY_FTC, obj, res, True, None)
    # shrink to one cluster, keep another controller's override patch, add the threshold annotation
    obj["spec"]["overrides"][0]["clusters"][1]["paths"].append({"path": "/spec/paused", "value": True})
    assert O.apply_scheduling_result(DEPLOY_FTC, obj, T.ScheduleResult({"a": 1}), False, 90 * 10**9)
    assert obj["spec"]["placements"][0]["placement"]["clusters"] == [{"name": "a"}]
    assert obj["spec"]["overrides"][0]["clusters"] == [
        {"clusterName": "a", "paths": [{"path": "/spec/replicas", "value": 1.0}]},
        {"clusterName": "b", "paths": [{"path": "/spec/paused", "value": True}]}]
    assert obj["metadata"]["annotations"] == {O.ENABLE_FOLLOWER_SCHEDULING_ANNOTATION: "false",
                                              O.POD_UNSCHEDULABLE_THRESHOLD_ANNOTATION: "1m30s"}
    # no clusters: placement entry removed, replicas overrides removed
    assert O.apply_scheduling_result(DEPLOY_FTC, obj, T.ScheduleResult({}), False, None)
    assert obj["spec"]["placements"] == []
    assert obj["spec"]["overrides"][0]["clusters"] == [
        {"clusterName": "b", "paths": [{"path": "/spec/paused", "value": True}]}]
    assert O.POD_UNSCHEDULABLE_THRESHOLD_ANNOTATION not in obj["metadata"]["annotations"]


def test_duplicate_mode_result_has_no_overrides():
    obj = _bare_obj()
    assert O.apply_scheduling_result(DEPLOY_FTC, obj, T.ScheduleResult({"a": None, "b": None}), True, None)
    assert "overrides" not in obj["spec"]
    assert O.get_current_replicas(DEPLOY_FTC, obj) == {"a": None, "b": None}


@pytest.mark.parametrize("ns,want", [(0, "0s"), (1, "1ns"), (1500, "1.5µs"), (2 * 10**6, "2ms"),
                                     (1500 * 10**6, "1.5s"), (90 * 10**9, "1m30s"), (3600 * 10**9, "1h0m0s"),
                                     (-61 * 10**9, "-1m1s"), (10**9 + 1, "1.000000001s")])
def test_duration_string(ns, want):  # time.Duration.String
    assert O.duration_string(ns) == want


@pytest.mark.parametrize("s,want", [("1m30s", 90 * 10**9), ("1.5h", 5400 * 10**9), ("300ms", 3 * 10**8),
                                    ("-2s", -2 * 10**9), ("0", 0), ("1h2m3s4ms5us6ns", 3723004005006)])
def test_parse_duration(s, want):
    assert O.parse_duration(s) == want


@pytest.mark.parametrize("s", ["", "1", "1x", "s", "--1s"])
def test_parse_duration_errors(s):
    with pytest.raises(O.ObjectError):
        O.parse_duration(s)


def test_add_annotation():
    obj = {}
    assert O.add_annotation(obj, O.SCHEDULING_TRIGGER_HASH_ANNOTATION, "123")
    assert not O.add_annotation(obj, O.SCHEDULING_TRIGGER_HASH_ANNOTATION, "123")
    assert O.add_annotation(obj, O.SCHEDULING_TRIGGER_HASH_ANNOTATION, "124")
    assert obj == {"metadata": {"annotations": {O.SCHEDULING_TRIGGER_HASH_ANNOTATION: "124"}}}


# ------------------------------------------------------------ Go sort / JSON encoding
def test_gosort_matches_oracle_with_inconsistent_comparators():
    rng = random.Random(5)
    comparators = [
        lambda a, b: a[0] < b[0],                                # ties (unstable pdqsort)
        lambda a, b: a[0] != b[0],                               # schedulingtriggers.go:249-250 style
        lambda a, b: (a[0] < b[0]) if a[1] != b[1] else a[0] != b[0],
    ]
    for trial in range(300):
        n = rng.choice([0, 1, 5, 12, 13, 20, 49, 50, 51, 80, 200])
        items = [(rng.randrange(6), rng.randrange(3), i) for i in range(n)]
        less = comparators[trial % 3]
        a = list(items)
        sort_slice(a, less)
        b = list(items)

        def lt(i, j, b=b, less=less):
            return less(b[i], b[j])

        def sw(i, j, b=b):
            b[i], b[j] = b[j], b[i]

        GoSort(lt, sw).sort(len(b))
        assert a == b, (trial, n)


@pytest.mark.parametrize("s", ["plain", "<a&b>", 'q"uo\\te', "ctl\x00\x01\x08\x0c\x1f\x7f", "nl\n\r\t",
                               "unié中\U0001f600", "sep  ", "sur\ud800x"])
def test_go_string_encoding(s):
    assert J.encode_string(s) == OT._go_string(s)


def _rand_str(rng, n=6):
    alphabet = "abcXYZ09-._/<>&\"\\ \né \x01"
    return "".join(rng.choice(alphabet) for _ in range(rng.randrange(n)))


def _rand_clusters(rng, C):
    out = []
    for i in range(C):
        labels = None if rng.random() < 0.2 else {_rand_str(rng): _rand_str(rng) for _ in range(rng.randrange(5))}
        taints = [T.Taint(rng.choice(["k1", "k2", "k3"]), rng.choice(["", "v", "w"]),
                          rng.choice(["NoSchedule", "NoExecute", "PreferNoSchedule"]))
                  for _ in range(rng.choice([0, 1, 3, 13, 30]))]
        apis = [T.APIResource(rng.choice(["", "apps", "batch"]), rng.choice(["v1", "v2"]),
                              rng.choice(["Deployment", "Job", "StatefulSet"]), rng.choice(["a", "b"]),
                              rng.choice(["Namespaced", "Cluster"])) for _ in range(rng.choice([0, 2, 12, 25]))]
        name = f"c{rng.randrange(C * 2)}" if rng.random() < 0.9 else _rand_str(rng) + str(i)
        out.append(T.FederatedCluster(name, labels, taints, apis))
    return out


def test_trigger_bytes_match_oracle_restatement():
    rng = random.Random(11)
    keys = list(OT.KNOWN) + ["other/annotation", OT.AUTO_MIGRATION_INFO]
    for trial in range(60):
        clusters = _rand_clusters(rng, rng.choice([0, 1, 4, 17]))
        suffix = O.trigger_suffix(clusters)
        for _ in range(5):
            ann = {k: _rand_str(rng, 12) for k in rng.sample(keys, rng.randrange(len(keys)))}
            obj = {"metadata": {"annotations": ann}, "spec": {"template": {"spec": {}}}}
            reps = rng.choice([None, 0, 5, -3, 2**40])
            if reps is not None:
                obj["spec"]["template"]["spec"]["replicas"] = reps
            ftc = O.FederatedTypeConfig(replicas_spec=rng.choice(["spec.replicas", ""]))
            pol = None
            if rng.random() < 0.8:
                pol = O.PropagationPolicy(_rand_str(rng), "ns", rng.randrange(100), O.PropagationPolicySpec(
                    auto_migration=O.AutoMigration() if rng.random() < 0.5 else None))
            got = O.trigger_prefix(ftc, obj, pol) + suffix
            rc = O.get_replica_count(ftc, obj)
            want = OT.trigger_json(ann, rc, None if pol is None else (pol.name, pol.generation,
                                                                      pol.spec.auto_migration is not None), clusters)
            assert got == want, trial
            assert json.loads(got.decode())  # well-formed


def test_trigger_hash_format():
    # strconv.FormatInt(int64(uint32)): always the unsigned decimal
    assert O.format_trigger_hash(0xFFFFFFFF) == "4294967295"
    b = O.trigger_prefix(DEPLOY_FTC, _bare_obj(), None) + O.trigger_suffix([])
    assert b == (b'{"schedulingAnnotations":[],"replicaCount":0,"resourceRequest":{"millicpu":0,"memory":0,'
                 b'"ephemeralStorage":0,"scalarResources":null},"policyName":"","policyGeneration":0,'
                 b'"clusterLabels":[],"clusterTaints":[],"clusterAPIResourceTypes":[]}')
    assert O.format_trigger_hash(fnv1_32(b)) == OT.trigger_hash({}, 0, None, [])


def test_go_string_encoder_equals_its_restatement():
    """gojson._enc_str (the C encoder where Go agrees, a translate table elsewhere) == the per-character
    restatement of encodeState.string, on strings over every class of character."""
    rng = random.Random(17)
    pool = [chr(c) for c in range(0x80)] + [" ", " ", "\ud800", "\udfff", "\ud83d", "é", "😀", "�"]
    for i in range(20000):
        s = "".join(rng.choice(pool) for _ in range(rng.randint(0, 24)))
        if i % 2:  # the fast path: nothing Go and Python encode differently
            s = "".join(ch for ch in s if ch not in "<>&\x08\x0c  " and not 0xD800 <= ord(ch) <= 0xDFFF)
        a, b = [], []
        J._enc_str(s, a)
        J._enc_str_ref(s, b)
        assert a == ["".join(b)], repr(s)

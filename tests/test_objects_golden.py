"""f2 — SchedulingUnit from federated objects and policies, against the reference's own test tables.

The cases come from ``tests/golden/schedulingunit.json`` and ``matched_policy.json``, which
``tests/golden/extract_golden.py`` reads out of the reference's tests (the literal objects, policies,
annotations and expected SchedulingUnits, with the file:line of each case):

* ``pkg/controllers/scheduler/scheduler_test.go`` TestGetSchedulingUnit, TestGetSchedulingUnitWithAnnotationOverrides,
  TestSchedulingMode
* ``pkg/controllers/scheduler/util_test.go`` TestMatchedPolicyKey

Each runs through the product's ``objects.scheduling_unit_for_fed_object`` / ``matched_policy_key`` and is compared
the way the Go test compares (gomega.Equal after the test's own field overwrites).
"""
import pytest

from golden_util import load
from kubeadmiral_amd import objects as O
from kubeadmiral_amd import types as T

SU = load("schedulingunit.json")
MP = load("matched_policy.json")


def _lower_keys(v):
    if isinstance(v, list):
        return [_lower_keys(x) for x in v]
    if isinstance(v, dict):
        return {k[0].lower() + k[1:]: _lower_keys(x) for k, x in v.items()}
    return v


def _want_su(d) -> T.SchedulingUnit:
    """The Go literal's framework.SchedulingUnit (Go field names) as the repo's type."""
    d = dict(d)
    if "ClusterNames" in d and isinstance(d["ClusterNames"], dict):
        d["ClusterNames"] = list(d["ClusterNames"])
    for k in ("Affinity", "Tolerations"):
        if d.get(k) is not None:
            d[k] = _lower_keys(d[k])
    return T.SchedulingUnit.from_json(d)


IGNORE_FIELDS = {"GroupVersion": ("group", "version"), "Kind": ("kind",), "Resource": ("resource",),
                 "Name": ("name",), "Namespace": ("namespace",), "Labels": ("labels",),
                 "Annotations": ("annotations",), "DesiredReplicas": ("desired_replicas",),
                 "CurrentClusters": ("current_clusters",), "ResourceRequest": ("resource_request",),
                 "AvoidDisruption": ("avoid_disruption",)}


def test_fixtures_cover_the_reference_tables():
    tests = {c["test"] for c in SU}
    assert tests == {"TestGetSchedulingUnit", "TestGetSchedulingUnitWithAnnotationOverrides", "TestSchedulingMode"}
    assert len(SU) == 11 and len(MP) == 8
    assert all(c["source"].startswith("pkg/controllers/scheduler/") for c in SU + MP)


@pytest.mark.parametrize("case", SU, ids=[c["name"] for c in SU])
def test_scheduling_unit_for_fed_object(case):
    tc = case["type_config"]
    ftc = O.FederatedTypeConfig(tc["group"], tc["version"], tc["kind"], tc["plural"], tc["scope"] or "Namespaced",
                                tc["replicas_spec"])
    pol = O.PropagationPolicy.from_json(case["policy"])
    got = O.scheduling_unit_for_fed_object(ftc, case["object"], pol)
    if case["ignore"] == "all but SchedulingMode":  # TestSchedulingMode compares su.SchedulingMode only
        assert got.scheduling_mode == case["want"]["SchedulingMode"], case["source"]
        return
    want = _want_su(case["want"])
    for f in case["ignore"]:  # the Go test copies these from the expectation before comparing
        for attr in IGNORE_FIELDS[f]:
            setattr(got, attr, getattr(want, attr))
    assert got == want, case["source"]


@pytest.mark.parametrize("case", MP, ids=[c["name"] for c in MP])
def test_matched_policy_key(case):
    labels = {}
    if case["pp"] is not None:
        labels[case["pp_label"]] = case["pp"]
    if case["cpp"] is not None:
        labels[case["cpp_label"]] = case["cpp"]
    assert case["pp_label"] == O.PROPAGATION_POLICY_NAME_LABEL
    assert case["cpp_label"] == O.CLUSTER_PROPAGATION_POLICY_NAME_LABEL
    obj = {"metadata": {"namespace": case["namespace"], "labels": labels}}
    got = O.matched_policy_key(obj, case["namespace"] != "")
    assert (got is not None) == case["found"], case["source"]
    if got is not None:
        assert got == (case["policy_namespace"], case["policy_name"]), case["source"]

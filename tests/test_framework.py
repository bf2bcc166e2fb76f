"""Product-side framework construction against the reference's own tests.

* ``profile_test.go:36-638`` — the 19 SchedulingProfile cases (``tests/golden/profile.json``) through
  ``kubeadmiral_amd.framework.apply_profile``, the function the batched reconcile caller uses
  (``controller.BatchReconciler._framework``), not the oracle's copy.
* ``framework/runtime/framework_test.go:213-370`` — ``TestNewFramework``'s registration and
  validation cases (enabled plugins respected, repeated / wrongly typed / unregistered plugins
  rejected, each enabled plugin constructed once, disabled ones never) through
  ``framework.new_framework`` and ``Framework``.
"""

import copy

import pytest

from golden_util import case_id, load
from kubeadmiral_amd import framework as F

PROFILE = load("profile.json")


@pytest.mark.parametrize("c", PROFILE, ids=[case_id(c) for c in PROFILE])
def test_profile_golden_through_product_apply_profile(c):
    b = c["base"]
    base = F.EnabledPlugins(list(b["FilterPlugins"] or []), list(b["ScorePlugins"] or []),
                            list(b["SelectPlugins"] or []), list(b["ReplicasPlugins"] or []))
    got = F.apply_profile(base, copy.deepcopy(c["plugins"]))
    w = c["want"]
    assert got.filter_plugins == list(w["FilterPlugins"] or [])
    assert got.score_plugins == list(w["ScorePlugins"] or [])
    assert got.select_plugins == list(w["SelectPlugins"] or [])
    assert got.replicas_plugins == list(w["ReplicasPlugins"] or [])


def test_reconciler_framework_is_apply_profile_over_defaults():
    """BatchReconciler._framework = createFramework (profile.go:84-113): defaults ⊕ profile."""
    from kubeadmiral_amd.controller import BatchReconciler

    prof = {"filter": {"disabled": [{"name": F.TaintToleration}]},
            "score": {"disabled": [{"name": "*"}], "enabled": [{"name": F.ClusterResourcesMostAllocated}]}}
    fwk = BatchReconciler._framework(None, _names_only(prof))
    assert fwk.enabled.filter_plugins == [F.APIResources, F.ClusterResourcesFit, F.PlacementFilter,
                                          F.ClusterAffinity]
    assert fwk.enabled.score_plugins == [F.ClusterResourcesMostAllocated]
    assert fwk.enabled.select_plugins == [F.MaxCluster]
    assert fwk.enabled.replicas_plugins == [F.ClusterCapacityWeight]


def _names_only(prof):
    return {k: {kk: [x["name"] for x in vv] for kk, vv in v.items()} for k, v in prof.items()}


# ------------------------------------------------------- TestNewFramework (framework_test.go:213-370)
class _Registry:
    """framework_test.go:221-283: fake plugins by the interfaces they implement; counts constructions."""

    KINDS = {
        "filter": {"FilterPlugin"},
        "score": {"ScorePlugin"},
        "select": {"SelectPlugin"},
        "replicas": {"ReplicasPlugin"},
        "filterAndScore": {"FilterPlugin", "ScorePlugin"},
        "scoreAndSelect": {"ScorePlugin", "SelectPlugin"},
        "notEnabled": {"FilterPlugin"},
    }

    def __init__(self):
        self.constructed = {}

    def factories(self):
        def make(name):
            def factory():
                if name == "notEnabled":
                    raise AssertionError("plugin not enabled should not be constructed")
                if self.constructed.get(name):
                    raise AssertionError(f"{name} constructed more than once")
                self.constructed[name] = True
                return frozenset(self.KINDS[name])
            return factory
        return {n: make(n) for n in self.KINDS}


NEW_FRAMEWORK_CASES = [
    ("enabled plugins are respected",
     F.EnabledPlugins(["filter"], ["score"], ["scoreAndSelect"], ["replicas"]),
     {"FilterPlugin": ["filter"], "ScorePlugin": ["score"], "SelectPlugin": ["scoreAndSelect"],
      "ReplicasPlugin": ["replicas"]}),
    ("enabled plugins are respected 2",
     F.EnabledPlugins(["filter", "filterAndScore"], ["score", "scoreAndSelect"], ["scoreAndSelect", "select"], []),
     {"FilterPlugin": ["filter", "filterAndScore"], "ScorePlugin": ["score", "scoreAndSelect"],
      "SelectPlugin": ["scoreAndSelect", "select"], "ReplicasPlugin": []}),
    ("repeated plugins returns error",
     F.EnabledPlugins(["filter"], ["score", "score"], ["scoreAndSelect"], ["replicas"]), "already registered"),
    ("incorrect type returns error",
     F.EnabledPlugins(["replicas"], ["score", "scoreAndSelect"], ["scoreAndSelect", "select"], ["filter"]),
     "does not implement"),
    ("plugins not found in registry returns error",
     F.EnabledPlugins(["filter"], ["score", "scoreAndSelect"], ["scoreAndSelect", "select", "notexists"],
                      ["replicas"]), "does not exist"),
]


@pytest.mark.parametrize("name,enabled,want", NEW_FRAMEWORK_CASES, ids=[c[0] for c in NEW_FRAMEWORK_CASES])
def test_new_framework_cases(name, enabled, want):
    reg = _Registry()
    if isinstance(want, str):
        with pytest.raises(F.FrameworkError, match=want):
            F.new_framework(reg.factories(), enabled)
        return
    assert F.new_framework(reg.factories(), enabled) == want
    assert set(reg.constructed) == {n for names in want.values() for n in names}


def test_in_tree_framework_validation():
    """Framework over the in-tree registry (profile.go:39-50) fails exactly where NewFramework does."""
    F.Framework()  # the default set is valid
    with pytest.raises(F.FrameworkError, match="does not implement ScorePlugin"):
        F.Framework(F.EnabledPlugins([], [F.APIResources], [], []))
    with pytest.raises(F.FrameworkError, match="already registered as FilterPlugin"):
        F.Framework(F.EnabledPlugins([F.TaintToleration, F.TaintToleration], [], [], []))
    with pytest.raises(F.FrameworkError, match="SelectPlugin nope does not exist"):
        F.Framework(F.EnabledPlugins([], [], ["nope"], []))
    # a registered webhook plugin: NewFramework succeeds, the device cannot run it
    with pytest.raises(F.UnsupportedPlugin):
        F.Framework(F.EnabledPlugins(["webhook-a"], [], [], []), registry=set(F.IN_TREE) | {"webhook-a"})
    # registered but not enabled: fine
    fw = F.Framework(F.default_enabled_plugins(), registry=set(F.IN_TREE) | {"webhook-a"})
    assert fw.select_plugin == 8 and fw.replicas_plugin == 9

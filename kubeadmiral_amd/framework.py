"""Framework / profile mirror of the reference (host side of the drop-in).

* plugin names            ← pkg/controllers/scheduler/framework/plugins/names/names.go:19-30
* in-tree registry        ← pkg/controllers/scheduler/profile.go:39-50
* EnabledPlugins          ← pkg/apis/core/types.go:21-43
* default plugin set      ← pkg/apis/core/v1alpha1/extensions_schedulingprofile.go:24-49
* applyProfile / reconcileExtPoint ← pkg/controllers/scheduler/profile.go:52-82
* NewFramework validation ← pkg/controllers/scheduler/framework/runtime/framework.go:45-95

``Framework(enabled)`` raises exactly where ``runtime.NewFramework`` returns an
error, and ``UnsupportedPlugin`` for plugins outside the in-tree set (e.g. the
out-of-process webhook plugins, ``extensions/webhook/v1alpha1/plugin.go``) —
the caller must keep the Go ``genericScheduler`` for such profiles.
"""

from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import Callable, Dict, FrozenSet, List, Mapping, Optional

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

# include/kad_sched.h enum kad_plugin
PLUGIN_ID = {
    APIResources: 0, TaintToleration: 1, ClusterResourcesFit: 2, PlacementFilter: 3, ClusterAffinity: 4,
    ClusterResourcesBalancedAllocation: 5, ClusterResourcesLeastAllocated: 6, ClusterResourcesMostAllocated: 7,
    MaxCluster: 8, ClusterCapacityWeight: 9,
}
FILTER_PLUGINS = {APIResources, TaintToleration, ClusterResourcesFit, PlacementFilter, ClusterAffinity}
SCORE_PLUGINS = {TaintToleration, ClusterResourcesBalancedAllocation, ClusterResourcesLeastAllocated,
                 ClusterResourcesMostAllocated, ClusterAffinity}
SELECT_PLUGINS = {MaxCluster}
REPLICAS_PLUGINS = {ClusterCapacityWeight}
IN_TREE = FILTER_PLUGINS | SCORE_PLUGINS | SELECT_PLUGINS | REPLICAS_PLUGINS

PROFILE_XORSHIFT_GO121 = 1


class FrameworkError(ValueError):
    """runtime.NewFramework error (framework.go:45-95)."""


class UnsupportedPlugin(FrameworkError):
    """A registered but non-in-tree plugin (webhook): not executable on the device."""


@dataclass
class EnabledPlugins:
    filter_plugins: List[str] = field(default_factory=list)
    score_plugins: List[str] = field(default_factory=list)
    select_plugins: List[str] = field(default_factory=list)
    replicas_plugins: List[str] = field(default_factory=list)

    def is_plugin_enabled(self, name: str) -> bool:  # pkg/apis/core/types.go:28-43
        return name in set(self.filter_plugins) | set(self.score_plugins) | set(self.select_plugins) | set(
            self.replicas_plugins)


def default_enabled_plugins() -> EnabledPlugins:
    return EnabledPlugins(
        [APIResources, TaintToleration, ClusterResourcesFit, PlacementFilter, ClusterAffinity],
        [TaintToleration, ClusterResourcesBalancedAllocation, ClusterResourcesLeastAllocated, ClusterAffinity],
        [MaxCluster],
        [ClusterCapacityWeight],
    )


def reconcile_ext_point(enabled, enabled_names, disabled_names):
    disabled = set(disabled_names or [])
    result = [] if "*" in disabled else [e for e in enabled if e not in disabled]
    result.extend(enabled_names or [])
    return result


def apply_profile(base: EnabledPlugins, plugins: Optional[dict]) -> EnabledPlugins:
    """SchedulingProfile.Spec.Plugins → EnabledPlugins. Replicas plugins cannot be changed (profile.go:52-60)."""
    if plugins is None:
        return base
    for point, attr in (("filter", "filter_plugins"), ("score", "score_plugins"), ("select", "select_plugins")):
        ps = plugins.get(point) or {}
        setattr(base, attr, reconcile_ext_point(getattr(base, attr), ps.get("enabled"), ps.get("disabled")))
    return base


class KadProfile(ctypes.Structure):
    """include/kad_sched.h: kad_profile."""

    _fields_ = [("filter_mask", ctypes.c_uint32), ("score_mask", ctypes.c_uint32),
                ("select_plugin", ctypes.c_int32), ("replicas_plugin", ctypes.c_int32),
                ("flags", ctypes.c_uint32), ("reserved", ctypes.c_uint32 * 3)]


EXTENSION_POINTS = ("FilterPlugin", "ScorePlugin", "SelectPlugin", "ReplicasPlugin")
# what each in-tree plugin implements (plugins/*: which framework interfaces the type satisfies)
IN_TREE_REGISTRY: Dict[str, Callable[[], FrozenSet[str]]] = {
    n: (lambda n=n: frozenset(p for p, kinds in zip(EXTENSION_POINTS, (FILTER_PLUGINS, SCORE_PLUGINS, SELECT_PLUGINS,
                                                                      REPLICAS_PLUGINS)) if n in kinds))
    for n in sorted(IN_TREE)
}


def new_framework(registry: Mapping[str, Callable[[], FrozenSet[str]]], enabled: EnabledPlugins) -> Dict[str, List[str]]:
    """runtime.NewFramework (framework/runtime/framework.go:45-95) over a registry of plugin factories.

    A factory returns the set of extension-point interfaces its plugin implements (the Go plugin's type).
    Every enabled plugin is constructed exactly once; plugins that are registered but not enabled are never
    constructed (IsPluginEnabled, pkg/apis/core/types.go:28-43). Each extension point is then filled in
    order, failing like addPlugins (:72-99): "<Point> <name> does not exist", "plugin <name> does not
    implement <Point>", "plugin <name> already registered as <Point>". Returns the plugin lists per point.
    """
    built = {name: factory() for name, factory in registry.items() if enabled.is_plugin_enabled(name)}
    out: Dict[str, List[str]] = {}
    for point, names in zip(EXTENSION_POINTS, (enabled.filter_plugins, enabled.score_plugins,
                                               enabled.select_plugins, enabled.replicas_plugins)):
        seen: List[str] = []
        for n in names:
            if n not in built:
                raise FrameworkError(f"{point} {n} does not exist")
            if point not in built[n]:
                raise FrameworkError(f"plugin {n} does not implement {point}")
            if n in seen:
                raise FrameworkError(f"plugin {n} already registered as {point}")
            seen.append(n)
        out[point] = seen
    return out


class Framework:
    """Validated framework = the device profile (kad_profile).

    ``registry``: None = the in-tree registry (profile.go:39-50); a set of names = the in-tree plugins
    among them plus, for any other name, a registered out-of-tree (webhook) plugin; or a mapping
    name → factory as :func:`new_framework` takes. Construction fails where ``runtime.NewFramework``
    does; a valid framework that enables an out-of-tree plugin raises :class:`UnsupportedPlugin` (the
    device runs only in-tree plugins, so such profiles keep the Go path).
    """

    def __init__(self, enabled: Optional[EnabledPlugins] = None, registry=None, flags: int = 0):
        enabled = enabled if enabled is not None else default_enabled_plugins()
        if registry is None:
            registry = IN_TREE_REGISTRY
        elif not isinstance(registry, Mapping):  # names: out-of-tree ones implement every point (webhook adapter)
            registry = {n: IN_TREE_REGISTRY.get(n, lambda: frozenset(EXTENSION_POINTS)) for n in registry}
        lists = new_framework(registry, enabled)
        for names in lists.values():
            for n in names:
                if n not in IN_TREE:
                    raise UnsupportedPlugin(f"plugin {n} is not an in-tree plugin")
        self.enabled = enabled
        self.flags = flags

    @property
    def filter_mask(self) -> int:
        m = 0
        for n in self.enabled.filter_plugins:
            m |= 1 << PLUGIN_ID[n]
        return m

    @property
    def score_mask(self) -> int:
        m = 0
        for n in self.enabled.score_plugins:
            m |= 1 << PLUGIN_ID[n]
        return m

    @property
    def select_plugin(self) -> int:
        return PLUGIN_ID[self.enabled.select_plugins[0]] if self.enabled.select_plugins else -1

    @property
    def replicas_plugin(self) -> int:
        return PLUGIN_ID[self.enabled.replicas_plugins[0]] if self.enabled.replicas_plugins else -1

    def has_filter(self, name) -> bool:
        return name in self.enabled.filter_plugins

    def has_score(self, name) -> bool:
        return name in self.enabled.score_plugins

    def to_c(self) -> KadProfile:
        p = KadProfile()
        p.filter_mask = self.filter_mask
        p.score_mask = self.score_mask
        p.select_plugin = self.select_plugin
        p.replicas_plugin = self.replicas_plugin
        p.flags = self.flags
        return p

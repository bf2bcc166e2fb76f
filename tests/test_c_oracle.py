"""The C restatement (oracle/kad_ref.c over packed blobs) == the pinned Python oracle (objects).

This validates, at once, the host packer (kubeadmiral_amd/pack.py: interning,
program compilation, resource conversion) and the C oracle that the GPU
parity tests and the CPU baseline use at sizes the Python oracle cannot reach.
"""

import numpy as np
import pytest

from kubeadmiral_amd import framework as F
from kubeadmiral_amd import pack, synth
from kubeadmiral_amd import types as T
from kubeadmiral_amd.results import to_schedule_result
from oracle import kad_oracle as O
from oracle import ref


def oracle_fwk(fwk):
    e = fwk.enabled
    return O.Framework(O.EnabledPlugins(e.filter_plugins, e.score_plugins, e.select_plugins, e.replicas_plugins))


def py_results(fwk, units, clusters):
    ofw = oracle_fwk(fwk)
    out = []
    for su in units:
        kind, val = O.schedule_or_error(ofw, su, clusters)
        out.append(T.ScheduleError(val) if kind == "error" else val)
    return out


def same(a, b):
    if isinstance(a, T.ScheduleError) or isinstance(b, T.ScheduleError):
        return isinstance(a, T.ScheduleError) and isinstance(b, T.ScheduleError) and a.stage == b.stage
    return a.suggested_clusters == b.suggested_clusters


def compare(clusters, units, fwk, n_threads=1):
    snap = pack.Snapshot(clusters)
    batch = pack.Batch(snap, fwk, units)
    res = ref.schedule(snap, batch, fwk, n_threads=n_threads)
    want = py_results(fwk, units, clusters)
    bad = []
    for w, su in enumerate(units):
        got = to_schedule_result(res, w, su, snap.names)
        if not same(got, want[w]):
            bad.append((w, su.name, got, want[w]))
    return bad


@pytest.mark.parametrize("seed", range(24))
def test_c_oracle_matches_python_oracle_fuzz(seed):
    clusters, units = synth.gen_fuzz(seed, W=50)
    fwk = synth.fuzz_framework(seed)
    bad = compare(clusters, units, fwk)
    assert not bad, bad[:3]


@pytest.mark.parametrize("seed,n_taints", [(901, 100), (902, 160), (903, 220)])
def test_c_oracle_matches_python_oracle_many_taint_words(seed, n_taints):
    """Taint ids over 2-4+ words (the packer's multi-word toleration / taint masks, SnapDev::TW > 1): the C
    oracle the GPU tests check against agrees with the object-level oracle under every fuzz profile."""
    from kubeadmiral_amd import pack
    clusters, units = synth.gen_fuzz(seed, W=40, C=30, n_taints=n_taints)
    assert pack.Snapshot(clusters).TW >= 2
    for i in range(len(synth.FUZZ_PROFILES)):
        bad = compare(clusters, units, synth.fuzz_framework(i))
        assert not bad, (i, bad[:3])


@pytest.mark.parametrize("seed", range(6))
def test_c_oracle_matches_python_oracle_discovery_lists(seed):
    """Production-shaped API-resource lists (~150 Kind-sorted discovery entries per cluster, 3 GVK words;
    clusterstatus.go:221-266) with units over 8 workload kinds and one no cluster serves: APIResources.Filter
    (apiresources.go:25-43) on GVK ids past the first word, under every fuzz profile."""
    clusters, units = synth.with_discovery(*synth.gen_fuzz(700 + seed, W=40), seed)
    snap = pack.Snapshot(clusters)
    assert snap.GW >= 3 and max(snap.gvk_id.values()) >= 128
    bad = compare(clusters, units, synth.fuzz_framework(seed))
    assert not bad, bad[:3]


def test_c_oracle_matches_python_oracle_c3r_small():
    clusters, units, fwk = synth.make_config("c3r", W=150, C=64)
    snap = pack.Snapshot(clusters)
    assert snap.GW >= 3
    assert sum(snap.gvk_id[(su.group, su.version, su.kind)] >= 64 for su in units) > 50
    assert not compare(clusters, units, fwk)


def test_c_oracle_matches_python_oracle_relaxed_resources():
    """c3p's cluster shapes (available < 0, empty allocatable: federatedcluster/util.go:178-214) with zero and
    non-zero requests: the C restatement equals the object-level oracle (fit.go's int64 compare, the
    capacity == 0 branches of least/most_allocated.go and fractionOfCapacity)."""
    clusters, units, fwk = synth.make_config("c3p", W=200, C=200)
    rng = np.random.default_rng(3)
    synth.production_resources(clusters, rng, p_over=0.3, p_empty=0.15)
    for su in units[::2]:
        su.resource_request = T.Resource(int(rng.integers(0, 64_001)), int(rng.integers(0, 1 << 38)))
    for f in (fwk, F.Framework(F.default_enabled_plugins())):
        assert not compare(clusters, units, f)


def test_c_oracle_matches_python_oracle_c1():
    clusters, units, fwk = synth.make_config("c1", W=200)
    assert not compare(clusters, units, fwk, n_threads=4)


def test_c_oracle_matches_python_oracle_c2_small():
    clusters, units, fwk = synth.make_config("c2", W=150, C=64)
    assert not compare(clusters, units, fwk)


def test_c_oracle_matches_python_oracle_c4_small():
    clusters, units, fwk = synth.make_config("c4", W=120, C=80)
    assert not compare(clusters, units, fwk)


def test_c_oracle_matches_python_oracle_c5_small():
    clusters, units, fwk = synth.make_config("c5", W=40, C=120)
    assert not compare(clusters, units, fwk)


def test_c_select_rows_match_python_sort():
    import numpy as np
    from oracle.gosem import go_sort_slice
    rng = np.random.default_rng(7)
    for _ in range(300):
        n = int(rng.integers(0, 200))
        scores = rng.integers(0, int(rng.integers(1, 12)), n).tolist()
        k = int(rng.integers(0, n + 2))
        items = [[i, s] for i, s in enumerate(scores)]
        go_sort_slice(items, lambda a, b: a[1] > b[1])
        want = [i for i, _ in items[:min(k, n)]]
        assert ref.select_row(scores, k) == want


@pytest.mark.parametrize("seed", range(6))
def test_c_oracle_matches_python_oracle_wide_prefs(seed):
    """The C oracle reads the i64 preference columns of a wide batch (values past int32) as the object oracle
    computes them."""
    from kubeadmiral_amd import pack
    clusters, units = synth.gen_fuzz(700 + seed, W=50)
    synth.widen_prefs(units, seed, share=0.5)
    fwk = synth.fuzz_framework(seed)
    assert pack.header_of(pack.Batch(pack.Snapshot(clusters), fwk, units).blob, pack.BatchHeader).flags == 0
    bad = compare(clusters, units, fwk)
    assert not bad, bad[:3]

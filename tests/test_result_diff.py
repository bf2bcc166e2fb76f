"""§8 f3 — the result-dependent half of applySchedulingResult (scheduler.go:632-695) as per-unit flags.

CPU: the oracle restatement over kad_result_state arrays (oracle/result_diff.py) agrees with the object-level
functions the product's reconciler applies (objects.set_placement_cluster_names / update_replicas_override, which
restate util/placement.go / scheduler/util.go on unstructured objects), on fuzz objects and C-oracle results.
GPU (-m gpu): kad_result_diff on the device, from the last kad_schedule's outputs, equals the oracle.
"""
import copy

import numpy as np
import pytest

from kubeadmiral_amd import objects as O
from kubeadmiral_amd import pack, synth
from kubeadmiral_amd import types as T
from kubeadmiral_amd.results import to_schedule_result
from oracle import ref
from oracle import result_diff as RD

FTC = O.FederatedTypeConfig("apps", "v1", "Deployment", "deployments", "Namespaced", "spec.replicas")


def _case(seed, W=120, C=30):
    clusters, units = synth.gen_fuzz(seed, W=W, C=C)
    fwk = synth.fuzz_framework(seed)
    snap = pack.Snapshot(clusters)
    batch = pack.Batch(snap, fwk, units)
    objs = synth.gen_result_objects(np.random.default_rng(seed), W, snap.names)
    return snap, batch, fwk, units, objs


def _object_level(snap, units, res, objs, errors):
    """What applySchedulingResult's two calls report on a copy of each object."""
    out = np.zeros(len(objs), np.uint32)
    for w, (su, obj) in enumerate(zip(units, objs)):
        if w in errors:
            continue
        r = to_schedule_result(res, w, su, snap.names)
        if isinstance(r, T.ScheduleError):
            out[w] = RD.SKIP
            continue
        if int(res.status[w]) == pack.ST_STICKY:
            out[w] = RD.STICKY
            continue
        f = 0
        if O.set_placement_cluster_names(copy.deepcopy(obj), O.PREFIXED_GLOBAL_SCHEDULER_NAME, r.cluster_set()):
            f |= RD.PLACEMENT
        desired = {c: n for c, n in (r.suggested_clusters or {}).items() if n is not None}
        if O.update_replicas_override(FTC, copy.deepcopy(obj), desired):
            f |= RD.OVERRIDES
        out[w] = f
    return out


@pytest.mark.parametrize("seed", range(12))
def test_oracle_equals_object_level(seed):
    snap, batch, fwk, units, objs = _case(seed)
    res = ref.schedule(snap, batch, fwk)
    state = O.result_states(FTC, objs, snap.names)
    got = RD.diff_flags(res, batch.out_off, state)
    want = _object_level(snap, units, res, objs, set(state["errors"]))
    ok = np.ones(len(objs), bool)
    ok[state["errors"]] = False
    assert np.array_equal(got[ok], want[ok])
    # every branch is exercised
    assert (got & RD.PLACEMENT).any() and (got & RD.OVERRIDES).any() and (got == 0).any()
    assert ((got & (RD.PLACEMENT | RD.OVERRIDES)) == RD.PLACEMENT).any()


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(6))
def test_gpu_result_diff_equals_oracle(seed):
    from kubeadmiral_amd import build, runtime
    build.build()
    ctx = runtime.Context(0)
    try:
        snap, batch, fwk, units, objs = _case(100 + seed, W=400, C=90)
        ctx.upload_snapshot(snap)
        res = ctx.run(fwk, batch)
        state = O.result_states(FTC, objs, snap.names)
        got = ctx.result_diff(state)
        want = RD.diff_flags(res, batch.out_off, state)
        assert np.array_equal(got, want), np.nonzero(got != want)[0][:10]
        assert (got & RD.OVERRIDES).any() and (got & RD.PLACEMENT).any()
    finally:
        ctx.close()

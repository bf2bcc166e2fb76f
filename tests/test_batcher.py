"""CoalescingScheduler: per-unit Schedule calls from worker threads coalesced into batches.

CPU tests drive the dispatcher with a recording stand-in for BatchScheduler
(host logic only: coalescing, grouping by framework and cluster list, error
propagation, shutdown); the GPU test runs real worker threads against the
HIP path and compares every unit with the C oracle (oracle/kad_ref.c).
"""

import os
import threading

import numpy as np
import pytest

from kubeadmiral_amd import framework as F
from kubeadmiral_amd import pack, synth
from kubeadmiral_amd import types as T
from kubeadmiral_amd.batcher import CoalescingScheduler


class Recorder:
    """Stands in for BatchScheduler.schedule: result = {unit name: desired replicas}; 'bad-*' units error."""

    def __init__(self, fail_batches=False):
        self.calls = []
        self.fail_batches = fail_batches

    def schedule(self, fwk, units, clusters):
        self.calls.append((bytes(fwk.to_c()), T.clusters_fingerprint(clusters), [u.name for u in units]))
        if self.fail_batches:
            raise RuntimeError("device lost")
        return [T.ScheduleError("score", "boom") if u.name.startswith("bad")
                else T.ScheduleResult({u.name: u.desired_replicas}) for u in units]


def _unit(name, d=1):
    return T.SchedulingUnit(group="apps", version="v1", kind="Deployment", namespace="ns", name=name,
                            desired_replicas=d)


def _run_workers(cs, jobs, n_threads=8):
    out = [None] * len(jobs)
    start = threading.Barrier(n_threads)

    def work(t):
        start.wait()
        for i in range(t, len(jobs), n_threads):
            fwk, su, cl = jobs[i]
            try:
                out[i] = cs.schedule(fwk, su, cl)
            except T.ScheduleError as e:
                out[i] = e
    th = [threading.Thread(target=work, args=(t,)) for t in range(n_threads)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    return out


def test_concurrent_calls_coalesce_and_keep_their_results():
    rec = Recorder()
    fwk = F.Framework()
    cl = []
    jobs = [(fwk, _unit(f"u{i}", i), cl) for i in range(400)]
    with CoalescingScheduler(rec, max_wait_s=0.02) as cs:
        out = _run_workers(cs, jobs)
    assert [r.suggested_clusters for r in out] == [{f"u{i}": i} for i in range(400)]
    assert sum(cs.batches) == 400 and len(cs.batches) < 400  # calls were coalesced
    assert sorted(n for c in rec.calls for n in c[2]) == sorted(f"u{i}" for i in range(400))


def test_batches_split_by_framework_and_cluster_list():
    rec = Recorder()
    f1 = F.Framework()
    f2 = F.Framework(F.EnabledPlugins([F.APIResources], [], [F.MaxCluster], [F.ClusterCapacityWeight]))
    cl_a, cl_b = [T.FederatedCluster("a")], [T.FederatedCluster("b")]
    jobs = [(f1 if i % 2 else f2, _unit(f"u{i}"), cl_a if i % 3 else cl_b) for i in range(120)]
    with CoalescingScheduler(rec, max_wait_s=0.05) as cs:
        _run_workers(cs, jobs, n_threads=4)
    for prof, fp, names in rec.calls:
        idx = [int(n[1:]) for n in names]
        assert len({bytes((f1 if i % 2 else f2).to_c()) for i in idx}) == 1
        assert {bytes((f1 if i % 2 else f2).to_c()) for i in idx} == {prof}
        assert {T.clusters_fingerprint(cl_a if i % 3 else cl_b) for i in idx} == {fp}


def test_equal_content_lists_share_a_batch():
    """The reference lists clusters afresh per reconcile (scheduler.go:334): every call brings its own
    list object. Equal content → one group per window; a changed label → its own group."""
    rec = Recorder()
    fwk = F.Framework()
    base = [T.FederatedCluster(f"c{i}", labels={"k": "v"}) for i in range(4)]
    changed = [T.FederatedCluster(f"c{i}", labels={"k": "w" if i == 2 else "v"}) for i in range(4)]
    cs = CoalescingScheduler(rec, max_wait_s=0.5, max_batch=64)
    futs = [cs.submit(fwk, _unit(f"u{i}"), [T.FederatedCluster(c.name, labels=dict(c.labels)) for c in base])
            for i in range(40)]
    futs += [cs.submit(fwk, _unit(f"x{i}"), list(changed)) for i in range(8)]
    for f in futs:
        f.result(timeout=10)
    cs.close()
    assert sum(cs.batches) == 48
    by_fp = {}
    for _, fp, names in rec.calls:
        by_fp.setdefault(fp, []).extend(names)
    assert sorted(by_fp[T.clusters_fingerprint(base)]) == sorted(f"u{i}" for i in range(40))
    assert sorted(by_fp[T.clusters_fingerprint(changed)]) == sorted(f"x{i}" for i in range(8))
    assert len(rec.calls) <= 2 * len(cs.batches)


def test_resource_version_identifies_content():
    a = T.FederatedCluster("c0", labels={"k": "v"}, resource_version="7")
    b = T.FederatedCluster("c0", labels={"k": "other"}, resource_version="7")
    assert T.clusters_fingerprint([a]) == T.clusters_fingerprint([b])  # same RV: the API server's promise
    b.resource_version = "8"
    assert T.clusters_fingerprint([a]) != T.clusters_fingerprint([b])
    c = T.FederatedCluster("c0", labels={"k": "v"})
    d = T.FederatedCluster("c0", labels={"k": "v"})
    assert T.clusters_fingerprint([c]) == T.clusters_fingerprint([d])
    d.labels["k"] = "w"  # edited in place, no RV: content decides
    assert T.clusters_fingerprint([c]) != T.clusters_fingerprint([d])


def test_unit_errors_raise_per_call_and_batch_failures_reach_every_caller():
    with CoalescingScheduler(Recorder(), max_wait_s=0.0) as cs:
        assert cs.schedule(F.Framework(), _unit("ok", 3), []).suggested_clusters == {"ok": 3}
        with pytest.raises(T.ScheduleError):
            cs.schedule(F.Framework(), _unit("bad-1"), [])
    with CoalescingScheduler(Recorder(fail_batches=True), max_wait_s=0.01) as cs:
        futs = [cs.submit(F.Framework(), _unit(f"u{i}"), []) for i in range(10)]
        for f in futs:
            with pytest.raises(RuntimeError, match="device lost"):
                f.result(timeout=10)
        # the dispatcher survives a failed batch
        cs.scheduler.fail_batches = False
        assert cs.schedule(F.Framework(), _unit("after", 2), []).suggested_clusters == {"after": 2}


def test_max_batch_bounds_a_dispatch():
    rec = Recorder()
    cs = CoalescingScheduler(rec, max_batch=16, max_wait_s=0.05)
    futs = [cs.submit(F.Framework(), _unit(f"u{i}"), []) for i in range(100)]
    for f in futs:
        f.result(timeout=10)
    cs.close()
    assert max(cs.batches) <= 16 and sum(cs.batches) == 100


def test_closed_scheduler_refuses_calls():
    cs = CoalescingScheduler(Recorder())
    cs.close()
    cs.close()  # idempotent
    with pytest.raises(RuntimeError, match="closed"):
        cs.submit(F.Framework(), _unit("late"), [])


def _norm(r):
    """ScheduleErrors compare by error class (parity is on the class, not the message)."""
    return ("error", r.stage) if isinstance(r, T.ScheduleError) else r


@pytest.mark.gpu
def test_gpu_worker_threads_match_oracle():
    from kubeadmiral_amd.results import to_schedule_result
    from oracle import ref

    cl, units, fwk = synth.make_config("c1", W=1000, seed=0xC1)
    snap = pack.Snapshot(cl)
    want_b = ref.schedule(snap, pack.Batch(snap, fwk, units), fwk, n_threads=min(8, os.cpu_count() or 1))
    want = [to_schedule_result(want_b, w, su, snap.names) for w, su in enumerate(units)]
    # every call brings its own copy of the cluster list, as the reference's reconcile does (scheduler.go:334)
    with CoalescingScheduler(max_wait_s=0.005) as cs:
        got = _run_workers(cs, [(fwk, su, list(cl)) for su in units], n_threads=8)
        uploads = cs.scheduler.full_uploads
    assert [_norm(r) for r in got] == [_norm(r) for r in want]
    assert len(cs.batches) < len(units) // 4  # coalesced across distinct but equal lists
    assert uploads == 1  # the resident snapshot is reused: equal content, no repack

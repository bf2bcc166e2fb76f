"""kad_group (one process, several GPUs): the batch split into contiguous unit ranges, one kad_ctx per member,
results in one view — bit-exact with a single kad_ctx over the whole batch.

The reference schedules each unit independently against the read-only cluster list (scheduler.go:246-309),
called from the scheduler's worker goroutines (worker.go:132-134, scheduler.go:507); a one-GPU box maps every
member onto device 0, so these tests run the group's split, shard uploads, offset downloads and peer-copied
snapshot exactly as on an 8-GPU node (the copies are same-device there).
"""

import numpy as np
import pytest

from gpu_util import assert_same, c_oracle
from kubeadmiral_amd import pack, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def single():
    from kubeadmiral_amd import build, runtime
    build.build()
    c = runtime.Context(0)
    yield c
    c.close()


@pytest.fixture(scope="module", params=[2, 4])
def group(request):
    from kubeadmiral_amd import runtime
    g = runtime.GroupContext([0] * request.param)
    yield g
    g.close()


def _same_arrays(got, want, batch, what):
    assert_same(got, want, what)
    # every written slot, byte for byte
    cnt = want.count.astype(np.int64)
    idx = np.repeat(np.asarray(batch.out_off[:-1], np.int64), cnt) + (
        np.arange(int(cnt.sum())) - np.repeat(np.cumsum(cnt) - cnt, cnt))
    assert np.array_equal(got.cluster[idx], want.cluster[idx]), what
    assert np.array_equal(got.replicas[idx], want.replicas[idx]), what


def _both(single, group, clusters, units, fwk):
    snap = pack.Snapshot(clusters)
    batch = pack.Batch(snap, fwk, units)
    single.upload_snapshot(snap)
    want = single.run(fwk, batch)
    group.upload_snapshot(snap)
    got = group.run(fwk, batch)
    return snap, batch, got, want


@pytest.mark.parametrize("seed", range(12))
def test_group_fuzz_equals_single(single, group, seed):
    clusters, units = synth.gen_fuzz(8100 + seed, W=97)
    fwk = synth.fuzz_framework(seed)
    snap, batch, got, want = _both(single, group, clusters, units, fwk)
    _same_arrays(got, want, batch, f"group fuzz {seed}")
    ulo, slo = group.ranges()
    assert ulo[-1] == batch.W and slo[-1] == batch.n_out_slots
    assert group.path_counts()["units"] == batch.W


@pytest.mark.parametrize("cfg,W", [("c2", 30_000), ("c4", 30_000), ("c3r", 20_000), ("c5", 600)])
def test_group_configs_equal_single_and_oracle(single, group, cfg, W):
    clusters, units, fwk = synth.make_config(cfg, W=W)
    snap, batch, got, want = _both(single, group, clusters, units, fwk)
    _same_arrays(got, want, batch, f"group {cfg}")
    assert_same(got, c_oracle(snap, batch, fwk), f"group {cfg} vs oracle")
    assert group.path_counts() == single.path_counts()


def test_group_fewer_units_than_members(single, group):
    """Members with empty ranges (W < n), and W = 0."""
    clusters, units = synth.gen_fuzz(8200, W=1, C=12)
    fwk = synth.fuzz_framework(1)
    snap, batch, got, want = _both(single, group, clusters, units, fwk)
    _same_arrays(got, want, batch, "group W=1")
    _, batch0, got0, _ = _both(single, group, clusters, [], fwk)
    assert len(got0.status) == 0


def test_group_snapshot_update_and_schedule_batch(single, group):
    """A cluster status event as a delta on every member; the resident batch stays valid; the all-in-one
    kad_group_schedule_batch gives the same rows."""
    rng = np.random.default_rng(8300)
    clusters, units = synth.gen_fuzz(8300, W=120, C=40)
    fwk = synth.fuzz_framework(1)
    snap, batch, got, want = _both(single, group, clusters, units, fwk)
    new, _ = synth.mutate_clusters(rng, clusters, 9, structural=True)
    delta = snap.diff(new)
    if delta is None:
        pytest.skip("mutation needed a vocabulary change")
    group.update_snapshot(delta)
    single.update_snapshot(delta)
    snap.commit(delta)
    group.schedule(fwk)
    single.schedule(fwk)
    want2 = single.download()
    _same_arrays(group.download(), want2, batch, "group after delta")
    _same_arrays(group.schedule_batch(fwk, batch), want2, batch, "group schedule_batch")


def test_batch_scheduler_and_coalescer_on_a_group():
    """BatchScheduler / CoalescingScheduler with devices=[...] schedule through a kad_group: per-unit results
    equal the C oracle's."""
    from kubeadmiral_amd.batcher import CoalescingScheduler
    from kubeadmiral_amd.results import to_schedule_result
    from kubeadmiral_amd.runtime import BatchScheduler
    clusters, units = synth.gen_fuzz(8400, W=150, C=60)
    fwk = synth.fuzz_framework(1)
    bs = BatchScheduler(devices=[0, 0, 0])
    out = bs.schedule(fwk, units, clusters)
    snap = pack.Snapshot(clusters)
    batch = pack.Batch(snap, fwk, units)
    want = c_oracle(snap, batch, fwk)
    for w, su in enumerate(units):
        a, b = out[w], to_schedule_result(want, w, su, snap.names)
        assert type(a) is type(b) and (getattr(a, "suggested_clusters", None) == getattr(b, "suggested_clusters", None))
    bs.ctx.close()
    with CoalescingScheduler(devices=[0, 0], max_wait_s=0.01) as cs:
        futs = [cs.submit(fwk, su, clusters) for su in units]
        res = [f.result() for f in futs]
    for w, su in enumerate(units):
        a, b = res[w], to_schedule_result(want, w, su, snap.names)
        assert type(a) is type(b) and (getattr(a, "suggested_clusters", None) == getattr(b, "suggested_clusters", None))

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


@pytest.mark.parametrize("cfg,W", [("c2", 30_000), ("c4", 30_000), ("c3r", 20_000), ("c3p", 20_000), ("c5", 600)])
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


def _slice_state(st, lo, hi):
    """The kad_result_state arrays of units [lo, hi)."""
    po, oo = st["place_off"], st["ovr_off"]
    return {"place_off": (po[lo:hi + 1] - po[lo]).astype(np.int32), "place_cluster": st["place_cluster"][po[lo]:po[hi]],
            "place_has": st["place_has"][lo:hi], "ovr_off": (oo[lo:hi + 1] - oo[lo]).astype(np.int32),
            "ovr_cluster": st["ovr_cluster"][oo[lo]:oo[hi]], "ovr_value": st["ovr_value"][oo[lo]:oo[hi]],
            "ovr_kind": st["ovr_kind"][oo[lo]:oo[hi]]}


def test_group_member_copy_and_diff(single, group):
    """A member ctx's kad_results_copy_device and kad_result_diff cover its shard (they read the
    whole batch's sizes from shard-sized buffers before): equal to the group's download and to the single
    context's diff over the same units."""
    import torch
    clusters, units = synth.gen_fuzz(8500, W=150, C=60)
    fwk = synth.fuzz_framework(2)
    snap, batch, got, want = _both(single, group, clusters, units, fwk)
    rng = np.random.default_rng(8500)
    W, C = batch.W, snap.C
    cnt = want.count.astype(np.int64)
    place, p_off, o_id, o_val, o_off = [], [0], [], [], [0]
    for w in range(W):
        sel = want.cluster[batch.out_off[w]:batch.out_off[w] + cnt[w]].tolist()
        r = rng.random()
        ids = sel if r < 0.4 else (sel[:-1] if r < 0.6 else rng.integers(-1, C, int(rng.integers(0, 5))).tolist())
        place += ids
        p_off.append(len(place))
        for cid in (sel[:2] if rng.random() < 0.5 else []):
            o_id.append(cid)
            o_val.append(int(rng.integers(0, 4)))
        o_off.append(len(o_id))
    state = {"place_off": np.asarray(p_off, np.int32), "place_cluster": np.asarray(place, np.int32),
             "place_has": (rng.random(W) < 0.9).astype(np.uint8), "ovr_off": np.asarray(o_off, np.int32),
             "ovr_cluster": np.asarray(o_id, np.int32), "ovr_value": np.asarray(o_val, np.int64),
             "ovr_kind": np.zeros(len(o_id), np.uint8)}
    full = single.result_diff(state)
    ulo, slo = group.ranges()
    for i in range(len(group.devices)):
        m = group.member(i)
        lo, hi, s0, s1 = int(ulo[i]), int(ulo[i + 1]), int(slo[i]), int(slo[i + 1])
        assert np.array_equal(m.result_diff(_slice_state(state, lo, hi)), full[lo:hi]), i
        dev = f"cuda:{group.devices[i]}"
        t = [torch.full((max(1, n),), -7, dtype=dt, device=dev) for n, dt in
             ((hi - lo, torch.int32), (hi - lo, torch.int32), (hi - lo, torch.int32), (s1 - s0, torch.int32),
              (s1 - s0, torch.int64))]
        m.copy_results_device(*(x.data_ptr() for x in t))
        torch.cuda.synchronize()
        for x, ref, n in zip(t, (got.status[lo:hi], got.count[lo:hi], got.flags[lo:hi], got.cluster[s0:s1],
                                 got.replicas[s0:s1]), (hi - lo,) * 3 + (s1 - s0,) * 2):
            assert np.array_equal(x.cpu().numpy()[:n].view(np.asarray(ref).dtype) if n else x.cpu().numpy()[:0],
                                  np.asarray(ref)[:n]), i
            if n < x.numel():  # nothing past the member's own results
                assert (x.cpu().numpy()[n:] == -7).all()


def test_group_schedule_batch_concurrent_callers(single, group):
    """kad_group_schedule_batch holds the group lock from upload to download: two threads with
    batches of different sizes never download each other's batch."""
    import threading
    clusters, units = synth.gen_fuzz(8600, W=400, C=50)
    fwk = synth.fuzz_framework(1)
    snap = pack.Snapshot(clusters)
    b_small, b_big = pack.Batch(snap, fwk, units[:97]), pack.Batch(snap, fwk, units)
    single.upload_snapshot(snap)
    w_small, w_big = single.run(fwk, b_small), single.run(fwk, b_big)
    group.upload_snapshot(snap)
    errs = []

    def worker(b, want):
        try:
            for _ in range(12):
                _same_arrays(group.schedule_batch(fwk, b), want, b, "concurrent schedule_batch")
        except Exception as e:  # noqa: BLE001 (reported below)
            errs.append(e)

    th = [threading.Thread(target=worker, args=a) for a in ((b_small, w_small), (b_big, w_big))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs[0]


def test_group_across_devices_equals_single():
    """Members on distinct GPUs (peer access, hipMemcpyPeerAsync snapshot copies, per-device streams): skipped
    on a one-GPU box — runs on a multi-GPU node."""
    from kubeadmiral_amd import runtime
    import torch
    n = torch.cuda.device_count()
    if n < 2:
        pytest.skip("one GPU: the cross-device path needs >= 2")
    clusters, units, fwk = synth.make_config("c3r", W=40_000)
    snap = pack.Snapshot(clusters)
    batch = pack.Batch(snap, fwk, units)
    c = runtime.Context(0)
    g = runtime.GroupContext(list(range(min(n, 8))))
    try:
        c.upload_snapshot(snap)
        want = c.run(fwk, batch)
        g.upload_snapshot(snap)
        _same_arrays(g.run(fwk, batch), want, batch, f"group over {min(n, 8)} devices")
        assert_same(want, c_oracle(snap, batch, fwk), "single vs oracle")
    finally:
        g.close()
        c.close()


def test_group_eight_members_full_c3_equals_single():
    """C3 at full size (1M units x 1000 clusters, the bench's own batch) over an 8-member group — every member
    on device 0, as the box has one GPU — bit-exact with a single context over the whole batch: the split
    the driver's 8-GPU run uses (125 000 units per member), each member's opening phase and work queue on its
    shard, the results at their offsets."""
    import os
    import sys
    import torch  # noqa: F401
    from kubeadmiral_amd import columns as CO
    from kubeadmiral_amd import runtime
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    W, C = synth.SIZES["c3"]
    clusters = bench.make_clusters("c3", C)
    snap = pack.Snapshot(clusters)
    fwk = synth.profile_for("c3")
    nb = CO.NativePacker(snap).pack(fwk, bench.make_columns("c3", 0, W, clusters))
    c = runtime.Context(0)
    g = runtime.GroupContext([0] * 8)
    try:
        c.upload_snapshot(snap)
        c.upload_batch(nb)
        c.schedule(fwk)
        want = c.download()
        g.upload_snapshot(snap)
        g.upload_batch(nb)
        g.schedule(fwk)
        got = g.download()
        ulo, _ = g.ranges()
        assert list(np.diff(ulo)) == [125_000] * 8
        _same_arrays(got, want, nb, "c3 1M over 8 members")
        assert g.path_counts()["units"] == W
    finally:
        g.close()
        c.close()

"""In-place snapshot updates (kad_snapshot_update): cluster update events within the vocabulary.

The reference re-reads the informer's cluster objects on every Schedule call
(generic_scheduler.go:96, cluster events scheduler.go:157-177), so the
property to hold is: scheduling a batch packed against the OLD snapshot on
the UPDATED snapshot gives exactly what a fresh snapshot + fresh batch of the
new cluster list gives (C oracle, oracle/kad_ref.c). CPU tests check the host
side and the delta format (a numpy restatement of the device scatter); the
GPU test applies the delta on the device and reschedules the resident batch.
"""

import os

import numpy as np
import pytest

from kubeadmiral_amd import pack, synth
from kubeadmiral_amd import types as T
from oracle import ref
from tests.gpu_util import assert_same


def _oracle(snap, batch, fwk):
    return ref.schedule(snap, batch, fwk, n_threads=min(8, os.cpu_count() or 1))


def _apply_delta_host(blob: np.ndarray, delta: pack.SnapshotDelta) -> np.ndarray:
    """What snapshot_delta_kernel does (csrc/kad_delta.hip), restated over the blobs."""
    out = blob.copy()
    sh = pack.SnapshotHeader.from_buffer_copy(bytes(blob[:pack.ctypes.sizeof(pack.SnapshotHeader)]))
    dh = pack.SnapshotDeltaHeader.from_buffer_copy(bytes(delta.blob[:pack.ctypes.sizeof(pack.SnapshotDeltaHeader)]))
    n, C = dh.n_changed, sh.n_clusters
    idx = delta.blob[dh.idx_off:dh.idx_off + 4 * n].view(np.int32)
    dims = {"S": sh.n_scalar, "GW": sh.n_gvk_words, "TW": sh.n_taint_words, "K": sh.n_label_keys, None: 1}
    for a, (dt, r) in enumerate(pack.Snapshot.ARRAYS):
        rows, es = dims[r], np.dtype(dt).itemsize
        src = delta.blob[dh.off[a]:dh.off[a] + rows * n * es].view(dt).reshape(rows, n)
        dst = out[sh.off[a]:sh.off[a] + rows * C * es].view(dt).reshape(rows, C)
        dst[:, idx] = src
    return out


CASES = [("fuzz", s) for s in range(6)] + [("c1", 0), ("c4", 1), ("c5", 2)]


def _workload(kind, seed):
    if kind == "fuzz":
        cl, units = synth.gen_fuzz(700 + seed, W=80)
        return cl, units, synth.fuzz_framework(seed)
    return synth.make_config(kind, W=300, C=96 if kind != "c5" else 160, seed=seed)


@pytest.mark.parametrize("kind,seed", CASES)
def test_update_equals_fresh_snapshot(kind, seed):
    cl, units, fwk = _workload(kind, seed)
    snap = pack.Snapshot(cl)
    batch = pack.Batch(snap, fwk, units)
    old_blob = snap.blob.copy()
    rng = np.random.default_rng(seed)
    new, idx = synth.mutate_clusters(rng, cl, max(1, len(cl) // 4))
    delta = snap.update(new)
    assert delta is not None and delta.changed == [i for i in idx if new[i] != cl[i]]
    # the delta carries exactly the host-side update
    assert np.array_equal(_apply_delta_host(old_blob, delta), snap.blob)
    fresh = pack.Snapshot(new)
    assert_same(_oracle(snap, batch, fwk), _oracle(fresh, pack.Batch(fresh, fwk, units), fwk), f"{kind}/{seed}")


def test_resource_only_update_is_byte_identical_to_repack():
    cl, units, fwk = synth.make_config("c2", W=50, C=200, seed=3)
    snap = pack.Snapshot(cl)
    new, _ = synth.mutate_clusters(np.random.default_rng(1), cl, 40, structural=False)
    assert snap.update(new) is not None
    assert np.array_equal(snap.blob, pack.Snapshot(new).blob)


def test_unchanged_list_gives_empty_delta():
    cl, _, _ = synth.make_config("c1", W=1, seed=4)
    snap = pack.Snapshot(cl)
    before = snap.blob.copy()
    d = snap.update(list(cl))
    assert d is not None and d.changed == [] and np.array_equal(before, snap.blob)


def test_vocabulary_growth_and_membership_need_a_full_upload():
    cl, _, _ = synth.make_config("c1", W=1, seed=5)
    snap = pack.Snapshot(cl)
    before = snap.blob.copy()
    import copy

    def with_change(f):
        new = copy.deepcopy(cl)
        f(new)
        return new

    cases = [
        with_change(lambda n: n[3].labels.__setitem__("key0", "never-seen")),       # new label value
        with_change(lambda n: n[3].labels.__setitem__("brand-new-key", "x")),       # new label key
        with_change(lambda n: n[2].taints.append(T.Taint("k", "v", "NoSchedule"))),  # new taint
        with_change(lambda n: n[1].api_resource_types.append(T.APIResource("g", "v9", "K"))),
        with_change(lambda n: n[0].allocatable.__setitem__("example.com/fpga", "2")),  # new scalar name
        cl[:-1],                                                                     # leave
        cl[1:] + cl[:1],                                                             # reorder
        with_change(lambda n: setattr(n[4], "name", "renamed")),
    ]
    for new in cases:
        assert snap.update(new) is None
    assert np.array_equal(before, snap.blob)  # a refused update leaves the snapshot untouched


def test_in_place_edits_and_replaced_elements_are_seen():
    """The same list object, an element replaced and another edited in place: both columns change."""
    cl, _, _ = synth.make_config("c2", W=1, C=40, seed=11)
    snap = pack.Snapshot(cl)
    import copy

    cl2 = list(cl)
    snap2 = pack.Snapshot(cl2)
    cl2[3] = copy.deepcopy(cl2[3])
    cl2[3].available = dict(cl2[3].available, cpu="0")
    cl2[7].available["memory"] = "0"  # edited in place (shared with ``cl``)
    d = snap2.diff(cl2)
    assert d is not None and d.changed == [3, 7]
    assert snap2.diff(cl2).changed == [3, 7]  # not committed yet: still pending
    snap2.commit(d)
    assert snap2.diff(cl2).changed == []
    assert np.array_equal(snap2.blob, pack.Snapshot(cl2).blob)
    del snap


def test_failed_device_update_is_not_committed():
    """BatchScheduler commits host columns only after kad_snapshot_update succeeded; after a failure the
    next call re-uploads the whole snapshot."""
    from kubeadmiral_amd.runtime import BatchScheduler

    class FakeCtx:
        def __init__(self):
            self.snap, self.fail, self.uploads, self.updates = None, False, 0, 0

        def upload_snapshot(self, snap):
            self.snap = snap
            self.uploads += 1

        def update_snapshot(self, delta):
            if self.fail:
                raise RuntimeError("device update failed")
            self.updates += 1

    ctx = FakeCtx()
    bs = BatchScheduler(ctx)
    cl, _, _ = synth.make_config("c1", W=1, seed=12)
    snap = bs.set_clusters(cl)
    before = snap.blob.copy()
    new, _ = synth.mutate_clusters(np.random.default_rng(3), cl, 4, structural=False)
    ctx.fail = True
    with pytest.raises(RuntimeError):
        bs.set_clusters(new)
    assert np.array_equal(before, snap.blob)  # host copy unchanged
    ctx.fail = False
    bs.set_clusters(new)
    assert ctx.uploads == 2 and ctx.updates == 0  # full re-upload after the failure
    newer, _ = synth.mutate_clusters(np.random.default_rng(4), new, 3, structural=False)
    bs.set_clusters(newer)
    assert ctx.updates == 1 and np.array_equal(ctx.snap.blob, pack.Snapshot(newer).blob)


def test_delta_header_layout():
    cl, _, _ = synth.make_config("c5", W=1, C=64, seed=6)
    snap = pack.Snapshot(cl)
    new, idx = synth.mutate_clusters(np.random.default_rng(2), cl, 10)
    d = snap.update(new)
    h = pack.SnapshotDeltaHeader.from_buffer_copy(bytes(d.blob[:pack.ctypes.sizeof(pack.SnapshotDeltaHeader)]))
    assert h.magic == pack.DELTA_MAGIC and h.fingerprint == snap.fingerprint and h.n_clusters == len(cl)
    assert h.total_bytes == d.blob.nbytes and h.n_changed == len(d.changed)
    assert all(o % pack.ALIGN == 0 for o in list(h.off) + [h.idx_off])
    assert list(d.blob[h.idx_off:h.idx_off + 4 * h.n_changed].view(np.int32)) == d.changed


def _norm(r):
    """ScheduleErrors compare by error class (parity is on the class, not the message)."""
    return ("error", r.stage) if isinstance(r, T.ScheduleError) else r


@pytest.mark.gpu
@pytest.mark.parametrize("kind,seed", CASES)
def test_gpu_delta_reschedules_resident_batch(kind, seed):
    from kubeadmiral_amd.runtime import Context

    cl, units, fwk = _workload(kind, seed)
    snap = pack.Snapshot(cl)
    batch = pack.Batch(snap, fwk, units)
    ctx = Context(0)
    ctx.upload_snapshot(snap)
    assert_same(ctx.run(fwk, batch), _oracle(snap, batch, fwk), f"{kind}/{seed} before")
    rng = np.random.default_rng(100 + seed)
    for step in range(3):  # several events in a row against the same resident batch
        new, _ = synth.mutate_clusters(rng, snap.clusters, max(1, len(cl) // (3 + step)))
        delta = snap.update(new)
        assert delta is not None
        ctx.update_snapshot(delta)
        ctx.schedule(fwk)  # resident batch, no re-upload
        assert_same(ctx.download(), _oracle(snap, batch, fwk), f"{kind}/{seed} step {step}")
    ctx.close()


@pytest.mark.gpu
def test_gpu_delta_rejects_foreign_vocabulary():
    from kubeadmiral_amd.runtime import Context, KadError

    cl, _, _ = synth.make_config("c1", W=1, seed=7)
    a, b = pack.Snapshot(cl), pack.Snapshot(cl[:-1])
    ctx = Context(0)
    ctx.upload_snapshot(b)
    new, _ = synth.mutate_clusters(np.random.default_rng(0), cl, 3)
    d = a.update(new)
    with pytest.raises(KadError, match="KAD_EINVAL"):
        ctx.update_snapshot(d)
    ctx.close()


@pytest.mark.gpu
def test_gpu_batch_scheduler_uses_deltas():
    from kubeadmiral_amd.results import to_schedule_result
    from kubeadmiral_amd.runtime import BatchScheduler

    cl, units, fwk = synth.make_config("c1", W=200, seed=8)
    bs = BatchScheduler()
    bs.schedule(fwk, units, cl)
    rng = np.random.default_rng(9)
    cur = cl
    for _ in range(3):
        cur, _ = synth.mutate_clusters(rng, cur, 5)
        got = bs.schedule(fwk, units, cur)
        fresh = pack.Snapshot(cur)
        want_b = pack.Batch(fresh, fwk, units)
        want = _oracle(fresh, want_b, fwk)
        assert [_norm(r) for r in got] == [_norm(to_schedule_result(want, w, su, fresh.names))
                                           for w, su in enumerate(units)]
    assert bs.full_uploads == 1 and bs.delta_updates == 3

"""Multi-rank layout of the hot path on CPU (gloo, world_size 2).

kubeadmiral_amd/shard.py: rank 0 packs the cluster snapshot and broadcasts the
blob; every rank checks it against its own packing (fingerprint), schedules a
contiguous shard of the units, and rank 0 gathers the rows. The gathered rows
must equal one unsharded run: units are independent in the reference
(generic_scheduler.go:92-150), so sharding is exact. The C oracle stands in for
the GPU here (tests only); bench.py runs the same layout over RCCL.
"""

import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from kubeadmiral_amd import shard, synth
from kubeadmiral_amd.pack import Batch, Snapshot
from oracle import ref


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _make(seed, W, C):
    clusters, units = synth.gen_fuzz(seed, W=W, C=C)
    return clusters, units, synth.fuzz_framework(seed)


def _worker(rank, world, port, seed, W, C, outdir):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        clusters, units, fwk = _make(seed, W, C)
        snap = Snapshot(clusters)
        blob = shard.broadcast_blob(snap.blob if rank == 0 else None, dist).numpy()
        shard.check_snapshot(blob, snap.fingerprint)
        assert np.array_equal(blob, snap.blob)
        lo, hi = shard.shard_range(len(units), rank, world)
        batch = Batch(snap, fwk, units[lo:hi])
        res = ref.schedule(snap, batch, fwk)
        rows = shard.gather_rows(shard.rows_of(res), dist)
        if rank == 0:
            with open(os.path.join(outdir, "rows.txt"), "w") as f:
                f.write(repr(rows))
    finally:
        dist.destroy_process_group()


def test_shard_range_covers():
    for n in (0, 1, 5, 64, 1001):
        for world in (1, 2, 3, 8):
            spans = [shard.shard_range(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [h - l for l, h in spans]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard.shard_range(10, 2, 2)


def test_check_snapshot_rejects_other_snapshot():
    a, _, _ = _make(3, 4, 8)
    b, _, _ = _make(4, 4, 9)
    sa, sb = Snapshot(a), Snapshot(b)
    shard.check_snapshot(sa.blob, sa.fingerprint)
    with pytest.raises(RuntimeError):
        shard.check_snapshot(sb.blob, sa.fingerprint)


@pytest.mark.parametrize("seed", [11, 12])
def test_gloo_world2_sharded_equals_unsharded(tmp_path, seed):
    W, C = 45, 23
    mp.start_processes(_worker, args=(2, _free_port(), seed, W, C, str(tmp_path)), nprocs=2, join=True,
                       start_method="spawn")
    with open(tmp_path / "rows.txt") as f:
        got = eval(f.read())  # our own repr of tuples/lists/ints
    clusters, units, fwk = _make(seed, W, C)
    snap = Snapshot(clusters)
    batch = Batch(snap, fwk, units)
    want = shard.rows_of(ref.schedule(snap, batch, fwk))
    assert len(got) == W
    assert got == want

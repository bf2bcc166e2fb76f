"""C4 and C5 at the sizes bench.py reports them, on the GPU, against the C oracle on every unit.

* C4: 1 000 000 Divide units x 512 clusters (weights, min/max replicas, capacity caps) — the planner
  (util/planner/planner.go:211-304) and ClusterCapacityWeight (plugins/rsp/rsp.go:65-181) on every row;
* C5: 100 000 units x 10 000 clusters (dense label affinity, 256 taint ids, API-resource gaps) —
  ClusterAffinity (plugins/clusteraffinity/cluster_affinity.go:50-140) and the long-row kernel.

Each batch is the bench's own (bench.make_clusters / make_columns → native packer), scheduled once through
the C ABI, compared row by row with oracle/kad_ref.c (16 threads, about 1 s of CPU each), then checked
for the size-independent properties: counts within the packed output bound, ascending cluster ids per
unit, Divide replicas >= 0 (C4), a byte-identical rerun.
"""

import os
import sys

import numpy as np
import pytest

from gpu_util import assert_same, c_oracle
from kubeadmiral_amd import columns as CO
from kubeadmiral_amd import pack, synth

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(cfg):
    import torch  # noqa: F401  (the HIP runtime is torch's: initialise it before libkad.so)
    sys.path.insert(0, ROOT)
    import bench
    from kubeadmiral_amd import build, runtime
    build.build()
    W, C = synth.SIZES[cfg]
    clusters = bench.make_clusters(cfg, C)
    cols = bench.make_columns(cfg, 0, W, clusters)
    snap = pack.Snapshot(clusters)
    fwk = synth.profile_for(cfg)
    nb = CO.NativePacker(snap).pack(fwk, cols)
    ctx = runtime.Context(0)
    ctx.upload_snapshot(snap)
    ctx.upload_batch(nb)
    ctx.schedule(fwk)
    res = ctx.download()
    return ctx, snap, nb, cols, fwk, res


def _structure(res, W, C):
    cnt = res.count.astype(np.int64)
    bound = np.diff(res.out_off)
    assert (cnt >= 0).all() and (cnt <= bound).all()
    assert (cnt[(res.status != pack.ST_OK) & (res.status != pack.ST_STICKY)] == 0).all()
    slot_unit = np.repeat(np.arange(W), cnt)
    pos = np.arange(len(slot_unit)) - np.repeat(np.cumsum(cnt) - cnt, cnt)
    idx = np.repeat(res.out_off[:-1], cnt) + pos
    ids = res.cluster[idx]
    assert ((ids >= 0) & (ids < C)).all()
    same = slot_unit[1:] == slot_unit[:-1]
    assert (np.diff(ids)[same] > 0).all()
    return idx


def _rerun_identical(ctx, fwk, res):
    ctx.schedule(fwk)
    res2 = ctx.download()
    for a in ("status", "count", "flags", "cluster", "replicas"):
        assert np.array_equal(getattr(res2, a), getattr(res, a)), a


@pytest.fixture(scope="module")
def full_c4():
    out = _run("c4")
    yield out
    out[0].close()


@pytest.fixture(scope="module")
def full_c5():
    out = _run("c5")
    yield out
    out[0].close()


def test_c4_full_equals_c_oracle(full_c4):
    ctx, snap, nb, cols, fwk, res = full_c4
    assert nb.W == 1_000_000 and snap.C == 512
    assert ctx.path_counts()["planner_rows"] > 0.5 * nb.W  # the planner runs on most rows
    assert_same(res, c_oracle(snap, nb, fwk), "c4 1M x 512")


def test_c4_full_properties(full_c4):
    ctx, snap, nb, cols, fwk, res = full_c4
    idx = _structure(res, nb.W, snap.C)
    ok = res.status == pack.ST_OK
    assert ok.mean() > 0.5
    # Divide units: every selected cluster carries a replica count (>= 0; Duplicate's nil pointer is -1)
    assert (res.replicas[idx] >= 0).all()
    _rerun_identical(ctx, fwk, res)


def test_c5_full_equals_c_oracle(full_c5):
    ctx, snap, nb, cols, fwk, res = full_c5
    assert nb.W == 100_000 and snap.C == 10_000
    assert ctx.path_counts()["row_kernel"] > 0  # long feasible lists take the row kernel
    assert_same(res, c_oracle(snap, nb, fwk), "c5 100k x 10k")


def test_c5_full_properties(full_c5):
    ctx, snap, nb, cols, fwk, res = full_c5
    _structure(res, nb.W, snap.C)
    hist = {int(s): int(n) for s, n in zip(*np.unique(res.status, return_counts=True))}
    assert hist.get(pack.ST_OK, 0) > 0.3 * nb.W, hist
    assert hist.get(pack.ST_NO_FEASIBLE, 0) > 0, hist  # the adversarial filters empty some units
    _rerun_identical(ctx, fwk, res)

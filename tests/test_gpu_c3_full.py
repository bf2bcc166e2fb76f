"""C3 at its full size on the GPU: 1 000 000 units x 1 000 clusters (BASELINE.json north_star config).

The batch is the bench's own (columnar generator → native packer, bench.py make_clusters / make_columns),
scheduled once through the C ABI, then
* against the C oracle on every unit (oracle/kad_ref.c, 16 threads: about 1 s of CPU for 1e9 decisions);
* under the properties SURVEY §8 asks at this size: status histogram, counts <= MaxClusters and <= the
  packed output bound, cluster ids in [0, C) strictly ascending per unit, byte-identical rerun.
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
W, C = 1_000_000, 1000


def _full(cfg):
    import torch  # noqa: F401  (the HIP runtime is torch's: initialise it before libkad.so)
    sys.path.insert(0, ROOT)
    import bench
    from kubeadmiral_amd import build, runtime
    build.build()
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


@pytest.fixture(scope="module")
def full_c3():
    out = _full("c3")
    yield out
    out[0].close()


def test_c3r_full_equals_c_oracle():
    """c3r at full size: C3 with ~150 Kind-sorted discovery API resources per cluster (3 GVK words) and units
    over 8 workload kinds — the APIResources filter on GVK ids past word 0 stays on the folded fast path (no
    unit on the full kernel) and every row equals the C oracle's."""
    ctx, snap, nb, cols, fwk, res = _full("c3r")
    try:
        assert snap.GW == 3
        assert ctx.path_counts()["full_kernel"] == 0
        assert_same(res, c_oracle(snap, nb, fwk), "c3r 1M x 1000")
    finally:
        ctx.close()


def test_c3_full_equals_c_oracle(full_c3):
    ctx, snap, nb, cols, fwk, res = full_c3
    assert_same(res, c_oracle(snap, nb, fwk), "c3 1M x 1000")


def test_c3_full_properties(full_c3):
    ctx, snap, nb, cols, fwk, res = full_c3
    st = res.status
    hist = {int(s): int(n) for s, n in zip(*np.unique(st, return_counts=True))}
    # C3's units have no placement / sticky / scalar requests: every unit is scheduled or has no feasible cluster
    assert set(hist) <= {pack.ST_OK, pack.ST_NO_FEASIBLE}, hist
    assert hist.get(pack.ST_OK, 0) > 0.5 * W, hist
    cnt = res.count.astype(np.int64)
    bound = np.diff(res.out_off)
    assert (cnt >= 0).all() and (cnt <= bound).all()
    has_max = (cols["flags"] & CO.SU_HAS_MAX_CLUSTERS) != 0
    assert has_max.all()  # the C3 generator always sets MaxClusters (1..16)
    assert (cnt <= cols["max_clusters"]).all()
    assert (cnt[st != pack.ST_OK] == 0).all()
    # selected cluster ids: in range, strictly ascending within a unit
    slot_unit = np.repeat(np.arange(W), cnt)
    starts = res.out_off[:-1]
    pos = np.arange(len(slot_unit)) - np.repeat(np.cumsum(cnt) - cnt, cnt)
    ids = res.cluster[np.repeat(starts, cnt) + pos]
    assert ((ids >= 0) & (ids < C)).all()
    same_unit = slot_unit[1:] == slot_unit[:-1]
    assert (np.diff(ids)[same_unit] > 0).all()
    # MaxCluster ties cut by the pdqsort replay are part of this batch
    assert (res.flags & pack.RF_TIE_STRADDLE).mean() > 0.05
    # byte-identical rerun
    ctx.schedule(fwk)
    res2 = ctx.download()
    for a in ("status", "count", "flags", "cluster", "replicas"):
        assert np.array_equal(getattr(res2, a), getattr(res, a)), a


def test_c3p_full_equals_c_oracle():
    """c3p at full size: c3r's snapshots with over-committed (available < 0) and fully cordoned (empty
    allocatable) clusters, units without ResourceRequest (the live controller's, schedulingtriggers.go:188-191).
    The relaxed snapshot stays on the exact-f64 fast path: the wide kernel, no unit on the full kernel, and
    every row equals the C oracle's."""
    ctx, snap, nb, cols, fwk, res = _full("c3p")
    try:
        paths = ctx.snapshot_paths()
        assert paths == {"resource_class": "relaxed", "exact_f64": True, "wide": True, "fold": True,
                         "fitfold": True}, paths
        assert ctx.path_counts()["full_kernel"] == 0
        assert_same(res, c_oracle(snap, nb, fwk), "c3p 1M x 1000")
    finally:
        ctx.close()

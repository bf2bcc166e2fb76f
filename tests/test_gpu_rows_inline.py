"""The wide kernel's opening phase (row_units on the wide blocks, BatchDev::early_rows) at the shape of round
5's GPU fault: the 8-GPU shard of C3 (its first 125 000 units), with more routed units than wide-kernel
blocks and routed units at the first and last index, bit-exact against the C oracle.

The fault (gpurun_out/r05inl2.log, "illegal memory access" in kad_sync after step_ab.py at 125k units) came
from an intermediate build whose noinline wide_rows read the kernel's arguments through the kernarg segment
pointer, which a callee does not receive (the pointer is 0 there): kubeadmiral_amd/isa_check.py now rejects
such code at build time (tests/test_isa_guard.py), and this test runs the shipped path on that shape."""

import os
import sys

import numpy as np
import pytest

from gpu_util import assert_same, c_oracle
from kubeadmiral_amd import columns as CO
from kubeadmiral_amd import synth
from kubeadmiral_amd import types as T

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
W, C = 125_000, 1000


def _open_unit(su):
    """su with every filter open: no affinity / selector, every taint tolerated, no request — all 1000
    clusters feasible (> WIDE_P = 512: prep routes it to the row body); MaxClusters 16 cuts ties."""
    su.affinity = None
    su.cluster_selector = None
    su.tolerations = [T.Toleration(key="", operator=T.TOLERATION_OP_EXISTS)]
    su.resource_request = T.Resource()
    su.max_clusters = 16
    return su


def test_c3_shard_routed_units_equal_c_oracle():
    import torch  # noqa: F401
    sys.path.insert(0, ROOT)
    import bench
    from kubeadmiral_amd import build, pack, runtime
    build.build()
    clusters = bench.make_clusters("c3", C)
    units = CO.to_units(bench.make_columns("c3", 0, W, clusters))
    opened = list(range(0, W, 97)) + [W - 2, W - 1]  # 1 290 routed units: ~5 per wide-kernel block
    for w in opened:
        _open_unit(units[w])
    snap = pack.Snapshot(clusters)
    fwk = synth.profile_for("c3")
    nb = CO.NativePacker(snap).pack(fwk, CO.from_units(units))
    ctx = runtime.Context(0)
    try:
        ctx.upload_snapshot(snap)
        assert ctx.snapshot_paths()["wide"]
        ctx.upload_batch(nb)
        ctx.schedule(fwk)
        res = ctx.download()
        pc = ctx.path_counts()
        assert pc["full_kernel"] == 0
        assert pc["row_kernel"] >= len(opened) > 256, pc
        want = c_oracle(snap, nb, fwk)
        assert_same(res, want, "c3 125k shard with routed units")
        # the opened units took 16 of their 1000 feasible clusters, most through a straddling tie
        assert (res.count[opened] == 16).all()
        assert res.status[W - 1] == 0 and res.count[W - 1] == 16
        # a second launch on the same resident batch (the work heads and the row list reset by the kernels)
        ctx.schedule(fwk)
        res2 = ctx.download()
        assert np.array_equal(res2.cluster, res.cluster) and np.array_equal(res2.status, res.status)
    finally:
        ctx.close()

"""Score and filter programs longer than the 64-word windows the kernels load them through.

The lean and wide kernels read a unit's ClusterAffinity score program as one 64-word window load and parse it
with v_readlane (affinity_score_pv, words past 63 from memory); prep_wave_kernel does the same with the filter
program; schedule_row_kernel stages at most ROW_PRE_PROG words in LDS. Units with 14-20 preferred terms of 1-4
expressions (score programs of ~50-120 words) and 6-9 required terms (filter programs past 64 words) at C = 200
(lean, 4 chunks), 700 (wide) and 5000 (prep_wave, lean / row kernels) against the C oracle
(cluster_affinity.go:50-140, MaxCluster's tie replay on the totals).
"""

import numpy as np
import pytest

from gpu_util import assert_same, c_oracle
from kubeadmiral_amd import framework as F
from kubeadmiral_amd import pack, synth
from kubeadmiral_amd import types as T

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import torch  # noqa: F401  (the HIP runtime is torch's: initialise it before libkad.so)
    from kubeadmiral_amd import build, runtime
    build.build()
    c = runtime.Context(0)
    yield c
    c.close()


def _units(rng, clusters, W):
    out = []
    for w in range(W):
        req = [T.ClusterSelectorTerm([synth._expr(rng, 8, 4, all_ops=True) for _ in range(int(rng.integers(2, 6)))])
               for _ in range(int(rng.integers(6, 10)))]
        prefs = [T.PreferredSchedulingTerm(int(rng.integers(1, 101)), T.ClusterSelectorTerm(
            [synth._expr(rng, 8, 4, all_ops=True) for _ in range(int(rng.integers(1, 5)))]))
            for _ in range(int(rng.integers(14, 21)))]
        out.append(T.SchedulingUnit(
            group="apps", version="v1", kind="Deployment", namespace="default", name=f"lp-{w}", desired_replicas=5,
            scheduling_mode=T.SCHEDULING_MODE_DUPLICATE if w % 2 else T.SCHEDULING_MODE_DIVIDE,
            max_clusters=int(rng.integers(1, 12)), affinity=T.Affinity(T.ClusterAffinity(T.ClusterSelector(req), prefs)),
            resource_request=T.Resource(int(rng.integers(0, 4000)), int(rng.integers(0, 8 * synth.GI)))))
    return out


@pytest.mark.parametrize("C", [200, 700, 5000])
def test_long_programs_equal_c_oracle(ctx, C):
    rng = np.random.default_rng(0x1060 + C)
    clusters = synth.gen_clusters(rng, C, n_keys=8, n_vals=4)
    units = _units(rng, clusters, 300)
    fwk = F.Framework(F.default_enabled_plugins())
    snap = pack.Snapshot(clusters)
    batch = pack.Batch(snap, fwk, units)
    ctx.upload_snapshot(snap)
    got = ctx.run(fwk, batch)
    want = c_oracle(snap, batch, fwk)
    assert_same(got, want, f"long programs C={C}")
    assert (want.status == pack.ST_OK).sum() > 30  # enough units pass the long filters to be scored

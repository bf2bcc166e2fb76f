"""prep_wave_kernel (one unit per wave, snapshots of 65-256 chunks) on every filter input it folds, against the
C oracle: ClusterNames placement lists and CurrentClusters (the per-chunk id-list words,
placement/filter.go:37-57 and taint_toleration.go:64-78), up to 256 taint ids, API-resource gaps, required
affinity terms (cluster_affinity.go:50-94) and the cpu / memory fit rows — at 65-80, 129-192 and 193-256
chunks (the <2>, <3> and <4> instantiations). C5's bench batch covers the affinity-heavy case at full size
(test_gpu_full_configs.py); its units have no placement or current clusters.
"""

import numpy as np
import pytest

from gpu_util import assert_same, c_oracle
from kubeadmiral_amd import framework as F
from kubeadmiral_amd import pack, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import torch  # noqa: F401  (the HIP runtime is torch's: initialise it before libkad.so)
    from kubeadmiral_amd import build, runtime
    build.build()
    c = runtime.Context(0)
    yield c
    c.close()


@pytest.mark.parametrize("C", [4500, 9000, 15000])
def test_prep_wave_placement_current_taints_affinity(ctx, C):
    rng = np.random.default_rng(0x9E0 + C)
    clusters = synth.gen_clusters(rng, C, n_keys=16, n_vals=8, n_taints=256, taints_per=(0, 6), p_gvk=0.9,
                                  gvks=synth.GVKS)
    units = synth.gen_units_c4(rng, 400, clusters) + synth.gen_units_c5(rng, 400, clusters, n_keys=16, n_vals=8)
    for su in units:  # tolerations over the whole id range
        su.tolerations = (su.tolerations or []) + synth._tolerations(rng, 256, 0, 4)
    fwk = F.Framework(F.default_enabled_plugins())
    snap = pack.Snapshot(clusters)
    batch = pack.Batch(snap, fwk, units)
    ctx.upload_snapshot(snap)
    got = ctx.run(fwk, batch)
    assert_same(got, c_oracle(snap, batch, fwk), f"prep_wave C={C}")
    # the C4-shaped units really carry placement and current-cluster lists through this path
    assert any(su.cluster_names for su in units) and any(su.current_clusters for su in units)

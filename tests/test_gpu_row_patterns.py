"""MaxCluster over long feasible lists with structured score sequences, through schedule_row_kernel's
workgroup-wide pdqsort replay (kad_select.h PdqWaveP::select_block / fused_block, then wave 0's
select_from): every cluster is feasible (n = C > the wide kernel's 512 positions), LeastAllocated gives
cluster c exactly the total s[c] (allocatable 100 cores / 100Gi, available s[c] of each), and MaxClusters
puts the cut inside a run of equal totals, so the first-k set depends on Go's exact swap sequence
(max_cluster.go:42-66, go1.19 sort.Slice → pdqsort_func). The patterns drive the rare branches of the replay
on ranges longer than the block threshold: already sorted (partialInsertionSort), reversed (choosePivot's
decreasing hint → reverseRange), organ pipe and sawtooth (unbalanced partitions → breakPatterns, the
heapSort fallback), a single value (partitionEqual), few values. Checked against the C oracle's full sort."""
import zlib

import numpy as np
import pytest

from gpu_util import assert_same, c_oracle
from kubeadmiral_amd import framework as F
from kubeadmiral_amd import pack
from kubeadmiral_amd import types as T

pytestmark = pytest.mark.gpu

# C = 1000: the wide path (5..16 chunks) routes units with more than 512 feasible clusters to the row kernel
# from prep_kernel (beside the wide kernel); C = 1500: the lean kernel's NCH = 0 path hands units with more
# than 256 to it after its own pass


def _patterns(rng, C):
    i = np.arange(C)
    return {
        "ascending": (i * 100) // C,
        "descending": 99 - (i * 100) // C,
        "organ_pipe": np.minimum(i, C - 1 - i) * 100 // (C // 2 + 1),
        "sawtooth7": i % 7,
        "sawtooth61": (i * 3) % 61,
        "constant": np.full(C, 42),
        "two_runs": np.where(i < 700, 10, 90),
        "few_values": rng.integers(0, 4, C),
        "mostly_sorted": np.sort(rng.integers(0, 30, C))[::-1].copy(),
        "random": rng.integers(0, 101, C),
    }


@pytest.fixture(scope="module")
def ctx():
    from kubeadmiral_amd import build, runtime
    build.build()
    c = runtime.Context(0)
    yield c
    c.close()


@pytest.mark.parametrize("C", [1000, 1500])
@pytest.mark.parametrize("pattern", ["ascending", "descending", "organ_pipe", "sawtooth7", "sawtooth61",
                                     "constant", "two_runs", "few_values", "mostly_sorted", "random"])
def test_row_kernel_replay_patterns(ctx, pattern, C):
    rng = np.random.default_rng(zlib.crc32(pattern.encode()) + C)
    s = _patterns(rng, C)[pattern].astype(int)
    assert s.min() >= 0 and s.max() <= 100
    clusters = [T.FederatedCluster(name=f"pc-{c:04d}", allocatable={"cpu": "100", "memory": "100Gi"},
                                   available={"cpu": str(int(v)), "memory": f"{int(v)}Gi"})
                for c, v in enumerate(s)]
    fwk = F.Framework(F.EnabledPlugins([F.ClusterResourcesFit], [F.ClusterResourcesLeastAllocated], [F.MaxCluster],
                                       []))
    ks = [1, 2, 13, 64, 257, 333, 499, 500, 501, 512, 700, 999, C - 1]
    units = [T.SchedulingUnit(group="apps", version="v1", kind="Deployment", namespace="ns", name=f"u{j}",
                              scheduling_mode=T.SCHEDULING_MODE_DUPLICATE, max_clusters=k)
             for j, k in enumerate(ks)]
    snap = pack.Snapshot(clusters)
    batch = pack.Batch(snap, fwk, units)
    ctx.upload_snapshot(snap)
    got = ctx.run(fwk, batch)
    want = c_oracle(snap, batch, fwk)
    assert (got.status == pack.ST_OK).all()
    assert (got.count == np.minimum(ks, C)).all()
    assert ctx.path_counts()["row_kernel"] == len(ks), "every unit must take schedule_row_kernel"
    assert_same(got, want, f"pattern {pattern} C={C}")

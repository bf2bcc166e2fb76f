"""HIP path (libkad.so on an MI355X) == the oracle, bit for bit.

* golden vectors of the reference's own tests, through the C ABI: filters,
  scores (debug output), MaxCluster (stage entry point), planner (stage entry
  point, with planner_test.go's convergence driver), rsp plugin (full pipeline)
* fuzz batches covering every branch vs the C oracle and the Python oracle
* config-scale batches (C1, C2 at full size, C4/C5 subsets) vs the C oracle
* large-C rows that spill the per-wave state to global scratch
* determinism (two runs, identical bytes)
"""

import os

import numpy as np
import pytest

from golden_util import case_id, load
from gpu_util import assert_same, c_oracle
from kubeadmiral_amd import framework as F
from kubeadmiral_amd import k8s, pack, synth
from kubeadmiral_amd import types as T
from kubeadmiral_amd.results import to_schedule_result

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from kubeadmiral_amd import build, runtime
    build.build()
    c = runtime.Context(0)
    yield c
    c.close()


def run(ctx, clusters, units, fwk):
    snap = pack.Snapshot(clusters)
    batch = pack.Batch(snap, fwk, units)
    ctx.upload_snapshot(snap)
    return snap, batch, ctx.run(fwk, batch)


# ------------------------------------------------------------------ golden
FILTERS = load("filters.json")
SCORES = load("scores.json")
MAXC = load("maxcluster.json")
PLANNER = load("planner.json")
RSP = load("rsp_plugin.json")


@pytest.mark.parametrize("c", FILTERS, ids=[case_id(c) for c in FILTERS])
def test_golden_filter_on_gpu(ctx, c):
    su = T.SchedulingUnit.from_json(c["su"])
    su.scheduling_mode = T.SCHEDULING_MODE_DUPLICATE
    su.sticky_cluster = False
    su.max_clusters = None
    cl = T.FederatedCluster.from_json(c["cluster"])
    fwk = F.Framework(F.EnabledPlugins([c["plugin"]], [], [], []))
    _, _, res = run(ctx, [cl], [su], fwk)
    st, pairs = res.row(0)
    feasible = st == pack.ST_OK and len(pairs) == 1
    if c["want"] == "Success":
        assert feasible
    else:
        assert st == pack.ST_NO_FEASIBLE


@pytest.mark.parametrize("c", SCORES, ids=[case_id(c) for c in SCORES])
def test_golden_score_on_gpu(ctx, c):
    su = T.SchedulingUnit.from_json(c["su"])
    su.scheduling_mode = T.SCHEDULING_MODE_DUPLICATE
    clusters = [T.FederatedCluster.from_json(x) for x in c["clusters"]]
    fwk = F.Framework(F.EnabledPlugins([], [c["plugin"]], [], []))
    snap = pack.Snapshot(clusters)
    batch = pack.Batch(snap, fwk, [su])
    ctx.upload_snapshot(snap)
    ctx.upload_batch(batch)
    feas, tot = ctx.debug_scores(fwk)
    assert feas[0].all()
    assert tot[0].tolist() == c["want"]


@pytest.mark.parametrize("c", MAXC, ids=[case_id(c) for c in MAXC])
def test_golden_maxcluster_on_gpu(ctx, c):
    su = T.SchedulingUnit.from_json(c["su"])
    names = [n for n, _ in c["scores"]]
    [(st, sel)] = ctx.select_rows([[s for _, s in c["scores"]]], [su.max_clusters])
    if c["want"] != "Success":
        assert st == pack.ST_ERR_SELECT
        return
    assert st == pack.ST_OK
    assert sorted(names[i] for i in sel) == sorted(c["want_clusters"])


def _gpu_plan(ctx, rsp, replicas, clusters, existing, est, avoid, keep):
    prefs = []
    for cl in clusters:
        p = rsp.get(cl, rsp.get("*"))
        if p is not None:
            prefs.append((cl, p))
    row = {"elems": [{"hash": k8s.fnv1_32(n.encode()), "weight": p.weight, "min": p.min_replicas,
                      "max": p.max_replicas, "cap": est.get(n), "current": (existing or {}).get(n, 0)}
                     for n, p in prefs], "total": replicas, "avoid": avoid, "keep": keep}
    [(plan, over)] = ctx.plan_rows([row])
    return ({n: v for (n, _), v in zip(prefs, plan)},
            {n: v for (n, _), v in zip(prefs, over) if v is not None})


@pytest.mark.parametrize("path", ["lanes", "ws", "pairs"])
@pytest.mark.parametrize("c", PLANNER, ids=[f"{case_id(c)}-a{int(c['avoidDisruption'])}k{int(c['keepUnschedulableReplicas'])}"
                                            for c in PLANNER])
def test_golden_planner_on_gpu(ctx, c, path, monkeypatch):
    """planner_test.go's cases through kad_plan_rows: the register planner (rows of K <= 64, plan_row_lanes),
    the LDS-workspace planner (kad_debug_plan_force_workspace 1, the path of rows with K > 64) and the
    half-wave pair planner (2: plan_row_pair, plan_pair_kernel's path for rows of K <= 32)."""
    from test_oracle_golden import run_planner_case
    ctx.plan_force_workspace({"lanes": 0, "ws": 1, "pairs": 2}[path])
    try:
        converged, plan, over = run_planner_case(
            c, lambda rsp, r, cl, ex, est, key, av, kp: _gpu_plan(ctx, rsp, r, cl, ex, est, av, kp))
    finally:
        ctx.plan_force_workspace(False)
    assert converged
    if plan or c["want_plan"]:
        assert plan == c["want_plan"]
    if over or c["want_overflow"]:
        assert over == c["want_overflow"]


@pytest.mark.parametrize("seed", range(6))
def test_plan_rows_lanes_equal_workspace(ctx, seed, monkeypatch):
    """Random rows (K 1..64, weights/minimums/maximums/capacities/current replicas incl. zero, tie-heavy
    hashes, avoid/keep both ways): the register planner and the LDS-workspace planner agree exactly."""
    rng = np.random.default_rng(seed)
    rows = []
    for _ in range(300):
        K = int(rng.integers(1, 65))
        hs = rng.integers(0, 4 if rng.random() < 0.3 else 1 << 32, K)
        elems = []
        for i in range(K):
            elems.append({"hash": int(hs[i]), "weight": int(rng.integers(0, 5 if rng.random() < 0.4 else 1000)),
                          "min": int(rng.integers(0, 6)) if rng.random() < 0.3 else 0,
                          "max": int(rng.integers(0, 200)) if rng.random() < 0.3 else None,
                          "cap": int(rng.integers(0, 300)) if rng.random() < 0.25 else None,
                          "current": int(rng.integers(0, 400)) if rng.random() < 0.5 else 0})
        rows.append({"elems": elems, "total": int(rng.integers(0, 20_000)), "avoid": bool(rng.random() < 0.5),
                     "keep": bool(rng.random() < 0.5)})
    lanes = ctx.plan_rows(rows)
    ctx.plan_force_workspace(True)
    try:
        ws = ctx.plan_rows(rows)
    finally:
        ctx.plan_force_workspace(False)
    assert lanes == ws


@pytest.mark.parametrize("seed", range(8))
def test_plan_rows_pairs_equal_lanes(ctx, seed):
    """The half-wave pair planner (two rows of K <= 32 per wave, plan_row_pair) against the 64-lane register
    planner on random rows: K 1..40 (pairs with one row past 32 fall back to one row per wave), tie-heavy
    hashes, weights up to 2^26 on some rows (the non-kbuf rank path), totals past 2^24 on some rows (the
    int64 desired-plan path beside a narrow row), minimums / maximums / capacities / current replicas,
    avoid / keep both ways."""
    rng = np.random.default_rng(700 + seed)
    rows = []
    for _ in range(400):
        K = int(rng.integers(1, 41)) if rng.random() < 0.9 else int(rng.integers(1, 9))
        hs = rng.integers(0, 4 if rng.random() < 0.3 else 1 << 32, K)
        wide_w = rng.random() < 0.05
        elems = []
        for i in range(K):
            elems.append({"hash": int(hs[i]),
                          "weight": int(rng.integers(0, (1 << 26) if wide_w else (5 if rng.random() < 0.4 else 1000))),
                          "min": int(rng.integers(0, 6)) if rng.random() < 0.3 else 0,
                          "max": int(rng.integers(0, 200)) if rng.random() < 0.3 else None,
                          "cap": int(rng.integers(0, 300)) if rng.random() < 0.25 else None,
                          "current": int(rng.integers(0, 400)) if rng.random() < 0.5 else 0})
        total = int(rng.integers(0, 20_000)) if rng.random() < 0.95 else int(rng.integers(1 << 24, 1 << 30))
        rows.append({"elems": elems, "total": total, "avoid": bool(rng.random() < 0.5),
                     "keep": bool(rng.random() < 0.5)})
    lanes = ctx.plan_rows(rows)
    ctx.plan_force_workspace(2)
    try:
        pairs = ctx.plan_rows(rows)
    finally:
        ctx.plan_force_workspace(0)
    assert pairs == lanes


@pytest.mark.parametrize("c", RSP, ids=[case_id(c) for c in RSP])
def test_golden_rsp_on_gpu(ctx, c):
    su = T.SchedulingUnit.from_json(c["su"])
    clusters = [T.FederatedCluster.from_json(x) for x in c["clusters"]]
    fwk = F.Framework(F.EnabledPlugins([], [], [], [F.ClusterCapacityWeight]))
    snap, _, res = run(ctx, clusters, [su], fwk)
    st, pairs = res.row(0)
    assert st == pack.ST_OK
    assert [[snap.names[cid], r] for cid, r in pairs] == c["want"]


# -------------------------------------------------------------------- fuzz
@pytest.mark.parametrize("seed", range(48))
def test_fuzz_gpu_equals_c_oracle(ctx, seed):
    clusters, units = synth.gen_fuzz(seed, W=80)
    fwk = synth.fuzz_framework(seed)
    snap, batch, res = run(ctx, clusters, units, fwk)
    assert_same(res, c_oracle(snap, batch, fwk), f"fuzz seed {seed}")


@pytest.mark.parametrize("seed", range(8))
def test_fuzz_wide_prefs_gpu_equals_c_oracle(ctx, seed):
    """Preference values past int32: the planner reads the i64 columns (KAD_BATCH_NARROW_PREFS off)."""
    clusters, units = synth.gen_fuzz(2000 + seed, W=80)
    synth.widen_prefs(units, seed, share=0.5)
    fwk = synth.fuzz_framework(seed)
    snap, batch, res = run(ctx, clusters, units, fwk)
    assert pack.header_of(batch.blob, pack.BatchHeader).flags == 0
    assert_same(res, c_oracle(snap, batch, fwk), f"wide fuzz seed {seed}")


@pytest.mark.parametrize("seed", range(6))
def test_fuzz_gpu_equals_python_oracle(ctx, seed):
    from test_c_oracle import py_results, same
    clusters, units = synth.gen_fuzz(1000 + seed, W=60)
    fwk = synth.fuzz_framework(seed)
    snap, batch, res = run(ctx, clusters, units, fwk)
    want = py_results(fwk, units, clusters)
    for w, su in enumerate(units):
        got = to_schedule_result(res, w, su, snap.names)
        assert same(got, want[w]), (w, got, want[w])


def test_xorshift_variant_profile_flag(ctx):
    clusters, units = synth.gen_fuzz(77, W=80, C=200)
    fwk = F.Framework(F.default_enabled_plugins(), flags=F.PROFILE_XORSHIFT_GO121)
    snap, batch, res = run(ctx, clusters, units, fwk)
    assert_same(res, c_oracle(snap, batch, fwk), "go1.21 xorshift")


# ------------------------------------------------------------ config scale
def test_c1_full(ctx):
    clusters, units, fwk = synth.make_config("c1")
    snap, batch, res = run(ctx, clusters, units, fwk)
    assert_same(res, c_oracle(snap, batch, fwk), "c1")


def test_c2_full_size(ctx):
    clusters, units, fwk = synth.make_config("c2")
    snap, batch, res = run(ctx, clusters, units, fwk)
    assert (res.status == pack.ST_OK).mean() > 0.5
    assert_same(res, c_oracle(snap, batch, fwk), "c2 100k x 256")
    # determinism: a second run gives identical bytes
    ctx.schedule(fwk)
    res2 = ctx.download()
    assert_same(res2, res, "c2 rerun")
    # timing is off by default (production callers pay no event records): no event times to read
    with pytest.raises(Exception, match="timing off"):
        ctx.timing()
    # timing on (bench's per-kernel times): same bytes, and the stage times are there
    ctx.set_timing(True)
    try:
        ctx.schedule(fwk)
        ctx.sync()
        assert_same(ctx.download(), res, "c2 timing on")
        assert ctx.timing()[1] > 0
    finally:
        ctx.set_timing(False)


def test_c4_subset(ctx):
    clusters, units, fwk = synth.make_config("c4", W=20_000)
    snap, batch, res = run(ctx, clusters, units, fwk)
    assert_same(res, c_oracle(snap, batch, fwk), "c4 20k x 512")


def test_c5_subset(ctx):
    clusters, units, fwk = synth.make_config("c5", W=1500, C=2000)
    snap, batch, res = run(ctx, clusters, units, fwk)
    assert_same(res, c_oracle(snap, batch, fwk), "c5 1.5k x 2k")


def test_c3_clusters_1000(ctx):
    """C3's defining cluster count (C = 1000, 16 chunks: the lean kernel's wide rows, feasible lists beyond
    256 positions) on 20k units of the C3 generator (seed 0xC3), against the C oracle."""
    clusters, units, fwk = synth.make_config("c3", W=20_000)
    assert len(clusters) == 1000
    snap, batch, res = run(ctx, clusters, units, fwk)
    assert (res.status == pack.ST_OK).mean() > 0.5
    assert (res.flags & pack.RF_TIE_STRADDLE).mean() > 0.05  # MaxCluster ties cut: pdqsort replays
    assert_same(res, c_oracle(snap, batch, fwk), "c3 20k x 1000")


@pytest.mark.parametrize("seed", [0xC31, 0xC32])
def test_c3_long_lists_routed_beside_the_wide_kernel(ctx, seed):
    """C = 1000 units whose feasible lists pass WIDE_P = 512 positions (a third of them: no selector, an
    Exists expression only, light requests): prep_kernel routes them to schedule_row_kernel, which runs on
    the side stream beside the wide kernel (BatchDev::early_rows); every row must equal the C oracle's and
    the row path must have taken units."""
    rng = np.random.default_rng(seed)
    clusters = synth.gen_clusters(rng, 1000)
    units = synth.gen_units_c2(rng, 3000)
    for i, su in enumerate(units):
        if i % 3 == 0:
            su.cluster_selector = None
            su.affinity = T.Affinity(T.ClusterAffinity(required=T.ClusterSelector([T.ClusterSelectorTerm(
                [T.ClusterSelectorRequirement(f"key{i % 8}", T.OP_EXISTS, [])])])))
            su.tolerations = [T.Toleration(operator=T.TOLERATION_OP_EXISTS)]
            su.resource_request = T.Resource(int(rng.integers(0, 100)), int(rng.integers(0, 1 << 20)))
    fwk = synth.profile_for("c3")
    snap, batch, res = run(ctx, clusters, units, fwk)
    assert ctx.path_counts()["row_kernel"] > 100
    assert_same(res, c_oracle(snap, batch, fwk), f"c3 long lists seed {seed}")


@pytest.mark.parametrize("seed,C,n_taints", [(7301, 30, 9), (7302, 300, 9), (7303, 1000, 9), (7304, 3000, 9),
                                             (7305, 800, 160), (7306, 500, 300)])
def test_fuzz_discovery_lists(ctx, seed, C, n_taints):
    """Production-shaped API-resource lists (~150 Kind-sorted discovery entries per cluster, GVK ids in 3
    words; clusterstatus.go:221-266) with units over 8 workload kinds and one no cluster serves, under every
    fuzz profile against the C oracle: APIResources.Filter (apiresources.go:25-43) from any GVK word's slice
    on folded snapshots (TW <= 4), from the full kernel on unfolded ones (the last case, TW = 5)."""
    clusters, units = synth.with_discovery(*synth.gen_fuzz(seed, W=120, C=C, n_taints=n_taints), seed)
    for i in range(len(synth.FUZZ_PROFILES)):
        fwk = synth.fuzz_framework(i)
        snap, batch, res = run(ctx, clusters, units, fwk)
        assert snap.GW >= 3
        assert_same(res, c_oracle(snap, batch, fwk), f"discovery fuzz seed {seed} profile {i}")


def test_c3r_clusters_1000(ctx):
    """c3r on 20k units: C3's generator with discovery-shaped API-resource lists and 8 workload kinds (most
    GVK ids >= 64). No unit may fall to the one-wave-per-unit full kernel (GVK ids past word 0
    routed there), and every row equals the C oracle's."""
    clusters, units, fwk = synth.make_config("c3r", W=20_000)
    snap, batch, res = run(ctx, clusters, units, fwk)
    gv = [snap.gvk_id.get((su.group, su.version, su.kind), -1) for su in units]
    assert sum(g >= 64 for g in gv) > 0.5 * len(units)
    assert ctx.path_counts()["full_kernel"] == 0
    assert (res.status == pack.ST_OK).mean() > 0.5
    assert_same(res, c_oracle(snap, batch, fwk), "c3r 20k x 1000")


def test_c3_default_set_divide_subrun(ctx):
    """'a parity sub-run with the full default plugin set in Divide mode' (C = 1000)."""
    rng = np.random.default_rng(synth.SEEDS["c3"] + 1)
    clusters = synth.gen_clusters(rng, 1000)
    units = synth.gen_units_c2(rng, 20_000, mode=T.SCHEDULING_MODE_DIVIDE)
    for i, su in enumerate(units):  # half static weights, half dynamic (rsp.go:69)
        if i % 2 == 0:
            su.weights = {clusters[int(j)].name: int(rng.integers(0, 10)) for j in rng.integers(0, 1000, 24)}
        su.avoid_disruption = bool(i % 3 == 0)
    fwk = F.Framework(F.default_enabled_plugins())
    snap, batch, res = run(ctx, clusters, units, fwk)
    assert (res.status == pack.ST_OK).mean() > 0.5
    assert (res.replicas[:batch.n_out_slots] > 0).any()
    assert_same(res, c_oracle(snap, batch, fwk), "c3 default-set Divide 20k x 1000")


def test_c5_clusters_10000(ctx):
    """C5's defining cluster count (C = 10 000: rows past the LDS budget, global-scratch replays, 256
    taint ids in 4 words, 64 label keys) on 1 000 units of the C5 generator, against the C oracle."""
    clusters, units, fwk = synth.make_config("c5", W=1000, C=10_000)
    assert len(clusters) == 10_000
    snap, batch, res = run(ctx, clusters, units, fwk)
    assert snap.TW == 4
    assert_same(res, c_oracle(snap, batch, fwk), "c5 1k x 10000")


@pytest.mark.parametrize("cfg,W,C", [("c2", 200, 256), ("c3", 60, 1000), ("c4", 100, 512), ("c5", 16, 10_000)])
def test_config_shaped_gpu_equals_python_oracle(ctx, cfg, W, C):
    """The object-level Python oracle (pinned by the reference's golden vectors) on samples of each
    config's own generator: pins the packer at config shape, not only through the C oracle."""
    from test_c_oracle import py_results, same
    clusters, units, fwk = synth.make_config(cfg, W=W, C=C)
    snap, batch, res = run(ctx, clusters, units, fwk)
    want = py_results(fwk, units, clusters)
    for w, su in enumerate(units):
        got = to_schedule_result(res, w, su, snap.names)
        assert same(got, want[w]), (cfg, w, got, want[w])


@pytest.mark.parametrize("seed,C,n_taints", [(5101, 40, 160), (5102, 300, 180), (5103, 1500, 120),
                                             (5104, 200, 100), (5105, 5000, 100), (5103, 1500, 200)])
def test_fuzz_many_taint_words(ctx, seed, C, n_taints):
    """Taint ids spread over 2-4 words (SnapDev::TW > 1): prep folds TaintToleration from the 8-id group
    tables of every word (NoExecute table for units with CurrentClusters), for the lean (NCH = 1..4 and 0)
    and wide kernels, against the C oracle under every fuzz profile; TW > 4 (the last case) runs unfolded."""
    clusters, units = synth.gen_fuzz(seed, W=120, C=C, n_taints=n_taints)
    for i in range(len(synth.FUZZ_PROFILES)):
        fwk = synth.fuzz_framework(i)
        snap, batch, res = run(ctx, clusters, units, fwk)
        assert snap.TW >= 2
        assert_same(res, c_oracle(snap, batch, fwk), f"many taints seed {seed} C={C} profile {i}")


@pytest.mark.parametrize("seed,C,prof", [(6101, 9000, 1), (6102, 3000, 2), (6103, 12000, 3), (6104, 1000, 1),
                                         (6105, 12289, 1)])
def test_row_kernel_long_feasible_lists(ctx, seed, C, prof):
    """Feasible lists longer than the lean (256) / wide (512) kernels' registers go to
    schedule_row_kernel (one workgroup per unit) on folded snapshots: tie-heavy fuzz clusters (half of
    them share one resource shape) so the k-th largest total cuts ties and wave 0 replays pdqsort over
    thousands of positions. C = 12289 is past ROW_MAX_C (those rows take the full kernel)."""
    clusters, units = synth.gen_fuzz(seed, W=300, C=C)
    fwk = synth.fuzz_framework(prof)
    snap, batch, res = run(ctx, clusters, units, fwk)
    ok = res.status == pack.ST_OK
    assert (res.count[ok] > 0).any()
    assert_same(res, c_oracle(snap, batch, fwk), f"rows seed {seed} C={C} profile {prof}")


@pytest.mark.parametrize("seed", [7101, 7102])
def test_requirement_value_rows_and_segments(ctx, seed):
    """Requirement masks from both paths: In / NotIn / Exists / DoesNotExist whose value ids are < 64 and
    at most 5, and the label-free ops (metadata.name, TRUE / FALSE) through req_row_kernel, and the rest —
    value ids >= 64 (a key with 150 distinct values), lists longer than 5, Gt / Lt — through the
    key-grouped segments (req_mask_kernel); ClusterAffinity filter and score against the C oracle."""
    rng = np.random.default_rng(seed)
    C = 700
    clusters = synth.gen_clusters(rng, C, n_keys=3, n_vals=4, n_int_keys=1)
    for c in clusters:  # "wide" has 150 distinct values; some clusters lack it
        if rng.random() < 0.85:
            c.labels = dict(c.labels or {}, wide=f"w{int(rng.integers(0, 150))}")
    names = [c.name for c in clusters]

    def req():
        r = rng.random()
        if r < 0.35:
            vals = [f"w{int(v)}" for v in rng.integers(0, 150, int(rng.integers(1, 9)))]
            return T.ClusterSelectorRequirement("wide", T.OP_IN if rng.random() < 0.5 else T.OP_NOT_IN, vals)
        if r < 0.5:
            return T.ClusterSelectorRequirement("wide", T.OP_EXISTS if rng.random() < 0.5 else T.OP_DOES_NOT_EXIST,
                                                None)
        if r < 0.6:
            return T.ClusterSelectorRequirement("num0", T.OP_GT if rng.random() < 0.5 else T.OP_LT,
                                                [str(int(rng.integers(0, 1000)))])
        return synth._expr(rng, 3, 4, 1, all_ops=True, p_invalid=0.03)

    units = []
    for w in range(400):
        terms = []
        for _ in range(int(rng.integers(1, 4))):
            fields = None
            if rng.random() < 0.2:
                fields = [T.ClusterSelectorRequirement("metadata.name", T.OP_NOT_IN,
                                                       [names[int(rng.integers(0, C))]])]
            terms.append(T.ClusterSelectorTerm([req() for _ in range(int(rng.integers(1, 3)))], fields))
        prefs = [T.PreferredSchedulingTerm(int(rng.integers(1, 50)), T.ClusterSelectorTerm([req()]))
                 for _ in range(int(rng.integers(0, 3)))]
        units.append(T.SchedulingUnit(
            group="apps", version="v1", kind="Deployment", namespace="default", name=f"vr-{w}", desired_replicas=3,
            scheduling_mode=T.SCHEDULING_MODE_DUPLICATE, max_clusters=int(rng.integers(1, 9)),
            affinity=T.Affinity(T.ClusterAffinity(T.ClusterSelector(terms), prefs or None))))
    for fwk in (F.Framework(F.default_enabled_plugins()),
                F.Framework(F.EnabledPlugins([F.ClusterAffinity], [F.ClusterAffinity], [F.MaxCluster], []))):
        snap, batch, res = run(ctx, clusters, units, fwk)
        assert (res.status == pack.ST_OK).mean() > 0.3
        assert_same(res, c_oracle(snap, batch, fwk), f"value rows seed {seed}")


@pytest.mark.parametrize("C", [333, 1000])
def test_label_free_requirements(ctx, C):
    """the label-free requirement ops computed on req_row_kernel without label loads —
    metadata.name In / NotIn on an existing and on an unknown cluster name, ClusterSelector entries on a key
    no cluster has (the Equals requirement is constant FALSE) and DoesNotExist on such a key (constant
    TRUE) — with C not a multiple of 64, ClusterAffinity filter + score against the C oracle."""
    rng = np.random.default_rng(C)
    clusters = synth.gen_clusters(rng, C, n_keys=3, n_vals=4)
    names = [c.name for c in clusters]

    def field():
        op = T.OP_IN if rng.random() < 0.5 else T.OP_NOT_IN
        name = names[int(rng.integers(0, C))] if rng.random() < 0.7 else "no-such-cluster"
        return T.ClusterSelectorRequirement("metadata.name", op, [name])

    def expr():
        r = rng.random()
        if r < 0.3:
            return T.ClusterSelectorRequirement("absent-key", T.OP_DOES_NOT_EXIST, None)
        if r < 0.45:
            return T.ClusterSelectorRequirement("absent-key", T.OP_IN, ["x"])
        return synth._expr(rng, 3, 4, 0, all_ops=False, p_invalid=0.0)

    units = []
    for w in range(500):
        terms = []
        for _ in range(int(rng.integers(1, 3))):
            fields = [field() for _ in range(int(rng.integers(0, 2)))] or None
            exprs = [expr() for _ in range(int(rng.integers(0, 3)))] or None
            terms.append(T.ClusterSelectorTerm(exprs, fields))
        prefs = [T.PreferredSchedulingTerm(int(rng.integers(1, 50)), T.ClusterSelectorTerm(None, [field()]))
                 for _ in range(int(rng.integers(0, 3)))]
        sel = {"absent-key": "v"} if rng.random() < 0.1 else None
        units.append(T.SchedulingUnit(
            group="apps", version="v1", kind="Deployment", namespace="default", name=f"lf-{w}", desired_replicas=3,
            scheduling_mode=T.SCHEDULING_MODE_DUPLICATE, max_clusters=int(rng.integers(1, 9)), cluster_selector=sel,
            affinity=T.Affinity(T.ClusterAffinity(T.ClusterSelector(terms), prefs or None))))
    for fwk in (F.Framework(F.default_enabled_plugins()),
                F.Framework(F.EnabledPlugins([F.ClusterAffinity], [F.ClusterAffinity], [F.MaxCluster], []))):
        snap, batch, res = run(ctx, clusters, units, fwk)
        st = np.bincount(res.status, minlength=6)
        assert st[pack.ST_OK] > 50 and st[pack.ST_NO_FEASIBLE] > 10, st
        assert_same(res, c_oracle(snap, batch, fwk), f"label-free C={C}")


def test_large_c_global_scratch(ctx):
    """C = 6000 does not fit the per-wave LDS budget: rows run from global scratch slabs."""
    clusters, units = synth.gen_fuzz(4242, W=200, C=6000)
    fwk = F.Framework(F.default_enabled_plugins())
    snap, batch, res = run(ctx, clusters, units, fwk)
    assert_same(res, c_oracle(snap, batch, fwk), "C=6000")


def test_tie_heavy_selection_rows(ctx):
    """Adversarial ties: the straddle path (pdqsort replay) against Go's full sort."""
    from test_pdq_select import full_first_k
    rng = np.random.default_rng(5)
    rows, ks, want = [], [], []
    for it in range(400):
        n = int(rng.integers(1, 1500))
        s = rng.integers(0, int(rng.integers(1, 6)), n).tolist()
        k = int(rng.integers(0, n + 1))
        rows.append(s)
        ks.append(k)
        want.append(full_first_k(s, k))
    got = ctx.select_rows(rows, ks)
    for (st, sel), w in zip(got, want):
        assert st == pack.ST_OK
        assert set(sel) == w


# ------------------------------------------------------- extreme values
def _extreme_batch(seed, C=200, W=120):
    """Fuzz batch pushed to the edges of the lean kernel's fast paths: capacities
    above 2^46 (Least/MostAllocated's exact int64 path), zero and negative
    quantities, and preferred-affinity weights of +-2^31 so totals span more
    than 2^32 (64-bit bisection; wide-key straddles go to the full kernel)."""
    rng = np.random.default_rng(seed)
    clusters, units = synth.gen_fuzz(seed, W=W, C=C)
    for c in clusters:
        r = rng.random()
        if r < 0.25:
            c.allocatable["memory"] = str(int(rng.integers(1 << 46, 1 << 52)))
            c.available["memory"] = str(int(rng.integers(0, 1 << 46)))
        elif r < 0.35:
            c.allocatable["cpu"] = "0"
            c.available["cpu"] = "0"
        elif r < 0.45:
            c.allocatable["cpu"] = f"{int(rng.integers(1, 1 << 40))}m"
            c.available["cpu"] = "1m"
    for su in units:
        ca = su.affinity.cluster_affinity if su.affinity is not None else None
        if ca is not None and ca.preferred:
            for p in ca.preferred:
                if rng.random() < 0.5:
                    p.weight = int(rng.choice([-(1 << 31), (1 << 31) - 1, -123456789, 987654321]))
    return clusters, units


@pytest.mark.parametrize("seed", range(8))
def test_extreme_values_gpu_equals_c_oracle(ctx, seed):
    clusters, units = _extreme_batch(500 + seed)
    fwk = F.Framework(F.default_enabled_plugins()) if seed % 2 == 0 else synth.fuzz_framework(seed)
    snap, batch, res = run(ctx, clusters, units, fwk)
    assert_same(res, c_oracle(snap, batch, fwk), f"extreme seed {seed}")


def test_ties_straddle_many_feasible(ctx):
    """C = 256 with identical clusters: every total ties, MaxCluster cuts inside the
    tie run on every unit (wave-parallel pdqsort replay over up to 256 positions)."""
    rng = np.random.default_rng(9)
    clusters = synth.gen_clusters(rng, 256, n_taints=0)
    for c in clusters:
        c.allocatable = {"cpu": "64", "memory": "256Gi"}
        c.available = {"cpu": str(int(rng.integers(30, 34))), "memory": "128Gi"}
        c.labels = {"key0": "val0"}
    units = synth.gen_units_c2(np.random.default_rng(10), 300)
    for su in units:
        su.affinity = None
        su.cluster_selector = None
        su.tolerations = None
        su.resource_request = T.Resource(int(rng.integers(0, 100)), int(rng.integers(0, 1 << 30)))
        su.max_clusters = int(rng.integers(1, 250))
    fwk = synth.profile_for("c2")
    snap, batch, res = run(ctx, clusters, units, fwk)
    assert (res.flags & 1).mean() > 0.5  # most rows straddle
    assert_same(res, c_oracle(snap, batch, fwk), "tie-heavy 256")


# ------------------------------------------------- clean-snapshot f64 path
def snapshot_is_clean(snap):
    """Host restatement of kad_api.hip res_clean: 1 <= alloc < 2^46, 0 <= used <= alloc (cpu, memory)."""
    h = pack.header_of(snap.blob, pack.SnapshotHeader)
    C = len(snap.names)
    a = [pack.array_of(snap.blob, h, i, np.int64, C) for i in (pack.S_ALLOC_CPU, pack.S_ALLOC_MEM)]
    u = [pack.array_of(snap.blob, h, i, np.int64, C) for i in (pack.S_USED_CPU, pack.S_USED_MEM)]
    return all(((x >= 1) & (x < (1 << 46)) & (y >= 0) & (y <= x)).all() for x, y in zip(a, u))


@pytest.mark.parametrize("seed", range(24))
def test_fuzz_clean_snapshot_gpu_equals_c_oracle(ctx, seed):
    """Snapshots whose cpu/memory satisfy SnapDev::clean at C = 16..256 (lean kernel
    instantiations NCH = 1..4 with the f64 resource columns), every fuzz profile
    (Least/Most/Balanced, taint and affinity scores), requests incl. zero and > capacity."""
    rng = np.random.default_rng(9000 + seed)
    C = [16, 64, 70, 130, 200, 256][seed % 6]
    clusters, units = synth.gen_fuzz(9000 + seed, W=90, C=C)
    for c in clusters:
        r = rng.random()
        if r < 0.3:  # large exact capacities near the 2^46 bound
            am = int(rng.integers(1 << 40, (1 << 46) - 1))
            c.allocatable["memory"] = str(am)
            c.available["memory"] = str(int(rng.integers(0, am + 1)))
        elif r < 0.5:  # fully used / fully free
            c.available["cpu"] = c.allocatable["cpu"] if rng.random() < 0.5 else "0"
    fwk = synth.fuzz_framework(seed) if seed % 3 else F.Framework(F.default_enabled_plugins())
    snap, batch, res = run(ctx, clusters, units, fwk)
    assert snapshot_is_clean(snap), "fixture must exercise the clean path"
    assert_same(res, c_oracle(snap, batch, fwk), f"clean fuzz seed {seed} C={C}")


@pytest.mark.parametrize("seed", range(16))
def test_fuzz_relaxed_snapshot_gpu_equals_c_oracle(ctx, seed):
    """Per-cluster clean (kad_api.hip res_clean class 1): some clusters with available < 0 (used >
    allocatable) and some with empty allocatable — the shapes aggregateResources reports
    (federatedcluster/util.go:178-214) — on the exact-f64 fast path of every kernel that has one: the lean
    kernel's clean instantiations (C <= 256), the wide kernel (C = 400..1000) and the row kernel's score
    columns (C = 1500, 3000: lean NCH = 0 + schedule_row_kernel). Requests zero and non-zero, every fuzz
    profile; the snapshot must stay on the fast path (snapshot_paths exact_f64)."""
    rng = np.random.default_rng(9500 + seed)
    C = [16, 64, 200, 256, 400, 700, 1000, 1500, 3000][seed % 9]
    W = 90 if C <= 1000 else 60
    clusters, units = synth.gen_fuzz(9500 + seed, W=W, C=C)
    synth.production_resources(clusters, rng, p_over=0.2, p_empty=0.1)
    cls = clusters[:2]  # at least one of each kind
    cls[0].allocatable, cls[0].available = {}, {}
    cls[1].available = dict(cls[1].available, cpu="-5", memory="-1Gi")
    for su in units[: W // 3]:  # zero requests: Fit returns early (fit.go:82-87), scores see request 0
        su.resource_request = T.Resource()
    fwk = synth.fuzz_framework(seed) if seed % 3 else F.Framework(F.default_enabled_plugins())
    snap, batch, res = run(ctx, clusters, units, fwk)
    paths = ctx.snapshot_paths()
    assert paths["resource_class"] == "relaxed", paths
    assert paths["exact_f64"] == (paths["fold"] and paths["fitfold"]), paths
    assert_same(res, c_oracle(snap, batch, fwk), f"relaxed fuzz seed {seed} C={C}")


@pytest.mark.parametrize("seed", range(16))
def test_zero_request_batches_gpu_equals_c_oracle(ctx, seed):
    """Batches in which no unit has a ResourceRequest (BatchDev::zero_req, what the live controller sends:
    schedulingtriggers.go:188-191) take the wide kernel's zero-request instantiation (the resource scores
    from the per-cluster column c_zs): C3's profile at 1 000 clusters (the LeastAllocated specialisation),
    the default set at 512 (the 8-chunk specialisation) and fuzz profiles at 400 / 700 (the generic one),
    on clean and relaxed snapshots (clusters over-committed or with empty allocatable); seeds 12-15 give one
    unit a request, so the same batch shape takes the exact-f64 instantiation."""
    rng = np.random.default_rng(9700 + seed)
    C = [1000, 512, 400, 700][seed % 4]
    clusters, units = synth.gen_fuzz(9700 + seed, W=120, C=C)
    if seed % 2:
        synth.production_resources(clusters, rng, p_over=0.2, p_empty=0.1)
        clusters[0].allocatable, clusters[0].available = {}, {}
    for su in units:
        su.resource_request = T.Resource()
    if seed >= 12:  # one unit with a request: the batch is not zero-request, every unit takes the exact path
        units[len(units) // 2].resource_request = T.Resource(250, 1 << 30)
    if C == 1000:
        fwk = synth.profile_for("c3")
    elif C == 512:
        fwk = F.Framework(F.default_enabled_plugins())
    else:
        fwk = synth.fuzz_framework(seed)
    snap, batch, res = run(ctx, clusters, units, fwk)
    assert_same(res, c_oracle(snap, batch, fwk), f"zero-request seed {seed} C={C} {ctx.snapshot_paths()}")

"""bench.py's host logic on CPU: the JSON line contract, the per-stage rooflines, the shard sweep and the
gathered-placement verification, with a stand-in for the GPU context whose results come from the C
restatement (oracle/kad_ref.c). No GPU here: this checks the bookkeeping, never a kernel; the GPU run of
bench.py (round end, and tests/test_gpu_bench_dist.py) uses the real libkad.so context."""
import argparse
import json

import numpy as np
import pytest

import bench
from kubeadmiral_amd import results, runtime, synth


class FakeContext:
    """runtime.Context's surface as bench.py uses it; schedule() runs the C oracle."""
    STAGES = runtime.Context.STAGES

    def __init__(self, device=0):
        self.device = device
        self.snap = self.batch = None
        self.res = None

    def upload_snapshot(self, snap):
        self.snap = snap

    def upload_snapshot_blob(self, blob, snap=None):
        import types
        self.snap = types.SimpleNamespace(blob=np.ascontiguousarray(blob, np.uint8))

    def upload_batch(self, batch):
        self.batch = batch

    def schedule(self, fwk):
        from oracle import ref
        self.res = ref.schedule(self.snap, self.batch, fwk, n_threads=4)
        self.fwk = fwk

    def sync(self):
        pass

    def download(self, out=None):
        if out is not None:  # the caller's buffers, as kad_results_download fills them
            W, n = len(self.res.status), len(self.res.cluster)
            for a, b in ((out.status, self.res.status), (out.count, self.res.count), (out.flags, self.res.flags),
                         (out.cluster, self.res.cluster), (out.replicas, self.res.replicas)):
                a[:len(b)] = b
            return type(self.res)(out.status[:W], out.count[:W], out.flags[:W], out.cluster[:n], out.replicas[:n],
                                  self.res.out_off)
        return self.res

    def path_counts(self):
        return {"units": self.batch.W, "full_kernel": 3, "row_kernel": 5, "planner_rows": 0}

    def snapshot_paths(self):
        return {"resource_class": "strict", "exact_f64": True, "wide": True, "fold": True, "fitfold": True}

    def set_timing(self, on):
        pass

    def stage_timing(self):
        return {"req_mask": 0.01, "prep": 0.02, "main": 0.2, "defer": 0.003, "planner": 0.0, "total": 0.25,
                "rows": 0.015}

    def close(self):
        pass


@pytest.fixture
def fake(monkeypatch):
    from kubeadmiral_amd import build
    build.build()
    monkeypatch.setattr(runtime, "Context", FakeContext)
    # pageable stand-ins for the page-locked result arrays (torch's pinned allocator needs a GPU)
    monkeypatch.setattr(results.BatchResult, "pinned", staticmethod(
        lambda W, n: results.BatchResult(np.zeros(max(1, W), np.int32), np.zeros(max(1, W), np.int32),
                                         np.zeros(max(1, W), np.uint32), np.zeros(max(1, n), np.int32),
                                         np.zeros(max(1, n), np.int64), np.zeros(1, np.int64))))
    monkeypatch.setitem(synth.SIZES, "c3", (3000, 1000))
    monkeypatch.setitem(synth.SIZES, "c2", (800, 256))


def _args(**kw):
    a = dict(gpus=1, steps=2, warmup=1, config="c3", units=None, cpu_seconds=0.05, no_cpu_baseline=False,
             no_extra=True, extras="c2", no_sweep=True, no_e2e=False, backend="nccl", share_gpu=False)
    a.update(kw)
    return argparse.Namespace(**a)


def test_line_contract_and_rooflines(fake):
    out = bench.bench_schedule(_args(), "c3", 0, 1, 0, None)
    json.dumps(out)  # serialisable
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline", "end_to_end"):
        assert k in out, k
    r = out["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in r, k
    # the dominant kernel is the stage with the longest (stand-in) time: the main kernel
    assert r["kernel"] == "schedule_wide_kernel" and r["time_ms"] == pytest.approx(0.2)
    assert r["frac"] == pytest.approx(r["achieved"] / r["peak"])
    assert set(r["kernels"]) == {"req_mask", "prep", "main", "rows", "defer"}
    assert out["cpu_baseline"]["kind"] == "port" and out["cpu_baseline"]["cores"] >= 1
    assert out["config"]["paths"]["row_kernel"] == 5
    e2e = out["end_to_end"]
    assert e2e["pipelined"]["chunks"] == 4 and e2e["sequential"]["units"] == 3000


def test_printed_lines_fit_the_driver_tail(fake, capsys, tmp_path, monkeypatch):
    """bench.py's stdout ends with the headline line, ≤ 3 KB and parseable, after one ≤ 1.5 KB line per extra
    config; the full result goes to a file. Built from a real bench result (c3 + embedded c2 + sweep) whose
    per-stage dicts are what made round 3's single 21 KB line unparseable."""
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    args = _args(no_extra=False, no_sweep=False)
    out = bench.bench_schedule(args, "c3", 0, 1, 0, None)
    out["extra"] = {"c2": bench.bench_schedule(args, "c2", 0, 1, 0, None),
                    "c4": bench.bench_schedule(args, "c2", 0, 1, 0, None)}
    out["shard_sweep"] = bench.shard_sweep(args, "c3", 0, out["ms_per_step"])
    assert len(json.dumps(out)) > 6000  # the uncompacted result would not fit
    bench.emit(out, "c3")
    lines = capsys.readouterr().out.strip().split("\n")
    assert len(lines) == 3
    head = lines[-1]
    assert len(head) <= bench.HEADLINE_MAX, len(head)
    h = json.loads(head)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline", "parity"):
        assert k in h, k
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in h["roofline"], k
    assert h["cpu_baseline"]["kind"] == "port" and h["cpu_baseline"]["cores"] >= 1
    assert h["parity"]["mismatches"] == 0 and h["parity"]["units_checked"] == 3000
    assert set(h["shard_sweep"]) == {"2", "4", "8"} and set(h["extra"]) == {"c2", "c4"}
    assert h["value"] == pytest.approx(out["value"], rel=1e-3)
    for s in lines[:-1]:
        assert len(s) <= bench.EXTRA_MAX, len(s)
        assert json.loads(s)["metric"] == h["metric"]
    full = json.loads((tmp_path / h["detail"]).read_text())
    assert "kernels" in full["roofline"]


def test_verify_rows_reports_mismatches(fake):
    """The bench's parity count catches a changed row (windows over the batch when no CPU pass is reused)."""
    out = bench.bench_schedule(_args(no_cpu_baseline=True, no_e2e=True), "c3", 0, 1, 0, None)
    assert out["parity"]["mismatches"] == 0 and out["parity"]["units_checked"] == 3000
    ctx = FakeContext()
    from kubeadmiral_amd import columns as CO
    from kubeadmiral_amd import pack
    clusters = bench.make_clusters("c3", 1000)
    snap = pack.Snapshot(clusters)
    fwk = synth.profile_for("c3")
    nb = CO.NativePacker(snap).pack(fwk, bench.make_columns("c3", 0, 3000, clusters))
    ctx.upload_snapshot(snap)
    ctx.upload_batch(nb)
    ctx.schedule(fwk)
    res = ctx.download()
    w = int(np.nonzero(res.count > 0)[0][7])
    res.cluster[nb.out_off[w]] += 1
    p = bench.verify_rows(snap, nb, fwk, res, max_units=1000)
    assert p["windows"] == 16 and p["units_checked"] == 16 * (1000 // 16)
    p = bench.verify_rows(snap, nb, fwk, res, max_units=10_000)
    assert p["mismatches"] == 1 and p["first_mismatch"] == w
    # a CPU pass that covered [0, 500) of a batch larger than max_units: the rest is sampled by 16 windows,
    # the last of which reaches the batch's tail
    from oracle import ref
    want = ref.schedule(snap, nb, fwk, 0, 500, 4)
    p = bench.verify_rows(snap, nb, fwk, res, want=want, n_want=500, max_units=1600)
    assert p["windows"] == 17 and p["units_checked"] > 500 + 16 * 90
    tail = nb.W - 1
    while res.count[tail] == 0:
        tail -= 1
    res.cluster[nb.out_off[tail]] += 1
    p2 = bench.verify_rows(snap, nb, fwk, res, want=want, n_want=500, max_units=nb.W * 16)
    assert p2["mismatches"] >= 1


def test_stale_pmc_is_not_used(fake, tmp_path, monkeypatch):
    """A PMC profile whose src_hash is not the code's is reported as stale, never mixed with live timing."""
    prof = tmp_path / "profiles"
    prof.mkdir()
    (prof / "pmc_c3.json").write_text(json.dumps({"units": 3000, "clusters": 1000, "src_hash": "0" * 16,
                                                  "kernels": {"schedule_wide_kernel<16>": {"SQ_INSTS_SALU": 1e9}}}))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    pmc, _, why = bench.load_pmc("c3", 3000, 1000)
    assert pmc is None and "stale" in why
    from kubeadmiral_amd.build import source_hash
    (prof / "pmc_c3.json").write_text(json.dumps({"units": 3000, "clusters": 1000, "src_hash": source_hash(),
                                                  "kernels": {"kad::schedule_wide_kernel<16>(kad::WideArgs)": {
                                                      "SQ_INSTS_SALU": 4.0e8, "SQ_INSTS_VALU": 1.0e8,
                                                      "hbm_bytes_corrected": 1e6}}}))
    pmc, _, why = bench.load_pmc("c3", 3000, 1000)
    assert pmc is not None and why is None
    r = bench.roofline_for("main", "schedule_wide_kernel", 1.0, 5e5, pmc, "x", None)
    assert r["bound"] == "salu_issue"
    assert r["frac"] == pytest.approx(4.0e8 / 1e-3 / bench.SALU_PEAK)
    assert r["traffic"] == 1e6 and r["hbm"]["measured_gbs"] == pytest.approx(1.0)


def test_shard_sweep_projection(fake):
    out = bench.shard_sweep(_args(), "c3", 0, t1_ms=1.0, ns=(2,))
    p = out["per_n"]["2"]
    assert len(p["shard_ms"]) == 2 and p["units_per_rank"] == 1500
    assert p["projected_efficiency"] == pytest.approx(1.0 / (2 * p["max_ms"]))


def _rank_worker(rank, world, port, outdir):
    import os

    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        runtime.Context = FakeContext
        synth.SIZES["c2"] = (900, 256)
        out = bench.bench_schedule(_args(gpus=world, backend="gloo", share_gpu=True, config="c2"), "c2", rank, world,
                                   0, dist)
        if rank == 0:
            with open(os.path.join(outdir, "line.json"), "w") as f:
                json.dump(out, f)
    finally:
        dist.destroy_process_group()


def test_two_ranks_gloo_line_and_gather_verification(tmp_path):
    """bench.py's N > 1 path on CPU (gloo, world size 2): snapshot broadcast, shard send, the timed steps, the
    placement all-gather and its check against single-rank runs of every shard, the max-over-ranks line."""
    import socket

    import torch.multiprocessing as mp
    from kubeadmiral_amd import build
    build.build()
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    mp.start_processes(_rank_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True, start_method="spawn")
    line = json.loads((tmp_path / "line.json").read_text())
    assert line["n_gpus"] == 2 and line["config"]["units_total"] == 900 and line["config"]["units_per_gpu"] == 450
    assert line["allgather"]["backend"] == "gloo"
    assert line["allgather"]["verified"] and "2 ranks" in line["allgather"]["verified"]


class FakeGroup:
    """runtime.GroupContext's surface as bench_group uses it: the members' shards of one batch, results
    from the C oracle over the whole batch."""

    def __init__(self, devices):
        self.devices = list(devices)
        self.ctx = FakeContext()
        self.timing = False

    def upload_snapshot(self, snap):
        self.ctx.upload_snapshot(snap)

    def upload_batch(self, batch):
        self.ctx.upload_batch(batch)

    def schedule(self, fwk):
        self.ctx.schedule(fwk)

    def sync(self):
        pass

    def download(self, out=None):
        return self.ctx.download()

    def path_counts(self):
        return self.ctx.path_counts()

    def member(self, i):
        return self.ctx

    def set_timing(self, on):
        self.timing = on

    def member_stage_timing(self, i):
        st = self.ctx.stage_timing()
        return {k: v * (1 + 0.1 * i) for k, v in st.items()}  # member i a little slower

    def ranges(self):
        W = self.ctx.batch.W
        n = len(self.devices)
        ulo = np.array([W * i // n for i in range(n + 1)], np.int64)
        return ulo, np.asarray(self.ctx.batch.out_off)[ulo]

    def close(self):
        pass


def test_group_mode_line(fake, monkeypatch):
    """bench_group (--gpus N, the default group mode): the contract fields, whole-batch parity, per-member
    stage times (the slowest member per stage), the group summary in the printed line."""
    monkeypatch.setattr(runtime, "GroupContext", FakeGroup)
    out = bench.bench_group(_args(gpus=4), "c3", [0, 1, 2, 3], None, 0)
    json.dumps(out)
    assert out["n_gpus"] == 4 and out["scaling"] == "strong" and out["value"] > 0
    assert out["config"]["units_total"] == 3000 and out["config"]["units_per_gpu"] == 750
    assert "kad_group" in out["config"]["parallelism"] and out["config"]["rccl_world_size"] is None
    assert out["parity"]["mismatches"] == 0 and out["parity"]["units_checked"] == 3000
    assert out["config"]["stage_ms"]["main"] == pytest.approx(0.2 * 1.3)  # member 3's
    assert len(out["group"]["member_total_ms"]) == 4
    line = bench.compact_line(out)
    assert line["group"]["devices"] == [0, 1, 2, 3] and line["group"]["mode"] == "group"
    assert out["cpu_baseline"] is None  # the CPU baseline is the N = 1 line's


def test_score_term_rows_counts_distinct_preferred_ids():
    """The rows stage's compulsory model reads each distinct preferred-term requirement row once: the parser
    walks every unit's score program (n_terms, then weight, n_expr, ids per term) and matches a direct count."""
    from kubeadmiral_amd import pack

    clusters, units, fwk = synth.make_config("c5", W=120, C=300)
    snap = pack.pack_snapshot(clusters)
    batch = pack.pack_batch(snap, fwk, units)
    h = pack.header_of(batch.blob, pack.BatchHeader)
    off = pack.array_of(batch.blob, h, pack.B_SPROG_OFF, np.int32, batch.W + 1)
    prog = pack.array_of(batch.blob, h, pack.B_SPROG, np.int32, int(off[-1]))
    want = set()
    for w in range(batch.W):
        p = prog[off[w]:off[w + 1]].tolist()
        if not p:
            continue
        i = 1
        for _ in range(p[0]):
            want.update(p[i + 2:i + 2 + p[i + 1]])
            i += 2 + p[i + 1]
        assert i == len(p), "score program layout"
    assert want and bench.score_term_rows(batch) == len(want)
    nch = (300 + 63) // 64
    b = bench.stage_bytes_model("rows", batch.W, 300, nch, batch, snap, 0, {"row_kernel": batch.W}, 0, 0)
    assert b == (64.0 + 8 * nch) * batch.W + 72.0 * 300 + 8.0 * nch * len(want)

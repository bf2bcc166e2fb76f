#!/usr/bin/env python3
"""Benchmark: scheduling decisions/s (workload × cluster evaluations per second).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3] [--units TOTAL]

Default: BASELINE.json's north_star configuration C3 — 1M SchedulingUnits × 1k
FederatedClusters (C2 generator, seed 0xC3) — on one MI355X, with the C2 line
(100k × 256) measured in the same run and embedded under ``extra``.

One step = one pass of the hot path (filter → score → select [→ replicas])
over the resident batch against the resident cluster snapshot (kad_schedule).
With ``--gpus N`` (N > 1) and no torch.distributed environment, bench.py
starts ``torch.distributed.run`` with N ranks as a child process before any
GPU call. The TOTAL batch is fixed and sharded over the ranks (strong
scaling, "1M workloads … sharded over 8×MI355X"): rank 0 generates the units
and packs every shard with the native packer (one packer, N schedulers),
RCCL-broadcasts the cluster snapshot and sends each rank its batch blob over
xGMI; every rank checks the snapshot fingerprint against its batch, times K
passes between barriers, and the step time is the max over ranks. After the
timed region the placements are all-gathered over RCCL (fixed per-rank slot
arrays) and timed as their own field.

Prints ONE JSON line (rank 0) with the driver's contract fields plus
``roofline`` (dominant kernel: compulsory bytes per launch ÷ its HIP-event
time vs 8 TB/s; the PMC-measured HBM bytes and the SALU/VALU issue fractions
from profiles/pmc_<cfg>.json when it matches the workload; SURVEY §8(d)'s
canonical algorithmic-byte model kept only for transparency),
``end_to_end`` (pack + H2D + schedule + D2H) and ``cpu_baseline`` (the C
restatement of the reference, oracle/kad_ref.c, on a bounded sample).
"""

from __future__ import annotations

import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0
CLOCK_HZ = 2.4e9
N_CU = 256
# issue capacity per second of the whole chip: one wave64 VALU instruction per SIMD every 2 cycles
# (SIMD-32), one SALU instruction per CU per cycle (MI355X_MICROARCH.md, Execution model)
VALU_PEAK = N_CU * 4 * CLOCK_HZ / 2
SALU_PEAK = N_CU * CLOCK_HZ
WORKLOAD_DESC = {
    "c1": "1k Deployment SchedulingUnits x 16 FederatedClusters, default plugin set, Divide",
    "c2": "100k SchedulingUnits x 256 FederatedClusters: Fit+Taint+Affinity(+APIResources) filters, "
          "LeastAllocated score, MaxCluster select, Duplicate",
    "c3": "1M SchedulingUnits x 1k FederatedClusters (c2 generator), sharded over the GPUs",
    "c3r": "c3 with production-shaped snapshots: ~150 Kind-sorted discovery API resources per cluster "
           "(clusterstatus.go:221-266) and units over 8 workload kinds",
    "c3p": "c3r with the live controller's inputs: ResourceRequest never set (schedulingtriggers.go:188-191) and "
           "1.5 % of clusters with available < 0, 0.5 % with empty allocatable (federatedcluster/util.go:178-214)",
    "c4": "1M Divide SchedulingUnits x 512 clusters: weights, min/max replicas, capacity caps",
    "c5": "100k SchedulingUnits x 10k clusters: dense label affinity, many taints, API-resource gaps",
    "t1": "scheduling-trigger hashes: 1k federated Deployments x 16 joined clusters",
    "t2": "scheduling-trigger hashes: 100k federated Deployments x 256 joined clusters (~1.6 MB cluster part)",
}
# Issue bound of one FNV-1 step per lane: the inner loop is one v_mul_lo_u32 (quarter rate: 16 SIMD cycles per
# wave64 instruction) + one v_bitop3_b32 per byte; the bound is the multiply, 4 steps/cycle/SIMD × 4 SIMDs × 256
# CUs × 2.4 GHz.
FNV_STEP_PEAK = 4.0 * 4 * 256 * 2.4e9


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def relaunch(args) -> int:
    """--gpus N > 1 without a torch.distributed environment: run N ranks under torch.distributed.run as a
    child process (nothing in this process has touched the GPU) and return its exit code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.call(cmd, env=env)


# ------------------------------------------------------------------------ workloads
def make_clusters(cfg: str, C: int):
    from kubeadmiral_amd import synth

    rng = np.random.default_rng(synth.SEEDS[cfg])
    if cfg == "c5":
        return synth.gen_clusters(rng, C, n_keys=64, n_vals=16, n_int_keys=4, n_taints=256, taints_per=(4, 16),
                                  p_gvk=0.9, gvks=synth.GVKS)
    cl = synth.gen_clusters(rng, C)
    if cfg in ("c3r", "c3p"):  # C3's clusters with discovery-shaped API-resource lists (their own random stream)
        for c, api in zip(cl, synth.discovery_api_resources(np.random.default_rng([synth.SEEDS[cfg], 0xA91]), C)):
            c.api_resource_types = api
    if cfg == "c3p":  # over-committed and fully cordoned clusters (their own random stream)
        synth.production_resources(cl, np.random.default_rng([synth.SEEDS[cfg], 0x9E5]))
    return cl


def make_columns(cfg: str, lo: int, hi: int, clusters):
    """Columns (kad_su_columns) of units [lo, hi) of the config's batch (seeded per shard)."""
    from kubeadmiral_amd import columns as CO
    from kubeadmiral_amd import synth

    rng = np.random.default_rng([synth.SEEDS[cfg], lo])
    if cfg in ("c2", "c3"):
        return synth.gen_units_c2_columns(rng, hi - lo, prefix=f"su{lo}")
    if cfg == "c3r":  # C3's units (same stream) over 8 workload kinds
        return synth.gen_units_c2_columns(rng, hi - lo, prefix=f"su{lo}", workloads=synth.C3R_WORKLOADS)
    if cfg == "c3p":  # c3r's units as the live controller builds them: no ResourceRequest
        cols = synth.gen_units_c2_columns(rng, hi - lo, prefix=f"su{lo}", workloads=synth.C3R_WORKLOADS)
        cols["req_cpu"][:] = 0
        cols["req_mem"][:] = 0
        return cols
    if cfg == "c4":  # vectorised generators: 1M C4 units in seconds (the object generator takes minutes)
        return synth.gen_units_c4_columns(rng, hi - lo, [c.name for c in clusters], prefix=f"c4-{lo}")
    if cfg == "c5":
        return synth.gen_units_c5_columns(rng, hi - lo, [c.name for c in clusters], prefix=f"c5-{lo}")
    units = synth.gen_units_c1(rng, hi - lo, clusters)
    for i, su in enumerate(units):
        su.name = f"{su.name}-{lo + i}"
    return CO.from_units(units)


def canonical_bytes(n_reqs, n_tols, count, C, TW, divide_counts):
    """SURVEY.md §8(d) model: W·C·B_pair + Σ_w B_w (+ Σ_w K_w·B_plan for Divide rows). Transparency only:
    it charges every pair its cluster operands as if streamed from HBM, which the kernels serve from LDS."""
    r = n_reqs.astype(np.float64)
    b_pair = 32 + 16 + 16 * (TW - 1) + 4 + 4 + 4 * r
    pair = float(np.sum(b_pair) * C)
    per_w = float(np.sum(128 + 16 * r + 8 * n_tols + 12 * count))
    plan = float(np.sum(divide_counts) * 48)
    return pair + per_w, plan


def load_pmc(cfg: str, W: int, C: int):
    """profiles/pmc_<cfg>.json (scripts/profile.sh → scripts/pmc_summary.py) when it was collected on this
    workload AND on this code (its ``src_hash`` = build.source_hash() of libkad.so's sources): counters of
    an older kernel are never reported against today's timing. Returns (pmc | None, path, why-not)."""
    from kubeadmiral_amd.build import source_hash

    path = os.path.join(ROOT, "profiles", f"pmc_{cfg}.json")
    if not os.path.exists(path):
        return None, path, "no PMC profile"
    with open(path) as f:
        pmc = json.load(f)
    if pmc.get("units") != W or pmc.get("clusters") != C:
        return None, path, f"PMC profile is for {pmc.get('units')} x {pmc.get('clusters')}"
    if pmc.get("src_hash") != source_hash():
        return None, path, f"PMC profile is stale (src_hash {pmc.get('src_hash')} != {source_hash()})"
    return pmc, path, None


# stage (kad_stage_timing) → the kernels it launches (rocprofv3 names contain these)
STAGE_KERNELS = {"req_mask": ("req_row_kernel", "req_mask_kernel"), "prep": ("prep_kernel",),
                 "main": ("schedule_wide_kernel", "schedule_lean_kernel"), "rows": ("schedule_row_kernel",),
                 "defer": ("schedule_kernel<",),
                 "planner": ("plan_hdr_kernel", "plan_pair_kernel", "plan_kernel")}


def pmc_kernel_sum(pmc, stage: str, main_name: str = None):
    """Per-launch counters of the stage's kernels summed (None without a profile)."""
    if pmc is None:
        return None
    names = (main_name,) if main_name else STAGE_KERNELS[stage]
    acc = {}
    for k, d in pmc.get("kernels", {}).items():
        if any(n in k for n in names):
            for c, v in d.items():
                if isinstance(v, (int, float)):
                    acc[c] = acc.get(c, 0.0) + v
    return acc or None


def roofline_for(stage: str, kernel: str, t_ms: float, compulsory: float, pmc, pmc_path, why_not):
    """The roofline of one kernel: HBM (compulsory bytes / live time; PMC-measured traffic beside it),
    VALU issue and SALU issue (PMC instruction counts / live time vs the chip's issue rates). ``bound`` is
    the largest fraction — the resource that binds — and ``achieved`` / ``peak`` / ``frac`` are its."""
    t = max(t_ms, 1e-9) * 1e-3
    d = pmc_kernel_sum(pmc, stage, None if stage != "main" else kernel)
    traffic = d.get("hbm_bytes_corrected") if d else None
    hbm_gbs = compulsory / t / 1e9
    cand = {"hbm": (traffic / t / 1e9 if traffic else hbm_gbs, HBM_PEAK_GBS, "GB/s")}
    issue = None
    if d and d.get("SQ_INSTS_VALU") is not None:
        cand["valu_issue"] = (d["SQ_INSTS_VALU"] / t, VALU_PEAK, "wave-instr/s")
        cand["salu_issue"] = (d["SQ_INSTS_SALU"] / t, SALU_PEAK, "wave-instr/s")
        issue = {"valu_insts": d["SQ_INSTS_VALU"], "salu_insts": d["SQ_INSTS_SALU"],
                 "valu_frac": d["SQ_INSTS_VALU"] / t / VALU_PEAK, "salu_frac": d["SQ_INSTS_SALU"] / t / SALU_PEAK,
                 "lds_insts": d.get("SQ_INSTS_LDS"),
                 "wait_frac": (d["SQ_WAIT_ANY"] / d["SQ_WAVE_CYCLES"]) if d.get("SQ_WAVE_CYCLES") else None,
                 "peaks": "VALU 1.23e12 wave-instr/s (256 CU x 4 SIMD x 2.4 GHz / 2), SALU 6.1e11 (256 CU x 2.4 GHz)"}
    bound = max(cand, key=lambda b: cand[b][0] / cand[b][1])
    ach, peak, unit = cand[bound]
    return {"bound": bound, "achieved": ach, "peak": peak, "unit": unit, "frac": ach / peak, "traffic": traffic,
            "kernel": kernel, "time_ms": t_ms, "compulsory_bytes_per_launch": compulsory,
            "hbm": {"compulsory_gbs": hbm_gbs, "compulsory_frac": hbm_gbs / HBM_PEAK_GBS,
                    "measured_gbs": traffic / t / 1e9 if traffic else None,
                    "measured_frac": traffic / t / 1e9 / HBM_PEAK_GBS if traffic else None},
            "issue": issue,
            "pmc": os.path.relpath(pmc_path, ROOT) if pmc is not None else why_not}


def host_cpus():
    """(worker threads for the CPU baseline, os.cpu_count(), the cgroup's CPU limit or None): one thread per CPU
    this process may both run on (len(sched_getaffinity)) and be given time on (ceil of the cgroup quota,
    /sys/fs/cgroup/cpu.max) — on the GPU box the affinity mask names the machine's 256 threads while the
    cgroup allows 16, and 256 threads under a 16-CPU quota are throttled, not faster. All three are reported."""
    try:
        usable = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        usable = os.cpu_count() or 1
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
            if q != "max":
                quota = int(q) / int(period)
    except (OSError, ValueError):
        pass
    threads = usable if quota is None else max(1, min(usable, math.ceil(quota)))
    return threads, os.cpu_count(), quota


def cpu_baseline(snap, batch, fwk, C, target_s):
    """The C restatement timed on the host (kind "port") over the first n units, n sized for ~target_s of
    work, one worker thread per CPU the process may use (host_cpus). Returns (line, oracle result of units
    [0, n), n) — the result doubles as the parity check of the GPU rows (verify_rows)."""
    from oracle import ref

    threads, n_machine, quota = host_cpus()
    n = min(batch.W, 2000)
    t0 = time.perf_counter()
    want = ref.schedule(snap, batch, fwk, 0, n, threads)
    dt = time.perf_counter() - t0
    n2 = int(min(batch.W, max(n, n * target_s / max(dt, 1e-6))))
    if n2 > n:
        t0 = time.perf_counter()
        want = ref.schedule(snap, batch, fwk, 0, n2, threads)
        dt = time.perf_counter() - t0
        n = n2
    reps = max(1, int(target_s / max(dt, 1e-6)))
    if reps > 1:
        t0 = time.perf_counter()
        for _ in range(reps):
            ref.schedule(snap, batch, fwk, 0, n, threads)
        dt = time.perf_counter() - t0
    line = {"value": reps * n * C / dt, "unit": "decisions/s", "cores": threads, "kind": "port",
            "cpu_count": n_machine, "cgroup_cpu_limit": quota,
            "sample": f"{reps} pass(es) over units [0, {n}) of {batch.W} x {C} clusters, oracle/kad_ref.c "
                      f"(C restatement of the Go reference, one unit per worker thread, {threads} threads = the "
                      f"CPUs this process may use within its cgroup limit {quota}; machine {n_machine}), "
                      f"{dt:.2f}s wall"}
    return line, want, n


def verify_rows(snap, batch, fwk, res, want=None, n_want=0, max_units=200_000):
    """Parity of the timed run's rows against the C oracle (oracle/kad_ref.c), outside every timed region:
    units [0, n_want) from the CPU baseline's own oracle pass when there was one (and the rest of a batch of
    at most max_units units by a pass of its own), else 16 equal windows spread over the batch holding
    ~max_units units. Rows compare status, count, (cluster, replicas) pairs and result flags."""
    from oracle import ref

    W = batch.W
    threads = min(16, os.cpu_count() or 1)
    if want is not None and n_want > 0:
        wins = [(0, n_want, want)]
        if n_want < W <= max_units:  # a time-bounded CPU pass stopped short: the remaining units too
            wins.append((n_want, W, None))
        elif n_want < W:  # ... of a large batch: 16 windows spread over the rest, so the tail is sampled too
            rest = W - n_want
            span = max(1, min(rest // 16, max_units // 16))
            wins += [(n_want + rest * i // 16, min(W, n_want + rest * i // 16 + span), None) for i in range(16)]
    elif W <= max_units:
        wins = [(0, W, None)]
    else:
        span = max_units // 16
        wins = [(W * i // 16, W * i // 16 + span, None) for i in range(16)]
    bad = 0
    first = None
    for lo, hi, have in wins:
        w = have if have is not None else ref.schedule(snap, batch, fwk, lo, hi, threads)
        sl = slice(lo, hi)
        eq = np.ones(hi - lo, bool)
        eq &= (res.status[sl] == w.status[sl]) & (res.count[sl] == w.count[sl]) & (res.flags[sl] == w.flags[sl])
        # slot contents within each row's written range
        cnt = w.count[sl].astype(np.int64)
        starts = np.asarray(batch.out_off[lo:hi], np.int64)
        idx = np.repeat(starts, cnt) + (np.arange(int(cnt.sum())) - np.repeat(np.cumsum(cnt) - cnt, cnt))
        rows = np.repeat(np.arange(hi - lo), cnt)
        d = (res.cluster[idx] != w.cluster[idx]) | (res.replicas[idx] != w.replicas[idx])
        eq[rows[d]] = False
        nb = int((~eq).sum())
        if nb and first is None:
            first = lo + int(np.nonzero(~eq)[0][0])
        bad += nb
    checked = sum(hi - lo for lo, hi, _ in wins)
    return {"units_checked": checked, "of": W, "mismatches": bad, "first_mismatch": first,
            "oracle": "oracle/kad_ref.c", "windows": len(wins)}


# ------------------------------------------------------------------------ scheduling bench
def bench_schedule(args, cfg, rank, world, local, dist, W_total=None, cpu_seconds=None):
    import torch  # noqa: F401  (HIP runtime initialised by torch before libkad.so)

    from kubeadmiral_amd import columns as CO
    from kubeadmiral_amd import pack, shard, synth
    from kubeadmiral_amd.runtime import Context

    W0, C = synth.SIZES[cfg]
    W_total = W_total if W_total is not None else (args.units if args.units is not None else W0)
    fwk = synth.profile_for(cfg)
    cpu_seconds = args.cpu_seconds if cpu_seconds is None else cpu_seconds
    lo, hi = shard.shard_range(W_total, rank, world)
    dev = f"cuda:{local}"
    # RCCL moves device tensors over xGMI; the gloo rehearsal mode (--backend gloo) moves host tensors
    cdev = dev if args.backend == "nccl" else "cpu"
    t_gen = t_pack = 0.0

    # rank 0: cluster list, snapshot, every shard's batch blob (one packer, N schedulers)
    snap = None
    blobs = {}
    stats0 = None
    if rank == 0:
        t0 = time.perf_counter()
        clusters = make_clusters(cfg, C)
        snap = pack.Snapshot(clusters)
        packer = CO.NativePacker(snap)
        for r in range(world):
            rlo, rhi = shard.shard_range(W_total, r, world)
            tg = time.perf_counter()
            cols = make_columns(cfg, rlo, rhi, clusters)
            tp = time.perf_counter()
            nb = packer.pack(fwk, cols)
            t_pack += time.perf_counter() - tp
            t_gen += tp - tg
            blobs[r] = nb
            if r == 0:
                stats0 = (cols, nb)
        log(f"[rank 0] {cfg}: {W_total} units x {C} clusters over {world} rank(s): generated in {t_gen:.1f}s, "
            f"packed in {t_pack:.2f}s ({W_total / max(t_pack, 1e-9):.0f} units/s native), "
            f"batch {sum(b.blob.nbytes for b in blobs.values()) / 1e6:.1f} MB, snapshot {snap.blob.nbytes / 1e3:.1f} kB "
            f"({time.perf_counter() - t0:.1f}s)")

    ctx = Context(local)
    if dist is not None:
        # snapshot: RCCL broadcast over xGMI, uploaded from device memory
        buf = shard.broadcast_blob(snap.blob if rank == 0 else None, dist, device=cdev)
        if cdev != "cpu":
            torch.cuda.synchronize()
        # batch blob: rank 0 → rank r (point-to-point over xGMI)
        if rank == 0:
            batch = blobs[0]
            for r in range(1, world):
                b = torch.from_numpy(blobs[r].blob).to(cdev)
                dist.send(torch.tensor([b.numel()], dtype=torch.int64, device=cdev), dst=r)
                dist.send(b, dst=r)
        else:
            n = torch.zeros(1, dtype=torch.int64, device=cdev)
            dist.recv(n, src=0)
            b = torch.empty(int(n.item()), dtype=torch.uint8, device=cdev)
            dist.recv(b, src=0)
            batch = CO.NativeBatch.from_blob(b.cpu().numpy(), fwk)
        # the received snapshot must be the one this rank's batch was packed against
        shard.check_snapshot(buf[:4096].cpu().numpy(), int(pack.header_of(batch.blob, pack.BatchHeader)
                                                             .snapshot_fingerprint))
        if cdev != "cpu":
            ctx.upload_snapshot_device(buf.data_ptr(), buf.numel(), snap)
        else:
            ctx.upload_snapshot_blob(buf.numpy())
        del buf
    else:
        batch = blobs[0]
        ctx.upload_snapshot(snap)
    ctx.upload_batch(batch)

    for _ in range(args.warmup):
        ctx.schedule(fwk)
        ctx.sync()
    if dist is not None:
        dist.barrier()
    ctx.sync()
    # timed region: K full passes back to back on the context's stream, timing events off
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ctx.schedule(fwk)
    ctx.sync()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    res = ctx.download()
    paths = ctx.path_counts()
    sp = ctx.snapshot_paths()  # the main kernel and the snapshot's resource class (per-cluster clean)
    paths["main"] = "wide" if sp["wide"] else "lean"
    paths["resource_class"] = sp["resource_class"]
    # per-stage device time (HIP events on the context's stream), outside the timed region
    ctx.set_timing(True)
    st = []
    for _ in range(max(3, min(args.steps, 10))):
        ctx.schedule(fwk)
        ctx.sync()
        st.append(ctx.stage_timing())
    ctx.set_timing(False)
    stage = {k: float(np.mean([s[k] for s in st])) for k in ctx.STAGES}
    ms = elapsed / max(1, args.steps) * 1e3

    # placements all-gathered over RCCL (fixed per-rank slot arrays), timed on its own
    allgather = None
    if dist is not None:
        allgather = gather_placements(ctx, batch, res, dist, world, cdev, blobs if rank == 0 else None, fwk)

    if dist is not None:
        t = torch.tensor([ms] + [stage[k] for k in ctx.STAGES], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ms = float(t[0])
        stage = {k: float(v) for k, v in zip(ctx.STAGES, t[1:].tolist())}

    out = None
    if rank == 0:
        out = schedule_line(args, cfg, world, W_total, C, batch, snap, fwk, res, stage, ms, stats0, paths)
        out["allgather"] = allgather
        if world == 1 and not args.no_e2e:
            out["end_to_end"] = end_to_end(ctx, snap, fwk, stats0[0], res, C, packer_for=snap)
        want, n_want = None, 0
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"], want, n_want = cpu_baseline(snap, batch, fwk, C, cpu_seconds)
        # rank 0's rows (its shard) against the C oracle; the other ranks' rows are checked against
        # single-rank runs of their shards in gather_placements
        out["parity"] = verify_rows(snap, batch, fwk, res, want, n_want)
        if out["parity"]["mismatches"]:
            log(f"[rank 0] {cfg}: PARITY FAILURE {out['parity']}")
    ctx.close()
    return out


def bench_group(args, cfg, devices, dist, rank):
    """--gpus N in one process (the default --mode group): the product's multi-GPU path, kad_group_* behind the
    C ABI (include/kad_sched.h) — the path a Go controller links, one scheduler process calling Schedule from
    its workers (worker.go:132-134, scheduler.go:507). One snapshot upload copied device to device, the whole
    batch split into N contiguous unit ranges, the members' pipelines issued concurrently from a host pool.
    The timed step is kad_group_schedule over all N devices (K back to back) between two kad_group_sync. Under
    torch.distributed.run (the driver's SCALE launch) rank 0 drives all N devices and the other ranks only
    join the barriers around the timed region; the max over ranks is rank 0's time."""
    import torch  # noqa: F401  (HIP runtime initialised by torch before libkad.so)

    from kubeadmiral_amd import columns as CO
    from kubeadmiral_amd import pack, synth
    from kubeadmiral_amd.runtime import GroupContext

    N = len(devices)
    W0, C = synth.SIZES[cfg]
    W_total = args.units if args.units is not None else W0
    fwk = synth.profile_for(cfg)
    g = snap = batch = stats0 = None
    if rank == 0:
        t0 = time.perf_counter()
        clusters = make_clusters(cfg, C)
        snap = pack.Snapshot(clusters)
        cols = make_columns(cfg, 0, W_total, clusters)
        batch = CO.NativePacker(snap).pack(fwk, cols)
        stats0 = (cols, batch)
        log(f"[group] {cfg}: {W_total} units x {C} clusters over devices {devices}: generated + packed in "
            f"{time.perf_counter() - t0:.1f}s, batch {batch.blob.nbytes / 1e6:.1f} MB")
        g = GroupContext(devices)
        t0 = time.perf_counter()
        g.upload_snapshot(snap)
        g.upload_batch(batch)
        upload_ms = (time.perf_counter() - t0) * 1e3
        for _ in range(args.warmup):
            g.schedule(fwk)
            g.sync()
    if dist is not None:
        dist.barrier()
    if g is not None:
        g.sync()
    t0 = time.perf_counter()
    if g is not None:
        for _ in range(args.steps):
            g.schedule(fwk)
        g.sync()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ms = elapsed / max(1, args.steps) * 1e3
    if dist is not None:  # max over ranks (rank 0 did the work; the others waited at the barriers)
        import torch

        t = torch.tensor([ms if rank == 0 else 0.0], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ms = float(t[0])
    if rank != 0:
        return None
    t1 = time.perf_counter()
    res = g.download()
    d2h_ms = (time.perf_counter() - t1) * 1e3
    paths = g.path_counts()
    sp = g.member(0).snapshot_paths()
    paths["main"] = "wide" if sp["wide"] else "lean"
    paths["resource_class"] = sp["resource_class"]
    # per-member stage times (timing on, outside the timed region): the slowest member per stage
    g.set_timing(True)
    per = []
    for _ in range(max(3, min(args.steps, 10))):
        g.schedule(fwk)
        g.sync()
        per.append([g.member_stage_timing(i) for i in range(N)])
    g.set_timing(False)
    from kubeadmiral_amd.runtime import Context

    stage = {k: float(np.mean([max(m[k] for m in run) for run in per])) for k in Context.STAGES}
    member_main = [float(np.mean([run[i]["total"] for run in per])) for i in range(N)]
    ulo, _ = g.ranges()
    out = schedule_line(args, cfg, N, W_total, C, batch, snap, fwk, res, stage, ms, stats0, paths)
    out["config"]["parallelism"] = f"dp{N} (kad_group: one process, {N} devices)"
    out["config"]["rccl_world_size"] = None
    out["config"]["units_per_gpu"] = int(np.max(np.diff(ulo)))
    out["group"] = {"devices": list(devices), "member_total_ms": member_main, "upload_ms": upload_ms,
                    "download_ms": d2h_ms, "mode": "group"}
    out["parity"] = verify_rows(snap, batch, fwk, res)
    if out["parity"]["mismatches"]:
        log(f"[group] {cfg}: PARITY FAILURE {out['parity']}")
    g.close()
    return out


def score_term_rows(batch) -> int:
    """Distinct requirement ids in the batch's score programs (ClusterAffinity preferred terms): the rows the
    row kernel's (term, chunk) word pass reads. Program layout: n_terms, then per term weight, n_expr, ids."""
    from kubeadmiral_amd import pack

    h = pack.header_of(batch.blob, pack.BatchHeader)
    W = int(h.n_units)
    off = pack.array_of(batch.blob, h, pack.B_SPROG_OFF, np.int32, W + 1)
    prog = pack.array_of(batch.blob, h, pack.B_SPROG, np.int32, int(off[W]))
    ids = set()
    for w in range(W):
        i, e = int(off[w]), int(off[w + 1])
        if i >= e:
            continue
        nt, pc = int(prog[i]), i + 1
        for _ in range(nt):
            ne = int(prog[pc + 1])
            ids.update(prog[pc + 2:pc + 2 + ne].tolist())
            pc += 2 + ne
    return len(ids)


def stage_bytes_model(stage, W, C, nch, batch, snap, out_bytes, paths, n_distinct_reqs, divide_slots):
    """Compulsory HBM bytes of one launch of each stage's kernels (inputs read once, outputs written once):
    * req_mask: every distinct requirement's row words written + the label columns read once;
    * prep: the batch blob read once + UnitRec (64 B) and static filter words (8 B x chunks) per unit written;
    * main: UnitRec + static words per unit, 56 B per cached cluster, 12 B per unit + 12 B per placement out;
    * rows: UnitRec + static words per unit the kernel takes, its cluster columns (72 B: f64 resources, f32
      inverses, 32-B PreferNoSchedule words), and its units' share of the distinct preferred-term requirement
      rows (8 B x chunks each; the share assumes the routed units hold a proportional part of them);
    * defer: UnitRec + static words per unit the kernel takes, its cached cluster columns;
    * planner: SURVEY §8(d) B_plan = 48 B per (Divide unit, selected cluster)."""
    K = snap.K if hasattr(snap, "K") else 0
    if stage == "req_mask":
        return 8.0 * nch * max(0, n_distinct_reqs) + 4.0 * K * C
    if stage == "prep":
        return float(batch.blob.nbytes) + (64.0 + 8 * nch) * W
    if stage == "main":
        return (64.0 + 8 * nch) * W + 56.0 * C + out_bytes
    if stage == "rows":
        R = paths["row_kernel"]
        terms = 8.0 * nch * score_term_rows(batch) * (R / max(1, W)) if R else 0.0
        return (64.0 + 8 * nch) * R + 72.0 * C + terms
    if stage == "defer":
        return (64.0 + 8 * nch) * paths["full_kernel"] + 56.0 * C
    if stage == "planner":
        return 48.0 * divide_slots
    return 0.0


def schedule_line(args, cfg, world, W_total, C, batch, snap, fwk, res, stage, ms, stats0, paths):
    """The bench line of one scheduling config (rank 0): value, stage times, the per-stage rooflines and
    the dominant kernel's roofline (the stage with the longest live HIP-event time)."""
    from kubeadmiral_amd import pack

    W0r = batch.W
    nch = (C + 63) // 64
    count = res.count.astype(np.int64)
    out_bytes = 12 * W0r + 12 * float(count.sum())
    cols0, nb0 = stats0
    divide = (nb0.flags & pack.W_DUPLICATE) == 0 if fwk.replicas_plugin >= 0 else np.zeros(W0r, bool)
    divide_slots = float(count[divide].sum())
    kbytes, pbytes = canonical_bytes(nb0.n_reqs, nb0.n_tols, count, C, snap.TW, count[divide])
    pmc, pmc_path, why_not = load_pmc(cfg, W0r, C)
    # the bench snapshots are clean (allocatable >= used >= 0): wide kernel for 5..16 chunks, else lean
    main_kernel = "schedule_wide_kernel" if 4 < nch <= 16 else "schedule_lean_kernel"
    kernels = {}
    for st in ("req_mask", "prep", "main", "rows", "defer", "planner"):
        t = stage.get(st, 0.0)
        if t < 0.002:  # not launched (events back to back)
            continue
        kname = main_kernel if st == "main" else " + ".join(STAGE_KERNELS[st])
        cb = stage_bytes_model(st, W0r, C, nch, batch, snap, out_bytes, paths, nb0.n_distinct_reqs, divide_slots)
        kernels[st] = roofline_for(st, kname, t, cb, pmc, pmc_path, why_not)
    dom = max(kernels, key=lambda k: kernels[k]["time_ms"])
    roof = dict(kernels[dom])
    fss_ms = sum(stage.get(k, 0.0) for k in ("req_mask", "prep", "main", "rows", "defer"))
    stage_b = batch.blob.nbytes + snap.blob.nbytes + out_bytes
    roof["stage"] = {"time_ms": fss_ms, "compulsory_bytes": stage_b,
                     "frac": stage_b / (fss_ms * 1e-3) / 1e9 / HBM_PEAK_GBS}
    roof["algorithmic_bytes_per_launch"] = kbytes
    roof["algorithmic_model_frac"] = kbytes / (fss_ms * 1e-3) / 1e9 / HBM_PEAK_GBS
    roof["algorithmic_note"] = ("SURVEY §8(d) per-pair model (charges every pair its cluster operands as if "
                                "streamed from HBM; the kernels serve them from LDS): transparency only")
    roof["kernels"] = {k: {f: v[f] for f in ("kernel", "time_ms", "bound", "frac", "traffic")} |
                       {"salu_frac": (v["issue"] or {}).get("salu_frac"), "valu_frac": (v["issue"] or {}).get("valu_frac"),
                        "hbm_measured_frac": v["hbm"]["measured_frac"], "hbm_compulsory_frac": v["hbm"]["compulsory_frac"]}
                       for k, v in kernels.items()}
    return {
        "metric": "scheduling decisions/sec (workload x cluster evals/s)",
        "value": W_total * C / (ms * 1e-3),
        "unit": "decisions/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "int64",
        "data": "synthetic (seeded SURVEY.md §8(d) generator; no cluster/dataset available)",
        "config": {"workload": f"{cfg}: {WORKLOAD_DESC[cfg]}", "units_total": W_total, "units_per_gpu": W0r,
                   "clusters": C, "parallelism": f"dp{world}", "rccl_world_size": world,
                   "stage_ms": stage, "paths": paths},
        "roofline": roof,
        "allgather": None,
        "end_to_end": None,
        "cpu_baseline": None,
    }


HEADLINE_MAX = 3000  # bytes of the last stdout line (the driver keeps a ~9 KB tail of stdout + stderr)
EXTRA_MAX = 1500


def _sig(x, n=4):
    """Floats to n significant digits (recursively); keeps the printed line short."""
    if isinstance(x, float):
        return float(f"{x:.{n}g}")
    if isinstance(x, dict):
        return {k: _sig(v, n) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_sig(v, n) for v in x]
    return x


def compact_line(out: dict, headline: bool = True) -> dict:
    """The printed form of a bench result: the driver's contract fields, a flat ``roofline`` for the
    dominant kernel (+ one [ms, bound, frac] triple per stage), ``cpu_baseline``, the parity count and
    short end-to-end / shard-sweep / extra-config summaries. The full result (per-stage kernel dicts,
    sweep shards, embedded configs) goes to a file (write_full)."""
    keep = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data")
    line = {k: out.get(k) for k in keep}
    c = out.get("config", {})
    if "stage_ms" in c:
        line["config"] = {k: c.get(k) for k in ("workload", "units_total", "units_per_gpu", "clusters", "parallelism",
                                                "rccl_world_size")}
        line["config"]["stage_ms"] = {k: v for k, v in c["stage_ms"].items() if v >= 0.002}
        if headline:
            line["config"]["paths"] = c.get("paths")
    else:  # trigger lines: their config is already short
        line["config"] = c
    r = out.get("roofline")
    if r:
        issue = r.get("issue") or {}
        hbm = r.get("hbm") or {}
        roof = {k: r.get(k) for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "kernel", "time_ms")}
        roof.update({"compulsory_bytes": r.get("compulsory_bytes_per_launch"),
                     "hbm_measured_frac": hbm.get("measured_frac"), "hbm_compulsory_frac": hbm.get("compulsory_frac"),
                     "salu_frac": issue.get("salu_frac"), "valu_frac": issue.get("valu_frac"),
                     "wait_frac": issue.get("wait_frac"), "pmc": r.get("pmc")})
        if headline:
            roof["algorithmic_bytes_per_launch"] = r.get("algorithmic_bytes_per_launch")
            roof["stages"] = {k: [v["time_ms"], v["bound"], v["frac"]] for k, v in (r.get("kernels") or {}).items()}
        line["roofline"] = roof
    cb = out.get("cpu_baseline")
    line["cpu_baseline"] = dict(cb) if cb else None
    if cb and not headline:
        line["cpu_baseline"]["sample"] = cb["sample"].split(",")[0]
    p = out.get("parity")
    line["parity"] = {k: p[k] for k in ("units_checked", "of", "mismatches")} if p else None
    e = out.get("end_to_end")
    if e:
        s = e["sequential"]
        line["end_to_end"] = {"decisions_per_s": e["decisions_per_s"],
                              "seq_ms": {k[:-3]: s[k] for k in ("pack_ms", "h2d_ms", "schedule_ms", "d2h_ms")},
                              "blob_mb": s["blob_mb"], "pipelined_decisions_per_s": e["pipelined"]["decisions_per_s"]}
    if out.get("group"):
        gr = out["group"]
        line["group"] = {"devices": gr["devices"], "member_total_ms": gr["member_total_ms"], "mode": gr["mode"]}
    if out.get("allgather"):
        a = out["allgather"]
        line["allgather"] = {"ms": a["ms"], "gbs": a["gbs"], "backend": a["backend"], "verified": a["verified"]}
    sw = out.get("shard_sweep")
    if sw:
        line["shard_sweep"] = {n: {"max_ms": v["max_ms"], "eff": v["projected_efficiency"]}
                               for n, v in sw["per_n"].items()}
    ex = out.get("extra")
    if ex:
        line["extra"] = {k: {"value": v["value"], "ms_per_step": v["ms_per_step"],
                             "parity_mismatches": (v.get("parity") or {}).get("mismatches")} for k, v in ex.items()}
    if out.get("detail"):
        line["detail"] = out["detail"]
    return _sig(line)


def write_full(out: dict, cfg: str):
    """The full result as one JSON file under gpurun_out/ (what the compact line leaves out)."""
    d = os.path.join(ROOT, "gpurun_out")
    try:
        os.makedirs(d, exist_ok=True)
        path = os.path.join(d, f"bench_full_{cfg}.json")
        with open(path, "w") as f:
            json.dump(out, f, indent=1)
        return os.path.relpath(path, ROOT)
    except OSError:
        return None


def emit(out: dict, cfg: str):
    """Rank 0's stdout: one compact line per extra config, then the headline line LAST (≤ HEADLINE_MAX)."""
    out["detail"] = write_full(out, cfg)
    lines = []
    for k, v in (out.get("extra") or {}).items():
        c = compact_line(v, headline=False)
        s = json.dumps(c)
        # over the budget: shed the least useful fields first, keeping roofline and cpu_baseline
        for path in (("end_to_end",), ("data",), ("config", "stage_ms"), ("roofline", "stages"),
                     ("roofline", "algorithmic_bytes_per_launch")):
            if len(s) <= EXTRA_MAX:
                break
            tgt = c
            for key in path[:-1]:
                tgt = tgt.get(key) if isinstance(tgt.get(key), dict) else {}
            tgt.pop(path[-1], None)
            s = json.dumps(c)
        if len(s) > EXTRA_MAX:
            s = json.dumps({f: c[f] for f in ("metric", "value", "unit", "ms_per_step", "config", "parity") if f in c})
        lines.append(s)
    head = json.dumps(compact_line(out))
    if len(head) > HEADLINE_MAX:  # never let the headline outgrow the driver's capture
        h = compact_line(out)
        for f in ("extra", "shard_sweep", "end_to_end", "detail"):
            h.pop(f, None)
            head = json.dumps(h)
            if len(head) <= HEADLINE_MAX:
                break
    sys.stderr.flush()
    for s in lines:
        print(s, flush=True)
    print(head, flush=True)
    return head


def shard_sweep(args, cfg, local, t1_ms, ns=(2, 4, 8)):
    """Step time of every rank's shard of the C3 batch for N = 2, 4, 8 ranks, each run alone on this GPU
    (the shards bench.py --gpus N would hand out: shard.shard_range, the same per-shard generator), and the
    strong-scaling efficiency they project, t(1 GPU) / (N * max_r t(shard r)), before any RCCL cost (the
    timed step has no collective)."""
    from kubeadmiral_amd import columns as CO
    from kubeadmiral_amd import pack, shard, synth
    from kubeadmiral_amd.runtime import Context

    W_total, C = synth.SIZES[cfg]
    fwk = synth.profile_for(cfg)
    clusters = make_clusters(cfg, C)
    snap = pack.Snapshot(clusters)
    packer = CO.NativePacker(snap)
    ctx = Context(local)
    ctx.upload_snapshot(snap)
    out = {"t1_ms": t1_ms, "steps": args.steps, "per_n": {}}
    for n in ns:
        ts, stages = [], []
        for r in range(n):
            lo, hi = shard.shard_range(W_total, r, n)
            ctx.upload_batch(packer.pack(fwk, make_columns(cfg, lo, hi, clusters)))
            for _ in range(max(2, args.warmup)):
                ctx.schedule(fwk)
            ctx.sync()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                ctx.schedule(fwk)
            ctx.sync()
            ts.append((time.perf_counter() - t0) / max(1, args.steps) * 1e3)
            if r == 0:  # rank 0's per-stage device times (HIP events), outside the timing
                ctx.set_timing(True)
                st = []
                for _ in range(3):
                    ctx.schedule(fwk)
                    ctx.sync()
                    st.append(ctx.stage_timing())
                ctx.set_timing(False)
                stages = {k: float(np.mean([x[k] for x in st])) for k in ctx.STAGES}
        tn = max(ts)
        out["per_n"][str(n)] = {"units_per_rank": W_total // n, "shard_ms": ts, "max_ms": tn, "rank0_stage_ms": stages,
                                "projected_decisions_per_s": W_total * C / (tn * 1e-3),
                                "projected_efficiency": t1_ms / (n * tn)}
        log(f"[sweep] N={n}: shard ms {['%.3f' % t for t in ts]} -> efficiency {t1_ms / (n * tn):.3f}")
    ctx.close()
    return out


def end_to_end(ctx, snap, fwk, cols, res, C, packer_for, chunks=4, packs=2):
    """The hot path as a caller sees it, from columnar units to downloaded placements, one rank, warm:
    * sequential: native pack (in place, page-locked) → kad_batch_upload (one DMA) → schedule → D2H;
    * pipelined: the batch in ``chunks`` unit ranges, two contexts alternating and ``packs`` chunk packs in
      flight on worker threads (ctypes releases the GIL; one packer each, plus the one being uploaded), so
      chunks i+1.. are packed on the host while chunk i is uploaded, scheduled and downloaded — what a
      batching caller (batcher.CoalescingScheduler) does with a stream of units. Two packs in flight overlap
      one pack's narrow phases with the other's parallel ones; the upload checks then run on the library's
      side pool instead of waiting behind a pack (kad_pool.h run_checks).
    Both must reproduce the timed run's rows exactly."""
    from concurrent.futures import ThreadPoolExecutor

    from kubeadmiral_amd import columns as CO
    from kubeadmiral_amd.results import BatchResult
    from kubeadmiral_amd.runtime import Context

    W = cols.n_units
    packer = CO.NativePacker(packer_for)
    nb = packer.pack(fwk, cols, take=False)  # warm (allocates the page-locked buffer)
    ctx.upload_batch(nb)
    ctx.sync()
    pinned = BatchResult.pinned(W, max(1, nb.n_out_slots))  # page-locked, reused (allocated outside the timing)
    t0 = time.perf_counter()
    nb = packer.pack(fwk, cols, take=False)
    t1 = time.perf_counter()
    ctx.upload_batch(nb)
    ctx.sync()
    t2 = time.perf_counter()
    ctx.schedule(fwk)
    ctx.sync()
    t3 = time.perf_counter()
    r2 = ctx.download(out=pinned)
    t4 = time.perf_counter()
    assert r2.equal_rows(res).all(), "end-to-end rerun differs from the timed run"
    tot = t4 - t0
    seq = {"pack_ms": (t1 - t0) * 1e3, "h2d_ms": (t2 - t1) * 1e3, "schedule_ms": (t3 - t2) * 1e3,
           "d2h_ms": (t4 - t3) * 1e3, "total_ms": tot * 1e3, "units": W, "decisions_per_s": W * C / tot,
           "pack_units_per_s": W / (t1 - t0), "blob_mb": nb.blob.nbytes / 1e6, "h2d_gbs": nb.blob.nbytes / (t2 - t1) / 1e9}
    # pipelined over chunks
    ctx2 = Context(ctx.device)
    ctx2.upload_snapshot(packer_for)
    ctxs = (ctx, ctx2)
    bounds = [W * i // chunks for i in range(chunks + 1)]
    parts = [cols.slice(bounds[i], bounds[i + 1]) for i in range(chunks)]
    bufs = None
    pipe = None
    tried = {}
    # one pack in flight (it takes the library's whole host pool) and two (one pack's narrow phases beside the
    # other's parallel ones): which wins depends on the host — on the round-5/6 boxes two in flight lost to the
    # sequential pass — so both run and the faster is reported
    for npk in sorted({1, packs}):
        packers = [packer] + [CO.NativePacker(packer_for) for _ in range(npk)]
        with ThreadPoolExecutor(max_workers=npk) as pool:
            for rep in range(2):  # first pass warms the packers / contexts and sizes the result buffers
                outs = []
                t0 = time.perf_counter()
                futs = {i: pool.submit(packers[i % len(packers)].pack, fwk, parts[i], 0, False)
                        for i in range(min(npk, chunks))}
                for i in range(chunks):
                    nbi = futs.pop(i).result()
                    if i + npk < chunks:
                        j = i + npk
                        futs[j] = pool.submit(packers[j % len(packers)].pack, fwk, parts[j], 0, False)
                    c = ctxs[i % 2]
                    c.upload_batch(nbi)
                    c.schedule(fwk)
                    r = c.download(out=bufs[i] if bufs else None)
                    r.out_off = np.array(r.out_off)  # a view into the packer's buffer, which chunk i + npk + 1 reuses
                    outs.append(r)
                tot = time.perf_counter() - t0
                if bufs is None:
                    bufs = [BatchResult.pinned(len(r.status), len(r.cluster)) for r in outs]
        tried[npk] = tot * 1e3
        if pipe is None or tot * 1e3 < pipe["total_ms"]:
            pipe = {"chunks": chunks, "packs_in_flight": npk, "total_ms": tot * 1e3, "decisions_per_s": W * C / tot}
    pipe["total_ms_by_packs_in_flight"] = tried
    ctx2.close()
    # every chunk's rows equal the timed run's rows of the same units
    for i, r in enumerate(outs):
        lo = bounds[i]
        for w in range(0, bounds[i + 1] - lo, max(1, (bounds[i + 1] - lo) // 2000)):
            assert r.row(w) == res.row(lo + w), f"pipelined chunk {i} unit {w} differs"
    return {"decisions_per_s": max(seq["decisions_per_s"], pipe["decisions_per_s"]), "sequential": seq,
            "pipelined": pipe,
            "note": "native packer from columnar units (page-locked blob, zero-copy upload) + H2D + schedule + D2H "
                    "(into page-locked result arrays reused across batches); pipelined: pack of chunk i+1 overlaps the GPU work of chunk i; not the "
                    "headline value"}


def gather_placements(ctx, batch, res, dist, world, dev, blobs=None, fwk=None):
    """All-gather of every rank's placements: status / count / flags [W_r] and (cluster, replicas) slots,
    each rank's arrays padded to the largest rank's sizes (fixed per-rank slots). RCCL on device buffers
    filled device-to-device from libkad (kad_results_copy_device); host tensors in the gloo rehearsal."""
    import torch

    W = batch.W
    S = batch.n_out_slots
    mx = torch.tensor([W, S], dtype=torch.int64, device=dev)
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    Wm, Sm = int(mx[0]), max(1, int(mx[1]))
    st = torch.zeros(3 * Wm, dtype=torch.int32, device=dev)  # status | count | flags
    cl = torch.full((Sm,), -1, dtype=torch.int32, device=dev)
    rp = torch.zeros(Sm, dtype=torch.int64, device=dev)
    if dev != "cpu":
        # the fills above run on torch's stream, libkad's copy on its own: the fills must land first
        torch.cuda.synchronize()
        ctx.copy_results_device(st.data_ptr(), st.data_ptr() + 4 * Wm, st.data_ptr() + 8 * Wm, cl.data_ptr(),
                                rp.data_ptr())
    else:
        st[:W] = torch.from_numpy(res.status[:W])
        st[Wm:Wm + W] = torch.from_numpy(res.count[:W])
        st[2 * Wm:2 * Wm + W] = torch.from_numpy(res.flags[:W].view(np.int32))
        cl[:S] = torch.from_numpy(res.cluster[:S])
        rp[:S] = torch.from_numpy(res.replicas[:S])
    g_st = [torch.empty_like(st) for _ in range(world)]
    g_cl = [torch.empty_like(cl) for _ in range(world)]
    g_rp = [torch.empty_like(rp) for _ in range(world)]
    times = []
    for _ in range(5):
        if dev != "cpu":
            torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        dist.all_gather(g_st, st)
        dist.all_gather(g_cl, cl)
        dist.all_gather(g_rp, rp)
        if dev != "cpu":
            torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    t = torch.tensor([float(np.median(times))], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    # this rank's own part of the gathered arrays equals its download
    r = dist.get_rank()
    assert np.array_equal(g_st[r][:W].cpu().numpy(), res.status[:W]), "all-gathered placements differ"
    assert np.array_equal(g_cl[r][:S].cpu().numpy(), res.cluster[:S]), "all-gathered placements differ"  # same buffer
    verified = None
    if r == 0 and blobs is not None:
        # every rank's gathered part equals a single-rank run of the same shard blob on rank 0
        for q in range(world):
            ctx.upload_batch(blobs[q])
            ctx.schedule(fwk)
            one = ctx.download()
            Wq, Sq = blobs[q].W, blobs[q].n_out_slots
            gs, gc, gr = g_st[q].cpu().numpy(), g_cl[q].cpu().numpy(), g_rp[q].cpu().numpy()
            # the written slots of each unit: [out_off[w], out_off[w] + count[w]) (the rest of a unit's bound
            # is never written, by either run)
            cnt = one.count[:Wq].astype(np.int64)
            valid = np.zeros(Sq, bool)
            starts = np.asarray(blobs[q].out_off[:Wq], np.int64)
            idx = np.repeat(starts, cnt) + (np.arange(int(cnt.sum())) - np.repeat(np.cumsum(cnt) - cnt, cnt))
            valid[idx] = True
            for what, got, want in (("status", gs[:Wq], one.status[:Wq]), ("count", gs[Wm:Wm + Wq], one.count[:Wq]),
                                    ("flags", gs[2 * Wm:2 * Wm + Wq], one.flags[:Wq].view(np.int32)),
                                    ("cluster", gc[:Sq][valid], one.cluster[:Sq][valid]),
                                    ("replicas", gr[:Sq][valid], one.replicas[:Sq][valid])):
                assert np.array_equal(got, want), f"gathered {what} of rank {q} differs from a single-rank run"
        verified = f"all {world} ranks' status/count/flags/cluster/replicas == single-rank runs of their shards"
    nbytes = world * (12 * Wm + 12 * Sm)
    return {"ms": float(t[0]) * 1e3, "bytes_gathered": nbytes, "per_rank_slots": Sm, "per_rank_units": Wm,
            "gbs": nbytes / (float(t[0]) + 1e-12) / 1e9, "backend": "rccl" if dev != "cpu" else "gloo",
            "verified": verified}


# ------------------------------------------------------------------------ trigger bench (§8 f4)
def bench_trigger(args, cfg, rank, world, local, dist):
    """computeSchedulingTriggerHash for a batch of objects (kad_trigger_*), weak scaling."""
    from kubeadmiral_amd import objects as O
    from kubeadmiral_amd import synth
    from kubeadmiral_amd.runtime import Context

    W0, C = synth.TRIGGER_SIZES[cfg]
    W = args.units if args.units is not None else W0
    rng = np.random.default_rng(0x7 + rank)
    ftc, clusters, objs, pols = synth.gen_trigger_workload(rng, W, C)
    suffix = O.trigger_suffix(clusters)
    prefixes = [O.trigger_prefix(ftc, o, p) for o, p in zip(objs, pols)]
    pre_bytes = sum(len(p) for p in prefixes)
    log(f"[rank {rank}] {cfg}: {W} objects, cluster part {len(suffix)} B, object parts {pre_bytes / max(1, W):.0f} B avg")
    ctx = Context(local)
    ctx.trigger_suffix_upload(suffix)
    ctx.trigger_prefixes_upload(prefixes)
    for _ in range(args.warmup):
        ctx.trigger_run()
        ctx.sync()
    if dist is not None:
        dist.barrier()
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ctx.trigger_run()
    ctx.sync()
    if dist is not None:
        dist.barrier()
    ms = (time.perf_counter() - t0) / max(1, args.steps) * 1e3
    tot, summ = [], []
    for _ in range(max(3, min(args.steps, 10))):
        ctx.trigger_run()
        a, b = ctx.trigger_timing()
        tot.append(a)
        summ.append(b)
    tot_ms, sum_ms = float(np.mean(tot)), float(np.mean(summ))
    units_total = W * world
    if dist is not None:
        import torch

        t = torch.tensor([ms, tot_ms, sum_ms], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ms, tot_ms, sum_ms = t.tolist()
    out = None
    if rank == 0:
        steps = 256.0 * len(suffix)  # FNV steps of the cluster-part summary (256 residue chains)
        obj_bytes = pre_bytes + 8 * (W + 1) + 4 * W
        out = {
            "metric": "scheduling-trigger hashes/sec (objects/s)", "value": units_total / (ms * 1e-3),
            "unit": "objects/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
            "data": "synthetic (seeded federated Deployments, policies and joined clusters)",
            "config": {"workload": f"{cfg}: {WORKLOAD_DESC[cfg]}", "objects_per_gpu": W, "objects_total": units_total,
                       "clusters": C, "cluster_part_bytes": len(suffix), "object_part_bytes_avg": pre_bytes / max(1, W),
                       "parallelism": f"dp{world}",
                       "kernel_ms": {"cluster_part_summary": sum_ms, "objects": tot_ms - sum_ms}},
            "roofline": {"bound": "valu", "achieved": steps / (sum_ms * 1e-3), "peak": FNV_STEP_PEAK,
                         "unit": "FNV steps/s", "frac": steps / (sum_ms * 1e-3) / FNV_STEP_PEAK, "traffic": None,
                         "kernel": "trig_segment_kernel + trig_compose_kernel (256 residue chains over the cluster part)",
                         "objects_kernel_gbs": obj_bytes / max(1e-9, (tot_ms - sum_ms) * 1e-3) / 1e9},
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_cpu_baseline:
            from oracle import ref

            threads, n_machine, quota = host_cpus()
            n = min(W, 64)
            t0 = time.perf_counter()
            ref.trigger_hashes(prefixes[:n], suffix, threads)
            dt = time.perf_counter() - t0
            n = int(min(W, max(n, n * args.cpu_seconds / max(dt, 1e-6))))
            t0 = time.perf_counter()
            ref.trigger_hashes(prefixes[:n], suffix, threads)
            dt = time.perf_counter() - t0
            out["cpu_baseline"] = {"value": n / dt, "unit": "objects/s", "cores": threads, "kind": "port",
                                   "cpu_count": n_machine, "cgroup_cpu_limit": quota,
                                   "sample": f"first {n} of {W} objects, oracle/kad_trigger_ref.c (each object's "
                                             f"bytes folded end to end, as schedulingtriggers.go:141-145; JSON "
                                             f"building not timed), {dt:.2f}s wall"}
    ctx.close()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c3", choices=sorted(WORKLOAD_DESC))
    ap.add_argument("--units", type=int, default=None, help="total units (default: the config's W)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip the embedded C2/C4/C5 lines of the default run")
    ap.add_argument("--extras", default="c3r,c3p,c2,c4,c5", help="configs embedded under `extra` in the default C3 run")
    ap.add_argument("--no-sweep", action="store_true", help="skip the C3 shard-size sweep of the default run")
    ap.add_argument("--no-e2e", action="store_true", help="skip the pack -> upload -> schedule -> download timing")
    ap.add_argument("--backend", default="nccl", choices=("nccl", "gloo"),
                    help="gloo: rehearse the multi-rank path with host-tensor transfers (e.g. ranks sharing one GPU)")
    ap.add_argument("--share-gpu", action="store_true", help="every rank uses device 0 (rehearsal on a 1-GPU box)")
    ap.add_argument("--mode", default="group", choices=("group", "ranks"),
                    help="--gpus N > 1: group = one process over N devices through kad_group_* (the C ABI's "
                         "multi-GPU path, default); ranks = one torch.distributed rank per GPU, snapshot and "
                         "shards over RCCL, placements all-gathered")
    ap.add_argument("--group-devices", default=None,
                    help="group mode: comma-separated HIP device ids (default 0..N-1; e.g. 0,0,0,0 rehearses "
                         "four members on a one-GPU box)")
    args = ap.parse_args()

    if args.mode == "group" and args.gpus > 1 and not args.config.startswith("t"):
        sys.exit(main_group(args))
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(relaunch(args))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = 0 if args.share_gpu else int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch with --nproc-per-node {args.gpus}")
    import torch

    dist = None
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")

    from kubeadmiral_amd import build

    if rank == 0:
        build.build()
    if dist is not None:
        dist.barrier()

    cfg = args.config
    if cfg.startswith("t"):
        out = bench_trigger(args, cfg, rank, world, local, dist)
    else:
        out = bench_schedule(args, cfg, rank, world, local, dist)
        default_run = cfg == "c3" and world == 1 and args.units is None
        # the default run also measures every other single-GPU config (C2 100k x 256, C4 1M x 512 Divide,
        # C5 100k x 10k) on the same box and embeds their full lines, sampled CPU baselines included
        if default_run and not args.no_extra:
            out["extra"] = {}
            for c2 in [c for c in args.extras.split(",") if c]:
                out["extra"][c2] = bench_schedule(args, c2, rank, world, local, dist, W_total=None,
                                                  cpu_seconds=args.cpu_seconds / 2)
        # and C3's shard sizes for N = 2, 4, 8 (the 1-GPU projection of strong scaling)
        if default_run and not args.no_sweep:
            out["shard_sweep"] = shard_sweep(args, cfg, local, out["ms_per_step"])
    if rank == 0 and out is not None:
        emit(out, cfg)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def main_group(args) -> int:
    """--mode group: this process (or rank 0 of a torch.distributed launch) drives all N devices."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world not in (1, args.gpus):
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    import torch  # noqa: F401

    dist = None
    if world > 1:  # launched one rank per GPU (the driver's SCALE run): a CPU process group for the barriers
        import torch.distributed as dist

        dist.init_process_group("gloo")
    devices = ([int(x) for x in args.group_devices.split(",")] if args.group_devices
               else list(range(args.gpus)))
    if len(devices) != args.gpus:
        raise SystemExit(f"--group-devices names {len(devices)} devices, --gpus {args.gpus}")
    from kubeadmiral_amd import build

    if rank == 0:
        build.build()
    if dist is not None:
        dist.barrier()
    out = bench_group(args, args.config, devices, dist, rank)
    if rank == 0 and out is not None:
        emit(out, args.config)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    main()

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
    return synth.gen_clusters(rng, C)


def make_columns(cfg: str, lo: int, hi: int, clusters):
    """Columns (kad_su_columns) of units [lo, hi) of the config's batch (seeded per shard)."""
    from kubeadmiral_amd import columns as CO
    from kubeadmiral_amd import synth

    rng = np.random.default_rng([synth.SEEDS[cfg], lo])
    if cfg in ("c2", "c3"):
        return synth.gen_units_c2_columns(rng, hi - lo, prefix=f"su{lo}")
    gen = {"c1": synth.gen_units_c1, "c4": synth.gen_units_c4, "c5": synth.gen_units_c5}[cfg]
    units = gen(rng, hi - lo, clusters)
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
    """profiles/pmc_<cfg>.json (scripts/profile.sh → scripts/pmc_summary.py) when it matches the workload."""
    path = os.path.join(ROOT, "profiles", f"pmc_{cfg}.json")
    if not os.path.exists(path):
        return None, path
    with open(path) as f:
        pmc = json.load(f)
    if pmc.get("units") != W or pmc.get("clusters") != C:
        return None, path
    return pmc, path


def cpu_baseline(snap, batch, fwk, C, target_s):
    from oracle import ref

    threads = min(16, os.cpu_count() or 1)
    n = min(batch.W, 2000)
    t0 = time.perf_counter()
    ref.schedule(snap, batch, fwk, 0, n, threads)
    dt = time.perf_counter() - t0
    n2 = int(min(batch.W, max(n, n * target_s / max(dt, 1e-6))))
    if n2 > n:
        t0 = time.perf_counter()
        ref.schedule(snap, batch, fwk, 0, n2, threads)
        dt = time.perf_counter() - t0
        n = n2
    reps = max(1, int(target_s / max(dt, 1e-6)))
    if reps > 1:
        t0 = time.perf_counter()
        for _ in range(reps):
            ref.schedule(snap, batch, fwk, 0, n, threads)
        dt = time.perf_counter() - t0
    return {"value": reps * n * C / dt, "unit": "decisions/s", "cores": threads, "kind": "port",
            "sample": f"{reps} pass(es) over the first {n} of {batch.W} units x {C} clusters, oracle/kad_ref.c "
                      f"(C restatement of the Go reference, one unit per worker thread), {dt:.2f}s wall"}


# ------------------------------------------------------------------------ scheduling bench
def bench_schedule(args, cfg, rank, world, local, dist, W_total=None, extra_line=False):
    import torch  # noqa: F401  (HIP runtime initialised by torch before libkad.so)

    from kubeadmiral_amd import columns as CO
    from kubeadmiral_amd import pack, shard, synth
    from kubeadmiral_amd.runtime import Context

    W0, C = synth.SIZES[cfg]
    W_total = W_total if W_total is not None else (args.units if args.units is not None else W0)
    fwk = synth.profile_for(cfg)
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
        allgather = gather_placements(ctx, batch, res, dist, world, cdev)

    if dist is not None:
        t = torch.tensor([ms] + [stage[k] for k in ctx.STAGES], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ms = float(t[0])
        stage = {k: float(v) for k, v in zip(ctx.STAGES, t[1:].tolist())}

    out = None
    if rank == 0:
        value = W_total * C / (ms * 1e-3)
        W0r = batch.W
        nch = (C + 63) // 64
        count = res.count.astype(np.int64)
        out_bytes = 12 * W0r + 12 * float(count.sum())
        # dominant kernel (the main schedule kernel): its compulsory bytes per launch — unit records,
        # static filter words, the cluster columns it caches, its outputs — over its HIP-event time
        main_bytes = 64 * W0r + 8 * nch * W0r + 56 * C + out_bytes
        t_main = stage["main"]
        main_gbs = main_bytes / (t_main * 1e-3) / 1e9
        # the whole filter/score/select stage: batch blob + snapshot + outputs once
        fss_ms = stage["req_mask"] + stage["prep"] + stage["main"] + stage["defer"]
        stage_bytes = batch.blob.nbytes + snap.blob.nbytes + out_bytes
        cols0, nb0 = stats0
        divide = (nb0.flags & pack.W_DUPLICATE) == 0 if fwk.replicas_plugin >= 0 else np.zeros(W0r, bool)
        kbytes, pbytes = canonical_bytes(nb0.n_reqs, nb0.n_tols, count, C, snap.TW, count[divide])
        pmc, pmc_path = load_pmc(cfg, W0r, C)
        traffic = issue = None
        if pmc is not None:
            k = pmc.get("main_kernel", {})
            traffic = k.get("hbm_bytes_per_launch")
            if k.get("SQ_INSTS_VALU") is not None:
                issue = {"valu_insts": k["SQ_INSTS_VALU"], "salu_insts": k["SQ_INSTS_SALU"],
                         "valu_frac": k["SQ_INSTS_VALU"] / (t_main * 1e-3 * VALU_PEAK),
                         "salu_frac": k["SQ_INSTS_SALU"] / (t_main * 1e-3 * SALU_PEAK),
                         "peaks": "VALU 1.23e12 wave-instr/s (256 CU x 4 SIMD x 2.4 GHz / 2), "
                                  "SALU 6.1e11 (256 CU x 2.4 GHz)", "source": os.path.relpath(pmc_path, ROOT)}
        out = {
            "metric": "scheduling decisions/sec (workload x cluster evals/s)",
            "value": value,
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
                       "stage_ms": stage},
            "roofline": {
                "bound": "hbm", "achieved": main_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": main_gbs / HBM_PEAK_GBS, "traffic": traffic,
                "kernel": "schedule_wide_kernel" if 4 < nch <= 16 else "schedule_lean_kernel",
                "time_ms": t_main, "compulsory_bytes_per_launch": main_bytes,
                "bytes_model": "64 B UnitRec + 8 B x chunks static filter words per unit, 56 B per cached "
                               "cluster, 12 B per unit + 12 B per placement out",
                "measured_hbm_gbs": (traffic / (t_main * 1e-3) / 1e9) if traffic else None,
                "stage": {"time_ms": fss_ms, "compulsory_bytes": stage_bytes,
                          "frac": stage_bytes / (fss_ms * 1e-3) / 1e9 / HBM_PEAK_GBS},
                "issue": issue,
                "algorithmic_bytes_per_launch": kbytes,
                "algorithmic_model_frac": kbytes / (fss_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                "planner": ({"time_ms": stage["planner"], "bytes": pbytes,
                             "frac": pbytes / (stage["planner"] * 1e-3) / 1e9 / HBM_PEAK_GBS}
                            if stage["planner"] > 0.001 else None),
            },
            "allgather": allgather,
            "end_to_end": None,
            "cpu_baseline": None,
        }
        if world == 1:
            out["end_to_end"] = end_to_end(ctx, snap, fwk, cols0, res, C, packer_for=snap)
            if not args.no_cpu_baseline:
                log(f"[rank 0] timing the CPU baseline (C restatement of the reference) on {cfg}")
                out["cpu_baseline"] = cpu_baseline(snap, batch, fwk, C, args.cpu_seconds)
    ctx.close()
    return out


def end_to_end(ctx, snap, fwk, cols, res, C, packer_for):
    """pack (native) + H2D (batch blob) + schedule + D2H (results), one rank, warm."""
    from kubeadmiral_amd import columns as CO

    packer = CO.NativePacker(packer_for)
    packer.pack(fwk, cols)  # warm
    t0 = time.perf_counter()
    nb = packer.pack(fwk, cols)
    t1 = time.perf_counter()
    ctx.upload_batch(nb)
    ctx.sync()
    t2 = time.perf_counter()
    ctx.schedule(fwk)
    ctx.sync()
    t3 = time.perf_counter()
    r2 = ctx.download()
    t4 = time.perf_counter()
    assert r2.equal_rows(res).all(), "end-to-end rerun differs from the timed run"
    tot = t4 - t0
    return {"pack_ms": (t1 - t0) * 1e3, "h2d_ms": (t2 - t1) * 1e3, "schedule_ms": (t3 - t2) * 1e3,
            "d2h_ms": (t4 - t3) * 1e3, "total_ms": tot * 1e3, "units": nb.W,
            "decisions_per_s": nb.W * C / tot, "pack_units_per_s": nb.W / (t1 - t0),
            "blob_mb": nb.blob.nbytes / 1e6,
            "note": "native packer (libkad.so kad_pack_batch) from columnar units; H2D/D2H through pageable "
                    "host buffers; not the headline value"}


def gather_placements(ctx, batch, res, dist, world, dev):
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
    assert np.array_equal(g_cl[r][:S].cpu().numpy(), res.cluster[:S]), "all-gathered placements differ"
    nbytes = world * (12 * Wm + 12 * Sm)
    return {"ms": float(t[0]) * 1e3, "bytes_gathered": nbytes, "per_rank_slots": Sm, "per_rank_units": Wm,
            "gbs": nbytes / (float(t[0]) + 1e-12) / 1e9, "backend": "rccl" if dev != "cpu" else "gloo"}


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

            threads = min(16, os.cpu_count() or 1)
            n = min(W, 64)
            t0 = time.perf_counter()
            ref.trigger_hashes(prefixes[:n], suffix, threads)
            dt = time.perf_counter() - t0
            n = int(min(W, max(n, n * args.cpu_seconds / max(dt, 1e-6))))
            t0 = time.perf_counter()
            ref.trigger_hashes(prefixes[:n], suffix, threads)
            dt = time.perf_counter() - t0
            out["cpu_baseline"] = {"value": n / dt, "unit": "objects/s", "cores": threads, "kind": "port",
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
    ap.add_argument("--no-extra", action="store_true", help="skip the embedded C2 line of the default run")
    ap.add_argument("--backend", default="nccl", choices=("nccl", "gloo"),
                    help="gloo: rehearse the multi-rank path with host-tensor transfers (e.g. ranks sharing one GPU)")
    ap.add_argument("--share-gpu", action="store_true", help="every rank uses device 0 (rehearsal on a 1-GPU box)")
    args = ap.parse_args()

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
        # the default run also measures C2 (100k x 256, one GPU) and embeds it
        if (cfg == "c3" and world == 1 and args.units is None and not args.no_extra):
            a2 = argparse.Namespace(**vars(args))
            a2.no_cpu_baseline = True
            o2 = bench_schedule(a2, "c2", rank, world, local, dist, W_total=None)
            if out is not None and o2 is not None:
                out["extra"] = {"c2": {k: o2[k] for k in ("value", "ms_per_step")} |
                                {"config": o2["config"], "roofline_frac": o2["roofline"]["frac"],
                                 "roofline_time_ms": o2["roofline"]["time_ms"],
                                 "end_to_end": o2["end_to_end"]}}
    if rank == 0 and out is not None:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Benchmark: scheduling decisions/s (workload × cluster evaluations per second).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2]

One step = one pass of the hot path (filter → score → select [→ replicas])
over the whole resident batch of SchedulingUnits against the resident
cluster snapshot (kad_schedule + stream sync). For N > 1 the driver launches
one process per GPU (torch.distributed.run); rank 0 packs the cluster snapshot
and RCCL-broadcasts the blob over xGMI, every rank schedules its own shard of
units (weak scaling: the per-GPU batch is the config's W), no collective runs
inside the timed region, and the time is the max over ranks.

Prints ONE JSON line (rank 0) with the driver's contract fields plus
``roofline`` (canonical algorithmic bytes of SURVEY.md §8(d) per launch of the
filter/score/select kernel ÷ its HIP-event time, against 8 TB/s) and
``cpu_baseline`` (the C restatement of the reference — oracle/kad_ref.c —
timed on a bounded sample on this host's cores).
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0
WORKLOAD_DESC = {
    "c1": "1k Deployment SchedulingUnits x 16 FederatedClusters, default plugin set, Divide",
    "c2": "100k SchedulingUnits x 256 FederatedClusters: Fit+Taint+Affinity(+APIResources) filters, "
          "LeastAllocated score, MaxCluster select, Duplicate",
    "c3": "1M SchedulingUnits x 1k FederatedClusters (c2 generator), sharded over GPUs",
    "c4": "1M Divide SchedulingUnits x 512 clusters: weights, min/max replicas, capacity caps",
    "c5": "100k SchedulingUnits x 10k clusters: dense label affinity, many taints, API-resource gaps",
    "t1": "scheduling-trigger hashes: 1k federated Deployments x 16 joined clusters",
    "t2": "scheduling-trigger hashes: 100k federated Deployments x 256 joined clusters (~1.6 MB cluster part)",
}
# Issue bound of one FNV-1 step per lane: the inner loop is one v_mul_lo_u32 (quarter rate: 16 SIMD cycles per
# wave64 instruction) + one v_bitop3_b32 per byte. The round-1 t2 run measured 3.64 steps/cycle/SIMD, above the
# 3.2 of issuing both back to back, so the bitop overlaps the multiply: the bound is the multiply alone,
# 4 steps/cycle/SIMD × 4 SIMDs × 256 CUs × 2.4 GHz.
FNV_STEP_PEAK = 4.0 * 4 * 256 * 2.4e9


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def canonical_bytes(batch, res, C, TW, divide_rows):
    """W·C·B_pair + Σ_w B_w + Σ_w K_w·B_plan (bytes per launch)."""
    r = batch.n_reqs.astype(np.float64)
    b_pair = 32 + 16 + 16 * (TW - 1) + 4 + 4 + 4 * r
    pair = float(np.sum(b_pair) * C)
    per_w = float(np.sum(128 + 16 * r + 8 * batch.n_tols + 12 * res.count))
    plan = float(np.sum(res.count[divide_rows]) * 48) if divide_rows is not None else 0.0
    return pair + per_w, plan


def cpu_baseline(snap, batch, fwk, C, target_s):
    from oracle import ref

    threads = min(16, os.cpu_count() or 1)
    n = min(batch.W, 2000)
    t0 = time.perf_counter()
    ref.schedule(snap, batch, fwk, 0, n, threads)
    dt = time.perf_counter() - t0
    # grow the sample to ~target_s of CPU work: first more units (bounded by
    # the batch), then repeated passes over them
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


def bench_trigger(args, cfg, rank, world, local, dist):
    """§8(f) f4: computeSchedulingTriggerHash for a batch of objects (kad_trigger_*)."""
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
        print(json.dumps(out), flush=True)
    ctx.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=sorted(WORKLOAD_DESC))
    ap.add_argument("--units", type=int, default=None, help="units per GPU (default: the config's W)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--pmc", default=None, help="JSON with per-launch HBM bytes from rocprofv3 (profiles/)")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist

        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from kubeadmiral_amd import build, pack, synth
    from kubeadmiral_amd.runtime import Context

    if rank == 0:
        build.build()
    if dist is not None:
        dist.barrier()

    cfg = args.config
    if cfg.startswith("t"):
        bench_trigger(args, cfg, rank, world, local, dist)
        if dist is not None:
            dist.barrier()
            dist.destroy_process_group()
        return
    W0, C = synth.SIZES[cfg]
    W = args.units if args.units is not None else (W0 if cfg not in ("c3", "c4") else W0 // max(1, world))
    log(f"[rank {rank}] generating {cfg}: {W} units x {C} clusters")
    t0 = time.time()
    rng = np.random.default_rng(synth.SEEDS[cfg])
    if cfg == "c5":
        clusters = synth.gen_clusters(rng, C, n_keys=64, n_vals=16, n_int_keys=4, n_taints=256, taints_per=(4, 16),
                                      p_gvk=0.9, gvks=synth.GVKS)
    else:
        clusters = synth.gen_clusters(rng, C)
    urng = np.random.default_rng(synth.SEEDS[cfg] * 1000 + rank)
    if cfg in ("c2", "c3"):
        units = synth.gen_units_c2(urng, W, prefix=f"r{rank}")
    elif cfg == "c1":
        units = synth.gen_units_c1(urng, W, clusters)
    elif cfg == "c4":
        units = synth.gen_units_c4(urng, W, clusters)
    else:
        units = synth.gen_units_c5(urng, W, clusters)
    fwk = synth.profile_for(cfg)
    snap = pack.Snapshot(clusters)
    batch = pack.Batch(snap, fwk, units)
    log(f"[rank {rank}] packed in {time.time() - t0:.1f}s: batch {batch.blob.nbytes / 1e6:.1f} MB, "
        f"snapshot {snap.blob.nbytes / 1e3:.1f} kB")

    ctx = Context(local)
    if dist is not None:
        # rank 0's packed snapshot is the one every rank schedules against: RCCL broadcast over xGMI
        import torch

        buf = torch.empty(snap.blob.nbytes, dtype=torch.uint8, device=f"cuda:{local}")
        if rank == 0:
            buf.copy_(torch.from_numpy(snap.blob))
        dist.broadcast(buf, src=0)
        torch.cuda.synchronize()
        ctx.upload_snapshot_device(buf.data_ptr(), snap.blob.nbytes, snap)
        del buf
    else:
        ctx.upload_snapshot(snap)
    ctx.upload_batch(batch)

    for _ in range(args.warmup):
        ctx.schedule(fwk)
        ctx.sync()
    if dist is not None:
        dist.barrier()
    ctx.sync()
    # timed region: K full passes enqueued back to back on the context's
    # stream (each pass: req_mask → prep → schedule → defer pass → planner);
    # no event records between them (the per-kernel times come from the loop below)
    ctx.set_timing(False)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ctx.schedule(fwk)
    ctx.sync()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    res = ctx.download()
    # per-kernel device time (HIP events on the context's stream), outside the timed region
    ctx.set_timing(True)
    kms, pms = [], []
    for _ in range(max(3, min(args.steps, 10))):
        ctx.schedule(fwk)
        ctx.sync()
        _, k1, k2 = ctx.timing()
        kms.append(k1)
        pms.append(k2)
    ms = elapsed / max(1, args.steps) * 1e3
    units_total = W * world
    if dist is not None:
        import torch

        t = torch.tensor([ms, float(np.mean(kms)), float(np.mean(pms))], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ms, kmax, pmax = t.tolist()
        n = torch.tensor([W], dtype=torch.int64, device=f"cuda:{local}")
        dist.all_reduce(n)
        units_total = int(n.item())
    else:
        kmax, pmax = float(np.mean(kms)), float(np.mean(pms))

    divide = np.nonzero(((batch.arrays[0] & pack.W_DUPLICATE) == 0))[0] if fwk.replicas_plugin >= 0 else None
    kbytes, pbytes = canonical_bytes(batch, res, C, snap.TW, divide)
    achieved = kbytes / (kmax * 1e-3) / 1e9
    traffic = None
    pmc_path = args.pmc or os.path.join(ROOT, "profiles", f"pmc_{cfg}.json")
    if os.path.exists(pmc_path):
        with open(pmc_path) as f:
            pmc = json.load(f)
        if pmc.get("units") == W and pmc.get("clusters") == C:
            traffic = pmc.get("hbm_bytes_per_launch")

    out = None
    if rank == 0:
        value = units_total * C / (ms * 1e-3)
        out = {
            "metric": "scheduling decisions/sec (workload x cluster evals/s)",
            "value": value,
            "unit": "decisions/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic (seeded SURVEY.md §8(d) generator; no cluster/dataset available)",
            "config": {"workload": f"{cfg}: {WORKLOAD_DESC[cfg]}", "units_per_gpu": W, "units_total": units_total,
                       "clusters": C, "parallelism": f"dp{world}",
                       "kernel_ms": {"filter_score_select": kmax, "replica_planner": pmax}},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "algorithmic_bytes_per_launch": kbytes,
                         # what actually crosses the HBM interface (rocprofv3 FETCH/WRITE, profiles/pmc_<cfg>.json)
                         # over the same time: the per-pair operands of the byte model are served from LDS
                         "measured_hbm_gbs": (traffic / (kmax * 1e-3) / 1e9) if traffic else None,
                         "time_ms": kmax, "timed": "req_mask + prep + schedule kernels (HIP events)"},
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_cpu_baseline:
            log("[rank 0] timing the CPU baseline (C restatement of the reference)")
            out["cpu_baseline"] = cpu_baseline(snap, batch, fwk, C, args.cpu_seconds)
        print(json.dumps(out), flush=True)
    ctx.close()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

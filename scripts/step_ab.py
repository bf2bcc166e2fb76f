#!/usr/bin/env python3
"""Step-time A/B of tuning knobs (a -DKAD_TUNING build, ablibs/libkad_tune.so: scripts/wide_exp.py --build) on one
workload, variants alternating within one process so that box-to-box spread cancels.

    python scripts/step_ab.py --config c3 --units 125000 --variants "base;KAD_ROWS_AFTER=1" [--rounds 3]

Each variant is ';'-separated, its knobs ','-separated NAME=VALUE pairs (tuning_env reads them per launch
for the knobs that are not cached; cached knobs need their own process — the script re-execs nothing).
Prints one JSON line: mean / min step ms per variant and rank-0 stage times."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--units", type=int, default=0)
    ap.add_argument("--variants", default="base")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--stages", action="store_true", help="also report mean per-stage times per variant")
    ap.add_argument("--lib", default=os.path.join(ROOT, "ablibs", "libkad_tune.so"))
    a = ap.parse_args()
    import torch  # noqa: F401

    import bench
    from kubeadmiral_amd import columns, runtime, synth
    from kubeadmiral_amd.pack import Snapshot

    runtime.load_library(a.lib)
    W0, C = synth.SIZES[a.config]
    clusters = bench.make_clusters(a.config, C)
    fwk = synth.profile_for(a.config)
    snap = Snapshot(clusters)
    batch = columns.NativePacker(snap).pack(fwk, bench.make_columns(a.config, 0, a.units or W0, clusters))
    ctx = runtime.Context(0)
    ctx.upload_snapshot(snap)
    ctx.upload_batch(batch)
    variants = [v.strip() for v in a.variants.split(";") if v.strip()]
    res = {v: [] for v in variants}
    stg = {}
    ref = None
    for r in range(a.rounds):
        for v in variants:
            env = {} if v == "base" else dict(kv.split("=") for kv in v.split(","))
            old = {k: os.environ.get(k) for k in env}
            os.environ.update(env)
            for _ in range(3):
                ctx.schedule(fwk)
            ctx.sync()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                ctx.schedule(fwk)
            ctx.sync()
            res[v].append((time.perf_counter() - t0) / a.steps * 1e3)
            if a.stages:  # per-stage HIP-event times of 3 more steps (timing on, outside the timed loop)
                ctx.set_timing(True)
                for _ in range(3):
                    ctx.schedule(fwk)
                    ctx.sync()
                    stg.setdefault(v, []).append(ctx.stage_timing())
                ctx.set_timing(False)
            out = ctx.download()
            if v == "base" and ref is None:
                ref = out
            elif ref is not None and not v.startswith("EXP"):
                assert out.equal_rows(ref).all(), f"variant {v} changed the results"
            for k, x in old.items():
                if x is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = x
    # a digest of the results (every unit's status / count / flags and its counted slots): equal across
    # libraries that schedule identically (a cross-library A/B's parity check)
    import hashlib

    st, cn = np.asarray(ref.status), np.asarray(ref.count)
    oo = np.asarray(ref.out_off)[: len(cn)]
    idx = np.repeat(oo, cn) + (np.arange(int(cn.sum())) - np.repeat(np.cumsum(cn) - cn, cn))
    h = hashlib.sha1()
    for x in (st, cn, np.asarray(ref.flags), np.asarray(ref.cluster)[idx], np.asarray(ref.replicas)[idx]):
        h.update(np.ascontiguousarray(x).tobytes())
    print(json.dumps({"config": a.config, "units": batch.W, "digest": h.hexdigest()[:16], "ms": {v: [round(x, 4) for x in xs] for v, xs in res.items()},
                      "mean": {v: round(float(np.mean(xs)), 4) for v, xs in res.items()},
                      "min": {v: round(float(np.min(xs)), 4) for v, xs in res.items()},
                      "stages": {v: {k: round(float(np.mean([d[k] for d in ds])), 4) for k in ds[0]} for v, ds in stg.items()}}),
          flush=True)


if __name__ == "__main__":
    main()

"""End-to-end probe (measurement only): where the pack -> upload -> schedule -> download time of one config
goes on the GPU box. Packer / upload laps come from KAD_PACK_TIMING / KAD_UPLOAD_TIMING (stderr); this script
times pageable vs page-locked downloads and the pipelined variants (chunks x packer threads).
    python scripts/e2e_prof.py --config c3 [--units N] --out gpurun_out/e2e.json"""
import argparse
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import bench  # noqa: E402
from kubeadmiral_amd import columns as CO  # noqa: E402
from kubeadmiral_amd import pack, synth  # noqa: E402
from kubeadmiral_amd import build as kbuild, runtime  # noqa: E402

# the packer / upload laps (KAD_PACK_TIMING / KAD_UPLOAD_TIMING) are compiled into measurement builds only
TUNE_LIB = os.path.join(os.path.dirname(kbuild.HERE), "ablibs", "libkad_tune.so")
kbuild.build(extra=["-DKAD_TUNING"], out=TUNE_LIB)
runtime.load_library(TUNE_LIB)
from kubeadmiral_amd.results import BatchResult  # noqa: E402
from kubeadmiral_amd.runtime import Context  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--units", type=int, default=0)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    W0, C = synth.SIZES[a.config]
    W = a.units or W0
    fwk = synth.profile_for(a.config)
    clusters = bench.make_clusters(a.config, C)
    snap = pack.Snapshot(clusters)
    cols = bench.make_columns(a.config, 0, W, clusters)
    ctx = Context(0)
    ctx.upload_snapshot(snap)
    packer = CO.NativePacker(snap)
    out = {"config": a.config, "units": W, "clusters": C, "threads": CO.default_threads(), "seq": [], "pipe": []}
    pinned = None
    for rep in range(a.reps):
        print(f"--- sequential rep {rep}", file=sys.stderr, flush=True)
        t0 = time.perf_counter()
        nb = packer.pack(fwk, cols, take=False)
        t1 = time.perf_counter()
        ctx.upload_batch(nb)
        ctx.sync()
        t2 = time.perf_counter()
        ctx.schedule(fwk)
        ctx.sync()
        t3 = time.perf_counter()
        r_pageable = ctx.download()
        t4 = time.perf_counter()
        if pinned is None:
            pinned = BatchResult.pinned(nb.W, max(1, nb.n_out_slots))
        t5 = time.perf_counter()
        r_pinned = ctx.download(out=pinned)
        t6 = time.perf_counter()
        assert r_pinned.equal_rows(r_pageable).all()
        out["seq"].append({"pack_ms": (t1 - t0) * 1e3, "upload_ms": (t2 - t1) * 1e3, "schedule_ms": (t3 - t2) * 1e3,
                           "d2h_pageable_ms": (t4 - t3) * 1e3, "d2h_pinned_ms": (t6 - t5) * 1e3,
                           "blob_mb": nb.blob.nbytes / 1e6, "n_out_slots": nb.n_out_slots})
        print(json.dumps(out["seq"][-1]), file=sys.stderr, flush=True)
    os.environ.pop("KAD_PACK_TIMING", None)
    ctx2 = Context(0)
    ctx2.upload_snapshot(snap)
    ctxs = (ctx, ctx2)
    packers = (packer, CO.NativePacker(snap))
    for chunks in (2, 4, 8):
        bounds = [W * i // chunks for i in range(chunks + 1)]
        parts = [cols.slice(bounds[i], bounds[i + 1]) for i in range(chunks)]
        for threads in (0, max(1, CO.default_threads() - 2)):
            bufs = None
            with ThreadPoolExecutor(max_workers=1) as pool:
                for rep in range(2):
                    outs = []
                    t0 = time.perf_counter()
                    fut = pool.submit(packers[0].pack, fwk, parts[0], threads, False)
                    t_wait = 0.0
                    for i in range(chunks):
                        tw = time.perf_counter()
                        nbi = fut.result()
                        t_wait += time.perf_counter() - tw
                        if i + 1 < chunks:
                            fut = pool.submit(packers[(i + 1) % 2].pack, fwk, parts[i + 1], threads, False)
                        c = ctxs[i % 2]
                        c.upload_batch(nbi)
                        c.schedule(fwk)
                        r = c.download(out=bufs[i] if bufs else None)
                        outs.append(r)
                    tot = time.perf_counter() - t0
                    if bufs is None:
                        bufs = [BatchResult.pinned(len(r.status), len(r.cluster)) for r in outs]
            rec = {"chunks": chunks, "threads": threads, "total_ms": tot * 1e3, "wait_pack_ms": t_wait * 1e3,
                   "decisions_per_s": W * C / tot}
            out["pipe"].append(rec)
            print(json.dumps(rec), file=sys.stderr, flush=True)
    ctx2.close()
    ctx.close()
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()

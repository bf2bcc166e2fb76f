#!/usr/bin/env python3
"""Per-unit timeline of the wide kernel (profiling build, GPU only): for every unit of the last launch its
realtime start (100 MHz), duration, feasible count, straddle flag and global wave, saved as .npz for
offline analysis of the kernel's tail (which units run last, how long, on which waves).

    python scripts/unit_trace.py --build                      # CPU side: ablibs/libkad_prof.so
    python scripts/unit_trace.py --units 125000 --out gpurun_out/utrace_125k.npz
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from kubeadmiral_amd import build as kbuild  # noqa: E402

PROF_LIB = os.environ.get("KAD_PROF_LIB", os.path.join(os.path.dirname(kbuild.HERE), "ablibs", "libkad_prof.so"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--units", type=int, default=0)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default="gpurun_out/utrace.npz")
    ap.add_argument("--build", action="store_true")
    a = ap.parse_args()
    if a.build:
        kbuild.build(force=True, extra=["-DKAD_PHASE_PROF"], out=PROF_LIB)
        return
    import ctypes

    import torch  # noqa: F401

    import bench
    from kubeadmiral_amd import columns, runtime, synth
    from kubeadmiral_amd.pack import Snapshot

    L = runtime.load_library(PROF_LIB)
    L.kad_debug_phase_counters.argtypes = [ctypes.c_void_p, ctypes.c_int]
    W0, C = synth.SIZES[a.config]
    W = a.units or W0
    clusters = bench.make_clusters(a.config, C)
    fwk = synth.profile_for(a.config)
    snap = Snapshot(clusters)
    batch = columns.NativePacker(snap).pack(fwk, bench.make_columns(a.config, 0, W, clusters))
    ctx = runtime.Context(0)
    ctx.upload_snapshot(snap)
    ctx.upload_batch(batch)
    out = {}
    for r in range(a.reps):
        ctx.schedule(fwk)
        ctx.sync()
        st = np.zeros(1 << 20, np.uint64)
        inf = np.zeros(1 << 20, np.uint64)
        assert L.kad_debug_phase_counters(st.ctypes.data, -3) > 0
        assert L.kad_debug_phase_counters(inf.ctypes.data, -4) > 0
        wt = np.zeros(8192 * 2, np.uint64)
        L.kad_debug_phase_counters(wt.ctypes.data, -1)
        out[f"start{r}"] = st[:W]
        out[f"info{r}"] = inf[:W]
        out[f"wavetime{r}"] = wt
    res = ctx.download()
    out["status"] = res.status
    out["count"] = res.count
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    np.savez_compressed(a.out, **out)
    print(f"saved {a.out}: {W} units x {a.reps} launches", flush=True)


if __name__ == "__main__":
    main()

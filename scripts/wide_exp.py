#!/usr/bin/env python3
"""Measurement-only variants of the wide kernel (KAD_WIDE_EXPERIMENT bits, a -DKAD_TUNING build): how much
of its time and of its instruction counts each phase costs. Results differ from the reference under any
bit; the product library ignores the variable.

    python scripts/wide_exp.py --build                  # builds ablibs/libkad_tune.so (CPU ok)
    KAD_WIDE_EXPERIMENT=<bits> python scripts/wide_exp.py [--config c3] [--units N]
bits: 1 no pdqsort replay, 2 stop after the filters, 4 no selection, 8 no output pass."""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from kubeadmiral_amd import build as kbuild  # noqa: E402

TUNE_LIB = os.path.join(os.path.dirname(kbuild.HERE), "ablibs", "libkad_tune.so")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--units", type=int, default=0)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--build", action="store_true")
    a = ap.parse_args()
    if a.build:
        kbuild.build(force=True, extra=["-DKAD_TUNING"], out=TUNE_LIB)
        return
    import bench
    from kubeadmiral_amd import columns, runtime, synth
    from kubeadmiral_amd.pack import Snapshot

    runtime.load_library(TUNE_LIB)
    W0, C = synth.SIZES[a.config]
    clusters = bench.make_clusters(a.config, C)
    fwk = synth.profile_for(a.config)
    snap = Snapshot(clusters)
    batch = columns.NativePacker(snap).pack(fwk, bench.make_columns(a.config, 0, a.units or W0, clusters))
    ctx = runtime.Context(0)
    ctx.upload_snapshot(snap)
    ctx.upload_batch(batch)
    ctx.schedule(fwk)
    ctx.sync()
    ctx.set_timing(True)
    st = []
    for _ in range(a.reps):
        ctx.schedule(fwk)
        ctx.sync()
        st.append(ctx.stage_timing())
    out = {"config": a.config, "units": batch.W, "exp": int(os.environ.get("KAD_WIDE_EXPERIMENT", "0")),
           "stage_ms": {k: float(np.mean([s[k] for s in st])) for k in ctx.STAGES}}
    print(json.dumps(out))
    ctx.close()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Native pack time of a config's full batch (KAD_PACK_TIMING=1 prints the packer's phases).

    python scripts/pack_time.py c4
"""
import sys, time, os; sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import bench
from kubeadmiral_amd import build as kbuild, columns, runtime, synth
# the packer's phase laps (KAD_PACK_TIMING=1) are compiled into measurement builds only
TUNE_LIB = os.path.join(os.path.dirname(kbuild.HERE), "ablibs", "libkad_tune.so")
kbuild.build(extra=["-DKAD_TUNING"], out=TUNE_LIB)
runtime.load_library(TUNE_LIB)
from kubeadmiral_amd.pack import Snapshot
cfg = sys.argv[1] if len(sys.argv) > 1 else "c4"
W0, C = synth.SIZES[cfg]
clusters = bench.make_clusters(cfg, C)
fwk = synth.profile_for(cfg)
snap = Snapshot(clusters)
cols = bench.make_columns(cfg, 0, W0, clusters)
pk = columns.NativePacker(snap)
for _ in range(4):
    t0 = time.perf_counter(); b = pk.pack(fwk, cols, take=False); t1 = time.perf_counter()
    print("pack ms %.1f" % ((t1 - t0) * 1e3), flush=True)

"""Summarise rocprofv3 csv output (kernel stats + per-dispatch counters) for profiles/.

    python scripts/pmc_summary.py <rocprof out dir> <config> [--units W --clusters C --json profiles/pmc_<cfg>.json]

Per kernel: average duration (kernel-trace pass) and the average per dispatch of
every counter collected in the separate --pmc passes. HBM bytes per launch of the
filter/score/select stage (req_mask_kernel + prep_kernel + schedule_lean_kernel
+ schedule_kernel) follow MI355X_MICROARCH.md's HBM/rocprofv3 section:
FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE counts half the bytes
of wide coalesced streaming reads, so the read side is doubled (the same
correction for every read of the stage: an upper bound for its narrower
accesses), WRITE_SIZE is taken as is.
"""
import argparse
import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kubeadmiral_amd.build import source_hash  # noqa: E402

STAGE = ("req_mask_kernel", "req_row_kernel", "prep_kernel", "schedule_lean_kernel", "schedule_wide_kernel",
         "schedule_row_kernel", "schedule_kernel")
# the step's kernels (bench.py picks its roofline kernel among them by live HIP-event time)
STEP = STAGE + ("plan_hdr_kernel", "plan_pair_kernel", "plan_kernel")

ap = argparse.ArgumentParser()
ap.add_argument("out")
ap.add_argument("cfg")
ap.add_argument("--units", type=int, default=None)
ap.add_argument("--clusters", type=int, default=None)
ap.add_argument("--json", default=None)
a = ap.parse_args()

res = {"config": a.cfg, "kernels": {}}
for f in glob.glob(os.path.join(a.out, "trace", "**", "*kernel_stats.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        res["kernels"].setdefault(r["Name"], {})["avg_ns"] = float(r["AverageNs"])
        res["kernels"][r["Name"]]["calls"] = int(r["Calls"])
for f in glob.glob(os.path.join(a.out, "*", "**", "*counter_collection.csv"), recursive=True):
    acc = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in acc.items():
        for cn, vals in d.items():
            # one value per dispatch per counter (summed over dimensions by rocprofv3)
            res["kernels"].setdefault(k, {})[cn] = sum(vals) / max(1, len(vals))
stage_bytes = 0.0
stage_ns = 0.0
for k, d in res["kernels"].items():
    if "FETCH_SIZE" in d or "WRITE_SIZE" in d:
        d["hbm_bytes_raw"] = (d.get("FETCH_SIZE", 0) + d.get("WRITE_SIZE", 0)) * 1024
        d["hbm_bytes_corrected"] = (2 * d.get("FETCH_SIZE", 0) + d.get("WRITE_SIZE", 0)) * 1024
    if any(s in k for s in STAGE):
        stage_bytes += d.get("hbm_bytes_corrected", 0.0)
        stage_ns += d.get("avg_ns", 0.0)
res["stage"] = {"kernels": list(STAGE), "hbm_bytes_per_launch": stage_bytes, "avg_ns_sum": stage_ns}
# the longest kernel of the step: traffic and instruction counts per launch
main = {}
for k, d in res["kernels"].items():
    if any(m in k for m in STEP) and d.get("avg_ns", 0) > main.get("avg_ns", 0):
        main = dict(d, name=k)
if main:
    main["hbm_bytes_per_launch"] = main.get("hbm_bytes_corrected")
res["main_kernel"] = main
print(json.dumps(res, indent=1))
if a.json:
    with open(a.json, "w") as f:
        json.dump({"config": a.cfg, "units": a.units, "clusters": a.clusters, "src_hash": source_hash(),
                   "hbm_bytes_per_launch": stage_bytes, "stage_avg_ns_sum": stage_ns,
                   "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes; (2*FETCH_SIZE + WRITE_SIZE)"
                             " KiB per dispatch summed over the stage kernels (MI355X_MICROARCH.md HBM section)",
                   "main_kernel": res["main_kernel"], "kernels": res["kernels"]}, f, indent=1)

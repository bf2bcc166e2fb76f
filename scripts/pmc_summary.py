"""Summarise rocprofv3 csv output (kernel stats + per-dispatch counters) for profiles/."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

out, cfg = sys.argv[1], sys.argv[2]
res = {"config": cfg, "kernels": {}}
for f in glob.glob(os.path.join(out, "trace", "**", "*kernel_stats.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        res["kernels"].setdefault(r["Name"], {})["avg_ns"] = float(r["AverageNs"])
        res["kernels"][r["Name"]]["calls"] = int(r["Calls"])
for f in glob.glob(os.path.join(out, "*", "**", "*counter_collection.csv"), recursive=True):
    acc = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in acc.items():
        for cn, vals in d.items():
            # one value per dispatch per counter (summed over dimensions by rocprofv3)
            res["kernels"].setdefault(k, {})[cn] = sum(vals) / max(1, len(vals))
for k, d in res["kernels"].items():
    if "FETCH_SIZE" in d or "WRITE_SIZE" in d:
        d["hbm_bytes_raw"] = (d.get("FETCH_SIZE", 0) + d.get("WRITE_SIZE", 0)) * 1024
print(json.dumps(res, indent=1))

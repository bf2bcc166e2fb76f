#!/usr/bin/env python3
"""Per-step timeline of a rocprofv3 kernel trace: kernel durations, their overlap and the idle gaps between them.

    rocprofv3 --kernel-trace --output-format csv -d OUT -o run -- python bench.py --config c3 --units 125000 ...
    python scripts/timeline.py OUT [--last N] [--json out.json]

The trace's dispatches are grouped into steps (a step starts at each req_row_kernel / req_mask_kernel /
prep_kernel that follows a gap): per step, the span from the first start to the last end, each kernel's
duration and start offset, and the GPU-idle time inside the span (no kernel running on any queue). Reports
the median over the last N steps (the timed region of bench.py is its last K + timing passes).
"""
import argparse
import csv
import glob
import json
import os
import statistics as stats
import sys


def load(d):
    files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        sys.exit(f"no kernel_trace.csv under {d}")
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    return rows


def short(name):
    n = name.replace("void ", "").replace("kad::", "")
    return n.split("(")[0]


STEP_FIRST = ("req_row_kernel", "req_mask_kernel", "prep_kernel")


def steps(rows):
    """Split the dispatches into pipeline passes: each occurrence of the pipeline's first kernel starts one."""
    names = [short(n) for _, _, n in rows]
    first = next((k for k in STEP_FIRST if any(x.startswith(k) for x in names)), names[0])
    out, cur = [], []
    for r, sn in zip(rows, names):
        if sn.startswith(first) and cur:
            out.append(cur)
            cur = []
        cur.append(r)
    if cur:
        out.append(cur)
    return out


def analyse(step):
    t0 = min(s for s, _, _ in step)
    t1 = max(e for _, e, _ in step)
    # idle: span minus the union of kernel intervals
    iv = sorted((s, e) for s, e, _ in step)
    busy, cs, ce = 0, iv[0][0], iv[0][1]
    for s, e in iv[1:]:
        if s > ce:
            busy += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    busy += ce - cs
    ks = [{"kernel": short(n), "start_us": (s - t0) / 1e3, "dur_us": (e - s) / 1e3} for s, e, n in step]
    return {"span_us": (t1 - t0) / 1e3, "idle_us": (t1 - t0 - busy) / 1e3, "kernels": ks}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--last", type=int, default=10)
    ap.add_argument("--skip-last", type=int, default=0, help="passes after the timed region (bench: its timing passes)")
    ap.add_argument("--json")
    a = ap.parse_args()
    allr = load(a.dir)
    sel = steps(allr)
    sel = sel[:len(sel) - a.skip_last] if a.skip_last else sel
    sel = sel[-a.last:]
    st = [analyse(s) for s in sel]
    med = {"steps": len(st), "span_us": stats.median(x["span_us"] for x in st),
           "idle_us": stats.median(x["idle_us"] for x in st)}
    # per kernel position in the step: median start / duration
    n_k = min(len(x["kernels"]) for x in st)
    med["kernels"] = [{"kernel": st[-1]["kernels"][i]["kernel"],
                       "start_us": stats.median(x["kernels"][i]["start_us"] for x in st),
                       "dur_us": stats.median(x["kernels"][i]["dur_us"] for x in st)} for i in range(n_k)]
    # step-to-step period (start of step k+1 - start of step k) over the last steps
    starts = []
    for s in sel:
        starts.append(min(x[0] for x in s))
    if len(starts) > 1:
        med["period_us"] = stats.median((b - a_) / 1e3 for a_, b in zip(starts, starts[1:]))
    print(json.dumps(med, indent=1))
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"median": med, "steps": st}, f, indent=1)


if __name__ == "__main__":
    main()

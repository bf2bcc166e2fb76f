#!/usr/bin/env python3
"""Per-phase cycle breakdown of schedule_kernel (profiling build, GPU only).

    python scripts/phase_prof.py [--config c2] [--units N] [--build]

Builds ablibs/libkad_prof.so with -DKAD_PHASE_PROF (s_memtime at the
phase boundaries of each SchedulingUnit, summed with atomics), runs a few
launches of the config and prints mean cycles per unit per phase. The
instrumentation perturbs timing (s_memtime ≈ +11 % wave cycles); the
counters are shader-clock cycles of wall time per unit, including cycles
the wave waits while other waves issue: use them for the relative split.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from kubeadmiral_amd import build as kbuild  # noqa: E402

PROF_LIB = os.environ.get("KAD_PROF_LIB", os.path.join(os.path.dirname(kbuild.HERE), "ablibs", "libkad_prof.so"))
NAMES = ["A_filter", "B_score", "C_normalize", "D_select", "E_output", "n_straddle", "n_select", "sum_feasible",
         "D_select_straddle", "row_units", "lean_A_filter", "lean_B_score", "lean_D_select", "lean_E_output",
         "lean_n_straddle", "lean_D_select_straddle", "plan_P0_setup", "plan_P1_weights", "plan_P2_plan",
         "plan_P3_output", "row_compact", "plan_rows", "row_score", "row_normalize",
         "replay_setup", "replay_partition", "replay_pivot", "replay_insertion", "replay_n_partitions",
         "replay_sum_n", "row_select", "row_replay", "row_terms", "row_positions"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--units", type=int, default=0)
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    if a.build or not os.path.exists(PROF_LIB):
        kbuild.build(force=True, extra=["-DKAD_PHASE_PROF"], out=PROF_LIB)
        if a.build:
            return
    import bench
    from kubeadmiral_amd import columns, runtime, synth
    from kubeadmiral_amd.pack import Snapshot

    L = runtime.load_library(PROF_LIB)
    L.kad_debug_phase_counters.argtypes = [ctypes.c_void_p, ctypes.c_int]
    W0, C = synth.SIZES[a.config]
    clusters = bench.make_clusters(a.config, C)
    fwk = synth.profile_for(a.config)
    snap = Snapshot(clusters)
    # the bench's workload (columnar generator + native packer)
    batch = columns.NativePacker(snap).pack(fwk, bench.make_columns(a.config, 0, a.units or W0, clusters))
    ctx = runtime.Context(0)
    ctx.upload_snapshot(snap)
    ctx.upload_batch(batch)
    cnt = np.zeros(40, dtype=np.uint64)
    ctx.schedule(fwk)
    ctx.sync()
    L.kad_debug_phase_counters(cnt.ctypes.data, 1)
    for _ in range(a.reps):
        ctx.schedule(fwk)
        ctx.sync()
    L.kad_debug_phase_counters(cnt.ctypes.data, 1)
    W = batch.W * a.reps
    out = {"config": a.config, "units": batch.W, "reps": a.reps}
    # lean kernel wave lifetimes of the last launch (s_memtime): mean lifetime / kernel span, start / end spread
    wt = np.zeros(8192 * 2, dtype=np.uint64)
    if L.kad_debug_phase_counters(wt.ctypes.data, -1) > 0:
        st, en = wt[0::2].astype(np.int64), wt[1::2].astype(np.int64)
        live = np.nonzero(en > 0)[0]
        if len(live):
            # s_memrealtime (100 MHz, device-wide); also split by XCD (4-wave blocks round-robin over 8 XCDs)
            wpb = 16 if a.config == "c3" else 4  # wide kernel: 16-wave blocks; lean: 4
            xcd = (live // wpb) % 8
            span_all = float(en[live].max() - st[live].min())
            out["lean_span_us"] = span_all / 100.0
            out["lean_wave_lifetime_frac"] = round(float((en[live] - st[live]).mean()) / span_all, 3)
            out["lean_start_p50_p90_max_frac"] = [round(float(np.percentile(st[live] - st[live].min(), q)) / span_all, 3)
                                                  for q in (50, 90, 100)]
            out["lean_end_p10_p50_min_frac"] = [round(float(np.percentile(en[live] - st[live].min(), q)) / span_all, 3)
                                                for q in (10, 50, 0)]
            fr, ss, es = [], [], []
            for x in range(8):
                sel = live[xcd == x]
                if not len(sel):
                    continue
                s0, e0 = st[sel], en[sel]
                span = float(e0.max() - s0.min())
                fr.append(float((e0 - s0).mean()) / span)
                ss.append(float(s0.max() - s0.min()) / span)
                es.append(float(e0.max() - e0.min()) / span)
            out["lean_waves"] = int(len(live))
            wx = np.zeros(8192 * 6, dtype=np.uint64)
            if a.config == "c3" and L.kad_debug_phase_counters(wx.ctypes.data, -2) > 0:
                # wide kernel: late waves (last 10 % of ends) vs the rest — units, longest unit, last dequeue
                units, umax, deq = wx[0::6].astype(np.int64), wx[1::6].astype(np.int64), wx[2::6].astype(np.int64)
                hwid, xcc = wx[4::6].astype(np.int64), wx[5::6].astype(np.int64)
                # per CU (XCC, SE, SH, CU from HW_ID): the CU's last wave end and its waves' mean end
                cu_key = (xcc[live] & 0xF) * 4096 + ((hwid[live] >> 13) & 7) * 512 + ((hwid[live] >> 12) & 1) * 16 + \
                    ((hwid[live] >> 8) & 15)
                endf_all = (en[live] - st[live].min()) / span_all
                keys = np.unique(cu_key)
                cu_last = np.array([endf_all[cu_key == k].max() for k in keys])
                cu_mean = np.array([endf_all[cu_key == k].mean() for k in keys])
                out["wide_cus"] = int(len(keys))
                out["wide_cu_last_end_p10_p50_p90_max"] = [round(float(np.percentile(cu_last, q)), 3) for q in (10, 50, 90, 100)]
                out["wide_cu_mean_end_p10_p50_p90_max"] = [round(float(np.percentile(cu_mean, q)), 3) for q in (10, 50, 90, 100)]
                out["wide_cu_of_last_wave"] = int(keys[np.argmax(cu_last)])
                out["wide_xcc_last_end"] = [round(float(endf_all[(xcc[live] & 0xF) == x].max()), 3) for x in range(8)]
                endf = (en[live] - st[live].min()) / span_all
                late = live[endf >= np.percentile(endf, 90)]
                rest = live[endf < np.percentile(endf, 90)]
                for nm, sel in (("late", late), ("rest", rest)):
                    out[f"wide_{nm}_units_mean"] = round(float(units[sel].mean()), 2)
                    out[f"wide_{nm}_maxunit_cycles_mean"] = round(float(umax[sel].mean()), 1)
                    out[f"wide_{nm}_last_dequeue_frac_mean"] = round(float((deq[sel] - st[live].min()).mean()) / span_all, 3)
                    out[f"wide_{nm}_end_frac_mean"] = round(float((en[sel] - st[live].min()).mean()) / span_all, 3)
                out["wide_units_p10_p50_p90"] = [int(np.percentile(units[live], q)) for q in (10, 50, 90)]
                out["wide_end_frac_hist10"] = np.histogram(endf, bins=10, range=(0, 1))[0].tolist()
            out["lean_wave_lifetime_frac_per_xcd"] = [round(v, 3) for v in fr]
            out["lean_start_spread_frac_per_xcd"] = [round(v, 3) for v in ss]
            out["lean_end_spread_frac_per_xcd"] = [round(v, 3) for v in es]
    if a.config == "c5" or os.environ.get("KAD_ROW_STAMPS"):
        # schedule_row_kernel blocks of the last launch (they overwrite the lean kernel's first slots): lifetime
        # over the row kernel's own span, and the end spread
        wt2 = np.zeros(8192 * 2, dtype=np.uint64)
        wx2 = np.zeros(8192 * 6, dtype=np.uint64)
        ctx.schedule(fwk)
        ctx.sync()
        L.kad_debug_phase_counters(wt2.ctypes.data, -1)
        L.kad_debug_phase_counters(wx2.ctypes.data, -2)
        nb = int(os.environ.get("KAD_ROW_BLOCKS", "512"))
        st2, en2 = wt2[0:2 * nb:2].astype(np.int64), wt2[1:2 * nb:2].astype(np.int64)
        ok = (en2 > st2)
        if ok.any():
            span = float(en2[ok].max() - st2[ok].min())
            out["row_blocks"] = int(ok.sum())
            out["row_span_us"] = span / 100.0
            out["row_block_lifetime_frac"] = round(float((en2[ok] - st2[ok]).mean()) / span, 3)
            out["row_block_end_p10_p50_p90_frac"] = [round(float(np.percentile(en2[ok] - st2[ok].min(), q)) / span, 3)
                                                     for q in (10, 50, 90)]
            out["row_block_units_p10_p50_p90"] = [int(np.percentile(wx2[0:6 * nb:6][ok], q)) for q in (10, 50, 90)]
    for i, nm in enumerate(NAMES):
        v = float(cnt[i])
        if nm == "-":
            continue
        if nm.startswith("plan_P"):
            out[nm + "_cycles_per_row"] = round(v / max(1.0, float(cnt[21])), 1)
            continue
        if nm.startswith("row_") and nm != "row_units":  # per unit of schedule_row_kernel
            out[nm + "_cycles_per_row"] = round(v / max(1.0, float(cnt[9])), 1)
            continue
        if nm.startswith("replay_"):  # per straddling unit (wide kernel)
            out[nm + "_per_straddle"] = round(v / max(1.0, float(cnt[14])), 1)
            continue
        if nm.startswith(("A_", "B_", "C_", "D_", "E_", "lean_A", "lean_B", "lean_D", "lean_E")):
            out[nm + "_cycles_per_unit"] = round(v / W, 1)
        else:
            out[nm + "_per_unit"] = round(v / W, 4)
    print(json.dumps(out, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()

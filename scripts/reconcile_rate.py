#!/usr/bin/env python3
"""Objects per second through BatchReconciler.reconcile and reconcile_texts (f1: policy lookup, trigger hashes on the GPU, units,
one packed batch per framework, schedule, result application), with the native object path
(include/kad_objects.h) and with objects.py, on synth.gen_trigger_workload objects. GPU required.

    python scripts/reconcile_rate.py [--objects 20000] [--clusters 64] [--out file.json]
"""
import argparse
import copy
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--objects", type=int, default=20000)
    ap.add_argument("--clusters", type=int, default=64)
    ap.add_argument("--out", default="")
    ap.add_argument("--profile", default="", help="cProfile the native first pass into this file (top functions)")
    ap.add_argument("--profile-texts", default="", help="cProfile the texts first pass into this file")
    a = ap.parse_args()
    import numpy as np

    from kubeadmiral_amd import synth
    from kubeadmiral_amd.controller import BatchReconciler

    ftc, clusters, objs0, pols = synth.gen_trigger_workload(np.random.default_rng(5), a.objects, a.clusters,
                                                            n_policies=16)
    by_key = {}
    for p in pols:
        if p.spec.auto_migration is not None:
            p.spec.auto_migration.when.pod_unschedulable_for = "2m"
        by_key[(p.namespace, p.name)] = p
    out = {"objects": a.objects, "clusters": a.clusters}
    results = {}
    for native in (True, False):
        rec = BatchReconciler(ftc, native_objects=native)
        objs = copy.deepcopy(objs0)
        t0 = time.perf_counter()
        if a.profile and native:
            import cProfile
            import pstats
            pr = cProfile.Profile()
            pr.enable()
        got = rec.reconcile(objs, by_key, clusters)  # first pass: every object is scheduled and applied
        t1 = time.perf_counter()
        if a.profile and native:
            pr.disable()
            with open(a.profile, "w") as f:
                pstats.Stats(pr, stream=f).sort_stats("tottime").print_stats(25)
        again = rec.reconcile(objs, by_key, clusters)  # second pass: every trigger hash unchanged
        t2 = time.perf_counter()
        name = "native" if native else "python"
        stages = {}
        for g in got:
            stages[g.stage] = stages.get(g.stage, 0) + 1
        out[name] = {"first_pass_objects_per_s": round(a.objects / (t1 - t0)),
                     "unchanged_pass_objects_per_s": round(a.objects / (t2 - t1)), "stages": stages,
                     "unchanged": sum(g.stage == "unchanged" for g in again)}
        results[name] = (objs, [(g.stage, g.result) for g in got])
        print(json.dumps({name: out[name]}), flush=True)
    out["same_outcome"] = results["native"][1] == results["python"][1] and results["native"][0] == results["python"][0]

    # the reconcile over the objects' JSON texts (reconcile_texts: every per-object step native)
    from kubeadmiral_amd import objects as O

    texts = [json.dumps(o).encode() for o in objs0]
    ptexts = [json.dumps(O.policy_to_json(p)) for p in by_key.values()]  # the informer's policies, once each
    rec = BatchReconciler(ftc)
    if a.profile_texts:
        import cProfile
        import pstats
        pr = cProfile.Profile()
        pr.enable()
    t0 = time.perf_counter()
    got, new = rec.reconcile_texts(texts, ptexts, clusters)
    t1 = time.perf_counter()
    if a.profile_texts:
        pr.disable()
        with open(a.profile_texts, "w") as f:
            pstats.Stats(pr, stream=f).sort_stats("tottime").print_stats(30)
    again, _ = rec.reconcile_texts([n if n is not None else t for n, t in zip(new, texts)], ptexts, clusters)
    t2 = time.perf_counter()
    stages = {}
    for g in got:
        stages[g.stage] = stages.get(g.stage, 0) + 1
    out["texts"] = {"first_pass_objects_per_s": round(a.objects / (t1 - t0)),
                    "unchanged_pass_objects_per_s": round(a.objects / (t2 - t1)), "stages": stages,
                    "unchanged": sum(g.stage == "unchanged" for g in again)}
    out["texts_same_outcome"] = ([(g.stage, g.result) for g in got] == results["python"][1] and
                                 all(json.loads(n) == o for n, o in zip(new, results["python"][0]) if n is not None))
    print(json.dumps({"texts": out["texts"]}), flush=True)
    print(json.dumps(out), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Host rates of the f2 / f3 / f4 object paths (no GPU): native kad_units_from_objects / kad_apply_results /
kad_trigger_prefixes vs the Python restatement (objects.py), on seeded federated objects of tests/test_native_objects.py's generator.

    python scripts/objects_rate.py [--objects 100000] [--threads 16] [--out file.json]
"""
import argparse
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--objects", type=int, default=100000)
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--python-sample", type=int, default=5000)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import test_native_objects as t
    from kubeadmiral_amd import columns as K

    rng = random.Random(5)
    policies = [t._policy(rng, f"p{i}", False) for i in range(8)]
    objs = [t._object(rng, policies) for _ in range(a.objects)]
    texts = [json.dumps(o, separators=(",", ":")).encode() for o in objs]
    off, cl, rep = t._results(rng, len(objs))
    fol, th = [True] * len(objs), [None] * len(objs)
    out = {"objects": a.objects, "bytes_per_object": round(sum(map(len, texts)) / len(texts), 1),
           "threads": a.threads or K.default_threads()}
    K.units_from_objects(t.DEPLOY, texts[:1000], policies, threads=a.threads)  # pool warm-up
    for name, fn in (("units", lambda: K.units_from_objects(t.DEPLOY, texts, policies, threads=a.threads)),
                     ("apply", lambda: K.apply_results(t.DEPLOY, texts, t.NAMES, off, cl, rep, fol, th,
                                                        threads=a.threads)),
                     ("trigger_prefixes", lambda: K.trigger_prefixes(t.DEPLOY, texts, policies, threads=a.threads))):
        best = 1e9
        for _ in range(3):
            t0 = time.perf_counter()
            fn()
            best = min(best, time.perf_counter() - t0)
        out[f"native_{name}_objects_per_s"] = round(a.objects / best)
    n = min(a.python_sample, a.objects)
    t0 = time.perf_counter()
    t.python_units(t.DEPLOY, texts[:n], policies)
    out["python_units_objects_per_s"] = round(n / (time.perf_counter() - t0))
    t0 = time.perf_counter()
    t.python_apply(t.DEPLOY, texts[:n], off[:n + 1], cl, rep, fol, th)
    out["python_apply_objects_per_s"] = round(n / (time.perf_counter() - t0))
    # objects.py's trigger prefix from the decoded objects (policy lookup as the reconcile does it)
    from kubeadmiral_amd import objects as O

    pols = {}
    for p in policies:
        try:
            pols[(p["metadata"].get("namespace", ""), p["metadata"]["name"])] = O.PropagationPolicy.from_json(p)
        except Exception:  # noqa: BLE001
            pass
    t0 = time.perf_counter()
    for x in texts[:n]:
        o = json.loads(x)
        key = O.matched_policy_key(o, t.DEPLOY.namespaced)
        try:
            O.trigger_prefix(t.DEPLOY, o, pols.get(key) if key else None)
        except O.ObjectError:
            pass
    out["python_trigger_prefixes_objects_per_s"] = round(n / (time.perf_counter() - t0))
    print(json.dumps(out), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()

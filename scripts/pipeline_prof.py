#!/usr/bin/env python3
"""Where the pipelined end-to-end time goes (bench.py end_to_end): the pack of the whole batch vs its chunks,
two packers at once, and (GPU present) the pipelined loop with per-phase timestamps.

    python scripts/pipeline_prof.py [--cfg c4] [--chunks 4] [--out file.json]
"""
import argparse
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", default="c4")
    ap.add_argument("--chunks", type=int, default=4)
    ap.add_argument("--units", type=int, default=0)
    ap.add_argument("--workers", type=int, default=1, help="chunk packs in flight in the pipelined loop")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import bench
    from kubeadmiral_amd import columns as CO
    from kubeadmiral_amd import pack, synth

    W, C = synth.SIZES[a.cfg]
    W = a.units or W
    fwk = synth.profile_for(a.cfg)
    clusters = bench.make_clusters(a.cfg, C)
    snap = pack.Snapshot(clusters)
    cols = bench.make_columns(a.cfg, 0, W, clusters)
    out = {"cfg": a.cfg, "units": W, "chunks": a.chunks}
    p1, p2 = CO.NativePacker(snap), CO.NativePacker(snap)
    bounds = [W * i // a.chunks for i in range(a.chunks + 1)]
    parts = [cols.slice(bounds[i], bounds[i + 1]) for i in range(a.chunks)]

    def t(f, reps=3):
        best = 1e9
        for _ in range(reps):
            t0 = time.perf_counter()
            f()
            best = min(best, time.perf_counter() - t0)
        return best * 1e3

    p1.pack(fwk, cols, take=False)
    p2.pack(fwk, cols, take=False)
    out["pack_whole_ms"] = t(lambda: p1.pack(fwk, cols, take=False))
    out["slice_ms"] = t(lambda: [cols.slice(bounds[i], bounds[i + 1]) for i in range(a.chunks)])
    out["pack_chunks_seq_ms"] = t(lambda: [p1.pack(fwk, p, 0, False) for p in parts])
    out["pack_chunk_ms"] = [t(lambda p=p: p1.pack(fwk, p, 0, False)) for p in parts]

    def two():
        with ThreadPoolExecutor(max_workers=2) as ex:
            f1 = ex.submit(lambda: [p1.pack(fwk, p, 0, False) for p in parts[0::2]])
            f2 = ex.submit(lambda: [p2.pack(fwk, p, 0, False) for p in parts[1::2]])
            f1.result()
            f2.result()
    out["pack_chunks_two_packers_ms"] = t(two)
    print(json.dumps(out), flush=True)

    from kubeadmiral_amd.results import BatchResult
    from kubeadmiral_amd.runtime import Context

    try:
        ctxs = (Context(0), Context(0))
    except Exception as e:  # noqa: BLE001 — no GPU here: the pack numbers alone
        print(f"no device: {e}", flush=True)
        ctxs = None
    if ctxs is not None:
        for c in ctxs:
            c.upload_snapshot(snap)
        nb = p1.pack(fwk, cols, take=False)
        ctxs[0].upload_batch(nb)
        ctxs[0].sync()
        ts = {}
        t0 = time.perf_counter()
        ctxs[0].upload_batch(nb)
        ctxs[0].sync()
        ts["h2d_whole_ms"] = (time.perf_counter() - t0) * 1e3
        t0 = time.perf_counter()
        ctxs[0].schedule(fwk)
        ctxs[0].sync()
        ts["schedule_whole_ms"] = (time.perf_counter() - t0) * 1e3
        t0 = time.perf_counter()
        ctxs[0].download()
        ts["d2h_whole_ms"] = (time.perf_counter() - t0) * 1e3
        out.update(ts)
        packers = [p1, p2] + [CO.NativePacker(snap) for _ in range(a.workers - 1)]
        for pk in packers[2:]:
            pk.pack(fwk, parts[0], 0, False)
        bufs = None
        out["workers"] = a.workers
        with ThreadPoolExecutor(max_workers=a.workers) as pool:
            for rep in range(3):
                ev = []
                t0 = time.perf_counter()

                def stamp(name, i):
                    ev.append((name, i, round((time.perf_counter() - t0) * 1e3, 3)))

                def packj(i):
                    stamp("pack_start", i)
                    r = packers[i % len(packers)].pack(fwk, parts[i], 0, False)
                    stamp("pack_end", i)
                    return r
                futs = {i: pool.submit(packj, i) for i in range(min(a.workers, a.chunks))}
                outs = []
                for i in range(a.chunks):
                    nbi = futs.pop(i).result()
                    if i + a.workers < a.chunks:
                        futs[i + a.workers] = pool.submit(packj, i + a.workers)
                    c = ctxs[i % 2]
                    stamp("upload_start", i)
                    c.upload_batch(nbi)
                    stamp("upload_end", i)
                    c.schedule(fwk)
                    stamp("schedule_queued", i)
                    r = c.download(out=bufs[i] if bufs else None)
                    stamp("download_end", i)
                    outs.append(r)
                tot = (time.perf_counter() - t0) * 1e3
                if bufs is None:
                    bufs = [BatchResult.pinned(len(r.status), len(r.cluster)) for r in outs]
                out[f"pipelined_rep{rep}"] = {"total_ms": round(tot, 3), "events": ev}
                print(json.dumps({f"pipelined_rep{rep}": out[f"pipelined_rep{rep}"]}), flush=True)
        for c in ctxs:
            c.close()
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()

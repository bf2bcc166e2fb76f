"""Native batch packer (include/kad_pack.h, libkad.so kad_pack_batch) against the Python packer.

The Python packer (kubeadmiral_amd/pack.py) is pinned to the object-level oracle by
tests/test_c_oracle.py; the native packer must produce the SAME blob byte for byte
(interning order, programs, CSR rows, toleration masks, output bounds) on every
fuzz batch and on samples of every config's generator, for every fuzz profile.
Host code only: runs on CPU (libkad.so loads without a GPU).
"""

import numpy as np
import pytest

from kubeadmiral_amd import columns as CO
from kubeadmiral_amd import framework as F
from kubeadmiral_amd import pack, synth
from kubeadmiral_amd import types as T


@pytest.fixture(scope="module", autouse=True)
def _lib():
    from kubeadmiral_amd import build
    build.build()


def _same(snap, fwk, units, threads=0):
    want = pack.Batch(snap, fwk, units)
    got = CO.NativePacker(snap).pack(fwk, CO.from_units(units), threads=threads)
    assert got.blob.nbytes == want.blob.nbytes
    if not np.array_equal(got.blob, want.blob):
        hw, hg = pack.header_of(want.blob, pack.BatchHeader), pack.header_of(got.blob, pack.BatchHeader)
        diff = [i for i in range(pack.B_NARRAYS)
                if not np.array_equal(pack.array_of(want.blob, hw, i, np.uint8), pack.array_of(got.blob, hg, i, np.uint8))]
        raise AssertionError(f"blobs differ in arrays {diff}")
    assert np.array_equal(got.n_reqs, want.n_reqs) and np.array_equal(got.n_tols, want.n_tols)
    assert got.n_distinct_reqs == want.n_distinct_reqs
    return got


@pytest.mark.parametrize("seed", range(60))
def test_fuzz_blob_identical(seed):
    clusters, units = synth.gen_fuzz(seed, W=70)
    _same(pack.Snapshot(clusters), synth.fuzz_framework(seed), units, threads=1 + seed % 4)


@pytest.mark.parametrize("cfg,W,C", [("c1", 600, 16), ("c2", 5000, 256), ("c3", 3000, 1000), ("c4", 2500, 512),
                                     ("c5", 400, 2000)])
def test_config_samples_blob_identical(cfg, W, C):
    clusters, units, fwk = synth.make_config(cfg, W=W, C=C)
    _same(pack.Snapshot(clusters), fwk, units)


@pytest.mark.parametrize("prof", range(len(synth.FUZZ_PROFILES)))
def test_profiles_change_output_bounds(prof):
    clusters, units = synth.gen_fuzz(900 + prof, W=120, C=30)
    _same(pack.Snapshot(clusters), synth.fuzz_framework(prof), units)


def test_threads_do_not_change_the_blob():
    clusters, units = synth.gen_fuzz(4242, W=6000, C=50)
    snap = pack.Snapshot(clusters)
    fwk = F.Framework()
    cols = CO.from_units(units)
    P = CO.NativePacker(snap)
    blobs = [P.pack(fwk, cols, threads=t).blob for t in (1, 2, 3, 8)]
    assert all(np.array_equal(blobs[0], b) for b in blobs[1:])


def test_concurrent_packers_share_the_worker_pool():
    """Packs from several host threads at once (a Go shim's goroutines): every packer's parallel loops go
    through libkad's one persistent worker pool (csrc/kad_pool.h), one job at a time, and each blob stays
    byte-identical to a serial pack of the same units — no deadlock, no cross-talk between jobs."""
    from concurrent.futures import ThreadPoolExecutor

    clusters, units = synth.gen_fuzz(4343, W=8000, C=60)
    snap = pack.Snapshot(clusters)
    fwk = F.Framework()
    parts = [CO.from_units(units[i::4]) for i in range(4)]
    want = [CO.NativePacker(snap).pack(fwk, p, threads=1).blob.copy() for p in parts]

    def job(i):
        P = CO.NativePacker(snap)
        out = []
        for _ in range(3):
            out.append(P.pack(fwk, parts[i], threads=0).blob.copy())
        return out

    with ThreadPoolExecutor(max_workers=4) as ex:
        got = list(ex.map(job, range(4)))
    for i in range(4):
        for b in got[i]:
            assert np.array_equal(b, want[i])


def test_pack_after_fork_in_the_child():
    """The worker pool is per process (kad_pool.h): a child forked after the parent's pool exists packs with a
    fresh pool (its parent's workers do not exist in it) — the same blob, no hang. Forked while another
    thread of the parent is packing, too (that thread's locks are not the child's)."""
    import os
    import threading

    clusters, units = synth.gen_fuzz(4545, W=9000, C=40)
    snap = pack.Snapshot(clusters)
    fwk = F.Framework()
    cols = CO.from_units(units)
    want = CO.NativePacker(snap).pack(fwk, cols, threads=8).blob.copy()  # the pool now exists
    stop = threading.Event()

    def busy():
        P = CO.NativePacker(snap)
        while not stop.is_set():
            P.pack(fwk, cols, threads=8)

    t = threading.Thread(target=busy)
    t.start()
    try:
        for _ in range(3):
            r, w = os.pipe()
            pid = os.fork()
            if pid == 0:  # child: pack twice, report, leave without running the parent's atexit handlers
                ok = 1
                try:
                    for _ in range(2):
                        ok &= int(np.array_equal(CO.NativePacker(snap).pack(fwk, cols, threads=8).blob, want))
                finally:
                    os.write(w, bytes([ok]))
                    os._exit(0)
            os.close(w)
            import select
            ready, _, _ = select.select([r], [], [], 60)
            assert ready, "child packer hung after fork"
            assert os.read(r, 1) == b"\x01"
            os.close(r)
            os.waitpid(pid, 0)
    finally:
        stop.set()
        t.join()


def test_in_place_batch_is_refused_once_stale():
    """pack(take=False) returns the packer's own buffer: the batch keeps the packer alive, and a batch the
    packer has since overwritten (or freed by close) is refused before any upload."""
    import gc

    clusters, units = synth.gen_fuzz(4646, W=300, C=20)
    snap = pack.Snapshot(clusters)
    fwk = F.Framework()
    cols = CO.from_units(units)
    want = CO.NativePacker(snap).pack(fwk, cols).blob.copy()
    P = CO.NativePacker(snap)
    nb = P.pack(fwk, cols, take=False)
    nb.check_current()
    del P
    gc.collect()
    assert np.array_equal(nb.blob, want)  # still the packer's live buffer
    P = nb.in_place[0]
    nb2 = P.pack(fwk, cols, take=False)
    nb2.check_current()
    with pytest.raises(ValueError, match="packed another batch"):
        nb.check_current()
    P.close()
    with pytest.raises(ValueError, match="closed"):
        nb2.check_current()


def test_download_refuses_wrong_dtypes():
    """kad_results_download writes 4 / 8 bytes per element: a caller buffer of another dtype is refused
    before the copy (checked on the host, no GPU needed)."""
    from kubeadmiral_amd import results, runtime

    clusters, units = synth.gen_fuzz(4747, W=50, C=20)
    snap = pack.Snapshot(clusters)
    fwk = F.Framework()
    nb = CO.NativePacker(snap).pack(fwk, CO.from_units(units))
    ctx = object.__new__(runtime.Context)
    ctx.h, ctx.batch = None, nb
    good = results.BatchResult.empty(nb)
    bad = results.BatchResult(good.status, good.count, good.flags, good.cluster, good.replicas.astype(np.int32),
                              good.out_off)
    with pytest.raises(ValueError, match="dtype"):
        ctx.download(out=bad)
    bad = results.BatchResult(good.status.astype(np.int16), good.count, good.flags, good.cluster, good.replicas,
                              good.out_off)
    with pytest.raises(ValueError, match="dtype"):
        ctx.download(out=bad)


def test_empty_batch():
    clusters, _ = synth.gen_fuzz(3, W=1, C=10)
    _same(pack.Snapshot(clusters), F.Framework(), [])


@pytest.mark.parametrize("seed", range(10))
def test_columns_round_trip(seed):
    """from_units -> to_units loses nothing the scheduler reads: the objects it gives back pack (through
    pack.py, the path pinned to the oracle) to the same blob as the originals, and a second round trip is
    the identity on the columns."""
    clusters, units = synth.gen_fuzz(seed, W=50)
    snap, fwk = pack.Snapshot(clusters), synth.fuzz_framework(seed)
    cols = CO.from_units(units)
    back = CO.to_units(cols)
    assert np.array_equal(pack.Batch(snap, fwk, back).blob, pack.Batch(snap, fwk, units).blob)
    again = CO.from_units(back)
    assert np.array_equal(again.str_off, cols.str_off) and np.array_equal(again.str_data, cols.str_data)
    assert all(np.array_equal(again.cols[k], cols.cols[k]) for k in cols.cols)


def test_columnar_generator_matches_its_objects():
    """synth.gen_units_c2_columns (the bench's C2/C3 input) packs to the same blob natively and through
    pack.py from the objects it describes, and has the C2 distributions."""
    rng = np.random.default_rng(0xC3)
    clusters = synth.gen_clusters(rng, 1000)
    snap = pack.Snapshot(clusters)
    fwk = synth.profile_for("c3")
    cols = synth.gen_units_c2_columns(np.random.default_rng(7), 4000)
    units = CO.to_units(cols)
    got = CO.NativePacker(snap).pack(fwk, cols)
    assert np.array_equal(got.blob, pack.Batch(snap, fwk, units).blob)
    assert all(1 <= u.max_clusters <= 16 and 1 <= u.desired_replicas <= 100 for u in units)
    assert 0.45 < np.mean([u.cluster_selector is not None for u in units]) < 0.55
    assert all(len(u.affinity.cluster_affinity.required.cluster_selector_terms) == 1 for u in units)
    assert {len(u.tolerations or []) for u in units} == {0, 1, 2, 3}


def test_malformed_columns_are_rejected():
    _, units = synth.gen_fuzz(5, W=20, C=12)
    clusters, _ = synth.gen_fuzz(5, W=1, C=12)
    snap = pack.Snapshot(clusters)
    P = CO.NativePacker(snap)
    good = CO.from_units(units)
    P.pack(F.Framework(), good)
    for field, idx, val in (("name", 0, 10 ** 6), ("tol_off", 1, -1), ("rq_key", 0, -7), ("rt_req", 0, 10 ** 6),
                            ("sel_off", 0, 3)):
        if len(good.cols[field]) <= idx:
            continue
        bad = CO.SUColumns(good.n_units, good.str_off, good.str_data, dict(good.cols))
        bad.cols[field] = bad.cols[field].copy()
        bad.cols[field][idx] = val
        with pytest.raises(RuntimeError, match="kad_pack_batch"):
            P.pack(F.Framework(), bad)
    P.pack(F.Framework(), good)  # still usable


def _create(v):
    import ctypes

    from kubeadmiral_amd.runtime import load_library

    L = load_library()
    L.kad_packer_create.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p)]
    L.kad_packer_error.argtypes = [ctypes.c_void_p]
    L.kad_packer_error.restype = ctypes.c_char_p
    L.kad_packer_destroy.argtypes = [ctypes.c_void_p]
    h = ctypes.c_void_p()
    rc = L.kad_packer_create(ctypes.byref(v), ctypes.byref(h))
    if rc == 0:
        L.kad_packer_destroy(h)
        return rc, ""
    return rc, L.kad_packer_error(None).decode()


def _bad_vocab_cases():
    """(name, mutate(vocab, keep)) — each breaks one rule kad_packer_create checks."""
    import ctypes

    def offs(v, field, arr):
        a = np.asarray(arr, np.int64)
        v._keep.append(a)
        getattr(v, field).off = a.ctypes.data

    def voff(v, arr):
        a = np.asarray(arr, np.int32)
        v._keep.append(a)
        v.label_val_off = a.ctypes.data

    return [
        ("gvk_count", lambda v: setattr(v.gvk_version, "n", v.gvk_group.n - 1)),
        ("taint_count", lambda v: setattr(v.taint_effect, "n", v.taint_key.n - 1)),
        ("label_val_off_null", lambda v: setattr(v, "label_val_off", None)),
        ("label_val_off_start", lambda v: voff(v, [1] + [v.label_vals.n] * v.label_keys.n)),
        ("label_val_off_decreasing", lambda v: voff(v, [0, 3, 2] + [v.label_vals.n] * (v.label_keys.n - 2))),
        ("label_val_off_past_end", lambda v: voff(v, [0] * v.label_keys.n + [v.label_vals.n + 1])),
        ("strs_negative_n", lambda v: setattr(v.cluster_names, "n", -1)),
        ("strs_not_from_zero", lambda v: offs(v, "cluster_names", [5] + [9] * v.cluster_names.n)),
        ("strs_decreasing", lambda v: offs(v, "label_keys", [0, 4, 2] + [8] * (v.label_keys.n - 2))),
        ("strs_null_off", lambda v: setattr(v.taint_key, "off", ctypes.c_void_p(None))),
        ("taint_words", lambda v: setattr(v, "n_taint_words", 0)),
    ]


@pytest.mark.parametrize("case", [c[0] for c in _bad_vocab_cases()])
def test_packer_create_rejects_malformed_vocab(case):
    """the vocabulary from a cross-language caller is validated (KAD_EINVAL + message)."""
    clusters, units, fwk = synth.make_config("c5", W=4, C=64)
    snap = pack.Snapshot(clusters)
    assert snap.TW >= 1 and len(snap.label_key_id) >= 3 and len(snap.taint_defs) >= 1 and len(snap.gvk_id) >= 1
    keep = []
    v = CO.vocab_of(snap, keep)
    v._keep = keep
    assert _create(v) == (0, "")
    mutate = dict(_bad_vocab_cases())[case]
    mutate(v)
    rc, msg = _create(v)
    assert rc == -1 and msg, (case, rc, msg)


@pytest.mark.parametrize("cfg,W,C", [("c4", 1500, 512), ("c4", 400, 100), ("c5", 300, 1500)])
def test_columnar_generators_blob_identical(cfg, W, C):
    """synth.gen_units_c4_columns / gen_units_c5_columns (the bench's vectorised C4 / C5 generators): the
    native packer's blob equals the Python packer's on the same units (columns → objects → pack.Batch)."""
    rng = np.random.default_rng(C + W)
    if cfg == "c4":
        clusters = synth.gen_clusters(rng, C)
        cols = synth.gen_units_c4_columns(rng, W, [c.name for c in clusters])
    else:
        clusters = synth.gen_clusters(rng, C, n_keys=64, n_vals=16, n_int_keys=4, n_taints=256, taints_per=(4, 16),
                                      p_gvk=0.9, gvks=synth.GVKS)
        cols = synth.gen_units_c5_columns(rng, W, [c.name for c in clusters])
    units = CO.to_units(cols)
    snap = pack.Snapshot(clusters)
    fwk = synth.profile_for(cfg)
    want = pack.Batch(snap, fwk, units)
    got = CO.NativePacker(snap).pack(fwk, cols)
    assert np.array_equal(got.blob, want.blob)
    # the distributions the docstrings promise
    if cfg == "c4":
        k = np.diff(cols["place_off"])
        assert k.min() >= min(8, C) and k.max() <= 64
        assert all(len(u.cluster_names) == n for u, n in zip(units, k))  # distinct clusters
        assert 0.35 < np.mean([u.weights is not None for u in units]) < 0.65
        assert 0.15 < np.mean([u.current_clusters is not None for u in units]) < 0.35
    else:
        assert all(2 <= len(u.affinity.cluster_affinity.required.cluster_selector_terms) <= 8 for u in units)
        ops = {r.operator for u in units for t in u.affinity.cluster_affinity.required.cluster_selector_terms
               for r in (t.match_expressions or [])}
        assert {"In", "NotIn", "Exists", "DoesNotExist", "Gt", "Lt", "Bogus"} <= ops
        assert any(t.match_fields for u in units for t in u.affinity.cluster_affinity.required.cluster_selector_terms)


@pytest.mark.parametrize("threads", [1, 3, 8])
def test_shared_requirement_entries(threads):
    """Units whose terms reference the same requirement entries (the column format allows it): the parallel
    interning falls back to one chunk and the blob still equals the Python packer's."""
    clusters, units = synth.gen_fuzz(4321, W=60, C=20)
    fwk = synth.fuzz_framework(1)
    cols = CO.from_units(units)
    c = cols.cols
    # point every required term of the second half at the first term's entries of unit 0 (when it has one)
    r0 = int(c["rterm_off"][0])
    if int(c["rterm_off"][1]) > r0:
        for w in range(30, 60):
            for t in range(int(c["rterm_off"][w]), int(c["rterm_off"][w + 1])):
                c["rt_req"][t] = c["rt_req"][r0]
                c["rt_n_expr"][t] = c["rt_n_expr"][r0]
                c["rt_n_field"][t] = c["rt_n_field"][r0]
    snap = pack.Snapshot(clusters)
    want = pack.Batch(snap, fwk, CO.to_units(cols))
    got = CO.NativePacker(snap).pack(fwk, cols, threads=threads)
    assert np.array_equal(got.blob, want.blob)


@pytest.mark.parametrize("cfg,W,C", [("c3", 2000, 1000), ("c4", 900, 512), ("c5", 300, 1500)])
def test_columns_slice_packs_like_its_units(cfg, W, C):
    """SUColumns.slice (the pipelined pack's chunks): a chunk's blob equals the Python packer's blob of the
    same units."""
    import bench
    clusters = bench.make_clusters(cfg, C) if cfg != "c5" else synth.gen_clusters(
        np.random.default_rng(5), C, n_keys=64, n_vals=16, n_int_keys=4, n_taints=256, taints_per=(4, 16),
        p_gvk=0.9, gvks=synth.GVKS)
    cols = bench.make_columns(cfg, 0, W, clusters)
    snap = pack.Snapshot(clusters)
    fwk = synth.profile_for(cfg)
    units = CO.to_units(cols)
    for lo, hi in ((0, W // 3), (W // 3, W - 7), (W - 7, W)):
        part = cols.slice(lo, hi)
        got = CO.NativePacker(snap).pack(fwk, part)
        want = pack.Batch(snap, fwk, units[lo:hi])
        assert np.array_equal(got.blob, want.blob), (lo, hi)


@pytest.mark.parametrize("seed", range(8))
def test_wide_preference_values_blob_identical(seed):
    """Preference values past int32 keep the i64 columns (KAD_BATCH_NARROW_PREFS off); both packers agree on the
    layout and the bytes, and batches within int32 get the narrow columns."""
    clusters, units = synth.gen_fuzz(300 + seed, W=80)
    snap, fwk = pack.Snapshot(clusters), synth.fuzz_framework(seed)
    narrow = _same(snap, fwk, units)
    assert pack.header_of(narrow.blob, pack.BatchHeader).flags == pack.BATCH_NARROW_PREFS
    synth.widen_prefs(units, seed, share=0.5)
    wide = _same(snap, fwk, units)
    assert pack.header_of(wide.blob, pack.BatchHeader).flags == 0
    assert wide.blob.nbytes > narrow.blob.nbytes

"""Build libkad.so (HIP, gfx950) in-tree, next to this file.

    python -m kubeadmiral_amd.build [--force] [--verbose]

hipcc cross-compiles for gfx950 without a GPU. ``-ffp-contract=off`` keeps
BalancedAllocation's and rsp's float64 arithmetic bit-identical to Go (no FMA
contraction, SURVEY.md §7 hard part 2).
"""

from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libkad.so")
SOURCES = ["kad_kernels.hip", "kad_trigger.hip", "kad_delta.hip", "kad_diff.hip", "kad_api.hip", "kad_pack.cpp", "kad_objects.cpp"]
HEADERS = ["kad_device.h", "kad_wave.h", "kad_select.h", "kad_plan.h", "kad_pool.h"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("KAD_OFFLOAD_ARCH", "gfx950")


def _inputs():
    return [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [
        os.path.join(os.path.dirname(HERE), "include", h) for h in ("kad_sched.h", "kad_pack.h", "kad_objects.h")]


# host code that no kernel launch depends on (the object formats either side of the batch; the native packer,
# whose blob the tests pin byte for byte to pack.py's; the host worker pool): left out of the profile hash,
# so that editing it does not invalidate the kernels' PMC profiles
HOST_ONLY = ("kad_objects.cpp", "kad_objects.h", "kad_pack.cpp", "kad_pool.h")


def source_hash() -> str:
    """16 hex digits of SHA-256 over the sources and headers the measured kernels depend on (libkad.so's,
    except ``HOST_ONLY``): profiles/pmc_<cfg>.json records the hash of the code it was collected on, and
    bench.py uses its counters only when they match."""
    import hashlib

    h = hashlib.sha256()
    for p in _inputs():
        if os.path.basename(p) in HOST_ONLY:
            continue
        with open(p, "rb") as f:
            h.update(os.path.basename(p).encode() + b"\0" + f.read())
    return h.hexdigest()[:16]


STAMP = LIB + ".sha256"  # SHA-256 of every input libkad.so was linked from (written by build())


def inputs_hash() -> str:
    """SHA-256 over every source and header libkad.so is compiled from (names and contents)."""
    import hashlib

    h = hashlib.sha256()
    for p in _inputs():
        with open(p, "rb") as f:
            h.update(os.path.basename(p).encode() + b"\0" + f.read())
    return h.hexdigest()


def up_to_date() -> bool:
    """libkad.so was built from exactly the current sources: its stamp holds their content hash (robust to
    copies and checkouts that reset modification times); a library without a stamp falls back to mtimes."""
    if not os.path.exists(LIB):
        return False
    if os.path.exists(STAMP):
        with open(STAMP) as f:
            return f.read().strip() == inputs_hash()
    t = os.path.getmtime(LIB)
    return all(os.path.getmtime(p) <= t for p in _inputs())


def _obj_dir(extra) -> str:
    """Object directory of one flag set (the plain build, or a variant such as -DKAD_PHASE_PROF)."""
    import hashlib

    tag = hashlib.sha256(" ".join(extra).encode()).hexdigest()[:8] if extra else "base"
    return os.path.join(HERE, "build_obj", f"{ARCH}-{tag}")


def build(force: bool = False, verbose: bool = False, extra=(), out: str = LIB) -> str:
    """Compile libkad.so (or a variant at `out`, e.g. the -DKAD_PHASE_PROF profiling build).

    Each source compiles to its own object in parallel (the kernels' file dominates: ~50 s of a ~90 s serial
    build), and only the objects older than their source or any header are rebuilt; then one link."""
    from concurrent.futures import ThreadPoolExecutor

    stamp = inputs_hash()  # of the sources as compiled below (an edit during the build leaves the stamp stale)
    if out == LIB and not force and up_to_date():
        if not os.path.exists(STAMP):  # up to date by modification times (a library from before stamps)
            _write_stamp(stamp)
        return LIB
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math", "-Wall",
             "-Wno-unused-function", "-pthread"] + list(extra)
    odir = _obj_dir(list(extra))
    os.makedirs(odir, exist_ok=True)
    hdr_t = max(os.path.getmtime(p) for p in _inputs() if not p.endswith((".hip", ".cpp")))

    def compile_one(f):
        src, obj = os.path.join(CSRC, f), os.path.join(odir, f + ".o")
        if not force and os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(src), hdr_t):
            return None
        cmd = [HIPCC] + flags + ["-c", src, "-o", obj + ".tmp"]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
        if r.returncode != 0:
            return cmd, r.stdout.decode(errors="replace")
        if verbose and r.stdout:
            sys.stdout.write(r.stdout.decode(errors="replace"))
        os.replace(obj + ".tmp", obj)
        return None

    with ThreadPoolExecutor(max_workers=len(SOURCES)) as ex:
        fails = [r for r in ex.map(compile_one, SOURCES) if r]
    if fails:
        # compiler warnings would flood the caller's stderr (bench.py's tail is what the driver keeps): shown
        # only when the build fails
        sys.stderr.write(fails[0][1][-20000:])
        raise subprocess.CalledProcessError(1, fails[0][0])
    # device functions called from kernels must not read the kernarg segment pointer (isa_check)
    from . import isa_check

    bad = []
    for src in SOURCES:
        if src.endswith(".hip"):
            bad += isa_check.null_kernarg_loads(os.path.join(odir, src + ".o"))
    if bad:
        raise RuntimeError("device functions load through a null kernarg segment pointer (pass the kernel's "
                           "argument pointer in instead): " + "; ".join(bad[:8]))
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    link = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-pthread", "-o", out + ".tmp"] + \
        [os.path.join(odir, f + ".o") for f in SOURCES]
    subprocess.run(link, check=True)
    if out == LIB and os.path.exists(STAMP):
        os.remove(STAMP)  # (no stamp while the library is being replaced)
    os.replace(out + ".tmp", out)
    if out == LIB:
        _write_stamp(stamp)
    return out


def _write_stamp(h: str) -> None:
    with open(STAMP + ".tmp", "w") as f:
        f.write(h + "\n")
    os.replace(STAMP + ".tmp", STAMP)


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True,
          extra=["-Rpass-analysis=kernel-resource-usage"] if "--resource-usage" in sys.argv else [])
    print(LIB)

"""The build's device-code guard (kubeadmiral_amd/isa_check.py): no device function reads its kernel's
arguments through a null kernarg segment pointer — the cause of round 5's GPU fault."""

import os
import subprocess
import textwrap

import pytest

from kubeadmiral_amd import build, isa_check

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

SNIPPET = textwrap.dedent("""
    #include <hip/hip_runtime.h>
    struct A { int* p; int n; };
    // the round-5 shape: a noinline callee reading the kernel's arguments itself
    __device__ __attribute__((noinline)) void callee_bad(int v) {
      const A* a = (const A*)__builtin_amdgcn_kernarg_segment_ptr();
      a->p[threadIdx.x] = v;
    }
    // the shipped shape: the kernel passes its argument pointer in
    __device__ __attribute__((noinline)) void callee_good(const A* a, int v) { a->p[threadIdx.x] = v; }
    __global__ void kb(A args) { callee_bad(args.n); }
    __global__ void kg(A args) { callee_good((const A*)__builtin_amdgcn_kernarg_segment_ptr(), args.n); }
""")


def _have_toolchain():
    return os.path.exists(HIPCC) and os.path.exists(os.path.join(isa_check.LLVM_BIN, "llvm-objdump"))


@pytest.mark.skipif(not _have_toolchain(), reason="hipcc / llvm tools absent")
def test_guard_flags_a_callee_reading_kernargs(tmp_path):
    src, obj = tmp_path / "k.hip", tmp_path / "k.o"
    src.write_text(SNIPPET)
    subprocess.run([HIPCC, f"--offload-arch={build.ARCH}", "-O3", "-c", str(src), "-o", str(obj)], check=True,
                   stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    found = isa_check.null_kernarg_loads(str(obj))
    assert found and all(f.startswith("_Z10callee_badi:") for f in found), found
    # kernels are told apart by their descriptors (<name>.kd)
    dis, kernels = isa_check.device_code(str(obj))
    assert {"_Z2kb1A", "_Z2kg1A"} <= kernels


def test_scan_tracks_redefinitions():
    dis = textwrap.dedent("""\
        0000000000000000 <callee>:
        \ts_mov_b64 s[4:5], 0
        \tv_readlane_b32 s4, v1, 0
        \tv_readlane_b32 s5, v1, 1
        \ts_load_dword s6, s[4:5], 0x0
        \ts_mov_b64 s[8:9], 0
        \ts_load_dwordx2 s[10:11], s[8:9], 0x10
        0000000000000100 <kern>:
        \ts_mov_b64 s[0:1], 0
        \ts_load_dword s2, s[0:1], 0x0
        """)
    found = isa_check.scan(dis, {"kern"})
    assert len(found) == 1 and "s[8:9]" in found[0], found


@pytest.mark.skipif(not _have_toolchain(), reason="hipcc / llvm tools absent")
def test_product_objects_are_clean():
    build.build()
    odir = build._obj_dir([])
    for src in build.SOURCES:
        if src.endswith(".hip"):
            assert isa_check.null_kernarg_loads(os.path.join(odir, src + ".o")) == [], src

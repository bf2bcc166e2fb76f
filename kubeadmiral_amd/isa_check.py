"""Build-time check of the gfx950 device code: no device function loads through a null base.

A device function that is not inlined into its kernel (``__attribute__((noinline))``) does not receive the
kernarg segment pointer: AMDGPU's calling convention passes the dispatch / queue / implicit-argument pointers
and the work-group ids to callees, not the kernarg segment. ``__builtin_amdgcn_kernarg_segment_ptr()``
evaluated in such a callee lowers to the constant 0 (``s_mov_b64 s[a:b], 0``), and every argument read
through it is a load from address 0 — an illegal memory access on the device. Round 5's one GPU fault was
this: an early version of ``wide_rows`` (the wide kernel's opening-phase row body, a noinline function so
that its registers stay out of the unit loop's allocation) read the kernel's arguments through
``wargs()`` itself; the shipped version takes the argument pointer from the kernel.

``null_kernarg_loads(obj)`` disassembles the gfx950 code object inside a hipcc object file and returns one
finding per non-kernel function that loads (scalar or vector memory) through a register pair it set to 0.
``build.build`` runs it on every HIP object before linking, so the mistake cannot ship again.
"""

from __future__ import annotations

import os
import re
import subprocess
import tempfile
from typing import Dict, List

LLVM_BIN = os.environ.get("KAD_LLVM_BIN", "/opt/rocm/lib/llvm/bin")
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"

_FUNC = re.compile(r"^[0-9a-f]+ <(.+)>:$")
_ZERO_PAIR = re.compile(r"^\s*s_mov_b64\s+s\[(\d+):(\d+)\],\s*0\s*(?:$|//)")
# a memory instruction's base operand: s_load*/s_buffer_load* "dst, s[a:b], off"; global_*/flat_* "..., s[a:b]"
_SMEM = re.compile(r"^\s*s_(?:load|buffer_load)\w*\s+s(?:\[\d+:\d+\]|\d+),\s*s\[(\d+):(\d+)\]")
_GMEM = re.compile(r"^\s*global_\w+\s+.*,\s*s\[(\d+):(\d+)\]")
_SREG = re.compile(r"^s(?:\[(\d+):(\d+)\]|(\d+))$")


def _written_sgprs(line: str) -> set:
    """SGPRs an instruction may write: its first operand (every instruction but stores), and the second of
    VALU forms with a scalar carry / compare destination (v_*_co_*, v_cmp*_e64, v_div_scale*)."""
    code = line.split("//", 1)[0].strip()
    if not code or " " not in code:
        return set()
    mn, ops = code.split(None, 1)
    if "store" in mn or mn.startswith(("s_waitcnt", "s_branch", "s_cbranch", "s_setpc", "s_swappc")):
        return set()
    parts = [o.strip() for o in ops.split(",")]
    cand = parts[:1]
    if mn.startswith("v_") and ("_co_" in mn or mn.startswith("v_cmp") or mn.startswith("v_div_scale")):
        cand = parts[:2]
    regs = set()
    for o in cand:
        m = _SREG.match(o)
        if m:
            regs |= {int(m.group(3))} if m.group(3) else set(range(int(m.group(1)), int(m.group(2)) + 1))
    return regs


def _run(args: List[str]) -> bytes:
    return subprocess.run(args, check=True, stdout=subprocess.PIPE, stderr=subprocess.PIPE).stdout


def _device_object(obj: str, d: str):
    """The gfx950 code object bundled in a hipcc object file (its .hip_fatbin section), or None without one."""
    secs = _run([os.path.join(LLVM_BIN, "llvm-readelf"), "-S", "--wide", obj]).decode(errors="replace")
    if ".hip_fatbin" not in secs:
        return None
    fb, co, junk = os.path.join(d, "fb.bin"), os.path.join(d, "dev.co"), os.path.join(d, "junk.o")
    _run([os.path.join(LLVM_BIN, "llvm-objcopy"), f"--dump-section=.hip_fatbin={fb}", obj, junk])
    _run([os.path.join(LLVM_BIN, "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={fb}",
          f"--targets={TARGET}", f"--output={co}"])
    return co


def device_code(obj: str):
    """(llvm-objdump -d text, kernel names = symbols with a <name>.kd descriptor) of the object's device code;
    ("", set()) for an object without device code."""
    with tempfile.TemporaryDirectory() as d:
        co = _device_object(obj, d)
        if co is None:
            return "", set()
        dis = _run([os.path.join(LLVM_BIN, "llvm-objdump"), "-d", "--no-show-raw-insn", co]).decode(errors="replace")
        syms = _run([os.path.join(LLVM_BIN, "llvm-readelf"), "--symbols", "--wide", co]).decode(errors="replace")
    return dis, {m.group(1) for m in re.finditer(r"\s(\S+)\.kd$", syms, re.M)}


def scan(disasm: str, kernels: set) -> List[str]:
    """Findings "function: line" for non-kernel functions loading through a register pair they zeroed."""
    funcs: Dict[str, List[str]] = {}
    cur = None
    for line in disasm.splitlines():
        m = _FUNC.match(line)
        if m:
            cur = m.group(1)
            funcs[cur] = []
        elif cur is not None:
            funcs[cur].append(line)
    out = []
    for name, body in funcs.items():
        if name in kernels:
            continue
        zero = set()  # register pairs (a, b) holding 0
        for ln in body:
            m = _ZERO_PAIR.match(ln)
            if m:
                zero.add((int(m.group(1)), int(m.group(2))))
                continue
            for rx in (_SMEM, _GMEM):
                mm = rx.match(ln)
                if mm and (int(mm.group(1)), int(mm.group(2))) in zero:
                    out.append(f"{name}: {ln.strip()}")
            if zero:  # a write to a zeroed register ends that pair's null value
                regs = _written_sgprs(ln)
                if regs:
                    zero = {p for p in zero if not (regs & {p[0], p[1]})}
    return out


def null_kernarg_loads(obj: str) -> List[str]:
    if not os.path.exists(obj):
        return []
    return scan(*device_code(obj))

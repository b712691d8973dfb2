"""LDS-visibility lint of libgsr's gfx950 code: every s_barrier must be preceded, on EVERY control-flow
path, by an `s_waitcnt` that drains lgkmcnt to 0 after the path's last LDS access.

Why: __syncthreads() is a workgroup release fence + s_barrier + acquire fence; the release has to wait
for the wave's outstanding LDS operations (lgkmcnt(0)) before the barrier, or another wave may read
the LDS word stale after it.  Round 3 found a build of k_render_fwd whose loop back edge went from a
no-return `ds_and_b32` straight to the loop-head `s_barrier` without that wait;
`lds_barrier()` (gsr_common.h) forces it.  This lint checks the shipped code object, so a compiler
that drops the wait anywhere -- any kernel, any barrier, any path -- fails the CPU suite.

Method: the .hip_fatbin section of the shared object holds one offload bundle per translation unit;
each gfx950 code object is disassembled with llvm-objdump, split into basic blocks at branch targets
and after branches, and a forward may-analysis propagates "an LDS access may be outstanding" (set by
any ds_* memory instruction, cleared by an s_waitcnt whose lgkmcnt field is 0) to a fixed point.

usage: python tools/lds_lint.py [libgsr.so]   (exit status 1 and one line per violation when any)
"""
from __future__ import annotations

import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
# ds_* ops that do not access LDS memory (cross-lane data movement through the LDS crossbar)
NON_MEMORY_DS = ("ds_swizzle", "ds_permute", "ds_bpermute", "ds_nop")

_INSN = re.compile(r"^\s+(?P<op>[a-z_0-9]+)(?P<args>[^/]*)//\s*(?P<addr>[0-9A-Fa-f]+):")
_FUNC = re.compile(r"^(?P<addr>[0-9a-f]+) <(?P<name>[^>]+)>:")
_TARGET = re.compile(r"<(?P<sym>[^>+]+)(?:\+0x(?P<off>[0-9a-f]+))?>\s*$")


def code_objects(lib: str) -> list[str]:
    """Disassembly text of every gfx950 code object embedded in `lib`."""
    with tempfile.TemporaryDirectory() as td:
        fb = os.path.join(td, "fatbin")
        subprocess.run([f"{LLVM}/llvm-objcopy", "--dump-section", f".hip_fatbin={fb}", lib, os.path.join(td, "x")],
                       check=True, capture_output=True)
        data = open(fb, "rb").read()
        starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
        out = []
        for k, s in enumerate(starts):
            part = os.path.join(td, f"b{k}")
            with open(part, "wb") as f:
                f.write(data[s:starts[k + 1] if k + 1 < len(starts) else len(data)])
            co = os.path.join(td, f"co{k}")
            r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={part}",
                                f"--targets={TARGET}", f"--output={co}"], capture_output=True)
            if r.returncode != 0 or not os.path.exists(co) or os.path.getsize(co) == 0:
                continue
            d = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", co], check=True,
                               capture_output=True, text=True)
            out.append(d.stdout)
        return out


def _functions(text: str):
    """{name: [(addr, op, args, branch_target or None)]} from llvm-objdump output."""
    funcs, cur, symaddr = {}, None, {}
    for line in text.splitlines():
        m = _FUNC.match(line)
        if m:
            cur = m.group("name")
            symaddr[cur] = int(m.group("addr"), 16)
            funcs[cur] = []
            continue
        m = _INSN.match(line)
        if m and cur is not None:
            op = m.group("op")
            tgt = None
            if op.startswith("s_branch") or op.startswith("s_cbranch"):
                t = _TARGET.search(line)
                if t:
                    tgt = (t.group("sym"), int(t.group("off") or "0", 16))
            funcs[cur].append((int(m.group("addr"), 16), op, m.group("args"), tgt))
    return {n: [(a, op, args, symaddr[t[0]] + t[1] if t and t[0] in symaddr else None)
                for a, op, args, t in ins] for n, ins in funcs.items()}


def _lgkm_zero(args: str) -> bool:
    """Does this s_waitcnt drain lgkmcnt?  (`lgkmcnt(0)`, or a bare `0`: every counter.)"""
    a = args.strip()
    if re.search(r"lgkmcnt\(0\)", a):
        return True
    return a == "0"


def lint_function(ins) -> list[int]:
    """Addresses of s_barrier instructions some path reaches with an LDS access outstanding."""
    if not ins:
        return []
    addrs = [a for a, *_ in ins]
    index = {a: i for i, a in enumerate(addrs)}
    leaders = {0}
    for i, (a, op, _args, tgt) in enumerate(ins):
        if tgt is not None and tgt in index:
            leaders.add(index[tgt])
        if op.startswith("s_branch") or op.startswith("s_cbranch") or op in ("s_endpgm", "s_setpc_b64"):
            if i + 1 < len(ins):
                leaders.add(i + 1)
    starts = sorted(leaders)
    blocks = [(s, (starts[k + 1] if k + 1 < len(starts) else len(ins))) for k, s in enumerate(starts)]
    bid = {s: k for k, (s, _e) in enumerate(blocks)}
    succ = []
    for s, e in blocks:
        a, op, _args, tgt = ins[e - 1]
        nx = []
        if tgt is not None and tgt in index:
            nx.append(bid[index[tgt]])
        if not (op.startswith("s_branch") or op in ("s_endpgm", "s_setpc_b64")) and e < len(ins):
            nx.append(bid[e])
        succ.append(nx)
    state_in = [False] * len(blocks)
    bad = set()
    work = list(range(len(blocks)))
    seen = [False] * len(blocks)
    while work:
        k = work.pop()
        pend = state_in[k]
        s, e = blocks[k]
        for i in range(s, e):
            a, op, args, _t = ins[i]
            if op.startswith("ds_") and not op.startswith(NON_MEMORY_DS):
                pend = True
            elif op == "s_waitcnt" and _lgkm_zero(args):
                pend = False
            elif op == "s_barrier" and pend:
                bad.add(a)
        for n in succ[k]:
            if (pend and not state_in[n]) or not seen[n]:
                state_in[n] = state_in[n] or pend
                seen[n] = True
                work.append(n)
    return sorted(bad)


def lint_library(lib: str) -> list[str]:
    out = []
    for text in code_objects(lib):
        for name, ins in _functions(text).items():
            for a in lint_function(ins):
                out.append(f"{name} @0x{a:x}: s_barrier reachable with an LDS access outstanding (no lgkmcnt(0))")
    return out


def kernel_count(lib: str) -> int:
    return sum(len(_functions(t)) for t in code_objects(lib))


if __name__ == "__main__":
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(
        os.path.dirname(os.path.abspath(__file__)), "..", "animating-gaussian-splats_amd",
        "diff_gaussian_rasterization", "libgsr.so")
    v = lint_library(lib)
    print(f"{kernel_count(lib)} functions checked, {len(v)} violation(s)")
    for line in v:
        print(line)
    sys.exit(1 if v else 0)

"""DPP data-hazard lint of libgsr's gfx950 code: a DPP instruction must not read a VGPR that a VALU
instruction wrote fewer than 2 wait states before it, on ANY control-flow path.

Why: on gfx9-family cores (gfx950 included) a DPP operand is read through the cross-lane network before
the VALU result forwarding covers it; the ISA requires 2 wait states between a VALU write of a VGPR and a
DPP instruction reading it (the compiler's hazard recognizer pads its own code with s_nop).  Inline
assembly is not padded: `row_halves3` (gsr_backward.hip, the pair reduction's v_add_f32_dpp stages)
carries its own `s_nop 1` and interleaves its three registers so that each stage reads a value written
two instructions earlier.  A violation does not fault: the DPP reads the register's OLD value when the
wave issues its instructions back to back, and the right one when other waves' instructions fall in
between -- so the sums come out wrong only sometimes, and differently from run to run (DESIGN.md 2.4f:
the round-5 C4 gradient mismatch).

Method: the same code objects, functions and basic blocks as tools/lds_lint.py; a forward analysis keeps,
per VGPR, the fewest wait states since a VALU instruction wrote it (s_nop N counts N + 1, every other
instruction 1; merged by minimum over a block's predecessors) and checks every *_dpp instruction's
source VGPRs.

usage: python tools/dpp_hazard_lint.py [libgsr.so]   (exit status 1 and one line per violation when any)
"""
from __future__ import annotations

import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import lds_lint  # noqa: E402

DPP_WAIT_STATES = 2
_VREG = re.compile(r"\bv(?:(\d+)|\[(\d+):(\d+)\])")
# VALU instructions that write both of their first two operands
TWO_DEFS = ("v_swap_b32", "v_permlane16_swap", "v_permlane32_swap")


def _vgprs(tok: str) -> list[int]:
    out = []
    for m in _VREG.finditer(tok):
        if m.group(1) is not None:
            out.append(int(m.group(1)))
        else:
            out.extend(range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def _operands(args: str) -> list[str]:
    # operands up to the first modifier (row_ror:8, row_mask:..., bound_ctrl, offset:...)
    ops = []
    for tok in args.split(","):
        tok = tok.strip()
        if not tok:
            continue
        ops.append(tok.split()[0])
    return ops


def _defs_uses(op: str, args: str):
    """(VGPRs written, VGPRs read) of a VALU instruction; ([], []) for anything else."""
    if not op.startswith("v_"):
        return [], []
    ops = _operands(args)
    if not ops:
        return [], []
    if op.startswith(TWO_DEFS):
        d = _vgprs(ops[0]) + (_vgprs(ops[1]) if len(ops) > 1 else [])
        return d, d
    return _vgprs(ops[0]), [r for o in ops[1:] for r in _vgprs(o)]


def _wait_states(op: str, args: str) -> int:
    if op == "s_nop":
        a = args.strip()
        try:
            return int(a, 0) + 1
        except ValueError:
            return 1
    return 1


def lint_function(ins) -> list[tuple[int, str]]:
    """(address, text) of DPP instructions some path reaches within 2 wait states of a VALU write of
    one of their source VGPRs."""
    if not ins:
        return []
    index = {a: i for i, (a, *_r) in enumerate(ins)}
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
        _a, op, _args, tgt = ins[e - 1]
        nx = []
        if tgt is not None and tgt in index:
            nx.append(bid[index[tgt]])
        if not (op.startswith("s_branch") or op in ("s_endpgm", "s_setpc_b64")) and e < len(ins):
            nx.append(bid[e])
        succ.append(nx)
    # state: {vgpr: wait states since its last VALU write} for writes still inside the hazard window
    state_in: list[dict | None] = [None] * len(blocks)
    state_in[0] = {}
    bad = {}
    work = [0]
    while work:
        k = work.pop()
        st = dict(state_in[k])
        s, e = blocks[k]
        for i in range(s, e):
            a, op, args, _t = ins[i]
            defs, uses = _defs_uses(op, args)
            if "_dpp" in op:
                near = [r for r in uses if st.get(r, DPP_WAIT_STATES) < DPP_WAIT_STATES]
                if near:
                    bad[a] = f"{op}{args.rstrip()} reads v{near[0]} {st[near[0]]} wait state(s) after its VALU write"
            ws = _wait_states(op, args)
            st = {r: d + ws for r, d in st.items() if d + ws < DPP_WAIT_STATES}
            for r in defs:
                st[r] = 0
        for n in succ[k]:
            if state_in[n] is None:
                state_in[n] = dict(st)
                work.append(n)
                continue
            merged = dict(state_in[n])
            changed = False
            for r, d in st.items():
                if d < merged.get(r, DPP_WAIT_STATES):
                    merged[r] = d
                    changed = True
            if changed:
                state_in[n] = merged
                work.append(n)
    return sorted(bad.items())


def lint_library(lib: str) -> list[str]:
    out = []
    for text in lds_lint.code_objects(lib):
        for name, ins in lds_lint._functions(text).items():
            for a, why in lint_function(ins):
                out.append(f"{name} @0x{a:x}: {why}")
    return out


def dpp_count(lib: str) -> int:
    return sum(1 for text in lds_lint.code_objects(lib) for ins in lds_lint._functions(text).values()
               for _a, op, _args, _t in ins if "_dpp" in op)


if __name__ == "__main__":
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(
        os.path.dirname(os.path.abspath(__file__)), "..", "animating-gaussian-splats_amd",
        "diff_gaussian_rasterization", "libgsr.so")
    v = lint_library(lib)
    print(f"{dpp_count(lib)} DPP instructions checked, {len(v)} violation(s)")
    for line in v:
        print(line)
    sys.exit(1 if v else 0)

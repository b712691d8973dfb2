"""Build a library whose pair reduction has the DPP data hazard that tools/dpp_hazard_lint.py checks for
(DESIGN.md 2.4f).  Form `seq`: row_halves3's three registers reduced one after another, one asm
statement per DPP stage and no s_nop -- each v_add_f32_dpp reads the register the previous instruction
wrote.  Form `nonop`: the shipped, interleaved asm without its leading s_nop -- only the first stages can
read a register the compiler's code wrote just before the asm.  Used to
reproduce the round-5 C4 mismatch on the GPU (tools/gpu_r06a.sh) and, built from a temporary copy of
the sources, by tests/test_lds_lint.py to prove the lint flags it.

usage: python tools/dpp_hazard_variant.py OUT.so [seq|nonop]"""
import os
import re
import shutil
import subprocess
import sys
import tempfile

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
HIPCC = "/opt/rocm/bin/hipcc"
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-slp-vectorize"]

HAZARD = '''__device__ inline void dpp_stage_nowait(float &v, int ror) {
    if (ror == 8) asm volatile("v_add_f32_dpp %0, %0, %0 row_ror:8 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(v));
    else if (ror == 4) asm volatile("v_add_f32_dpp %0, %0, %0 row_ror:4 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(v));
    else asm volatile("v_add_f32_dpp %0, %0, %0 row_ror:2 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(v));
}
__device__ inline void row_halves3(float &X, float &Y, float &Z) {
    dpp_stage_nowait(X, 8); dpp_stage_nowait(X, 4); dpp_stage_nowait(X, 2);
    dpp_stage_nowait(Y, 8); dpp_stage_nowait(Y, 4); dpp_stage_nowait(Y, 2);
    dpp_stage_nowait(Z, 8); dpp_stage_nowait(Z, 4); dpp_stage_nowait(Z, 2);
}
'''


def make_variant(out: str, form: str = "seq", sources=None, csrc: str | None = None) -> None:
    csrc = csrc or os.path.join(REPO, "animating-gaussian-splats_amd", "csrc")
    with tempfile.TemporaryDirectory() as td:
        src = os.path.join(td, "csrc")
        shutil.copytree(csrc, src)
        shutil.copytree(os.path.join(REPO, "include"), os.path.join(td, "include"))
        for f in os.listdir(src):
            if f.endswith((".hip", ".h")):
                p = os.path.join(src, f)
                t = open(p).read().replace("../../include/gsr.h", "../include/gsr.h")
                open(p, "w").write(t)
        p = os.path.join(src, "gsr_backward.hip")
        t = open(p).read()
        if form == "seq":
            m = re.search(r"__device__ inline void row_halves3\(float &X, float &Y, float &Z\) \{.*?\n\}\n", t, re.S)
            assert m, "row_halves3 not found"
            t = t[:m.start()] + HAZARD + t[m.end():]
        else:
            assert t.count('asm("s_nop 1\\n\\t"') == 1, "row_halves3's s_nop not found"
            t = t.replace('asm("s_nop 1\\n\\t"', 'asm(')
        open(p, "w").write(t)
        srcs = sources or ["gsr_api.hip", "gsr_forward.hip", "gsr_backward.hip", "gsr_loss.hip", "gsr_densify.hip",
                           "gsr_adam.hip", "gsr_io.hip"]
        subprocess.run([HIPCC, *FLAGS, "-shared", "-o", os.path.abspath(out), *srcs], cwd=src, check=True,
                       capture_output=True)


if __name__ == "__main__":
    make_variant(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "seq")

"""CPU: the shipped gfx950 code object has no workgroup barrier that a path reaches with an LDS access
outstanding (tools/lds_lint.py).  The round-3 nondeterminism came from exactly such a path: k_render_fwd's
loop back edge went from a no-return ds_and_b32 to the loop-head s_barrier without s_waitcnt lgkmcnt(0)
(DESIGN.md 2.4c).  The lint also has to find that defect when it is present: a copy of the sources whose
lds_barrier() lacks the explicit wait is built and must be flagged at k_render_fwd."""
import os
import shutil
import subprocess

import pytest

from conftest import PKG, REPO

import sys
sys.path.insert(0, os.path.join(REPO, "tools"))
import lds_lint  # noqa: E402

LIB = os.path.join(PKG, "diff_gaussian_rasterization", "libgsr.so")
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(LIB), reason="libgsr.so not built")
def test_shipped_library_has_no_unwaited_lds_barrier():
    assert lds_lint.kernel_count(LIB) >= 40  # every translation unit's kernels were inspected
    assert lds_lint.lint_library(LIB) == []


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_lint_flags_the_round3_defect(tmp_path):
    src = tmp_path / "csrc"
    shutil.copytree(os.path.join(PKG, "csrc"), src)
    shutil.copytree(os.path.join(REPO, "include"), tmp_path / "include")
    for f in src.iterdir():
        if f.suffix in (".hip", ".h"):
            f.write_text(f.read_text().replace("../../include/gsr.h", "../include/gsr.h"))
    common = src / "gsr_common.h"
    text = common.read_text()
    wait = "__builtin_amdgcn_s_waitcnt(0xC07F);"
    assert text.count(wait) == 1
    common.write_text(text.replace(wait, ""))
    so = tmp_path / "broken.so"
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
                    "-fno-slp-vectorize", "-shared", "-o", str(so), "gsr_forward.hip"],
                   cwd=src, check=True, capture_output=True)
    bad = lds_lint.lint_library(str(so))
    assert any("k_render_fwd" in b for b in bad), bad


# ---- DPP data hazards (tools/dpp_hazard_lint.py) ---------------------------------------
import dpp_hazard_lint  # noqa: E402
import dpp_hazard_variant  # noqa: E402


@pytest.mark.skipif(not os.path.exists(LIB), reason="libgsr.so not built")
def test_shipped_library_has_no_dpp_hazard():
    """Every DPP instruction of the shipped code object -- the compiler's and row_halves3's inline
    v_add_f32_dpp stages -- reads VGPRs written at least 2 wait states earlier on every path."""
    assert dpp_hazard_lint.dpp_count(LIB) > 100
    assert dpp_hazard_lint.lint_library(LIB) == []


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_dpp_lint_flags_the_round5_defect(tmp_path):
    """The pair reduction with one asm statement per DPP stage and no s_nop (the round-5 work-in-progress
    form) must be flagged at k_render_bwd."""
    so = tmp_path / "dpphaz.so"
    dpp_hazard_variant.make_variant(str(so), sources=["gsr_backward.hip"])
    bad = dpp_hazard_lint.lint_library(str(so))
    assert any("k_render_bwd" in b and "v_add_f32_dpp" in b for b in bad), bad

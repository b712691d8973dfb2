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

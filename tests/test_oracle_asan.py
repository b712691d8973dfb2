"""The CPU oracle under AddressSanitizer + UndefinedBehaviorSanitizer ("-fsanitize=address
on the CPU oracle"): ``make -C oracle asan`` builds oracle/asan_check.c against gsr_oracle.c twice,
sanitized and plain; the sanitized run must exit cleanly (any out-of-bounds access, use after free,
leak or UB aborts it) and print the same checksums as the plain build."""
import os
import shutil
import subprocess

import pytest

ORACLE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle")


@pytest.mark.skipif(shutil.which("gcc") is None and shutil.which("cc") is None, reason="no C compiler")
def test_oracle_clean_under_asan_and_ubsan():
    subprocess.run(["make", "-s", "-C", ORACLE, "asan"], check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0", UBSAN_OPTIONS="halt_on_error=1")
    san = subprocess.run([os.path.join(ORACLE, "_san", "asan_check")], capture_output=True, text=True,
                         env=env, timeout=300)
    assert san.returncode == 0, san.stderr[-4000:]
    assert "ERROR: AddressSanitizer" not in san.stderr and "runtime error" not in san.stderr, san.stderr[-4000:]
    plain = subprocess.run([os.path.join(ORACLE, "_san", "plain_check")], capture_output=True, text=True,
                           timeout=300, check=True)
    assert san.stdout == plain.stdout
    assert len(san.stdout.strip().splitlines()) == 3

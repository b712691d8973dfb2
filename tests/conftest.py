"""Shared pytest setup: import paths, the ``gpu`` marker, and helpers used across test files."""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "animating-gaussian-splats_amd")
for p in (PKG, REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs the HIP kernels)")


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:  # noqa: BLE001
        return False


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but no GPU is visible")
    return torch.device("cuda:0")


@pytest.fixture(autouse=True, scope="session")
def _dump_parity_stats():
    """At the end of the session, the parity tests' outside-tolerance fractions (test_gpu_parity.STATS)
    go to gpurun_out/parity_stats.json when that directory exists (GPU runs)."""
    yield
    mod = sys.modules.get("test_gpu_parity")
    out = os.path.join(REPO, "gpurun_out")
    if mod is not None and getattr(mod, "STATS", None) and os.path.isdir(out):
        import json
        with open(os.path.join(out, "parity_stats.json"), "w") as f:
            json.dump(mod.STATS, f, indent=0)

"""Shared test setup.

Markers: ``gpu`` -- needs an MI355X (run with ``-m gpu`` on the GPU box);
everything else runs on the CPU-only build container.
"""
import json
import os
import sys
from pathlib import Path

import numpy as np
import pytest

# torch (ROCm 7.0 wheel) and libhspmv (linked against /opt/rocm 7.2) share the
# libamdhip64.so.7 SONAME: whichever loads first serves both.  torch only works
# with its own copy, so load torch before any test touches libhspmv.
import torch  # noqa: F401

REPO = Path(__file__).resolve().parent.parent
GOLDEN = REPO / "tests" / "golden"
sys.path.insert(0, str(REPO / "heterogeneous-spmv_amd"))
sys.path.insert(0, str(REPO / "oracle"))
os.environ.setdefault("OMP_SCHEDULE", "static")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP GPU (MI355X)")


@pytest.fixture(scope="session")
def manifest():
    return json.loads((GOLDEN / "manifest.json").read_text())


@pytest.fixture(scope="session")
def golden_names(manifest):
    return sorted(k for k, v in manifest["fixtures"].items() if "same_as" not in v)


def load_golden(name):
    return dict(np.load(GOLDEN / f"{name}.npz"))


def fp64_tol_ok(y, y64, absrow):
    """SURVEY.md §8c / north star: |y - y64| <= 1e-6 |y64| + 1e-12 sum|a x|."""
    err = np.abs(np.asarray(y, np.float64) - y64)
    return bool(np.all(err <= 1e-6 * np.abs(y64) + 1e-12 * absrow))

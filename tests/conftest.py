"""Shared pytest setup.

* registers the ``gpu`` marker (parity tests that need an MI355X);
* puts the repo root (for ``oracle``) and ``nano-hevc_amd/`` (for the drop-in
  ``nano_hevc`` package) on sys.path;
* loads the golden fixtures generated from the reference (tests/golden/).
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "nano-hevc_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    if os.environ.get("NH_TEST_AB") == "1":   # tools: run the parity tests on the A/B library (its NH_* knobs)
        from nano_hevc import _lib
        _lib.use_ab(True)


@pytest.fixture(scope="session")
def golden():
    def load(name):
        with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
            return {k: z[k] for k in z.files}
    return load

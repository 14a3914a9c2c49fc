import os
import subprocess
import sys

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
PKG = os.path.join(ROOT, "fia-kdd-19_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")
LIB = os.path.join(PKG, "influence", "libfia.so")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm GPU) and the built HIP library")


@pytest.fixture(scope="session")
def libfia_path():
    """Path of libfia.so, building it (hipcc cross-compiles without a GPU) if absent."""
    if not os.path.exists(LIB):
        subprocess.check_call(["make", "-C", os.path.join(PKG, "csrc"), "-j8"], stdout=subprocess.DEVNULL)
    return LIB

"""pytest configuration: the `gpu` marker, import paths and shared fixture loaders."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "sdr-for-android-lib_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


# torch wheels bundle their own libamdhip64.so.7 (same SONAME as /opt/rocm's).  Whichever loads first is the
# one every library in the process uses, and torch only works on its own build, so torch is imported before
# libsdrg.so is loaded; libsdrg.so then runs on that runtime (see DESIGN.md "HIP runtime").
try:
    import torch  # noqa: F401
except Exception:  # the CPU suite does not need torch
    torch = None


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) and the built HIP library")


def load_golden(name: str) -> dict:
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


GOLDEN_CASES = ["golden_cs8_16384", "golden_cs16_65536", "golden_cu8_8192_fs2400k", "golden_cf32_4096_fs2500k",
                "golden_cs8_256", "golden_cs8_128"]


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle as O
    O.lib()
    return O

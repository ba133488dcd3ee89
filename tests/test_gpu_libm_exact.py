"""csrc/glibc_logf.h on the GPU against the host's glibc on every non-negative float: the device logf / log10f
(the statistics kernels' dB) bit-exact with glibc, with the table in constant memory and in LDS
(tests/cpp/libm_exact.hip)."""
import os
import subprocess

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def test_glibc_logf_device_exhaustive(tmp_path):
    exe = tmp_path / "libm_exact_gpu"
    inc = os.path.join(ROOT, "sdr-for-android-lib_amd", "csrc")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                    "-fno-builtin", f"-I{inc}", os.path.join(ROOT, "tests", "cpp", "libm_exact.hip"), "-o", str(exe),
                    "-lpthread"], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "mismatches logf 0 log10f 0 lds_vs_const 0" in r.stdout, r.stdout + r.stderr

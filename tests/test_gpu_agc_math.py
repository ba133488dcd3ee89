"""GPU check of the AGC's correctly rounded sqrt/division (sdr-for-android-lib_amd/csrc/ssb_math.h): the packed
sequences the SSB pipeline uses must equal IEEE sqrtf and operator/ bit for bit over every float the AGC's sqrt
operand can take (adaptiveAGC, src/ssb/ssb_demod_opt.cpp:104-107).  Exhaustive: ~1.3e9 operands x 4 targets."""
import os
import subprocess

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def test_agc_desired_exact_exhaustive(tmp_path):
    exe = tmp_path / "agc_exact"
    src = os.path.join(ROOT, "tests", "cpp", "agc_exact.hip")
    inc = os.path.join(ROOT, "sdr-for-android-lib_amd", "csrc")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                    f"-I{inc}", src, "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "mismatches 0 " in r.stdout, r.stdout + r.stderr

"""csrc/glibc_logf.h on the host against the running glibc on every non-negative float (2^31 - 2^23 + 1 values,
about 15 s on 8 cores): the restatement of glibc 2.35's logf / log10f that the statistics kernels use for every dB
value (fft_process.cpp:146-155, :196-210, :256, :282, :304) is bit-exact with the C library the reference's
x86-64 build links, and both are monotone non-decreasing (the statistics rely on it to evaluate the focus window's
dB only near its largest power).  The device instantiation is checked the same way by tests/test_gpu_libm_exact.py."""
import os
import subprocess

from conftest import ROOT


def test_glibc_logf_restatement_exhaustive(tmp_path):
    exe = tmp_path / "libm_exact"
    subprocess.run(["g++", "-O2", "-std=c++17", "-fopenmp", "-ffp-contract=off", "-fno-builtin",
                    f"-I{os.path.join(ROOT, 'sdr-for-android-lib_amd', 'csrc')}",
                    os.path.join(ROOT, "tests", "cpp", "libm_exact.cpp"), "-o", str(exe), "-lm"], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "mismatches logf 0 log10f 0 monotone 0 negative/nan 0" in r.stdout, r.stdout + r.stderr

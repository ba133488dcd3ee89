"""GPU test of the JNI glue logic (sdr-for-android-lib_amd/jni/sdrg_jni_bridge.hpp): a C++ driver with a
recording fake of the JNI calls (no JVM here) checks the full read() callback surface — order, signatures,
payloads bit-identical to the engine's C ABI outputs, setters mid-stream, stopReading and close."""
import os
import subprocess

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def test_jni_bridge_callbacks(tmp_path):
    exe = tmp_path / "jni_bridge_test"
    libdir = os.path.join(ROOT, "sdr-for-android-lib_amd", "lib")
    subprocess.run(["g++", "-O2", "-std=c++17", f"-I{os.path.join(ROOT, 'include')}",
                    f"-I{os.path.join(ROOT, 'sdr-for-android-lib_amd', 'jni')}",
                    os.path.join(ROOT, "tests", "cpp", "jni_bridge_test.cpp"), "-o", str(exe), f"-L{libdir}", "-lsdrg",
                    f"-Wl,-rpath,{libdir}"], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("OK"), r.stdout

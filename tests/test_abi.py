"""CPU tests of the boundary: libsdrg.so loads, exports every entry point include/sdrg.h declares, and its
host-only helpers (SSB filter design, PCM length) agree with the reference build's numbers.  No compute
call touches a GPU here."""
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, ROOT

import sdrg


def _header_symbols():
    text = open(os.path.join(ROOT, "include", "sdrg.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(sdrg_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    declared = _header_symbols()
    assert len(declared) >= 18
    assert sorted(sdrg.EXPORTS) == declared
    out = subprocess.run(["nm", "-D", "--defined-only", sdrg.lib_path()], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT (sdrg_[a-z0-9_]+)$", out, flags=re.M))
    missing = [s for s in declared if s not in exported]
    assert not missing, missing
    L = sdrg.load()
    for s in declared:
        assert hasattr(L, s)
    assert L.sdrg_abi_version() == 1


def test_library_is_gfx950_code():
    blob = open(sdrg.lib_path(), "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    assert b"sm_" not in blob.split(b"amdgcn")[0][-64:]  # no CUDA targets bundled


def test_pcm_len_matches_reference_geometry(oracle_mod):
    O = oracle_mod
    for n in (64, 128, 255, 256, 1024, 4096, 8192, 16384, 65536):
        for fs in (1_000_000, 2_000_000, 2_048_000, 2_400_000, 2_500_000, 10_000_000):
            assert sdrg.ssb_pcm_len(n, fs) == O.ssb_pcm_len(n, fs), (n, fs)
    assert sdrg.ssb_pcm_len(16384, 2_000_000) == 394


def _bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


def test_engine_filter_design_is_bit_exact_with_reference():
    """The host design code (csrc/design.cpp) against coefficients/taps read from the reference build."""
    with np.load(os.path.join(GOLDEN, "golden_ssb_design.npz"), allow_pickle=False) as z:
        d = {k: z[k] for k in z.files}
    for fs in (2_000_000, 2_400_000, 2_500_000):
        for mode, fc in ((1, 3200), (2, 2200), (0, 2200)):
            got = sdrg.ssb_design(16384, fs, mode)
            np.testing.assert_array_equal(_bits(got["lpf"]), _bits(d[f"lpf_{fs}_{fc}"]))
            np.testing.assert_array_equal(_bits(got["hp"]), _bits(d["hp_48000_1200"]))
            np.testing.assert_array_equal(_bits(got["bp"]), _bits(d["bp_48000_2400"]))
    for key in [k for k in d if k.startswith("taps_")]:
        size, dec = (int(x) for x in key.split("_")[1:])
        fs = {41: 2_000_000, 50: 2_400_000, 52: 2_500_000}[dec]
        got = sdrg.ssb_design(size, fs, 1)["taps"]
        want = d[key]
        nz = want != 0
        assert got.size == want.size
        np.testing.assert_array_equal(got == 0, ~nz)
        np.testing.assert_array_equal(_bits(got[nz]), _bits(want[nz]), err_msg=key)


def test_engine_create_without_gpu_reports_status():
    """On a machine without a gfx950 device the engine refuses loudly (no CPU fallback)."""
    try:
        import torch
        if torch.cuda.device_count() > 0:
            pytest.skip("a GPU is visible; covered by the gpu tests")
    except Exception:
        pass
    with pytest.raises(sdrg.SdrgError) as ei:
        sdrg.Engine(sdrg.SDRConfig(), 4)
    assert "SDRG_E_NODEVICE" in str(ei.value)


def test_invalid_configs_rejected_before_device():
    with pytest.raises(sdrg.SdrgError) as ei:
        sdrg.Engine(sdrg.SDRConfig(samplesPerReading=0), 1)
    assert "UNSUPPORTED" in str(ei.value)


def test_jni_bridge_and_dropins_compile(tmp_path):
    """The JNI glue template (with the test's JNI fake) and the C++ drop-in programs compile against the
    public headers (no GPU needed to build; the GPU tests run them)."""
    inc = os.path.join(ROOT, "include")
    jni = os.path.join(ROOT, "sdr-for-android-lib_amd", "jni")
    for src in ("jni_bridge_test.cpp", "compat_main.cpp", "compat_pulse.cpp"):
        subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-Wall", "-Wextra", f"-I{inc}", f"-I{jni}",
                        os.path.join(ROOT, "tests", "cpp", src)], check=True)


def test_product_library_reads_no_lab_knobs():
    """The lab environment knobs exist only in -DSDRG_LAB=1 builds: the product library neither imports getenv nor
    carries a knob's name (tests/test_gpu_lab_knobs.py checks the behaviour on the GPU)."""
    import sdrg
    dyn = subprocess.run(["nm", "-D", "--undefined-only", sdrg.lib_path()], capture_output=True, text=True,
                         check=True).stdout
    assert "getenv" not in dyn
    blob = open(sdrg.lib_path(), "rb").read()
    for knob in (b"SDRG_PIPE_SKIP", b"SDRG_PIPE_MAP", b"SDRG_CU_SPLIT", b"SDRG_PIPE_PRIO", b"SDRG_SPECTRUM_GRID",
                 b"SDRG_SSB_REFERENCE_KERNELS", b"SDRG_STREAM_PRIO", b"SDRG_EVENT_FENCE", b"SDRG_PIPE_STAMPS"):
        assert knob not in blob, knob

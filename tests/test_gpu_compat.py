"""GPU test of the C++ drop-ins (include/sdrg_compat.hpp): a C++ program written like the reference bridge
(FFTProcessor::configure/process/get*, processSSB_opt) is compiled against libsdrg.so and checked against
the oracle: PCM bit-exact, spectrum within the FFT tolerance, statistics on that spectrum bit-exact."""
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def test_cpp_dropins_match_oracle(tmp_path):
    import oracle as O
    n, F, fs, cf, focus, mode = 16384, 3, 2_000_000, 100_000_000, 5, 1
    exe = tmp_path / "compat_main"
    inc = os.path.join(ROOT, "include")
    libdir = os.path.join(ROOT, "sdr-for-android-lib_amd", "lib")
    subprocess.run(["g++", "-O2", "-std=c++17", f"-I{inc}", os.path.join(ROOT, "tests", "cpp", "compat_main.cpp"),
                    "-o", str(exe), f"-L{libdir}", "-lsdrg", f"-Wl,-rpath,{libdir}"], check=True)
    raw = O.synth_frames(F, n, O.CS8, tone_hz=-1700.0, fs=fs)
    iqs = np.stack([O.unpack(O.CS8, raw[f], n) for f in range(F)])
    (tmp_path / "in.bin").write_bytes(iqs.astype(np.float32).tobytes())
    subprocess.run([str(exe), str(tmp_path / "in.bin"), str(tmp_path / "out.bin"), str(n), str(F), str(fs), str(cf),
                    str(focus), str(mode)], check=True)
    buf = (tmp_path / "out.bin").read_bytes()
    fst, sst = O.FftState(cf, fs, n, focus), O.SsbState()
    off = 0
    for f in range(F):
        spec = np.frombuffer(buf, np.float32, n, off); off += 4 * n
        rec = np.frombuffer(buf, np.float64, 11, off); off += 88
        c = int(np.frombuffer(buf, np.int32, 1, off)[0]); off += 4
        pcm = np.frombuffer(buf, np.int16, c, off); off += 2 * c
        ref = O.power_shifted(iqs[f], use_f64=True)
        assert np.all(np.abs(spec - ref) <= 1e-4 * ref + 1e-6 * ref.max())
        want = fst.signal_strength(spec.copy(), 1000 + 100 * f)
        fields = ["mean_snr_db", "mean_snr_sigma", "tracking_frequency", "detection_flag", "peak_above_noise_mean_db",
                  "max_bin_snr_db", "max_bin_snr_sigma", "best1khz_snr_db", "best1khz_snr_sigma",
                  "best1khz_center_freq_hz", "per_bin_mean"]
        for i, k in enumerate(fields):
            assert rec[i] == np.float64(want[k]), (f, k, rec[i], want[k])  # same spectrum: bit-exact
        np.testing.assert_array_equal(pcm, sst.process(iqs[f], fs, mode))


def test_cpp_pulse_dropins_match_reference_fixtures(tmp_path):
    """SpectralPulseDetector / AudioPulseDetector drop-ins, written like the bridge uses them, against the
    reference fixtures (bit-exact getters)."""
    import pulse_inputs as PI
    from conftest import load_golden
    exe = tmp_path / "compat_pulse"
    inc = os.path.join(ROOT, "include")
    libdir = os.path.join(ROOT, "sdr-for-android-lib_amd", "lib")
    subprocess.run(["g++", "-O2", "-std=c++17", f"-I{inc}", os.path.join(ROOT, "tests", "cpp", "compat_pulse.cpp"),
                    "-o", str(exe), f"-L{libdir}", "-lsdrg", f"-Wl,-rpath,{libdir}"], check=True)
    dt = np.dtype([("strength", "<f4"), ("live_etat", "<i4"), ("level", "<i4"), ("locked", "<i4"),
                   ("period_s", "<f4"), ("est_freq_hz", "<f4")])
    g = load_golden("pulse_spectral")
    name, fs, n, kw, _ = PI.SPECTRAL_CASES[0]
    x, f = PI.spectral_case(n=n, fs_energy=fs, **kw)
    (tmp_path / "s.bin").write_bytes(np.stack([x, f], axis=1).astype(np.float32).tobytes())
    subprocess.run([str(exe), "spectral", repr(fs), str(tmp_path / "s.bin"), str(tmp_path / "so.bin")], check=True)
    got = np.frombuffer((tmp_path / "so.bin").read_bytes(), dt)
    for k in dt.names:
        a, b = np.ascontiguousarray(g[name][k]), np.ascontiguousarray(got[k])
        assert a.tobytes() == b.tobytes(), k
    ga = load_golden("pulse_audio")
    name, n, block, kw = PI.AUDIO_CASES[0]
    s = PI.audio_case(n=n, **kw)
    (tmp_path / "a.bin").write_bytes(s.tobytes())
    subprocess.run([str(exe), "audio", str(block), str(tmp_path / "a.bin"), str(tmp_path / "ao.bin")], check=True)
    got = np.frombuffer((tmp_path / "ao.bin").read_bytes(), dt)
    for k in ("strength", "live_etat", "level", "locked", "period_s"):
        assert np.ascontiguousarray(ga[name][k]).tobytes() == np.ascontiguousarray(got[k]).tobytes(), k

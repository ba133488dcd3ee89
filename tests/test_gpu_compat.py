"""GPU test of the C++ drop-ins (include/sdrg_compat.hpp): a C++ program written like the reference bridge
(FFTProcessor::configure/process/get*, processSSB_opt) is compiled against libsdrg.so and checked against
the oracle: PCM bit-exact, spectrum and statistics within the parity tolerances."""
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
            assert abs(rec[i] - float(want[k])) <= 2e-4 + 2e-5 * abs(float(want[k])), (f, k, rec[i], want[k])
        np.testing.assert_array_equal(pcm, sst.process(iqs[f], fs, mode))

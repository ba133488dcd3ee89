"""evaluateSignalStrength (fft_process.cpp:122-379) on the GPU across window geometries: every statistics kernel
variant the host picks from the geometry (csrc/stats.hip: the narrow one-wave-per-frame kernel with its pooled
bins in 8 or 24 registers per lane or visited in LDS, and the wide 256-thread kernel once the windows exceed the
narrow kernel's staging budget; a rocprofv3 trace of this file shows all four launched) against the oracle restatement on the SAME GPU spectrum: integer outputs exact,
floats to 2e-5 relative + 2e-4 absolute (only libm ulps differ), as in tests/test_gpu_parity.py.  The grid spans
frame sizes, sample rates and focus widths from 1 kHz to 200 kHz, including geometries where fewer than two
reference windows fit (the stale-output branch, :218-225)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

FLOAT_FIELDS = ["mean_snr_db", "mean_snr_sigma", "peak_above_noise_mean_db", "max_bin_snr_db", "max_bin_snr_sigma",
                "best1khz_snr_db", "best1khz_snr_sigma", "best1khz_center_freq_hz", "per_bin_mean", "abs_peak_db",
                "signal_power_db"]
INT_FIELDS = ["detection_flag", "peak_bin", "valid", "n_ref_windows", "tracking_frequency"]

GEOMETRIES = [(n, fs, focus) for n in (8192, 16384, 65536) for fs in (2_000_000, 2_500_000)
              for focus in (1, 2, 10, 20, 50, 100, 200)]


@pytest.fixture(scope="module")
def S():
    import sdrg
    return sdrg


@pytest.fixture(scope="module")
def O():
    import oracle
    return oracle


@pytest.mark.parametrize("n,fs,focus", GEOMETRIES)
def test_stats_geometry_vs_oracle(S, O, n, fs, focus):
    fmt = O.CS16 if n >= 65536 else O.CS8
    B, F = 4, 2
    rng = np.random.default_rng(n + fs // 1000 + focus)
    raw = []
    for b in range(B):  # a tone inside the focus, one outside, a weak one, noise only
        tone = [float(rng.uniform(-0.4, 0.4)) * focus * 1e3, float(rng.uniform(0.3, 0.45)) * fs, 500.0, 0.0][b]
        amp = [0.5, 0.3, 0.01, 0.0][b] * (8000.0 if fmt == O.CS16 else 60.0)
        raw.append(O.synth_frames(F, n, fmt, tone_hz=tone, fs=fs, amp=amp, seed=7 * n + focus + b))
    raw = np.stack(raw)
    cfg = S.SDRConfig(centerFrequency=100_000_000, samplesPerReading=n, sampleRate=fs, freqFocusRangeKhz=focus,
                      soundMode=1)
    eng = S.Engine(cfg, B)
    fst = [O.FftState(100_000_000, fs, n, focus) for _ in range(B)]
    for f in range(F):
        now = 1000 + 350 * f
        spec, rec, _ = eng.process(raw[:, f], fmt=fmt, stages=S.STAGE_SPECTRUM | S.STAGE_STATS, now_ms=now)
        want = np.zeros(B, dtype=rec.dtype)
        for b in range(B):
            want[b] = fst[b].signal_strength(spec[b], now)
        for fld in INT_FIELDS:
            np.testing.assert_array_equal(rec[fld], want[fld], err_msg=f"n{n} fs{fs} focus{focus} f{f} {fld}")
        for fld in FLOAT_FIELDS:
            a, c = rec[fld].astype(np.float64), want[fld].astype(np.float64)
            ok = np.abs(a - c) <= 2e-4 + 2e-5 * np.abs(c)
            assert ok.all(), (n, fs, focus, f, fld, a[~ok][:4], c[~ok][:4])
    eng.close()

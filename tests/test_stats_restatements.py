"""Two independent restatements of evaluateSignalStrength (src/dsp/fft_process.cpp:122-379) must agree: the C
oracle (oracle/sdrg_oracle.c, which the GPU statistics kernel is tested against) and a numpy restatement written
separately from the reference text (oracle/stats_np.py).  The reference's own fft_process.cpp cannot be built here
(jni.h and an FFTW library are absent), so this cross-check stands in for a reference pin of the statistics: a
shared misreading would have to be made twice, independently.

Randomised spectra cover noise, tones in and out of focus, ties (equal window means, equal peak bins, constant
spectra), invalid focus (< 2 reference windows), non-power-of-two and odd N, the 65536-bin / 200 kHz geometry,
and multi-frame sequences through the tracking latch and the detection ring."""
import numpy as np
import pytest

import stats_np

INTS = ["detection_flag", "peak_bin", "valid", "n_ref_windows", "tracking_frequency"]
FLOATS = ["mean_snr_db", "mean_snr_sigma", "peak_above_noise_mean_db", "max_bin_snr_db", "max_bin_snr_sigma",
          "best1khz_snr_db", "best1khz_snr_sigma", "best1khz_center_freq_hz", "per_bin_mean", "abs_peak_db",
          "signal_power_db"]


def spectrum(rng, n, kind):
    if kind == "noise":
        return rng.exponential(1.0, n).astype(np.float32)
    if kind == "tone":
        p = rng.exponential(1.0, n).astype(np.float32)
        p[rng.integers(n // 2 - n // 64, n // 2 + n // 64)] += np.float32(rng.uniform(10, 1e4))
        return p
    if kind == "const":  # every window mean equal, every bin a tie
        return np.full(n, np.float32(rng.uniform(0.1, 10)), np.float32)
    if kind == "steps":  # windows of equal means in several groups, peaks repeated
        p = np.repeat(rng.choice([0.5, 1.0, 2.0], size=n // 16 + 1), 16)[:n].astype(np.float32)
        p[n // 2 - 3: n // 2 + 3] = 50.0
        return p
    if kind == "quantised":  # few distinct values: ties everywhere, in gaps and medians too
        return rng.integers(1, 5, n).astype(np.float32)
    if kind == "tiny":  # dB floor (1e-20) and zeros
        p = rng.exponential(1e-22, n).astype(np.float32)
        p[rng.random(n) < 0.2] = 0.0
        return p
    raise ValueError(kind)


CASES = [(4096, 2_000_000, 5), (16384, 2_000_000, 5), (2048, 2_500_000, 5), (1536, 2_000_000, 5),
         (4099, 2_048_000, 3), (65536, 2_000_000, 200), (65536, 2_000_000, 5), (1000, 2_000_000, 50),
         (16384, 2_000_000, 400), (8192, 2_400_000, 10), (12288, 3_200_000, 7), (256, 2_000_000, 5)]
KINDS = ["noise", "tone", "const", "steps", "quantised", "tiny"]


def compare(got, want, ctx):
    """Every output bit-identical: both restatements run the same float32 operations in the reference's order
    with the same C-library log10f / logf (IEEE sqrt and division), so any difference is a reading difference."""
    for f in INTS:
        assert int(got[f]) == int(want[f]), (ctx, f, got[f], want[f])
    for f in FLOATS:
        a, b = np.float32(got[f]), np.float32(want[f])
        assert a.tobytes() == b.tobytes() or (np.isnan(a) and np.isnan(b)), (ctx, f, float(a), float(b))


@pytest.mark.parametrize("n,fs,focus", CASES)
def test_numpy_and_c_restatements_agree(oracle_mod, n, fs, focus):
    O = oracle_mod
    rng = np.random.default_rng(n * 7 + focus)
    frames = 60 if n <= 16384 else 12
    cf = 100_000_000
    c_state = O.FftState(cf, fs, n, focus)
    np_state = stats_np.SignalStrength(cf, fs, focus)
    now = 1000
    for f in range(frames):
        kind = KINDS[f % len(KINDS)] if f % 3 else "tone"
        p = spectrum(rng, n, kind)
        now += int(rng.integers(1, 200))
        if f == frames // 2:  # setFrequency mid-run: configure + isCenterFrequencyChanged
            cf += 25_000
            c_state.configure(cf, fs, n, focus)
            c_state.set_center_frequency_changed()
            np_state.configure(cf, fs, focus)
            np_state.cf_changed = True
        want = c_state.signal_strength(p, now)
        got = np_state.evaluate(p, now)
        compare(got, want, (n, fs, focus, f, kind))


def test_restatements_agree_on_thousands_of_random_spectra(oracle_mod):
    O = oracle_mod
    rng = np.random.default_rng(2026)
    count = 0
    for trial in range(40):
        n = int(rng.choice([512, 777, 1024, 2000, 4096, 6144, 8192]))
        fs = int(rng.choice([1_000_000, 2_000_000, 2_048_000, 2_400_000, 3_200_000]))
        focus = int(rng.choice([1, 2, 5, 10, 20, 100]))
        c_state = O.FftState(100_000_000, fs, n, focus)
        np_state = stats_np.SignalStrength(100_000_000, fs, focus)
        now = 0
        for f in range(50):
            p = spectrum(rng, n, KINDS[int(rng.integers(0, len(KINDS)))])
            now += int(rng.integers(1, 150))
            compare(np_state.evaluate(p, now), c_state.signal_strength(p, now), (trial, f, n, fs, focus))
            count += 1
    assert count == 2000

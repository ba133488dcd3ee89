"""CPU tests: pin the oracle (oracle/sdrg_oracle.c) before trusting it as the parity checker.

* SSB: bit-for-bit against the reference's own ssb_demod_opt.cpp (tests/golden fixtures written by
  tests/golden/make_golden.py from oracle/_ref/ref_ssb) and, when the reference build is present,
  against fresh reference runs at the stage level.
* Spectrum: against numpy's float64 DFT (the fixtures' `spectra`).
* Window geometry: against the table the survey measured on the reference (tests/golden/geometry.json).
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, GOLDEN_CASES, load_golden


def _bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


@pytest.mark.parametrize("case", GOLDEN_CASES)
def test_oracle_ssb_matches_reference_fixtures(oracle_mod, case):
    O = oracle_mod
    g = load_golden(case)
    S, F = g["raw"].shape[:2]
    n, fs, fmt = int(g["n"]), int(g["fs"]), int(g["fmt"])
    for s in range(S):
        st = O.SsbState()
        for f in range(F):
            iq = O.unpack(fmt, g["raw"][s, f], n)
            pcm = st.process(iq, fs, int(g["modes"][s, f]))
            np.testing.assert_array_equal(pcm, g["pcm"][s, f], err_msg=f"{case} stream {s} frame {f}")


def test_oracle_filter_design_matches_reference(oracle_mod):
    O = oracle_mod
    with np.load(os.path.join(GOLDEN, "golden_ssb_design.npz"), allow_pickle=False) as z:
        d = {k: z[k] for k in z.files}
    for fs in (2_000_000, 2_400_000, 2_500_000):
        for fc, q in ((3200.0, 0.9), (2200.0, 1.2)):
            np.testing.assert_array_equal(_bits(O.lpf_coefs(float(fs), fc, q)), _bits(d[f"lpf_{fs}_{int(fc)}"]))
    np.testing.assert_array_equal(_bits(O.hp_coefs(48000.0, 1200.0, 0.7)), _bits(d["hp_48000_1200"]))
    np.testing.assert_array_equal(_bits(O.bp_coefs(48000.0, 2400.0, 0.6)), _bits(d["bp_48000_2400"]))
    for key in [k for k in d if k.startswith("taps_")]:
        size, dec = (int(x) for x in key.split("_")[1:])
        got, want = O.fir_taps(size, dec), d[key]
        # taps are read back from the reference as impulse responses (0 + 1*h[p]), which maps -0 to +0
        nz = want != 0
        np.testing.assert_array_equal(got == 0, ~nz, err_msg=key)
        np.testing.assert_array_equal(_bits(got[nz]), _bits(want[nz]), err_msg=key)


@pytest.mark.parametrize("case", [c for c in GOLDEN_CASES if c != "golden_cs8_128"])
def test_oracle_spectrum_matches_float64_dft(oracle_mod, case):
    O = oracle_mod
    g = load_golden(case)
    n, fmt = int(g["n"]), int(g["fmt"])
    for (s, f), want in zip(g["spectra_idx"], g["spectra"]):
        iq = O.unpack(fmt, g["raw"][s, f], n)
        for use_f64 in (False, True):
            got = O.power_shifted(iq, use_f64)
            tol = 1e-4 * want + 1e-6 * want.max()
            assert np.all(np.abs(got - want) <= tol), (case, use_f64, np.max(np.abs(got - want) / (tol)))


def test_oracle_geometry_matches_survey(oracle_mod):
    O = oracle_mod
    with open(os.path.join(GOLDEN, "geometry.json")) as f:
        geo = json.load(f)
    for c in geo["cases"]:
        lo, hi, w, wins = O.window_geometry(c["sample_rate"], c["n"], c["focus_khz"])
        assert [lo, hi] == c["focus"]
        assert len(wins) == c["n_ref"]
        if "win_bins_1k" in c:
            assert w == c["win_bins_1k"]
        if "windows_first_two" in c:
            assert [list(x) for x in wins[:2]] == c["windows_first_two"]
            assert [list(x) for x in wins[-2:]] == c["windows_last_two"]
            assert sum(h - l + 1 for l, h in wins) == c["ref_bins_total"]
            assert O.ssb_decim(c["sample_rate"]) == c["decim"]
            assert O.ssb_pcm_len(c["n"], c["sample_rate"]) == c["pcm_len"]
        if "window_len" in c:
            assert all(h - l + 1 == c["window_len"] for l, h in wins)
    cw = geo["cw_peak"]
    raw = O.synth_frames(1, cw["n"], O.CS8, tone_hz=cw["tone_hz"], fs=cw["sample_rate"])
    st = O.FftState(100_000_000, cw["sample_rate"], cw["n"], 5)
    _, rec = st.process(O.unpack(O.CS8, raw[0], cw["n"]), 1000)
    assert rec["peak_bin"] == cw["peak_bin"]


def test_oracle_stats_analytic_cases(oracle_mod):
    """Hand-checkable statistics: flat spectrum and a single-bin spike."""
    O = oracle_mod
    n, fs = 16384, 2_000_000
    st = O.FftState(100_000_000, fs, n, 5)
    P = np.full(n, 1e-4, dtype=np.float32)
    rec = st.signal_strength(P, 1000)
    # flat: every window mean = focus mean -> SNR 0, noise level -40 dB, MAD floors apply
    assert rec["valid"] == 1 and rec["n_ref_windows"] == 10
    assert abs(rec["mean_snr_db"]) < 1e-5 and abs(rec["per_bin_mean"] + 40.0) < 1e-4
    assert rec["detection_flag"] == 0
    P2 = P.copy()
    P2[8200] = 1.0
    rec2 = st.signal_strength(P2, 1100)
    assert rec2["peak_bin"] == 8200 and abs(rec2["abs_peak_db"]) < 1e-6
    assert abs(rec2["peak_above_noise_mean_db"] - 40.0) < 1e-3
    # best 1 kHz window containing the spike starts at or before 8200; centre frequency is on the grid
    fpb = np.float32(fs) / np.float32(n)
    k = (rec2["best1khz_center_freq_hz"] - (100_000_000 - 1_000_000)) / fpb
    assert abs(k - round(k)) < 1e-2 and 8200 - 9 < round(k) <= 8200 + 9
    # peak latch: tracking follows the peak only after 300 ms
    assert rec2["tracking_frequency"] == 100_000_000
    rec3 = st.signal_strength(P2, 1401)
    assert rec3["tracking_frequency"] == round(8200 * fpb + np.float32(100_000_000) - np.float32(1_000_000))


def test_oracle_invalid_when_focus_too_wide(oracle_mod):
    """focus so wide that fewer than 2 reference windows fit: outputs zeroed, detection 0 (:218-225)."""
    O = oracle_mod
    st = O.FftState(100_000_000, 2_000_000, 4096, 400)
    P = np.random.default_rng(1).random(4096).astype(np.float32)
    rec = st.signal_strength(P, 1000)
    assert rec["valid"] == 0 and rec["mean_snr_db"] == 0 and rec["detection_flag"] == 0


@pytest.mark.skipif(not os.path.exists(os.path.join(os.path.dirname(GOLDEN), "..", "oracle", "_ref", "ref_ssb")),
                    reason="reference build (oracle/_ref) only exists where /root/reference is mounted")
def test_oracle_ssb_stages_match_reference_live(oracle_mod):
    O = oracle_mod
    raw = O.synth_frames(1, 16384, O.CS8, tone_hz=900.0, seed=77)
    iq = O.unpack(O.CS8, raw[0], 16384).reshape(-1, 2)
    want = O.ref_ssb_stages(iq, 2_000_000, 3200.0, 0.9, 0.35, 0.006, 0.55)
    _, got = O.SsbState().process(iq, 2_000_000, 1, stages=True)
    for k in ("dc_re", "lpf", "agc", "fir", "eq"):
        np.testing.assert_array_equal(_bits(got[k]), _bits(want[k]), err_msg=k)


def test_power_shifted_any_n_vs_numpy(oracle_mod):
    """The oracle's any-N double DFT (Bluestein for non-powers of two) against numpy's float64 FFT, with the
    reference's fftshift loop (fft_process.cpp:92-97): for odd N element N-1 is never written (stays 0 in a fresh
    vector) and bin N-1 is dropped."""
    O = oracle_mod
    rng = np.random.default_rng(8)
    for n in (1, 2, 3, 5, 7, 12, 97, 1000, 1536, 3072, 4099, 10240, 12289, 20000, 24576):
        x = (rng.normal(0, 0.3, 2 * n)).astype(np.float32)
        got = O.power_shifted(x, use_f64=True)
        X = np.fft.fft(x[0::2].astype(np.float64) + 1j * x[1::2].astype(np.float64))
        p = (X.real.astype(np.float32) ** 2 + X.imag.astype(np.float32) ** 2).astype(np.float32)
        half = n // 2
        want = np.zeros(n, np.float32)
        want[:half] = p[half:2 * half]
        want[half:2 * half] = p[:half]
        tol = 1e-5 * want + 1e-9 * want.max()
        assert np.all(np.abs(got - want) <= tol), (n, np.max(np.abs(got - want)))
        if n % 2:
            assert got[n - 1] == 0.0

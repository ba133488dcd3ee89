"""Statistics decided by the last ulp: the GPU's evaluateSignalStrength (csrc/stats.hip) against the oracle on
crafted spectra fed through sdrg_engine_signal_strength_host, every record field bit-exact.

The reference turns powers into dB with glibc's log10f (fft_process.cpp:146-155, :196-210, :256) and then decides
  * the focus peak: the FIRST bin whose dB is strictly greater than every earlier one (:146-154);
  * the window order: std::sort by meanDb (:218-247), whose bottom windows feed the pooled per-bin statistics
    (sequential sum in sorted order, :252-269, and the MAD of their gaps);
so two bins whose powers differ by an ulp or two can land on the same dB float under one libm and on different
floats under another, and then the peak index, the window set and every downstream value differ.  The kernels
compute dB through a restatement of glibc's log10f (csrc/glibc_logf.h, exhaustively equal to glibc:
tests/test_libm_exact.py, tests/test_gpu_libm_exact.py), and these spectra are built so that those decisions hang
on the rounding:
  * focus bins drawn from a handful of adjacent floats around p0 (many dB ties, and pairs an ulp apart that tie
    or not depending on the log's rounding), at p0 across 40 decades and in denormals;
  * reference windows holding the same multiset of values in different orders (equal or ulp-apart window means);
  * both kernels: the narrow one (16384 / 5 kHz) and the wide one (65536 / 200 kHz)."""
import numpy as np
import pytest

from test_gpu_parity import assert_records_equal

pytestmark = pytest.mark.gpu

FS, CF = 2_000_000, 100_000_000


@pytest.fixture(scope="module")
def S():
    import sdrg
    return sdrg


@pytest.fixture(scope="module")
def O():
    import oracle
    return oracle


def ulps_around(p0, k, size, rng):
    """size float32 values p0 + j ulps, j uniform in [0, k)."""
    base = np.array([p0], np.float32).view(np.uint32)[0]
    return (base + rng.integers(0, k, size).astype(np.uint32)).view(np.float32)


def crafted(O, n, focus, B, rng, p0s):
    lo, hi, _, wins = O.window_geometry(FS, n, focus)
    spec = np.empty((B, n), np.float32)
    for b in range(B):
        p0 = np.float32(p0s[b % len(p0s)])
        kind = b % 4
        # background: a noise floor near p0 / 100 so every window mean is finite and distinct-ish
        spec[b] = (rng.exponential(1.0, n) * p0 / 100).astype(np.float32)
        if kind == 0:    # focus: a plateau of ulp-neighbours (dB ties decide the first maximum)
            spec[b, lo:hi + 1] = ulps_around(p0, 4, hi - lo + 1, rng)
        elif kind == 1:  # plateau plus one bin a single ulp above the plateau, late in the window
            spec[b, lo:hi + 1] = np.float32(p0)
            spec[b, hi - 3] = (np.array([p0], np.float32).view(np.uint32) + np.uint32(1)).view(np.float32)[0]
        elif kind == 2:  # every reference window: one shared multiset of values, permuted per window
            vals = (rng.exponential(1.0, max(h - l + 1 for l, h in wins)) * p0).astype(np.float32)
            for l, h in wins:
                spec[b, l:h + 1] = rng.permutation(vals[:h - l + 1])
            spec[b, lo:hi + 1] = ulps_around(p0 * 10, 3, hi - lo + 1, rng)
        else:            # reference windows of ulp-neighbours (window means tie or differ by an ulp)
            for l, h in wins:
                spec[b, l:h + 1] = ulps_around(p0, 3, h - l + 1, rng)
            spec[b, lo:hi + 1] = ulps_around(p0 * 3, 8, hi - lo + 1, rng)
    return spec


P0S = [1e-38, 3e-30, 1.7e-12, 6.1e-7, 2.3e-3, 0.5, 1.0, 1.0000001, 9.99e2, 4.4e7, 1.2e19]


@pytest.mark.parametrize("n,focus", [(16384, 5), (65536, 5), (65536, 200)])
def test_ulp_ties_bit_exact(S, O, n, focus):
    rng = np.random.default_rng(n + focus)
    B, F = 44, 3
    eng = S.Engine(S.SDRConfig(centerFrequency=CF, samplesPerReading=n, sampleRate=FS, freqFocusRangeKhz=focus,
                               soundMode=1), B)
    fst = [O.FftState(CF, FS, n, focus) for _ in range(B)]
    ties = 0
    lo, hi = O.window_geometry(FS, n, focus)[:2]
    for f in range(F):
        spec = crafted(O, n, focus, B, rng, P0S)
        now = 1000 + 200 * f
        rec = eng.signal_strength(spec, now)
        want = np.stack([fst[b].signal_strength(spec[b], now) for b in range(B)])
        assert_records_equal(rec, want, msg=f"n{n} focus{focus} call{f}")
        # the crafted focus windows do put the decision on a tie: the first maximum of dB is not the first
        # maximum of power in many frames
        ties += int(np.sum(rec["peak_bin"] != lo + np.argmax(spec[:, lo:hi + 1], axis=1)))
    assert ties > 0
    eng.close()


@pytest.mark.parametrize("n,focus", [(16384, 5), (65536, 200)])
def test_denormal_and_zero_spectra_bit_exact(S, O, n, focus):
    """Powers in the denormal range and exact zeros (the 1e-20 floor dominates) through both log branches; at 65536 /
    200 kHz the wide kernel's focus peak from the largest power meets dB plateaus thousands of floats wide."""
    B = 8
    rng = np.random.default_rng(5)
    spec = np.zeros((B, n), np.float32)
    for b in range(1, B):
        spec[b] = rng.integers(1, 1 << (3 * b), n).astype(np.uint32).view(np.float32)  # denormals of growing size
    spec[B - 1, ::7] = 0.0
    eng = S.Engine(S.SDRConfig(centerFrequency=CF, samplesPerReading=n, sampleRate=FS, freqFocusRangeKhz=focus), B)
    fst = [O.FftState(CF, FS, n, focus) for _ in range(B)]
    rec = eng.signal_strength(spec, 1000)
    want = np.stack([fst[b].signal_strength(spec[b], 1000) for b in range(B)])
    assert_records_equal(rec, want, msg="denormal")
    eng.close()

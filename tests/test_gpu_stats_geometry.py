"""evaluateSignalStrength (fft_process.cpp:122-379) on the GPU across window geometries: every statistics kernel
variant the host picks from the geometry (csrc/stats.hip: the narrow one-wave-per-frame kernel with its pooled
bins in 8 or 24 registers per lane or visited in LDS, and the wide 256-thread kernel once the windows exceed the
narrow kernel's staging budget; a rocprofv3 trace of this file shows all four launched) against the oracle restatement on the SAME GPU spectrum: every field bit-exact (dB through the
glibc log10f restatement, csrc/glibc_logf.h), as in tests/test_gpu_parity.py.  The grid spans
frame sizes, sample rates and focus widths from 1 kHz to 200 kHz, including geometries where fewer than two
reference windows fit (the stale-output branch, :218-225)."""
import numpy as np
import pytest

from test_gpu_parity import assert_records_equal

pytestmark = pytest.mark.gpu

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
        assert_records_equal(rec, want, msg=f"n{n} fs{fs} focus{focus} f{f}")
    eng.close()


@pytest.mark.parametrize("n,fs,focus", [(65536, 2_000_000, 200), (65536, 2_500_000, 100), (16384, 2_000_000, 200),
                                        (65536, 2_000_000, 20)])
@pytest.mark.parametrize("B", [1, 6, 9])
def test_wide_statistics_partial_groups(S, O, n, fs, focus, B):
    """The wide statistics kernel runs several frames per workgroup (csrc/stats.hip, stats_wide_multi_kernel): stream
    counts that leave the last workgroup partly empty, on caller spectra (sdrg_engine_signal_strength_host), every
    field bit-exact against the oracle, the stream state carried over three calls."""
    rng = np.random.default_rng(n + B + focus)
    cfg = S.SDRConfig(centerFrequency=100_000_000, samplesPerReading=n, sampleRate=fs, freqFocusRangeKhz=focus,
                      soundMode=1)
    eng = S.Engine(cfg, B)
    fst = [O.FftState(100_000_000, fs, n, focus) for _ in range(B)]
    for f in range(3):
        spec = rng.exponential(1.0, size=(B, n)).astype(np.float32)
        for b in range(B):  # a peak in the focus; a plateau of 40 equal maxima; one of 400 (more near-maximum bins
            # than the multi-frame kernel keeps as candidates per lane: its focus re-scan); noise only
            if b % 4 == 0:
                spec[b, n // 2 + int(rng.integers(-50, 50))] = np.float32(1e4 * (1 + f))
            elif b % 4 == 1:
                spec[b, n // 2 - 20:n // 2 + 20] = np.float32(77.0)
            elif b % 4 == 2:
                spec[b, n // 2 - 200:n // 2 + 200] = np.float32(55.0 + f)
        now = 1000 + 333 * f
        rec = eng.signal_strength(spec, now_ms=now)
        want = np.zeros(B, dtype=rec.dtype)
        for b in range(B):
            want[b] = fst[b].signal_strength(spec[b], now)
        assert_records_equal(rec, want, msg=f"n{n} fs{fs} focus{focus} B{B} f{f}")
    eng.close()

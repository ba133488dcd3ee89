"""Spectrum for ANY frame size the reference accepts (fftwf_plan_dft_1d(sampCount, ...) plans every N,
src/dsp/fft_process.cpp:77-79; SDRConfig only recommends multiples of 512, SDRBridge.kt:25-26): the engine's
mixed-radix / four-step / Bluestein kernels (csrc/fftany.hip) against the float64 DFT (oracle_dft_f64_any, pinned to
numpy in tests/test_oracle.py) with the SURVEY 8c bound |dP| <= 1e-4 P + 1e-6 max(P), the reference's fftshift
loop for odd N (element N-1 never written), peak bin exact, and the statistics on the engine's spectrum equal to
the oracle's bit for bit (wide windows at N > 65536 exercise the global pooled-bin path)."""
import numpy as np
import pytest

from test_gpu_parity import assert_records_equal

pytestmark = pytest.mark.gpu

FS, CF = 2_000_000, 100_000_000

# VERDICT r1's list, then the edges: tiny N, odd and prime N (Bluestein in one workgroup and four-step), powers
# of two above 65536, 3 * 2^18 (four-step mixed radix), and the largest prime below 2^20
SIZES = [1536, 3072, 10240, 12288, 20000, 24576, 131072,
         1, 2, 3, 7, 97, 1000, 4099, 12289, 65537, 786432, 1048576, 999983]


@pytest.fixture(scope="module")
def S():
    import sdrg
    return sdrg


@pytest.fixture(scope="module")
def O():
    import oracle
    return oracle


@pytest.mark.parametrize("n", SIZES)
def test_any_n_spectrum_vs_f64_dft(S, O, n):
    B = 3 if n <= 65536 else 2
    fmts = [O.CS8, O.CS16, O.CF32]
    fmt = fmts[n % 3]
    raw = np.stack([O.synth_frames(1, n, fmt, tone_hz=1100.0 + 700.0 * b, fs=FS, seed=n + b)[0] for b in range(B)])
    cfg = S.SDRConfig(centerFrequency=CF, samplesPerReading=n, sampleRate=FS, freqFocusRangeKhz=5, soundMode=1)
    eng = S.Engine(cfg, B)
    spec, rec, _ = eng.process(raw, fmt=fmt, stages=S.STAGE_SPECTRUM | S.STAGE_STATS, now_ms=1000)
    last = n - 1 if n % 2 else n  # odd N: element N-1 is not part of the reference's output (stays 0 here)
    for b in range(B):
        iq = O.unpack(fmt, raw[b], n)
        want = O.power_shifted(iq, use_f64=True)
        ok = np.abs(spec[b][:last] - want[:last]) <= 1e-4 * want[:last] + 1e-6 * want.max()
        assert ok.all(), (n, b, np.argwhere(~ok)[:5].ravel(), spec[b][~ok][:3], want[:last][~ok][:3])
        if n % 2:
            assert spec[b][n - 1] == 0.0
        st = O.FftState(CF, FS, n, 5)
        w = st.signal_strength(spec[b], 1000)
        assert_records_equal(rec[b:b + 1], np.array([w], dtype=rec.dtype), msg=f"n{n} stream {b}")
        if n >= 64:  # the tone's bin: exact against the float64 reference's first maximum in the focus window
            lo, hi = O.window_geometry(FS, n, 5)[:2]
            if hi >= lo:
                db = 10.0 * np.log10(want[lo:hi + 1].astype(np.float32) + np.float32(1e-20))
                assert rec[b]["peak_bin"] == lo + int(np.argmax(db)), (n, b)
    eng.close()


def test_any_n_second_frame_keeps_odd_tail(S, O):
    """Odd N: power_shifted[N-1] keeps the vector's previous value (never written); through the host path the
    engine's own per-stream output buffer plays the reference's member vector."""
    n = 4099
    raw = O.synth_frames(2, n, O.CS8, tone_hz=900.0, fs=FS, seed=3)
    eng = S.Engine(S.SDRConfig(centerFrequency=CF, samplesPerReading=n, sampleRate=FS), 1)
    for f in range(2):
        spec, _, _ = eng.process(raw[f][None], fmt=S.CS8, stages=S.STAGE_SPECTRUM)
        assert spec[0][n - 1] == 0.0
    eng.close()

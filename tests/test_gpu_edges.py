"""GPU edge cases through the C ABI against the oracle (bars as in test_gpu_parity.py):

* partial batches at the benchmark frame size: 1 and 21 streams (the persistent spectrum kernel with fewer
  frames than workgroups, an SSB pipeline workgroup with 5 of its 16 streams live);
* degenerate frames: all-zero IQ (the statistics' log floors), full-scale DC (every sample -128 / -32768:
  one bin holds all the power, the SSB AGC and clamps saturate) and a full-scale Nyquist tone.
"""
import numpy as np
import pytest

from test_gpu_parity import assert_records_equal, engine, spectrum_ok

pytestmark = pytest.mark.gpu

N, FS = 16384, 2_000_000


@pytest.fixture(scope="module")
def S():
    import sdrg
    return sdrg


@pytest.fixture(scope="module")
def O():
    import oracle
    return oracle


def _check_calls(S, O, raw, fmt, n, fs):
    """raw [B][F][2n]: run F calls, compare every output with the oracle run stream by stream."""
    B, F = raw.shape[0], raw.shape[1]
    eng = engine(S, n, fs, B)
    fst = [O.FftState(100_000_000, fs, n, 5) for _ in range(B)]
    sst = [O.SsbState() for _ in range(B)]
    for f in range(F):
        now = 1000 + 200 * f
        spec, rec, pcm = eng.process(raw[:, f], fmt=fmt, now_ms=now)
        want = np.zeros(B, dtype=rec.dtype)
        for b in range(B):
            iq = O.unpack(fmt, raw[b, f], n)
            ok = spectrum_ok(spec[b], O.power_shifted(iq, use_f64=True))
            assert ok.all(), (b, f, np.argwhere(~ok)[:5].ravel())
            want[b] = fst[b].signal_strength(spec[b], now)
            np.testing.assert_array_equal(pcm[b], sst[b].process(iq, fs, 1), err_msg=f"pcm stream {b} call {f}")
        assert_records_equal(rec, want, msg=f"call {f}")
    eng.close()


@pytest.mark.parametrize("B", [1, 21])
def test_partial_batches(S, O, B):
    F = 2
    rng = np.random.default_rng(B)
    raw = np.stack([O.synth_frames(F, N, O.CS8, tone_hz=float(rng.uniform(-4000, 4000)), fs=FS, seed=50 + b)
                    for b in range(B)])
    _check_calls(S, O, raw, O.CS8, N, FS)


@pytest.mark.parametrize("fmt_name", ["CS8", "CS16"])
def test_degenerate_frames(S, O, fmt_name):
    fmt = getattr(O, fmt_name)
    dt, lo = (np.int8, -128) if fmt == O.CS8 else (np.int16, -32768)
    hi = -lo - 1
    zero = np.zeros(2 * N, dt)
    dc = np.full(2 * N, lo, dt)
    nyq = np.empty(2 * N, dt)
    nyq[0::2] = np.where(np.arange(N) % 2 == 0, hi, lo)  # I alternates full scale, Q = 0
    nyq[1::2] = 0
    frames = [zero, dc, nyq, zero]
    raw = np.stack([np.stack([frames[b], frames[(b + 1) % 4]]) for b in range(4)])  # [4][2 calls][2N]
    _check_calls(S, O, raw, fmt, N, FS)


def test_page_locked_host_buffers(S, O):
    """process(out=...) into sdrg.HostBuffer arrays (sdrg_host_alloc, page-locked) gives the same bytes as the
    default pageable arrays, with the input also page-locked."""
    B, n = 8, 4096
    raw = np.stack([O.synth_frames(1, n, O.CS8, tone_hz=700.0 * b - 2000.0, fs=FS, seed=90 + b)[0] for b in range(B)])
    e1, e2 = engine(S, n, FS, B), engine(S, n, FS, B)
    hb = [S.HostBuffer((B, 2 * n), np.int8), S.HostBuffer((B, n), np.float32), S.HostBuffer((B,), S.RECORD_DTYPE),
          S.HostBuffer((B, e2.pcm_len), np.int16)]
    hb[0].array[...] = raw
    for k in range(2):
        a = e1.process(raw, fmt=O.CS8, now_ms=1000 + 8 * k)
        b = e2.process(hb[0].array, fmt=O.CS8, now_ms=1000 + 8 * k, out=(hb[1].array, hb[2].array, hb[3].array))
        assert a[0].tobytes() == b[0].tobytes() and a[2].tobytes() == b[2].tobytes()
        for f in S.RECORD_DTYPE.names:  # fields: the struct's padding bytes are unspecified
            assert a[1][f].tobytes() == b[1][f].tobytes(), f
    with pytest.raises(S.SdrgError):
        e2.process(raw, fmt=O.CS8, out=(hb[1].array, None, hb[3].array))  # STATS requested, no records array
    for h in hb:
        h.close()
    e1.close()
    e2.close()

"""GPU parity of the NCO / short-FIR SSB variant (a build extension, include/sdrg.h sdrg_engine_set_ssb_variant)
against its CPU restatement (oracle/sdrg_oracle.c; pinned as described in tests/test_ssb_variant.py).

Bar: PCM bit-exact, every stream, every call (the NCO phase runs on across calls), through both SSB kernel
families: the pipelined kernel (2 MHz: decimation 41; LDS-DMA loader for whole 512-B batches, direct loads
otherwise) and the lane-per-stream kernels (250 kHz: decimation 5, which the pipeline does not cover).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def S():
    import sdrg
    return sdrg


@pytest.fixture(scope="module")
def O():
    import oracle
    return oracle


def _batch(O, B, F, n, fmt, fs, f_nco, seed):
    rng = np.random.default_rng(seed)
    raws = []
    for b in range(B):
        off = float(rng.uniform(-3000, 3000)) if b % 3 else float(rng.uniform(20e3, 90e3))
        raws.append(O.synth_frames(F, n, fmt, tone_hz=f_nco + off, fs=fs, seed=seed * 100 + b))
    return np.stack(raws)  # [B][F][2n]


@pytest.mark.parametrize("fmt_name,n,fs,f_nco,taps", [
    ("CS8", 16384, 2_000_000, 250e3, 127),      # the BASELINE configs[2] shape: pipeline, LDS-DMA loader
    ("CS16", 16384, 2_000_000, -312.5e3, 127),  # negative offset, CS16 DMA unpack
    ("CF32", 4000, 2_000_000, 61e3 + 0.37, 91),  # 4000 % 64 != 0: direct loads, partial last chunk
    ("CU8", 8192, 2_400_000, 480e3, 255),       # NCO only, reference FIR length
    ("CS8", 16384, 2_000_000, 0.0, 127),        # short FIR only, no mixer
    ("CS8", 4096, 250_000, 40e3, 127),          # decimation 5: the lane-per-stream kernels
])
def test_variant_pcm_bit_exact(S, O, fmt_name, n, fs, f_nco, taps):
    fmt = getattr(O, fmt_name)
    B, F = 48, 3
    raw = _batch(O, B, F, n, fmt, fs, f_nco, seed=n % 97 + taps)
    cfg = S.SDRConfig(centerFrequency=100_000_000, samplesPerReading=n, sampleRate=fs, freqFocusRangeKhz=5, soundMode=1)
    eng = S.Engine(cfg, B)
    eng.set_ssb_variant(f_nco, taps)
    v = eng.ssb_variant()
    assert v["fir_taps"] == taps and v["nco_increment"] == (O.nco_increment(f_nco, fs) if f_nco else 0)
    assert eng.pcm_len == O.ssb_pcm_len(n, fs, taps)
    sst = [O.SsbState() for _ in range(B)]
    for st in sst:
        st.set_variant(f_nco, fs, taps)
    for f in range(F):
        _, _, pcm = eng.process(raw[:, f], fmt=fmt, now_ms=1000 + 100 * f, stages=S.STAGE_SSB)
        assert pcm.shape == (B, eng.pcm_len)
        for b in range(B):
            want = sst[b].process(O.unpack(fmt, raw[b, f], n), fs, 1)
            np.testing.assert_array_equal(pcm[b], want, err_msg=f"{fmt_name} fs={fs} nco={f_nco} stream {b} call {f}")
        assert eng.ssb_variant()["nco_phase"] == (O.nco_increment(f_nco, fs) * n * (f + 1)) % 2**32 if f_nco else True
    eng.close()


def test_variant_switch_back_to_reference_chain(S, O):
    """Variant on for two calls, then off: the taps and chunk table are re-derived and the PCM is the reference
    chain's again (filter state carried through, as the restatement carries it)."""
    n, fs, B = 16384, 2_000_000, 32
    raw = _batch(O, B, 4, n, O.CS8, fs, 250e3, seed=5)
    cfg = S.SDRConfig(centerFrequency=100_000_000, samplesPerReading=n, sampleRate=fs, freqFocusRangeKhz=5, soundMode=1)
    eng = S.Engine(cfg, B)
    sst = [O.SsbState() for _ in range(B)]
    for f in range(4):
        on = f < 2
        eng.set_ssb_variant(250e3 if on else 0.0, 127 if on else 0) if f in (0, 2) else None
        if f in (0, 2):
            for st in sst:
                st.set_variant(250e3 if on else 0.0, fs, 127 if on else 0)
        _, _, pcm = eng.process(raw[:, f], fmt=O.CS8, now_ms=1000 + 100 * f, stages=S.STAGE_SSB)
        assert pcm.shape[1] == (397 if on else 394)
        for b in range(B):
            np.testing.assert_array_equal(pcm[b], sst[b].process(O.unpack(O.CS8, raw[b, f], n), fs, 1),
                                          err_msg=f"stream {b} call {f}")
    eng.close()


def test_variant_rejects_bad_arguments(S):
    cfg = S.SDRConfig(centerFrequency=100_000_000, samplesPerReading=4096, sampleRate=2_000_000)
    eng = S.Engine(cfg, 4)
    for taps in (2, 256, -1, 1):
        with pytest.raises(Exception):
            eng.set_ssb_variant(1e3, taps)
    with pytest.raises(Exception):
        eng.set_ssb_variant(float("nan"), 0)
    eng.close()

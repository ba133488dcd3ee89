"""CPU tests of the NCO / short-FIR SSB variant's CPU restatement (oracle/sdrg_oracle.c, include/sdrg.h
sdrg_engine_set_ssb_variant).

The variant is a BUILD EXTENSION named by BASELINE.json configs[2] ("SSB (USB) NCO + FIR-decimate to 48 kHz
PCM, 127-tap FIR"); the reference chain has no NCO and a 255-tap FIR (ssb_demod_opt.cpp:122, SURVEY.md
section 7h), so there is no reference output to pin it to ("parity unpinned" against the reference).  What
pins it instead:
  * with the variant off ((0 Hz, 0 taps) or (0 Hz, 255 taps)) the restatement is the reference-pinned chain,
    bit for bit (test_ssb_golden / test_oracle_* pin that chain to the reference build);
  * the NCO phasor agrees with e^{-j 2 pi ph / 2^32} in float64 to the table's truncation error;
  * the chain tunes: a tone at nco_hz + 1 kHz comes out as a 1 kHz tone, a tone at 0 Hz is rejected;
  * the phase is continuous across calls (a call's first sample continues the previous call's phase).
The GPU kernels are held to this restatement bit for bit (tests/test_gpu_ssb_variant.py).
"""
import numpy as np
import pytest

FS = 2_000_000
N = 16384


def _tone_iq(O, hz, n=N, frames=1, amp=0.5, seed=3, noise=None):
    return [O.unpack(O.CF32, f, n)
            for f in O.synth_frames(frames, n, O.CF32, tone_hz=hz, fs=FS, amp=amp, seed=seed, noise=noise)]


def test_variant_off_is_the_reference_chain(oracle_mod):
    O = oracle_mod
    frames = _tone_iq(O, 1800.0, frames=3)
    a, b, c = O.SsbState(), O.SsbState(), O.SsbState()
    b.set_variant(0.0, FS, 0)
    c.set_variant(0.0, FS, 255)
    for iq in frames:
        pa = a.process(iq, FS, 1)
        np.testing.assert_array_equal(pa, b.process(iq, FS, 1))
        np.testing.assert_array_equal(pa, c.process(iq, FS, 1))


def test_pcm_len_and_tap_count(oracle_mod):
    O = oracle_mod
    assert O.ssb_pcm_len(N, FS) == (N - 255) // 41 + 1 == 394
    assert O.ssb_pcm_len(N, FS, 127) == (N - 127) // 41 + 1 == 397
    h = np.zeros(256, np.float32)
    assert O.lib().oracle_fir_taps_n(N, 41, np.float32(0.45), 127, h.ctypes.data) == 127
    assert abs(float(h[:127].astype(np.float64).sum()) - 1.0) < 1e-5  # unity DC gain after normalisation
    np.testing.assert_allclose(h[:127], h[:127][::-1], rtol=1e-5, atol=1e-8)  # linear phase (to float rounding)
    assert O.lib().oracle_fir_taps_n(101, 41, np.float32(0.45), 127, h.ctypes.data) == 101  # n|1 when n < taps


@pytest.mark.parametrize("hz", [250e3, -250e3, 1234.5, -0.3, 999_999.0])
def test_nco_increment_and_phasor(oracle_mod, hz):
    O = oracle_mod
    inc = O.nco_increment(hz, FS)
    assert inc == int(round((hz / FS) % 1.0 * 2**32)) % 2**32
    L = O.lib()
    rng = np.random.default_rng(7)
    ph = rng.integers(0, 2**32, 2000, dtype=np.uint64)
    xr, xi = rng.uniform(-1, 1, 2000), rng.uniform(-1, 1, 2000)
    got = np.array([L.oracle_nco_mix(int(p), float(a), float(b)) for p, a, b in zip(ph, xr, xi)])
    want = np.real((xr.astype(np.float32) + 1j * xi.astype(np.float32)) * np.exp(-2j * np.pi * ph.astype(np.float64) / 2**32))
    # 12 truncated phase bits (2 pi 2^-20 rad) + float rounding of the tables and products
    assert np.max(np.abs(got - want)) < 1.2e-5


def _pcm_tone_hz(pcm):
    x = pcm.astype(np.float64)
    x = x - x.mean()
    p = np.abs(np.fft.rfft(x * np.hanning(x.size))) ** 2
    return np.argmax(p) * 48780.49 / x.size, float(np.sum(x ** 2))  # 2 MHz / 41 PCM rate


def test_variant_tunes_to_the_nco_frequency(oracle_mod):
    """A noise-free tone at nco_hz + 1 kHz: the variant brings it to 1 kHz; the reference chain (no NCO)
    leaves it 251 kHz out, where the low-pass rejects it."""
    O = oracle_mod
    f_nco = 250e3
    on = O.SsbState()
    on.set_variant(f_nco, FS, 127)
    plain = O.SsbState()
    plain.set_variant(0.0, FS, 127)
    pcm_on, pcm_off = [], []
    for iq in _tone_iq(O, f_nco + 1000.0, frames=6, noise=0.0):
        pcm_on.append(on.process(iq, FS, 1))
        pcm_off.append(plain.process(iq, FS, 1))
    assert all(p.size == 397 for p in pcm_on)
    f_peak, e_on = _pcm_tone_hz(np.concatenate(pcm_on[2:]))  # after the AGC settles
    assert abs(f_peak - 1000.0) < 60.0, f_peak
    _, e_off = _pcm_tone_hz(np.concatenate(pcm_off[2:]))
    assert e_off < 1e-3 * e_on, (e_off, e_on)


def test_phase_continuous_across_calls(oracle_mod):
    """A call's samples are mixed with phase inc * (k * samp_count + t): check through the chain's first stage
    (removeDC taps) against the same frame mixed with an explicitly offset phase."""
    O = oracle_mod
    f_nco = 123456.7
    inc = O.nco_increment(f_nco, FS)
    frames = _tone_iq(O, f_nco + 2500.0, frames=2, amp=0.4)
    st = O.SsbState()
    st.set_variant(f_nco, FS, 127)
    st.process(frames[0], FS, 1)
    _, taps = st.process(frames[1], FS, 1, stages=True)
    L = O.lib()
    iq = frames[1].reshape(-1, 2)
    ph0 = (inc * N) % 2**32
    mixed = np.array([L.oracle_nco_mix((ph0 + inc * t) % 2**32, float(iq[t, 0]), float(iq[t, 1])) for t in range(N)],
                     dtype=np.float32)
    dc = np.float32(0.0)
    want = np.empty(N, np.float32)
    for t in range(N):  # removeDC (:49-55), float32, no contraction
        dc = np.float32(np.float32(0.9995) * dc) + np.float32(np.float32(1.0) - np.float32(0.9995)) * mixed[t]
        want[t] = mixed[t] - dc
    np.testing.assert_array_equal(taps["dc_re"], want)

"""GPU parity tests of the pulse detectors (csrc/pulse.hip) through the C ABI.

Bar: bit-exact.  The detectors are integer/branch state machines over float inputs whose float (and, for
the frequency estimate, double) expressions the kernels replay in the reference's order, so every getter
value must equal the reference's bit for bit:
  * against tests/golden/pulse_*.npz (the reference's own spectral_pulse_detector.cpp /
    audio_pulse_detector.cpp, oracle/_ref/ref_pulse), with thousands of streams per call;
  * end to end in the engine: the spectral detector against the oracle fed with the GPU's own per-frame
    records, the audio detector against the oracle fed with the GPU's own PCM (isolates the detectors from
    the FFT's float tolerance), including the callbacks' arguments.
"""
import numpy as np
import pytest

import pulse_inputs as PI
from conftest import load_golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def S():
    import sdrg
    return sdrg


@pytest.fixture(scope="module")
def O():
    import oracle
    return oracle


def _one(rec):
    """A single np.void output record as a length-1 array."""
    return np.array([rec], dtype=rec.dtype)


def _same(ref, got, fields, msg=""):
    for k in fields:
        a, b = np.ascontiguousarray(ref[k]), np.ascontiguousarray(got[k])
        if a.dtype.kind == "f":
            a, b = a.view(np.uint32), b.view(np.uint32)
        bad = np.flatnonzero(a != b)
        assert bad.size == 0, f"{msg} {k}: {bad.size} differ, first at {bad[0]}: want {ref[k][bad[0]]} got {got[k][bad[0]]}"


def test_spectral_bank_vs_reference_fixtures_many_streams(S, O):
    """4096 streams, stream s running fixture case s % 7 (all at fsEnergy = 2 MHz / 16384), 3300 frames."""
    g = load_golden("pulse_spectral")
    cases = [c for c in PI.SPECTRAL_CASES if c[1] == float(PI.FS16K)]
    ins = [PI.spectral_case(n=c[2], fs_energy=c[1], **c[3]) for c in cases]
    n_frames = cases[0][2]
    B = 4096
    idx = np.arange(B) % len(cases)
    X = np.stack([ins[k][0] for k in range(len(cases))])[idx]  # [B][frames]
    F = np.stack([ins[k][1] for k in range(len(cases))])[idx]
    bank = S.PulseBank(S.PULSE_SPECTRAL, B, S.PulseConfig.default(S.PULSE_SPECTRAL, fs_energy=float(PI.FS16K)))
    outs = np.empty((n_frames, B), S.PULSE_OUTPUT_DTYPE)
    for f in range(n_frames):
        outs[f] = bank.process_spectral(X[:, f], F[:, f])
    for k, c in enumerate(cases):
        for s in (k, k + len(cases) * 300, B - len(cases) + k):
            if s % len(cases) == k and s < B:
                _same(g[c[0]], outs[:, s], O.PULSE_REF_FIELDS, f"{c[0]} stream {s}")
    assert outs["overflow"].max() == 0


def test_spectral_bank_configure_regrow_and_reset(S, O):
    """configure() keeps the state, including across a ring regrow (fsEnergy 20 -> 40); reset() restarts."""
    g = load_golden("pulse_spectral")
    name, fs, n, kw, (k_re, fs2) = [c for c in PI.SPECTRAL_CASES if c[0] == "reconfigure"][0]
    x, f = PI.spectral_case(n=n, fs_energy=fs, **kw)
    B = 3
    bank = S.PulseBank(S.PULSE_SPECTRAL, B, S.PulseConfig.default(S.PULSE_SPECTRAL, fs_energy=fs))
    outs = []
    for t in range(n):
        if t == k_re:
            bank.configure(S.PulseConfig.default(S.PULSE_SPECTRAL, fs_energy=fs2))
        outs.append(bank.process_spectral(np.full(B, x[t]), np.full(B, f[t])))
    outs = np.stack(outs)
    for s in range(B):
        _same(g[name], outs[:, s], O.PULSE_REF_FIELDS, f"stream {s}")
    bank.reset()
    bank.configure(S.PulseConfig.default(S.PULSE_SPECTRAL, fs_energy=fs))
    again = np.stack([bank.process_spectral(np.full(B, x[t]), np.full(B, f[t])) for t in range(k_re)])
    _same(g[name][:k_re], again[:, 0], O.PULSE_REF_FIELDS, "after reset")


@pytest.mark.parametrize("case", PI.AUDIO_CASES, ids=[c[0] for c in PI.AUDIO_CASES])
def test_audio_bank_vs_reference_fixtures(S, O, case):
    """256 streams: even streams carry the fixture case, odd streams a time-reversed copy (checked
    against the oracle) so neighbouring streams never share a trajectory."""
    name, n, block, kw = case
    g = load_golden("pulse_audio")
    s = PI.audio_case(n=n, **kw)
    B = 256
    rev = s[::-1].copy()
    bank = S.PulseBank(S.PULSE_AUDIO, B)
    outs = []
    for k in range(0, n, block):
        a, b = s[k:k + block], rev[k:k + block]
        blk = np.empty((B, a.size), np.int16)
        blk[0::2] = a
        blk[1::2] = b
        outs.append(bank.process_audio(blk))
    outs = np.stack(outs)
    fields = ("strength", "live_etat", "level", "locked", "period_s", "input")
    for st in (0, 2, B - 2):
        _same(g[name], outs[:, st], fields, f"{name} stream {st}")
    want_rev = O.PulseDetector(O.PULSE_AUDIO).audio_blocks(rev, block)
    _same(want_rev, outs[:, 1], fields, f"{name} reversed")
    _same(want_rev, outs[:, B - 1], fields, f"{name} reversed")


def test_audio_bank_float_input_and_empty_blocks(S, O):
    s = PI.audio_case(seed=21, n=48000 * 6, period=1.3)
    x = (s.astype(np.float32) * np.float32(1.0 / 20000.0)).astype(np.float32)
    B = 4
    bank = S.PulseBank(S.PULSE_AUDIO, B)
    ref = O.PulseDetector(O.PULSE_AUDIO)
    for k in range(0, x.size, 700):
        blk = np.repeat(x[None, k:k + 700], B, axis=0)
        got = bank.process_audio(blk)
        want = ref.audio(x[k:k + 700])
        empty = bank.process_audio(np.zeros((B, 0), np.float32))  # process(empty pcm): state unchanged
        for st in range(B):
            _same(_one(want), got[st:st + 1], ("strength", "live_etat", "level", "locked", "period_s"))
            _same(_one(want), empty[st:st + 1], ("strength", "live_etat", "level", "locked", "period_s"))


def _beacon_frames(n_streams, n, fs, frame0, n_frames, seed=5):
    """CS8 IQ: a +2 kHz carrier keyed on for 0.15 s every 1.75 s (a different phase per stream) over noise."""
    rng = np.random.default_rng(seed + frame0)
    t0 = (frame0 + np.arange(n_frames))[:, None, None] * n + np.arange(n)[None, None, :]
    t = t0 / fs
    phase0 = 0.37 * np.arange(n_streams)[None, :, None]
    on = (np.mod(t + phase0, 1.75) < 0.15).astype(np.float64)
    amp = 4.0 + 40.0 * on
    ph = 2 * np.pi * 2000.0 * t
    shape = (n_frames, n_streams, n)
    i = amp * np.cos(ph) + rng.normal(0, 6.0, shape)
    q = amp * np.sin(ph) + rng.normal(0, 6.0, shape)
    iq = np.empty((n_frames, n_streams, 2 * n), np.int8)
    iq[..., 0::2] = np.clip(np.round(i), -128, 127)
    iq[..., 1::2] = np.clip(np.round(q), -128, 127)
    return iq


def test_engine_pulse_stages_end_to_end(S, O):
    """Engine with STAGE_ALL over 520 frames (4.3 s at 2 MHz / 16384): the spectral and audio detectors must
    equal the oracle detectors fed the engine's own records and PCM, and the callbacks must carry them."""
    n, fs, B, T = 16384, 2_000_000, 6, 520
    cfg = S.SDRConfig(centerFrequency=100_000_000, samplesPerReading=n, sampleRate=fs, freqFocusRangeKhz=5,
                      soundMode=1)
    eng = S.Engine(cfg, B)
    cb_spec, cb_audio = [], []
    eng.read(spectralPulseCallback=lambda s, a, b, c: cb_spec.append((s, a, b, c)),
             audioPulseCallback=lambda s, a, b: cb_audio.append((s, a, b)))
    fs_e = float(np.float32(fs) / np.float32(n))
    o_spec = [O.PulseDetector(O.PULSE_SPECTRAL, fs_energy=fs_e) for _ in range(B)]
    o_aud = [O.PulseDetector(O.PULSE_AUDIO) for _ in range(B)]
    live_seen = 0
    for f0 in range(0, T, 40):
        frames = _beacon_frames(B, n, fs, f0, 40)
        for k in range(frames.shape[0]):
            cb_spec.clear()
            cb_audio.clear()
            _, rec, pcm = eng.process(frames[k], fmt=S.CS8, stages=S.STAGE_ALL, now_ms=1000 + f0 + k)
            ps, pa = eng.pulse_outputs()
            for s in range(B):
                ws = o_spec[s].spectral(rec["best1khz_snr_sigma"][s:s + 1], rec["best1khz_center_freq_hz"][s:s + 1])
                _same(ws, ps[s:s + 1], O.PULSE_REF_FIELDS, f"spectral frame {f0 + k} stream {s}")
                wa = o_aud[s].audio(pcm[s])
                _same(_one(wa), pa[s:s + 1], ("strength", "live_etat", "level", "locked", "period_s"),
                      f"audio frame {f0 + k} stream {s}")
                assert cb_spec[s][0] == s and np.float32(cb_spec[s][1]) == ws["input"][0]
                assert cb_spec[s][2] == ws["live_etat"][0] and cb_spec[s][3] == ws["est_freq_hz_rounded"][0]
                assert cb_audio[s][0] == s and np.float32(cb_audio[s][1]) == wa["strength"]
                assert cb_audio[s][2] == wa["live_etat"]
            live_seen = max(live_seen, int(ps["live_etat"].max()), int(pa["live_etat"].max()))
    assert live_seen >= 1, "the beacon never produced an admitted ROI: the test proves little"


def test_engine_pulse_stage_dependencies(S):
    cfg = S.SDRConfig(centerFrequency=100_000_000, samplesPerReading=4096, sampleRate=2_000_000)
    eng = S.Engine(cfg, 2)
    iq = np.zeros((2, 2 * 4096), np.int8)
    with pytest.raises(S.SdrgError):
        eng.process(iq, fmt=S.CS8, stages=S.STAGE_SPECTRUM | S.STAGE_SPECTRAL_PULSE)
    with pytest.raises(S.SdrgError):
        eng.process(iq, fmt=S.CS8, stages=S.STAGE_SPECTRUM | S.STAGE_AUDIO_PULSE)
    eng.process(iq, fmt=S.CS8, stages=S.STAGE_ALL)
    sp, au = eng.pulse_outputs()
    assert (sp["live_etat"] == 0).all() and (au["live_etat"] == 0).all() and (sp["n_energy"] == 1).all()


@pytest.mark.parametrize("case", PI.SPECTRAL_CUSTOM_CASES, ids=[c[0] for c in PI.SPECTRAL_CUSTOM_CASES])
def test_spectral_bank_custom_config_vs_reference(S, O, case):
    name, fs, n, kw, ov = case
    g = load_golden("pulse_spectral")
    x, f = PI.spectral_case(n=n, fs_energy=fs, **kw)
    B = 70  # not a multiple of 64
    bank = S.PulseBank(S.PULSE_SPECTRAL, B, S.PulseConfig.default(S.PULSE_SPECTRAL, fs_energy=fs,
                                                                  **O.pulse_overrides(ov)))
    outs = np.stack([bank.process_spectral(np.full(B, x[t]), np.full(B, f[t])) for t in range(n)])
    for s in (0, 63, 64, B - 1):
        _same(g[name], outs[:, s], O.PULSE_REF_FIELDS, f"{name} stream {s}")


@pytest.mark.parametrize("case", PI.AUDIO_CUSTOM_CASES, ids=[c[0] for c in PI.AUDIO_CUSTOM_CASES])
def test_audio_bank_custom_config_vs_reference(S, O, case):
    """Custom band / noise reference / rates, 67 streams (the front-end kernel's last wave partly empty)."""
    name, n, block, kw, ov = case
    g = load_golden("pulse_audio")
    s = PI.audio_case(n=n, **kw)
    B = 67
    bank = S.PulseBank(S.PULSE_AUDIO, B, S.PulseConfig.default(S.PULSE_AUDIO, **O.pulse_overrides(ov)))
    outs = np.stack([bank.process_audio(np.repeat(s[None, k:k + block], B, axis=0)) for k in range(0, n, block)])
    for st in (0, 63, 64, B - 1):
        _same(g[name], outs[:, st], ("strength", "live_etat", "level", "locked", "period_s", "input"), f"{name} {st}")

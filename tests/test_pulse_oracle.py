"""CPU tests: pin the pulse-detector oracle (oracle/pulse_oracle.c) before trusting it as the checker.

* Against tests/golden/pulse_{spectral,audio}.npz: outputs of the reference's own
  spectral_pulse_detector.cpp / audio_pulse_detector.cpp (oracle/_ref/ref_pulse), bit for bit, over the
  deterministic cases of tests/pulse_inputs.py (lock, period switch, jitter and missed pulses, confusion
  spikes, noise only, a mid-run configure(), >10 s energy-buffer trimming and >20 s ROI trimming).
* When the reference build exists (container only): fresh reference runs on extra random cases.
"""
import os

import numpy as np
import pytest

import pulse_inputs as PI
from conftest import load_golden


def _same(ref, got, fields):
    for k in fields:
        a, b = np.ascontiguousarray(ref[k]), np.ascontiguousarray(got[k])
        if a.dtype.kind == "f":
            a, b = a.view(np.uint32), b.view(np.uint32)
        bad = np.flatnonzero(a != b)
        assert bad.size == 0, f"{k}: {bad.size} frames differ, first at {bad[0]}: ref {ref[k][bad[0]]} got {got[k][bad[0]]}"


def _run_spectral(O, fs, x, f, reconf):
    d = O.PulseDetector(O.PULSE_SPECTRAL, fs_energy=fs)
    if reconf is None:
        return d.spectral(x, f)
    k, fs2 = reconf
    a = d.spectral(x[:k], f[:k])
    d.configure(fs_energy=fs2)  # SpectralPulseDetector::configure: state kept
    return np.concatenate([a, d.spectral(x[k:], f[k:])])


@pytest.mark.parametrize("case", PI.SPECTRAL_CASES, ids=[c[0] for c in PI.SPECTRAL_CASES])
def test_spectral_oracle_matches_reference_fixture(oracle_mod, case):
    O = oracle_mod
    name, fs, n, kw, reconf = case
    g = load_golden("pulse_spectral")
    x, f = PI.spectral_case(n=n, fs_energy=fs, **kw)
    assert PI.digest(x, f) == str(g[name + "__digest"]), "input generator drifted"
    _same(g[name], _run_spectral(O, fs, x, f, reconf), O.PULSE_REF_FIELDS)


@pytest.mark.parametrize("case", PI.AUDIO_CASES, ids=[c[0] for c in PI.AUDIO_CASES])
def test_audio_oracle_matches_reference_fixture(oracle_mod, case):
    O = oracle_mod
    name, n, block, kw = case
    g = load_golden("pulse_audio")
    s = PI.audio_case(n=n, **kw)
    assert PI.digest(s) == str(g[name + "__digest"]), "input generator drifted"
    got = O.PulseDetector(O.PULSE_AUDIO).audio_blocks(s, block)
    _same(g[name], got, ("strength", "live_etat", "level", "locked", "period_s", "input"))


def test_fixtures_exercise_the_state_machine():
    """The fixtures must reach every live state band, lock, and the trimming paths (else they prove little)."""
    g = load_golden("pulse_spectral")
    live = np.concatenate([g[c[0]]["live_etat"] for c in PI.SPECTRAL_CASES])
    assert set(np.unique(live)) >= {0, 1, 2, 3, 4, 5}
    assert any(g[c[0]]["locked"].any() for c in PI.SPECTRAL_CASES)
    assert not g["noise_only"]["live_etat"].any()
    assert len(g["beacon_clean"]) / float(PI.FS16K) > 20.0  # > 20 s: ROI trim + 10 s buffer trim
    a = load_golden("pulse_audio")
    assert a["burst_394"]["live_etat"].max() == 5 and a["burst_394"]["locked"].any()


def test_spectral_reset_and_defaults(oracle_mod):
    O = oracle_mod
    c = O.pulse_config_default(O.PULSE_SPECTRAL)[0]
    assert np.float32(c["fs_energy"]) == np.float32(20.0) and np.float32(c["snr_strong"]) == np.float32(4.0)
    c = O.pulse_config_default(O.PULSE_AUDIO)[0]
    assert np.float32(c["fs_energy"]) == np.float32(100.0) and c["noise_ref_far"] == 80
    x, f = PI.spectral_case(seed=1, n=800, fs_energy=float(PI.FS16K))
    d = O.PulseDetector(O.PULSE_SPECTRAL, fs_energy=float(PI.FS16K))
    a = d.spectral(x, f)
    d.reset()
    b = d.spectral(x, f)
    _same(a, b, O.PULSE_REF_FIELDS)


@pytest.mark.skipif(not os.path.exists(os.path.join(os.path.dirname(__file__), "..", "oracle", "_ref", "ref_pulse")),
                    reason="reference build (oracle/_ref) only exists where /root/reference is mounted")
@pytest.mark.parametrize("seed", [101, 202, 303])
def test_oracle_matches_reference_live(oracle_mod, seed):
    O = oracle_mod
    rng = np.random.default_rng(seed)
    fs = float(np.float32(rng.choice([20.0, 61.03515625, 122.0703125, 244.140625])))
    n = int(fs * 26)
    x, f = PI.spectral_case(seed=seed, n=n, fs_energy=fs, period=float(rng.uniform(0.8, 3.0)),
                            amp=float(rng.uniform(1.5, 8.0)), jitter=float(rng.uniform(0.0, 0.2)),
                            miss=float(rng.uniform(0.0, 0.3)), extra=float(rng.uniform(0.0, 0.003)))
    _same(O.ref_pulse_spectral(x, f, fs), _run_spectral(O, fs, x, f, None), O.PULSE_REF_FIELDS)
    s = PI.audio_case(seed=seed, n=48000 * 8, period=float(rng.uniform(0.6, 2.5)), amp=int(rng.integers(500, 9000)))
    block = int(rng.choice([97, 394, 480, 1256]))
    _same(O.ref_pulse_audio(s, block), O.PulseDetector(O.PULSE_AUDIO).audio_blocks(s, block),
          ("strength", "live_etat", "level", "locked", "period_s"))


@pytest.mark.parametrize("case", PI.SPECTRAL_CUSTOM_CASES, ids=[c[0] for c in PI.SPECTRAL_CUSTOM_CASES])
def test_spectral_oracle_custom_config_matches_reference(oracle_mod, case):
    O = oracle_mod
    name, fs, n, kw, ov = case
    g = load_golden("pulse_spectral")
    x, f = PI.spectral_case(n=n, fs_energy=fs, **kw)
    assert PI.digest(x, f) == str(g[name + "__digest"])
    d = O.PulseDetector(O.PULSE_SPECTRAL, fs_energy=fs, **O.pulse_overrides(ov))
    _same(g[name], d.spectral(x, f), O.PULSE_REF_FIELDS)


@pytest.mark.parametrize("case", PI.AUDIO_CUSTOM_CASES, ids=[c[0] for c in PI.AUDIO_CUSTOM_CASES])
def test_audio_oracle_custom_config_matches_reference(oracle_mod, case):
    O = oracle_mod
    name, n, block, kw, ov = case
    g = load_golden("pulse_audio")
    s = PI.audio_case(n=n, **kw)
    assert PI.digest(s) == str(g[name + "__digest"])
    got = O.PulseDetector(O.PULSE_AUDIO, **O.pulse_overrides(ov)).audio_blocks(s, block)
    _same(g[name], got, ("strength", "live_etat", "level", "locked", "period_s", "input"))

"""Generate tests/golden/pulse_spectral.npz and pulse_audio.npz (run in the container that has /root/reference).

Expected outputs come from the REFERENCE's own src/dsp/spectral_pulse_detector.cpp and
src/ssb/audio_pulse_detector.cpp, built unmodified by `make -C oracle ref` into oracle/_ref/ref_pulse
(driver: oracle/ref_pulse_driver.cpp).  Inputs are the deterministic cases of tests/pulse_inputs.py; each
case stores the SHA-256 of its generated input so a test can tell a generator drift from a parity failure.
Only the fields the reference getters expose are meaningful (oracle.PULSE_REF_FIELDS).

    make -C oracle ref && python tests/golden/make_pulse_golden.py
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle as O  # noqa: E402
import pulse_inputs as PI  # noqa: E402


def main() -> None:
    assert O.have_ref() and os.path.exists(O.REF_PULSE), "run `make -C oracle ref` first"
    spec = {}
    for name, fs, n, kw, reconf in PI.SPECTRAL_CASES:
        x, f = PI.spectral_case(n=n, fs_energy=fs, **kw)
        spec[name] = O.ref_pulse_spectral(x, f, fs, reconf)
        spec[name + "__digest"] = np.array(PI.digest(x, f))
    for name, fs, n, kw, ov in PI.SPECTRAL_CUSTOM_CASES:
        x, f = PI.spectral_case(n=n, fs_energy=fs, **kw)
        spec[name] = O.ref_pulse_spectral(x, f, fs, None, ov)
        spec[name + "__digest"] = np.array(PI.digest(x, f))
    np.savez_compressed(os.path.join(HERE, "pulse_spectral.npz"), **spec)
    aud = {}
    for name, n, block, kw in PI.AUDIO_CASES:
        s = PI.audio_case(n=n, **kw)
        aud[name] = O.ref_pulse_audio(s, block)
        aud[name + "__digest"] = np.array(PI.digest(s))
    for name, n, block, kw, ov in PI.AUDIO_CUSTOM_CASES:
        s = PI.audio_case(n=n, **kw)
        aud[name] = O.ref_pulse_audio(s, block, ov)
        aud[name + "__digest"] = np.array(PI.digest(s))
    np.savez_compressed(os.path.join(HERE, "pulse_audio.npz"), **aud)
    print("wrote pulse_spectral.npz, pulse_audio.npz")


if __name__ == "__main__":
    main()

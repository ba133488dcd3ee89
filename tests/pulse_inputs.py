"""Deterministic synthetic inputs for the pulse-detector parity tests and fixtures.

Everything is built from a counter-based integer hash (splitmix64 over numpy uint64) and IEEE float64
+ - * / only (no libm transcendental), so the same bytes come out on any machine; the fixtures in
tests/golden/pulse_*.npz also store a SHA-256 of the generated inputs, which the tests check first.

  spectral_case(...)  -> (snr_sigma float32[n], freq_hz float32[n])  one value pair per FFT frame, a
                         pulsed beacon in best1kHzSnrSigma units over a noisy floor plus a drifting
                         best-1-kHz centre frequency (the inputs SpectralPulseDetector::process receives,
                         sdr-bridge-java-soapy.cpp:477-479)
  audio_case(...)     -> int16[n] PCM at 48 kHz: 2 kHz triangle-wave bursts in noise (the SSB output
                         AudioPulseDetector::process receives, ssb_processor.cpp:109)
"""
from __future__ import annotations

import hashlib

import numpy as np

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix(seed: int, idx: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = (np.uint64(seed) * np.uint64(0x9E3779B97F4A7C15) + idx.astype(np.uint64) * np.uint64(0xBF58476D1CE4E5B9)) & _M64
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def uniform(seed: int, n: int, lane: int = 0) -> np.ndarray:
    """float64 uniforms in [0, 1) from the top 53 bits of the hash of (seed, 4*i + lane)."""
    idx = np.arange(n, dtype=np.uint64) * np.uint64(4) + np.uint64(lane)
    return (_splitmix(seed, idx) >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def gaussish(seed: int, n: int) -> np.ndarray:
    """Approximately unit-variance noise: (sum of 4 uniforms - 2) * sqrt(3)."""
    s = uniform(seed, n, 0) + uniform(seed, n, 1) + uniform(seed, n, 2) + uniform(seed, n, 3)
    return (s - 2.0) * 1.7320508075688772


def _pulse_times(seed: int, duration: float, period: float, jitter: float, miss: float, t_first: float):
    k = int(duration / period) + 2
    u = uniform(seed ^ 0x5A5A, k, 0)
    m = uniform(seed ^ 0xA5A5, k, 1)
    times = t_first + np.arange(k) * period + (u - 0.5) * 2.0 * jitter
    return times[m >= miss]


def spectral_case(seed: int, n: int, fs_energy: float, period: float = 1.75, width: float = 0.12,
                  amp: float = 6.0, floor: float = 0.3, noise: float = 0.6, jitter: float = 0.03,
                  miss: float = 0.0, f0: float = 100004800.0, drift: float = 3.0, fnoise: float = 40.0,
                  period2: float | None = None, switch_t: float = 0.0, extra: float = 0.0):
    t = np.arange(n) / fs_energy
    dur = n / fs_energy
    x = floor + noise * gaussish(seed, n)
    times = _pulse_times(seed, dur, period, jitter, miss, 0.9)
    if period2 is not None:  # the beacon changes period at switch_t
        t2 = _pulse_times(seed ^ 0x77, dur, period2, jitter, miss, switch_t)
        times = np.concatenate([times[times < switch_t], t2[t2 >= switch_t]])
    amps = amp * (0.6 + 0.8 * uniform(seed ^ 0x1234, len(times), 2))
    for tk, ak in zip(times, amps):
        x = x + ak * np.maximum(0.0, 1.0 - np.abs(t - tk) / width)
    if extra > 0.0:  # spurious isolated spikes (confusion)
        sp = uniform(seed ^ 0x4321, n, 3) < extra
        x = x + sp * amp * 0.9
    f = f0 + drift * t + fnoise * gaussish(seed ^ 0x9999, n)
    return x.astype(np.float32), f.astype(np.float32)


def audio_case(seed: int, n: int, period: float = 1.75, burst: float = 0.2, amp: int = 6000,
               noise: float = 900.0, jitter: float = 0.02, miss: float = 0.0, rate: float = 48000.0,
               hum: int = 0):
    t = np.arange(n) / rate
    times = _pulse_times(seed, n / rate, period, jitter, miss, 0.8)
    gate = np.zeros(n, dtype=np.float64)
    for tk in times:
        gate = np.maximum(gate, ((t >= tk) & (t < tk + burst)).astype(np.float64))
    ph = np.arange(n) % 24  # 2 kHz triangle at 48 kHz: 24-sample period
    tri = np.where(ph < 12, ph - 6, 18 - ph).astype(np.float64) / 6.0
    x = amp * gate * tri + noise * gaussish(seed, n)
    if hum:  # out-of-band 250 Hz square wave (192-sample period), removed by the band-pass
        x = x + hum * np.where((np.arange(n) % 192) < 96, 1.0, -1.0)
    return np.clip(np.round(x), -32768, 32767).astype(np.int16)


def digest(*arrays: np.ndarray) -> str:
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


# The fixture cases.  fs_energy 122.0703125 = 2 MHz / 16384 (the bench configuration, what applyConfig
# sets, sdr-bridge-java-soapy.cpp:1130-1138); 20 is the detector's own default.
FS16K = np.float32(2e6) / np.float32(16384)
SPECTRAL_CASES = [
    # name, fs_energy, n_frames, kwargs, reconfigure (frame, fs2) or None
    ("beacon_clean", float(FS16K), 3300, dict(seed=1), None),
    ("beacon_weak", float(FS16K), 3300, dict(seed=2, amp=2.6, noise=0.5), None),
    ("beacon_jitter_miss", float(FS16K), 3300, dict(seed=3, jitter=0.12, miss=0.25), None),
    ("period_switch", float(FS16K), 3300, dict(seed=4, period=1.2, period2=2.1, switch_t=12.0), None),
    ("noise_only", float(FS16K), 3300, dict(seed=5, amp=0.0, noise=1.1), None),
    ("confusion", float(FS16K), 3300, dict(seed=6, extra=0.004, jitter=0.2), None),
    ("fast_beacon", float(FS16K), 3300, dict(seed=7, period=0.6, width=0.05), None),
    ("default_fs20", 20.0, 700, dict(seed=8, width=0.3), None),
    ("reconfigure", 20.0, 900, dict(seed=9, width=0.3), (400, 40.0)),
]
AUDIO_CASES = [
    # name, n_samples, block, kwargs
    ("burst_394", 48000 * 24, 394, dict(seed=11)),
    ("weak_394", 48000 * 24, 394, dict(seed=12, amp=1500, noise=700.0, miss=0.2)),
    ("hum_noise_1000", 48000 * 24, 1000, dict(seed=13, amp=0, hum=4000)),
    ("fast_100", 48000 * 12, 100, dict(seed=14, period=0.7, burst=0.08, hum=2500)),
]

# Non-default configurations (reference Config field names), pinned against the reference build too.
SPECTRAL_CUSTOM_CASES = [
    # name, fs_energy, n_frames, input kwargs, Config overrides
    ("custom_thresholds", float(FS16K), 2600, dict(seed=31, amp=3.2, jitter=0.08),
     {"snrMin": 1.2, "snrRhythm": 2.0, "snrStrong": 3.0, "liveDivisor": 2.0, "liveWindowT": 3.0}),
    ("custom_period", 40.0, 1200, dict(seed=32, period=2.6, width=0.25),
     {"tTargetInit": 2.5, "dtTolS": 0.25, "zDefaultS": 1.0, "sumNMax": 5, "dispersionMax": 0.9}),
]
AUDIO_CUSTOM_CASES = [
    # name, n_samples, block, input kwargs, Config overrides
    ("custom_band_noise_ref", 48000 * 16, 394, dict(seed=41, amp=2500, noise=600.0),
     {"fMin": 1200.0, "fMax": 3000.0, "noiseRefFar": 60, "noiseRefNear": 25, "snrStrong": 1.8, "snrMin": 1.05}),
    ("custom_rates", 32000 * 16, 512, dict(seed=42, rate=32000.0, period=1.4),
     {"sampleRate": 32000.0, "fsEnergy": 50.0, "smoothCutoff": 4.0, "tTargetInit": 1.4, "liveDivisor": 2.5}),
]


"""ctypes binding of oracle/liboracle.so — TEST INFRASTRUCTURE ONLY.

The CPU restatement of the reference hot path (see sdrg_oracle.c's header for what it restates and how
it is pinned).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module; the product package never does.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
REF_SSB = os.path.join(HERE, "_ref", "ref_ssb")

# include/sdrg.h formats / stages
CF32, CS8, CU8, CS16 = 0, 1, 2, 3
STAGE_SPECTRUM, STAGE_STATS, STAGE_SSB, STAGE_HOT_PATH = 1, 2, 4, 7
STAGE_SPECTRAL_PULSE, STAGE_AUDIO_PULSE, STAGE_ALL = 8, 16, 31

RECORD_DTYPE = np.dtype(
    [
        ("tracking_frequency", "<i8"),
        ("mean_snr_db", "<f4"),
        ("mean_snr_sigma", "<f4"),
        ("peak_above_noise_mean_db", "<f4"),
        ("max_bin_snr_db", "<f4"),
        ("max_bin_snr_sigma", "<f4"),
        ("best1khz_snr_db", "<f4"),
        ("best1khz_snr_sigma", "<f4"),
        ("best1khz_center_freq_hz", "<f4"),
        ("per_bin_mean", "<f4"),
        ("detection_flag", "<i4"),
        ("peak_bin", "<i4"),
        ("abs_peak_db", "<f4"),
        ("signal_power_db", "<f4"),
        ("valid", "<i4"),
        ("n_ref_windows", "<i4"),
    ],
    align=True,
)

# include/sdrg.h sdrg_pulse_config / sdrg_pulse_output
PULSE_SPECTRAL, PULSE_AUDIO = 0, 1
PULSE_CONFIG_DTYPE = np.dtype(
    [(k, "<f4") for k in ("fs_energy", "z_default_s", "t_target_init", "dt_tol_s", "snr_min", "snr_rhythm",
                          "snr_strong", "dispersion_max")]
    + [("sum_n_max", "<i4"), ("live_window_t", "<f4"), ("live_divisor", "<f4"), ("sample_rate", "<f4"),
       ("f_min", "<f4"), ("f_max", "<f4"), ("smooth_cutoff", "<f4"), ("noise_ref_far", "<i4"),
       ("noise_ref_near", "<i4")],
    align=True,
)
PULSE_OUTPUT_DTYPE = np.dtype(
    [
        ("strength", "<f4"),
        ("live_etat", "<i4"),
        ("level", "<i4"),
        ("locked", "<i4"),
        ("period_s", "<f4"),
        ("est_freq_hz", "<f4"),
        ("est_freq_hz_rounded", "<i8"),
        ("input", "<f4"),
        ("n_energy", "<i4"),
        ("n_rois", "<i4"),
        ("overflow", "<i4"),
    ],
    align=True,
)
# fields the reference getters expose (n_energy / n_rois / overflow are engine diagnostics)
PULSE_REF_FIELDS = ("strength", "live_etat", "level", "locked", "period_s", "est_freq_hz", "est_freq_hz_rounded",
                    "input")

_lib = None


def build() -> None:
    """Compile liboracle.so (and, when /root/reference exists, oracle/_ref/ref_ssb)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    if os.path.isdir("/root/reference/src/ssb"):
        subprocess.run(["make", "-s", "-C", HERE, "ref"], check=True)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        i32, i64, u32, f32 = ctypes.c_int32, ctypes.c_int64, ctypes.c_uint32, ctypes.c_float
        sig = {
            "oracle_unpack": (ctypes.c_int, [ctypes.c_int, P, i64, P]),
            "oracle_power_shifted": (ctypes.c_int, [P, ctypes.c_int, ctypes.c_int, P]),
            "oracle_fft_state_size": (ctypes.c_int, []),
            "oracle_fft_state_init": (None, [P]),
            "oracle_fft_configure": (None, [P, u32, u32, i32, i32]),
            "oracle_fft_set_center_frequency_changed": (None, [P]),
            "oracle_window_geometry": (ctypes.c_int, [u32, i32, i32, P, P, P, P, P]),
            "oracle_signal_strength": (ctypes.c_int, [P, P, i32, i64, P]),
            "oracle_fft_process": (ctypes.c_int, [P, P, i32, i64, ctypes.c_int, P, P]),
            "oracle_ssb_state_size": (ctypes.c_int, []),
            "oracle_ssb_state_init": (None, [P]),
            "oracle_iir2_lowpass": (None, [f32, f32, f32, P]),
            "oracle_biquad_highpass": (None, [f32, f32, f32, P]),
            "oracle_biquad_bandpass": (None, [f32, f32, f32, P]),
            "oracle_fir_taps": (ctypes.c_int, [i64, ctypes.c_int, f32, P]),
            "oracle_ssb_decim": (ctypes.c_int, [u32]),
            "oracle_ssb_pcm_len": (ctypes.c_int, [i64, u32]),
            "oracle_ssb_pcm_len_n": (ctypes.c_int, [i64, u32, ctypes.c_int]),
            "oracle_fir_taps_n": (ctypes.c_int, [i64, ctypes.c_int, f32, ctypes.c_int, P]),
            "oracle_nco_increment": (u32, [ctypes.c_double, u32]),
            "oracle_nco_mix": (f32, [u32, f32, f32]),
            "oracle_ssb_set_variant": (None, [P, ctypes.c_double, u32, ctypes.c_int]),
            "oracle_ssb_process": (ctypes.c_int, [P, P, i64, u32, ctypes.c_int, ctypes.c_int, P, P, P]),
            "oracle_run_streams": (ctypes.c_int, [P, ctypes.c_int, i32, i32, i32, u32, u32, i32, ctypes.c_int,
                                                  ctypes.c_int, P, P]),
            "oracle_pulse_config_default": (ctypes.c_int, [ctypes.c_int, P]),
            "oracle_pulse_create": (P, [ctypes.c_int, P]),
            "oracle_pulse_destroy": (None, [P]),
            "oracle_pulse_configure": (ctypes.c_int, [P, P]),
            "oracle_pulse_reset": (None, [P]),
            "oracle_pulse_spectral": (ctypes.c_int, [P, P, P, ctypes.c_int, P]),
            "oracle_pulse_audio": (ctypes.c_int, [P, P, ctypes.c_int, ctypes.c_int, P]),
            "oracle_pulse_output_size": (ctypes.c_int, []),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def bytes_per_sample(fmt: int) -> int:
    return {CF32: 8, CS8: 2, CU8: 2, CS16: 4}[fmt]


def unpack(fmt: int, raw: np.ndarray, n: int) -> np.ndarray:
    raw = np.ascontiguousarray(raw)
    out = np.empty(2 * n, dtype=np.float32)
    rc = lib().oracle_unpack(fmt, _ptr(raw), n, _ptr(out))
    assert rc == 0, rc
    return out


def power_shifted(iq: np.ndarray, use_f64: bool = False) -> np.ndarray:
    iq = np.ascontiguousarray(iq, dtype=np.float32).reshape(-1)
    n = iq.size // 2
    out = np.zeros(n, dtype=np.float32)  # a fresh vector: for odd n element n-1 is never written (stays 0)
    rc = lib().oracle_power_shifted(_ptr(iq), n, int(use_f64), _ptr(out))
    assert rc == 0, rc
    return out


def window_geometry(sample_rate: int, n: int, focus_khz: int):
    lo, hi, w, nr = (ctypes.c_int32() for _ in range(4))
    wins = np.zeros(20, dtype=np.int32)
    lib().oracle_window_geometry(sample_rate, n, focus_khz, ctypes.byref(lo), ctypes.byref(hi), ctypes.byref(w),
                                 ctypes.byref(nr), _ptr(wins))
    return lo.value, hi.value, w.value, [(int(wins[2 * i]), int(wins[2 * i + 1])) for i in range(nr.value)]


class FftState:
    """FFTProcessor member state (fft_process.h:57-109) for one stream."""

    def __init__(self, center_frequency: int, sample_rate: int, n: int, focus_khz: int):
        self.buf = np.zeros(lib().oracle_fft_state_size(), dtype=np.uint8)
        lib().oracle_fft_state_init(_ptr(self.buf))
        self.configure(center_frequency, sample_rate, n, focus_khz)

    def configure(self, center_frequency: int, sample_rate: int, n: int, focus_khz: int) -> None:
        self.n = n
        lib().oracle_fft_configure(_ptr(self.buf), center_frequency & 0xFFFFFFFF, sample_rate & 0xFFFFFFFF, n,
                                   focus_khz)

    def set_center_frequency_changed(self) -> None:
        lib().oracle_fft_set_center_frequency_changed(_ptr(self.buf))

    def signal_strength(self, spectrum: np.ndarray, now_ms: int):
        spectrum = np.ascontiguousarray(spectrum, dtype=np.float32)
        rec = np.zeros(1, dtype=RECORD_DTYPE)
        rc = lib().oracle_signal_strength(_ptr(self.buf), _ptr(spectrum), spectrum.size, now_ms, _ptr(rec))
        assert rc == 0, rc
        return rec[0]

    def process(self, iq: np.ndarray, now_ms: int, use_f64: bool = False):
        iq = np.ascontiguousarray(iq, dtype=np.float32).reshape(-1)
        n = iq.size // 2
        # power_shifted_vec persists across frames (fft_process.h:59): resize keeps its prefix, new elements are 0
        # (for odd n the shift never writes element n-1, which keeps the vector's old value)
        old = getattr(self, "_vec", None)
        if old is None or old.size != n:
            self._vec = np.zeros(n, dtype=np.float32)
            if old is not None:
                k = min(n, old.size)
                self._vec[:k] = old[:k]
        rec = np.zeros(1, dtype=RECORD_DTYPE)
        rc = lib().oracle_fft_process(_ptr(self.buf), _ptr(iq), n, now_ms, int(use_f64), _ptr(self._vec), _ptr(rec))
        assert rc == 0, rc
        return self._vec.copy(), rec[0]


def lpf_coefs(fs: float, fc: float, q: float) -> np.ndarray:
    c = np.zeros(5, dtype=np.float32)
    lib().oracle_iir2_lowpass(fs, fc, q, _ptr(c))
    return c


def hp_coefs(fs: float, f0: float, q: float) -> np.ndarray:
    c = np.zeros(5, dtype=np.float32)
    lib().oracle_biquad_highpass(fs, f0, q, _ptr(c))
    return c


def bp_coefs(fs: float, f0: float, q: float) -> np.ndarray:
    c = np.zeros(5, dtype=np.float32)
    lib().oracle_biquad_bandpass(fs, f0, q, _ptr(c))
    return c


def fir_taps(in_size: int, decim: int, cutoff_rel: float = 0.45) -> np.ndarray:
    h = np.zeros(256, dtype=np.float32)
    n = lib().oracle_fir_taps(in_size, decim, cutoff_rel, _ptr(h))
    return h[:n].copy()


def ssb_decim(sample_rate: int) -> int:
    return lib().oracle_ssb_decim(sample_rate)


def ssb_pcm_len(n: int, sample_rate: int, fir_taps: int = 0) -> int:
    return lib().oracle_ssb_pcm_len_n(n, sample_rate, fir_taps)


def nco_increment(hz: float, sample_rate: int) -> int:
    """NCO variant (build extension, include/sdrg.h): round(hz / fs * 2^32) mod 2^32."""
    return lib().oracle_nco_increment(hz, sample_rate)


class _Taps(ctypes.Structure):
    _fields_ = [(k, ctypes.c_void_p) for k in ("dc_re", "lpf", "agc", "fir", "eq")]


class SsbState:
    """processSSB_opt's function statics (ssb_demod_opt.cpp:17-28, 223-282) for one stream."""

    def __init__(self):
        self.buf = np.zeros(lib().oracle_ssb_state_size(), dtype=np.uint8)
        lib().oracle_ssb_state_init(_ptr(self.buf))
        self.frozen = 0
        self.fir_taps = 0

    def set_variant(self, nco_hz: float, sample_rate: int, fir_taps: int = 0) -> None:
        """The NCO/short-FIR variant (a build extension; sdrg_engine_set_ssb_variant).  Restarts the phase."""
        lib().oracle_ssb_set_variant(_ptr(self.buf), nco_hz, sample_rate, fir_taps)
        self.fir_taps = fir_taps

    def process(self, iq: np.ndarray, sample_rate: int, mode: int = 1, upper: bool = True, stages: bool = False):
        iq = np.ascontiguousarray(iq, dtype=np.float32).reshape(-1)
        n = iq.size // 2
        if self.frozen == 0:
            self.frozen = n
        S = self.frozen
        m = max(ssb_pcm_len(S, sample_rate, self.fir_taps), 1)
        pcm = np.zeros(m, dtype=np.int16)
        plen = ctypes.c_int32()
        taps = None
        arrs = None
        if stages:
            arrs = {k: np.zeros(S if k in ("dc_re", "lpf", "agc") else m, dtype=np.float32)
                    for k in ("dc_re", "lpf", "agc", "fir", "eq")}
            taps = _Taps(**{k: v.ctypes.data for k, v in arrs.items()})
        rc = lib().oracle_ssb_process(_ptr(self.buf), _ptr(iq), n, sample_rate, int(upper), mode, _ptr(pcm),
                                      ctypes.byref(plen), ctypes.byref(taps) if taps is not None else None)
        assert rc == 0, rc
        out = pcm[: plen.value].copy()
        if stages:
            arrs["fir"] = arrs["fir"][: plen.value]
            arrs["eq"] = arrs["eq"][: plen.value]
            return out, arrs
        return out


def run_streams(raw: np.ndarray, fmt: int, n: int, f0: int, f1: int, sample_rate: int, center_frequency: int,
                focus_khz: int, stages: int = STAGE_ALL, mode: int = 1) -> None:
    """CPU-baseline worker: frames [f0, f1) of raw, each processed as a fresh stream (GIL released)."""
    spec = np.empty(n, dtype=np.float32)
    pcm = np.empty(max(ssb_pcm_len(n, sample_rate), 1), dtype=np.int16)
    rc = lib().oracle_run_streams(_ptr(raw), fmt, n, f0, f1, sample_rate, center_frequency, focus_khz, stages, mode,
                                  _ptr(spec), _ptr(pcm))
    assert rc == 0, rc


# ---------------------------------------------------------------------------------------------------------
# Reference SSB (oracle/_ref/ref_ssb, the reference's own ssb_demod_opt.cpp) — container only
# ---------------------------------------------------------------------------------------------------------
def pulse_config_default(kind: int) -> np.ndarray:
    c = np.zeros(1, PULSE_CONFIG_DTYPE)
    lib().oracle_pulse_config_default(kind, _ptr(c))
    return c


class PulseDetector:
    """One SpectralPulseDetector (kind 0) or AudioPulseDetector (kind 1), restated in pulse_oracle.c."""

    def __init__(self, kind: int, cfg: np.ndarray | None = None, **overrides):
        self.kind = kind
        self.cfg = pulse_config_default(kind) if cfg is None else cfg.copy()
        for k, v in overrides.items():
            self.cfg[k] = v
        self.h = lib().oracle_pulse_create(kind, _ptr(self.cfg))
        assert self.h

    def __del__(self):
        if getattr(self, "h", None):
            lib().oracle_pulse_destroy(self.h)
            self.h = None

    def configure(self, **overrides) -> None:
        for k, v in overrides.items():
            self.cfg[k] = v
        assert lib().oracle_pulse_configure(self.h, _ptr(self.cfg)) == 0

    def reset(self) -> None:
        lib().oracle_pulse_reset(self.h)

    def spectral(self, snr_sigma: np.ndarray, freq_hz: np.ndarray) -> np.ndarray:
        a = np.ascontiguousarray(snr_sigma, np.float32)
        b = np.ascontiguousarray(freq_hz, np.float32)
        out = np.zeros(a.size, PULSE_OUTPUT_DTYPE)
        assert lib().oracle_pulse_spectral(self.h, _ptr(a), _ptr(b), a.size, _ptr(out)) == 0
        return out

    def audio(self, block: np.ndarray) -> np.ndarray:
        a = np.ascontiguousarray(block)
        fmt = 0 if a.dtype == np.int16 else 1
        if fmt:
            a = a.astype(np.float32)
        out = np.zeros(1, PULSE_OUTPUT_DTYPE)
        assert lib().oracle_pulse_audio(self.h, _ptr(a), fmt, a.size, _ptr(out)) == 0
        return out[0]

    def audio_blocks(self, samples: np.ndarray, block: int) -> np.ndarray:
        outs = [self.audio(samples[k:k + block]) for k in range(0, samples.size, block)]
        return np.array(outs, PULSE_OUTPUT_DTYPE)


REF_PULSE = os.path.join(HERE, "_ref", "ref_pulse")


# reference Config field name -> sdrg_pulse_config field name
PULSE_CFG_NAMES = {"fsEnergy": "fs_energy", "zDefaultS": "z_default_s", "tTargetInit": "t_target_init",
                   "dtTolS": "dt_tol_s", "snrMin": "snr_min", "snrRhythm": "snr_rhythm", "snrStrong": "snr_strong",
                   "dispersionMax": "dispersion_max", "sumNMax": "sum_n_max", "liveWindowT": "live_window_t",
                   "liveDivisor": "live_divisor", "sampleRate": "sample_rate", "fMin": "f_min", "fMax": "f_max",
                   "smoothCutoff": "smooth_cutoff", "noiseRefFar": "noise_ref_far", "noiseRefNear": "noise_ref_near"}


def pulse_overrides(ref_names: dict) -> dict:
    """Reference Config overrides -> sdrg_pulse_config field overrides."""
    return {PULSE_CFG_NAMES[k]: v for k, v in ref_names.items()}


def _kv(overrides: dict | None):
    return [f"{k}={repr(float(np.float32(v))) if isinstance(v, float) else v}" for k, v in (overrides or {}).items()]


def ref_pulse_spectral(snr_sigma: np.ndarray, freq_hz: np.ndarray, fs_energy: float, reconf=None,
                       overrides: dict | None = None) -> np.ndarray:
    """The reference's own SpectralPulseDetector (oracle/_ref/ref_pulse, container only); overrides use the
    reference Config field names."""
    inp = np.stack([np.asarray(snr_sigma, np.float32), np.asarray(freq_hz, np.float32)], axis=1)
    args = [REF_PULSE, "spectral", repr(float(np.float32(fs_energy)))]
    if reconf is not None:
        args += [str(int(reconf[0])), repr(float(np.float32(reconf[1])))]
    args += _kv(overrides)
    out = subprocess.run(args, input=inp.tobytes(), capture_output=True, check=True).stdout
    return np.frombuffer(out, PULSE_OUTPUT_DTYPE).copy()


def ref_pulse_audio(samples: np.ndarray, block: int, overrides: dict | None = None) -> np.ndarray:
    """The reference's own AudioPulseDetector over int16 / float32 samples in blocks (container only)."""
    a = np.ascontiguousarray(samples)
    fmt = 0 if a.dtype == np.int16 else 1
    if fmt:
        a = a.astype(np.float32)
    out = subprocess.run([REF_PULSE, "audio", str(fmt), str(block)] + _kv(overrides), input=a.tobytes(),
                         capture_output=True, check=True).stdout
    return np.frombuffer(out, PULSE_OUTPUT_DTYPE).copy()


def have_ref() -> bool:
    return os.path.exists(REF_SSB)


def _hexfloats(text: str) -> np.ndarray:
    return np.array([float.fromhex(t) for t in text.split()], dtype=np.float32)


def ref_taps(in_size: int, decim: int) -> np.ndarray:
    out = subprocess.run([REF_SSB, "taps", str(in_size), str(decim)], check=True, capture_output=True, text=True).stdout
    vals = out.split()
    return _hexfloats(" ".join(vals[1:]))


def ref_coefs(kind: str, fs: float, f0: float, q: float) -> np.ndarray:
    out = subprocess.run([REF_SSB, kind, repr(fs), repr(f0), repr(q)], check=True, capture_output=True,
                         text=True).stdout
    return _hexfloats(out)


def ref_ssb_run(frames: np.ndarray, sample_rate: int, modes, upper: bool = True):
    """frames: [F][n][2] float32 CF32; returns list of int16 PCM arrays (fresh reference process)."""
    frames = np.ascontiguousarray(frames, dtype=np.float32)
    F, n = frames.shape[0], frames.shape[1]
    assert len(modes) == F
    res = subprocess.run([REF_SSB, "run", str(sample_rate), str(int(upper)), str(n)] + [str(m) for m in modes],
                         input=frames.tobytes(), check=True, capture_output=True)
    buf = res.stdout
    out, off = [], 0
    for _ in range(F):
        c = int(np.frombuffer(buf, dtype=np.int32, count=1, offset=off)[0])
        off += 4
        out.append(np.frombuffer(buf, dtype=np.int16, count=c, offset=off).copy())
        off += 2 * c
    return out


def ref_ssb_stages(frame: np.ndarray, sample_rate: int, fc: float, q: float, target: float, fast: float,
                   coeff: float):
    frame = np.ascontiguousarray(frame, dtype=np.float32)
    n = frame.shape[0]
    res = subprocess.run([REF_SSB, "stages", str(sample_rate), str(n), repr(fc), repr(q), repr(target), repr(fast),
                          repr(coeff)], input=frame.tobytes(), check=True, capture_output=True)
    buf, off, out = res.stdout, 0, {}
    for k in ("dc_re", "lpf", "agc", "fir", "eq"):
        c = int(np.frombuffer(buf, dtype=np.int32, count=1, offset=off)[0])
        off += 4
        out[k] = np.frombuffer(buf, dtype=np.float32, count=c, offset=off).copy()
        off += 4 * c
    return out


# ---------------------------------------------------------------------------------------------------------
# Synthetic inputs: CW tone + seeded Gaussian noise, quantised to the raw format
# ---------------------------------------------------------------------------------------------------------
def synth_frames(n_frames: int, n: int, fmt: int = CS8, tone_hz: float = 1500.0, fs: float = 2e6,
                 amp: float | None = None, noise: float | None = None, seed: int = 0x5D12,
                 phase_continuous: bool = True) -> np.ndarray:
    """Raw interleaved IQ frames [n_frames][n*2] in `fmt` (int8 / uint8 / int16 / float32)."""
    rng = np.random.default_rng(seed)
    if fmt in (CS8, CU8):
        amp = 60.0 if amp is None else amp
        noise = 4.0 if noise is None else noise
    elif fmt == CS16:
        amp = 8000.0 if amp is None else amp
        noise = 400.0 if noise is None else noise
    else:
        amp = 0.5 if amp is None else amp
        noise = 0.03 if noise is None else noise
    t = np.arange(n, dtype=np.float64)
    out = []
    for f in range(n_frames):
        t0 = f * n if phase_continuous else 0
        ph = 2 * np.pi * tone_hz * (t + t0) / fs
        i = amp * np.cos(ph) + rng.normal(0, noise, n)
        q = amp * np.sin(ph) + rng.normal(0, noise, n)
        iq = np.stack([i, q], axis=1).reshape(-1)
        if fmt == CS8:
            out.append(np.clip(np.round(iq), -128, 127).astype(np.int8))
        elif fmt == CU8:
            out.append(np.clip(np.round(iq + 127.4), 0, 255).astype(np.uint8))
        elif fmt == CS16:
            out.append(np.clip(np.round(iq), -32768, 32767).astype(np.int16))
        else:
            out.append(iq.astype(np.float32))
    return np.stack(out)

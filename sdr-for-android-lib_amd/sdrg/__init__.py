"""Python binding of libsdrg.so (include/sdrg.h) — host-side mirror of the reference's SDRBridge surface.

The reference exposes the hot path to Kotlin through JNI (java/fr/intuite/sdr/bridge/SDRBridge.kt:23-154):
`SDRConfig`, `applyConfig(...)`, `read(12 callbacks)` and per-field setters.  This module mirrors that
surface over the engine's C ABI with the same names and argument meaning:

    cfg = SDRConfig(centerFrequency=100_000_000, sampleRate=2_000_000, samplesPerReading=16384)
    eng = Engine(cfg, n_streams=4096)          # one reference "process" per stream
    eng.applyConfig(cfg); eng.setFrequency(...); eng.setFrequencyFocusRange(...); eng.setSoundMode(...)
    eng.read(fftCallback=..., meanSnrCallback=..., pcmCallback=...)   # register callbacks (JNI read)
    spectra, records, pcm = eng.process(iq_frames, fmt=CS8)           # one frame per stream

Everything runs in the HIP kernels of libsdrg.so; there is no CPU fallback.  If the library is missing
or no gfx950 device is present, the calls raise.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
LIB_PATH = os.environ.get("SDRG_LIB_PATH") or os.path.join(PKG, "lib", "libsdrg.so")  # override: diagnostic builds

# include/sdrg.h
CF32, CS8, CU8, CS16, CS12 = 0, 1, 2, 3, 4
STAGE_SPECTRUM, STAGE_STATS, STAGE_SSB, STAGE_HOT_PATH = 1, 2, 4, 7
STAGE_SPECTRAL_PULSE, STAGE_AUDIO_PULSE, STAGE_ALL = 8, 16, 31
PIPELINE_OFF, PIPELINE_ON, PIPELINE_INPUTS_READY = 0, 1, 2  # sdrg_engine_set_pipelining modes
PIPELINE_STATS_ASYNC = 4  # OR'ed with ON / INPUTS_READY: statistics on a stream of their own
PULSE_SPECTRAL, PULSE_AUDIO = 0, 1
STATUS = {0: "SDRG_OK", -1: "SDRG_E_INVALID", -2: "SDRG_E_UNSUPPORTED", -3: "SDRG_E_NOMEM", -4: "SDRG_E_HIP",
          -5: "SDRG_E_NODEVICE"}
BYTES_PER_SAMPLE = {CF32: 8, CS8: 2, CU8: 2, CS16: 4}
NUMPY_DTYPE = {CF32: np.float32, CS8: np.int8, CU8: np.uint8, CS16: np.int16}

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

# Every entry point include/sdrg.h declares (checked by tests/test_abi.py).
EXPORTS = [
    "sdrg_abi_version", "sdrg_last_error", "sdrg_ssb_pcm_len", "sdrg_focus_window", "sdrg_host_alloc", "sdrg_host_free", "sdrg_ssb_design", "sdrg_engine_create", "sdrg_engine_destroy",
    "sdrg_engine_apply_config", "sdrg_engine_set_frequency", "sdrg_engine_set_frequency_focus_range",
    "sdrg_engine_set_sound_mode", "sdrg_engine_set_sample_rate", "sdrg_engine_set_samples_per_reading",
    "sdrg_engine_input_released", "sdrg_engine_wait_input_released", "sdrg_engine_wait_outputs", "sdrg_engine_set_upper_sideband", "sdrg_engine_get_config", "sdrg_engine_n_streams", "sdrg_engine_pcm_len",
    "sdrg_engine_reset_state", "sdrg_engine_process_device", "sdrg_engine_synchronize", "sdrg_engine_set_stream",
    "sdrg_engine_set_pipelining", "sdrg_engine_set_ssb_variant", "sdrg_engine_get_ssb_variant",
    "sdrg_engine_process_host", "sdrg_engine_signal_strength_device", "sdrg_engine_signal_strength_host",
    "sdrg_engine_set_callbacks", "sdrg_engine_set_profiling", "sdrg_engine_get_timings",
    "sdrg_engine_get_timing_stats", "sdrg_engine_reset_timing_stats",
    "sdrg_engine_set_spectral_pulse_config", "sdrg_engine_set_audio_pulse_config", "sdrg_engine_pulse_outputs",
    "sdrg_engine_get_pulse_outputs",
    "sdrg_pulse_config_default", "sdrg_pulse_bank_create", "sdrg_pulse_bank_destroy", "sdrg_pulse_bank_configure",
    "sdrg_pulse_bank_get_config", "sdrg_pulse_bank_reset", "sdrg_pulse_bank_process_spectral_device",
    "sdrg_pulse_bank_process_audio_device", "sdrg_pulse_bank_process_spectral_host",
    "sdrg_pulse_bank_process_audio_host", "sdrg_pulse_bank_synchronize", "sdrg_pulse_bank_set_stream",
    "sdrg_ingest_create", "sdrg_ingest_destroy", "sdrg_ingest_output_format", "sdrg_ingest_push", "sdrg_ingest_status",
    "sdrg_ingest_pop_batch", "sdrg_ingest_pop", "sdrg_ingest_set_samples_per_reading",
    "sdrg_ssb_processor_create", "sdrg_ssb_processor_destroy", "sdrg_ssb_processor_start", "sdrg_ssb_processor_stop",
    "sdrg_ssb_processor_enqueue", "sdrg_ssb_processor_set_sound_mode", "sdrg_ssb_processor_set_pulse_config",
    "sdrg_ssb_processor_get_ambient_energy", "sdrg_ssb_processor_get_current_ratio", "sdrg_ssb_processor_drain",
    "sdrg_ssb_processor_counters",
    "sdrg_dist_unique_id", "sdrg_dist_create", "sdrg_dist_destroy", "sdrg_dist_info", "sdrg_dist_set_one_rank_rccl",
    "sdrg_engine_gather",
    "sdrg_engine_gather_records", "sdrg_engine_gather_focus", "sdrg_engine_gather_spectra", "sdrg_engine_gather_pcm",
    "sdrg_device_alloc", "sdrg_device_free", "sdrg_memcpy", "sdrg_measure_hbm_copy",
]
DIST_ID_BYTES = 128  # SDRG_DIST_ID_BYTES (ncclUniqueId)


class SdrgError(RuntimeError):
    pass


class _Config(ctypes.Structure):
    _fields_ = [
        ("center_frequency", ctypes.c_int64),
        ("sample_rate", ctypes.c_int64),
        ("samples_per_reading", ctypes.c_int32),
        ("freq_focus_range_khz", ctypes.c_int32),
        ("gain", ctypes.c_int32),
        ("sound_mode", ctypes.c_int32),
        ("refresh_fft_ms", ctypes.c_int64),
        ("refresh_peak_ms", ctypes.c_int64),
        ("refresh_signal_strength_ms", ctypes.c_int64),
    ]


class PulseConfig(ctypes.Structure):
    """sdrg_pulse_config: SpectralPulseDetector::Config / AudioPulseDetector::Config (include/sdrg.h)."""
    _fields_ = [(k, ctypes.c_float) for k in ("fs_energy", "z_default_s", "t_target_init", "dt_tol_s", "snr_min",
                                              "snr_rhythm", "snr_strong", "dispersion_max")] + [
        ("sum_n_max", ctypes.c_int32), ("live_window_t", ctypes.c_float), ("live_divisor", ctypes.c_float),
        ("sample_rate", ctypes.c_float), ("f_min", ctypes.c_float), ("f_max", ctypes.c_float),
        ("smooth_cutoff", ctypes.c_float), ("noise_ref_far", ctypes.c_int32), ("noise_ref_near", ctypes.c_int32)]

    @classmethod
    def default(cls, kind: int, **overrides) -> "PulseConfig":
        c = cls()
        _check(load().sdrg_pulse_config_default(kind, ctypes.byref(c)), "sdrg_pulse_config_default")
        for k, v in overrides.items():
            setattr(c, k, v)
        return c


class _Timings(ctypes.Structure):
    _fields_ = [("spectrum_ms", ctypes.c_float), ("stats_ms", ctypes.c_float), ("ssb_ms", ctypes.c_float),
                ("total_ms", ctypes.c_float)]


_V = ctypes.c_void_p
_I32, _I64, _F = ctypes.c_int32, ctypes.c_int64, ctypes.c_float
CB_FFT = ctypes.CFUNCTYPE(None, _V, _I32, ctypes.POINTER(ctypes.c_float), _I32)
CB_I = ctypes.CFUNCTYPE(None, _V, _I32, _I32)
CB_F = ctypes.CFUNCTYPE(None, _V, _I32, _F)
CB_J = ctypes.CFUNCTYPE(None, _V, _I32, _I64)
CB_PCM = ctypes.CFUNCTYPE(None, _V, _I32, ctypes.POINTER(ctypes.c_int16), _I32)
CB_FF = ctypes.CFUNCTYPE(None, _V, _I32, _F, _F)
CB_FIJ = ctypes.CFUNCTYPE(None, _V, _I32, _F, _I32, _I64)
CB_FI = ctypes.CFUNCTYPE(None, _V, _I32, _F, _I32)


class _Callbacks(ctypes.Structure):
    _fields_ = [
        ("user", _V),
        ("fft", CB_FFT),
        ("detection_flag", CB_I),
        ("mean_snr", CB_F),
        ("mean_snr_sigma", CB_F),
        ("peak_frequency", CB_J),
        ("pcm", CB_PCM),
        ("peak_above_noise_mean", CB_F),
        ("max_bin", CB_FF),
        ("best1khz", CB_FF),
        ("noise_level", CB_F),
        ("spectral_pulse", CB_FIJ),
        ("audio_pulse", CB_FI),
    ]


CB_SSB_PCM = ctypes.CFUNCTYPE(None, _V, ctypes.POINTER(ctypes.c_int16), _I32)
CB_SSB_PULSE = ctypes.CFUNCTYPE(None, _V, _F, _I32)


class _SsbCallbacks(ctypes.Structure):
    _fields_ = [("user", _V), ("pcm", CB_SSB_PCM), ("pulse", CB_SSB_PULSE)]


class _GatherBuffers(ctypes.Structure):
    _fields_ = [(k, _V) for k in ("records", "records_out", "focus_spectra", "focus_out", "spectra", "spectra_out",
                                  "pcm", "pcm_out")]


_lib = None


def lib_path() -> str:
    return LIB_PATH


def load() -> ctypes.CDLL:
    """Load libsdrg.so; raise if it has not been built (no CPU fallback exists)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise SdrgError(f"{LIB_PATH} not built: run `make -C sdr-for-android-lib_amd` "
                        "(or __graft_entry__.build())")
    L = ctypes.CDLL(LIB_PATH)
    P = ctypes.c_void_p
    sig = {
        "sdrg_abi_version": (_I32, []),
        "sdrg_last_error": (ctypes.c_char_p, []),
        "sdrg_ssb_pcm_len": (_I32, [_I32, _I64]),
        "sdrg_ssb_design": (_I32, [_I32, _I64, _I32, P, P, P, P, ctypes.POINTER(_I32)]),
        "sdrg_engine_create": (_I32, [ctypes.POINTER(_Config), _I32, _I32, ctypes.POINTER(P)]),
        "sdrg_engine_destroy": (_I32, [P]),
        "sdrg_engine_apply_config": (_I32, [P, ctypes.POINTER(_Config)]),
        "sdrg_engine_set_frequency": (_I32, [P, _I64]),
        "sdrg_engine_set_frequency_focus_range": (_I32, [P, _I32]),
        "sdrg_engine_set_sound_mode": (_I32, [P, _I32]),
        "sdrg_engine_set_sample_rate": (_I32, [P, _I64]),
        "sdrg_engine_set_samples_per_reading": (_I32, [P, _I32]),
        "sdrg_engine_input_released": (_I32, [P, ctypes.POINTER(_I32)]),
        "sdrg_engine_wait_input_released": (_I32, [P, P]),
        "sdrg_engine_set_upper_sideband": (_I32, [P, _I32]),
        "sdrg_engine_get_config": (_I32, [P, ctypes.POINTER(_Config)]),
        "sdrg_engine_n_streams": (_I32, [P]),
        "sdrg_engine_pcm_len": (_I32, [P]),
        "sdrg_engine_reset_state": (_I32, [P]),
        "sdrg_engine_process_device": (_I32, [P, P, _I32, _I32, P, P, P, _I64]),
        "sdrg_engine_synchronize": (_I32, [P]),
        "sdrg_engine_wait_outputs": (_I32, [P, P]),
        "sdrg_engine_set_stream": (_I32, [P, P]),
        "sdrg_engine_set_pipelining": (_I32, [P, _I32]),
        "sdrg_engine_set_ssb_variant": (_I32, [P, ctypes.c_double, _I32]),
        "sdrg_focus_window": (_I32, [_I64, _I32, _I32, P, P]),
        "sdrg_host_alloc": (_I32, [ctypes.c_size_t, P]),
        "sdrg_host_free": (_I32, [P]),
        "sdrg_engine_get_ssb_variant": (_I32, [P, P, P, P, P]),
        "sdrg_engine_process_host": (_I32, [P, P, _I32, _I32, P, P, P, _I64]),
        "sdrg_engine_signal_strength_device": (_I32, [P, P, P, _I64]),
        "sdrg_engine_signal_strength_host": (_I32, [P, P, P, _I64]),
        "sdrg_engine_set_callbacks": (_I32, [P, ctypes.POINTER(_Callbacks)]),
        "sdrg_engine_set_profiling": (_I32, [P, _I32]),
        "sdrg_engine_get_timings": (_I32, [P, ctypes.POINTER(_Timings)]),
        "sdrg_engine_get_timing_stats": (_I32, [P, ctypes.POINTER(_Timings), ctypes.POINTER(_I32)]),
        "sdrg_engine_reset_timing_stats": (_I32, [P]),
        "sdrg_engine_set_spectral_pulse_config": (_I32, [P, ctypes.POINTER(PulseConfig)]),
        "sdrg_engine_set_audio_pulse_config": (_I32, [P, ctypes.POINTER(PulseConfig)]),
        "sdrg_engine_pulse_outputs": (_I32, [P, ctypes.POINTER(P), ctypes.POINTER(P)]),
        "sdrg_engine_get_pulse_outputs": (_I32, [P, P, P]),
        "sdrg_pulse_config_default": (_I32, [_I32, ctypes.POINTER(PulseConfig)]),
        "sdrg_pulse_bank_create": (_I32, [_I32, ctypes.POINTER(PulseConfig), _I32, _I32, ctypes.POINTER(P)]),
        "sdrg_pulse_bank_destroy": (_I32, [P]),
        "sdrg_pulse_bank_configure": (_I32, [P, ctypes.POINTER(PulseConfig)]),
        "sdrg_pulse_bank_get_config": (_I32, [P, ctypes.POINTER(PulseConfig)]),
        "sdrg_pulse_bank_reset": (_I32, [P]),
        "sdrg_pulse_bank_process_spectral_device": (_I32, [P, P, P, _I32, P]),
        "sdrg_pulse_bank_process_audio_device": (_I32, [P, P, _I32, _I32, _I32, P]),
        "sdrg_pulse_bank_process_spectral_host": (_I32, [P, P, P, P]),
        "sdrg_pulse_bank_process_audio_host": (_I32, [P, P, _I32, _I32, P]),
        "sdrg_pulse_bank_synchronize": (_I32, [P]),
        "sdrg_pulse_bank_set_stream": (_I32, [P, P]),
        "sdrg_ingest_create": (_I32, [_I32, _I32, _I32, _I32, ctypes.POINTER(P)]),
        "sdrg_ingest_destroy": (_I32, [P]),
        "sdrg_ingest_output_format": (_I32, [P]),
        "sdrg_ingest_push": (_I32, [P, _I32, P, _I64]),
        "sdrg_ingest_status": (_I32, [P, _I32, ctypes.POINTER(_I32), ctypes.POINTER(_I32), ctypes.POINTER(_I64)]),
        "sdrg_ingest_pop_batch": (_I32, [P, P, ctypes.POINTER(_I32)]),
        "sdrg_ingest_pop": (_I32, [P, _I32, P, ctypes.POINTER(_I32)]),
        "sdrg_ingest_set_samples_per_reading": (_I32, [P, _I32]),
        "sdrg_ssb_processor_create": (_I32, [_I32, _I32, ctypes.POINTER(P)]),
        "sdrg_ssb_processor_destroy": (_I32, [P]),
        "sdrg_ssb_processor_start": (_I32, [P, ctypes.POINTER(_SsbCallbacks)]),
        "sdrg_ssb_processor_stop": (_I32, [P]),
        "sdrg_ssb_processor_enqueue": (_I32, [P, P, _I32, _I32, _I64]),
        "sdrg_ssb_processor_set_sound_mode": (_I32, [P, _I32]),
        "sdrg_ssb_processor_set_pulse_config": (_I32, [P, ctypes.POINTER(PulseConfig)]),
        "sdrg_ssb_processor_get_ambient_energy": (_F, [P]),
        "sdrg_ssb_processor_get_current_ratio": (_F, [P]),
        "sdrg_ssb_processor_drain": (_I32, [P]),
        "sdrg_ssb_processor_counters": (_I32, [P, ctypes.POINTER(_I64), ctypes.POINTER(_I64), ctypes.POINTER(_I64),
                                              ctypes.POINTER(_I32)]),
        "sdrg_dist_unique_id": (_I32, [P, _I32]),
        "sdrg_dist_create": (_I32, [P, _I32, _I32, _I32, ctypes.POINTER(P)]),
        "sdrg_dist_destroy": (_I32, [P]),
        "sdrg_dist_info": (_I32, [P, ctypes.POINTER(_I32), ctypes.POINTER(_I32), ctypes.POINTER(_I32),
                                  ctypes.POINTER(_I32)]),
        "sdrg_dist_set_one_rank_rccl": (_I32, [P, _I32]),
        "sdrg_engine_gather": (_I32, [P, P, _I32, ctypes.POINTER(_GatherBuffers)]),
        "sdrg_engine_gather_records": (_I32, [P, P, _I32, P, P]),
        "sdrg_engine_gather_focus": (_I32, [P, P, _I32, P, P]),
        "sdrg_engine_gather_spectra": (_I32, [P, P, _I32, P, P]),
        "sdrg_engine_gather_pcm": (_I32, [P, P, _I32, P, P]),
        "sdrg_device_alloc": (_I32, [_I32, ctypes.c_size_t, ctypes.POINTER(P)]),
        "sdrg_device_free": (_I32, [_I32, P]),
        "sdrg_memcpy": (_I32, [_I32, P, P, ctypes.c_size_t]),
        "sdrg_measure_hbm_copy": (_I32, [_I32, ctypes.c_size_t, _I32, ctypes.POINTER(ctypes.c_double)]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def _check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().sdrg_last_error()
        raise SdrgError(f"{what}: {STATUS.get(rc, rc)}: {msg.decode() if msg else ''}")


def ssb_pcm_len(n: int, sample_rate: int) -> int:
    return int(load().sdrg_ssb_pcm_len(n, sample_rate))


class HostBuffer:
    """Page-locked host memory (sdrg_host_alloc) viewed as a numpy array, for Engine.process outputs and inputs
    at the full PCIe rate.  Freed by close() or when garbage-collected."""

    def __init__(self, shape, dtype):
        self.dtype = np.dtype(dtype)
        nbytes = int(np.prod(shape)) * self.dtype.itemsize
        p = ctypes.c_void_p()
        _check(load().sdrg_host_alloc(max(nbytes, 1), ctypes.byref(p)), "sdrg_host_alloc")
        self._p = p
        buf = (ctypes.c_char * max(nbytes, 1)).from_address(p.value)
        self.array = np.frombuffer(buf, dtype=self.dtype, count=int(np.prod(shape))).reshape(shape)

    def close(self) -> None:
        if getattr(self, "_p", None) is not None and self._p.value:
            self.array = None
            load().sdrg_host_free(self._p)
            self._p = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DeviceBuffer:
    """Device memory through the C ABI (sdrg_device_alloc): a torch-free host can feed the engine and the gathers.
    upload / download are synchronous copies (not ordered with the engine's streams: synchronize the engine first)."""

    def __init__(self, nbytes: int, device: int = 0):
        self.device, self.nbytes = device, int(nbytes)
        p = ctypes.c_void_p()
        _check(load().sdrg_device_alloc(device, max(self.nbytes, 1), ctypes.byref(p)), "sdrg_device_alloc")
        self._p = p

    @property
    def ptr(self) -> int:
        return self._p.value

    def upload(self, a: np.ndarray) -> None:
        a = np.ascontiguousarray(a)
        if a.nbytes > self.nbytes:
            raise ValueError(f"{a.nbytes} bytes into a {self.nbytes}-byte device buffer")
        _check(load().sdrg_memcpy(self.device, self._p, a.ctypes.data_as(ctypes.c_void_p), a.nbytes), "sdrg_memcpy")

    def download(self, shape, dtype) -> np.ndarray:
        out = np.empty(shape, dtype)
        if out.nbytes > self.nbytes:
            raise ValueError(f"{out.nbytes} bytes from a {self.nbytes}-byte device buffer")
        _check(load().sdrg_memcpy(self.device, out.ctypes.data_as(ctypes.c_void_p), self._p, out.nbytes), "sdrg_memcpy")
        return out

    def close(self) -> None:
        if getattr(self, "_p", None) is not None and self._p.value:
            load().sdrg_device_free(self.device, self._p)
            self._p = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def measure_hbm_copy(device: int = 0, nbytes: int = 1 << 30, reps: int = 10) -> float:
    """Read + write GB/s of the library's float4 streaming copy of nbytes (sdrg_measure_hbm_copy): the achievable
    HBM rate behind bench.py's roofline basis."""
    g = ctypes.c_double(0.0)
    _check(load().sdrg_measure_hbm_copy(device, nbytes, reps, ctypes.byref(g)), "sdrg_measure_hbm_copy")
    return g.value


def dist_unique_id() -> bytes:
    """ncclGetUniqueId (sdrg_dist_unique_id) on one rank; hand the bytes to every rank of the job."""
    buf = ctypes.create_string_buffer(DIST_ID_BYTES)
    _check(load().sdrg_dist_unique_id(buf, DIST_ID_BYTES), "sdrg_dist_unique_id")
    return buf.raw


class Dist:
    """An RCCL communicator over the job's ranks (sdrg_dist_create: one process per GPU).  Engine.gather moves the
    per-frame outputs of every rank's engine to a root rank with it."""

    def __init__(self, unique_id: bytes, world_size: int, rank: int, device: int = 0):
        if len(unique_id) != DIST_ID_BYTES:
            raise ValueError(f"unique id must be {DIST_ID_BYTES} bytes")
        h = ctypes.c_void_p()
        _check(load().sdrg_dist_create(ctypes.c_char_p(unique_id), world_size, rank, device, ctypes.byref(h)),
               "sdrg_dist_create")
        self._h, self.world_size, self.rank, self.device = h, world_size, rank, device

    def set_one_rank_rccl(self, on: bool) -> None:
        """One rank: gathers through ncclGather (True) or as device copies (False, the default)."""
        _check(load().sdrg_dist_set_one_rank_rccl(self._h, 1 if on else 0), "sdrg_dist_set_one_rank_rccl")

    def info(self) -> dict:
        r, w, v, x = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        _check(load().sdrg_dist_info(self._h, ctypes.byref(r), ctypes.byref(w), ctypes.byref(v), ctypes.byref(x)),
               "sdrg_dist_info")
        return {"rank": r.value, "world_size": w.value, "rccl_version": v.value, "rccl_data": bool(x.value)}

    def close(self) -> None:
        if getattr(self, "_h", None):
            load().sdrg_dist_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def focus_window(sample_rate: int, n: int, focus_khz: int) -> tuple[int, int]:
    """(first_bin, n_bins) of evaluateSignalStrength's focus window in the fftshifted spectrum (host-side)."""
    lo, nb = ctypes.c_int32(), ctypes.c_int32()
    _check(load().sdrg_focus_window(sample_rate, n, focus_khz, ctypes.byref(lo), ctypes.byref(nb)), "focus_window")
    return lo.value, nb.value


def ssb_design(samp_count: int, sample_rate: int, sound_mode: int = 1) -> dict:
    """The engine's SSB filter design for a configuration (host-side, no device)."""
    lpf, hp, bp = (np.zeros(5, np.float32) for _ in range(3))
    taps = np.zeros(256, np.float32)
    nt = ctypes.c_int32()
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    _check(load().sdrg_ssb_design(samp_count, sample_rate, sound_mode, p(lpf), p(hp), p(bp), p(taps),
                                  ctypes.byref(nt)), "ssb_design")
    return {"lpf": lpf, "hp": hp, "bp": bp, "taps": taps[: nt.value].copy()}


@dataclass
class SDRConfig:
    """Kotlin SDRConfig (SDRBridge.kt:23-37): same field names and defaults."""
    centerFrequency: int = 430_000_000
    samplesPerReading: int = 16384
    sampleRate: int = 2_500_000
    gain: int = 10
    freqFocusRangeKhz: int = 5
    refreshFFTMs: int = 50
    refreshPeakMs: int = 200
    refreshSignalStrengthMs: int = 30
    soundMode: int = 1

    def _c(self) -> _Config:
        return _Config(self.centerFrequency, self.sampleRate, self.samplesPerReading, self.freqFocusRangeKhz,
                       self.gain, self.soundMode, self.refreshFFTMs, self.refreshPeakMs, self.refreshSignalStrengthMs)


class Engine:
    """n_streams independent receivers on one GPU; each process call consumes one frame per stream."""

    def __init__(self, cfg: SDRConfig, n_streams: int, device: int = 0):
        L = load()
        h = ctypes.c_void_p()
        c = cfg._c()
        _check(L.sdrg_engine_create(ctypes.byref(c), n_streams, device, ctypes.byref(h)), "sdrg_engine_create")
        self._h = h
        self.n_streams = n_streams
        self.cfg = cfg
        self._cbs = None

    # ---- SDRBridge surface -------------------------------------------------------------------------
    def applyConfig(self, cfg: SDRConfig) -> bool:
        c = cfg._c()
        _check(load().sdrg_engine_apply_config(self._h, ctypes.byref(c)), "applyConfig")
        self.cfg = cfg
        return True

    def setFrequency(self, frequency: int) -> None:
        _check(load().sdrg_engine_set_frequency(self._h, frequency), "setFrequency")
        self.cfg.centerFrequency = frequency

    def setFrequencyFocusRange(self, khz: int) -> None:
        _check(load().sdrg_engine_set_frequency_focus_range(self._h, khz), "setFrequencyFocusRange")
        self.cfg.freqFocusRangeKhz = khz

    def setSoundMode(self, mode: int) -> None:
        _check(load().sdrg_engine_set_sound_mode(self._h, mode), "setSoundMode")
        self.cfg.soundMode = mode

    def setSampleRate(self, sample_rate: int) -> None:
        """JNI setSampleRate: BridgeConfig only (the SSB sees it next frame; the statistics at the next configure)."""
        _check(load().sdrg_engine_set_sample_rate(self._h, sample_rate), "setSampleRate")
        self.cfg.sampleRate = sample_rate

    def setSamplesPerReading(self, n: int) -> None:
        """JNI setSamplesPerReading: BridgeConfig only; the frame size of the next calls."""
        _check(load().sdrg_engine_set_samples_per_reading(self._h, n), "setSamplesPerReading")
        self.cfg.samplesPerReading = n

    def input_released(self) -> bool:
        """True once every kernel of the last call that reads its iq buffer has finished (non-blocking)."""
        r = ctypes.c_int32()
        _check(load().sdrg_engine_input_released(self._h, ctypes.byref(r)), "input_released")
        return bool(r.value)

    def wait_input_released(self, hip_stream: int | None = None) -> None:
        """Make hip_stream (None: the engine's main stream) wait until the last call has released its iq buffer."""
        _check(load().sdrg_engine_wait_input_released(self._h, hip_stream), "wait_input_released")

    def setUpperSideband(self, upper: bool) -> None:
        _check(load().sdrg_engine_set_upper_sideband(self._h, int(upper)), "setUpperSideband")

    def read(self, fftCallback=None, detectionFlagCallback=None, meanSnrCallback=None, meanSnrSigmaCallback=None,
             peakFrequencyCallback=None, pcmCallback=None, peakAboveNoiseMeanCallback=None, maxBinCallback=None,
             best1kHzCallback=None, noiseLevelCallback=None, spectralPulseCallback=None,
             audioPulseCallback=None) -> None:
        """Register per-frame callbacks (JNI read(), SDRBridge.kt:141-154).  Each receives the stream index
        first, then the reference callback's arguments; arrays arrive as numpy copies."""
        def wrap(fn, ctype, conv):
            if fn is None:
                return ctype()
            return ctype(lambda _u, s, *a: fn(s, *conv(*a)))

        n_of = lambda p, n: (np.ctypeslib.as_array(p, shape=(n,)).copy(),)  # noqa: E731
        ident = lambda *a: a  # noqa: E731
        self._cbs = _Callbacks(
            None,
            wrap(fftCallback, CB_FFT, n_of),
            wrap(detectionFlagCallback, CB_I, ident),
            wrap(meanSnrCallback, CB_F, ident),
            wrap(meanSnrSigmaCallback, CB_F, ident),
            wrap(peakFrequencyCallback, CB_J, ident),
            wrap(pcmCallback, CB_PCM, n_of),
            wrap(peakAboveNoiseMeanCallback, CB_F, ident),
            wrap(maxBinCallback, CB_FF, ident),
            wrap(best1kHzCallback, CB_FF, ident),
            wrap(noiseLevelCallback, CB_F, ident),
            wrap(spectralPulseCallback, CB_FIJ, ident),
            wrap(audioPulseCallback, CB_FI, ident),
        )
        _check(load().sdrg_engine_set_callbacks(self._h, ctypes.byref(self._cbs)), "read")

    def stopReading(self) -> None:
        _check(load().sdrg_engine_set_callbacks(self._h, None), "stopReading")
        self._cbs = None

    # ---- engine ------------------------------------------------------------------------------------
    @property
    def pcm_len(self) -> int:
        return int(load().sdrg_engine_pcm_len(self._h))

    def reset_state(self) -> None:
        _check(load().sdrg_engine_reset_state(self._h), "reset_state")

    def set_spectral_pulse_config(self, cfg: PulseConfig) -> None:
        """SpectralPulseDetector::configure for every stream (state kept)."""
        _check(load().sdrg_engine_set_spectral_pulse_config(self._h, ctypes.byref(cfg)), "set_spectral_pulse_config")

    def setPulseConfig(self, cfg: PulseConfig) -> None:
        """SSBProcessor::setPulseConfig: fresh AudioPulseDetectors with cfg from the next frame."""
        _check(load().sdrg_engine_set_audio_pulse_config(self._h, ctypes.byref(cfg)), "setPulseConfig")

    def pulse_outputs(self, spectral: bool = True, audio: bool = True):
        """Host copies of the last call's pulse-detector outputs (PULSE_OUTPUT_DTYPE arrays, or None)."""
        sp = np.zeros(self.n_streams, PULSE_OUTPUT_DTYPE) if spectral else None
        au = np.zeros(self.n_streams, PULSE_OUTPUT_DTYPE) if audio else None
        ptr = lambda a: None if a is None else a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        _check(load().sdrg_engine_get_pulse_outputs(self._h, ptr(sp), ptr(au)), "get_pulse_outputs")
        return sp, au

    def pulse_output_ptrs(self):
        """Device pointers of the last call's pulse outputs (valid until the next call)."""
        a, b = ctypes.c_void_p(), ctypes.c_void_p()
        _check(load().sdrg_engine_pulse_outputs(self._h, ctypes.byref(a), ctypes.byref(b)), "pulse_outputs")
        return a.value, b.value

    def process(self, iq: np.ndarray, fmt: int = CS8, stages: int = STAGE_ALL, now_ms: int = 0, out=None):
        """Host path: iq is [n_streams][samplesPerReading * 2] raw samples. Returns (spectra, records, pcm).

        out: optional (spectra, records, pcm) arrays to write into (e.g. HostBuffer arrays, page-locked, for the
        full PCIe rate); entries for stages not run may be None.  By default fresh arrays are allocated."""
        n = self.cfg.samplesPerReading
        iq = np.ascontiguousarray(iq, dtype=NUMPY_DTYPE[fmt])
        if iq.size != self.n_streams * n * 2:
            raise SdrgError(f"iq has {iq.size} values, expected {self.n_streams}x{n}x2")
        plen = self.pcm_len
        if out is not None:
            spec, recs, pcm = out
            for a, shape, dt in ((spec, (self.n_streams, n), np.float32), (recs, (self.n_streams,), RECORD_DTYPE),
                                 (pcm, (self.n_streams, max(plen, 0)), np.int16)):
                if a is not None and (a.shape != shape or a.dtype != dt or not a.flags.c_contiguous):
                    raise SdrgError(f"out array {a.shape} {a.dtype}: expected contiguous {shape} {np.dtype(dt)}")
            if (stages & STAGE_SPECTRUM and spec is None) or (stages & STAGE_STATS and recs is None) or \
                    (stages & STAGE_SSB and pcm is None):
                raise SdrgError("out lacks an array for a requested stage")
        else:
            spec = np.empty((self.n_streams, n), np.float32) if stages & STAGE_SPECTRUM else None
            recs = np.zeros(self.n_streams, RECORD_DTYPE) if stages & STAGE_STATS else None
            pcm = np.empty((self.n_streams, max(plen, 0)), np.int16) if stages & STAGE_SSB else None
        ptr = lambda a: None if a is None else a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        _check(load().sdrg_engine_process_host(self._h, ptr(iq), fmt, stages, ptr(spec), ptr(recs),
                                               ptr(pcm) if (pcm is not None and plen > 0) else None, now_ms),
               "process_host")
        return spec, recs, pcm

    def signal_strength(self, spectra: np.ndarray, now_ms: int = 0) -> np.ndarray:
        """evaluateSignalStrength alone on caller spectra ([n_streams][samplesPerReading] fftshifted linear power,
        fft_process.cpp:122-379): returns the records; each stream's statistics state advances as in process()."""
        n = self.cfg.samplesPerReading
        spectra = np.ascontiguousarray(spectra, dtype=np.float32)
        if spectra.shape != (self.n_streams, n):
            raise SdrgError(f"spectra {spectra.shape}: expected ({self.n_streams}, {n})")
        recs = np.zeros(self.n_streams, RECORD_DTYPE)
        _check(load().sdrg_engine_signal_strength_host(self._h, spectra.ctypes.data_as(ctypes.c_void_p),
                                                       recs.ctypes.data_as(ctypes.c_void_p), now_ms),
               "signal_strength_host")
        return recs

    def process_device(self, iq_ptr: int, fmt: int, stages: int, spectra_ptr: int | None, records_ptr: int | None,
                       pcm_ptr: int | None, now_ms: int = 0) -> None:
        """Device path: raw device pointers (e.g. torch tensor .data_ptr()); asynchronous."""
        _check(load().sdrg_engine_process_device(self._h, iq_ptr, fmt, stages, spectra_ptr, records_ptr, pcm_ptr,
                                                 now_ms), "process_device")

    def synchronize(self) -> None:
        _check(load().sdrg_engine_synchronize(self._h), "synchronize")

    def wait_outputs(self, hip_stream: int | None = None) -> None:
        """Enqueue on hip_stream (None: the engine's main stream) a wait for every output of the last call."""
        _check(load().sdrg_engine_wait_outputs(self._h, hip_stream), "wait_outputs")

    def set_pipelining(self, mode) -> None:
        """Overlap each call's SSB stages with the next call's spectrum (see include/sdrg.h): False/PIPELINE_OFF,
        True/PIPELINE_ON, or PIPELINE_INPUTS_READY (iq complete at call time: no wait on the main stream); ON or
        INPUTS_READY | PIPELINE_STATS_ASYNC also runs each call's statistics beside the next call's spectrum."""
        _check(load().sdrg_engine_set_pipelining(self._h, int(mode)), "set_pipelining")

    def set_ssb_variant(self, nco_hz: float = 0.0, fir_taps: int = 0) -> None:
        """BUILD EXTENSION (not a reference interface): NCO mixer at nco_hz before the SSB chain and a
        fir_taps-long decimating FIR (0 = the reference's 255).  (0, 0) is the reference chain."""
        _check(load().sdrg_engine_set_ssb_variant(self._h, float(nco_hz), int(fir_taps)), "set_ssb_variant")

    def ssb_variant(self) -> dict:
        hz, taps, inc, ph = ctypes.c_double(), ctypes.c_int32(), ctypes.c_uint32(), ctypes.c_uint32()
        _check(load().sdrg_engine_get_ssb_variant(self._h, ctypes.byref(hz), ctypes.byref(taps), ctypes.byref(inc),
                                                  ctypes.byref(ph)), "get_ssb_variant")
        return {"nco_hz": hz.value, "fir_taps": taps.value, "nco_increment": inc.value, "nco_phase": ph.value}

    def gather(self, dist: "Dist", root: int = 0, records=None, records_out=None, focus_spectra=None, focus_out=None,
               spectra=None, spectra_out=None, pcm=None, pcm_out=None) -> None:
        """sdrg_engine_gather: gathers of this rank's per-frame outputs (device pointers, ints) to `root`, one RCCL group
        behind the last call's outputs on the engine stream that produced them (device copies on a one-rank
        communicator unless Dist.set_one_rank_rccl(True)); *_out only on the root."""
        b = _GatherBuffers(records, records_out, focus_spectra, focus_out, spectra, spectra_out, pcm, pcm_out)
        _check(load().sdrg_engine_gather(self._h, dist._h, root, ctypes.byref(b)), "sdrg_engine_gather")

    def set_stream(self, hip_stream: int | None) -> None:
        """Enqueue on the caller's HIP stream (e.g. torch.cuda.current_stream().cuda_stream); None = own."""
        _check(load().sdrg_engine_set_stream(self._h, hip_stream), "set_stream")

    def set_profiling(self, on: bool) -> None:
        _check(load().sdrg_engine_set_profiling(self._h, int(on)), "set_profiling")

    def timings(self) -> dict:
        t = _Timings()
        _check(load().sdrg_engine_get_timings(self._h, ctypes.byref(t)), "get_timings")
        return {"spectrum_ms": t.spectrum_ms, "stats_ms": t.stats_ms, "ssb_ms": t.ssb_ms, "total_ms": t.total_ms}

    def timing_stats(self) -> dict:
        t = _Timings()
        c = ctypes.c_int32()
        _check(load().sdrg_engine_get_timing_stats(self._h, ctypes.byref(t), ctypes.byref(c)), "get_timing_stats")
        return {"spectrum_ms": t.spectrum_ms, "stats_ms": t.stats_ms, "ssb_ms": t.ssb_ms, "total_ms": t.total_ms,
                "count": c.value}

    def reset_timing_stats(self) -> None:
        _check(load().sdrg_engine_reset_timing_stats(self._h), "reset_timing_stats")

    def close(self) -> None:
        if getattr(self, "_h", None):
            load().sdrg_engine_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class PulseBank:
    """n_streams beacon pulse detectors of one kind (SpectralPulseDetector or AudioPulseDetector) on one GPU."""

    def __init__(self, kind: int, n_streams: int, cfg: PulseConfig | None = None, device: int = 0):
        L = load()
        self.kind = kind
        self.n_streams = n_streams
        c = cfg if cfg is not None else PulseConfig.default(kind)
        h = ctypes.c_void_p()
        _check(L.sdrg_pulse_bank_create(kind, ctypes.byref(c), n_streams, device, ctypes.byref(h)),
               "sdrg_pulse_bank_create")
        self._h = h

    def configure(self, cfg: PulseConfig) -> None:
        _check(load().sdrg_pulse_bank_configure(self._h, ctypes.byref(cfg)), "pulse_bank_configure")

    def config(self) -> PulseConfig:
        c = PulseConfig()
        _check(load().sdrg_pulse_bank_get_config(self._h, ctypes.byref(c)), "pulse_bank_get_config")
        return c

    def reset(self) -> None:
        _check(load().sdrg_pulse_bank_reset(self._h), "pulse_bank_reset")

    def set_stream(self, hip_stream: int | None) -> None:
        _check(load().sdrg_pulse_bank_set_stream(self._h, hip_stream), "pulse_bank_set_stream")

    def process_spectral(self, snr_sigma: np.ndarray, freq_hz: np.ndarray) -> np.ndarray:
        a = np.ascontiguousarray(snr_sigma, np.float32)
        b = np.ascontiguousarray(freq_hz, np.float32)
        if a.size != self.n_streams or b.size != self.n_streams:
            raise SdrgError("one value per stream expected")
        out = np.zeros(self.n_streams, PULSE_OUTPUT_DTYPE)
        p = lambda x: x.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        _check(load().sdrg_pulse_bank_process_spectral_host(self._h, p(a), p(b), p(out)), "process_spectral_host")
        return out

    def process_audio(self, block: np.ndarray) -> np.ndarray:
        """block: [n_streams][n] int16 (or float32) samples, one block per stream."""
        a = np.ascontiguousarray(block)
        fmt = 0 if a.dtype == np.int16 else 1
        if fmt:
            a = np.ascontiguousarray(a, np.float32)
        if a.ndim != 2 or a.shape[0] != self.n_streams:
            raise SdrgError("block must be [n_streams][n]")
        out = np.zeros(self.n_streams, PULSE_OUTPUT_DTYPE)
        p = lambda x: x.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        _check(load().sdrg_pulse_bank_process_audio_host(self._h, p(a), fmt, a.shape[1], p(out)), "process_audio_host")
        return out

    def process_spectral_device(self, snr_ptr: int, freq_ptr: int, stride_bytes: int, out_ptr: int) -> None:
        _check(load().sdrg_pulse_bank_process_spectral_device(self._h, snr_ptr, freq_ptr, stride_bytes, out_ptr),
               "process_spectral_device")

    def process_audio_device(self, audio_ptr: int, sample_format: int, n: int, stride: int, out_ptr: int) -> None:
        _check(load().sdrg_pulse_bank_process_audio_device(self._h, audio_ptr, sample_format, n, stride, out_ptr),
               "process_audio_device")

    def synchronize(self) -> None:
        _check(load().sdrg_pulse_bank_synchronize(self._h), "pulse_bank_synchronize")

    def close(self) -> None:
        if getattr(self, "_h", None):
            load().sdrg_pulse_bank_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class SSBProcessor:
    """SSBProcessor (src/ssb/ssb_processor.h:24-58): a worker thread fed through a queue of at most queue_max
    frames (the reference's 3) that drops the oldest frame when full; each frame runs the SSB chain and the audio
    pulse detector on the GPU, then pcm_cb(pcm int16 array) (only when non-empty) and pulse_cb(strength, live_etat)
    are called on the worker thread."""

    def __init__(self, device: int = 0, queue_max: int = 0):
        h = ctypes.c_void_p()
        _check(load().sdrg_ssb_processor_create(device, queue_max, ctypes.byref(h)), "sdrg_ssb_processor_create")
        self._h = h
        self._cbs = None

    def startProcessing(self, pcm_cb=None, pulse_cb=None) -> None:
        def pcm(_u, p, n):
            if pcm_cb is not None:
                pcm_cb(np.ctypeslib.as_array(p, shape=(n,)).copy())

        def pulse(_u, strength, live):
            if pulse_cb is not None:
                pulse_cb(strength, live)

        self._cbs = _SsbCallbacks(None, CB_SSB_PCM(pcm), CB_SSB_PULSE(pulse))
        _check(load().sdrg_ssb_processor_start(self._h, ctypes.byref(self._cbs)), "startProcessing")

    def stopProcessing(self) -> None:
        _check(load().sdrg_ssb_processor_stop(self._h), "stopProcessing")

    def enqueueData(self, iq: np.ndarray, sample_rate: int, fmt: int = CF32) -> None:
        """iq: one frame of raw samples in `fmt` (CF32: complex64 or interleaved float32)."""
        a = np.ascontiguousarray(iq)
        if fmt == CF32 and np.iscomplexobj(a):
            a = np.ascontiguousarray(a, np.complex64).view(np.float32)
        a = np.ascontiguousarray(a, NUMPY_DTYPE[fmt])
        _check(load().sdrg_ssb_processor_enqueue(self._h, a.ctypes.data_as(ctypes.c_void_p), fmt, a.size // 2,
                                                 sample_rate), "enqueueData")

    def setSoundMode(self, mode: int) -> None:
        _check(load().sdrg_ssb_processor_set_sound_mode(self._h, mode), "setSoundMode")

    def setPulseConfig(self, cfg: PulseConfig) -> None:
        _check(load().sdrg_ssb_processor_set_pulse_config(self._h, ctypes.byref(cfg)), "setPulseConfig")

    def getAmbientEnergy(self) -> float:
        return float(load().sdrg_ssb_processor_get_ambient_energy(self._h))

    def getCurrentRatio(self) -> float:
        return float(load().sdrg_ssb_processor_get_current_ratio(self._h))

    def drain(self) -> None:
        _check(load().sdrg_ssb_processor_drain(self._h), "drain")

    def counters(self) -> dict:
        e, d, p, st = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int32()
        _check(load().sdrg_ssb_processor_counters(self._h, ctypes.byref(e), ctypes.byref(d), ctypes.byref(p),
                                                  ctypes.byref(st)), "counters")
        return {"enqueued": e.value, "dropped": d.value, "processed": p.value, "last_status": st.value}

    def close(self) -> None:
        if getattr(self, "_h", None):
            load().sdrg_ssb_processor_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


IN_BYTES_PER_SAMPLE = {CF32: 8, CS16: 4, CS8: 2, CU8: 2, CS12: 3}


class Ingest:
    """Exact-N re-chunking of raw reads per stream (rx_reading_thread, sdr-bridge-java-soapy.cpp:503-575)."""

    def __init__(self, n_streams: int, samples_per_reading: int, in_format: int = CS8, queue_max: int = 20):
        h = ctypes.c_void_p()
        _check(load().sdrg_ingest_create(n_streams, samples_per_reading, in_format, queue_max, ctypes.byref(h)),
               "sdrg_ingest_create")
        self._h = h
        self.n_streams, self.n, self.in_format = n_streams, samples_per_reading, in_format
        self.out_format = int(load().sdrg_ingest_output_format(h))

    def push(self, stream: int, raw: np.ndarray) -> None:
        """raw: the bytes of whole complex samples in the input format (any numpy dtype)."""
        b = np.ascontiguousarray(raw).view(np.uint8).reshape(-1)
        bps = IN_BYTES_PER_SAMPLE[self.in_format]
        if b.size % bps:
            raise SdrgError("partial sample")
        _check(load().sdrg_ingest_push(self._h, stream, b.ctypes.data_as(ctypes.c_void_p), b.size // bps),
               "ingest_push")

    def status(self, stream: int):
        q, p, d = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int64()
        _check(load().sdrg_ingest_status(self._h, stream, ctypes.byref(q), ctypes.byref(p), ctypes.byref(d)),
               "ingest_status")
        return q.value, p.value, d.value

    def _frame_dtype(self):
        return NUMPY_DTYPE[self.out_format]

    def pop_batch(self):
        """[n_streams][N*2] frames in the output format, or None when some stream has no frame yet."""
        out = np.empty((self.n_streams, 2 * self.n), self._frame_dtype())
        got = ctypes.c_int32()
        _check(load().sdrg_ingest_pop_batch(self._h, out.ctypes.data_as(ctypes.c_void_p), ctypes.byref(got)),
               "ingest_pop_batch")
        return out if got.value else None

    def pop(self, stream: int):
        out = np.empty(2 * self.n, self._frame_dtype())
        got = ctypes.c_int32()
        _check(load().sdrg_ingest_pop(self._h, stream, out.ctypes.data_as(ctypes.c_void_p), ctypes.byref(got)),
               "ingest_pop")
        return out if got.value else None

    def set_samples_per_reading(self, n: int) -> None:
        _check(load().sdrg_ingest_set_samples_per_reading(self._h, n), "ingest_set_samples_per_reading")
        self.n = n

    def close(self) -> None:
        if getattr(self, "_h", None):
            load().sdrg_ingest_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

"""A SECOND restatement of FFTProcessor::evaluateSignalStrength, in numpy, written directly from the reference text
(src/dsp/fft_process.cpp:122-379, members from fft_process.h:57-109) and NOT derived from oracle/sdrg_oracle.c.

TEST INFRASTRUCTURE ONLY (like everything under oracle/): tests/test_stats_restatements.py compares it with the C
restatement (oracle_signal_strength) on thousands of randomized spectra.  The reference's fft_process.cpp cannot be
built in this image (it needs jni.h and an FFTW library), so the statistics are not pinned by the reference itself;
two restatements written independently agreeing on every field guards against one misreading of the text.

Float semantics: every quantity is a numpy float32 and every float operation is done in float32 with round to
nearest, in the reference's order.  Sequential float sums (the reference's loops) use np.cumsum(dtype=float32),
which adds left to right (np.sum would add pairwise and round differently).  log10f / logf come from numpy's
float32 arithmetic, and log10f / logf are the C library's (glibc, through ctypes), as in the reference's x86-64
build: numpy's own float32 log10 can differ by an ulp, which flips the reference's window sort where two window
means tie to within an ulp (seen on near-silent frames).
"""
from __future__ import annotations

import ctypes
import ctypes.util

import numpy as np

f32 = np.float32
_libm = ctypes.CDLL(ctypes.util.find_library("m") or "libm.so.6")
_libm.log10f.restype = ctypes.c_float
_libm.log10f.argtypes = [ctypes.c_float]
_libm.logf.restype = ctypes.c_float
_libm.logf.argtypes = [ctypes.c_float]
_log10f = np.frompyfunc(lambda x: _libm.log10f(float(x)), 1, 1)


def log10f(x):
    return np.asarray(_log10f(np.asarray(x, dtype=np.float32)), dtype=np.float32)


def logf(x):
    return f32(_libm.logf(float(f32(x))))


def _seq_sum(a: np.ndarray) -> np.float32:
    """((a0 + a1) + a2) + ... in float32, starting from 0.0f (the reference's `float s = 0; for (...) s += x`)."""
    if a.size == 0:
        return f32(0.0)
    return np.cumsum(np.concatenate([np.zeros(1, np.float32), a.astype(np.float32)]), dtype=np.float32)[-1]


def _db(p):
    """10.0f * log10f(p / refPower + 1e-20f), refPower = 1 (fft_process.h:74-75)."""
    p = np.asarray(p, dtype=np.float32)
    return (f32(10.0) * log10f((p / f32(1.0)) + f32(1e-20))).astype(np.float32)


class SignalStrength:
    """The FFTProcessor members evaluateSignalStrength reads and writes, for one stream."""

    def __init__(self, center_frequency: int, sample_rate: int, focus_khz: int):
        # FftProcessorConfig (fft_process.h:20-26) as configure() stores it (uint32 fields)
        self.cf = np.uint32(center_frequency & 0xFFFFFFFF)
        self.fs = np.uint32(sample_rate & 0xFFFFFFFF)
        self.focus_khz = int(focus_khz)
        self.tracking_frequency = f32(0.0)
        self.max_peak = None                      # maxPeakAndFrequency (empty until configure/first use)
        self.t_last_max = 0                       # timeOfLastMaxPeak (ms)
        self.t_last_update = 0                    # timeOfLastMaxPeakUpdate (ms)
        self.peak_confirmed = 0
        self.det_buf = [0, 0, 0]                  # detectionFlagBuffer (remanance 3)
        self.det_idx = 0
        self.cf_changed = False                   # sdr_bridge_internal::isCenterFrequencyChanged
        self.out = dict(mean_snr_db=f32(0), mean_snr_sigma=f32(0), detection_flag=0, peak_above_noise_mean_db=f32(0),
                        max_bin_snr_db=f32(0), max_bin_snr_sigma=f32(0), best1khz_snr_db=f32(0),
                        best1khz_snr_sigma=f32(0), best1khz_center_freq_hz=f32(0), per_bin_mean=f32(0))
        self.configure(center_frequency, sample_rate, focus_khz)

    def configure(self, center_frequency: int, sample_rate: int, focus_khz: int) -> None:
        self.cf = np.uint32(center_frequency & 0xFFFFFFFF)
        self.fs = np.uint32(sample_rate & 0xFFFFFFFF)
        self.focus_khz = int(focus_khz)
        if self.max_peak is None:  # fft_process.cpp:33-35
            self.max_peak = [f32(-130.0), f32(self.cf)]

    def evaluate(self, P: np.ndarray, now_ms: int) -> dict:
        """One frame (fft_process.cpp:122-379); returns the getters plus the diagnostics of a frame record."""
        P = np.asarray(P, dtype=np.float32)
        n = P.size
        o = self.out
        diag = dict(peak_bin=-1, abs_peak_db=f32(-130.0), signal_power_db=f32(0.0), valid=0, n_ref_windows=0)
        freq_per_bin = f32(self.fs) / f32(n)
        X = f32(self.focus_khz) * f32(1000.0)
        nyq = f32(self.fs) / f32(2.0)

        def off_to_bin(off):
            return int((f32(off) + nyq) / freq_per_bin)  # static_cast<int>: truncation toward zero

        focus_lo = max(0, off_to_bin(-X))
        focus_hi = min(n - 1, off_to_bin(X) - 1)
        focus_len = focus_hi - focus_lo + 1
        if focus_len <= 0:
            return self._record(diag)  # :140 returns before anything else (no tracking, no detection)

        # 6.2: first maximum of dB (strict >, seeded at -130), mean power
        fdb = _db(P[focus_lo:focus_hi + 1])
        abs_peak = f32(-130.0)
        peak_in_focus = 0
        above = np.nonzero(fdb > abs_peak)[0]
        if above.size:
            k = int(np.argmax(fdb))  # first index of the maximum; it is > -130 because some value is
            abs_peak, peak_in_focus = fdb[k], k
        sig_sum = _seq_sum(P[focus_lo:focus_hi + 1])
        signal_power_db = _db(sig_sum / f32(focus_len))
        diag.update(peak_bin=focus_lo + peak_in_focus, abs_peak_db=abs_peak, signal_power_db=signal_power_db)

        w = max(1, int(np.ceil(f32(1000.0) / freq_per_bin)))

        def best1k_mean(lo, hi):  # :163-180
            ln = hi - lo + 1
            if ln <= 0:
                return f32(0.0)
            if ln < w:
                return _seq_sum(P[lo:hi + 1]) / f32(ln)
            init = _seq_sum(P[lo:lo + w])
            diffs = (P[lo + w:hi + 1] - P[lo:hi + 1 - w]).astype(np.float32)  # P[s+w-1] - P[s-1], s = lo+1 ..
            runs = np.cumsum(np.concatenate([[init], diffs]).astype(np.float32), dtype=np.float32)
            return np.max(runs / f32(w))

        wins = []  # (meanDb, maxBinDb, best1kDb, lo, hi) in collection order (:182-216)
        for k in range(1, 6):
            near = f32(4 * k - 2) * X
            far = f32(4 * k) * X
            if far >= nyq:
                break
            for lo, hi in ((max(0, off_to_bin(near)), min(n - 1, off_to_bin(far) - 1)),
                           (max(0, off_to_bin(-far)), min(n - 1, off_to_bin(-near) - 1))):
                if hi <= lo:
                    continue
                seg = P[lo:hi + 1]
                wins.append((_db(_seq_sum(seg) / f32(hi - lo + 1)), _db(np.max(seg)), _db(best1k_mean(lo, hi)), lo, hi))
        n_ref = len(wins)
        valid = n_ref >= 2
        diag.update(valid=int(valid), n_ref_windows=n_ref)
        if not valid:
            for key in ("mean_snr_db", "mean_snr_sigma", "peak_above_noise_mean_db", "max_bin_snr_db",
                        "max_bin_snr_sigma", "best1khz_snr_db", "best1khz_snr_sigma"):
                o[key] = f32(0.0)  # per_bin_mean and best1khz_center_freq_hz keep their old values
        else:
            order = np.argsort(np.array([wv[0] for wv in wins], np.float32), kind="stable")  # quietest first
            wins = [wins[i] for i in order]
            n_bottom = max(1, int(f32(n_ref) * f32(0.4)))
            # 6.4a
            means = np.array([wins[i][0] for i in range(n_bottom)], np.float32)
            mean = _seq_sum(means) / f32(n_bottom)
            gaps = np.sort(np.abs(means - mean))
            sigma = max(f32(1.4816) * gaps[n_bottom // 2], f32(0.5))
            snr_db = signal_power_db - mean
            o["mean_snr_db"], o["mean_snr_sigma"] = snr_db, snr_db / sigma
            # 6.4b
            pooled = np.concatenate([_db(P[wins[j][3]:wins[j][4] + 1]) for j in range(n_bottom)])
            sigma_bin, per_bin_mean = f32(1.0), f32(0.0)
            if pooled.size:
                per_bin_mean = _seq_sum(pooled) / f32(pooled.size)
                o["per_bin_mean"] = per_bin_mean
                g = np.sort(np.abs(pooled - per_bin_mean))
                sigma_bin = max(f32(1.4816) * g[g.size // 2], f32(1.0))
            o["peak_above_noise_mean_db"] = abs_peak - per_bin_mean
            # 6.4c
            log_n = logf(f32(focus_len))
            s2 = np.sqrt(f32(2.0) * log_n)
            loc = per_bin_mean + sigma_bin * s2
            with np.errstate(divide="ignore", invalid="ignore"):  # focusLen = 1: / 0 -> inf, as in C
                scale = max((sigma_bin * f32(3.14159)) / (np.sqrt(f32(6.0)) * s2), f32(0.5))
            o["max_bin_snr_db"] = abs_peak - loc
            o["max_bin_snr_sigma"] = o["max_bin_snr_db"] / scale
            # 6.4d
            b1k = np.array([wins[i][2] for i in range(n_bottom)], np.float32)
            mean1k = _seq_sum(b1k) / f32(n_bottom)
            g1k = np.sort(np.abs(b1k - mean1k))
            floor1k = sigma_bin / np.sqrt(f32(w))
            sigma1k = max(f32(1.4816) * g1k[n_bottom // 2], floor1k, f32(0.5))
            focus_best = best1k_mean(focus_lo, focus_hi)
            if focus_best > f32(0.0):
                o["best1khz_snr_db"] = _db(focus_best) - mean1k
                o["best1khz_snr_sigma"] = o["best1khz_snr_db"] / sigma1k
                best_start = focus_lo
                if focus_len >= w:
                    init = _seq_sum(P[focus_lo:focus_lo + w])
                    diffs = (P[focus_lo + w:focus_hi + 1] - P[focus_lo:focus_hi + 1 - w]).astype(np.float32)
                    runs = np.cumsum(np.concatenate([[init], diffs]).astype(np.float32), dtype=np.float32)
                    best_start = focus_lo + int(np.argmax(runs))  # first strict maximum
                o["best1khz_center_freq_hz"] = f32(best_start + w // 2) * freq_per_bin + (f32(self.cf) - nyq)
            else:
                o["best1khz_snr_db"] = o["best1khz_snr_sigma"] = f32(0.0)

        # 6.5 frequency tracking (clock injected as now_ms)
        if self.tracking_frequency == f32(0.0):
            self.tracking_frequency = f32(self.cf)
        if self.cf_changed:
            self.tracking_frequency = f32(self.cf)
            self.cf_changed = False
        if self.max_peak is None:
            self.max_peak = [f32(-130.0), f32(self.cf)]
        if valid and abs_peak > self.max_peak[0]:
            self.max_peak = [abs_peak, f32(focus_lo + peak_in_focus) * freq_per_bin + (f32(self.cf) - nyq)]
            self.t_last_max = now_ms
        if self.t_last_update < self.t_last_max and now_ms - self.t_last_max > 300:
            self.tracking_frequency = self.max_peak[1]
            self.t_last_update = now_ms
            self.max_peak[0] = f32(-130.0)
        # 6.6 detection
        above_thr = valid and o["mean_snr_sigma"] >= f32(4.0)
        if above_thr:
            if self.peak_confirmed < 1:  # confirmation = 1
                self.peak_confirmed += 1
        else:
            self.peak_confirmed = 0
        flag = 3 if (above_thr and self.peak_confirmed >= 1) else 0
        self.det_buf[self.det_idx] = flag
        self.det_idx = (self.det_idx + 1) % 3
        o["detection_flag"] = max(self.det_buf)
        return self._record(diag)

    def _record(self, diag: dict) -> dict:
        r = dict(self.out)
        # getTrackingFrequency rounds the float latch to the nearest integer (fft_process.h:41)
        t = float(self.tracking_frequency)  # std::round: halves away from zero
        r["tracking_frequency"] = int(np.sign(t) * np.floor(abs(t) + 0.5))
        r.update(diag)
        return r

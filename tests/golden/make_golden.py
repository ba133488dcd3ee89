"""Generate the golden fixtures in tests/golden/ (run in the container that has /root/reference).

Every expected SSB output comes from the REFERENCE's own src/ssb/ssb_demod_opt.cpp, built unmodified by
`make -C oracle ref` into oracle/_ref/ref_ssb; each stream runs in a fresh reference process, because
processSSB_opt keeps its filter state in function statics (ssb_demod_opt.cpp:223-282).

Every expected spectrum comes from numpy's float64 FFT (the DFT that fftwf_plan_dft_1d computes,
fft_process.cpp:77-79), squared and fftshifted like fft_process.cpp:83-97.  The vendored FFTW is a
prebuilt archive and is never linked, so the DFT definition is the pin for the spectrum.

Window geometry is the table SURVEY.md section 8 measured on the reference build.

Inputs are stored as raw bytes (never regenerated from cos/sin on another machine).

    python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402


def np_unpack(fmt: int, raw: np.ndarray) -> np.ndarray:
    """Same conventions as include/sdrg.h, in numpy float32 arithmetic (IEEE, no contraction)."""
    if fmt == O.CS8:
        return raw.astype(np.float32) * np.float32(1.0 / 128.0)
    if fmt == O.CU8:
        return (raw.astype(np.float32) - np.float32(127.4)) * np.float32(1.0 / 128.0)
    if fmt == O.CS16:
        return raw.astype(np.float32) * np.float32(1.0 / 32768.0)
    return raw.astype(np.float32)


def np_power_shifted_f64(iq: np.ndarray) -> np.ndarray:
    c = iq[0::2].astype(np.float64) + 1j * iq[1::2].astype(np.float64)
    X = np.fft.fft(c)
    return np.fft.fftshift((X.real ** 2 + X.imag ** 2)).astype(np.float32)


def make_case(name: str, fmt: int, n: int, fs: int, stream_modes, tones, spectra_frames, seed: int, **synth):
    S = len(stream_modes)
    F = len(stream_modes[0])
    raw = np.stack([O.synth_frames(F, n, fmt, tone_hz=tones[s], fs=fs, seed=seed + s, **synth) for s in range(S)])
    pcm_len = O.ssb_pcm_len(n, fs)
    pcm = np.zeros((S, F, pcm_len), dtype=np.int16)
    for s in range(S):
        frames = np.stack([np_unpack(fmt, raw[s, f]).reshape(n, 2) for f in range(F)])
        outs = O.ref_ssb_run(frames, fs, stream_modes[s])
        for f in range(F):
            assert outs[f].size == pcm_len, (outs[f].size, pcm_len)
            pcm[s, f] = outs[f]
    spectra = np.stack([np_power_shifted_f64(np_unpack(fmt, raw[s, f])) for (s, f) in spectra_frames]) \
        if spectra_frames else np.zeros((0, n), np.float32)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), raw=raw, fmt=np.int32(fmt), n=np.int32(n),
                        fs=np.int64(fs), modes=np.array(stream_modes, dtype=np.int32), pcm=pcm,
                        spectra_idx=np.array(spectra_frames, dtype=np.int32).reshape(-1, 2), spectra=spectra,
                        tones=np.array(tones, dtype=np.float64))
    print(name, raw.shape, raw.dtype, "pcm", pcm.shape)


def main() -> None:
    if not O.have_ref():
        O.build()
    assert O.have_ref(), "oracle/_ref/ref_ssb missing: needs /root/reference"

    # C1/C2/C3 shape: CS8, N=16384, fs=2 MHz, 4 streams x 3 frames, mixed sound modes (mode 3 = unknown:
    # keeps the previous mode's globals, ssb_demod_opt.cpp:230-255)
    make_case("golden_cs8_16384", O.CS8, 16384, 2_000_000, [[1, 1, 1], [2, 2, 2], [0, 1, 2], [1, 3, 2]],
              [1500.0, 1000.0, -2500.0, 400.0], [(0, 0), (1, 0)], seed=0x5D12)
    # C5 shape: CS16 (LimeSDR path), N=65536
    make_case("golden_cs16_65536", O.CS16, 65536, 2_000_000, [[1, 1]], [3000.0], [(0, 0)], seed=0x5D13)
    # RTL-SDR CU8 at 2.4 MHz (decim 50), and CF32 at the SDRConfig default 2.5 MHz (decim 52)
    make_case("golden_cu8_8192_fs2400k", O.CU8, 8192, 2_400_000, [[1, 1], [0, 0]], [700.0, -1200.0], [(0, 1)],
              seed=0x5D14)
    make_case("golden_cf32_4096_fs2500k", O.CF32, 4096, 2_500_000, [[1, 2]], [2000.0], [(0, 0)], seed=0x5D15)
    # edges: exactly one FIR output (N=256), and no output at all (N=128 -> 129 taps > 128 samples)
    make_case("golden_cs8_256", O.CS8, 256, 2_000_000, [[1, 1, 1]], [5000.0], [(0, 2)], seed=0x5D16)
    make_case("golden_cs8_128", O.CS8, 128, 2_000_000, [[1, 1]], [5000.0], [], seed=0x5D17)

    # filter design parameters from the reference build (bit patterns)
    coefs = {}
    for fs in (2_000_000, 2_400_000, 2_500_000):
        for (fc, q) in ((3200.0, 0.9), (2200.0, 1.2)):
            coefs[f"lpf_{fs}_{int(fc)}"] = O.ref_coefs("lpf", float(fs), fc, q)
    coefs["hp_48000_1200"] = O.ref_coefs("hp", 48000.0, 1200.0, 0.7)
    coefs["bp_48000_2400"] = O.ref_coefs("bp", 48000.0, 2400.0, 0.6)
    for (size, dec) in ((16384, 41), (65536, 41), (8192, 50), (4096, 52), (256, 41), (129, 41)):
        coefs[f"taps_{size}_{dec}"] = O.ref_taps(size, dec)
    np.savez_compressed(os.path.join(HERE, "golden_ssb_design.npz"), **coefs)
    print("design", sorted(coefs))

    # window geometry as measured on the reference build (preamble and 8(a) row 7)
    geometry = {
        "source": "SURVEY.md section 8 (computed by the survey with the reference's own float expressions)",
        "cases": [
            {"sample_rate": 2000000, "n": 16384, "focus_khz": 5, "focus": [8151, 8231], "win_bins_1k": 9,
             "n_bottom": 4, "n_ref": 10,
             "windows_first_two": [[8273, 8354], [8028, 8109]], "windows_last_two": [[8929, 9010], [7372, 7453]],
             "ref_bins_total": 820, "decim": 41, "pcm_len": 394},
            {"sample_rate": 2000000, "n": 65536, "focus_khz": 5, "focus": [32604, 32930], "win_bins_1k": 33,
             "n_ref": 10},
            {"sample_rate": 2000000, "n": 65536, "focus_khz": 200, "focus": [26214, 39320], "n_ref": 2,
             "window_len": 13107, "n_bottom": 1},
        ],
        "cw_peak": {"sample_rate": 2000000, "n": 16384, "tone_hz": 1000.0, "peak_bin": 8200},
    }
    with open(os.path.join(HERE, "geometry.json"), "w") as f:
        json.dump(geometry, f, indent=1)


if __name__ == "__main__":
    main()

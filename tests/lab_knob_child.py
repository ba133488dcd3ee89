"""Child process of tests/test_gpu_lab_knobs.py: one engine, two calls over 64 streams (every stage), prints a
sha256 per output.  Run with and without lab environment variables set before anything touches the GPU."""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sdr-for-android-lib_amd"), os.path.join(ROOT, "oracle")]

import numpy as np  # noqa: E402

import oracle as O  # noqa: E402
import sdrg  # noqa: E402

n, fs, B = 16384, 2_000_000, 64
raw = np.stack([O.synth_frames(2, n, O.CS8, tone_hz=150.0 * b - 4000.0, fs=fs, seed=b) for b in range(B)])
eng = sdrg.Engine(sdrg.SDRConfig(centerFrequency=100_000_000, samplesPerReading=n, sampleRate=fs,
                                 freqFocusRangeKhz=5, soundMode=1), B)
h = {k: hashlib.sha256() for k in ("spectra", "records", "pcm")}
for f in range(2):
    spec, rec, pcm = eng.process(raw[:, f], fmt=sdrg.CS8, stages=sdrg.STAGE_ALL, now_ms=1000 + 8 * f)
    h["spectra"].update(spec.tobytes())
    for fld in sdrg.RECORD_DTYPE.names:
        h["records"].update(np.ascontiguousarray(rec[fld]).tobytes())
    h["pcm"].update(pcm.tobytes())
eng.close()
print(" ".join(f"{k}={v.hexdigest()}" for k, v in h.items()))

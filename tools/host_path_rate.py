"""PCIe-inclusive rate of the host-buffer path (sdrg_engine_process_host): raw CS8 frames in host memory, spectra,
records and PCM back to host memory per call, as the JNI read() loop uses it.  Not the bench metric.

    python tools/host_path_rate.py [streams] [calls]
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "sdr-for-android-lib_amd"))
import torch  # noqa: E402,F401  (load torch's HIP runtime first)
import sdrg  # noqa: E402


def main() -> None:
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    calls = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    n, fs = 16384, 2_000_000
    cfg = sdrg.SDRConfig(centerFrequency=100_000_000, samplesPerReading=n, sampleRate=fs, freqFocusRangeKhz=5,
                         soundMode=1)
    eng = sdrg.Engine(cfg, B)
    rng = np.random.default_rng(1)
    iq = rng.integers(-20, 20, size=(B, 2 * n), dtype=np.int8)
    hb = [sdrg.HostBuffer((B, 2 * n), np.int8), sdrg.HostBuffer((B, n), np.float32),
          sdrg.HostBuffer((B,), sdrg.RECORD_DTYPE), sdrg.HostBuffer((B, eng.pcm_len), np.int16)]
    hb[0].array[...] = iq
    for pinned in (False, True):
        src = hb[0].array if pinned else iq
        out = (hb[1].array, hb[2].array, hb[3].array) if pinned else None
        for stages, name in ((sdrg.STAGE_ALL, "all stages, spectra + records + PCM to host"),
                             (sdrg.STAGE_SSB | sdrg.STAGE_AUDIO_PULSE, "SSB only, PCM to host")):
            eng.process(src, fmt=sdrg.CS8, stages=stages, now_ms=1000, out=out)  # warm-up (allocations, first touch)
            t0 = time.perf_counter()
            for k in range(calls):
                eng.process(src, fmt=sdrg.CS8, stages=stages, now_ms=1010 + 8 * k, out=out)
            dt = (time.perf_counter() - t0) / calls
            print(f"{name}: {dt * 1e3:.2f} ms/call for {B} x {n} = {B * n / dt / 1e6:.0f} M IQ samples/s "
                  f"({'page-locked sdrg.HostBuffer' if pinned else 'pageable numpy'} buffers)", flush=True)
    for h in hb:
        h.close()
    eng.close()


if __name__ == "__main__":
    main()

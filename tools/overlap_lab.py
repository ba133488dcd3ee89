"""Lab: can the SSB pipeline (on part of the chip) and the spectrum kernel (on the rest) run side by side?
Two engines on their own HIP streams: A runs SSB for S_A streams (one pipeline workgroup per 16 streams, one
per CU), B runs the spectrum (+stats) for 4096 frames with a persistent grid limited by SDRG_SPECTRUM_GRID.
Prints per-step ms alone and together."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sdr-for-android-lib_amd"), ROOT]
import sdrg  # noqa: E402
from bench import synth_device_frames  # noqa: E402

N, FS = 16384, 2_000_000
dev = torch.device("cuda", 0)
S_A = int(os.environ.get("S_A", "2048"))
S_B = 4096
cfg = sdrg.SDRConfig(centerFrequency=100_000_000, samplesPerReading=N, sampleRate=FS, freqFocusRangeKhz=5, soundMode=1)
A = sdrg.Engine(cfg, S_A)
B = sdrg.Engine(cfg, S_B)
iq = synth_device_frames(torch, dev, S_B, seed=7)
spec = torch.empty((S_B, N), dtype=torch.float32, device=dev)
rec = torch.zeros((S_B, sdrg.RECORD_DTYPE.itemsize), dtype=torch.uint8, device=dev)
pcm = torch.empty((S_B, A.pcm_len), dtype=torch.int16, device=dev)
torch.cuda.synchronize()


def run(which, steps=20):
    for it in range(steps + 3):
        if it == 3:
            A.synchronize(); B.synchronize(); t0 = time.perf_counter()
        if "a" in which:
            A.process_device(iq.data_ptr(), sdrg.CS8, sdrg.STAGE_SSB, None, None, pcm.data_ptr(), 1000 + it)
        if "b" in which:
            B.process_device(iq.data_ptr(), sdrg.CS8, sdrg.STAGE_SPECTRUM | sdrg.STAGE_STATS, spec.data_ptr(),
                             rec.data_ptr(), None, 1000 + it)
        if "s" in which:  # serial: B waits for A each step
            A.synchronize()
    A.synchronize(); B.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


out = {"S_A": S_A, "grid": os.environ.get("SDRG_SPECTRUM_GRID"), "ssb_alone": run("a"), "spec_alone": run("b"),
       "both": run("ab")}
print(json.dumps(out))

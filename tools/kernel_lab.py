#!/usr/bin/env python3
"""Kernel lab driver (profiling only, not a benchmark): repeated engine calls of chosen stages on resident
synthetic inputs (3 rotated batches), so rocprofv3 counter passes see only the kernels of interest.
    python tools/kernel_lab.py --stages spectrum --calls 20            # spectrum16k_kernel alone
    python tools/kernel_lab.py --stages spectrum+stats --n 65536 --fmt CS16 --streams 1024 --focus 200
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "sdr-for-android-lib_amd"))

import bench  # noqa: E402  (synth_device_frames)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stages", default="spectrum", choices=["spectrum", "spectrum+stats", "ssb", "all"])
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--fmt", default="CS8", choices=["CS8", "CS16"])
    ap.add_argument("--streams", type=int, default=4096)
    ap.add_argument("--focus", type=int, default=5)
    ap.add_argument("--calls", type=int, default=20)
    ap.add_argument("--pipelined", type=int, default=0)
    a = ap.parse_args()
    import torch
    import sdrg
    dev = torch.device("cuda", 0)
    cs16 = a.fmt == "CS16"
    fmt = sdrg.CS16 if cs16 else sdrg.CS8
    eng = sdrg.Engine(sdrg.SDRConfig(centerFrequency=100_000_000, samplesPerReading=a.n, sampleRate=2_000_000,
                                     freqFocusRangeKhz=a.focus, soundMode=1), a.streams)
    iqs = [bench.synth_device_frames(torch, dev, a.streams, seed=11 + k, n=a.n, cs16=cs16) for k in range(3)]
    spec = torch.empty((a.streams, a.n), dtype=torch.float32, device=dev)
    rec = torch.zeros((a.streams, sdrg.RECORD_DTYPE.itemsize), dtype=torch.uint8, device=dev)
    pcm = torch.empty((a.streams, max(eng.pcm_len, 1)), dtype=torch.int16, device=dev)
    st = {"spectrum": sdrg.STAGE_SPECTRUM, "spectrum+stats": sdrg.STAGE_SPECTRUM | sdrg.STAGE_STATS,
          "ssb": sdrg.STAGE_SSB, "all": sdrg.STAGE_ALL}[a.stages]
    eng.set_pipelining(bool(a.pipelined))
    eng.set_profiling(True)
    torch.cuda.synchronize()
    for k in range(a.calls):
        eng.process_device(iqs[k % 3].data_ptr(), fmt, st, spec.data_ptr(), rec.data_ptr(), pcm.data_ptr(), 1000 + 8 * k)
    eng.synchronize()
    print({k: round(v, 4) for k, v in eng.timing_stats().items()})
    eng.close()


if __name__ == "__main__":
    main()

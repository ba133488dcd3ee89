# lab: the first steps after a host synchronisation, for a kernel trace (rocprofv3 --kernel-trace, then
# tools/lab/startup_blocks.py).  After a pre-roll, phases of 5 blocks each, every block after eng.synchronize():
#   P1: 20 c3 steps (STAGE_ALL) right after the synchronisation (the driver command's timed region)
#   P2: 20 c3 steps after a further 20 ms idle
#   P3: 40 FFT + statistics steps (~130 us each: is the dip at a call count or at a time after the start?)
#   P4: 20 SSB-only steps
# Phases are 50 ms apart.  python tools/lab/startup_trace.py
import os, sys, time
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "sdr-for-android-lib_amd"))
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch
import bench
import sdrg
dev = torch.device("cuda", 0)
cfg = sdrg.SDRConfig(centerFrequency=bench.CF, samplesPerReading=bench.N, sampleRate=bench.FS, freqFocusRangeKhz=5, soundMode=1)
eng = sdrg.Engine(cfg, bench.B)
iqs = [bench.synth_device_frames(torch, dev, bench.B, seed=7 + k, n=bench.N, cs16=False) for k in range(3)]
specs = [torch.empty((bench.B, bench.N), dtype=torch.float32, device=dev) for _ in range(2)]
recs = [torch.zeros((bench.B, sdrg.RECORD_DTYPE.itemsize), dtype=torch.uint8, device=dev) for _ in range(2)]
pcm = torch.empty((bench.B, eng.pcm_len), dtype=torch.int16, device=dev)
eng.set_pipelining(1 | sdrg.PIPELINE_STATS_ASYNC)
eng.set_profiling(True)
torch.cuda.synchronize()
calls, now = [0], [1000]


def step(st):
    k = calls[0]
    calls[0] += 1
    eng.process_device(iqs[k % 3].data_ptr(), sdrg.CS8, st, specs[k % 2].data_ptr(),
                       recs[k % 2].data_ptr() if st & sdrg.STAGE_STATS else None,
                       pcm.data_ptr() if st & sdrg.STAGE_SSB else None, now[0])
    now[0] += 8


def block(st, k, idle_ms=0.0):
    eng.synchronize()
    torch.cuda.synchronize()
    if idle_ms:
        time.sleep(idle_ms / 1e3)
    t0 = time.perf_counter()
    for _ in range(k):
        step(st)
    eng.synchronize()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / k * 1e3


for _ in range(8):  # pre-roll
    block(sdrg.STAGE_ALL, 25)
FS = sdrg.STAGE_SPECTRUM | sdrg.STAGE_STATS
for name, st, k, idle in (("P1", sdrg.STAGE_ALL, 20, 0), ("P2", sdrg.STAGE_ALL, 20, 20), ("P3", FS, 40, 0),
                          ("P4", sdrg.STAGE_SSB, 20, 0)):
    time.sleep(0.05)
    ms = [block(st, k, idle) for _ in range(5)]
    print(name, "ms/step", " ".join(f"{x:.4f}" for x in ms), flush=True)

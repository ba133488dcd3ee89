# lab: ms/step of consecutive 25-step blocks of the pipelined c3 step from a cold engine, per pipelining mode
# (how many steps the schedule takes to settle); one process per mode: python tools/lab/warm_trace.py MODE
import os, sys, time
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "sdr-for-android-lib_amd"))
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch
import bench
import sdrg
mode = int(sys.argv[1])
dev = torch.device("cuda", 0)
cfg = sdrg.SDRConfig(centerFrequency=bench.CF, samplesPerReading=bench.N, sampleRate=bench.FS, freqFocusRangeKhz=5, soundMode=1)
eng = sdrg.Engine(cfg, bench.B)
iqs = [bench.synth_device_frames(torch, dev, bench.B, seed=7 + k, n=bench.N, cs16=False) for k in range(3)]
spec = torch.empty((bench.B, bench.N), dtype=torch.float32, device=dev)
rec = torch.zeros((bench.B, sdrg.RECORD_DTYPE.itemsize), dtype=torch.uint8, device=dev)
pcm = torch.empty((bench.B, eng.pcm_len), dtype=torch.int16, device=dev)
eng.set_pipelining(mode)
eng.set_profiling(True)
torch.cuda.synchronize()
now, out = 1000, []
for blk in range(16):
    t0 = time.perf_counter()
    for i in range(25):
        eng.process_device(iqs[i % 3].data_ptr(), sdrg.CS8, sdrg.STAGE_ALL, spec.data_ptr(), rec.data_ptr(), pcm.data_ptr(), now)
        now += 8
    eng.synchronize()
    out.append((time.perf_counter() - t0) / 25 * 1e3)
print(f"mode {mode}: " + " ".join(f"{x:.3f}" for x in out), flush=True)

# lab: pipelined default steps with and without the engine's per-call profiling events
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
spec = torch.empty((bench.B, bench.N), dtype=torch.float32, device=dev)
rec = torch.zeros((bench.B, sdrg.RECORD_DTYPE.itemsize), dtype=torch.uint8, device=dev)
pcm = torch.empty((bench.B, eng.pcm_len), dtype=torch.int16, device=dev)
eng.set_pipelining(sdrg.PIPELINE_INPUTS_READY if os.environ.get("INPUTS_READY") else True)
now = [1000]
def run(k, prof):
    eng.set_profiling(prof)
    eng.synchronize(); torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(k):
        eng.process_device(iqs[i % 3].data_ptr(), sdrg.CS8, sdrg.STAGE_ALL, spec.data_ptr(), rec.data_ptr(), pcm.data_ptr(), now[0])
        now[0] += 8
    eng.synchronize(); torch.cuda.synchronize()
    return (time.perf_counter() - t0) / k * 1e3
run(100, False)
for rep in range(3):
    a = run(200, False); b = run(200, True)
    print(f"no events {a:.4f} ms/step   events {b:.4f} ms/step")
# host-side enqueue cost: calls issued back to back without waiting (the GPU queue absorbs them)
eng.set_profiling(False)
eng.synchronize(); torch.cuda.synchronize()
ts = []
for i in range(40):
    t = time.perf_counter()
    eng.process_device(iqs[i % 3].data_ptr(), sdrg.CS8, sdrg.STAGE_ALL, spec.data_ptr(), rec.data_ptr(), pcm.data_ptr(), now[0])
    ts.append((time.perf_counter() - t) * 1e3)
eng.synchronize()
ts.sort()
print(f"host enqueue per call: median {ts[20]:.4f} ms, min {ts[0]:.4f}, max {ts[-1]:.4f}")

# lab: pipelined steps of the c3 batch with and without the pulse detectors (the upper bound of taking them off
# the two streams' critical paths), alternating, profiling off
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
eng.set_pipelining(int(os.environ.get("LAB_PIPE_MODE", "2")))
now = [1000]
def run(k, stages, prof=False):
    eng.set_profiling(prof)
    eng.synchronize(); torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(k):
        eng.process_device(iqs[i % 3].data_ptr(), sdrg.CS8, stages, spec.data_ptr(), rec.data_ptr(), pcm.data_ptr(), now[0])
        now[0] += 8
    eng.synchronize(); torch.cuda.synchronize()
    return (time.perf_counter() - t0) / k * 1e3
legs = {"all": sdrg.STAGE_ALL, "no spectral pulse": sdrg.STAGE_ALL & ~sdrg.STAGE_SPECTRAL_PULSE,
        "no audio pulse": sdrg.STAGE_ALL & ~sdrg.STAGE_AUDIO_PULSE, "no pulse": sdrg.STAGE_HOT_PATH}
for st in legs.values():
    run(60, st)
for rep in range(3):
    print("  ".join(f"{name} {run(50, st):.4f}" for name, st in legs.items()), flush=True)
for name, st in legs.items():  # per-kernel device times (events), profiled run
    eng.reset_timing_stats() if hasattr(eng, "reset_timing_stats") else None
    ms = run(50, st, True)
    print(f"{name}: {ms:.4f} ms/step, timing stats {eng.timing_stats()}", flush=True)

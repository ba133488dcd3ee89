# lab: ms/step of the pipelined c3 batch (all stages) and the engine's per-kernel event times, one process
# (so per-process env knobs such as SDRG_PIPE_MAP apply); prints one line
import os, sys, time
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "sdr-for-android-lib_amd"))
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch
import bench
import sdrg
label = sys.argv[1] if len(sys.argv) > 1 else "run"
stages = int(sys.argv[2]) if len(sys.argv) > 2 else sdrg.STAGE_ALL
dev = torch.device("cuda", 0)
cfg = sdrg.SDRConfig(centerFrequency=bench.CF, samplesPerReading=bench.N, sampleRate=bench.FS, freqFocusRangeKhz=5, soundMode=1)
eng = sdrg.Engine(cfg, bench.B)
iqs = [bench.synth_device_frames(torch, dev, bench.B, seed=7 + k, n=bench.N, cs16=False) for k in range(3)]
spec = torch.empty((bench.B, bench.N), dtype=torch.float32, device=dev)
rec = torch.zeros((bench.B, sdrg.RECORD_DTYPE.itemsize), dtype=torch.uint8, device=dev)
pcm = torch.empty((bench.B, eng.pcm_len), dtype=torch.int16, device=dev)
eng.set_pipelining(int(os.environ.get("LAB_PIPE_MODE", "2")))
if os.environ.get("LAB_NCO") == "1":  # the configs[2] variant: NCO at +250 kHz, 127-tap FIR (bench.py's configs2_nco127)
    eng.set_ssb_variant(bench.NCO_HZ, 127)
now = [1000]
def run(k, prof):
    eng.set_profiling(prof)
    eng.reset_timing_stats()
    eng.synchronize(); torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(k):
        eng.process_device(iqs[i % 3].data_ptr(), sdrg.CS8, stages, spec.data_ptr(), rec.data_ptr(), pcm.data_ptr(), now[0])
        now[0] += 8
    eng.synchronize(); torch.cuda.synchronize()
    return (time.perf_counter() - t0) / k * 1e3
run(10, False)
a = [run(50, False) for _ in range(3)]
b = run(50, True)
t = eng.timing_stats()
print(f"{label}: ms/step {' '.join(f'{x:.4f}' for x in a)} | profiled {b:.4f} spectrum {t['spectrum_ms']:.4f} "
      f"stats {t['stats_ms']:.4f} ssb {t['ssb_ms']:.4f}", flush=True)

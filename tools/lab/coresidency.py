# lab: which co-resident kernel costs the SSB stream its ~20 us per step over the SSB stage alone (the loop's cycles are
# the same, r5ar stamps): pipelined c3 steps with every stage, without the statistics, without the spectrum, and the
# SSB stage alone; ms per step and the engine's per-stream timings (profiled), alternating
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
eng.set_pipelining(int(os.environ.get("LAB_PIPE_MODE", "6")))
now = [1000]
calls = [0]


def run(k, stages):
    eng.reset_timing_stats()
    eng.synchronize()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k):
        c = calls[0]
        calls[0] += 1
        eng.process_device(iqs[c % 3].data_ptr(), sdrg.CS8, stages, specs[c % 2].data_ptr(), recs[c % 2].data_ptr(),
                           pcm.data_ptr(), now[0])
        now[0] += 8
    eng.synchronize()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / k * 1e3


S = sdrg
legs = {"all": S.STAGE_ALL,
        "no stats": S.STAGE_SPECTRUM | S.STAGE_SSB | S.STAGE_AUDIO_PULSE,
        "no spectrum": S.STAGE_SSB | S.STAGE_AUDIO_PULSE,
        "ssb only": S.STAGE_SSB}
eng.set_profiling(True)
for st in legs.values():
    run(100, st)
for rep in range(3):
    out = []
    for name, st in legs.items():
        ms = run(150, st)
        t = eng.timing_stats()
        out.append(f"{name} {ms:.4f} (ssb {t['ssb_ms']:.4f} spec {t['spectrum_ms']:.4f} stats {t['stats_ms']:.4f})")
    print(" | ".join(out), flush=True)

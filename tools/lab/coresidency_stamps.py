# lab (r5bg): the SSB workgroups' start skew and loop cycles per co-resident stage set (lab stamps build,
# SDRG_PIPE_STAMPS=1); a stamps report follows each BLOCK line.  Formerly: where the SSB kernel's time outside its workgroups' loops goes (lab stamps build, SDRG_PIPE_STAMPS=1, under
# rocprofv3 --kernel-trace): blocks of pipelined c3 steps and of SSB-only steps; the engine's stamps report prints,
# per call, the first workgroup entry, the first loop start and the last loop end (s_memrealtime, 10 ns units), to be
# set against the trace's start / end of the same SSB kernels (tools/lab/ssb_boundary_join.py)
import os, sys
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
now, calls = [1000], [0]


def block(k, stages):
    for _ in range(k):
        c = calls[0]
        calls[0] += 1
        eng.process_device(iqs[c % 3].data_ptr(), sdrg.CS8, stages, specs[c % 2].data_ptr(), recs[c % 2].data_ptr(),
                           pcm.data_ptr(), now[0])
        now[0] += 8
    eng.synchronize()
    torch.cuda.synchronize()


S = sdrg
legs = [("all", S.STAGE_ALL)] if os.environ.get("LAB_ALL_ONLY") else [("all", S.STAGE_ALL),
        ("no-stats", S.STAGE_SPECTRUM | S.STAGE_SSB | S.STAGE_AUDIO_PULSE),
        ("no-audio", S.STAGE_ALL & ~S.STAGE_AUDIO_PULSE),
        ("spectrum+ssb", S.STAGE_SPECTRUM | S.STAGE_SSB),
        ("no-spectrum", S.STAGE_SSB | S.STAGE_AUDIO_PULSE),
        ("ssb", S.STAGE_SSB)]
for _ in range(3):
    block(25, S.STAGE_ALL)
for name, st in legs:
    block(20, st)
    print("BLOCK " + name, file=sys.stderr, flush=True)
    block(60, st)
print("done", file=sys.stderr, flush=True)

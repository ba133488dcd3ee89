"""Lab: the spectrum stage alone on resident IQ (engine process_device, STAGE_SPECTRUM), HIP events around K calls,
and a hash of the last call's spectra (to check two kernels for the same bits).
python tools/lab/spec_time.py [n] [fmt cs8|cs16|cu8|cf32] [streams] [calls]  (SDRG_LIB_PATH selects a variant library)"""
import hashlib
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "sdr-for-android-lib_amd"))
import torch  # noqa: E402
import sdrg  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
fmt_name = sys.argv[2] if len(sys.argv) > 2 else "cs8"
B = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
K = int(sys.argv[4]) if len(sys.argv) > 4 else 50
fmt = {"cs8": sdrg.CS8, "cs16": sdrg.CS16, "cu8": sdrg.CU8, "cf32": sdrg.CF32}[fmt_name]
bps = {"cs8": 2, "cu8": 2, "cs16": 4, "cf32": 8}[fmt_name]
dev = torch.device("cuda", 0)
eng = sdrg.Engine(sdrg.SDRConfig(centerFrequency=100_000_000, samplesPerReading=n, sampleRate=2_000_000,
                                 freqFocusRangeKhz=5, soundMode=1), B)
g = torch.Generator(device=dev)
g.manual_seed(7)
if fmt_name == "cf32":
    iq = torch.randn((B, 2 * n), dtype=torch.float32, device=dev, generator=g)
else:
    iq = torch.randint(0, 256, (B, n * bps), dtype=torch.uint8, device=dev, generator=g)
spec = torch.empty((B, n), dtype=torch.float32, device=dev)
# lab: SPEC_TIME_DIST=rccl (a one-rank sdrg.Dist communicator first) / gloo (a one-rank gloo group) / both
_d = os.environ.get("SPEC_TIME_DIST", "")
if _d in ("gloo", "both"):
    import torch.distributed as tdist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29555")
    tdist.init_process_group("gloo", rank=0, world_size=1)
if _d in ("rccl", "both"):
    _comm = sdrg.Dist(sdrg.dist_unique_id(), 1, 0, device=0)
work = torch.cuda.Stream(dev)
eng.set_stream(work.cuda_stream)
torch.cuda.synchronize()


def call(k):
    eng.process_device(iq.data_ptr(), fmt, sdrg.STAGE_SPECTRUM, spec.data_ptr(), None, None, 1000 + k)


for k in range(5):
    call(k)
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
with torch.cuda.stream(work):
    a.record()
    for k in range(K):
        call(5 + k)
    b.record()
b.synchronize()
us = a.elapsed_time(b) / K * 1e3
gbs = B * n * (bps + 4) / (us * 1e-6) / 1e9
h = hashlib.sha256(spec.cpu().numpy().tobytes()).hexdigest()[:16]
print(f"spectrum n={n} {fmt_name} B={B}: {us:.1f} us per call, {gbs:.0f} GB/s ({gbs / 8000:.3f} of 8 TB/s) "
      f"hash {h} ({os.path.basename(os.environ.get('SDRG_LIB_PATH', 'product'))} "
      f"alone={os.environ.get('SDRG_K16_ALONE', '-')} dist={_d or '-'})", flush=True)
eng.set_stream(None)
eng.close()

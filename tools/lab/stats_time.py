"""Lab: the statistics kernel alone on resident spectra (sdrg_engine_signal_strength_device), HIP events around K calls.
python tools/lab/stats_time.py [n] [focus_khz] [streams] [calls]  (SDRG_LIB_PATH selects a variant library)"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "sdr-for-android-lib_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import sdrg  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
focus = int(sys.argv[2]) if len(sys.argv) > 2 else 200
B = int(sys.argv[3]) if len(sys.argv) > 3 else 1024
K = int(sys.argv[4]) if len(sys.argv) > 4 else 30
dev = torch.device("cuda", 0)
eng = sdrg.Engine(sdrg.SDRConfig(centerFrequency=100_000_000, samplesPerReading=n, sampleRate=2_000_000,
                                 freqFocusRangeKhz=focus, soundMode=1), B)
g = torch.Generator(device=dev)
g.manual_seed(1)
spec = torch.empty((B, n), dtype=torch.float32, device=dev).exponential_(1.0, generator=g)
spec[:, n // 2 + 37] *= 1e4
rec = torch.zeros((B, sdrg.RECORD_DTYPE.itemsize), dtype=torch.uint8, device=dev)
work = torch.cuda.Stream(dev)
eng.set_stream(work.cuda_stream)
lib = sdrg.load()
torch.cuda.synchronize()


def call(k):
    rc = lib.sdrg_engine_signal_strength_device(eng._h, ctypes.c_void_p(spec.data_ptr()), ctypes.c_void_p(rec.data_ptr()),
                                                 ctypes.c_int64(1000 + k))
    assert rc == 0, rc


for k in range(5):
    call(k)
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
with torch.cuda.stream(work):
    a.record()
    for k in range(K):
        call(5 + k)
    b.record()
b.synchronize()
print(f"stats n={n} focus={focus} B={B}: {a.elapsed_time(b) / K * 1e3:.1f} us per call "
      f"({os.environ.get('SDRG_LIB_PATH', 'product')}, single={os.environ.get('SDRG_WIDE_SINGLE', '0')})", flush=True)
eng.set_stream(None)
eng.close()

"""BASELINE configs[3]'s collective on the one GPU of the box: a ONE-rank RCCL process group
(backend "nccl", device_id cuda:0) started in a fresh spawned interpreter before any GPU call, the real engine
pipelined on a torch stream for several steps, and every step's records, focus-window spectra and full spectra (the
fftCallback payload, sdr-bridge-java-soapy.cpp:456-466) gathered with sdrg.shard on HIP tensors, with no host
synchronisation between the steps -- the collectives are ordered after each step's kernels on the stream alone.
The gathered buffers must equal the engine's own outputs bit for bit, and dist.get_backend() must be "nccl"."""
import os
import socket
import sys

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

N, FS, CF, FOCUS, B, STEPS = 16384, 2_000_000, 100_000_000, 5, 256, 4


def _worker(port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
    sys.path[:0] = [os.path.join(ROOT, "sdr-for-android-lib_amd"), os.path.join(ROOT, "oracle")]
    try:
        import torch
        import torch.distributed as dist
        import oracle as O
        import sdrg
        from sdrg import shard

        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
        backend = dist.get_backend()
        raws = np.stack([O.synth_frames(STEPS, N, O.CS8, tone_hz=170.0 * (s % 23) - 1900.0, fs=FS, seed=4400 + s)
                         for s in range(B)], axis=1)
        eng = sdrg.Engine(sdrg.SDRConfig(centerFrequency=CF, samplesPerReading=N, sampleRate=FS,
                                         freqFocusRangeKhz=FOCUS, soundMode=1), B, device=0)
        work = torch.cuda.Stream(dev)
        torch.cuda.set_stream(work)  # the collectives and the engine share this stream
        eng.set_stream(work.cuda_stream)
        eng.set_pipelining(sdrg.PIPELINE_INPUTS_READY)
        iq = [torch.from_numpy(raws[k]).to(dev) for k in range(STEPS)]
        spec = [torch.empty((B, N), dtype=torch.float32, device=dev) for _ in range(STEPS)]
        rec = [torch.zeros((B, sdrg.RECORD_DTYPE.itemsize), dtype=torch.uint8, device=dev) for _ in range(STEPS)]
        pcm = torch.empty((B, eng.pcm_len), dtype=torch.int16, device=dev)
        lo, nb = sdrg.focus_window(FS, N, FOCUS)
        g_rec = [torch.full_like(r, 0xEE) for r in rec]
        g_foc = [torch.full((B, nb), -1.0, dtype=torch.float32, device=dev) for _ in range(STEPS)]
        g_spec = [torch.full_like(s, -1.0) for s in spec]
        stage = torch.empty((B, nb), dtype=torch.float32, device=dev)
        torch.cuda.synchronize()
        for k in range(STEPS):  # no host synchronisation inside the loop
            eng.process_device(iq[k].data_ptr(), sdrg.CS8, sdrg.STAGE_ALL, spec[k].data_ptr(), rec[k].data_ptr(),
                               pcm.data_ptr(), 1000 + 8 * k)
            r = shard.gather_records(rec[k], 1, 0, out=g_rec[k])
            f = shard.gather_focus(spec[k], lo, nb, 1, 0, out=g_foc[k], staging=stage)
            s = shard.gather_spectra(spec[k], 1, 0, out=g_spec[k])
            assert r is g_rec[k] and f is g_foc[k] and s is g_spec[k]
        eng.synchronize()
        torch.cuda.synchronize()
        ok = {}
        for k in range(STEPS):
            ok[f"records{k}"] = torch.equal(g_rec[k], rec[k])
            ok[f"focus{k}"] = torch.equal(g_foc[k], spec[k][:, lo:lo + nb])
            ok[f"spectra{k}"] = torch.equal(g_spec[k], spec[k])
        # the engine really produced distinct steps (not one buffer gathered four times)
        ok["distinct"] = not torch.equal(spec[0], spec[1])
        eng.set_stream(None)
        eng.close()
        dist.destroy_process_group()
        q.put(("ok", backend, ok))
    except Exception as exc:  # reported to the parent
        q.put(("error", repr(exc), None))
        raise


def test_one_rank_rccl_gathers_equal_engine_outputs():
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(port, q))
    p.start()
    status, backend, ok = q.get(timeout=240)
    p.join(timeout=120)
    assert status == "ok", backend
    assert p.exitcode == 0
    assert backend == "nccl"
    assert ok and all(ok.values()), ok

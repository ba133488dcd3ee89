"""BASELINE configs[3]'s path on the GPU: streams sharded over ranks, each rank running the REAL HIP
engine for its block of streams on a torch stream (sdrg_engine_set_stream), pipelined, and gathering every step's
72-byte records and focus-window spectra to rank 0 (sdrg.shard, the same calls bench.py makes at N > 1), then the
PCM of all steps.  Two ranks on the one GPU of the box, gloo (gathers staged through host memory), spawned as fresh
interpreters.  Rank 0's gathered data must equal one engine over all 2B streams bit for bit."""
import os
import socket
import sys

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

N, FS, CF, FOCUS, B, STEPS = 16384, 2_000_000, 100_000_000, 5, 96, 3


def _inputs(first, last):
    """[STEPS][last-first][2N] int8: stream s's frames depend only on its global id s."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    per = [O.synth_frames(STEPS, N, O.CS8, tone_hz=150.0 * (s % 29) - 2100.0, fs=FS, seed=9000 + s)
           for s in range(first, last)]
    return np.stack(per, axis=1)


def _run_engine(torch, sdrg, first, last, dev, gather=None):
    """STEPS pipelined calls over streams [first, last) on a torch stream; gather(step, rec, spec) per step."""
    nb = last - first
    raws = _inputs(first, last)
    eng = sdrg.Engine(sdrg.SDRConfig(centerFrequency=CF, samplesPerReading=N, sampleRate=FS, freqFocusRangeKhz=FOCUS,
                                     soundMode=1), nb, device=0)
    work = torch.cuda.Stream(dev)
    torch.cuda.set_stream(work)
    eng.set_stream(work.cuda_stream)
    eng.set_pipelining(True)
    iq = [torch.from_numpy(raws[k]).to(dev) for k in range(STEPS)]
    spec = torch.empty((nb, N), dtype=torch.float32, device=dev)
    rec = torch.zeros((nb, sdrg.RECORD_DTYPE.itemsize), dtype=torch.uint8, device=dev)
    pcm = [torch.empty((nb, eng.pcm_len), dtype=torch.int16, device=dev) for _ in range(STEPS)]
    out = []
    for k in range(STEPS):
        eng.process_device(iq[k].data_ptr(), sdrg.CS8, sdrg.STAGE_ALL, spec.data_ptr(), rec.data_ptr(),
                           pcm[k].data_ptr(), 1000 + 8 * k)
        out.append(gather(k, rec, spec) if gather else (rec.cpu(), spec.cpu()))
    eng.synchronize()
    torch.cuda.synchronize()
    eng.set_stream(None)
    eng.close()
    return out, [p.cpu() for p in pcm]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path[:0] = [os.path.join(ROOT, "sdr-for-android-lib_amd")]
    try:
        import torch
        import torch.distributed as dist
        import sdrg
        from sdrg import shard

        dist.init_process_group("gloo", rank=rank, world_size=world)
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        first, last = shard.stream_range(rank, world, B)
        lo, nb = sdrg.focus_window(FS, N, FOCUS)
        rec_out = torch.empty((world * B, sdrg.RECORD_DTYPE.itemsize), dtype=torch.uint8) if rank == 0 else None

        def gather(k, rec, spec):
            r = shard.gather_records(rec.cpu(), world, rank, dst=0, out=None if rec_out is None else rec_out.clone())
            f = shard.gather_records(spec[:, lo:lo + nb].contiguous().cpu(), world, rank, dst=0)
            return (r, f)

        steps, pcms = _run_engine(torch, sdrg, first, last, dev, gather)
        pcm_all = [shard.gather_records(p.view(torch.uint8), world, rank, dst=0) for p in pcms]  # int16 as bytes
        dist.barrier()
        dist.destroy_process_group()
        if rank == 0:
            q.put(("ok", [(r.numpy(), f.numpy()) for r, f in steps], [p.numpy() for p in pcm_all]))
    except Exception as exc:  # reported to the parent
        q.put(("error", f"rank {rank}: {exc!r}", None))
        raise


def test_sharded_gpu_engines_equal_single_engine():
    import torch.multiprocessing as mp
    world = 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    status, steps, pcm = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
    assert status == "ok", steps
    for p in procs:
        assert p.exitcode == 0
    # the same 2B streams through one engine in this process
    import torch
    import sdrg
    dev = torch.device("cuda", 0)
    lo, nb = sdrg.focus_window(FS, N, FOCUS)
    want, want_pcm = _run_engine(torch, sdrg, 0, world * B, dev)
    torch.cuda.set_stream(torch.cuda.default_stream(dev))
    for k in range(STEPS):
        r, f = steps[k]
        # field by field: the record's 4 tail padding bytes are unspecified
        got_r = np.ascontiguousarray(r).view(sdrg.RECORD_DTYPE).reshape(-1)
        want_r = np.ascontiguousarray(want[k][0].numpy()).view(sdrg.RECORD_DTYPE).reshape(-1)
        for fld in sdrg.RECORD_DTYPE.names:
            np.testing.assert_array_equal(got_r[fld], want_r[fld], err_msg=f"records.{fld} step {k}")
        np.testing.assert_array_equal(f, want[k][1].numpy()[:, lo:lo + nb], err_msg=f"focus spectra step {k}")
        np.testing.assert_array_equal(pcm[k], want_pcm[k].view(torch.uint8).numpy(), err_msg=f"pcm step {k}")

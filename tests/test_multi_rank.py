"""world_size-2 test of the sharded multi-GPU path on CPU (gloo): each rank owns a contiguous block of streams
and runs them for three steps (the per-rank engine is stood in for by the oracle here: no GPU in this suite);
the records gathered to rank 0 must equal a single-process run over all streams bit for bit, and so must the
focus-window spectrum slices gathered beside them (shard.gather_focus)."""
import os
import socket
import sys

import numpy as np
import torch.multiprocessing as mp

from conftest import ROOT

N, FS, CF, FOCUS, B, STEPS = 4096, 2_500_000, 100_000_000, 5, 3, 3


def _records(O, first, last, spectra=None):
    raw = O.synth_frames((last) * STEPS, N, O.CS8, tone_hz=1200.0, fs=FS)
    states = {s: O.FftState(CF, FS, N, FOCUS) for s in range(first, last)}
    out = []
    for step in range(STEPS):
        recs = []
        specs = []
        for s in range(first, last):
            iq = O.unpack(O.CS8, raw[s * STEPS + step], N)
            spec, rec = states[s].process(iq, 1000 + 10 * step)
            recs.append(rec)
            specs.append(np.asarray(spec, np.float32).copy())
        if spectra is not None:
            spectra.append(np.stack(specs))
        arr = np.zeros(len(recs), dtype=O.RECORD_DTYPE)  # fields only: the struct's tail padding is unspecified
        for f in O.RECORD_DTYPE.names:
            arr[f] = [r[f] for r in recs]
        out.append(arr)
    return out


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "sdr-for-android-lib_amd")]
    import torch
    import torch.distributed as dist
    import oracle as O
    import sdrg
    from sdrg import shard

    dist.init_process_group("gloo", rank=rank, world_size=world)
    first, last = shard.stream_range(rank, world, B)
    lo, nb = sdrg.focus_window(FS, N, FOCUS)
    got, got_focus = [], []
    out = None
    specs = []
    for k, recs in enumerate(_records(O, first, last, specs)):
        t = torch.from_numpy(recs.view(np.uint8).reshape(B, -1).copy())
        if rank == 0 and k > 0 and out is None:  # later steps gather into a preallocated buffer (bench.py)
            out = torch.empty((world * B, t.shape[1]), dtype=torch.uint8)
        g = shard.gather_records(t, world, rank, out=out)
        gf = shard.gather_focus(torch.from_numpy(specs[k]), lo, nb, world, rank)
        if rank == 0:
            got.append(g.numpy().copy())
            got_focus.append(gf.numpy().copy())
    dist.barrier()
    dist.destroy_process_group()
    if rank == 0:
        q.put((got, got_focus))


def test_sharded_records_equal_single_process(oracle_mod):
    O = oracle_mod
    world = 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got, got_focus = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    specs = []
    want = _records(O, 0, world * B, specs)
    lo, hi = O.window_geometry(FS, N, FOCUS)[:2]
    assert len(got) == STEPS and len(got_focus) == STEPS
    for step in range(STEPS):
        np.testing.assert_array_equal(got[step], want[step].view(np.uint8).reshape(world * B, -1))
        np.testing.assert_array_equal(got_focus[step], specs[step][:, lo:hi + 1])


def test_stream_range():
    sys.path.insert(0, os.path.join(ROOT, "sdr-for-android-lib_amd"))
    from sdrg import shard
    assert shard.stream_range(0, 2, 4096) == (0, 4096)
    assert shard.stream_range(1, 2, 4096) == (4096, 8192)


def _one_rank_worker(port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
    sys.path[:0] = [os.path.join(ROOT, "sdr-for-android-lib_amd")]
    try:
        import torch
        import torch.distributed as dist
        from sdrg import shard
        rec = torch.arange(5 * 72, dtype=torch.int64).remainder(251).to(torch.uint8).reshape(5, 72)
        bare = shard.gather_records(rec, 1, 0)  # no process group: the tensor itself
        dist.init_process_group("gloo", rank=0, world_size=1)
        out = torch.zeros_like(rec)
        got = shard.gather_records(rec, 1, 0, out=out)  # a one-rank group: the collective runs
        spec = torch.rand(5, 64)
        foc = shard.gather_focus(spec, 10, 7, 1, 0)
        dist.destroy_process_group()
        q.put(("ok", bare is rec, got is out and torch.equal(out, rec), torch.equal(foc, spec[:, 10:17])))
    except Exception as exc:  # reported to the parent
        q.put(("error", repr(exc), None, None))


def test_one_rank_group_runs_the_collective():
    """with a process group initialised, shard.gather_* run the collective at world size 1 too
    (the one-GPU box then drives the same RCCL path bench.py uses at N > 1); without one they return the input."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_one_rank_worker, args=(port, q))
    p.start()
    res = q.get(timeout=120)
    p.join(timeout=60)
    assert res == ("ok", True, True, True), res

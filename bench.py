#!/usr/bin/env python3
"""bench.py — IQ Msamples/s of the reference hot path on MI355X (BASELINE.json metric).

A "step" is one pass of the hot path over one batch: every one of B = 4096 independent streams hands one
16384-sample CS8 frame (2 Msps) to the engine, which runs IQ unpack -> 16384-pt FFT -> |X|^2 -> fftshift ->
signal-strength statistics (FFTProcessor::process, src/dsp/fft_process.cpp:42-379) and the SSB chain ->
int16 PCM (processSSB_opt, src/ssb/ssb_demod_opt.cpp:221-296; the reference's 255-tap FIR, decim 41).
Inputs are synthetic CW tones + noise, resident in HBM before the timed region; every step does the full
work (the per-stream filter state advances from step to step like a live receiver).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu-baseline]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (one process per GPU)

`python bench.py --gpus N` with N > 1 and no WORLD_SIZE in the environment starts the N rank processes itself
(torch.distributed.run as a child process, before anything touches a GPU) and exits with their status.
With N > 1 every rank runs its own 4096 streams (weak scaling) and the per-frame records (+ focus-window
spectra) of each step are gathered to rank 0 by libsdrg.so's own RCCL ncclGather (sdrg_dist_create +
sdrg_engine_gather, the C ABI a C/C++ host behind JNI calls; torch.distributed only carries the control plane:
the communicator id, barriers and the max-over-ranks time, over gloo); value = all ranks' samples /
max-over-ranks time.  The full-spectra gather (the fftCallback payload) is timed after the timed region and
reported separately.
Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "sdr-for-android-lib_amd"))

import numpy as np  # noqa: E402

N = 16384
FS = 2_000_000
CF = 100_000_000
NCO_HZ = 250e3  # --ssb-variant nco127: the NCO offset of the BASELINE configs[2] variant
B = 4096
HBM_PEAK_GBS = 8000.0  # MI355X spec (MI355X_MICROARCH.md)
ALG_BYTES_PER_SAMPLE = {"spectrum": 6.0}  # CS8: 2 B in + 4 B fftshifted float32 power out
ISO_LAUNCHES = 30  # launches of the spectrum stage alone behind roofline_isolated
N_INPUTS = 3  # distinct input batches rotated per step: 3 x 128 MiB > the 256 MiB Infinity Cache
SSB_ISO_CALLS = 20  # joined SSB-only calls timed for ssb_latency_floor.ssb_ms_alone
PROFILED_STEPS = 20  # labelled lines: steps of the separate profiled pass behind their per-kernel times
# labelled lines: timed steps at least this many (the headline times exactly --steps): a labelled line's own timed region
# carries the same fixed fill / drain / clock cost (~0.3 ms) as the headline's, which over the driver's 20
# steps hid their steady rate (configs[2] 9 % under it); each labelled dict records its steps
LABELLED_MIN_STEPS = 100
LAB_HOST_TIMES = os.environ.get("SDRG_BENCH_HOST_TIMES") == "1"
LAB_NO_STEP_GATHER = os.environ.get("SDRG_BENCH_NO_STEP_GATHER") == "1"  # lab: the N > 1 path without its per-step gathers
N_OUTPUTS = 3  # spectra / records buffers rotated per step (asynchronous statistics read a call's spectra late)
# SSB floor: the sample-serial low-pass wave's own instruction issue.  Per sample it issues 6 VALU instructions
# (the packed product of the previous output, 4 dependent adds, the packed product of the output before it) and
# 0.5 LDS instructions (a 16-byte read and write per 4 samples); one wave issues at most one instruction per
# 4 cycles and a dependent VALU op completes in 4 (tools/lab/lat.hip, dep_add.hip), so no
# bit-exact schedule runs the recurrence faster than 26 cycles per sample at the chip's 2.4 GHz maximum clock
SSB_CHAIN_CYCLES = 26
MAX_CLOCK_GHZ = 2.4


def log(msg: str) -> None:
    print(msg, file=sys.stderr, flush=True)


def synth_device_frames(torch, dev, n_streams: int, seed: int, n: int = N, cs16: bool = False):
    """CW tone per stream (inside the 5 kHz focus) + Gaussian noise, generated on the GPU: CS8 (amplitude 60,
    noise 4) or CS16 (amplitude 8000, noise 400), SURVEY 8d C1 / C5."""
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    amp, sig, lo, hi, dt = (8000.0, 400.0, -32768, 32767, torch.int16) if cs16 else (60.0, 4.0, -128, 127, torch.int8)
    tones = (torch.rand(n_streams, 1, device=dev, generator=g, dtype=torch.float64) * 9000.0 - 4500.0)
    t = torch.arange(n, device=dev, dtype=torch.float64)[None, :]
    ph = 2 * np.pi * tones * t / FS
    i = torch.round(amp * torch.cos(ph) + sig * torch.randn(n_streams, n, device=dev, generator=g, dtype=torch.float64))
    q = torch.round(amp * torch.sin(ph) + sig * torch.randn(n_streams, n, device=dev, generator=g, dtype=torch.float64))
    iq = torch.stack([i, q], dim=2).clamp_(lo, hi).to(dt).reshape(n_streams, 2 * n).contiguous()
    return iq


def pmc_traffic(kernel: str, streams: int):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary (profiles/*_hbm_pmc.json, made by
    tools/profile_round.sh + tools/profile_summary.py on this same bench command), or None."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_hbm_pmc.json"))):  # round tags sort in order
        try:
            d = json.load(open(f))
            t = d["kernels"][kernel]["traffic_bytes"]
        except (KeyError, ValueError, OSError):
            continue
        if t is not None and streams == B:
            best = (t, os.path.basename(f))
    return best


def d2d_copy_gbs(torch, dev, nbytes: int = 1 << 30, reps: int = 10) -> float:
    """Measured HBM bandwidth: a device-to-device copy of nbytes, (read + write) bytes per second, HIP events."""
    a = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    b = torch.empty_like(a)
    b.copy_(a)
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(reps):
        b.copy_(a)
    t1.record()
    t1.synchronize()
    ms = t0.elapsed_time(t1) / reps
    del a, b
    return 2 * nbytes / (ms * 1e-3) / 1e9


def host_cores() -> tuple[int, str]:
    """Cores this process may use: its CPU affinity, capped by the cgroup CPU quota when one is set (a GPU box
    shows the whole machine's CPUs in the affinity mask but grants this job a share of them)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        pass
    cores = min(aff, quota) if quota else aff
    return cores, f"sched_getaffinity {aff}" + (f", cgroup cpu.max quota {quota}" if quota else "")


def cpu_baseline(threads: int, target_cpu_s: float = 15.0) -> dict:
    """The oracle (our C restatement of the reference path: FFT + stats + SSB + pulse detectors per frame), one fresh stream per
    frame, timed on the host cores with `threads` worker threads (ctypes releases the GIL)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    O.lib()
    frames = 64
    raw = O.synth_frames(frames, N, O.CS8, tone_hz=1500.0, fs=FS)
    # calibrate single-thread cost per frame
    t0 = time.perf_counter()
    O.run_streams(raw, O.CS8, N, 0, 8, FS, CF, 5)
    per_frame = (time.perf_counter() - t0) / 8
    per_thread = max(8, int(target_cpu_s / threads / per_frame))

    def work():
        done = 0
        while done < per_thread:
            k = min(frames, per_thread - done)
            O.run_streams(raw, O.CS8, N, 0, k, FS, CF, 5)
            done += k

    ts = [threading.Thread(target=work) for _ in range(threads)]
    t0 = time.perf_counter()
    for th in ts:
        th.start()
    for th in ts:
        th.join()
    wall = time.perf_counter() - t0
    total = per_thread * threads
    return {"value": round(total * N / wall / 1e6, 3), "unit": "IQ Msamples/s", "cores": threads, "kind": "port",
            "sample": f"{total} frames x {N} CS8 samples (FFT+stats+SSB+pulse detectors per frame, fresh stream "
                      "each), "
                      f"{threads} threads = every host core granted ({host_cores()[1]}), {wall:.2f} s wall, "
                      f"{per_frame * 1e3:.3f} ms/frame single-thread"}


def rehearsal_verify(torch, dist, world, rank, streams, rec, f_stage, pcm, gather_pcm, gathered, f_out, p_out):
    """--rehearse-gloo: after the timed steps, every rank hashes what it contributed to the last step's gathers
    (records, focus slices, PCM bytes) and rank 0 checks that each rank's block of its gathered buffers hashes
    the same -- the gather delivered every rank's data, in rank order, bit for bit."""
    import hashlib
    torch.cuda.synchronize()

    def digest(t):
        return hashlib.sha256(t.detach().cpu().contiguous().numpy().tobytes()).hexdigest()

    mine = {"records": digest(rec)}
    if f_stage is not None:
        mine["focus"] = digest(f_stage)
    if gather_pcm:
        mine["pcm"] = digest(pcm.view(torch.uint8))
    every = [None] * world
    dist.all_gather_object(every, mine)
    if rank != 0:
        return None
    result = {}
    for key, buf in (("records", gathered), ("focus", f_out), ("pcm", p_out)):
        if buf is None:
            continue
        ok = all(digest(buf[r * streams:(r + 1) * streams]) == every[r][key] for r in range(world))
        result[key] = "ok" if ok else "MISMATCH"
    result["ranks"] = world
    return result


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_command(gpus: int, argv: list[str], port: int) -> list[str]:
    """The one-process-per-GPU launch of this script (the driver's own form of the command)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + argv


def maybe_launch(args, argv: list[str]) -> int | None:
    """--gpus N > 1 without WORLD_SIZE: start the N ranks as a child torch.distributed.run (nothing in this
    process has touched a GPU: counting devices does not initialise one on this image) and return its exit
    status; None when this process is a rank (or N == 1)."""
    if args.gpus < 1:
        log(f"bench: --gpus must be >= 1 (got {args.gpus})")
        return 2
    if args.gpus == 1 or "WORLD_SIZE" in os.environ:
        return None
    if not args.rehearse_gloo:
        import torch
        have = torch.cuda.device_count()
        if have < args.gpus:
            log(f"bench: --gpus {args.gpus} but only {have} GPU(s) visible")
            return 3
    cmd = launch_command(args.gpus, argv, free_port())
    if args.launch_dry_run:
        print(json.dumps({"launch": cmd}), flush=True)
        return 0
    import subprocess
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    return subprocess.run(cmd, env=env).returncode


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    # the chip takes ~50 steps (~20 ms) of this load from idle to a steady clock (tools/lab/warm_trace.py:
    # 25-step blocks at 0.36, 0.345, then 0.34 ms/step), so the default warmup covers that ramp
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--streams", type=int, default=B)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 (default): every core granted (host_cores)")
    ap.add_argument("--no-labelled", action="store_true", help="skip the labelled configs[1]/configs[2] legs")
    ap.add_argument("--pipelined", type=int, default=2, choices=[0, 1, 2],
                    help="2 (default): each step's SSB stages run beside the next step's spectrum, inputs resident "
                         "(SDRG_PIPELINE_INPUTS_READY: the SSB stage does not wait on the main stream); 1: the same with "
                         "the SSB stage forked from the main stream (SDRG_PIPELINE_ON); 0: each step joins its SSB "
                         "stream.  Every stage of every step runs in all three")
    ap.add_argument("--stages", default=None, choices=["all", "hot", "spectrum", "spectrum+stats", "ssb"],
                    help="ablation only: the metric is defined on 'all' (the c3 default)")
    ap.add_argument("--config", default="c3", choices=["c3", "c2", "c5"],
                    help="c3 (default, the metric's workload): BASELINE configs[1]+SSB, every stage; c2: BASELINE "
                         "configs[1] as written (FFT + power + stats only); c5: BASELINE configs[4] (65536-pt CS16, "
                         "1024 streams, FFT + stats, --focus kHz); c2 and c5 print separately labelled lines")
    ap.add_argument("--focus", type=int, default=5, help="c5: freqFocusRangeKhz (SURVEY 8d: 5 and 200)")
    ap.add_argument("--ssb-variant", default="reference", choices=["reference", "nco127"],
                    help="nco127: the BASELINE configs[2] variant (a build extension, not the reference chain): NCO "
                         "mixer at +250 kHz + 127-tap FIR (sdrg_engine_set_ssb_variant); a separately labelled line")
    ap.add_argument("--gather", default="records+focus", choices=["records", "records+pcm", "records+focus",
                                                                  "records+pcm+focus"],
                    help="N > 1: what each step gathers to rank 0 over RCCL (sdrg_engine_gather): the 72-B frame records "
                         "(peak indices and statistics) and, by default, each frame's focus-window spectrum slice "
                         "(BASELINE configs[3] gathers spectra + peak indices), optionally each frame's PCM (SURVEY 8e)")
    ap.add_argument("--rehearse-gloo", action="store_true",
                    help="rehearsal of the N > 1 path on a one-GPU box: every rank on cuda:0, gloo backend, the gathers "
                         "staged through host memory (not a measurement)")
    ap.add_argument("--spectra-gather-steps", type=int, default=10,
                    help="N > 1: after the timed region, time this many gathers of every rank's full spectra (the "
                         "fftCallback payload, 4 B x N bins per frame) to rank 0, reported as spectra_gather_ms (0: skip)")
    ap.add_argument("--prewarm-ms", type=float, default=100.0,
                    help="untimed pre-roll before --warmup: the same step, in blocks of 25, until this much wall time has "
                         "passed, so the timed steps run at the chip's steady clock whatever --warmup is (reported as "
                         "prewarm_ms)")
    ap.add_argument("--stats-async", default="auto", choices=["auto", "0", "1"],
                    help="1: pipelined calls run their statistics on a stream of their own beside the next call's spectrum "
                         "(SDRG_PIPELINE_STATS_ASYNC; every stage of every call still runs); 0: after the spectrum on the "
                         "main stream; auto (default): 1 for the 65536-point configs[4] lines, whose four-step FFT leaves "
                         "room beside it (measured 8 %% / 2 %% faster at 5 / 200 kHz), and for the c3 step with the SSB "
                         "stage, whose statistics then run beside the SSB pipeline and the next spectrum (1.2 %% faster); "
                         "0 for FFT + statistics alone at 16384 points (configs[1]), whose persistent spectrum kernel "
                         "loses more to co-resident statistics than they gain (0.148 vs 0.128 ms/step), and for N > 1 "
                         "(the per-step gathers read the records on the main stream)")
    ap.add_argument("--process-group", action="store_true",
                    help="N = 1: run the N > 1 code path anyway on the one GPU -- a one-rank communicator from the C "
                         "ABI with the per-step gathers behind each step's outputs (device copies at one rank; "
                         "SDRG_BENCH_ONE_RANK_RCCL=1 keeps RCCL's kernel), barriers, max-over-ranks timing, the "
                         "full-spectra gather (a rehearsal line)")
    ap.add_argument("--launch-dry-run", action="store_true", help=argparse.SUPPRESS)
    argv = sys.argv[1:]
    args = ap.parse_args(argv)
    rc = maybe_launch(args, argv)
    if rc is not None:
        return rc
    # this process is a rank: the ONE JSON line goes to the real stdout, everything else (RCCL's version banner,
    # which it prints on stdout at communicator creation, library warnings) to stderr
    json_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)

    import torch
    import torch.distributed as dist
    import sdrg
    from sdrg import shard

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist_on = world > 1 or args.process_group  # a process group (one rank included): the N > 1 code path
    rehearse = args.rehearse_gloo and dist_on
    # the data path of a real N > 1 run: libsdrg.so's own RCCL communicator and gathers (C ABI); torch.distributed
    # (gloo) carries the control plane only.  --rehearse-gloo (every rank on cuda:0, where RCCL refuses two ranks on
    # one device) gathers through sdrg.shard over gloo instead
    capi = dist_on and not rehearse
    if dist_on and world == 1:  # a one-rank group started without torch.distributed.run
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(free_port()))
    if world > 1 and args.gpus not in (1, world):
        log(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}")
        return 3
    if world > 1 and not rehearse and torch.cuda.device_count() < world:
        log(f"bench: WORLD_SIZE={world} but only {torch.cuda.device_count()} GPU(s) visible")
        return 3
    if rehearse:
        local = 0
    if dist_on:
        dist.init_process_group("gloo")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    ranks_info = None
    if dist_on:
        if dist.get_world_size() != world:
            log(f"bench: process group has {dist.get_world_size()} ranks, expected {world}")
            return 3
        props = torch.cuda.get_device_properties(dev)
        mine = {"rank": rank, "local_rank": local, "device": dev.index, "name": props.name,
                "pci_bus_id": getattr(props, "pci_bus_id", None), "uuid": str(getattr(props, "uuid", ""))}
        every = [None] * world
        dist.all_gather_object(every, mine)
        distinct = len({e["uuid"] or (e["pci_bus_id"], e["device"]) for e in every}) == world
        ranks_info = {"ranks_seen": dist.get_world_size(),
                      "backend": "rccl (sdrg_engine_gather, C ABI)" if capi else "gloo (sdrg.shard, host-staged)",
                      "control_backend": dist.get_backend(), "distinct_devices": distinct,
                      "devices": [{k: v for k, v in e.items() if v not in (None, "")} for e in every]}
        if not rehearse and not distinct:
            log(f"bench: warning: ranks may share a GPU: {every}")

    c5 = args.config == "c5"
    n = 65536 if c5 else N
    fmt = sdrg.CS16 if c5 else sdrg.CS8
    fmt_name = "CS16" if c5 else "CS8"
    focus_khz = args.focus if c5 else 5
    streams = (1024 if args.streams == B else args.streams) if c5 else args.streams
    if args.stages is None:
        args.stages = "all" if args.config == "c3" else "spectrum+stats"
    cfg = sdrg.SDRConfig(centerFrequency=CF, samplesPerReading=n, sampleRate=FS, freqFocusRangeKhz=focus_khz,
                         soundMode=1)
    eng = sdrg.Engine(cfg, streams, device=local)
    variant = args.ssb_variant != "reference"
    if variant:
        eng.set_ssb_variant(NCO_HZ, 127)
    # N_INPUTS distinct batches rotated per step, so no step reads inputs the Infinity Cache kept from the last
    iqs = [synth_device_frames(torch, dev, streams, seed=0x5D12 + 7919 * rank + k, n=n, cs16=c5)
           for k in range(N_INPUTS)]
    specs = [torch.empty((streams, n), dtype=torch.float32, device=dev) for _ in range(N_OUTPUTS)]
    recs = [torch.zeros((streams, sdrg.RECORD_DTYPE.itemsize), dtype=torch.uint8, device=dev) for _ in range(N_OUTPUTS)]
    spec, rec = specs[0], recs[0]
    plen = eng.pcm_len
    pcm = torch.empty((streams, plen), dtype=torch.int16, device=dev)
    torch.cuda.synchronize()

    now = [1000]

    stages = {"all": sdrg.STAGE_ALL, "hot": sdrg.STAGE_HOT_PATH, "spectrum": sdrg.STAGE_SPECTRUM, "ssb": sdrg.STAGE_SSB,
              "spectrum+stats": sdrg.STAGE_SPECTRUM | sdrg.STAGE_STATS}[args.stages]

    gdev = torch.device("cpu") if rehearse else dev  # gloo gathers host tensors
    gathered = torch.empty((world * streams, rec.shape[1]), dtype=torch.uint8, device=gdev) if rank == 0 else None
    focus = "focus" in args.gather
    gather_pcm = "pcm" in args.gather
    # PCM travels as bytes: neither RCCL nor gloo has a 16-bit integer type
    p_out = torch.empty((world * streams, 2 * plen), dtype=torch.uint8, device=gdev) if gather_pcm and rank == 0 else None
    f_lo, f_n = sdrg.focus_window(FS, n, focus_khz)
    # host-staged focus slices of the gloo rehearsal (the C ABI packs them on the device itself)
    f_stages = ([torch.empty((streams, f_n), dtype=torch.float32, device=dev) for _ in range(N_OUTPUTS)]
                if focus and rehearse else None)
    f_stage = f_stages[0] if f_stages else None
    f_out = torch.empty((world * streams, f_n), dtype=torch.float32, device=gdev) if focus and rank == 0 else None
    host = (lambda t: t.cpu()) if rehearse else (lambda t: t)
    dcomm = None
    if capi:
        # the communicator: rank 0's ncclGetUniqueId bytes to every rank over the control plane, then
        # ncclCommInitRank inside libsdrg.so on this rank's GPU
        uid = [sdrg.dist_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        dcomm = sdrg.Dist(uid[0], world, rank, device=local)
        if os.environ.get("SDRG_BENCH_ONE_RANK_RCCL") == "1":  # lab: RCCL's one-rank kernel instead of device copies
            dcomm.set_one_rank_rccl(True)
        di = dcomm.info()
        ranks_info["rccl_version"] = di["rccl_version"]
        # one rank: device copies unless set_one_rank_rccl (RCCL's one-rank kernel slows the pipeline: DESIGN 7)
        ranks_info["gather_data_path"] = "rccl" if di["rccl_data"] else "device copies (one rank)"
    elif rehearse:
        # the engine enqueues on a torch stream, so the host-staged gathers' copies follow each step's kernels
        work_stream = torch.cuda.Stream(dev)
        torch.cuda.set_stream(work_stream)
        eng.set_stream(work_stream.cuda_stream)

    calls = [0]
    host_t = [0.0, 0.0, 0]  # lab (SDRG_BENCH_HOST_TIMES=1): host seconds in process_device, in gather; calls

    def ptr(t):
        return t.data_ptr() if t is not None else None

    def step(st=None):
        nonlocal spec, rec, f_stage
        iq = iqs[calls[0] % N_INPUTS]
        spec, rec = specs[calls[0] % N_OUTPUTS], recs[calls[0] % N_OUTPUTS]
        if focus and f_stages is not None:
            f_stage = f_stages[calls[0] % N_OUTPUTS]
        calls[0] += 1
        h0 = time.perf_counter()
        eng.process_device(iq.data_ptr(), fmt, stages if st is None else st, spec.data_ptr(), rec.data_ptr(),
                           pcm.data_ptr(), now[0])
        h1 = time.perf_counter()
        now[0] += n // 2000  # frame duration in ms at 2 Msps (8 ms for 16384)
        if capi:  # one gather group behind this step's outputs, on the stream that produced them (sdrg_engine_gather)
            if not LAB_NO_STEP_GATHER:
                eng.gather(dcomm, 0, records=rec.data_ptr(), records_out=ptr(gathered),
                           focus_spectra=spec.data_ptr() if focus else None, focus_out=ptr(f_out),
                           pcm=pcm.data_ptr() if gather_pcm else None, pcm_out=ptr(p_out))
        elif dist_on:
            shard.gather_records(host(rec), world, rank, dst=0, out=gathered)  # records (peaks, stats) to rank 0
            if gather_pcm:
                shard.gather_records(host(pcm.view(torch.uint8)), world, rank, dst=0, out=p_out)
            if focus:
                if rehearse:
                    f_stage.copy_(spec[:, f_lo:f_lo + f_n])
                    shard.gather_records(f_stage.cpu(), world, rank, dst=0, out=f_out)
                else:
                    shard.gather_focus(spec, f_lo, f_n, world, rank, dst=0, out=f_out, staging=f_stage)
        if LAB_HOST_TIMES:
            host_t[0] += h1 - h0
            host_t[1] += time.perf_counter() - h1
            host_t[2] += 1

    # the inputs are generated before the timed region and synchronised, so they are complete at every call.  The
    # host-staged rehearsal copies the PCM on the main stream, so its per-step PCM gather needs the joined schedule
    # (sdrg_engine_gather orders a pipelined call's PCM itself)
    pipelined = args.pipelined if not (gather_pcm and rehearse) else 0
    # asynchronous statistics need gathers ordered after the statistics' own stream: sdrg_engine_gather does that (it
    # waits for them on the GPU); the host-staged rehearsal gathers on a torch stream and keeps them on the main stream
    async_ok = bool(pipelined and (capi or not dist_on))
    with_ssb = args.stages == "all"
    stats_async = async_ok and (args.stats_async == "1" or (args.stats_async == "auto" and (c5 or with_ssb)))
    pipe_mode = pipelined | (sdrg.PIPELINE_STATS_ASYNC if stats_async else 0)
    c5_mode = pipelined | (sdrg.PIPELINE_STATS_ASYNC if async_ok and args.stats_async != "0" else 0)
    if pipelined:
        eng.set_pipelining(pipe_mode)
    eng.set_profiling(True)
    # pre-roll: from idle the chip needs ~50 steps (~20 ms) of this load to reach its steady clock
    # (tools/lab/warm_trace.py), more than a short --warmup covers; blocks of 25 steps until prewarm_ms has passed
    t_pre = time.perf_counter()
    prewarm_steps = 0
    while (time.perf_counter() - t_pre) * 1e3 < args.prewarm_ms:
        for _ in range(25):
            step()
        prewarm_steps += 25
        eng.synchronize()
    prewarm_ms = (time.perf_counter() - t_pre) * 1e3
    for _ in range(args.warmup):
        step()
    eng.synchronize()
    torch.cuda.synchronize()
    eng.reset_timing_stats()
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    host_t[:] = [0.0, 0.0, 0]
    for _ in range(args.steps):
        step()
    eng.synchronize()  # every step's gathers (on the engine's streams) complete inside the timed region
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if LAB_HOST_TIMES and host_t[2]:
        log(f"bench: host us per step: process_device {host_t[0] / host_t[2] * 1e6:.1f}, gather "
            f"{host_t[1] / host_t[2] * 1e6:.1f} over {host_t[2]} timed calls")
    spectra_gather = None
    if dist_on and args.spectra_gather_steps > 0:
        # the full spectra of every frame (fftCallback payload) to rank 0, timed on its own: outside the metric
        eng.synchronize()
        s_out = torch.empty((world * streams, n), dtype=torch.float32, device=gdev) if rank == 0 else None
        s_src = host(spec)

        def gather_spectra():
            if capi:
                eng.gather(dcomm, 0, spectra=s_src.data_ptr(), spectra_out=ptr(s_out))
            else:
                shard.gather_spectra(s_src, world, rank, dst=0, out=s_out)

        gather_spectra()  # untimed first gather
        eng.synchronize()
        torch.cuda.synchronize()
        dist.barrier()
        tg = time.perf_counter()
        for _ in range(args.spectra_gather_steps):
            gather_spectra()
        eng.synchronize()
        torch.cuda.synchronize()
        dist.barrier()
        tgt = torch.tensor([time.perf_counter() - tg], dtype=torch.float64)
        dist.all_reduce(tgt, op=dist.ReduceOp.MAX)
        g_ms = float(tgt.item()) / args.spectra_gather_steps * 1e3
        into0 = (world - 1) * streams * n * 4
        spectra_gather = {"spectra_gather_ms": round(g_ms, 4), "bytes_per_rank": streams * n * 4,
                          "bytes_into_rank0": into0, "GBs_into_rank0": round(into0 / (g_ms * 1e-3) / 1e9, 1),
                          "steps": args.spectra_gather_steps,
                          "note": "every rank's full [streams, N] float32 spectra gathered to rank 0 (the fftCallback "
                                  "payload, SURVEY 8e), after the timed region; not part of value"}
        del s_out
    # every rank hashes what it contributed to the last step's gathers; rank 0 checks its gathered blocks (any backend)
    if dist_on:
        eng.synchronize()
        f_mine = (f_stage if rehearse else spec[:, f_lo:f_lo + f_n].contiguous()) if focus else None
        rehearsal_check = rehearsal_verify(torch, dist, world, rank, streams, rec, f_mine, pcm, gather_pcm, gathered,
                                           f_out, p_out)
    else:
        rehearsal_check = None
    ts = eng.timing_stats()
    # the spectrum kernel alone (no SSB sharing the chip), a few launches after the timed region: its
    # isolated HBM rate, reported beside the timed-region one
    eng.set_pipelining(False)
    for k in range(5 + ISO_LAUNCHES):  # 5 untimed launches, then ISO_LAUNCHES timed ones
        if k == 5:
            eng.synchronize()
            eng.reset_timing_stats()
        eng.process_device(iqs[k % N_INPUTS].data_ptr(), fmt, sdrg.STAGE_SPECTRUM, spec.data_ptr(), None, None, now[0])
    eng.synchronize()
    spec_iso_ms = eng.timing_stats()["spectrum_ms"]
    ssb_iso_ms = None
    if args.stages == "all":  # the SSB stage alone (nothing else on the chip), for its latency-floor fraction
        for k in range(5 + SSB_ISO_CALLS):  # 5 untimed calls, then SSB_ISO_CALLS timed ones
            if k == 5:
                eng.synchronize()
                eng.reset_timing_stats()
            eng.process_device(iqs[k % N_INPUTS].data_ptr(), fmt, sdrg.STAGE_SSB, None, None, pcm.data_ptr(), now[0])
        eng.synchronize()
        ssb_iso_ms = eng.timing_stats()["ssb_ms"]
    d2d = d2d_copy_gbs(torch, dev)
    stream_gbs = sdrg.measure_hbm_copy(local, 1 << 30, 10)  # the library's float4 streaming copy (roofline basis)

    def labelled_rate(st, k_steps, variant_on=False, mode=None):
        """A separately labelled line measured in this same run: k_steps pipelined steps of stages st with profiling
        off (value, ms_per_step), then a separate profiled pass of up to PROFILED_STEPS steps for the per-kernel times
        (HIP events on each kernel's stream, as kernel_ms; an event marker costs a stream a few us, so it never sits in
        the timed pass), so a change of the line between two records can be attributed to a kernel."""
        if variant_on:
            eng.set_ssb_variant(NCO_HZ, 127)
        eng.set_pipelining(pipe_mode if mode is None else mode)
        eng.set_profiling(False)
        for _ in range(10):  # untimed, after the variant / schedule switch
            step(st)
        eng.synchronize()
        t1 = time.perf_counter()
        for _ in range(k_steps):
            step(st)
        eng.synchronize()
        dt = time.perf_counter() - t1
        eng.set_profiling(True)
        eng.reset_timing_stats()
        for _ in range(min(k_steps, PROFILED_STEPS)):
            step(st)
        eng.synchronize()
        tm = eng.timing_stats()
        eng.set_profiling(False)
        if variant_on:
            eng.set_ssb_variant(0.0, 0)
        r = {"value": round(k_steps * streams * n / dt / 1e6, 2), "ms_per_step": round(dt / k_steps * 1e3, 4), "steps": k_steps,
             "spectrum_ms": round(tm["spectrum_ms"], 4), "stats_ms": round(tm["stats_ms"], 4)}
        if st & sdrg.STAGE_SSB:
            r["ssb_ms"] = round(tm["ssb_ms"], 4)
        return r

    def c5_line(focus_c5: int, k_steps: int) -> dict:
        """BASELINE configs[4] in this same run: 1024 streams x 65536-pt CS16 frames, FFT + |X|^2 + fftshift + stats
        over a focus_c5 kHz focus, its own engine and rotated inputs."""
        n5, s5 = 65536, 1024
        e5 = sdrg.Engine(sdrg.SDRConfig(centerFrequency=CF, samplesPerReading=n5, sampleRate=FS,
                                        freqFocusRangeKhz=focus_c5, soundMode=1), s5, device=local)
        iq5 = [synth_device_frames(torch, dev, s5, seed=0xC5 + k, n=n5, cs16=True) for k in range(N_INPUTS)]
        sp5 = [torch.empty((s5, n5), dtype=torch.float32, device=dev) for _ in range(N_OUTPUTS)]
        rc5 = [torch.zeros((s5, sdrg.RECORD_DTYPE.itemsize), dtype=torch.uint8, device=dev) for _ in range(N_OUTPUTS)]
        st5 = sdrg.STAGE_SPECTRUM | sdrg.STAGE_STATS
        torch.cuda.synchronize()
        if pipelined:  # each call's statistics beside the next call's spectrum (--stats-async)
            e5.set_pipelining(c5_mode)
        t5 = [1000]

        def run(k):
            for i in range(k):
                e5.process_device(iq5[i % N_INPUTS].data_ptr(), sdrg.CS16, st5, sp5[i % N_OUTPUTS].data_ptr(),
                                  rc5[i % N_OUTPUTS].data_ptr(), None, t5[0])
                t5[0] += n5 // 2000
        run(20)
        e5.synchronize()
        t1 = time.perf_counter()
        run(k_steps)  # profiling off: the value and ms_per_step
        e5.synchronize()
        dt = time.perf_counter() - t1
        e5.set_profiling(True)  # a separate profiled pass for the per-kernel times
        e5.reset_timing_stats()
        run(min(k_steps, PROFILED_STEPS))
        e5.synchronize()
        tm = e5.timing_stats()
        e5.close()
        ms = dt / k_steps * 1e3
        fft_bytes = 8.0 * s5 * n5  # CS16: 4 B in + 4 B float32 power out per sample
        step_b = fft_bytes + s5 * sdrg.RECORD_DTYPE.itemsize
        del iq5, sp5, rc5
        return {"value": round(k_steps * s5 * n5 / dt / 1e6, 2), "ms_per_step": round(ms, 4), "steps": k_steps,
                "spectrum_ms": round(tm["spectrum_ms"], 4), "stats_ms": round(tm["stats_ms"], 4),
                "roofline_fft": {"kernel": "four_step_a + four_step_b", "achieved": round(fft_bytes / tm["spectrum_ms"]
                                                                                          / 1e6, 1),
                                 "frac": round(fft_bytes / tm["spectrum_ms"] / 1e6 / HBM_PEAK_GBS, 4)},
                "roofline_step_frac": round(step_b / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                "stats_async": bool(c5_mode & sdrg.PIPELINE_STATS_ASYNC),
                "workload": f"BASELINE configs[4]: {s5} streams x {n5}-pt CS16 frames @2 Msps, four-step FFT + |X|^2 "
                            f"+ fftshift + signal-strength stats over a {focus_c5} kHz focus; no SSB"}

    labelled = {}
    k_lab = max(args.steps, LABELLED_MIN_STEPS)
    if not dist_on and args.config == "c3" and args.stages == "all" and not variant and not args.no_labelled:
        eng.set_profiling(False)
        # FFT + statistics alone: the statistics after the spectrum on one stream (--stats-async auto) unless forced
        c1_mode = pipelined | (sdrg.PIPELINE_STATS_ASYNC if async_ok and args.stats_async == "1" else 0)
        labelled["configs1_fft_stats"] = dict(labelled_rate(sdrg.STAGE_SPECTRUM | sdrg.STAGE_STATS, k_lab,
                                                            mode=c1_mode),
                                              stats_async=bool(c1_mode & sdrg.PIPELINE_STATS_ASYNC),
                                              workload="BASELINE configs[1]: same batch, FFT + |X|^2 + fftshift + "
                                                       "log-mag/peak/signal-strength stats, no SSB")
        if async_ok:  # the other statistics schedule of the same line, measured right after it (an A/B in the record)
            alt = pipelined | (0 if c1_mode & sdrg.PIPELINE_STATS_ASYNC else sdrg.PIPELINE_STATS_ASYNC)
            labelled["configs1_fft_stats_other_schedule"] = dict(
                labelled_rate(sdrg.STAGE_SPECTRUM | sdrg.STAGE_STATS, k_lab, mode=alt),
                stats_async=bool(alt & sdrg.PIPELINE_STATS_ASYNC),
                note="configs1_fft_stats with the statistics schedule flipped (--stats-async), not the line's choice")
        labelled["configs2_nco127"] = dict(labelled_rate(sdrg.STAGE_ALL, k_lab, variant_on=True),
                                           workload="BASELINE configs[2] as written (a build extension, not the "
                                                    f"reference chain): SSB with an NCO mixer at +{NCO_HZ / 1e3:g} kHz "
                                                    "+ 127-tap FIR decim 41, every other stage as the headline")
        labelled["configs4_c5_5khz"] = c5_line(5, k_lab)
        labelled["configs4_c5_200khz"] = c5_line(200, k_lab)
    if dist_on:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    samples = args.steps * streams * n * world
    value = samples / elapsed / 1e6
    ms_per_step = elapsed / args.steps * 1e3
    spec_ms = ts["spectrum_ms"]
    alg_bytes = (8.0 if c5 else ALG_BYTES_PER_SAMPLE["spectrum"]) * streams * n  # CS16: 4 B in + 4 B out
    achieved = alg_bytes / (spec_ms * 1e-3) / 1e9 if spec_ms > 0 else 0.0
    kname = "four_step_a + four_step_b" if c5 else "spectrum16k_kernel"
    traffic = pmc_traffic("spectrum16k_kernel", streams) if args.config == "c3" else None
    workload = {
        "c3": (f"C3: {streams} streams x {n}-pt CS8 frames @2 Msps per GPU; FFT + |X|^2 + fftshift "
               "+ signal-strength stats + SSB (DC, LPF, AGC, 255-tap FIR decim 41, EQ, PCM) + spectral "
               "and audio pulse detectors"),
        "c2": (f"C2 (BASELINE configs[1]): {streams} streams x {n}-pt CS8 frames @2 Msps per GPU; FFT + |X|^2 + "
               "fftshift + signal-strength stats (peak, log-magnitude statistics); no SSB"),
        "c5": (f"C5 (BASELINE configs[4]): {streams} streams x {n}-pt CS16 frames @2 Msps per GPU; four-step FFT + "
               f"|X|^2 + fftshift + signal-strength stats over a {focus_khz} kHz focus; no SSB"),
    }[args.config]
    achieved_iso = alg_bytes / (spec_iso_ms * 1e-3) / 1e9 if spec_iso_ms > 0 else 0.0
    # whole-step algorithmic bytes: IQ in + spectra out + 72-B records + PCM out (~6.05 B/sample CS8)
    in_bps = 4.0 if c5 else 2.0
    step_bytes = streams * n * (in_bps + 4.0) + streams * (sdrg.RECORD_DTYPE.itemsize + 2 * plen * (args.stages == "all"))
    step_gbs = step_bytes / (ms_per_step * 1e-3) / 1e9
    out = {
        "metric": "IQ Msamples/s (16384-pt FFT+SSB) at 1/2/4/8 GPUs; % HBM roofline",
        "value": round(value, 2),
        "unit": "IQ Msamples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32 (int16 CS16 in)" if c5 else "f32 (int8 CS8 in, int16 PCM out)",
        "data": f"synthetic {fmt_name} CW tones + Gaussian noise, generated on device",
        "config": {"workload": workload if not variant else
                               (f"C3-variant (BASELINE configs[2], build extension, not the reference chain): {streams} "
                                f"streams x {n}-pt CS8 frames @2 Msps per GPU; FFT + stats + SSB with NCO mixer "
                                f"(+{NCO_HZ / 1e3:g} kHz) + 127-tap FIR decim 41 (397 PCM/frame) + pulse detectors"),
                   "streams_per_gpu": streams, "samples_per_frame": n, "sample_rate": FS, "format": fmt_name,
                   "focus_khz": focus_khz,
                   "parallelism": f"streams sharded {streams}/GPU x {world} GPU(s)" + (
                       ((", RCCL gather (sdrg_engine_gather) of records" if capi else ", gloo gather of records")
                        + (" + PCM" if gather_pcm else "") + (f" + {f_n}-bin focus spectra" if focus else ""))
                       if dist_on else "")},
        "kernel_ms": {k: round(v, 4) for k, v in ts.items() if k != "count"},
        "roofline": {"kernel": f"{kname} (unpack+FFT+|X|^2+fftshift)", "bound": "hbm",
                     "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic[0] if traffic else None,
                     "traffic_source": traffic[1] if traffic else None,
                     "alg_bytes_per_launch": alg_bytes,
                     "measured": ("HIP events on the kernel's stream over the timed region"
                                  + (", where each step's SSB pipeline shares the chip with the next step's spectrum"
                                     if pipelined else ""))},
        "roofline_isolated": {"kernel": kname, "bound": "hbm", "achieved": round(achieved_iso, 1),
                              "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved_iso / HBM_PEAK_GBS, 4),
                              "measured": f"{ISO_LAUNCHES} launches of the spectrum stage alone after the timed region"},
        "hbm_measured": {"stream_copy_GBs": round(stream_gbs, 1),
                         "d2d_copy_GBs": round(d2d, 1),
                         "note": "stream_copy: the library's float4 streaming copy of 1 GiB (sdrg_measure_hbm_copy: "
                                 "nontemporal loads/stores, 16 workgroups per CU), read + write bytes per second, the "
                                 "achievable rate the fractions below are priced against (MI355X_MICROARCH.md: 6.29 TB/s); "
                                 "d2d_copy: a hipMemcpy D2D of 1 GiB, for comparison (the copy path is slower)",
                         "frac_timed": round(achieved / stream_gbs, 4) if stream_gbs else None,
                         "frac_isolated": round(achieved_iso / stream_gbs, 4) if stream_gbs else None},
        "roofline_step": {"bound": "hbm", "achieved": round(step_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                          "frac": round(step_gbs / HBM_PEAK_GBS, 4),
                          "bytes_per_sample": round(step_bytes / (streams * n), 4),
                          "measured": "whole-step algorithmic bytes (IQ in, spectra, records, PCM out) / ms_per_step"},
        "pipelined": {0: "off (each step joins its SSB stream)",
                      1: "on (SSB stage forked from the main stream each step)",
                      2: "on, inputs ready (resident inputs: the SSB stage does not wait on the main stream)"}[pipelined]
                     + ("; statistics on a stream of their own beside the next step's spectrum (SDRG_PIPELINE_STATS_ASYNC),"
                        f" {N_OUTPUTS} spectra/records buffers rotated" if stats_async else ""),
        "inputs": f"{N_INPUTS} distinct {streams}x{n} {fmt_name} batches ({N_INPUTS * streams * n * in_bps / 2**20:.0f} "
                  "MiB) rotated per step in every leg, so inputs are not served from the 256 MiB Infinity Cache",
    }
    if args.stages == "all":
        # the step cannot beat its slowest bound: the SSB chain's serial floor (one frame's recurrences) or the HBM
        # time of its algorithmic bytes; as a fraction of HBM peak that ceiling is what ">= 60 % of HBM" can reach
        floor_ms = n * SSB_CHAIN_CYCLES / (MAX_CLOCK_GHZ * 1e9) * 1e3
        hbm_ms = step_bytes / (HBM_PEAK_GBS * 1e9) * 1e3
        ceil_ms = max(floor_ms, hbm_ms)
        out["roofline_step"]["ceiling"] = {
            "step_ceiling_frac": round(hbm_ms / ceil_ms, 4), "ceiling_ms": round(ceil_ms, 4),
            "bound_by": "ssb serial floor" if floor_ms >= hbm_ms else "hbm",
            "hbm_ms_at_peak": round(hbm_ms, 4), "ssb_floor_ms": round(floor_ms, 4),
            "frac_of_ceiling": round(ceil_ms / ms_per_step, 4),
            "note": "step algorithmic bytes / max(SSB serial floor, HBM time at peak) / peak: the highest "
                    "roofline_step.frac any bit-exact schedule of this step can reach"}
    out["prewarm_ms"] = round(prewarm_ms, 1)
    out["prewarm_steps"] = prewarm_steps
    if ranks_info:
        out.update(ranks_info)
    if dist_on:
        out["gather_mode"] = ("sdrg_engine_gather: one gather group per step behind the step's outputs on the stream "
                              "that produced them (the statistics stream when asynchronous), no host synchronisation; "
                              "RCCL ncclGather at N > 1, device copies on one rank" if capi else
                              "host-staged gloo gathers (rehearsal)")
    if spectra_gather:
        out["spectra_gather"] = spectra_gather
    if ssb_iso_ms:
        floor_ms = n * SSB_CHAIN_CYCLES / (MAX_CLOCK_GHZ * 1e9) * 1e3
        out["ssb_latency_floor"] = {
            "kernel": "ssb_pipe_kernel (the reference's sample-serial SSB chain, bit-exact)",
            "bound": "serial issue", "floor_ms": round(floor_ms, 4),
            "basis": f"{n} samples x {SSB_CHAIN_CYCLES} cycles (the low-pass wave's 6 VALU + 0.5 LDS instructions "
                     f"per sample at one instruction per 4 cycles, tools/lab/lat.hip) / {MAX_CLOCK_GHZ} GHz max clock",
            "ssb_ms_alone": round(ssb_iso_ms, 4), "frac_alone": round(floor_ms / ssb_iso_ms, 4),
            "ssb_ms_coresident": round(ts["ssb_ms"], 4),
            "frac_coresident": round(floor_ms / ts["ssb_ms"], 4) if ts["ssb_ms"] > 0 else None,
            "coresident_basis": ("every timed step: the SSB stream's time per step in the pipelined timed region, from "
                                 "one step's SSB end marker to the next (the SSB pipeline kernels and their launch "
                                 "gaps; the audio pulse detector runs on a stream of its own; the first step from its "
                                 "own start marker)"
                                 if pipelined else "every timed step: the SSB stream's start to end marker")}
        # the same kernel against HBM: the step's longest kernel by GPU time, and latency-bound (the floor above)
        ssb_bytes = streams * n * in_bps + streams * 2 * plen
        ssb_traffic = pmc_traffic("ssb_pipe_kernel", streams)
        if ts["ssb_ms"] > 0:
            ssb_gbs = ssb_bytes / (ts["ssb_ms"] * 1e-3) / 1e9
            out["roofline_ssb"] = {
                "kernel": "ssb_pipe_kernel", "bound": "hbm", "achieved": round(ssb_gbs, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(ssb_gbs / HBM_PEAK_GBS, 4), "alg_bytes_per_launch": ssb_bytes,
                "traffic": ssb_traffic[0] if ssb_traffic else None,
                "traffic_source": ssb_traffic[1] if ssb_traffic else None,
                "note": "the longest kernel by GPU time, measured co-resident in the timed region; it is bound by the "
                        "sample-serial recurrences (ssb_latency_floor), not by HBM: IQ in (I used) + PCM out"}
    if args.stages == "all" and ts["ssb_ms"] > 0:
        # the kernel with the most GPU time per step, against HBM: pipelined, the SSB stream (the pipeline kernel; the
        # audio detector runs on a stream of its own, s_ap) and the main stream (spectrum, statistics, spectral
        # detector) each fill the step
        cand = {"ssb_pipe_kernel": (ts["ssb_ms"], streams * n * in_bps + streams * 2 * plen),
                "spectrum16k_kernel" if not c5 else "four_step_a + four_step_b": (spec_ms, alg_bytes),
                "stats_kernel": (ts["stats_ms"], None)}
        dom = max((k for k in cand if cand[k][1] is not None), key=lambda k: cand[k][0])
        d_ms, d_bytes = cand[dom]
        d_gbs = d_bytes / (d_ms * 1e-3) / 1e9
        d_traffic = pmc_traffic(dom, streams)
        out["roofline_dominant"] = {
            "kernel": dom, "ms_per_step": round(d_ms, 4), "bound": "hbm", "achieved": round(d_gbs, 1),
            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(d_gbs / HBM_PEAK_GBS, 4), "alg_bytes_per_launch": d_bytes,
            "traffic": d_traffic[0] if d_traffic else None, "traffic_source": d_traffic[1] if d_traffic else None,
            "kernel_ms_per_step": {k: round(v[0], 4) for k, v in cand.items()},
            "note": "the kernel with the most GPU time per step (its stream time in the timed region); ssb_pipe_kernel "
                    "is bound by the sample-serial recurrences (ssb_latency_floor), not by HBM"}
    if labelled:
        out["labelled"] = labelled
    if rehearse:
        out["rehearsal"] = "gloo, every rank on cuda:0: a functional check of the N > 1 path, not a measurement"
    if dist_on:
        out["rehearsal_check" if rehearse else "gather_check"] = rehearsal_check
    if variant:
        out["ssb_variant"] = {"nco_hz": NCO_HZ, "fir_taps": 127, "note": "not the reference's chain; no CPU baseline"}
    if args.config != "c3":
        out["labelled_config"] = args.config
    elif args.stages != "all":
        out["ablation_stages"] = args.stages
    if (rank == 0 and not dist_on and not args.no_cpu_baseline and args.stages == "all" and not variant
            and args.config == "c3"):
        try:
            out["cpu_baseline"] = cpu_baseline(args.cpu_threads or host_cores()[0])
        except Exception as exc:  # the baseline is informative; never fail the bench line on it
            out["cpu_baseline"] = {"error": repr(exc)}
    if rank == 0:
        print(json.dumps(out), file=json_out, flush=True)
    eng.close()
    if dcomm is not None:
        dcomm.close()
    if dist_on:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())

"""GPU tests of the engine's host contract (include/sdrg.h): input release in pipelined mode, profiling reads
across pipelined calls, rejected calls leaving no state behind, the BridgeConfig-only setters
(setSampleRate / setSamplesPerReading, sdr-bridge-java-soapy.cpp:931-1023) and engines driven from several
threads at once."""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N, FS = 16384, 2_000_000


@pytest.fixture(scope="module")
def S():
    import sdrg
    return sdrg


@pytest.fixture(scope="module")
def O():
    import oracle
    return oracle


def engine(S, n, fs, streams, cf=100_000_000, focus=5, mode=1):
    cfg = S.SDRConfig(centerFrequency=cf, samplesPerReading=n, sampleRate=fs, freqFocusRangeKhz=focus, soundMode=mode)
    return S.Engine(cfg, streams)


def frames(O, B, F, n=N, fs=FS):
    return np.stack([np.stack([O.synth_frames(1, n, O.CS8, tone_hz=250.0 * (b % 17) - 2000.0, fs=fs,
                                              seed=1000 * f + b)[0] for b in range(B)]) for f in range(F)])


def run_device(S, torch, raws, B, pipelined, refill_one_buffer=False, wait_release=True):
    """F calls on device buffers; returns (spectra, records, pcm) stacked over calls, after synchronize.
    refill_one_buffer: every call reads ONE iq buffer that is refilled on the engine's stream before each call
    (the live-receiver pattern), after sdrg_engine_wait_input_released when wait_release."""
    dev = torch.device("cuda:0")
    F = raws.shape[0]
    eng = engine(S, N, FS, B)
    eng.set_pipelining(pipelined)
    work = torch.cuda.Stream(dev)
    eng.set_stream(work.cuda_stream)
    src = [torch.from_numpy(raws[f]).to(dev) for f in range(F)]
    one = torch.empty_like(src[0])
    spec = [torch.empty((B, N), dtype=torch.float32, device=dev) for _ in range(F)]
    rec = [torch.zeros((B, S.RECORD_DTYPE.itemsize), dtype=torch.uint8, device=dev) for _ in range(F)]
    pcm = [torch.empty((B, eng.pcm_len), dtype=torch.int16, device=dev) for _ in range(F)]
    torch.cuda.synchronize()
    for f in range(F):
        if refill_one_buffer:
            if wait_release:
                eng.wait_input_released(work.cuda_stream)
            with torch.cuda.stream(work):
                one.copy_(src[f])
            iq = one
        else:
            iq = src[f]
        eng.process_device(iq.data_ptr(), S.CS8, S.STAGE_ALL, spec[f].data_ptr(), rec[f].data_ptr(),
                           pcm[f].data_ptr(), 1000 + 8 * f)
    eng.synchronize()
    assert eng.input_released()
    out = (torch.stack(spec).cpu(), torch.stack(rec).cpu(), torch.stack(pcm).cpu())
    eng.set_stream(None)
    eng.close()
    return out


def test_pipelined_refill_after_input_release_equals_joined(S, O):
    """One iq buffer refilled on the engine's stream before every pipelined call, after wait_input_released:
    bit-identical to the joined schedule with a fresh buffer per call (the SSB pipeline of call k still reads
    the buffer while call k+1's spectrum runs, so without the wait the refill would overwrite its input)."""
    import torch
    B, F = 256, 4
    raws = frames(O, B, F)
    want = run_device(S, torch, raws, B, pipelined=False)
    got = run_device(S, torch, raws, B, pipelined=True, refill_one_buffer=True)
    for a, b in zip(want, got):
        assert torch.equal(a, b)


def test_input_released_query(S, O):
    import torch
    B = 64
    dev = torch.device("cuda:0")
    eng = engine(S, N, FS, B)
    assert eng.input_released()  # nothing enqueued yet
    iq = torch.from_numpy(frames(O, B, 1)[0]).to(dev)
    pcm = torch.empty((B, eng.pcm_len), dtype=torch.int16, device=dev)
    eng.set_pipelining(True)
    torch.cuda.synchronize()
    eng.process_device(iq.data_ptr(), S.CS8, S.STAGE_SSB, None, None, pcm.data_ptr(), 1000)
    eng.synchronize()
    assert eng.input_released()
    eng.close()


def test_timings_right_after_pipelined_call_and_ring_wrap(S, O):
    """get_timings straight after a pipelined call must wait for the unjoined SSB stream, and more
    than 64 profiled pipelined calls (the event ring) must fold without hipErrorNotReady."""
    import torch
    B = 128
    dev = torch.device("cuda:0")
    eng = engine(S, N, FS, B)
    eng.set_pipelining(True)
    eng.set_profiling(True)
    iq = torch.from_numpy(frames(O, B, 1)[0]).to(dev)
    spec = torch.empty((B, N), dtype=torch.float32, device=dev)
    rec = torch.zeros((B, S.RECORD_DTYPE.itemsize), dtype=torch.uint8, device=dev)
    pcm = torch.empty((B, eng.pcm_len), dtype=torch.int16, device=dev)
    torch.cuda.synchronize()
    eng.process_device(iq.data_ptr(), S.CS8, S.STAGE_ALL, spec.data_ptr(), rec.data_ptr(), pcm.data_ptr(), 1000)
    t = eng.timings()  # no synchronize before it
    assert t["ssb_ms"] > 0 and t["spectrum_ms"] > 0
    for k in range(70):
        eng.process_device(iq.data_ptr(), S.CS8, S.STAGE_ALL, spec.data_ptr(), rec.data_ptr(), pcm.data_ptr(),
                           1008 + 8 * k)
    st = eng.timing_stats()
    assert st["count"] == 71 and st["ssb_ms"] > 0
    eng.close()


def test_ssb_ms_after_profiling_pause(S, O):
    """a pipelined call's ssb_ms is measured from the previous call's SSB end marker only when that call
    was profiled and came right before it.  Turning profiling off for some calls (and idling) and on again without
    resetting the statistics must not hand the first profiled call an interval spanning the pause."""
    import time

    import torch
    B = 256
    dev = torch.device("cuda:0")
    eng = engine(S, N, FS, B)
    eng.set_pipelining(S.PIPELINE_INPUTS_READY)
    iq = torch.from_numpy(frames(O, B, 1)[0]).to(dev)
    spec = torch.empty((B, N), dtype=torch.float32, device=dev)
    rec = torch.zeros((B, S.RECORD_DTYPE.itemsize), dtype=torch.uint8, device=dev)
    pcm = torch.empty((B, eng.pcm_len), dtype=torch.int16, device=dev)
    torch.cuda.synchronize()
    now = [1000]

    def call():
        eng.process_device(iq.data_ptr(), S.CS8, S.STAGE_ALL, spec.data_ptr(), rec.data_ptr(), pcm.data_ptr(), now[0])
        now[0] += 8

    eng.set_profiling(True)
    for _ in range(12):
        call()
    per_call = eng.timing_stats()["ssb_ms"]
    assert per_call > 0
    eng.set_profiling(False)
    for _ in range(10):
        call()
    eng.synchronize()
    time.sleep(0.05)  # 50 ms idle: far above a call's SSB time
    eng.set_profiling(True)
    call()
    t = eng.timings()
    assert 0 < t["ssb_ms"] < 3 * per_call + 0.5, (t, per_call)
    for _ in range(3):  # the calls after it chain from its end marker again
        call()
    t = eng.timings()
    assert 0 < t["ssb_ms"] < 3 * per_call + 0.5, (t, per_call)
    st = eng.timing_stats()  # the window's mean holds no pause either
    assert st["ssb_ms"] < 3 * per_call + 0.5, (st, per_call)
    eng.close()


def test_rejected_call_freezes_nothing(S, O):
    """a call rejected after the SSB statics would have been set (null pcm) must not freeze the SSB
    frame size: the first SUCCESSFUL call freezes it (processSSB_opt's static sampCount, :224-227)."""
    import torch
    n0, n1 = 8192, 4096
    eng = engine(S, n0, FS, 1)
    dev = torch.device("cuda:0")
    iq0 = torch.from_numpy(O.synth_frames(1, n0, O.CS8, seed=3)[0]).to(dev)
    torch.cuda.synchronize()
    with pytest.raises(S.SdrgError):
        eng.process_device(iq0.data_ptr(), S.CS8, S.STAGE_SSB, None, None, None, 1000)  # null pcm: rejected
    eng.setSamplesPerReading(n1)
    raw = O.synth_frames(3, n1, O.CS8, tone_hz=900.0, seed=4)
    st = O.SsbState()
    for f in range(3):
        _, _, pcm = eng.process(raw[f][None], fmt=S.CS8, stages=S.STAGE_SSB)
        np.testing.assert_array_equal(pcm[0], st.process(O.unpack(O.CS8, raw[f], n1), FS, 1))
    eng.close()


def test_pipelining_modes(S, O):
    """sdrg_engine_set_pipelining takes SDRG_PIPELINE_OFF / _ON / _INPUTS_READY; anything else is SDRG_E_INVALID
    and leaves the mode unchanged (the next pipelined calls still equal the joined schedule: test_gpu_parity)."""
    eng = engine(S, N, FS, 2)
    for mode in (S.PIPELINE_OFF, S.PIPELINE_ON, S.PIPELINE_INPUTS_READY, S.PIPELINE_OFF):
        eng.set_pipelining(mode)
    for bad in (-1, 3, 7):
        with pytest.raises(S.SdrgError):
            eng.set_pipelining(bad)
    eng.close()


def test_set_sample_rate_is_bridge_config_only(S, O):
    """setSampleRate (:931-953) changes BridgeConfig only: the SSB chain sees the new rate from the next frame
    (handed the bridge's rate per frame, :441-442), the statistics keep FFTProcessor::config_'s rate until the next
    configure() (here setFrequencyFocusRange), and the spectral pulse detector keeps the fsEnergy applyConfig gave
    it (the bridge setters used to reconfigure it)."""
    n, fs0, fs1, B, F = 4096, 2_000_000, 2_400_000, 4, 6
    eng = engine(S, n, fs0, B)
    raw = np.stack([O.synth_frames(F, n, O.CS8, tone_hz=600.0 * (b + 1), fs=fs0, seed=50 + b) for b in range(B)])
    fst = [O.FftState(100_000_000, fs0, n, 5) for _ in range(B)]
    sst = [O.SsbState() for _ in range(B)]
    fs_energy0 = float(np.float32(fs0) / np.float32(n))
    spd = [O.PulseDetector(O.PULSE_SPECTRAL, fs_energy=fs_energy0) for _ in range(B)]
    for f in range(F):
        fs_ssb = fs0 if f < 2 else fs1
        if f == 2:
            eng.setSampleRate(fs1)
        if f == 4:  # a configure() point: the statistics now use the new rate too
            eng.setFrequencyFocusRange(5)
            for st in fst:
                st.configure(100_000_000, fs1, n, 5)
        spec, rec, pcm = eng.process(raw[:, f], fmt=S.CS8, stages=S.STAGE_ALL, now_ms=1000 + 10 * f)
        sp, _ = eng.pulse_outputs(audio=False)
        for b in range(B):
            iq = O.unpack(O.CS8, raw[b, f], n)
            np.testing.assert_array_equal(pcm[b], sst[b].process(iq, fs_ssb, 1), err_msg=f"pcm {b} {f}")
            want = fst[b].signal_strength(spec[b], 1000 + 10 * f)
            assert rec[b]["peak_bin"] == want["peak_bin"]
            assert np.float32(rec[b]["best1khz_center_freq_hz"]) == pytest.approx(
                float(want["best1khz_center_freq_hz"]), rel=1e-6), (b, f)
            ws = spd[b].spectral(rec["best1khz_snr_sigma"][b:b + 1], rec["best1khz_center_freq_hz"][b:b + 1])[0]
            for k in ("live_etat", "level", "locked", "n_energy"):
                assert sp[b][k] == ws[k], (k, b, f)
    eng.close()


def test_engines_in_concurrent_threads(S, O):
    """Two engines created and run from two threads at once (the dynamic-LDS attribute is set per device under a
    lock): each reproduces a single-threaded engine's outputs bit for bit."""
    n, B = 16384, 16
    raw = frames(O, B, 2)
    want = []
    eng = engine(S, n, FS, B)
    for f in range(2):
        want.append(eng.process(raw[f], fmt=S.CS8, now_ms=1000 + f))
    eng.close()
    results = [None, None]
    errors = []

    def worker(k):
        try:
            e = engine(S, n, FS, B)
            results[k] = [e.process(raw[f], fmt=S.CS8, now_ms=1000 + f) for f in range(2)]
            e.close()
        except Exception as exc:  # surfaced below
            errors.append(exc)

    ts = [threading.Thread(target=worker, args=(k,)) for k in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert not errors, errors
    for k in range(2):
        for f in range(2):
            for a, b in zip(results[k][f], want[f]):
                assert a.tobytes() == b.tobytes()  # records included: their tail padding is written as zeros


def test_dynamic_lds_limit_survives_large_small_large(S, O):
    """The max-dynamic-LDS attribute is one limit per (kernel, device): the engine only ever raises it
    (csrc/engine.cpp ensure_dynamic_lds), so a large, small, large sequence of frame sizes on ONE engine (the any-N
    FFT kernels size their LDS from N; 12288 points need more than the 64 KiB default) keeps every launch valid and
    every call's spectrum and records equal to a fresh engine's."""
    fs = 2_000_000
    eng = engine(S, 12288, fs, 2)
    for k, n in enumerate((12288, 1536, 12288, 6144, 12288)):
        cfg = S.SDRConfig(centerFrequency=100_000_000, samplesPerReading=n, sampleRate=fs, freqFocusRangeKhz=5,
                          soundMode=1)
        assert eng.applyConfig(cfg)
        raw = np.stack([O.synth_frames(1, n, O.CS8, tone_hz=900.0 + 300 * b, fs=fs, seed=10 * k + b)[0]
                        for b in range(2)])
        spec, rec, _ = eng.process(raw, fmt=S.CS8, stages=S.STAGE_SPECTRUM | S.STAGE_STATS, now_ms=1000 + k)
        fresh = engine(S, n, fs, 2)
        spec1, rec1, _ = fresh.process(raw, fmt=S.CS8, stages=S.STAGE_SPECTRUM | S.STAGE_STATS, now_ms=1000 + k)
        fresh.close()
        assert spec.tobytes() == spec1.tobytes(), n
        np.testing.assert_array_equal(rec["peak_bin"], rec1["peak_bin"])
    eng.close()


def _ss_after_calls(S, O, torch, raws, ss_spec, n, fs, focus, mode):
    """F calls (spectrum + statistics on device buffers), each followed by signal_strength on host spectra, on one
    engine in pipelining `mode`; returns every record (device calls and signal_strength calls) as bytes."""
    dev = torch.device("cuda:0")
    B, F = raws.shape[1], raws.shape[0]
    eng = engine(S, n, fs, B, focus=focus)
    if mode:
        eng.set_pipelining(mode)
    src = [torch.from_numpy(raws[f]).to(dev) for f in range(F)]
    spec = [torch.empty((B, n), dtype=torch.float32, device=dev) for _ in range(F)]
    rec = [torch.zeros((B, S.RECORD_DTYPE.itemsize), dtype=torch.uint8, device=dev) for _ in range(F)]
    torch.cuda.synchronize()
    ss = []
    for f in range(F):
        eng.process_device(src[f].data_ptr(), S.CS8, S.STAGE_SPECTRUM | S.STAGE_STATS, spec[f].data_ptr(),
                           rec[f].data_ptr(), None, 1000 + 33 * f)
        ss.append(eng.signal_strength(ss_spec[f], now_ms=1010 + 33 * f).tobytes())
    eng.synchronize()
    out = [r.cpu().numpy().tobytes() for r in rec], ss
    eng.close()
    return out


def test_signal_strength_follows_async_statistics(S, O):
    """signal_strength after a pipelined call with asynchronous statistics (SDRG_PIPELINE_STATS_ASYNC)
    must wait for them -- both update the same stream state (tracking latch, detection ring).  Records of the device
    calls and of the signal_strength calls equal the joined schedule's bit for bit (65536 points, 200 kHz focus:
    the wide statistics kernel, the longest asynchronous launch)."""
    import torch
    n, fs, B, F = 65536, 2_000_000, 32, 4
    raws = frames(O, B, F, n=n, fs=fs)
    rng = np.random.default_rng(5)
    ss_spec = rng.exponential(1.0, size=(F, B, n)).astype(np.float32)
    ss_spec[:, :, n // 2 + 100] *= 1e4  # a peak inside the focus
    want = _ss_after_calls(S, O, torch, raws, ss_spec, n, fs, 200, 0)
    got = _ss_after_calls(S, O, torch, raws, ss_spec, n, fs, 200, S.PIPELINE_INPUTS_READY | S.PIPELINE_STATS_ASYNC)
    for k in range(F):
        assert got[0][k] == want[0][k], f"device call {k}"
        assert got[1][k] == want[1][k], f"signal_strength call {k}"


def test_signal_strength_host_keeps_odd_n_carried_bin(S, O):
    """for odd N the spectrum never writes bin N-1 (fft_process.cpp:92-97) and the host path carries the
    stream's own value there (0 from a fresh vector); a signal_strength call on caller spectra in between must not
    replace it (it stages the caller's spectra in a buffer of its own)."""
    n, fs, B = 4099, 2_000_000, 4
    eng = engine(S, n, fs, B)
    raw = np.stack([O.synth_frames(2, n, O.CS8, tone_hz=500.0 * (b + 1), fs=fs, seed=60 + b) for b in range(B)])
    spec0, _, _ = eng.process(raw[:, 0], fmt=S.CS8, stages=S.STAGE_SPECTRUM | S.STAGE_STATS, now_ms=1000)
    assert np.all(spec0[:, n - 1] == 0)
    eng.signal_strength(np.full((B, n), 7.0, np.float32), now_ms=1005)
    spec1, _, _ = eng.process(raw[:, 1], fmt=S.CS8, stages=S.STAGE_SPECTRUM | S.STAGE_STATS, now_ms=1010)
    assert np.all(spec1[:, n - 1] == 0), spec1[:, n - 1]
    eng.close()


def test_hbm_copy_probe(S):
    """sdrg_measure_hbm_copy (bench.py's roofline basis): a float4 streaming copy reports a plausible read + write rate
    (well above PCIe, below the 8 TB/s spec), and bad arguments are rejected with a status, not a crash."""
    gbs = S.measure_hbm_copy(0, 256 << 20, 5)
    assert 1000.0 < gbs < 8000.0, gbs
    with pytest.raises(S.SdrgError):
        S.measure_hbm_copy(0, 8, 1)  # fewer than 16 bytes
    with pytest.raises(S.SdrgError):
        S.measure_hbm_copy(1 << 20, 1 << 20, 1)  # no such device

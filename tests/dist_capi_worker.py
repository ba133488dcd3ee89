"""Worker of tests/test_gpu_dist_capi.py, run as its own interpreter WITHOUT torch: the multi-GPU data path through
the C ABI alone (include/sdrg.h "Multi-GPU": sdrg_dist_* + sdrg_engine_gather, RCCL loaded by libsdrg.so itself),
device memory from sdrg_device_alloc.  A one-rank RCCL communicator, a pipelined engine (inputs ready, asynchronous
statistics) and STEPS calls with their gathers -- records, focus-window slices, full spectra and PCM -- enqueued
after each call with no host synchronisation in the loop; the PCM buffer is shared by every call, so each gather must
read it before the next call's SSB stage overwrites it.  A second, joined engine on the same inputs gives the
expected outputs.  Prints one JSON line: {"ok": {...}, "torch_loaded": bool, "rccl_version": int, "rccl_data": bool}."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sdr-for-android-lib_amd"), os.path.join(ROOT, "oracle")]

import numpy as np  # noqa: E402

import oracle as O  # noqa: E402  (test infrastructure: input synthesis only)
import sdrg  # noqa: E402

N, FS, CF, FOCUS, B, STEPS = 16384, 2_000_000, 100_000_000, 5, 256, 4


def main() -> int:
    raws = np.stack([O.synth_frames(STEPS, N, O.CS8, tone_hz=170.0 * (s % 23) - 1900.0, fs=FS, seed=5100 + s)
                     for s in range(B)], axis=1)  # [STEPS][B][2N] int8
    cfg = sdrg.SDRConfig(centerFrequency=CF, samplesPerReading=N, sampleRate=FS, freqFocusRangeKhz=FOCUS, soundMode=1)
    rec_b = B * sdrg.RECORD_DTYPE.itemsize
    lo, nb = sdrg.focus_window(FS, N, FOCUS)

    # expected: a joined engine, one synchronised call per step
    ref = sdrg.Engine(cfg, B, device=0)
    plen = ref.pcm_len
    iq = [sdrg.DeviceBuffer(raws[k].nbytes) for k in range(STEPS)]
    for k in range(STEPS):
        iq[k].upload(raws[k])
    r_spec, r_rec, r_pcm = sdrg.DeviceBuffer(B * N * 4), sdrg.DeviceBuffer(rec_b), sdrg.DeviceBuffer(B * plen * 2)
    want = []
    for k in range(STEPS):
        ref.process_device(iq[k].ptr, sdrg.CS8, sdrg.STAGE_ALL, r_spec.ptr, r_rec.ptr, r_pcm.ptr, 1000 + 8 * k)
        ref.synchronize()
        want.append((r_rec.download(rec_b, np.uint8), r_spec.download((B, N), np.float32),
                     r_pcm.download((B, plen), np.int16)))
    ref.close()

    dist = sdrg.Dist(sdrg.dist_unique_id(), 1, 0, device=0)
    dist.set_one_rank_rccl(os.environ.get("DIST_CAPI_ONE_RANK_RCCL") == "1")
    info = dist.info()
    # MODE all: records, focus, spectra and PCM (the gather runs on the audio detector's stream); nopcm: no PCM (on the
    # asynchronous statistics' stream); sync: no PCM, statistics on the main stream (on the main stream).  The spectra
    # and records buffers rotate over two, so call k + 2 rewrites what gather k reads and must wait for it on the GPU.
    mode = os.environ.get("DIST_CAPI_MODE", "all")
    eng = sdrg.Engine(cfg, B, device=0)
    eng.set_pipelining(sdrg.PIPELINE_INPUTS_READY | (0 if mode == "sync" else sdrg.PIPELINE_STATS_ASYNC))
    spec = [sdrg.DeviceBuffer(B * N * 4) for _ in range(2)]
    rec = [sdrg.DeviceBuffer(rec_b) for _ in range(2)]
    pcm = sdrg.DeviceBuffer(B * plen * 2)  # one buffer for every call
    g_rec = [sdrg.DeviceBuffer(rec_b) for _ in range(STEPS)]
    g_foc = [sdrg.DeviceBuffer(B * nb * 4) for _ in range(STEPS)]
    g_spec = [sdrg.DeviceBuffer(B * N * 4) for _ in range(STEPS)]
    g_pcm = [sdrg.DeviceBuffer(B * plen * 2) for _ in range(STEPS)]
    with_pcm = mode == "all"
    for k in range(STEPS):  # no host synchronisation inside the loop
        eng.process_device(iq[k].ptr, sdrg.CS8, sdrg.STAGE_ALL, spec[k % 2].ptr, rec[k % 2].ptr, pcm.ptr, 1000 + 8 * k)
        eng.gather(dist, 0, records=rec[k % 2].ptr, records_out=g_rec[k].ptr, focus_spectra=spec[k % 2].ptr,
                   focus_out=g_foc[k].ptr, spectra=spec[k % 2].ptr, spectra_out=g_spec[k].ptr,
                   pcm=pcm.ptr if with_pcm else None, pcm_out=g_pcm[k].ptr if with_pcm else None)
    eng.synchronize()
    ok = {}
    for k in range(STEPS):
        w_rec, w_spec, w_pcm = want[k]
        ok[f"records{k}"] = bool(np.array_equal(g_rec[k].download(rec_b, np.uint8), w_rec))
        if k >= STEPS - 2:
            ok[f"engine_records{k}"] = bool(np.array_equal(rec[k % 2].download(rec_b, np.uint8), w_rec))
        ok[f"focus{k}"] = bool(np.array_equal(g_foc[k].download((B, nb), np.float32).view(np.uint32),
                                              w_spec[:, lo:lo + nb].view(np.uint32)))
        ok[f"spectra{k}"] = bool(np.array_equal(g_spec[k].download((B, N), np.float32).view(np.uint32),
                                                w_spec.view(np.uint32)))
        if with_pcm:
            ok[f"pcm{k}"] = bool(np.array_equal(g_pcm[k].download((B, plen), np.int16), w_pcm))
    ok["distinct_steps"] = not np.array_equal(want[0][2], want[1][2])
    # refused before anything is enqueued: a root outside the communicator, a missing output buffer on the root
    def refused(**kw):
        try:
            eng.gather(dist, kw.pop("root", 0), **kw)
            return False
        except sdrg.SdrgError as exc:
            return "SDRG_E_INVALID" in str(exc)
    ok["bad_root_refused"] = refused(root=1, records=rec[0].ptr, records_out=g_rec[0].ptr)
    ok["null_records_out_refused"] = refused(records=rec[0].ptr)
    ok["null_focus_out_refused"] = refused(focus_spectra=spec[0].ptr)
    ok["null_pcm_out_refused"] = refused(pcm=pcm.ptr)
    ok["empty_selection_ok"] = not refused()  # nothing selected: a no-op
    eng.close()
    dist.close()
    print(json.dumps({"ok": ok, "torch_loaded": "torch" in sys.modules, "rccl_version": info["rccl_version"],
                      "world": info["world_size"], "rccl_data": info["rccl_data"], "mode": mode}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())

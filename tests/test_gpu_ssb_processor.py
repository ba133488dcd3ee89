"""SSBProcessor queue semantics (src/ssb/ssb_processor.cpp:51-115) on the GPU path (sdrg_ssb_processor):
a consumer that falls behind loses the OLDEST queued frames (queue of 3), the worker processes the frame it holds
and then the newest three, and the SSB filter state runs on across exactly the frames that were processed —
checked bit for bit against the oracle fed that same frame sequence."""
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


def test_slow_consumer_drops_oldest_and_keeps_continuity(S, O):
    raw = O.synth_frames(10, N, O.CF32, tone_hz=1300.0, fs=FS, seed=77)  # float32 interleaved
    entered, gate = threading.Event(), threading.Event()
    got, pulses = [], []

    def on_pcm(pcm):
        got.append(pcm)
        if len(got) == 1:
            entered.set()
            assert gate.wait(timeout=60)  # the consumer is slow: frame 0's callback blocks the worker

    proc = S.SSBProcessor()
    proc.startProcessing(on_pcm, lambda s, live: pulses.append((s, live)))
    proc.enqueueData(raw[0], FS)
    assert entered.wait(timeout=60)
    for f in range(1, 10):  # the worker is blocked: the queue keeps the newest 3 (7, 8, 9)
        proc.enqueueData(raw[f], FS)
    c = proc.counters()
    assert c["enqueued"] == 10 and c["dropped"] == 6
    gate.set()
    proc.drain()
    c = proc.counters()
    assert c["processed"] == 4 and c["last_status"] == 0, c
    assert len(got) == 4 and len(pulses) == 4
    st = O.SsbState()
    for k, f in enumerate([0, 7, 8, 9]):
        want = st.process(raw[f], FS, 1)
        np.testing.assert_array_equal(got[k], want, err_msg=f"processed frame {k} (input frame {f})")
    assert proc.getCurrentRatio() == 0.0
    proc.stopProcessing()
    proc.enqueueData(raw[0], FS)  # ignored once stopped (:53)
    assert proc.counters()["enqueued"] == 10
    proc.close()


def test_queue_keeps_up_with_sound_mode_switch(S, O):
    """Frames enqueued one at a time and drained: every frame processed, in order, with the sound mode the
    worker reads when it takes the frame (BridgeConfig::getSoundMode, :102)."""
    raw = O.synth_frames(6, 8192, O.CF32, tone_hz=700.0, fs=FS, seed=78)
    got = []
    proc = S.SSBProcessor()
    proc.startProcessing(lambda p: got.append(p))
    st = O.SsbState()
    want = []
    for f in range(6):
        mode = 1 if f < 3 else 2
        proc.setSoundMode(mode)
        proc.enqueueData(raw[f], FS)
        proc.drain()
        want.append(st.process(raw[f], FS, mode))
    assert proc.counters()["dropped"] == 0
    assert len(got) == 6
    for a, b in zip(got, want):
        np.testing.assert_array_equal(a, b)
    proc.close()


def test_callback_cannot_destroy_its_own_processor(S, O):
    """A callback on the worker thread may stop its processor (the loop ends after the frame) but not destroy it
    (the worker is still inside that frame): destroy returns SDRG_E_INVALID there and succeeds afterwards from
    another thread; start from the stopped worker's callback is refused likewise."""
    raw = O.synth_frames(2, 8192, O.CF32, tone_hz=900.0, fs=FS, seed=79)
    lib = S.load()
    rcs = {}
    proc = S.SSBProcessor()

    def on_pcm(_p):
        rcs["destroy"] = lib.sdrg_ssb_processor_destroy(proc._h)
        rcs["stop"] = lib.sdrg_ssb_processor_stop(proc._h)
        rcs["start"] = lib.sdrg_ssb_processor_start(proc._h, None)

    proc.startProcessing(on_pcm)
    proc.enqueueData(raw[0], FS)
    proc.drain()
    assert rcs == {"destroy": -1, "stop": 0, "start": -1}, rcs
    assert proc.counters()["processed"] == 1
    proc.stopProcessing()  # joins the ended loop
    proc.startProcessing(lambda p: rcs.setdefault("again", len(p)))  # restartable from another thread
    proc.enqueueData(raw[1], FS)
    proc.drain()
    assert rcs.get("again", 0) > 0
    proc.close()

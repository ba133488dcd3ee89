"""CPU tests of the ingest re-chunker (csrc/ingest.cpp, host-only): exact-N cutting, drop-oldest queueing and
the CS12 repack, against a Python model of the reference's rx_reading_thread loop
(src/sdr-bridge-java-soapy.cpp:541-573: accBuffer.insert, while size >= N cut a chunk, rx_queue drops its
front at RX_QUEUE_MAX = 20).

CS12: the layout is SoapySDR's published CS12 -> CS16 converter (I = b0 | (b1 & 0xf) << 8 and
Q = b1 >> 4 | b2 << 4, each in the top 12 bits of an int16).  SoapySDR is not in the reference tree and has
no fixture here, so this convention is parity-unpinned; the test pins our code to the published formula.
"""
import numpy as np
import pytest

import sdrg


class RefReader:
    """The reference's accumulate-and-cut loop for one stream (frames kept as raw bytes)."""

    def __init__(self, n, bps, queue_max=20):
        self.n, self.bps, self.qmax = n, bps, queue_max
        self.acc = b""
        self.queue = []
        self.dropped = 0

    def push(self, raw: bytes):
        self.acc += raw                                        # accBuffer.insert (:543-547)
        fb = self.n * self.bps
        while len(self.acc) >= fb:                             # while (accBuffer.size() >= N) (:550)
            if len(self.queue) >= self.qmax:                   # rx_queue.pop_front (:560-561)
                self.queue.pop(0)
                self.dropped += 1
            self.queue.append(self.acc[:fb])
            self.acc = self.acc[fb:]                           # accBuffer.erase (:566-569)


def cs12_to_cs16(raw: np.ndarray) -> np.ndarray:
    b = raw.reshape(-1, 3).astype(np.uint16)
    i = ((b[:, 1] << 12) | (b[:, 0] << 4)) & 0xFFFF
    q = ((b[:, 2] << 8) | (b[:, 1] & 0xF0)) & 0xFFFF
    return np.stack([i, q], axis=1).reshape(-1).astype(np.uint16).view(np.int16)


@pytest.mark.parametrize("fmt", [sdrg.CS8, sdrg.CU8, sdrg.CS16, sdrg.CF32])
def test_exact_n_cutting_matches_reference_loop(fmt):
    rng = np.random.default_rng(fmt + 7)
    n, streams, qmax = 1000, 3, 5
    bps = sdrg.IN_BYTES_PER_SAMPLE[fmt]
    ing = sdrg.Ingest(streams, n, fmt, qmax)
    refs = [RefReader(n, bps, qmax) for _ in range(streams)]
    popped = [[] for _ in range(streams)]
    want = [[] for _ in range(streams)]
    for it in range(300):
        s = int(rng.integers(streams))
        k = int(rng.choice([0, 1, 7, 333, 999, 1000, 1001, 2500, 4096]))
        raw = rng.integers(0, 256, k * bps, dtype=np.uint8)
        ing.push(s, raw)
        refs[s].push(raw.tobytes())
        if it % 3 == 0:  # the processing thread pops sometimes (queue overflows in between)
            for t in range(streams):
                f = ing.pop(t)
                if refs[t].queue:
                    want[t].append(refs[t].queue.pop(0))
                    assert f is not None
                    popped[t].append(f.view(np.uint8).tobytes())
                else:
                    assert f is None
        for t in range(streams):
            q, part, dropped = ing.status(t)
            assert q == len(refs[t].queue) and part * bps == len(refs[t].acc) and dropped == refs[t].dropped
    for t in range(streams):
        assert popped[t] == want[t]


def test_pop_batch_waits_for_every_stream():
    n = 64
    ing = sdrg.Ingest(2, n, sdrg.CS8)
    a = np.arange(2 * n, dtype=np.int8)
    ing.push(0, a)
    assert ing.pop_batch() is None
    ing.push(1, a[: n])          # half a frame
    assert ing.pop_batch() is None
    ing.push(1, a[n:])
    out = ing.pop_batch()
    assert out.shape == (2, 2 * n) and (out[0] == a).all() and (out[1] == a).all()
    assert ing.pop_batch() is None


def test_cs12_repacked_to_cs16():
    rng = np.random.default_rng(12)
    n = 500
    raw = rng.integers(0, 256, 3 * n * 2, dtype=np.uint8)  # two frames
    ing = sdrg.Ingest(1, n, sdrg.CS12)
    assert ing.out_format == sdrg.CS16
    ing.push(0, raw[: 3 * 377])
    ing.push(0, raw[3 * 377:])
    want = cs12_to_cs16(raw)
    f0, f1 = ing.pop(0), ing.pop(0)
    assert f0.dtype == np.int16 and (f0 == want[: 2 * n]).all() and (f1 == want[2 * n:]).all()
    # the 12-bit two's-complement value sits in the top bits: v12 = int16 >> 4
    b = raw[:3].astype(np.int32)
    i12 = ((b[1] & 0xF) << 8) | b[0]
    i12 = i12 - 4096 if i12 >= 2048 else i12
    assert f0[0] >> 4 == i12


def test_set_samples_per_reading_keeps_partial_samples():
    ing = sdrg.Ingest(1, 100, sdrg.CS16)
    x = np.arange(2 * 250, dtype=np.int16)
    ing.push(0, x)                       # two frames queued + 50 samples pending
    assert ing.status(0)[:2] == (2, 50)
    ing.set_samples_per_reading(40)      # queued 100-sample frames dropped, 50 pending -> one 40 frame + 10
    assert ing.status(0)[:2] == (1, 10)
    f = ing.pop(0)
    assert (f == x[2 * 200: 2 * 240]).all()


def test_errors():
    with pytest.raises(sdrg.SdrgError):
        sdrg.Ingest(1, 0, sdrg.CS8)
    with pytest.raises(sdrg.SdrgError):
        sdrg.Ingest(1, 16, 9)
    ing = sdrg.Ingest(2, 16, sdrg.CS16)
    with pytest.raises(sdrg.SdrgError):
        ing.push(2, np.zeros(4, np.int16))
    with pytest.raises(sdrg.SdrgError):
        ing.push(0, np.zeros(3, np.uint8))  # not a whole sample

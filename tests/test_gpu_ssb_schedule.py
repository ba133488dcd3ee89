"""SSB pipeline schedule edges (csrc/ssb.hip): the low-pass lookahead ring (3 slots, the whole-loop asm block when
the frame is whole 64-sample chunks, the C++ path for a partial last chunk), frames of 1-3 chunks, partial
workgroups, the direct-load path (CF32: no LDS-DMA at 256-B batches), sound-mode switches and several calls in a
row: PCM bit-exact against the oracle's processSSB_opt restatement (ssb_demod_opt.cpp:221-296), which the
reference build pins (tests/golden)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def S():
    import sdrg
    return sdrg


@pytest.fixture(scope="module")
def O():
    import oracle
    return oracle


# n: 64 (1 chunk), 192 (3), 100 / 1000 / 1500 (partial last chunk), 4096; fs with decimation 41 or 50
@pytest.mark.parametrize("fmt_name,n,fs", [("CS8", 64, 2_000_000), ("CS8", 100, 2_000_000), ("CS8", 192, 2_000_000),
                                           ("CS8", 1000, 2_000_000), ("CU8", 1500, 2_400_000),
                                           ("CS16", 4096, 2_000_000), ("CF32", 1000, 2_500_000),
                                           ("CF32", 4096, 2_000_000)])
@pytest.mark.parametrize("B", [21, 45])
def test_ssb_schedule_edges_vs_oracle(S, O, fmt_name, n, fs, B):
    fmt = getattr(O, fmt_name)
    # 21 streams: one workgroup of 32 with its second 16-stream group partly live (16 + 5); 45: a full workgroup and
    # one of 13 streams whose second group is empty (lab builds of 16-stream workgroups: 1 full + 1 partial, 2 + 1)
    F = 4
    raw = np.stack([O.synth_frames(F, n, fmt, tone_hz=300.0 * (b + 1) - 3000.0, fs=fs, seed=77 + b) for b in range(B)])
    cfg = S.SDRConfig(centerFrequency=100_000_000, samplesPerReading=n, sampleRate=fs, freqFocusRangeKhz=5,
                      soundMode=1)
    eng = S.Engine(cfg, B)
    sst = [O.SsbState() for _ in range(B)]
    modes = [1, 1, 2, 0]  # mode switches between calls (setSoundMode -> the next call's parameters)
    for f in range(F):
        eng.setSoundMode(modes[f])
        _, _, pcm = eng.process(raw[:, f], fmt=fmt, stages=S.STAGE_SSB)
        for b in range(B):
            want = sst[b].process(O.unpack(fmt, raw[b, f], n), fs, modes[f])
            np.testing.assert_array_equal(pcm[b], want, err_msg=f"{fmt_name} n={n} stream {b} frame {f}")
    eng.close()

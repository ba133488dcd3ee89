// ref_pulse_driver.cpp — TEST INFRASTRUCTURE ONLY (container-side).
//
// A command-line driver around the REFERENCE's own pulse detectors, which oracle/Makefile compiles from
// /root/reference (unmodified, g++ -O2 -std=c++20, the reference's x86-64 flags) into oracle/_ref/ref_pulse:
//   src/dsp/spectral_pulse_detector.cpp   src/ssb/audio_pulse_detector.cpp
// Used to pin oracle/pulse_oracle.c and to write the tests/golden/pulse_*.npz fixtures.  This file is our
// code: it only calls the public members declared in the two reference headers.
//
//   ref_pulse spectral <fs_energy> [<k> <fs_energy2>]
//       stdin: float32 pairs (snrSigma, freqHz), one per frame.  Builds SpectralPulseDetector with the default
//       Config but fsEnergy = <fs_energy> (what applyConfig does, sdr-bridge-java-soapy.cpp:1130-1138); before
//       frame <k> calls configure() with fsEnergy = <fs_energy2>.  stdout: one sdrg_pulse_output per frame.
//   ref_pulse audio <fmt> <block>
//       stdin: int16 (fmt 0) or float32 (fmt 1) samples; AudioPulseDetector with the default Config (what
//       SSBProcessor uses, setPulseConfig being a no-op in the bridge) processes them in blocks of <block>
//       samples (the last block may be shorter).  stdout: one sdrg_pulse_output per block.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "audio_pulse_detector.h"
#include "spectral_pulse_detector.h"
#include "../include/sdrg.h"

static void emit(const sdrg_pulse_output &o) { std::fwrite(&o, sizeof(o), 1, stdout); }

int main(int argc, char **argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: ref_pulse spectral <fs> [<k> <fs2>] | audio <fmt> <block>\n");
        return 2;
    }
    if (!std::strcmp(argv[1], "spectral")) {
        SpectralPulseDetector::Config cfg;
        cfg.fsEnergy = std::strtof(argv[2], nullptr);
        SpectralPulseDetector det;
        det.configure(cfg);
        const long k_re = argc > 4 ? std::strtol(argv[3], nullptr, 10) : -1;
        const float fs2 = argc > 4 ? std::strtof(argv[4], nullptr) : 0.f;
        float in[2];
        for (long k = 0; std::fread(in, sizeof(float), 2, stdin) == 2; k++) {
            if (k == k_re) {
                SpectralPulseDetector::Config c2;
                c2.fsEnergy = fs2;
                det.configure(c2);
            }
            det.process(in[0], in[1]);
            sdrg_pulse_output o;
            std::memset(&o, 0, sizeof(o));
            o.strength = det.lastPulseStrength();
            o.live_etat = det.liveEtat();
            o.level = static_cast<int32_t>(det.pulseDetected());
            o.locked = det.isLocked() ? 1 : 0;
            o.period_s = det.lockedPeriodS();
            o.est_freq_hz = det.estimatedFreqHz();
            o.est_freq_hz_rounded = std::llround(det.estimatedFreqHz());
            o.input = in[0];
            emit(o);
        }
        return 0;
    }
    if (!std::strcmp(argv[1], "audio") && argc >= 4) {
        const int fmt = std::atoi(argv[2]);
        const size_t block = (size_t)std::atol(argv[3]);
        AudioPulseDetector det;
        const size_t es = fmt == 0 ? 2 : 4;
        std::vector<char> buf(block * es);
        for (;;) {
            const size_t got = std::fread(buf.data(), es, block, stdin);
            if (got == 0) break;
            if (fmt == 0) {
                std::vector<int16_t> pcm(got);
                std::memcpy(pcm.data(), buf.data(), got * es);
                det.process(pcm);
            } else {
                std::vector<float> a(got);
                std::memcpy(a.data(), buf.data(), got * es);
                det.process(a);
            }
            sdrg_pulse_output o;
            std::memset(&o, 0, sizeof(o));
            o.strength = det.lastPulseStrength();
            o.live_etat = det.liveEtat();
            o.level = static_cast<int32_t>(det.pulseDetected());
            o.locked = det.isLocked() ? 1 : 0;
            o.period_s = det.lockedPeriodS();
            o.input = det.lastPulseStrength();
            emit(o);
            if (got < block) break;
        }
        return 0;
    }
    std::fprintf(stderr, "bad arguments\n");
    return 2;
}

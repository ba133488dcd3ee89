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
//   ref_pulse audio <fmt> <block> [key=value ...]
//       stdin: int16 (fmt 0) or float32 (fmt 1) samples; AudioPulseDetector with the default Config (what
//       SSBProcessor uses, setPulseConfig being a no-op in the bridge) processes them in blocks of <block>
//       samples (the last block may be shorter).  stdout: one sdrg_pulse_output per block.
//   Both kinds take optional Config overrides as key=value (the reference Config field names), e.g.
//   snrStrong=3.5 liveDivisor=2 (spectral: after fs_energy / the reconfigure pair).
#include <cmath>
#include <string>
#include <type_traits>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "audio_pulse_detector.h"
#include "spectral_pulse_detector.h"
#include "../include/sdrg.h"

static void emit(const sdrg_pulse_output &o) { std::fwrite(&o, sizeof(o), 1, stdout); }

// key=value Config overrides (field names of the reference Config structs)
template <class C>
static bool set_field(C &c, const char *kv) {
    const char *eq = std::strchr(kv, '=');
    if (!eq) return false;
    const std::string k(kv, eq - kv);
    const float v = std::strtof(eq + 1, nullptr);
    const int iv = std::atoi(eq + 1);
#define F(name) if (k == #name) { c.name = v; return true; }
#define I(name) if (k == #name) { c.name = iv; return true; }
    F(fsEnergy) F(zDefaultS) F(tTargetInit) F(dtTolS) F(snrMin) F(snrRhythm) F(snrStrong) F(dispersionMax)
    I(sumNMax) F(liveWindowT) F(liveDivisor)
    if constexpr (std::is_same_v<C, AudioPulseDetector::Config>) {
        F(sampleRate) F(fMin) F(fMax) F(smoothCutoff) I(noiseRefFar) I(noiseRefNear)
    }
#undef F
#undef I
    return false;
}

int main(int argc, char **argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: ref_pulse spectral <fs> [<k> <fs2>] | audio <fmt> <block>\n");
        return 2;
    }
    if (!std::strcmp(argv[1], "spectral")) {
        SpectralPulseDetector::Config cfg;
        cfg.fsEnergy = std::strtof(argv[2], nullptr);
        int a = 3;
        long k_re = -1;
        float fs2 = 0.f;
        if (argc > 4 && !std::strchr(argv[3], '=')) {
            k_re = std::strtol(argv[3], nullptr, 10);
            fs2 = std::strtof(argv[4], nullptr);
            a = 5;
        }
        for (; a < argc; a++)
            if (!set_field(cfg, argv[a])) { std::fprintf(stderr, "bad override %s\n", argv[a]); return 2; }
        SpectralPulseDetector det(cfg);
        float in[2];
        for (long k = 0; std::fread(in, sizeof(float), 2, stdin) == 2; k++) {
            if (k == k_re) {
                SpectralPulseDetector::Config c2 = cfg;
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
        AudioPulseDetector::Config cfg;
        for (int a = 4; a < argc; a++)
            if (!set_field(cfg, argv[a])) { std::fprintf(stderr, "bad override %s\n", argv[a]); return 2; }
        AudioPulseDetector det(cfg);
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

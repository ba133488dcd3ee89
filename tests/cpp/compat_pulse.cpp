// compat_pulse.cpp — exercises the pulse-detector drop-ins (include/sdrg_compat.hpp) the way the reference
// bridge and SSBProcessor call them (sdr-bridge-java-soapy.cpp:477-488, ssb_processor.cpp:109-113).
//   compat_pulse spectral <fs_energy> <in.bin> <out.bin>   in: float32 (snrSigma, freqHz) pairs
//   compat_pulse audio <block> <in.bin> <out.bin>          in: int16 PCM, processed in blocks
// out: per call float strength, int32 liveEtat, int32 level, int32 locked, float period, float estFreq
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "sdrg_compat.hpp"

using namespace sdrg::compat;

template <class D>
static void emit(FILE *fo, const D &d, float est) {
    const float f[2] = {d.lastPulseStrength(), d.lockedPeriodS()};
    const int32_t i[3] = {d.liveEtat(), static_cast<int32_t>(d.pulseDetected()), d.isLocked() ? 1 : 0};
    std::fwrite(&f[0], 4, 1, fo);
    std::fwrite(i, 4, 3, fo);
    std::fwrite(&f[1], 4, 1, fo);
    std::fwrite(&est, 4, 1, fo);
}

int main(int argc, char **argv) {
    if (argc != 5) return 2;
    FILE *fi = std::fopen(argv[3], "rb");
    FILE *fo = std::fopen(argv[4], "wb");
    if (!fi || !fo) return 3;
    if (!std::strcmp(argv[1], "spectral")) {
        SpectralPulseDetector::Config cfg;
        cfg.fsEnergy = std::strtof(argv[2], nullptr);
        SpectralPulseDetector det;
        det.configure(cfg);  // applyConfig (sdr-bridge-java-soapy.cpp:1130-1138)
        float in[2];
        while (std::fread(in, 4, 2, fi) == 2) {
            det.process(in[0], in[1]);
            if (det.lastStatus()) { std::fprintf(stderr, "%s\n", sdrg_last_error()); return 5; }
            emit(fo, det, det.estimatedFreqHz());
        }
    } else {
        const size_t block = (size_t)std::atol(argv[2]);
        AudioPulseDetector det;
        std::vector<int16_t> pcm(block);
        for (;;) {
            const size_t got = std::fread(pcm.data(), 2, block, fi);
            if (!got) break;
            pcm.resize(got);
            det.process(pcm);
            if (det.lastStatus()) { std::fprintf(stderr, "%s\n", sdrg_last_error()); return 5; }
            emit(fo, det, 0.f);
            if (got < block) break;
            pcm.resize(block);
        }
    }
    std::fclose(fi);
    std::fclose(fo);
    return 0;
}

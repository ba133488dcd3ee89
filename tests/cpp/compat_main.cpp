// compat_main.cpp — exercises the C++ drop-ins (include/sdrg_compat.hpp) the way the reference bridge
// calls FFTProcessor and processSSB_opt (sdr-bridge-java-soapy.cpp:441-455, ssb_processor.cpp:103).
//   compat_main <in.bin> <out.bin> <n> <frames> <fs> <cf> <focus_khz> <mode>
// in.bin : frames x n x complex<float>;  out.bin: per frame n floats spectrum, 11 record floats/ints as
// float64, int32 pcm count + int16 pcm.
#include <complex>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "sdrg_compat.hpp"

using namespace sdrg::compat;

int main(int argc, char **argv) {
    if (argc != 9) return 2;
    const int n = std::atoi(argv[3]), frames = std::atoi(argv[4]);
    const uint32_t fs = (uint32_t)std::strtoul(argv[5], nullptr, 10), cf = (uint32_t)std::strtoul(argv[6], nullptr, 10);
    const int focus = std::atoi(argv[7]), mode = std::atoi(argv[8]);
    FILE *fi = std::fopen(argv[1], "rb");
    FILE *fo = std::fopen(argv[2], "wb");
    if (!fi || !fo) return 3;
    FFTProcessor fft;
    fft.configure(FftProcessorConfig{cf, fs, n, focus});
    std::vector<std::complex<float>> buf(n);
    for (int f = 0; f < frames; f++) {
        if (std::fread(buf.data(), sizeof(buf[0]), n, fi) != (size_t)n) return 4;
        fft.processAt(buf.data(), (uint32_t)n, 1000 + 100 * f);
        if (fft.lastStatus() != 0) { std::fprintf(stderr, "fft status %d: %s\n", fft.lastStatus(), sdrg_last_error()); return 5; }
        std::vector<int16_t> pcm;
        bool pulse = false;
        processSSB_opt(buf, fs, true, pcm, pulse, mode);
        if (lastSsbStatus() != 0) { std::fprintf(stderr, "ssb status %d: %s\n", lastSsbStatus(), sdrg_last_error()); return 6; }
        const std::vector<float> &p = fft.getPowerSpectrum();
        std::fwrite(p.data(), sizeof(float), p.size(), fo);
        const double rec[11] = {fft.getMeanSnrDb(), fft.getMeanSnrSigma(), (double)fft.getTrackingFrequency(),
                                (double)fft.getDetectionFlag(), fft.getPeakAboveNoiseMeanDb(), fft.getMaxBinSnrDb(),
                                fft.getMaxBinSnrSigma(), fft.getBest1kHzSnrDb(), fft.getBest1kHzSnrSigma(),
                                fft.getBest1kHzCenterFreqHz(), fft.getPerBinMean()};
        std::fwrite(rec, sizeof(double), 11, fo);
        const int32_t c = (int32_t)pcm.size();
        std::fwrite(&c, sizeof(c), 1, fo);
        std::fwrite(pcm.data(), sizeof(int16_t), pcm.size(), fo);
    }
    std::fclose(fi);
    std::fclose(fo);
    return 0;
}

// ref_ssb_driver.cpp — TEST INFRASTRUCTURE ONLY (container-side).
//
// A command-line driver around the REFERENCE's own src/ssb/ssb_demod_opt.cpp, which oracle/Makefile
// compiles from /root/reference (unmodified, g++ -O2 -std=c++20, the reference's x86-64 flags) into
// oracle/_ref/ref_ssb.  Used to pin oracle/sdrg_oracle.c bit-for-bit and to write tests/golden fixtures.
// This file is our code: it only calls the public functions declared in ssb_demod_opt.h.
//
//   ref_ssb taps  <in_size> <decim>            FIR taps of simpleFIRDecimate (impulse responses), %a per line
//   ref_ssb lpf   <fs> <fc> <Q>                 iir2InitLowpass coefficients a0 a1 a2 b1 b2
//   ref_ssb hp    <fs> <f0> <Q>                 biquadInitHighpass coefficients
//   ref_ssb bp    <fs> <f0> <Q>                 biquadInitBandpass coefficients
//   ref_ssb run   <fs> <upper> <n> <mode>...    one frame of n CF32 samples per mode from stdin through
//                                               processSSB_opt (statics live for this process); writes
//                                               per frame int32 count + int16 pcm to stdout
//   ref_ssb stages <fs> <n> <fc> <Q> <target> <fast> <coeff>
//                                               one CF32 frame from stdin through the individual stage
//                                               functions; writes int32 count + float32[] for dc_re,
//                                               lpf, agc, fir, eq
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <complex>
#include <algorithm>

#include "ssb_demod_opt.h"

static void print_hex(const float *v, int n) {
    for (int i = 0; i < n; i++) std::printf("%a\n", (double)v[i]);
}

static bool read_frame(std::vector<std::complex<float>> &iq, size_t n) {
    iq.resize(n);
    return std::fread(iq.data(), sizeof(std::complex<float>), n, stdin) == n;
}

static void write_floats(const std::vector<float> &v) {
    int32_t c = (int32_t)v.size();
    std::fwrite(&c, sizeof(c), 1, stdout);
    if (c) std::fwrite(v.data(), sizeof(float), v.size(), stdout);
}

int main(int argc, char **argv) {
    if (argc < 2) return 2;
    const std::string cmd = argv[1];
    if (cmd == "taps" && argc == 4) {
        const size_t in_size = std::strtoull(argv[2], nullptr, 10);
        const int decim = std::atoi(argv[3]);
        // impulse at p: output 0 = sum_k in[k] h[k] = h[p] exactly (every other product is +-0)
        std::vector<float> taps;
        for (size_t p = 0; p < 255 && p < in_size; p++) {
            std::vector<float> in(in_size, 0.0f);
            in[p] = 1.0f;
            std::vector<float> out = simpleFIRDecimate(in, decim, 0.45f);
            if (out.empty()) break;
            taps.push_back(out[0]);
        }
        std::printf("%d\n", (int)taps.size());
        print_hex(taps.data(), (int)taps.size());
        return 0;
    }
    if ((cmd == "lpf" || cmd == "hp" || cmd == "bp") && argc == 5) {
        const float fs = std::strtof(argv[2], nullptr), f0 = std::strtof(argv[3], nullptr), q = std::strtof(argv[4], nullptr);
        float c[5];
        if (cmd == "lpf") {
            IIR2 f; iir2InitLowpass(f, fs, f0, q);
            c[0] = f.a0; c[1] = f.a1; c[2] = f.a2; c[3] = f.b1; c[4] = f.b2;
        } else {
            Biquad f;
            if (cmd == "hp") biquadInitHighpass(f, fs, f0, q); else biquadInitBandpass(f, fs, f0, q);
            c[0] = f.a0; c[1] = f.a1; c[2] = f.a2; c[3] = f.b1; c[4] = f.b2;
        }
        print_hex(c, 5);
        return 0;
    }
    if (cmd == "run" && argc >= 6) {
        const uint32_t fs = (uint32_t)std::strtoul(argv[2], nullptr, 10);
        const bool upper = std::atoi(argv[3]) != 0;
        const size_t n = std::strtoull(argv[4], nullptr, 10);
        for (int a = 5; a < argc; a++) {
            std::vector<std::complex<float>> iq;
            if (!read_frame(iq, n)) return 3;
            std::vector<int16_t> pcm;
            bool pulse = false;
            processSSB_opt(iq, fs, upper, pcm, pulse, std::atoi(argv[a]));
            int32_t c = (int32_t)pcm.size();
            std::fwrite(&c, sizeof(c), 1, stdout);
            if (c) std::fwrite(pcm.data(), sizeof(int16_t), pcm.size(), stdout);
        }
        return 0;
    }
    if (cmd == "stages" && argc == 9) {
        const uint32_t fs = (uint32_t)std::strtoul(argv[2], nullptr, 10);
        const size_t n = std::strtoull(argv[3], nullptr, 10);
        const float fc = std::strtof(argv[4], nullptr), q = std::strtof(argv[5], nullptr);
        const float target = std::strtof(argv[6], nullptr), fast = std::strtof(argv[7], nullptr);
        const float coeff = std::strtof(argv[8], nullptr);
        std::vector<std::complex<float>> iq;
        if (!read_frame(iq, n)) return 3;
        removeDC(iq, 0.9995f);
        std::vector<float> dc_re(n);
        for (size_t i = 0; i < n; i++) dc_re[i] = iq[i].real();
        IIR2 rf; iir2InitLowpass(rf, (float)fs, fc, q);
        iir2Process(rf, iq);
        std::vector<float> lpf(n);
        for (size_t i = 0; i < n; i++) lpf[i] = iq[i].real();
        std::vector<float> audio;
        demodSSB(iq, audio, true);
        adaptiveAGC(audio, target, fast, 0.00035f);
        const int decim = std::max(1, static_cast<int>(fs / 48000.0f));
        std::vector<float> fir = simpleFIRDecimate(audio, decim, 0.45f);
        std::vector<float> eq = fir;
        Biquad hp, bp;
        biquadInitHighpass(hp, 48000.0f, 1200.0f, 0.7f);
        biquadInitBandpass(bp, 48000.0f, 2400.0f, 0.6f);
        if (!eq.empty()) {
            biquadProcess(hp, eq);
            biquadProcess(bp, eq);
            transientBoost(eq, coeff);
        }
        write_floats(dc_re);
        write_floats(lpf);
        write_floats(audio);
        write_floats(fir);
        write_floats(eq);
        return 0;
    }
    return 2;
}

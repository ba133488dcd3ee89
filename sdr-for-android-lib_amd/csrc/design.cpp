// design.cpp — host-side filter design and window geometry, with the reference's own float expressions.
//
// Everything here is per configuration, not per sample, so it runs on the host once and the kernels
// receive the resulting coefficients.  The expressions are kept exactly as the reference writes them
// (mixed double/float promotions included) and this file is compiled without FP contraction, so the
// coefficients are bit-identical to the reference's x86-64 build (checked by tests/test_engine_host.py
// against tests/golden/golden_ssb_design.npz, which comes from the reference build).
#include <math.h>

#include <cmath>
#include <stdint.h>

#include "design.h"
#include "glibc_logf.h"

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif


namespace sdrg {

// iir2InitLowpass (src/ssb/ssb_demod_opt.cpp:60-73)
void design_lowpass(float fs, float fc, float Q, float c[5]) {
    float w0 = 2.0f * M_PI * fc / fs;
    float cosw0 = cosf(w0);
    float sinw0 = sinf(w0);
    float alpha = sinw0 / (2.0f * Q);
    float norm = 1.0f / (1.0f + alpha);
    c[0] = (1.0f - cosw0) / 2.0f * norm;
    c[1] = (1.0f - cosw0) * norm;
    c[2] = c[0];
    c[3] = -2.0f * cosw0 * norm;
    c[4] = (1.0f - alpha) * norm;
}

// biquadInitHighpass (:148-164)
void design_highpass(float fs, float f0, float Q, float c[5]) {
    float w0 = 2.0f * M_PI * f0 / fs;
    float cosw0 = cosf(w0);
    float sinw0 = sinf(w0);
    float alpha = sinw0 / (2.0f * Q);
    float b0 = (1 + cosw0) / 2.0f;
    float b1 = -(1 + cosw0);
    float b2 = (1 + cosw0) / 2.0f;
    float a0 = 1 + alpha;
    float a1 = -2 * cosw0;
    float a2 = 1 - alpha;
    c[0] = b0 / a0;
    c[1] = b1 / a0;
    c[2] = b2 / a0;
    c[3] = a1 / a0;
    c[4] = a2 / a0;
}

// biquadInitBandpass (:166-175)
void design_bandpass(float fs, float f0, float Q, float c[5]) {
    float w0 = 2.0f * M_PI * f0 / fs;
    float alpha = sinf(w0) / (2.0f * Q);
    float cosw0 = cosf(w0);
    float b0 = alpha, b1 = 0.0f, b2 = -alpha;
    float a0 = 1.0f + alpha, a1 = -2.0f * cosw0, a2 = 1.0f - alpha;
    c[0] = b0 / a0;
    c[1] = b1 / a0;
    c[2] = b2 / a0;
    c[3] = a1 / a0;
    c[4] = a2 / a0;
}

// simpleFIRDecimate's Hann-windowed sinc (:121-134); returns the tap count.  taps0: the length asked
// for (0 = the reference's 255; other values only through the NCO/short-FIR variant, sdrg.h)
int design_fir(int64_t in_size, int decim, float cutoff_rel, float *h, int taps0) {
    int N = ssb_taps_for(in_size, taps0);
    int M = N - 1;
    float fc = cutoff_rel / decim;
    for (int n = 0; n < N; n++) {
        int k = n - M / 2;
        float sinc = (k == 0) ? 2.0f * M_PI * fc : sinf(2.0f * M_PI * fc * k) / (float)k;
        float w = 0.5f - 0.5f * cosf(2.0f * M_PI * n / M);
        h[n] = (sinc / M_PI) * w;
    }
    float sum = 0.0f;
    for (int n = 0; n < N; n++) sum += h[n];
    if (sum != 0.0f)
        for (int n = 0; n < N; n++) h[n] /= sum;
    return N;
}

int ssb_decim(uint32_t sample_rate) {  // processSSB_opt :273
    const int d = (int)(sample_rate / 48000.0f);
    return d > 1 ? d : 1;
}

int ssb_taps_for(int64_t samp_count, int taps0) {
    int N = taps0 > 0 ? taps0 : 255;
    if (N > (int)samp_count) N = (int)samp_count | 1;
    return N;
}

int ssb_pcm_len(int64_t samp_count, uint32_t sample_rate, int taps0) {
    const int N = ssb_taps_for(samp_count, taps0);
    if (samp_count < N) return 0;
    return (int)((samp_count - N) / ssb_decim(sample_rate) + 1);
}

static int off_to_bin(float offset_hz, float nyquist, float freq_per_bin) {  // fft_process.cpp:131-133
    return (int)((offset_hz + nyquist) / freq_per_bin);
}

// Window geometry of evaluateSignalStrength (fft_process.cpp:124-216)
StatsGeometry stats_geometry(uint32_t sample_rate, uint32_t center_frequency, int n, int focus_khz) {
    StatsGeometry g{};
    g.n = n;
    const float freq_per_bin = static_cast<float>(sample_rate) / static_cast<float>(n);
    const float X_hz = focus_khz * 1000.0f;
    const float nyquist = sample_rate / 2.0f;
    int lo = off_to_bin(-X_hz, nyquist, freq_per_bin);
    int hi = off_to_bin(+X_hz, nyquist, freq_per_bin) - 1;
    g.focus_lo = lo > 0 ? lo : 0;
    g.focus_hi = hi < n - 1 ? hi : n - 1;
    g.focus_len = g.focus_hi - g.focus_lo + 1;
    // the Gumbel term's logN (:282): geometry only, so computed here with the reference's libm (glibc's logf,
    // restated in glibc_logf.h so the value does not depend on the host's C library)
    g.log_focus_len = g.focus_len > 0 ? glibc::logf(static_cast<float>(g.focus_len)) : 0.0f;
    const int w = (int)ceilf(1000.0f / freq_per_bin);
    g.win_bins_1k = w > 1 ? w : 1;
    int nr = 0;
    for (int k = 1; k <= 5; k++) {
        const float nearX = (4 * k - 2) * X_hz;
        const float farX = 4 * k * X_hz;
        if (farX >= nyquist) break;
        for (int side = 0; side < 2; side++) {
            int l, h;
            if (side == 0) {
                l = off_to_bin(+nearX, nyquist, freq_per_bin);
                h = off_to_bin(+farX, nyquist, freq_per_bin) - 1;
            } else {
                l = off_to_bin(-farX, nyquist, freq_per_bin);
                h = off_to_bin(-nearX, nyquist, freq_per_bin) - 1;
            }
            l = l > 0 ? l : 0;
            h = h < n - 1 ? h : n - 1;
            if (h <= l) continue;
            g.win_lo[nr] = l;
            g.win_hi[nr] = h;
            nr++;
        }
    }
    g.n_ref = nr;
    // pooled bins: the nBottom longest windows bound the pool whatever the sort order
    int lens[10];
    for (int i = 0; i < nr; i++) lens[i] = g.win_hi[i] - g.win_lo[i] + 1;
    for (int i = 1; i < nr; i++)
        for (int j = i; j > 0 && lens[j] > lens[j - 1]; j--) {
            const int t = lens[j];
            lens[j] = lens[j - 1];
            lens[j - 1] = t;
        }
    const int nb0 = (int)(nr * 0.4f);
    const int n_bottom = nb0 > 1 ? nb0 : 1;
    int pool = 0;
    for (int i = 0; i < n_bottom && i < nr; i++) pool += lens[i];
    g.max_pool = pool;
    int slo = g.focus_lo, shi = g.focus_hi;
    for (int i = 0; i < nr; i++) {
        slo = g.win_lo[i] < slo ? g.win_lo[i] : slo;
        shi = g.win_hi[i] > shi ? g.win_hi[i] : shi;
    }
    g.span_lo = slo;
    g.span_len = g.focus_len > 0 ? shi - slo + 1 : 0;
    g.freq_per_bin = freq_per_bin;
    g.nyquist = nyquist;
    g.cf_float = static_cast<float>(center_frequency);
    g.cf_minus_nyq = static_cast<float>(center_frequency) - nyquist;  // :327
    g.cf_u32_minus_nyq = (center_frequency - nyquist);                // :350, uint32 promoted to float
    g.cf_changed = 0;
    return g;
}

// Bilinear-transform Butterworth sections of the audio pulse detector, in float with the reference's
// expression order (audio_pulse_detector.cpp:4, :29-55).
void design_pulse_sos(float fs, float fc, bool highpass, float c[5]) {
    const float pi = 3.14159265358979f;
    const float Q = 0.7071f;
    const float K = tanf(pi * fc / fs);
    const float K2 = K * K;
    const float norm = K2 + K / Q + 1.f;
    if (highpass) {
        c[0] = 1.f / norm;
        c[1] = -2.f / norm;
        c[2] = 1.f / norm;
    } else {
        c[0] = K2 / norm;
        c[1] = 2.f * K2 / norm;
        c[2] = K2 / norm;
    }
    c[3] = 2.f * (K2 - 1.f) / norm;
    c[4] = (K2 - K / Q + 1.f) / norm;
}

// NCO of the SSB variant (sdrg.h, sdrg_engine_set_ssb_variant): phase increment per sample of a 32-bit
// phase accumulator, round(hz / fs * 2^32) modulo 2^32 (negative frequencies wrap)
uint32_t nco_increment(double hz, uint32_t sample_rate) {
    const double turns = hz / (double)sample_rate;
    const double frac = turns - std::floor(turns);  // [0, 1)
    return (uint32_t)(uint64_t)std::llround(frac * 4294967296.0);  // 2^32 wraps to 0 through the cast
}

// e^{-j 2 pi ph / 2^32} = hi[ph >> 22] * lo[(ph >> 12) & 1023]: hi[a] = e^{-j 2 pi a / 2^10}, lo[b] =
// e^{-j 2 pi b / 2^20}, each computed in double and rounded to float; interleaved {re, im}, hi then lo
void nco_tables(float *tab) {
    for (int a = 0; a < 1024; a++) {
        const double t = 2.0 * M_PI * (double)a / 1024.0;
        tab[2 * a] = (float)std::cos(t);
        tab[2 * a + 1] = (float)-std::sin(t);
    }
    for (int b = 0; b < 1024; b++) {
        const double t = 2.0 * M_PI * (double)b / 1048576.0;
        tab[2048 + 2 * b] = (float)std::cos(t);
        tab[2048 + 2 * b + 1] = (float)-std::sin(t);
    }
}

}  // namespace sdrg

/*
 * sdrg_oracle.c — TEST INFRASTRUCTURE ONLY.  CPU restatement of the reference hot path, used as the
 * parity checker by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.  The product
 * (libsdrg.so) never links, loads or calls this file.
 *
 * Restates, line by line and with the same float operation order (built with gcc -O2, no FMA
 * contraction, the reference's own x86-64 flags):
 *   - IQ unpack                 : convertIQ (src/ssb/ssb_demod_opt.cpp:33-44) + the CS8/CS16 conventions
 *                                 of include/sdrg.h (the Soapy driver conversions are not in the tree)
 *   - FFTProcessor::process     : src/dsp/fft_process.cpp:42-105 (FFT, |X|^2, fftshift)
 *   - evaluateSignalStrength    : src/dsp/fft_process.cpp:122-379 (focus window, reference windows,
 *                                 OS-CFAR stats, frequency tracking with an injected clock, detection)
 *   - processSSB_opt + stages   : src/ssb/ssb_demod_opt.cpp:49-296 with the function statics made an
 *                                 explicit per-stream state struct
 *
 * Pinning (see DESIGN.md "Oracle"): the SSB restatement is checked bit-for-bit against the reference's
 * own ssb_demod_opt.cpp compiled from /root/reference (oracle/_ref, tests/golden fixtures).  The FFT is
 * checked against numpy's float64 DFT (FFTW's published algorithm is the DFT; the vendored FFTW is a
 * prebuilt archive that may not be linked).  evaluateSignalStrength cannot be built from the reference
 * here (fft_process.cpp needs jni.h through sdr-bridge-internal.h and an FFTW library), so its
 * arithmetic is pinned only through the window geometry the survey measured on the reference
 *  and through analytic cases: parity of the stats arithmetic is PARTIALLY UNPINNED.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/sdrg.h"

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

#define ORACLE_API __attribute__((visibility("default")))

/* ------------------------------------------------------------------------------------------------
 * IQ unpack
 * ---------------------------------------------------------------------------------------------- */
ORACLE_API int oracle_unpack(int fmt, const void *src, int64_t n, float *iq) {
    if (!src || !iq || n < 0) return -1;
    switch (fmt) {
    case SDRG_IQ_CF32:
        memcpy(iq, src, (size_t)n * 2 * sizeof(float));
        return 0;
    case SDRG_IQ_CS8: {
        const int8_t *b = (const int8_t *)src;
        for (int64_t i = 0; i < 2 * n; i++) iq[i] = (float)b[i] * (1.0f / 128.0f);
        return 0;
    }
    case SDRG_IQ_CU8: {
        /* ssb_demod_opt.cpp:37-43: (buffer[k] - offset) * scale, offset 127.4f, scale 1/128 */
        const uint8_t *b = (const uint8_t *)src;
        const float offset = 127.4f, scale = 1.0f / 128.0f;
        for (int64_t i = 0; i < 2 * n; i++) iq[i] = ((float)b[i] - offset) * scale;
        return 0;
    }
    case SDRG_IQ_CS16: {
        const int16_t *b = (const int16_t *)src;
        for (int64_t i = 0; i < 2 * n; i++) iq[i] = (float)b[i] * (1.0f / 32768.0f);
        return 0;
    }
    default:
        return -2;
    }
}

/* ------------------------------------------------------------------------------------------------
 * FFT.  fft_process.cpp:77-79 runs fftwf_plan_dft_1d(N, FORWARD, ESTIMATE): X[k] = sum x[n] e^{-2 pi i kn/N},
 * unnormalised, no window.  Restated as an iterative radix-2 DIT transform (power-of-two N) in float
 * with twiddles rounded from double (the CPU-baseline arithmetic, same class as scalar FFTW), or in
 * double (the accuracy reference).
 * ---------------------------------------------------------------------------------------------- */
static int is_pow2(int n) { return n > 0 && (n & (n - 1)) == 0; }

static void bitrev_permute_f(float *re, float *im, int n) {
    for (int i = 1, j = 0; i < n; i++) {
        int bit = n >> 1;
        for (; j & bit; bit >>= 1) j ^= bit;
        j ^= bit;
        if (i < j) {
            float t = re[i]; re[i] = re[j]; re[j] = t;
            t = im[i]; im[i] = im[j]; im[j] = t;
        }
    }
}

static void bitrev_permute_d(double *re, double *im, int n) {
    for (int i = 1, j = 0; i < n; i++) {
        int bit = n >> 1;
        for (; j & bit; bit >>= 1) j ^= bit;
        j ^= bit;
        if (i < j) {
            double t = re[i]; re[i] = re[j]; re[j] = t;
            t = im[i]; im[i] = im[j]; im[j] = t;
        }
    }
}

/* Twiddle tables are cached per size (float and double). */
typedef struct { int n; float *c, *s; double *cd, *sd; } tw_cache;
static __thread tw_cache g_tw = {0, 0, 0, 0, 0};

static int ensure_twiddles(int n) {
    if (g_tw.n == n) return 0;
    free(g_tw.c); free(g_tw.s); free(g_tw.cd); free(g_tw.sd);
    g_tw.c = (float *)malloc(sizeof(float) * (size_t)(n / 2 + 1));
    g_tw.s = (float *)malloc(sizeof(float) * (size_t)(n / 2 + 1));
    g_tw.cd = (double *)malloc(sizeof(double) * (size_t)(n / 2 + 1));
    g_tw.sd = (double *)malloc(sizeof(double) * (size_t)(n / 2 + 1));
    if (!g_tw.c || !g_tw.s || !g_tw.cd || !g_tw.sd) { g_tw.n = 0; return -1; }
    for (int k = 0; k <= n / 2; k++) {
        double a = -2.0 * M_PI * (double)k / (double)n;
        g_tw.cd[k] = cos(a);
        g_tw.sd[k] = sin(a);
        g_tw.c[k] = (float)g_tw.cd[k];
        g_tw.s[k] = (float)g_tw.sd[k];
    }
    g_tw.n = n;
    return 0;
}

/* In-place forward DFT of (re, im), length n (power of two). */
ORACLE_API int oracle_fft_f32(float *re, float *im, int n) {
    if (!is_pow2(n)) return -2;
    if (ensure_twiddles(n)) return -3;
    bitrev_permute_f(re, im, n);
    for (int len = 2; len <= n; len <<= 1) {
        const int half = len >> 1, step = n / len;
        for (int base = 0; base < n; base += len) {
            for (int k = 0; k < half; k++) {
                const float wr = g_tw.c[k * step], wi = g_tw.s[k * step];
                const int a = base + k, b = a + half;
                const float tr = re[b] * wr - im[b] * wi;
                const float ti = re[b] * wi + im[b] * wr;
                re[b] = re[a] - tr; im[b] = im[a] - ti;
                re[a] = re[a] + tr; im[a] = im[a] + ti;
            }
        }
    }
    return 0;
}

ORACLE_API int oracle_fft_f64(double *re, double *im, int n) {
    if (!is_pow2(n)) return -2;
    if (ensure_twiddles(n)) return -3;
    bitrev_permute_d(re, im, n);
    for (int len = 2; len <= n; len <<= 1) {
        const int half = len >> 1, step = n / len;
        for (int base = 0; base < n; base += len) {
            for (int k = 0; k < half; k++) {
                const double wr = g_tw.cd[k * step], wi = g_tw.sd[k * step];
                const int a = base + k, b = a + half;
                const double tr = re[b] * wr - im[b] * wi;
                const double ti = re[b] * wi + im[b] * wr;
                re[b] = re[a] - tr; im[b] = im[a] - ti;
                re[a] = re[a] + tr; im[a] = im[a] + ti;
            }
        }
    }
    return 0;
}

/* Forward DFT in double for ANY n >= 1 (FFTW plans every size, fft_process.cpp:77-79): the radix-2 transform above
 * for powers of two; otherwise Bluestein's chirp-z over the power of two M >= 2n - 1, X_k = conj(b_k) sum_j
 * (x_j conj(b_j)) b_(k-j) with b_m = exp(i pi m^2 / n) (m^2 reduced mod 2n exactly), the convolution done with
 * three double FFTs.  Relative error ~1e-15 of the frame's energy: an accuracy reference, like the pow-2 path. */
ORACLE_API int oracle_dft_f64_any(double *re, double *im, int n) {
    if (n < 1) return -1;
    if (is_pow2(n)) return oracle_fft_f64(re, im, n);
    int m = 1;
    while (m < 2 * n - 1) m <<= 1;
    double *br = (double *)malloc(sizeof(double) * (size_t)n), *bi = (double *)malloc(sizeof(double) * (size_t)n);
    double *ar = (double *)calloc((size_t)m, sizeof(double)), *ai = (double *)calloc((size_t)m, sizeof(double));
    double *cr = (double *)calloc((size_t)m, sizeof(double)), *ci = (double *)calloc((size_t)m, sizeof(double));
    if (!br || !bi || !ar || !ai || !cr || !ci) {
        free(br); free(bi); free(ar); free(ai); free(cr); free(ci);
        return -3;
    }
    for (int64_t k = 0; k < n; k++) {
        const int64_t q = (k * k) % (2 * (int64_t)n);
        const double t = M_PI * (double)q / (double)n;
        br[k] = cos(t);
        bi[k] = sin(t);
    }
    for (int k = 0; k < n; k++) {  /* a = x conj(b) */
        ar[k] = re[k] * br[k] + im[k] * bi[k];
        ai[k] = im[k] * br[k] - re[k] * bi[k];
    }
    cr[0] = br[0];
    ci[0] = bi[0];
    for (int k = 1; k < n; k++) {
        cr[k] = cr[m - k] = br[k];
        ci[k] = ci[m - k] = bi[k];
    }
    oracle_fft_f64(ar, ai, m);
    oracle_fft_f64(cr, ci, m);
    for (int k = 0; k < m; k++) {  /* conj(A C) for the inverse through a forward transform */
        const double pr = ar[k] * cr[k] - ai[k] * ci[k], pi = ar[k] * ci[k] + ai[k] * cr[k];
        ar[k] = pr;
        ai[k] = -pi;
    }
    oracle_fft_f64(ar, ai, m);
    for (int k = 0; k < n; k++) {  /* X_k = conj(b_k) conj(.)/m */
        const double zr = ar[k] / m, zi = -ai[k] / m;
        re[k] = zr * br[k] + zi * bi[k];
        im[k] = zi * br[k] - zr * bi[k];
    }
    free(br); free(bi); free(ar); free(ai); free(cr); free(ci);
    return 0;
}

/* fft_process.cpp:77-97: FFT of the CF32 frame, power[i] = re*re + im*im (float), then fftshift.
 * use_f64 != 0 computes the transform in double and rounds X to float before the power. */
ORACLE_API int oracle_power_shifted(const float *iq, int n, int use_f64, float *out_shifted) {
    if (!iq || !out_shifted || n < 1) return -1;
    float *power = (float *)malloc(sizeof(float) * (size_t)n);
    if (!power) return -3;
    if (use_f64 || !is_pow2(n)) {  /* sizes the float radix-2 restatement does not cover: the double DFT */
        double *re = (double *)malloc(sizeof(double) * (size_t)n), *im = (double *)malloc(sizeof(double) * (size_t)n);
        if (!re || !im) { free(re); free(im); free(power); return -3; }
        for (int i = 0; i < n; i++) { re[i] = iq[2 * i]; im[i] = iq[2 * i + 1]; }
        oracle_dft_f64_any(re, im, n);
        for (int i = 0; i < n; i++) {
            const float xr = (float)re[i], xi = (float)im[i];
            power[i] = xr * xr + xi * xi;
        }
        free(re); free(im);
    } else {
        float *re = (float *)malloc(sizeof(float) * (size_t)n), *im = (float *)malloc(sizeof(float) * (size_t)n);
        if (!re || !im) { free(re); free(im); free(power); return -3; }
        for (int i = 0; i < n; i++) { re[i] = iq[2 * i]; im[i] = iq[2 * i + 1]; }
        oracle_fft_f32(re, im, n);
        for (int i = 0; i < n; i++) power[i] = re[i] * re[i] + im[i] * im[i];   /* :83-86 */
        free(re); free(im);
    }
    /* :92-97; for odd n the loop leaves out_shifted[n-1] as it was (the reference's vector keeps its old value)
     * and drops power[n-1] */
    const int half = n / 2;
    for (int i = 0; i < half; i++) {
        out_shifted[i] = power[i + half];
        out_shifted[i + half] = power[i];
    }
    free(power);
    return 0;
}

/* ------------------------------------------------------------------------------------------------
 * evaluateSignalStrength (fft_process.cpp:122-379) with FFTProcessor's members as explicit state.
 * ---------------------------------------------------------------------------------------------- */
typedef struct oracle_fft_state {
    /* FftProcessorConfig (fft_process.h:20-26) */
    uint32_t center_frequency;
    uint32_t sample_rate;
    int32_t samples_per_reading;
    int32_t freq_focus_range_khz;
    /* frequency tracking (fft_process.h:68-72) */
    float tracking_frequency;
    float max_peak_db, max_peak_freq;   /* maxPeakAndFrequency */
    int32_t max_peak_set;               /* !maxPeakAndFrequency.empty() */
    int64_t time_last_max_peak_ms, time_last_update_ms;
    int32_t center_frequency_changed;   /* sdr_bridge_internal::isCenterFrequencyChanged */
    /* detection (fft_process.h:77-86) */
    int32_t peak_confirmed;
    int32_t det_buf[3];
    int32_t det_idx;
    /* outputs (fft_process.h:88-109) — they persist across frames (stale semantics) */
    int32_t detection_flag_sent;
    float mean_snr_db, mean_snr_sigma, peak_above_noise_mean_db, max_bin_snr_db, max_bin_snr_sigma;
    float best1khz_snr_db, best1khz_snr_sigma, best1khz_center_freq_hz, per_bin_mean;
} oracle_fft_state;

ORACLE_API int oracle_fft_state_size(void) { return (int)sizeof(oracle_fft_state); }

/* FFTProcessor() + configure() (fft_process.cpp:8-39). */
ORACLE_API void oracle_fft_state_init(oracle_fft_state *s) { memset(s, 0, sizeof(*s)); }

ORACLE_API void oracle_fft_configure(oracle_fft_state *s, uint32_t center_frequency, uint32_t sample_rate,
                                     int32_t samples_per_reading, int32_t focus_khz) {
    s->center_frequency = center_frequency;
    s->sample_rate = sample_rate;
    s->samples_per_reading = samples_per_reading;
    s->freq_focus_range_khz = focus_khz;
    if (!s->max_peak_set) {                    /* :33-35 */
        s->max_peak_db = -130.0f;
        s->max_peak_freq = (float)center_frequency;
        s->max_peak_set = 1;
    }
}

ORACLE_API void oracle_fft_set_center_frequency_changed(oracle_fft_state *s) { s->center_frequency_changed = 1; }

static int off_to_bin(float offset_hz, float nyquist, float freq_per_bin) {        /* :131-133 */
    return (int)((offset_hz + nyquist) / freq_per_bin);
}

static float best1k_mean(const float *P, int lo, int hi, int w) {                  /* :163-180 */
    const int len = hi - lo + 1;
    if (len <= 0) return 0.0f;
    if (len < w) {
        float s = 0.0f;
        for (int i = lo; i <= hi; i++) s += P[i];
        return s / len;
    }
    float run_sum = 0.0f;
    for (int i = lo; i < lo + w; i++) run_sum += P[i];
    float best = run_sum / w;
    for (int start = lo + 1; start + w - 1 <= hi; start++) {
        run_sum += P[start + w - 1] - P[start - 1];
        const float m = run_sum / w;
        if (m > best) best = m;
    }
    return best;
}

typedef struct { float mean_db, max_bin_db, best1k_db; int lo, hi; } ref_window;

static float fmax_ref(float a, float b) { return (a < b) ? b : a; }   /* std::max(a, b) */

static int cmp_float(const void *a, const void *b) {
    const float x = *(const float *)a, y = *(const float *)b;
    return (x < y) ? -1 : (x > y) ? 1 : 0;
}

/* Window geometry (focus window + reference windows), shared with the geometry tests. */
ORACLE_API int oracle_window_geometry(uint32_t sample_rate, int32_t samp_count, int32_t focus_khz,
                                      int32_t *focus_lo, int32_t *focus_hi, int32_t *win_bins_1k,
                                      int32_t *n_ref, int32_t *ref_lo_hi /* [20] */) {
    const float freq_per_bin = (float)sample_rate / (float)samp_count;
    const float X_hz = focus_khz * 1000.0f;
    const float nyquist = sample_rate / 2.0f;
    const int lo = off_to_bin(-X_hz, nyquist, freq_per_bin);
    const int hi = off_to_bin(+X_hz, nyquist, freq_per_bin) - 1;
    *focus_lo = lo > 0 ? lo : 0;
    *focus_hi = hi < samp_count - 1 ? hi : samp_count - 1;
    const int w = (int)ceilf(1000.0f / freq_per_bin);
    *win_bins_1k = w > 1 ? w : 1;
    int nr = 0;
    for (int k = 1; k <= 5; k++) {                                                  /* :190-216 */
        const float nearX = (4 * k - 2) * X_hz;
        const float farX = 4 * k * X_hz;
        if (farX >= nyquist) break;
        int l0 = off_to_bin(+nearX, nyquist, freq_per_bin), h0 = off_to_bin(+farX, nyquist, freq_per_bin) - 1;
        l0 = l0 > 0 ? l0 : 0; h0 = h0 < samp_count - 1 ? h0 : samp_count - 1;
        if (h0 > l0) { ref_lo_hi[2 * nr] = l0; ref_lo_hi[2 * nr + 1] = h0; nr++; }
        int l1 = off_to_bin(-farX, nyquist, freq_per_bin), h1 = off_to_bin(-nearX, nyquist, freq_per_bin) - 1;
        l1 = l1 > 0 ? l1 : 0; h1 = h1 < samp_count - 1 ? h1 : samp_count - 1;
        if (h1 > l1) { ref_lo_hi[2 * nr] = l1; ref_lo_hi[2 * nr + 1] = h1; nr++; }
    }
    *n_ref = nr;
    return 0;
}

/* evaluateSignalStrength(sampCount, power_shifted, sampleRate, centerFrequency), now_ms = steady clock. */
ORACLE_API int oracle_signal_strength(oracle_fft_state *st, const float *P, int32_t samp_count, int64_t now_ms,
                                      sdrg_frame_record *rec) {
    const uint32_t sample_rate = st->sample_rate, center_frequency = st->center_frequency;
    const float ref_power = 1.0f;                                                  /* fft_process.h:74-75 */
    const float freq_per_bin = (float)sample_rate / (float)samp_count;             /* :124 */
    const float X_hz = st->freq_focus_range_khz * 1000.0f;
    const float nyquist = sample_rate / 2.0f;

    int focus_lo = off_to_bin(-X_hz, nyquist, freq_per_bin);                        /* :136-138 */
    if (focus_lo < 0) focus_lo = 0;
    int focus_hi = off_to_bin(+X_hz, nyquist, freq_per_bin) - 1;
    if (focus_hi > samp_count - 1) focus_hi = samp_count - 1;
    const int focus_len = focus_hi - focus_lo + 1;
    if (rec) {
        rec->peak_bin = -1; rec->abs_peak_db = -130.0f; rec->signal_power_db = 0.0f;
        rec->valid = 0; rec->n_ref_windows = 0;
    }
    if (focus_len <= 0) goto fill_record;                                           /* :139 */

    {
        float abs_peak_db = -130.0f;                                                /* :142-154 */
        int peak_bin_in_focus = 0;
        float signal_power_sum = 0.0f;
        for (int i = focus_lo; i <= focus_hi; i++) {
            const float p = P[i];
            signal_power_sum += p;
            const float dB = 10.0f * log10f(p / ref_power + 1e-20f);
            if (dB > abs_peak_db) { abs_peak_db = dB; peak_bin_in_focus = i - focus_lo; }
        }
        const float signal_power_db = 10.0f * log10f((signal_power_sum / focus_len) / ref_power + 1e-20f);

        const int w1k0 = (int)ceilf(1000.0f / freq_per_bin);                       /* :160 */
        const int win_bins_1k = w1k0 > 1 ? w1k0 : 1;

        ref_window win[10];
        int n_ref = 0;
        for (int k = 1; k <= 5; k++) {                                              /* :191-216 */
            const float nearX = (4 * k - 2) * X_hz;
            const float farX = 4 * k * X_hz;
            if (farX >= nyquist) break;
            for (int side = 0; side < 2; side++) {
                int lo, hi;
                if (side == 0) {
                    lo = off_to_bin(+nearX, nyquist, freq_per_bin);
                    hi = off_to_bin(+farX, nyquist, freq_per_bin) - 1;
                } else {
                    lo = off_to_bin(-farX, nyquist, freq_per_bin);
                    hi = off_to_bin(-nearX, nyquist, freq_per_bin) - 1;
                }
                if (lo < 0) lo = 0;
                if (hi > samp_count - 1) hi = samp_count - 1;
                if (hi <= lo) continue;                                             /* collectWindow :197 */
                const int n = hi - lo + 1;
                float sum = 0.0f, maxP = 0.0f;
                for (int i = lo; i <= hi; i++) {
                    sum += P[i];
                    if (P[i] > maxP) maxP = P[i];
                }
                win[n_ref].mean_db = 10.0f * log10f((sum / n) / ref_power + 1e-20f);
                win[n_ref].max_bin_db = 10.0f * log10f(maxP / ref_power + 1e-20f);
                win[n_ref].best1k_db = 10.0f * log10f(best1k_mean(P, lo, hi, win_bins_1k) / ref_power + 1e-20f);
                win[n_ref].lo = lo;
                win[n_ref].hi = hi;
                n_ref++;
            }
        }

        const int valid = (n_ref >= 2);                                             /* :218-225 */
        if (rec) {
            rec->peak_bin = focus_lo + peak_bin_in_focus;
            rec->abs_peak_db = abs_peak_db;
            rec->signal_power_db = signal_power_db;
            rec->valid = valid;
            rec->n_ref_windows = n_ref;
        }
        if (!valid) {
            st->mean_snr_db = st->mean_snr_sigma = 0.0f;
            st->peak_above_noise_mean_db = st->max_bin_snr_db = st->max_bin_snr_sigma = 0.0f;
            st->best1khz_snr_db = st->best1khz_snr_sigma = 0.0f;
        } else {
            /* std::sort by meanDb; libstdc++ sorts <=16 elements by (stable) insertion sort */
            for (int i = 1; i < n_ref; i++) {
                ref_window v = win[i];
                int j = i;
                while (j > 0 && v.mean_db < win[j - 1].mean_db) { win[j] = win[j - 1]; j--; }
                win[j] = v;
            }
            const int nb0 = (int)(n_ref * 0.4f);                                    /* :232 */
            const int n_bottom = nb0 > 1 ? nb0 : 1;

            {   /* 6.4a :235-247 */
                float mean = 0.0f;
                for (int i = 0; i < n_bottom; i++) mean += win[i].mean_db;
                mean /= n_bottom;
                float gaps[10];
                for (int i = 0; i < n_bottom; i++) gaps[i] = fabsf(win[i].mean_db - mean);
                qsort(gaps, (size_t)n_bottom, sizeof(float), cmp_float);
                const float sigma = fmax_ref(1.4816f * gaps[n_bottom / 2], 0.5f);
                const float snr_db = signal_power_db - mean;
                st->mean_snr_db = snr_db;
                st->mean_snr_sigma = snr_db / sigma;
            }

            /* 6.4b :252-269 */
            size_t n_pool = 0;
            for (int j = 0; j < n_bottom; j++) n_pool += (size_t)(win[j].hi - win[j].lo + 1);
            float *pooled = (float *)malloc(sizeof(float) * (n_pool ? n_pool : 1));
            float *gaps = (float *)malloc(sizeof(float) * (n_pool ? n_pool : 1));
            if (!pooled || !gaps) { free(pooled); free(gaps); return -3; }
            size_t q = 0;
            for (int j = 0; j < n_bottom; j++)
                for (int i = win[j].lo; i <= win[j].hi; i++) pooled[q++] = 10.0f * log10f(P[i] / ref_power + 1e-20f);
            float sigma_bin = 1.0f;
            float per_bin_mean = 0.0f;
            if (n_pool > 0) {
                for (size_t i = 0; i < n_pool; i++) per_bin_mean += pooled[i];
                per_bin_mean /= (float)n_pool;
                st->per_bin_mean = per_bin_mean;
                for (size_t i = 0; i < n_pool; i++) gaps[i] = fabsf(pooled[i] - per_bin_mean);
                qsort(gaps, n_pool, sizeof(float), cmp_float);
                sigma_bin = fmax_ref(1.4816f * gaps[n_pool / 2], 1.0f);
            }
            free(pooled); free(gaps);

            st->peak_above_noise_mean_db = abs_peak_db - per_bin_mean;              /* :274 */

            {   /* 6.4c :281-288 */
                const float logN = logf((float)focus_len);
                const float sqrt2logN = sqrtf(2.0f * logN);
                const float gumbel_loc = per_bin_mean + sigma_bin * sqrt2logN;
                const float gumbel_sig = fmax_ref(sigma_bin * 3.14159f / (sqrtf(6.0f) * sqrt2logN), 0.5f);
                st->max_bin_snr_db = abs_peak_db - gumbel_loc;
                st->max_bin_snr_sigma = st->max_bin_snr_db / gumbel_sig;
            }

            {   /* 6.4d :292-327 */
                float mean1k = 0.0f;
                for (int i = 0; i < n_bottom; i++) mean1k += win[i].best1k_db;
                mean1k /= n_bottom;
                float g1k[10];
                for (int i = 0; i < n_bottom; i++) g1k[i] = fabsf(win[i].best1k_db - mean1k);
                qsort(g1k, (size_t)n_bottom, sizeof(float), cmp_float);
                const float sigma_floor_1k = sigma_bin / sqrtf((float)win_bins_1k);
                /* std::max({a, b, c}) = first largest */
                float sigma1k = 1.4816f * g1k[n_bottom / 2];
                if (sigma1k < sigma_floor_1k) sigma1k = sigma_floor_1k;
                if (sigma1k < 0.5f) sigma1k = 0.5f;

                const float focus_best1k_linear = best1k_mean(P, focus_lo, focus_hi, win_bins_1k);
                if (focus_best1k_linear > 0.0f) {
                    const float focus_best1k_db = 10.0f * log10f(focus_best1k_linear / ref_power + 1e-20f);
                    st->best1khz_snr_db = focus_best1k_db - mean1k;
                    st->best1khz_snr_sigma = st->best1khz_snr_db / sigma1k;
                    const int len = focus_hi - focus_lo + 1;
                    int best_start = focus_lo;
                    if (len >= win_bins_1k) {
                        float rs = 0.f;
                        for (int i = focus_lo; i < focus_lo + win_bins_1k; i++) rs += P[i];
                        float bv = rs;
                        for (int s = focus_lo + 1; s + win_bins_1k - 1 <= focus_hi; s++) {
                            rs += P[s + win_bins_1k - 1] - P[s - 1];
                            if (rs > bv) { bv = rs; best_start = s; }
                        }
                    }
                    st->best1khz_center_freq_hz = (best_start + win_bins_1k / 2) * freq_per_bin
                                                  + ((float)center_frequency - nyquist);
                } else {
                    st->best1khz_snr_db = st->best1khz_snr_sigma = 0.0f;
                }
            }
        }

        /* 6.5 frequency tracking :333-361 */
        if (st->tracking_frequency == 0.0f) st->tracking_frequency = (float)center_frequency;
        if (st->center_frequency_changed) {
            st->tracking_frequency = (float)center_frequency;
            st->center_frequency_changed = 0;
        }
        if (!st->max_peak_set) {
            st->max_peak_db = -130.0f;
            st->max_peak_freq = (float)center_frequency;
            st->max_peak_set = 1;
        }
        if (valid && abs_peak_db > st->max_peak_db) {
            st->max_peak_db = abs_peak_db;
            st->max_peak_freq = (float)((focus_lo + peak_bin_in_focus) * freq_per_bin
                                        + ((float)center_frequency - nyquist));
            st->time_last_max_peak_ms = now_ms;
        }
        {
            const int64_t ms_since_peak = now_ms - st->time_last_max_peak_ms;
            if (st->time_last_update_ms < st->time_last_max_peak_ms && ms_since_peak > 300) {
                st->tracking_frequency = st->max_peak_freq;
                st->time_last_update_ms = now_ms;
                st->max_peak_db = -130.0f;
            }
        }

        /* 6.6 detection :365-378 */
        const int above = valid && (st->mean_snr_sigma >= 4.0f);
        if (above) {
            if (st->peak_confirmed < 1) st->peak_confirmed++;
        } else {
            st->peak_confirmed = 0;
        }
        const int current_flag = (above && st->peak_confirmed >= 1) ? 3 : 0;
        st->det_buf[st->det_idx] = current_flag;
        st->det_idx = (st->det_idx + 1) % 3;
        int m = st->det_buf[0];
        for (int i = 1; i < 3; i++) if (st->det_buf[i] > m) m = st->det_buf[i];
        st->detection_flag_sent = m;
    }

fill_record:
    if (rec) {
        rec->tracking_frequency = (int64_t)roundf(st->tracking_frequency);         /* fft_process.h:41 */
        rec->mean_snr_db = st->mean_snr_db;
        rec->mean_snr_sigma = st->mean_snr_sigma;
        rec->peak_above_noise_mean_db = st->peak_above_noise_mean_db;
        rec->max_bin_snr_db = st->max_bin_snr_db;
        rec->max_bin_snr_sigma = st->max_bin_snr_sigma;
        rec->best1khz_snr_db = st->best1khz_snr_db;
        rec->best1khz_snr_sigma = st->best1khz_snr_sigma;
        rec->best1khz_center_freq_hz = st->best1khz_center_freq_hz;
        rec->per_bin_mean = st->per_bin_mean;
        rec->detection_flag = st->detection_flag_sent;
    }
    return 0;
}

/* FFTProcessor::process (fft_process.cpp:42-105) on a CF32 frame: spectrum + stats. */
ORACLE_API int oracle_fft_process(oracle_fft_state *st, const float *iq, int32_t n, int64_t now_ms, int use_f64,
                                  float *out_shifted, sdrg_frame_record *rec) {
    int rc = oracle_power_shifted(iq, n, use_f64, out_shifted);
    if (rc) return rc;
    return oracle_signal_strength(st, out_shifted, n, now_ms, rec);
}

/* ------------------------------------------------------------------------------------------------
 * SSB chain (ssb_demod_opt.cpp).  All float, same operation order, no contraction.
 * ---------------------------------------------------------------------------------------------- */
typedef struct oracle_ssb_state {
    int64_t samp_count;                 /* static size_t sampCount (:224), 0 = not yet frozen */
    /* mode globals (:17-28), persistent */
    float agc_target, agc_fast, agc_slow, gain, lowpass_bd, lowpass_q, transient_coeff;
    int32_t rf_init;                    /* static bool rfInit (:262) */
    float lpf[5], lpf_z1, lpf_z2;       /* static IIR2 rfFilter: a0 a1 a2 b1 b2, z1 z2 */
    int32_t eq_init;                    /* static bool eqInit (:277) */
    float hp[5], hp_z1, hp_z2;
    float bp[5], bp_z1, bp_z2;
    /* NCO/short-FIR variant (a build extension, include/sdrg.h sdrg_engine_set_ssb_variant; all 0 = the
     * reference chain) */
    int32_t nco_on, fir_taps;
    uint32_t nco_inc, nco_phase;
} oracle_ssb_state;

ORACLE_API int oracle_ssb_state_size(void) { return (int)sizeof(oracle_ssb_state); }

ORACLE_API void oracle_ssb_state_init(oracle_ssb_state *s) {
    memset(s, 0, sizeof(*s));
    s->agc_target = 0.35f;       /* :17-28 initial values */
    s->agc_fast = 0.006f;
    s->agc_slow = 0.00035f;
    s->gain = 0.5f;
    s->lowpass_bd = 3200.0f;
    s->lowpass_q = 0.9f;
    s->transient_coeff = 0.55f;
}

/* iir2InitLowpass (:60-73) -> {a0, a1, a2, b1, b2} */
ORACLE_API void oracle_iir2_lowpass(float fs, float fc, float Q, float *c) {
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

/* biquadInitHighpass (:148-164) */
ORACLE_API void oracle_biquad_highpass(float fs, float f0, float Q, float *c) {
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
    c[0] = b0 / a0; c[1] = b1 / a0; c[2] = b2 / a0;
    c[3] = a1 / a0; c[4] = a2 / a0;
}

/* biquadInitBandpass (:166-175) */
ORACLE_API void oracle_biquad_bandpass(float fs, float f0, float Q, float *c) {
    float w0 = 2.0f * M_PI * f0 / fs;
    float alpha = sinf(w0) / (2.0f * Q);
    float cosw0 = cosf(w0);
    float b0 = alpha, b1 = 0.0f, b2 = -alpha;
    float a0 = 1.0f + alpha, a1 = -2.0f * cosw0, a2 = 1.0f - alpha;
    c[0] = b0 / a0; c[1] = b1 / a0; c[2] = b2 / a0;
    c[3] = a1 / a0; c[4] = a2 / a0;
}

/* simpleFIRDecimate's tap design (:121-134) at length taps0 (0 = the reference's 255); returns the tap
 * count N (taps written to h[0..N)). */
ORACLE_API int oracle_fir_taps_n(int64_t in_size, int decim, float cutoff_rel, int taps0, float *h) {
    int N = taps0 > 0 ? taps0 : 255;
    if (N > (int)in_size) N = (int)in_size | 1;
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

ORACLE_API int oracle_fir_taps(int64_t in_size, int decim, float cutoff_rel, float *h) {
    return oracle_fir_taps_n(in_size, decim, cutoff_rel, 0, h);
}

/* ---- NCO variant (BUILD EXTENSION: no reference counterpart; include/sdrg.h) ----
 * A 32-bit phase accumulator; the phasor e^{-j 2 pi ph / 2^32} is the product of two table entries,
 * hi[ph >> 22] = e^{-j 2 pi a / 2^10} and lo[(ph >> 12) & 1023] = e^{-j 2 pi b / 2^20}, each evaluated in
 * double and rounded to float.  Written independently of design.cpp / ssb.hip from the sdrg.h contract. */
ORACLE_API uint32_t oracle_nco_increment(double hz, uint32_t sample_rate) {
    double turns = hz / (double)sample_rate;
    turns -= floor(turns);
    return (uint32_t)(uint64_t)llround(turns * 4294967296.0);
}

static float nco_hi[2048], nco_lo[2048];
static int nco_ready = 0;

static void nco_init(void) {
    if (nco_ready) return;
    for (int k = 0; k < 1024; k++) {
        double a = 2.0 * M_PI * (double)k / 1024.0, b = 2.0 * M_PI * (double)k / 1048576.0;
        nco_hi[2 * k] = (float)cos(a);
        nco_hi[2 * k + 1] = (float)(-sin(a));
        nco_lo[2 * k] = (float)cos(b);
        nco_lo[2 * k + 1] = (float)(-sin(b));
    }
    nco_ready = 1;
}

/* Re((xr + j xi) w(ph)) */
ORACLE_API float oracle_nco_mix(uint32_t ph, float xr, float xi) {
    nco_init();
    const float *h = nco_hi + 2 * (ph >> 22), *l = nco_lo + 2 * ((ph >> 12) & 1023u);
    float wr = h[0] * l[0] - h[1] * l[1];
    float wi = h[0] * l[1] + h[1] * l[0];
    return xr * wr - xi * wi;
}

/* Select the variant for this stream's chain (nco_hz 0 = no mixer; fir_taps 0 = 255); restarts the phase. */
ORACLE_API void oracle_ssb_set_variant(oracle_ssb_state *s, double nco_hz, uint32_t sample_rate, int fir_taps) {
    s->nco_on = nco_hz != 0.0;
    s->nco_inc = s->nco_on ? oracle_nco_increment(nco_hz, sample_rate) : 0u;
    s->nco_phase = 0u;
    s->fir_taps = fir_taps;
}

ORACLE_API int oracle_ssb_decim(uint32_t sample_rate) {                             /* :273 */
    int d = (int)(sample_rate / 48000.0f);
    return d > 1 ? d : 1;
}

ORACLE_API int oracle_ssb_pcm_len_n(int64_t samp_count, uint32_t sample_rate, int taps0) {
    int N = taps0 > 0 ? taps0 : 255;
    if (N > (int)samp_count) N = (int)samp_count | 1;
    const int decim = oracle_ssb_decim(sample_rate);
    if (samp_count < N) return 0;
    return (int)((samp_count - N) / decim + 1);
}

ORACLE_API int oracle_ssb_pcm_len(int64_t samp_count, uint32_t sample_rate) {
    return oracle_ssb_pcm_len_n(samp_count, sample_rate, 0);
}

static float clampf_ref(float v, float lo, float hi) { return (v < lo) ? lo : (hi < v) ? hi : v; }

/* Optional stage taps for stage-level parity: each non-NULL array receives the chain's values. */
typedef struct oracle_ssb_taps {
    float *dc_re;     /* after removeDC, real part      [samp_count] */
    float *lpf;       /* after iir2Process (re == im)   [samp_count] */
    float *agc;       /* after adaptiveAGC              [samp_count] */
    float *fir;       /* after simpleFIRDecimate        [pcm_len]    */
    float *eq;        /* after HP, BP, transientBoost   [pcm_len]    */
} oracle_ssb_taps;

/* processSSB_opt(iq, sampleRate, upperSideband, pcmOut, pulse, mode) (:221-296).
 * iq: CF32 frame of n samples.  pcm_out must hold oracle_ssb_pcm_len(frozen count, fs) samples. */
ORACLE_API int oracle_ssb_process(oracle_ssb_state *s, const float *iq, int64_t n, uint32_t sample_rate,
                                  int upper, int mode, int16_t *pcm_out, int32_t *pcm_len,
                                  const oracle_ssb_taps *taps) {
    if (s->samp_count == 0) s->samp_count = n;                                    /* :224 static init */
    const int64_t S = s->samp_count;                                               /* iq.resize(sampCount) */

    if (mode == 2) {                                                               /* :230-255 */
        s->agc_target = 0.45f; s->agc_fast = 0.008f; s->gain = 4.5f;
        s->lowpass_bd = 2200.0f; s->lowpass_q = 1.2f; s->transient_coeff = 0.7f;
    } else if (mode == 0) {
        s->agc_target = 0.45f; s->agc_fast = 0.008f; s->gain = 10.0f;
        s->lowpass_bd = 2200.0f; s->lowpass_q = 1.2f; s->transient_coeff = 0.7f;
    } else if (mode == 1) {
        s->agc_target = 0.35f; s->agc_fast = 0.006f; s->agc_slow = 0.00035f; s->gain = 0.5f;
        s->lowpass_bd = 3200.0f; s->lowpass_q = 0.9f; s->transient_coeff = 0.55f;
    }

    float *audio = (float *)malloc(sizeof(float) * (size_t)(S > 0 ? S : 1));
    if (!audio) return -3;

    if (!s->rf_init) {                                                             /* :262-263 */
        oracle_iir2_lowpass((float)sample_rate, s->lowpass_bd, s->lowpass_q, s->lpf);
        s->lpf_z1 = s->lpf_z2 = 0.0f;
        s->rf_init = 1;
    }

    /* removeDC(iq, 0.9995f) (:49-55) — the imaginary part never reaches the output (:75-84 reads re) */
    {
        const float alpha = 0.9995f;
        const float one_minus = 1.0f - alpha;
        float dc = 0.0f;
        const float a0 = s->lpf[0], a1 = s->lpf[1], a2 = s->lpf[2], b1 = s->lpf[3], b2 = s->lpf[4];
        float z1 = s->lpf_z1, z2 = s->lpf_z2;
        for (int64_t i = 0; i < S; i++) {
            float re = (i < n) ? iq[2 * i] : 0.0f;
            /* variant: the NCO mixer on the present samples; the iq.resize() padding stays 0 */
            if (s->nco_on) re = (i < n) ? oracle_nco_mix(s->nco_phase + s->nco_inc * (uint32_t)i, iq[2 * i], iq[2 * i + 1]) : 0.0f;
            dc = alpha * dc + one_minus * re;
            const float x = re - dc;
            if (taps && taps->dc_re) taps->dc_re[i] = x;
            /* iir2Process (:75-84) */
            const float y = a0 * x + a1 * z1 + a2 * z2 - b1 * z1 - b2 * z2;
            z2 = z1; z1 = y;
            if (taps && taps->lpf) taps->lpf[i] = y;
            /* demodSSB (:89-96): iq[i] = {y, y} */
            audio[i] = upper ? (y + y) : (y - y);
        }
        s->lpf_z1 = z1; s->lpf_z2 = z2;
    }

    /* adaptiveAGC(audio, target, fast, 0.00035f) (:101-115) */
    {
        const float target = s->agc_target, fast = s->agc_fast, slow = 0.00035f;
        float gain = 1.0f;
        for (int64_t i = 0; i < S; i++) {
            const float x = audio[i];
            const float mag = fabsf(x) + 1e-8f;
            const float desired = target / (sqrtf(mag) + 1e-6f);
            const float rate = (desired < gain) ? fast : slow;
            gain = gain * (1.0f - rate) + desired * rate;
            audio[i] = clampf_ref(x * gain, -1.0f, 1.0f);
        }
        if (taps && taps->agc) memcpy(taps->agc, audio, sizeof(float) * (size_t)S);
    }

    /* simpleFIRDecimate(audio, decim, 0.45f) (:121-143) */
    const int decim = oracle_ssb_decim(sample_rate);
    float h[256];
    const int N = oracle_fir_taps_n(S, decim, 0.45f, s->fir_taps, h);
    int n_out = 0;
    float *out48 = (float *)malloc(sizeof(float) * (size_t)(S / decim + 4));
    if (!out48) { free(audio); return -3; }
    for (int64_t i = 0; i + N <= S; i += decim) {
        float acc = 0.0f;
        for (int k = 0; k < N; k++) acc += audio[i + k] * h[k];
        out48[n_out++] = acc;
    }
    if (taps && taps->fir) memcpy(taps->fir, out48, sizeof(float) * (size_t)n_out);

    if (!s->eq_init) {                                                             /* :277-282 */
        oracle_biquad_highpass(48000.0f, 1200.0f, 0.7f, s->hp);
        oracle_biquad_bandpass(48000.0f, 2400.0f, 0.6f, s->bp);
        s->hp_z1 = s->hp_z2 = s->bp_z1 = s->bp_z2 = 0.0f;
        s->eq_init = 1;
    }
    if (n_out > 0) {                                                               /* :283-289 */
        float z1 = s->hp_z1, z2 = s->hp_z2;
        for (int i = 0; i < n_out; i++) {                                          /* biquadProcess :177-186 */
            const float in = out48[i];
            const float y = s->hp[0] * in + s->hp[1] * z1 + s->hp[2] * z2 - s->hp[3] * z1 - s->hp[4] * z2;
            z2 = z1; z1 = y;
            out48[i] = y;
        }
        s->hp_z1 = z1; s->hp_z2 = z2;
        z1 = s->bp_z1; z2 = s->bp_z2;
        for (int i = 0; i < n_out; i++) {
            const float in = out48[i];
            const float y = s->bp[0] * in + s->bp[1] * z1 + s->bp[2] * z2 - s->bp[3] * z1 - s->bp[4] * z2;
            z2 = z1; z1 = y;
            out48[i] = y;
        }
        s->bp_z1 = z1; s->bp_z2 = z2;
        float prev = 0.0f;                                                         /* transientBoost :191-198 */
        const float coeff = s->transient_coeff;
        for (int i = 0; i < n_out; i++) {
            const float diff = out48[i] - prev;
            prev = out48[i];
            out48[i] = out48[i] + coeff * diff;
        }
    }
    if (taps && taps->eq) memcpy(taps->eq, out48, sizeof(float) * (size_t)n_out);

    for (int i = 0; i < n_out; i++) {                                              /* floatToPCM :203-210 */
        const float v = clampf_ref(out48[i] * s->gain, -1.0f, 1.0f);
        pcm_out[i] = (int16_t)(v * 32767.0f);
    }
    *pcm_len = n_out;
    s->nco_phase += s->nco_inc * (uint32_t)S;
    free(out48);
    free(audio);
    return 0;
}

/* ------------------------------------------------------------------------------------------------
 * Whole-frame helper used by the CPU baseline: unpack + FFTProcessor::process + processSSB_opt.
 * ---------------------------------------------------------------------------------------------- */
ORACLE_API int oracle_frame(oracle_fft_state *fst, oracle_ssb_state *sst, const void *raw, int fmt, int32_t n,
                            int64_t now_ms, int stages, int mode, float *spectrum, sdrg_frame_record *rec,
                            int16_t *pcm, int32_t *pcm_len) {
    float *iq = (float *)malloc(sizeof(float) * 2 * (size_t)n);
    if (!iq) return -3;
    int rc = oracle_unpack(fmt, raw, n, iq);
    if (!rc && (stages & SDRG_STAGE_SPECTRUM)) {
        rc = oracle_power_shifted(iq, n, 0, spectrum);
        if (!rc && (stages & SDRG_STAGE_STATS)) rc = oracle_signal_strength(fst, spectrum, n, now_ms, rec);
    }
    if (!rc && (stages & SDRG_STAGE_SSB)) {
        rc = oracle_ssb_process(sst, iq, n, fst->sample_rate, 1, mode, pcm, pcm_len, NULL);
    }
    free(iq);
    return rc;
}

/* pulse_oracle.c */
typedef struct oracle_pulse oracle_pulse;
int oracle_pulse_config_default(int kind, sdrg_pulse_config *c);
oracle_pulse *oracle_pulse_create(int kind, const sdrg_pulse_config *cfg);
void oracle_pulse_destroy(oracle_pulse *p);
int oracle_pulse_spectral(oracle_pulse *p, const float *snr_sigma, const float *freq_hz, int n_frames,
                          sdrg_pulse_output *out);
int oracle_pulse_audio(oracle_pulse *p, const void *audio, int fmt, int n, sdrg_pulse_output *out);

/* Batched CPU baseline: frames [f0, f1) of a [n_frames][n] raw buffer, each an independent stream (with the
 * pulse detectors of soapyCallback / the SSB worker when stages has SDRG_STAGE_SPECTRAL_PULSE /
 * SDRG_STAGE_AUDIO_PULSE). */
ORACLE_API int oracle_run_streams(const void *raw, int fmt, int32_t n, int32_t f0, int32_t f1, uint32_t sample_rate,
                                  uint32_t center_frequency, int32_t focus_khz, int stages, int mode, float *spectrum_scratch,
                                  int16_t *pcm_scratch) {
    const size_t bps = (fmt == SDRG_IQ_CF32) ? 8 : (fmt == SDRG_IQ_CS16) ? 4 : 2;
    oracle_fft_state fst;
    oracle_ssb_state sst;
    sdrg_frame_record rec;
    int32_t pcm_len = 0;
    for (int32_t f = f0; f < f1; f++) {
        oracle_fft_state_init(&fst);
        oracle_fft_configure(&fst, center_frequency, sample_rate, n, focus_khz);
        oracle_ssb_state_init(&sst);
        int rc = oracle_frame(&fst, &sst, (const char *)raw + (size_t)f * (size_t)n * bps, fmt, n, 1000, stages, mode,
                              spectrum_scratch, &rec, pcm_scratch, &pcm_len);
        if (rc) return rc;
        if (stages & (SDRG_STAGE_SPECTRAL_PULSE | SDRG_STAGE_AUDIO_PULSE)) {
            sdrg_pulse_config pc;
            sdrg_pulse_output po;
            if (stages & SDRG_STAGE_SPECTRAL_PULSE) {
                oracle_pulse_config_default(SDRG_PULSE_SPECTRAL, &pc);
                pc.fs_energy = (float)sample_rate / (float)n;
                oracle_pulse *d = oracle_pulse_create(SDRG_PULSE_SPECTRAL, &pc);
                if (!d) return -3;
                oracle_pulse_spectral(d, &rec.best1khz_snr_sigma, &rec.best1khz_center_freq_hz, 1, &po);
                oracle_pulse_destroy(d);
            }
            if (stages & SDRG_STAGE_AUDIO_PULSE) {
                oracle_pulse_config_default(SDRG_PULSE_AUDIO, &pc);
                oracle_pulse *d = oracle_pulse_create(SDRG_PULSE_AUDIO, &pc);
                if (!d) return -3;
                oracle_pulse_audio(d, pcm_scratch, 0, pcm_len, &po);
                oracle_pulse_destroy(d);
            }
        }
    }
    return 0;
}

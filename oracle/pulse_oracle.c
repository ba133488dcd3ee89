/*
 * pulse_oracle.c — TEST INFRASTRUCTURE ONLY.  CPU restatement of the reference's two beacon pulse
 * detectors, used as the parity checker for the engine's pulse kernels (csrc/pulse.hip).  The product
 * (libsdrg.so) never links, loads or calls this file.
 *
 *   SpectralPulseDetector  src/dsp/spectral_pulse_detector.h:19-79, spectral_pulse_detector.cpp:1-196
 *   AudioPulseDetector     src/ssb/audio_pulse_detector.h:15-104,  audio_pulse_detector.cpp:1-256
 *
 * Both detectors share one state machine (energy buffer -> local-maximum ROIs -> rhythm / phase lock ->
 * live state); they differ in the ROI score (spectral: the value itself; audio: value / trailing noise
 * mean), the base-state thresholds and the audio front end (band-pass, RMS per energy frame, low-pass).
 * The reference's std::deque members become plain arrays with pop-front by memmove; every float
 * expression keeps the reference's operand order, and the frequency regression is done in double as in
 * spectral_pulse_detector.cpp:148-170.  Built with the reference's x86-64 flags (gcc -O2, no FMA).
 *
 * Pinning: tests/golden/pulse_*.npz hold outputs of the reference's own two .cpp files compiled from
 * /root/reference by `make -C oracle ref` (oracle/_ref/ref_pulse, driver oracle/ref_pulse_driver.cpp), and
 * tests/test_oracle.py checks this restatement against them bit for bit.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/sdrg.h"

#define ORACLE_API __attribute__((visibility("default")))

typedef struct {
    float b0, b1, b2, a1, a2, z1, z2;
} pulse_sos;

typedef struct {
    int kind;
    sdrg_pulse_config cfg;
    /* energy buffer eBuf_ / freqBuf_ with its time origin eBufT0_ */
    float *e, *f;
    int n, cap;
    float t0;
    /* ROIs (t, etat) and the spectral frequency history (t, f), oldest first */
    float *roi_t;
    int *roi_etat;
    int n_rois, roi_cap;
    float fh_t[30], fh_f[30];
    int n_fh;
    float t_last_roi;
    int last_scan_idx;
    /* phase lock */
    int locked;
    float t_target;
    float last3[3];
    int n_last3;
    float hist_dts[5];
    int hist_n[5];
    int n_hist;
    /* outputs */
    int live_etat;
    float last_snr;
    int last_level;
    /* audio front end */
    pulse_sos band[2], low;
    int frame_samples, frame_count;
    float frame_acc;
} oracle_pulse;

static const float k_pi = 3.14159265358979f; /* audio_pulse_detector.cpp:4 */

/* makeLP2 / makeHP2 (audio_pulse_detector.cpp:29-55): bilinear Butterworth sections in float */
static pulse_sos design_sos(float fs, float fc, int highpass) {
    const float Q = 0.7071f;
    const float K = tanf(k_pi * fc / fs);
    const float K2 = K * K;
    const float norm = K2 + K / Q + 1.f;
    pulse_sos s;
    if (highpass) {
        s.b0 = 1.f / norm;
        s.b1 = -2.f / norm;
        s.b2 = 1.f / norm;
    } else {
        s.b0 = K2 / norm;
        s.b1 = 2.f * K2 / norm;
        s.b2 = K2 / norm;
    }
    s.a1 = 2.f * (K2 - 1.f) / norm;
    s.a2 = (K2 - K / Q + 1.f) / norm;
    s.z1 = s.z2 = 0.f;
    return s;
}

/* applyChain (audio_pulse_detector.cpp:57-65): direct form II transposed */
static float sos_step(pulse_sos *s, float x) {
    const float y = s->b0 * x + s->z1;
    s->z1 = s->b1 * x - s->a1 * y + s->z2;
    s->z2 = s->b2 * x - s->a2 * y;
    return y;
}

ORACLE_API int oracle_pulse_config_default(int kind, sdrg_pulse_config *c) {
    memset(c, 0, sizeof(*c));
    c->z_default_s = 0.666f;
    c->t_target_init = 1.75f;
    c->dt_tol_s = 0.150f;
    c->dispersion_max = 1.3f;
    c->sum_n_max = 7;
    c->live_window_t = 4.0f;
    c->live_divisor = 3.0f;
    c->sample_rate = 48000.f;
    c->f_min = 1500.f;
    c->f_max = 4000.f;
    c->smooth_cutoff = 5.f;
    c->noise_ref_far = 80;
    c->noise_ref_near = 40;
    if (kind == SDRG_PULSE_SPECTRAL) { /* spectral_pulse_detector.h:23-35 */
        c->fs_energy = 20.f;
        c->snr_min = 1.5f;
        c->snr_rhythm = 2.5f;
        c->snr_strong = 4.0f;
    } else { /* audio_pulse_detector.h:19-37 */
        c->fs_energy = 100.f;
        c->snr_min = 1.0f;
        c->snr_rhythm = 1.1f;
        c->snr_strong = 2.0f;
    }
    return 0;
}

static int ensure_cap(oracle_pulse *p) {
    const int max_buf = (int)(10.f * p->cfg.fs_energy);
    const int want = (max_buf > 0 ? max_buf : 0) + 8;
    if (p->cap < want) {
        float *e = (float *)realloc(p->e, sizeof(float) * (size_t)want);
        if (!e) return -3;
        p->e = e;
        float *f = (float *)realloc(p->f, sizeof(float) * (size_t)want);
        if (!f) return -3;
        p->f = f;
        p->cap = want;
    }
    return 0;
}

static void clear_detector(oracle_pulse *p) {
    p->n = 0;
    p->t0 = 0.f;
    p->n_rois = 0;
    p->n_fh = 0;
    p->t_last_roi = -1.f;
    p->last_scan_idx = 0;
    p->locked = 0;
    p->t_target = p->cfg.t_target_init;
    p->n_last3 = 0;
    p->n_hist = 0;
    p->live_etat = 0;
    p->last_snr = 0.f;
    p->last_level = 0;
    p->frame_count = 0;
    p->frame_acc = 0.f;
    for (int k = 0; k < 2; k++) p->band[k].z1 = p->band[k].z2 = 0.f;
    p->low.z1 = p->low.z2 = 0.f;
}

static void setup_audio(oracle_pulse *p) {
    /* constructor (audio_pulse_detector.cpp:8-24) */
    p->band[0] = design_sos(p->cfg.sample_rate, p->cfg.f_min, 1);
    p->band[1] = design_sos(p->cfg.sample_rate, p->cfg.f_max, 0);
    p->low = design_sos(p->cfg.fs_energy, p->cfg.smooth_cutoff, 0);
    const int fsamp = (int)(p->cfg.sample_rate / p->cfg.fs_energy);
    p->frame_samples = fsamp > 1 ? fsamp : 1;
}

ORACLE_API oracle_pulse *oracle_pulse_create(int kind, const sdrg_pulse_config *cfg) {
    oracle_pulse *p = (oracle_pulse *)calloc(1, sizeof(oracle_pulse));
    if (!p) return NULL;
    p->kind = kind;
    p->cfg = *cfg;
    p->roi_cap = 64;
    p->roi_t = (float *)malloc(sizeof(float) * (size_t)p->roi_cap);
    p->roi_etat = (int *)malloc(sizeof(int) * (size_t)p->roi_cap);
    if (!p->roi_t || !p->roi_etat || ensure_cap(p)) return NULL;
    clear_detector(p);
    if (kind == SDRG_PULSE_AUDIO) setup_audio(p);
    return p;
}

ORACLE_API void oracle_pulse_destroy(oracle_pulse *p) {
    if (!p) return;
    free(p->e);
    free(p->f);
    free(p->roi_t);
    free(p->roi_etat);
    free(p);
}

/* SpectralPulseDetector::configure (spectral_pulse_detector.cpp:6-8): config only, state kept */
ORACLE_API int oracle_pulse_configure(oracle_pulse *p, const sdrg_pulse_config *cfg) {
    p->cfg = *cfg;
    return ensure_cap(p);
}

ORACLE_API void oracle_pulse_reset(oracle_pulse *p) { clear_detector(p); }

/* timeOfIdx (spectral :13-15, audio :69-71) */
static float time_of(const oracle_pulse *p, int i) { return p->t0 + (float)i / p->cfg.fs_energy; }

/* noiseRef (audio_pulse_detector.cpp:78-90): trailing mean over [i-far, i-near), -1 if not enough history */
static float noise_ref(const oracle_pulse *p, int i) {
    int lo = i - p->cfg.noise_ref_far, hi = i - p->cfg.noise_ref_near;
    if (hi <= 0 || lo >= hi) return -1.f;
    if (lo < 0) lo = 0;
    if (hi > p->n) hi = p->n;
    if (lo >= hi) return -1.f;
    float acc = 0.f;
    for (int j = lo; j < hi; j++) acc += p->e[j];
    return acc / (float)(hi - lo);
}

static void push_bounded_f(float *a, int *n, int cap, float v) {
    if (*n == cap) {
        memmove(a, a + 1, sizeof(float) * (size_t)(cap - 1));
        (*n)--;
    }
    a[(*n)++] = v;
}

static void push_bounded_i(int *a, int *n, int cap, int v) {
    if (*n == cap) {
        memmove(a, a + 1, sizeof(int) * (size_t)(cap - 1));
        (*n)--;
    }
    a[(*n)++] = v;
}

static int last3_spread_ok(const oracle_pulse *p) {
    if (p->n_last3 != 3) return 0;
    float mn = p->last3[0], mx = p->last3[0];
    for (int k = 1; k < 3; k++) {
        if (p->last3[k] < mn) mn = p->last3[k];
        if (mx < p->last3[k]) mx = p->last3[k];
    }
    return mx - mn < p->cfg.dt_tol_s;
}

/* detectRois (spectral :46-143, audio :132-237) */
static void detect_rois(oracle_pulse *p) {
    const sdrg_pulse_config *c = &p->cfg;
    const int audio = p->kind == SDRG_PULSE_AUDIO;
    const float z_s = p->locked ? 0.75f * p->t_target : c->z_default_s;
    int idx_z = (int)(z_s * c->fs_energy);
    if (idx_z < 1) idx_z = 1;
    const int safe = p->n - idx_z;
    if (safe <= idx_z) return;
    int i = p->last_scan_idx > idx_z ? p->last_scan_idx : idx_z;
    for (; i < safe; i++) {
        const float val = p->e[i];
        int is_max = 1;
        for (int j = i - idx_z; j <= i + idx_z && is_max; j++)
            if (j != i && p->e[j] >= val) is_max = 0;
        if (!is_max) continue;

        float snr = val;
        if (audio) {
            const float noise = noise_ref(p, i);
            if (noise <= 0.f) continue;
            snr = val / noise;
        }
        if (snr < c->snr_min) continue;

        const float t_roi = time_of(p, i);
        const float dt = (p->t_last_roi >= 0.f) ? t_roi - p->t_last_roi : 0.f;
        int n_cyc = 1;
        float norm_dt = dt;
        if (dt > 0.f) {
            n_cyc = (int)roundf(dt / p->t_target);
            if (n_cyc < 1) n_cyc = 1;
            if (n_cyc > 1 && fabsf(dt - (float)n_cyc * p->t_target) > c->dt_tol_s) n_cyc = 1;
            norm_dt = dt / (float)n_cyc;
        }
        const int in_rhythm = (dt > 0.f) && (fabsf(norm_dt - p->t_target) < c->dt_tol_s);
        if (!(snr >= c->snr_strong || (snr >= c->snr_rhythm && in_rhythm))) continue;

        if (dt > 0.f) {
            push_bounded_f(p->last3, &p->n_last3, 3, norm_dt);
            if (last3_spread_ok(p)) {
                p->locked = 1;
                p->t_target = (p->last3[0] + p->last3[1] + p->last3[2]) / 3.f;
            }
            int nh = p->n_hist;
            push_bounded_f(p->hist_dts, &nh, 5, norm_dt);
            nh = p->n_hist;
            push_bounded_i(p->hist_n, &nh, 5, n_cyc);
            p->n_hist = nh;
        }

        int base;
        if (audio) /* audio_pulse_detector.cpp:194-198: fixed thresholds */
            base = (snr >= 2.0f) ? 5 : (snr >= 1.5f) ? 4 : (snr >= 1.2f) ? 3 : (snr >= 1.1f) ? 2 : 1;
        else /* spectral_pulse_detector.cpp:106-110 */
            base = (snr >= c->snr_strong) ? 5 : (snr >= 3.0f) ? 4 : (snr >= c->snr_rhythm) ? 3 : (snr >= 2.0f) ? 2 : 1;
        const int pen_rhythm = (dt > 0.f && !in_rhythm) ? 2 : 0;
        int pen_conf = 0;
        if (p->n_hist >= 4) {
            float disp = 0.f;
            for (int j = 1; j < p->n_hist; j++) disp += fabsf(p->hist_dts[j] - p->hist_dts[j - 1]);
            int sum_n = 0;
            for (int j = 0; j < p->n_hist; j++) sum_n += p->hist_n[j];
            if (disp > c->dispersion_max || sum_n > c->sum_n_max) pen_conf = 2;
        }
        if (last3_spread_ok(p)) pen_conf = 0;
        int etat = base - pen_rhythm - pen_conf;
        if (etat < 0) etat = 0;

        if (p->n_rois == p->roi_cap) {
            p->roi_cap *= 2;
            p->roi_t = (float *)realloc(p->roi_t, sizeof(float) * (size_t)p->roi_cap);
            p->roi_etat = (int *)realloc(p->roi_etat, sizeof(int) * (size_t)p->roi_cap);
        }
        p->roi_t[p->n_rois] = t_roi;
        p->roi_etat[p->n_rois] = etat;
        p->n_rois++;
        p->t_last_roi = t_roi;
        p->last_snr = snr;
        if (!audio) { /* freqHistory_ (spectral :130-131) */
            if (p->n_fh == 30) {
                memmove(p->fh_t, p->fh_t + 1, sizeof(float) * 29);
                memmove(p->fh_f, p->fh_f + 1, sizeof(float) * 29);
                p->n_fh--;
            }
            p->fh_t[p->n_fh] = t_roi;
            p->fh_f[p->n_fh] = p->f[i];
            p->n_fh++;
        }
        const float cutoff = t_roi - 20.f;
        int drop = 0;
        while (drop < p->n_rois && p->roi_t[drop] < cutoff) drop++;
        if (drop) {
            memmove(p->roi_t, p->roi_t + drop, sizeof(float) * (size_t)(p->n_rois - drop));
            memmove(p->roi_etat, p->roi_etat + drop, sizeof(int) * (size_t)(p->n_rois - drop));
            p->n_rois -= drop;
        }
        i += idx_z;
        p->last_scan_idx = i + 1;
    }
    if (p->last_scan_idx < safe) p->last_scan_idx = safe;
}

/* computeLiveEtat + toLevel (spectral :147-163, audio :241-256) */
static void update_live(oracle_pulse *p) {
    int live = 0;
    if (p->n_rois > 0) {
        const float now = time_of(p, p->n - 1);
        const float start = now - p->cfg.live_window_t * p->t_target;
        float acc = 0.f;
        for (int k = 0; k < p->n_rois; k++)
            if (p->roi_t[k] >= start) acc += (float)p->roi_etat[k];
        live = (int)floorf(acc / p->cfg.live_divisor);
        if (live > 5) live = 5;
    }
    p->live_etat = live;
    p->last_level = live >= 5 ? 3 : live >= 3 ? 2 : live >= 1 ? 1 : 0;
}

/* onEnergyFrame (spectral :27-42, audio :113-128) */
static void energy_frame(oracle_pulse *p, float v, float freq) {
    if (p->n == 0) p->t0 = 0.f;
    p->e[p->n] = v;
    p->f[p->n] = freq;
    p->n++;
    const int max_buf = (int)(10.f * p->cfg.fs_energy);
    int drop = 0;
    while (p->n - drop > max_buf) {
        drop++;
        p->t0 += 1.f / p->cfg.fs_energy;
        if (p->last_scan_idx > 0) p->last_scan_idx--;
    }
    if (drop) {
        memmove(p->e, p->e + drop, sizeof(float) * (size_t)(p->n - drop));
        memmove(p->f, p->f + drop, sizeof(float) * (size_t)(p->n - drop));
        p->n -= drop;
    }
    detect_rois(p);
    update_live(p);
}

/* estimatedFreqHz (spectral_pulse_detector.cpp:148-170): OLS in double over the admitted ROIs */
static float est_freq(const oracle_pulse *p) {
    const int n = p->n_fh;
    if (n < 2) return 0.f;
    const float t_now = time_of(p, p->n - 1);
    double st = 0, sf = 0, stt = 0, stf = 0;
    for (int k = 0; k < n; k++) {
        const float t = p->fh_t[k], f = p->fh_f[k];
        st += t;
        sf += f;
        stt += t * t; /* float product, as in the reference */
        stf += t * f;
    }
    const double den = n * stt - st * st;
    if (fabs(den) < 1e-9) return (float)(sf / n);
    const double a = (n * stf - st * sf) / den;
    const double b = (sf - a * st) / n;
    return (float)(a * t_now + b);
}

static void fill_output(const oracle_pulse *p, float input, sdrg_pulse_output *o) {
    memset(o, 0, sizeof(*o));
    o->strength = p->last_snr;
    o->live_etat = p->live_etat;
    o->level = p->last_level;
    o->locked = p->locked;
    o->period_s = p->t_target;
    if (p->kind == SDRG_PULSE_SPECTRAL) {
        o->est_freq_hz = est_freq(p);
        o->est_freq_hz_rounded = llroundf(o->est_freq_hz);
        o->input = input;
    } else {
        o->input = p->last_snr;
    }
    o->n_energy = p->n;
    o->n_rois = p->n_rois;
}

/* SpectralPulseDetector::process (spectral_pulse_detector.cpp:10-13) for n_frames consecutive frames */
ORACLE_API int oracle_pulse_spectral(oracle_pulse *p, const float *snr_sigma, const float *freq_hz, int n_frames,
                                     sdrg_pulse_output *out) {
    for (int k = 0; k < n_frames; k++) {
        if (ensure_cap(p)) return -3;
        energy_frame(p, snr_sigma[k], freq_hz[k]);
        if (out) fill_output(p, snr_sigma[k], &out[k]);
    }
    return 0;
}

/* AudioPulseDetector::process (audio_pulse_detector.cpp:92-110) on one block; format 0 int16, 1 float */
ORACLE_API int oracle_pulse_audio(oracle_pulse *p, const void *audio, int fmt, int n, sdrg_pulse_output *out) {
    const float inv = 1.f / 32767.f;
    for (int k = 0; k < n; k++) {
        const float x = fmt == 0 ? (float)((const int16_t *)audio)[k] * inv : ((const float *)audio)[k];
        float y = sos_step(&p->band[0], x);
        y = sos_step(&p->band[1], y);
        p->frame_acc += y * y;
        p->frame_count++;
        if (p->frame_count >= p->frame_samples) {
            const float rms = sqrtf(p->frame_acc / (float)p->frame_samples);
            if (ensure_cap(p)) return -3;
            energy_frame(p, sos_step(&p->low, rms), 0.f);
            p->frame_acc = 0.f;
            p->frame_count = 0;
        }
    }
    if (out) fill_output(p, 0.f, out);
    return 0;
}

ORACLE_API int oracle_pulse_output_size(void) { return (int)sizeof(sdrg_pulse_output); }

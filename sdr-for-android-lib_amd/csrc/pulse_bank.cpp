// pulse_bank.cpp — host side of the pulse detectors: configuration, per-stream state and rings in HBM,
// kernel launches (pulse.hip) and the sdrg_pulse_bank_* C ABI.
//
//   SpectralPulseDetector(cfg) / configure / reset   src/dsp/spectral_pulse_detector.cpp:3-8, :179-196
//   AudioPulseDetector(cfg) / reset                  src/ssb/audio_pulse_detector.cpp:8-24, :242-256
//
// Ring capacity: eBuf_ never holds more than maxBuf = (int)(10 * fsEnergy) values after a push, and ROIs
// are at least two energy frames apart (detectRois resumes at i + idx_z + 1, idx_z >= 1) while the list keeps
// 20 s, so at most 10 * fsEnergy + 2 ROIs are held.  One power-of-two capacity >= maxBuf + 8 covers both.
// A configure() that raises fsEnergy past the capacity re-lays the rings out on the host (synchronously,
// after the in-flight launches): configuration changes are rare and off the per-frame path.
#include "pulse_bank.h"

#include <math.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "design.h"

using namespace sdrg;

#define PB_TRY(expr)                                                                               \
    do {                                                                                           \
        hipError_t e_ = (expr);                                                                    \
        if (e_ != hipSuccess) return fail(SDRG_E_HIP, "%s: %s", #expr, hipGetErrorString(e_));    \
    } while (0)

namespace {

int max_buf_of(const sdrg_pulse_config &c) { return (int)(10.f * c.fs_energy); }  // spectral :31, audio :118

int cap_for(const sdrg_pulse_config &c) {
    const int need = std::max(max_buf_of(c), 0) + 8;
    int cap = 16;
    while (cap < need) cap <<= 1;
    return cap;
}

PulseParams params_of(const sdrg_pulse_bank *b) {
    const sdrg_pulse_config &c = b->cfg;
    PulseParams p;
    memset(&p, 0, sizeof(p));
    p.cap_mask = b->cap - 1;
    p.max_buf = max_buf_of(c);
    p.fs_energy = c.fs_energy;
    p.inv_fs = 1.f / c.fs_energy;
    p.z_default_s = c.z_default_s;
    p.dt_tol_s = c.dt_tol_s;
    p.snr_min = c.snr_min;
    p.snr_rhythm = c.snr_rhythm;
    p.snr_strong = c.snr_strong;
    p.dispersion_max = c.dispersion_max;
    p.sum_n_max = c.sum_n_max;
    p.live_window_t = c.live_window_t;
    p.live_divisor = c.live_divisor;
    p.noise_far = c.noise_ref_far;
    p.noise_near = c.noise_ref_near;
    if (b->kind == SDRG_PULSE_AUDIO) {  // constructor (audio_pulse_detector.cpp:8-24)
        design_pulse_sos(c.sample_rate, c.f_min, true, p.band[0]);
        design_pulse_sos(c.sample_rate, c.f_max, false, p.band[1]);
        design_pulse_sos(c.fs_energy, c.smooth_cutoff, false, p.low);
        p.frame_samples = std::max(1, (int)(c.sample_rate / c.fs_energy));
    }
    return p;
}

template <typename T>
int32_t dev_alloc(T **p, size_t n) {
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    PB_TRY(hipMalloc(reinterpret_cast<void **>(p), std::max<size_t>(n, 1) * sizeof(T)));
    return SDRG_OK;
}

int32_t alloc_rings(sdrg_pulse_bank *b, int cap) {
    const size_t n = (size_t)b->n_streams * (size_t)cap;
    int32_t rc;
    if ((rc = dev_alloc(&b->d_e, n)) || (rc = dev_alloc(&b->d_rt, n)) || (rc = dev_alloc(&b->d_re, n))) return rc;
    if (b->kind == SDRG_PULSE_SPECTRAL && (rc = dev_alloc(&b->d_f, n))) return rc;
    b->cap = cap;
    return SDRG_OK;
}

// Re-lay every stream's rings out at a larger capacity, keeping the logical contents (deque order).
// every stream the bank's kernels may still run on
int32_t sync_streams(sdrg_pulse_bank *b) {
    if (b->last_stream) PB_TRY(hipStreamSynchronize(b->last_stream));
    if (b->detect_stream && b->detect_stream != b->last_stream) PB_TRY(hipStreamSynchronize(b->detect_stream));
    return SDRG_OK;
}

int32_t regrow(sdrg_pulse_bank *b, int new_cap) {
    if (int32_t rc = sync_streams(b)) return rc;
    if (b->reset_pending) return alloc_rings(b, new_cap);  // nothing to keep
    const int S = b->n_streams, oc = b->cap, om = oc - 1;
    const bool spectral = b->kind == SDRG_PULSE_SPECTRAL;
    std::vector<PulseStreamState> st(S);
    PB_TRY(hipMemcpy(st.data(), b->d_state, sizeof(PulseStreamState) * S, hipMemcpyDeviceToHost));
    float *ne = nullptr, *nf = nullptr, *nrt = nullptr;
    int *nre = nullptr;
    const size_t nn = (size_t)S * new_cap;
    int32_t rc;
    if ((rc = dev_alloc(&ne, nn)) || (rc = dev_alloc(&nrt, nn)) || (rc = dev_alloc(&nre, nn)) ||
        (spectral && (rc = dev_alloc(&nf, nn))))
        return rc;
    const int G = 256;  // streams per host batch
    std::vector<float> he((size_t)G * oc), hf(spectral ? (size_t)G * oc : 0), hrt((size_t)G * oc);
    std::vector<int> hre((size_t)G * oc);
    std::vector<float> ge((size_t)G * new_cap, 0.f), gf(spectral ? (size_t)G * new_cap : 0, 0.f),
        grt((size_t)G * new_cap, 0.f);
    std::vector<int> gre((size_t)G * new_cap, 0);
    for (int s0 = 0; s0 < S; s0 += G) {
        const int g = std::min(G, S - s0);
        const size_t o = (size_t)s0 * oc, cnt = (size_t)g * oc;
        PB_TRY(hipMemcpy(he.data(), b->d_e + o, cnt * 4, hipMemcpyDeviceToHost));
        if (spectral) PB_TRY(hipMemcpy(hf.data(), b->d_f + o, cnt * 4, hipMemcpyDeviceToHost));
        PB_TRY(hipMemcpy(hrt.data(), b->d_rt + o, cnt * 4, hipMemcpyDeviceToHost));
        PB_TRY(hipMemcpy(hre.data(), b->d_re + o, cnt * 4, hipMemcpyDeviceToHost));
        for (int k = 0; k < g; k++) {
            PulseStreamState &x = st[s0 + k];
            const size_t so = (size_t)k * oc, dn = (size_t)k * new_cap;
            for (int j = 0; j < x.n; j++) {
                ge[dn + j] = he[so + ((x.head + j) & om)];
                if (spectral) gf[dn + j] = hf[so + ((x.head + j) & om)];
            }
            for (int j = 0; j < x.n_rois; j++) {
                grt[dn + j] = hrt[so + ((x.roi_head + j) & om)];
                gre[dn + j] = hre[so + ((x.roi_head + j) & om)];
            }
            x.head = 0;
            x.roi_head = 0;
        }
        const size_t no = (size_t)s0 * new_cap, ncnt = (size_t)g * new_cap;
        PB_TRY(hipMemcpy(ne + no, ge.data(), ncnt * 4, hipMemcpyHostToDevice));
        if (spectral) PB_TRY(hipMemcpy(nf + no, gf.data(), ncnt * 4, hipMemcpyHostToDevice));
        PB_TRY(hipMemcpy(nrt + no, grt.data(), ncnt * 4, hipMemcpyHostToDevice));
        PB_TRY(hipMemcpy(nre + no, gre.data(), ncnt * 4, hipMemcpyHostToDevice));
    }
    PB_TRY(hipMemcpy(b->d_state, st.data(), sizeof(PulseStreamState) * S, hipMemcpyHostToDevice));
    void *old[] = {b->d_e, b->d_f, b->d_rt, b->d_re};
    for (void *p : old)
        if (p) (void)hipFree(p);
    b->d_e = ne;
    b->d_f = nf;
    b->d_rt = nrt;
    b->d_re = nre;
    b->cap = new_cap;
    return SDRG_OK;
}

// callers hold a DeviceScope for b->device
int32_t before_launch(sdrg_pulse_bank *b, hipStream_t stream) {
    if (b->reset_pending) {
        PB_TRY(launch_pulse_reset(b->d_state, b->n_streams, b->cfg.t_target_init, stream));
        b->reset_pending = false;
    }
    b->last_stream = stream;
    return SDRG_OK;
}

hipStream_t call_stream(const sdrg_pulse_bank *b) { return b->user_stream ? b->user_stream : b->own_stream; }

}  // namespace

namespace sdrg {

int32_t pulse_config_check(int kind, const sdrg_pulse_config *c) {
    if (!c) return fail(SDRG_E_INVALID, "null pulse config");
    if (kind != SDRG_PULSE_SPECTRAL && kind != SDRG_PULSE_AUDIO) return fail(SDRG_E_INVALID, "bad pulse kind %d", kind);
    if (!(c->fs_energy > 0.f) || !isfinite(c->fs_energy)) return fail(SDRG_E_INVALID, "fs_energy must be > 0");
    if (max_buf_of(*c) > (1 << 24)) return fail(SDRG_E_UNSUPPORTED, "fs_energy %g: energy buffer too large", c->fs_energy);
    if (kind == SDRG_PULSE_AUDIO && !(c->sample_rate > 0.f)) return fail(SDRG_E_INVALID, "sample_rate must be > 0");
    return SDRG_OK;
}

int32_t pulse_bank_init(sdrg_pulse_bank *b, int kind, const sdrg_pulse_config *cfg, int n_streams, int device) {
    int32_t rc = pulse_config_check(kind, cfg);
    if (rc) return rc;
    if (n_streams <= 0) return fail(SDRG_E_INVALID, "n_streams must be > 0");
    b->kind = kind;
    b->cfg = *cfg;
    b->n_streams = n_streams;
    b->device = device;
    DeviceScope dscope_(device);
    PB_TRY(dscope_.error());
    if ((rc = dev_alloc(&b->d_state, (size_t)n_streams)) || (rc = dev_alloc(&b->d_out, (size_t)n_streams))) return rc;
    if (kind == SDRG_PULSE_SPECTRAL && (rc = dev_alloc(&b->d_fh, (size_t)n_streams * 2 * PULSE_FH_SLOTS))) return rc;
    if (kind == SDRG_PULSE_AUDIO && (rc = dev_alloc(&b->d_new_count, (size_t)n_streams * sdrg_pulse_bank::NEW_SETS)))
        return rc;
    if ((rc = alloc_rings(b, cap_for(*cfg)))) return rc;
    // (the null stream's fill, waited for: the bank's kernels run on non-blocking streams)
    PB_TRY(hipMemset(b->d_out, 0, sizeof(sdrg_pulse_output) * (size_t)n_streams));
    PB_TRY(hipStreamSynchronize(nullptr));
    b->reset_pending = true;
    return SDRG_OK;
}

void pulse_bank_release(sdrg_pulse_bank *b) {
    DeviceScope dscope_(b->device);
    (void)sync_streams(b);
    void *bufs[] = {b->d_state, b->d_e, b->d_f, b->d_rt, b->d_re, b->d_fh, b->d_out, b->d_in, b->d_new, b->d_new_count};
    for (void *p : bufs)
        if (p) (void)hipFree(p);
    if (b->own_stream) (void)hipStreamDestroy(b->own_stream);
}

int32_t pulse_bank_configure(sdrg_pulse_bank *b, const sdrg_pulse_config *cfg) {
    int32_t rc = pulse_config_check(b->kind, cfg);
    if (rc) return rc;
    DeviceScope dscope_(b->device);
    PB_TRY(dscope_.error());
    b->cfg = *cfg;
    if (b->kind == SDRG_PULSE_AUDIO) b->reset_pending = true;  // AudioPulseDetector(pendingConfig_)
    const int need = cap_for(*cfg);
    if (need > b->cap) return regrow(b, need);
    return SDRG_OK;
}

int32_t pulse_bank_spectral(sdrg_pulse_bank *b, const float *snr_sigma, const float *freq_hz, int stride_bytes,
                            sdrg_pulse_output *out, hipStream_t stream) {
    DeviceScope dscope_(b->device);
    PB_TRY(dscope_.error());
    if (b->kind != SDRG_PULSE_SPECTRAL) return fail(SDRG_E_INVALID, "not a spectral pulse bank");
    if (!snr_sigma || !freq_hz || !out) return fail(SDRG_E_INVALID, "null pointer");
    if (stride_bytes < 0 || (stride_bytes & 3)) return fail(SDRG_E_INVALID, "stride must be a multiple of 4");
    int32_t rc = before_launch(b, stream);
    if (rc) return rc;
    PB_TRY(launch_spectral_pulse(params_of(b), b->n_streams, b->d_state, b->d_e, b->d_f, b->d_rt, b->d_re, b->d_fh,
                                 snr_sigma, freq_hz, stride_bytes, out, stream));
    return SDRG_OK;
}

int32_t pulse_bank_audio_front(sdrg_pulse_bank *b, int n, AudioFront *af, hipStream_t stream, int set) {
    DeviceScope dscope_(b->device);
    PB_TRY(dscope_.error());
    if (b->kind != SDRG_PULSE_AUDIO) return fail(SDRG_E_INVALID, "not an audio pulse bank");
    if (set < 0 || set >= sdrg_pulse_bank::NEW_SETS) return fail(SDRG_E_INVALID, "energy-frame set %d", set);
    const PulseParams p = params_of(b);
    const size_t max_new = (size_t)std::max(n, 0) / (size_t)p.frame_samples + 2;  // (frameCount_ + n) / frameSamples_ < this
    if (max_new > b->new_slots || !b->d_new) {
        if (int32_t rc = sync_streams(b)) return rc;  // the old buffer may be in use
        int32_t rc = dev_alloc(&b->d_new, (size_t)sdrg_pulse_bank::NEW_SETS * b->n_streams * max_new);
        if (rc) return rc;
        b->new_slots = max_new;
    }
    // a pending reset runs before the front end reads the state, and after every detector that still uses it
    if (b->reset_pending && b->detect_stream && b->detect_stream != stream) PB_TRY(hipStreamSynchronize(b->detect_stream));
    int32_t rc = before_launch(b, stream);
    if (rc) return rc;
    memcpy(af->band, p.band, sizeof(af->band));
    memcpy(af->low, p.low, sizeof(af->low));
    af->frame_samples = p.frame_samples;
    af->max_new = (int)b->new_slots;
    af->state = b->d_state;
    af->new_e = b->d_new + (size_t)set * b->n_streams * b->new_slots;
    af->new_count = b->d_new_count + (size_t)set * b->n_streams;
    return SDRG_OK;
}

int32_t pulse_bank_audio_detect(sdrg_pulse_bank *b, sdrg_pulse_output *out, hipStream_t stream, int set) {
    if (set < 0 || set >= sdrg_pulse_bank::NEW_SETS) return fail(SDRG_E_INVALID, "energy-frame set %d", set);
    if (stream != b->last_stream) b->detect_stream = stream;
    PB_TRY(launch_audio_detect(params_of(b), b->n_streams, b->d_state, b->d_e, b->d_rt, b->d_re,
                               b->d_new + (size_t)set * b->n_streams * b->new_slots, (int)b->new_slots,
                               b->d_new_count + (size_t)set * b->n_streams, out, stream));
    return SDRG_OK;
}

int32_t pulse_bank_audio(sdrg_pulse_bank *b, const void *audio, int fmt, int n, int stride, sdrg_pulse_output *out,
                         hipStream_t stream) {
    DeviceScope dscope_(b->device);
    PB_TRY(dscope_.error());
    if (b->kind != SDRG_PULSE_AUDIO) return fail(SDRG_E_INVALID, "not an audio pulse bank");
    if (fmt != 0 && fmt != 1) return fail(SDRG_E_INVALID, "sample_format must be 0 (int16) or 1 (float)");
    if (n < 0 || (n > 0 && (!audio || stride < n))) return fail(SDRG_E_INVALID, "bad audio block (n %d, stride %d)", n, stride);
    if (!out) return fail(SDRG_E_INVALID, "null out");
    AudioFront af;
    int32_t rc = pulse_bank_audio_front(b, n, &af, stream);
    if (rc) return rc;
    PB_TRY(launch_audio_front(af, audio, fmt, n, stride, b->n_streams, stream));
    return pulse_bank_audio_detect(b, out, stream);
}

}  // namespace sdrg

extern "C" {

int32_t sdrg_pulse_config_default(int32_t kind, sdrg_pulse_config *c) {
    if (!c) return fail(SDRG_E_INVALID, "null config");
    if (kind != SDRG_PULSE_SPECTRAL && kind != SDRG_PULSE_AUDIO) return fail(SDRG_E_INVALID, "bad pulse kind %d", kind);
    memset(c, 0, sizeof(*c));
    c->z_default_s = 0.666f;  // spectral_pulse_detector.h:23-35, audio_pulse_detector.h:19-37
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
    if (kind == SDRG_PULSE_SPECTRAL) {
        c->fs_energy = 20.f;
        c->snr_min = 1.5f;
        c->snr_rhythm = 2.5f;
        c->snr_strong = 4.0f;
    } else {
        c->fs_energy = 100.f;
        c->snr_min = 1.0f;
        c->snr_rhythm = 1.1f;
        c->snr_strong = 2.0f;
    }
    return SDRG_OK;
}

int32_t sdrg_pulse_bank_create(int32_t kind, const sdrg_pulse_config *cfg, int32_t n_streams, int32_t device,
                               sdrg_pulse_bank **out) {
    if (!out) return fail(SDRG_E_INVALID, "null out");
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return fail(SDRG_E_NODEVICE, "no HIP device");
    if (device < 0 || device >= count) return fail(SDRG_E_INVALID, "device %d out of range", device);
    hipDeviceProp_t prop;
    PB_TRY(hipGetDeviceProperties(&prop, device));
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(SDRG_E_NODEVICE, "device %d is %s, this build targets gfx950", device, prop.gcnArchName);
    sdrg_pulse_bank *b = new sdrg_pulse_bank();
    int32_t rc = pulse_bank_init(b, kind, cfg, n_streams, device);
    if (!rc && hipStreamCreateWithFlags(&b->own_stream, hipStreamNonBlocking) != hipSuccess)
        rc = fail(SDRG_E_HIP, "hipStreamCreate failed");
    if (rc) {
        pulse_bank_release(b);
        delete b;
        return rc;
    }
    *out = b;
    return SDRG_OK;
}

int32_t sdrg_pulse_bank_destroy(sdrg_pulse_bank *b) {
    if (!b) return SDRG_OK;
    pulse_bank_release(b);
    delete b;
    return SDRG_OK;
}

int32_t sdrg_pulse_bank_configure(sdrg_pulse_bank *b, const sdrg_pulse_config *cfg) {
    if (!b) return fail(SDRG_E_INVALID, "null bank");
    return pulse_bank_configure(b, cfg);
}

int32_t sdrg_pulse_bank_get_config(const sdrg_pulse_bank *b, sdrg_pulse_config *out) {
    if (!b || !out) return fail(SDRG_E_INVALID, "null argument");
    *out = b->cfg;
    return SDRG_OK;
}

int32_t sdrg_pulse_bank_reset(sdrg_pulse_bank *b) {
    if (!b) return fail(SDRG_E_INVALID, "null bank");
    b->reset_pending = true;
    return SDRG_OK;
}

int32_t sdrg_pulse_bank_set_stream(sdrg_pulse_bank *b, void *hip_stream) {
    if (!b) return fail(SDRG_E_INVALID, "null bank");
    b->user_stream = static_cast<hipStream_t>(hip_stream);
    return SDRG_OK;
}

int32_t sdrg_pulse_bank_process_spectral_device(sdrg_pulse_bank *b, const float *snr_sigma, const float *freq_hz,
                                                int32_t stride_bytes, sdrg_pulse_output *out) {
    if (!b) return fail(SDRG_E_INVALID, "null bank");
    return pulse_bank_spectral(b, snr_sigma, freq_hz, stride_bytes, out, call_stream(b));
}

int32_t sdrg_pulse_bank_process_audio_device(sdrg_pulse_bank *b, const void *audio, int32_t sample_format, int32_t n,
                                             int32_t stride, sdrg_pulse_output *out) {
    if (!b) return fail(SDRG_E_INVALID, "null bank");
    return pulse_bank_audio(b, audio, sample_format, n, stride, out, call_stream(b));
}

int32_t sdrg_pulse_bank_synchronize(sdrg_pulse_bank *b) {
    if (!b) return fail(SDRG_E_INVALID, "null bank");
    DeviceScope dscope_(b->device);
    PB_TRY(dscope_.error());
    PB_TRY(hipStreamSynchronize(call_stream(b)));
    return SDRG_OK;
}

static int32_t stage_in(sdrg_pulse_bank *b, size_t bytes) {
    if (b->in_bytes >= bytes && b->d_in) return SDRG_OK;
    if (b->d_in) (void)hipFree(b->d_in);
    b->d_in = nullptr;
    b->in_bytes = 0;
    PB_TRY(hipMalloc(&b->d_in, std::max<size_t>(bytes, 16)));
    b->in_bytes = bytes;
    return SDRG_OK;
}

int32_t sdrg_pulse_bank_process_spectral_host(sdrg_pulse_bank *b, const float *snr_sigma, const float *freq_hz,
                                              sdrg_pulse_output *out) {
    if (!b || !snr_sigma || !freq_hz || !out) return fail(SDRG_E_INVALID, "null argument");
    DeviceScope dscope_(b->device);
    PB_TRY(dscope_.error());
    const size_t S = (size_t)b->n_streams;
    int32_t rc = stage_in(b, 2 * S * sizeof(float));
    if (rc) return rc;
    hipStream_t st = call_stream(b);
    float *d = static_cast<float *>(b->d_in);
    PB_TRY(hipMemcpyAsync(d, snr_sigma, S * 4, hipMemcpyHostToDevice, st));
    PB_TRY(hipMemcpyAsync(d + S, freq_hz, S * 4, hipMemcpyHostToDevice, st));
    if ((rc = pulse_bank_spectral(b, d, d + S, 4, b->d_out, st))) return rc;
    PB_TRY(hipMemcpyAsync(out, b->d_out, S * sizeof(sdrg_pulse_output), hipMemcpyDeviceToHost, st));
    PB_TRY(hipStreamSynchronize(st));
    return SDRG_OK;
}

int32_t sdrg_pulse_bank_process_audio_host(sdrg_pulse_bank *b, const void *audio, int32_t sample_format, int32_t n,
                                           sdrg_pulse_output *out) {
    if (!b || !out || (n > 0 && !audio)) return fail(SDRG_E_INVALID, "null argument");
    if (sample_format != 0 && sample_format != 1) return fail(SDRG_E_INVALID, "bad sample_format");
    if (n < 0) return fail(SDRG_E_INVALID, "negative n");
    DeviceScope dscope_(b->device);
    PB_TRY(dscope_.error());
    const size_t S = (size_t)b->n_streams, es = sample_format == 0 ? 2 : 4;
    int32_t rc = stage_in(b, S * (size_t)n * es);
    if (rc) return rc;
    hipStream_t st = call_stream(b);
    if (n > 0) PB_TRY(hipMemcpyAsync(b->d_in, audio, S * (size_t)n * es, hipMemcpyHostToDevice, st));
    if ((rc = pulse_bank_audio(b, b->d_in, sample_format, n, n, b->d_out, st))) return rc;
    PB_TRY(hipMemcpyAsync(out, b->d_out, S * sizeof(sdrg_pulse_output), hipMemcpyDeviceToHost, st));
    PB_TRY(hipStreamSynchronize(st));
    return SDRG_OK;
}

}  // extern "C"

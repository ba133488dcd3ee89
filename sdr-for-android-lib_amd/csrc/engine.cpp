// engine.cpp — the C ABI (include/sdrg.h): configuration, per-stream state in HBM, kernel orchestration.
//
// Host-side equivalent of the reference's bridge + FFTProcessor + processSSB_opt control logic:
//   BridgeConfig::initialize / setters     src/bridge-config.h:17-65
//   FFTProcessor::configure                src/dsp/fft_process.cpp:20-39
//   processSSB_opt's static initialisation src/ssb/ssb_demod_opt.cpp:223-282 (mode globals, rfInit, eqInit)
//   soapyCallback's per-frame dispatch     src/sdr-bridge-java-soapy.cpp:424-493
// Everything that runs per sample runs in the HIP kernels (spectrum.hip, stats.hip, ssb.hip).
//
// Work is enqueued on a main HIP stream (spectrum -> stats) and a forked SSB stream that joins back,
// so the two independent halves of the hot path overlap on the GPU and a caller sees one stream.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <tuple>
#include <vector>

#include "design.h"
#include "pulse_bank.h"
#include "sdrg_internal.h"

using namespace sdrg;

namespace {
thread_local std::string g_last_error;
}  // namespace

int32_t sdrg::fail(int32_t code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

// The attribute is one limit per (kernel, device) that each set overwrites, and launches asking for more than it
// fail; requests vary with the geometry (statistics) and N (any-N FFT), so the limit only ever rises: the largest
// value set so far is cached per (kernel, device), and a smaller request leaves it as it is.
hipError_t sdrg::ensure_dynamic_lds(const void *kernel, int bytes) {
    static std::mutex mu;
    static std::map<std::pair<const void *, int>, int> limit;  // (kernel, device) -> largest limit set
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    std::lock_guard<std::mutex> lk(mu);
    const auto key = std::make_pair(kernel, dev);
    auto it = limit.find(key);
    if (it != limit.end() && it->second >= bytes) return hipSuccess;
    e = hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e == hipSuccess) limit[key] = bytes;
    return e;
}

namespace {

#define HIP_TRY(expr)                                                                              \
    do {                                                                                           \
        hipError_t e_ = (expr);                                                                    \
        if (e_ != hipSuccess) return fail(SDRG_E_HIP, "%s: %s", #expr, hipGetErrorString(e_));    \
    } while (0)


// processSSB_opt's statics that every stream of an engine shares (they only depend on the call sequence)
struct SsbControl {
    int64_t samp_count = 0;  // static size_t sampCount, frozen at the first call (:224)
    float agc_target = 0.35f, agc_fast = 0.006f, agc_slow = 0.00035f, gain = 0.5f;  // :17-28
    float lowpass_bd = 3200.0f, lowpass_q = 0.9f, transient_coeff = 0.55f;
    bool rf_init = false;
    float lpf[5] = {0, 0, 0, 0, 0};
    bool eq_init = false;
    float hp[5] = {0, 0, 0, 0, 0}, bp[5] = {0, 0, 0, 0, 0};
    // FIR taps currently uploaded (depend on samp_count, decim and the variant's tap count)
    int64_t taps_samp = -1;
    int taps_decim = -1, taps_req = -1, n_taps = 0;
};

// Page-locked host array (hipHostMalloc) for the host path's engine-owned copies: device-to-host copies into
// pageable memory go through the runtime's staging at a fraction of the PCIe rate.
template <class T>
struct PinnedVec {
    T *p = nullptr;
    size_t n = 0, cap = 0;
    PinnedVec() = default;
    PinnedVec(const PinnedVec &) = delete;
    PinnedVec &operator=(const PinnedVec &) = delete;
    ~PinnedVec() {
        if (p) (void)hipHostFree(p);
    }
    bool resize(size_t k) {  // contents are not preserved on growth (every use refills the array)
        if (k > cap) {
            if (p) (void)hipHostFree(p);
            p = nullptr;
            cap = n = 0;
            if (hipHostMalloc(reinterpret_cast<void **>(&p), sizeof(T) * k, hipHostMallocDefault) != hipSuccess) {
                p = nullptr;
                return false;
            }
            cap = k;
        }
        n = k;
        return true;
    }
    void assign(const T *a, const T *b) {
        if (resize((size_t)(b - a))) memcpy(p, a, sizeof(T) * (size_t)(b - a));
    }
    T *data() { return p; }
    T &operator[](size_t i) { return p[i]; }
};

struct EvSet {
    hipEvent_t t0 = nullptr, spec = nullptr, stats = nullptr, ssb0 = nullptr, ssb1 = nullptr, end = nullptr;
    bool has_spec = false, has_stats = false, has_ssb = false, pending = false;
    bool ssb_timed = false;  // ssb0 recorded: this call's SSB duration is measured from its own start marker
    int64_t seq = -1;        // the call's number among ALL calls (pipelined SSB: interval to call seq - 1, if profiled)
    bool stats_marked = false;  // `stats` recorded after the statistics (joined calls, whose `end` follows the join)
};

}  // namespace

struct sdrg_engine {
    sdrg_config cfg{};  // BridgeConfig: what the next frame is cut, demodulated and reported with
    // FFTProcessor::config_ (fft_process.h:88, :20-39): the centre frequency, sample rate and focus the statistics
    // use, copied from cfg at each configure() point (create, applyConfig, setFrequency, setFrequencyFocusRange).
    // setSampleRate / setSamplesPerReading / setSoundMode change cfg only (sdr-bridge-java-soapy.cpp:931-1023).
    uint32_t fft_fc = 0, fft_fs = 0;
    int32_t fft_focus = 0;
    int n_streams = 0;
    int device = 0;
    hipStream_t s_main = nullptr, s_ssb = nullptr;
    // CU split (SDRG_CU_SPLIT, lab): the SSB stream and a spectrum/statistics stream restricted to disjoint
    // halves of the CUs (hipExtStreamCreateWithCUMask), so the latency-bound SSB waves share no SIMD with the
    // spectrum's; s_spec is forked from / joined into s_main per call like the SSB stream
    hipStream_t s_spec = nullptr;
    int spec_cus = 0;
    hipEvent_t ev_fork_spec = nullptr, ev_join_spec = nullptr;
    hipStream_t s_own = nullptr;  // the engine's own main stream (s_main is it, or the caller's via set_stream)
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    // input release: recorded after the last kernel of a call that reads its iq buffer on each stream (the
    // spectrum on s_main, the SSB pipeline on s_ssb); sdrg_engine_input_released / _wait_input_released
    hipEvent_t ev_in_main = nullptr, ev_in_ssb = nullptr;
    // the markers the last call recorded after its iq readers (ev_in_* or the profiling ring's events)
    hipEvent_t last_in_main = nullptr, last_in_ssb = nullptr;
    // profiling: a ring of event sets so consecutive calls are timed without host synchronisation
    static constexpr int RING = 64;
    EvSet ring[RING];
    bool ring_created = false;
    int ring_next = 0, ring_last = -1;
    bool profiling = false;
    sdrg_timings last_timings{};
    double sum_spec = 0, sum_stats = 0, sum_ssb = 0, sum_total = 0;
    int n_acc = 0, n_ssb = 0;
    int64_t calls_total = 0;  // every enqueue, profiled or not: two calls are consecutive only if their seqs are
    int64_t seq_reset = 0;    // seq of the first call after the last reset of the timing statistics

    // device state / buffers
    StatsState *d_stats = nullptr;
    SsbStreamState *d_ssb = nullptr;
    float *d_twiddles = nullptr;
    int tw_n = 0;
    float *d_taps = nullptr;
    int *d_chunk_table = nullptr;     // per SSB pipeline chunk: FIR outputs overlapping / completed
    size_t chunk_table_elems = 0;
    float *d_ssb_scratch = nullptr;
    size_t ssb_scratch_elems = 0;
    float *d_spec_scratch = nullptr;
    size_t spec_scratch_elems = 0;
    float *d_focus_stage = nullptr;   // sdrg_engine_gather: the focus-window slices, packed for ncclGather
    size_t focus_stage_elems = 0;
    // sdrg_engine_gather runs on a stream of its own after the outputs it reads; a later call that writes a buffer
    // still being gathered (same pointer) waits for the gather on the GPU first, so a caller rotating its output
    // buffers never delays its next call's kernels behind a gather
    bool last_async_stats = false;  // the last call with a statistics stage ran it on s_stats
    bool lab_ssb_first = false;     // lab SDRG_SSB_FIRST: host launch order of a forked SSB stage
    bool lab_stats_cus = false;     // lab SDRG_STATS_CUS: s_stats and s_spec on disjoint CU masks
    hipStream_t s_gather = nullptr;   // lab (SDRG_GATHER_STREAM=1): the gathers on a stream of their own
    hipStream_t s_last_gather = nullptr;  // the stream of the last gather
    hipEvent_t ev_gather = nullptr;  // the last gather's end (wait_outputs, synchronize)
    // each gather's end in a ring; a buffer a gather read maps to that gather's slot, so a call that rewrites it waits
    // for that gather only (waiting on the last gather instead made call k + 3's spectrum wait for gather k + 2, and
    // with it for call k + 2's asynchronous statistics)
    static constexpr int GRING = 8;
    hipEvent_t ev_g[GRING] = {};
    int64_t g_calls = 0;
    struct GBuf {
        uintptr_t lo, hi;  // the byte range [lo, hi) a gather reads
        int slot;
        int64_t seq;       // g_calls of that gather (gathers run in call order: the latest covers the earlier ones)
    };
    std::vector<GBuf> g_bufs;  // byte ranges read by gathers no later call has yet waited for
    // the event of the latest gather that reads any byte of [p, p + bytes) (ranges, not base pointers: an output
    // written at an offset into, or as a slice of, a gathered allocation still waits)
    hipEvent_t gathering(const void *p, size_t bytes) const {
        if (!p || !bytes) return nullptr;
        const uintptr_t lo = reinterpret_cast<uintptr_t>(p), hi = lo + bytes;
        const GBuf *best = nullptr;
        for (const GBuf &g : g_bufs)
            if (g.lo < hi && lo < g.hi && (!best || g.seq > best->seq)) best = &g;
        return best ? ev_g[best->slot] : nullptr;
    }
    float *d_fft_scratch = nullptr;   // four-step intermediate (N > 16384)
    size_t fft_scratch_elems = 0;
    sdrg_frame_record *d_rec_scratch = nullptr;
    float *d_pool = nullptr;          // statistics' pooled bins beyond the LDS bound (wide focus, N > 65536)
    size_t pool_elems = 0;
    // host-path staging
    void *d_iq_stage = nullptr;
    size_t iq_stage_bytes = 0;
    float *d_spec_stage = nullptr;
    size_t spec_stage_elems = 0;
    float *d_ss_stage = nullptr;  // signal_strength_host's copy of the caller's spectra
    size_t ss_stage_elems = 0;
    sdrg_frame_record *d_rec_stage = nullptr;
    int16_t *d_pcm_stage = nullptr;
    size_t pcm_stage_elems = 0;
    PinnedVec<float> h_spec;
    PinnedVec<sdrg_frame_record> h_rec;
    PinnedVec<int16_t> h_pcm;

    SsbControl ssb;
    // pulse detectors (created at the first call that runs their stage)
    sdrg_pulse_config spec_pulse_cfg{}, audio_pulse_cfg{};
    sdrg_pulse_bank spec_bank, audio_bank;
    bool spec_bank_live = false, audio_bank_live = false;
    PinnedVec<sdrg_pulse_output> h_pspec, h_paudio;
    bool cf_changed_pending = false;
    bool pipelined = false;  // sdrg_engine_set_pipelining: no join of the SSB stream per call
    bool inputs_ready = false;  // SDRG_PIPELINE_INPUTS_READY: no fork wait on the main stream either
    // SDRG_PIPELINE_STATS_ASYNC: a pipelined call's statistics (+ spectral pulse detector) run on s_stats after its
    // spectrum, beside the next call's spectrum.  The engine keeps the spectra a call's statistics read intact:
    // a call that writes the same spectra buffer as the call before waits (on the GPU) for that call's statistics,
    // and the host waits for the statistics of the call two before (so a caller rotating two or more spectra
    // buffers never waits on the GPU).
    bool stats_async = false;
    hipStream_t s_stats = nullptr;
    hipEvent_t ev_spec_done = nullptr;  // after a call's spectrum on s_main, waited by s_stats
    static constexpr int SA_RING = 3;
    hipEvent_t ev_stats_end[SA_RING] = {};  // end of the statistics of call (sa_calls - k) at slot % SA_RING
    const float *sa_spec[SA_RING] = {};     // the spectra buffer each of those calls' statistics read
    bool sa_live[SA_RING] = {};
    int64_t sa_calls = 0;
    hipEvent_t last_stats_end = nullptr;    // the last asynchronous statistics (wait_outputs, synchronize)
    // the audio pulse detector (AudioPulseDetector::process after processSSB_opt, ssb_processor.cpp:109) runs on s_ap
    // after the call's SSB pipeline, so the SSB stream (the pipelined step's critical path) carries the SSB kernels
    // alone.  Call k's front end (inside its SSB kernel) writes energy-frame set k % NEW_SETS; before it does, the host
    // waits for the detector of call k - NEW_SETS, which read that set.
    hipStream_t s_ap = nullptr;
    hipEvent_t ev_ap_end[sdrg_pulse_bank::NEW_SETS] = {};
    bool ap_live[sdrg_pulse_bank::NEW_SETS] = {};
    int64_t ap_calls = 0;
    hipEvent_t last_ap_end = nullptr;       // the last detector (outputs, joins)
    // NCO/short-FIR SSB variant (sdrg_engine_set_ssb_variant; a build extension, off by default)
    double nco_hz = 0.0;
    int fir_taps = 0;            // 0: the reference's 255
    uint32_t nco_phase = 0;      // phase of the next call's first sample (advances by inc * samp_count)
    float *d_nco_tab = nullptr;  // nco_tables(), uploaded once
    int upper = 1;
    bool has_cbs = false;
    sdrg_callbacks cbs{};
};

namespace {

// applyConfig's SpectralPulseDetector configuration (sdr-bridge-java-soapy.cpp:1130-1138): the default
// Config with fsEnergy = sampleRate / samplesPerReading (20 when samplesPerReading <= 0)
sdrg_pulse_config spectral_pulse_cfg_for(const sdrg_config &c) {
    sdrg_pulse_config p;
    sdrg_pulse_config_default(SDRG_PULSE_SPECTRAL, &p);
    p.fs_energy = c.samples_per_reading > 0 ? (float)c.sample_rate / (float)c.samples_per_reading : 20.f;
    return p;
}

// FFTProcessor::configure(FftProcessorConfig{cf, fs, N, focus}) with the bridge's current values
void configure_fft(sdrg_engine *e) {
    e->fft_fc = (uint32_t)e->cfg.center_frequency;
    e->fft_fs = (uint32_t)e->cfg.sample_rate;
    e->fft_focus = e->cfg.freq_focus_range_khz;
}

int32_t validate_config(const sdrg_config *cfg) {
    if (!cfg) return fail(SDRG_E_INVALID, "null config");
    if (cfg->samples_per_reading < 1 || cfg->samples_per_reading > (1 << 20))
        return fail(SDRG_E_UNSUPPORTED, "samples_per_reading %d outside [1, 2^20]", cfg->samples_per_reading);
    if ((uint32_t)cfg->sample_rate == 0) return fail(SDRG_E_INVALID, "sample_rate must be > 0");
    if (cfg->freq_focus_range_khz < 0) return fail(SDRG_E_INVALID, "freq_focus_range_khz must be >= 0");
    return SDRG_OK;
}

// hipMemset is enqueued on the null stream, which the engine's non-blocking streams are not ordered with: without
// the wait, a kernel or copy enqueued next on s_main could run before (or under) the fill -- e.g. a fresh staging
// buffer zeroed after the caller's spectra were copied into it.  Fills happen at allocation and reset only.
hipError_t memset_sync(void *p, int v, size_t bytes) {
    hipError_t e = hipMemset(p, v, bytes);
    if (e == hipSuccess) e = hipStreamSynchronize(nullptr);
    return e;
}

template <typename T>
int32_t ensure_device(T **p, size_t *have, size_t need, bool zero = false) {
    if (*have >= need && *p) return SDRG_OK;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *have = 0;
    if (need == 0) return SDRG_OK;
    HIP_TRY(hipMalloc(reinterpret_cast<void **>(p), need * sizeof(T)));
    if (zero) HIP_TRY(memset_sync(*p, 0, need * sizeof(T)));
    *have = need;
    return SDRG_OK;
}

int32_t upload_twiddles(sdrg_engine *e, int n) {
    if (e->tw_n == n && e->d_twiddles) return SDRG_OK;
    std::vector<float> tw(spectrum_twiddle_floats(n));
    spectrum_fill_twiddles(n, tw.data());
    if (e->d_twiddles) (void)hipFree(e->d_twiddles);
    e->d_twiddles = nullptr;
    e->tw_n = 0;
    HIP_TRY(hipMalloc(reinterpret_cast<void **>(&e->d_twiddles), tw.size() * sizeof(float)));
    HIP_TRY(hipMemcpy(e->d_twiddles, tw.data(), tw.size() * sizeof(float), hipMemcpyHostToDevice));
    e->tw_n = n;
    return SDRG_OK;
}

int64_t ssb_frozen_or(const sdrg_engine *e) {
    return e->ssb.samp_count ? e->ssb.samp_count : e->cfg.samples_per_reading;
}

// Resolve one ring slot's events into timings and add them to the running sums.
int32_t fold_slot(sdrg_engine *e, int slot) {
    EvSet &ev = e->ring[slot];
    if (!ev.pending) return SDRG_OK;
    HIP_TRY(hipEventSynchronize(ev.end));
    sdrg_timings t{};
    float ms = 0.0f;
    if (ev.has_spec) {
        HIP_TRY(hipEventElapsedTime(&ms, ev.t0, ev.spec));
        t.spectrum_ms = ms;
    }
    if (ev.has_stats) {
        if (ev.stats_marked) HIP_TRY(hipEventSynchronize(ev.stats));  // asynchronous statistics end on s_stats
        HIP_TRY(hipEventElapsedTime(&ms, ev.has_spec ? ev.spec : ev.t0, ev.stats_marked ? ev.stats : ev.end));
        t.stats_ms = ms;
    }
    bool ssb_measured = false;
    if (ev.has_ssb && ev.ssb_timed) {
        // pipelined calls never join the SSB stream into ev.end's stream: wait for its own end event
        HIP_TRY(hipEventSynchronize(ev.ssb1));
        HIP_TRY(hipEventElapsedTime(&ms, ev.ssb0, ev.ssb1));
        t.ssb_ms = ms;
        ssb_measured = true;
    } else if (ev.has_ssb) {
        // pipelined: no start marker (it would sit on the SSB stream, the step's critical path); the call's SSB
        // stream time is the interval from the previous call's SSB end marker to its own.  The previous slot still
        // holds that marker while its seq is this call's - 1 (enqueue folds a slot's successor before reusing it).
        const EvSet &pv = e->ring[(slot + sdrg_engine::RING - 1) % sdrg_engine::RING];
        if (pv.seq == ev.seq - 1 && pv.has_ssb && ev.seq > e->seq_reset) {
            HIP_TRY(hipEventSynchronize(ev.ssb1));
            HIP_TRY(hipEventElapsedTime(&ms, pv.ssb1, ev.ssb1));
            t.ssb_ms = ms;
            ssb_measured = true;
        }
    }
    HIP_TRY(hipEventElapsedTime(&ms, ev.t0, ev.end));
    t.total_ms = ms;
    ev.pending = false;
    if (slot == e->ring_last) e->last_timings = t;
    e->sum_spec += t.spectrum_ms;
    e->sum_stats += t.stats_ms;
    if (ssb_measured) {
        e->sum_ssb += t.ssb_ms;
        e->n_ssb++;
    }
    e->sum_total += t.total_ms;
    e->n_acc++;
    return SDRG_OK;
}

int32_t fold_all(sdrg_engine *e) {
    // oldest first
    for (int k = 0; k < sdrg_engine::RING; k++) {
        int32_t rc = fold_slot(e, (e->ring_next + k) % sdrg_engine::RING);
        if (rc) return rc;
    }
    return SDRG_OK;
}

// processSSB_opt's per-call control logic (:223-282) -> kernel parameters.  Works on copies of the engine's
// SSB control statics (c) and NCO phase (nco_phase) that the caller commits only once the call's launches have
// succeeded, so a rejected call freezes no frame size and advances no phase.  The taps and chunk table it may
// upload are keyed by the committed statics: a rejected call's upload is simply redone by the next call.
int32_t prepare_ssb(sdrg_engine *e, SsbControl &c, uint32_t &nco_phase, SsbParams *p) {
    const uint32_t fs = (uint32_t)e->cfg.sample_rate;
    if (c.samp_count == 0) c.samp_count = e->cfg.samples_per_reading;  // static size_t sampCount = iq.size()
    const int mode = e->cfg.sound_mode;
    if (mode == 2) {
        c.agc_target = 0.45f; c.agc_fast = 0.008f; c.gain = 4.5f;
        c.lowpass_bd = 2200.0f; c.lowpass_q = 1.2f; c.transient_coeff = 0.7f;
    } else if (mode == 0) {
        c.agc_target = 0.45f; c.agc_fast = 0.008f; c.gain = 10.0f;
        c.lowpass_bd = 2200.0f; c.lowpass_q = 1.2f; c.transient_coeff = 0.7f;
    } else if (mode == 1) {
        c.agc_target = 0.35f; c.agc_fast = 0.006f; c.agc_slow = 0.00035f; c.gain = 0.5f;
        c.lowpass_bd = 3200.0f; c.lowpass_q = 0.9f; c.transient_coeff = 0.55f;
    }
    if (!c.rf_init) {
        design_lowpass((float)fs, c.lowpass_bd, c.lowpass_q, c.lpf);
        c.rf_init = true;
    }
    const int decim = ssb_decim(fs);
    if (c.taps_samp != c.samp_count || c.taps_decim != decim || c.taps_req != e->fir_taps || !e->d_taps) {
        // an earlier call's SSB kernels may still read the taps and the chunk table (non-blocking streams)
        HIP_TRY(hipStreamSynchronize(e->s_ssb));
        // the device tables change now, before this call commits its SSB state: the committed key no longer
        // describes them, so a call that fails after this point leaves the next one to upload again
        e->ssb.taps_samp = -1;
        float h[256];
        c.n_taps = design_fir(c.samp_count, decim, 0.45f, h, e->fir_taps);
        c.taps_req = e->fir_taps;
        if (!e->d_taps) HIP_TRY(hipMalloc(reinterpret_cast<void **>(&e->d_taps), 256 * sizeof(float)));
        HIP_TRY(hipMemcpy(e->d_taps, h, sizeof(float) * (size_t)c.n_taps, hipMemcpyHostToDevice));
        c.taps_samp = c.samp_count;
        c.taps_decim = decim;
        // FIR output ranges per pipeline chunk (the kernel then needs no integer division):
        // overlapping: D*o <= t1-1 and D*o + NT - 1 >= t0 ; completed: t0 <= D*o + NT - 1 < t1
        const int CH = ssb_pipe_chunk(), D = decim, NT = c.n_taps;
        const int S = (int)c.samp_count, PL = ssb_pcm_len(c.samp_count, fs, e->fir_taps);
        const int nch = (S + CH - 1) / CH;
        std::vector<int> tab(4 * (size_t)nch);
        int ov_lo = 0, ov_hi = -1, dn_lo = 0, dn_hi = -1;
        for (int ch = 0; ch < nch; ch++) {
            const int t0 = ch * CH, t1 = std::min(t0 + CH, S);
            while (ov_lo < PL && D * ov_lo + NT - 1 < t0) ov_lo++;
            while (ov_hi + 1 < PL && D * (ov_hi + 1) <= t1 - 1) ov_hi++;
            dn_lo = dn_hi + 1;
            while (dn_hi + 1 < PL && D * (dn_hi + 1) + NT - 1 < t1) dn_hi++;
            tab[4 * ch] = ov_lo;
            tab[4 * ch + 1] = ov_hi;
            tab[4 * ch + 2] = dn_lo;
            tab[4 * ch + 3] = dn_hi;
        }
        int32_t rc = ensure_device(&e->d_chunk_table, &e->chunk_table_elems, tab.size());
        if (rc) return rc;
        HIP_TRY(hipMemcpy(e->d_chunk_table, tab.data(), tab.size() * sizeof(int), hipMemcpyHostToDevice));
    }
    if (!c.eq_init) {
        design_highpass(48000.0f, 1200.0f, 0.7f, c.hp);
        design_bandpass(48000.0f, 2400.0f, 0.6f, c.bp);
        c.eq_init = true;
    }
    memset(p, 0, sizeof(*p));
    p->samp_count = (int32_t)c.samp_count;
    p->n_in = e->cfg.samples_per_reading;
    p->upper = e->upper;  // SSBProcessor always asks for the upper sideband (ssb_processor.cpp:103)
    p->decim = decim;
    p->n_taps = c.n_taps;
    p->pcm_len = ssb_pcm_len(c.samp_count, fs, e->fir_taps);
    p->agc_target = c.agc_target;
    p->agc_fast = c.agc_fast;
    p->agc_slow = c.agc_slow;
    p->gain = c.gain;
    p->transient_coeff = c.transient_coeff;
    memcpy(p->lpf, c.lpf, sizeof(p->lpf));
    memcpy(p->hp, c.hp, sizeof(p->hp));
    memcpy(p->bp, c.bp, sizeof(p->bp));
    if (e->nco_hz != 0.0) {
        if (!e->d_nco_tab) {
            std::vector<float> tab(4096);
            nco_tables(tab.data());
            HIP_TRY(hipMalloc(reinterpret_cast<void **>(&e->d_nco_tab), sizeof(float) * tab.size()));
            HIP_TRY(hipMemcpy(e->d_nco_tab, tab.data(), sizeof(float) * tab.size(), hipMemcpyHostToDevice));
        }
        p->nco_on = 1;
        p->nco_inc = nco_increment(e->nco_hz, fs);
        p->nco_phase = nco_phase;
        p->nco_tab = e->d_nco_tab;
        nco_phase += p->nco_inc * (uint32_t)c.samp_count;  // phase-continuous across calls
    }
    return SDRG_OK;
}

int32_t alloc_state(sdrg_engine *e) {
    HIP_TRY(hipMalloc(reinterpret_cast<void **>(&e->d_stats), sizeof(StatsState) * (size_t)e->n_streams));
    HIP_TRY(hipMalloc(reinterpret_cast<void **>(&e->d_ssb), sizeof(SsbStreamState) * (size_t)e->n_streams));
    HIP_TRY(memset_sync(e->d_stats, 0, sizeof(StatsState) * (size_t)e->n_streams));
    HIP_TRY(memset_sync(e->d_ssb, 0, sizeof(SsbStreamState) * (size_t)e->n_streams));
    return SDRG_OK;
}

// FFTProcessor::configure (fft_process.cpp:33-35): maxPeakAndFrequency = {-130, cf} on first configure.
// The device state starts zeroed; max_peak_set = 0 makes the kernel seed it at the first frame with the
// centre frequency of that frame's configuration, which is what configure() stored.
int32_t bytes_per_sample(int fmt) {
    switch (fmt) {
    case SDRG_IQ_CF32: return 8;
    case SDRG_IQ_CS16: return 4;
    case SDRG_IQ_CS8:
    case SDRG_IQ_CU8: return 2;
    default: return 0;
    }
}

int32_t enqueue(sdrg_engine *e, const void *iq, int32_t fmt, int32_t stages, float *spectra,
                sdrg_frame_record *records, int16_t *pcm, int64_t now_ms, bool join) {
    const int n = e->cfg.samples_per_reading;
    const int B = e->n_streams;
    if (!iq) return fail(SDRG_E_INVALID, "null iq");
    if (bytes_per_sample(fmt) == 0) return fail(SDRG_E_INVALID, "unknown iq format %d", fmt);
    if (stages & ~SDRG_STAGE_ALL) return fail(SDRG_E_INVALID, "unknown stage bits 0x%x", stages);
    if ((stages & SDRG_STAGE_STATS) && !(stages & SDRG_STAGE_SPECTRUM))
        return fail(SDRG_E_INVALID, "STATS needs SPECTRUM");
    if ((stages & SDRG_STAGE_SPECTRAL_PULSE) && !(stages & SDRG_STAGE_STATS))
        return fail(SDRG_E_INVALID, "SPECTRAL_PULSE needs STATS");
    if ((stages & SDRG_STAGE_AUDIO_PULSE) && !(stages & SDRG_STAGE_SSB))
        return fail(SDRG_E_INVALID, "AUDIO_PULSE needs SSB");
    const bool do_spec = stages & SDRG_STAGE_SPECTRUM, do_stats = stages & SDRG_STAGE_STATS,
               do_ssb = stages & SDRG_STAGE_SSB, do_sp = stages & SDRG_STAGE_SPECTRAL_PULSE,
               do_ap = stages & SDRG_STAGE_AUDIO_PULSE;
    if (do_sp && !e->spec_bank_live) {
        int32_t rc = pulse_bank_init(&e->spec_bank, SDRG_PULSE_SPECTRAL, &e->spec_pulse_cfg, B, e->device);
        if (rc) return rc;
        e->spec_bank_live = true;
    }
    if (do_ap && !e->audio_bank_live) {
        int32_t rc = pulse_bank_init(&e->audio_bank, SDRG_PULSE_AUDIO, &e->audio_pulse_cfg, B, e->device);
        if (rc) return rc;
        e->audio_bank_live = true;
    }
    if (do_spec && !spectrum_supported(n))
        return fail(SDRG_E_UNSUPPORTED, "spectrum for N=%d not supported by this build", n);

    float *spec = spectra;
    if (do_spec && !spec) {
        // zeroed: for odd N the reference never writes power_shifted[N-1] (fft_process.cpp:92-97), which keeps the
        // value its vector held -- 0 for a fresh vector, the same stream's last value afterwards
        int32_t rc = ensure_device(&e->d_spec_scratch, &e->spec_scratch_elems, (size_t)B * n, true);
        if (rc) return rc;
        spec = e->d_spec_scratch;
    }
    sdrg_frame_record *recs = records;
    if (do_stats && !recs) {
        size_t have = e->d_rec_scratch ? (size_t)B : 0;
        int32_t rc = ensure_device(&e->d_rec_scratch, &have, (size_t)B);
        if (rc) return rc;
        recs = e->d_rec_scratch;
    }
    // the byte ranges this call writes (checked against the ranges pending gathers read)
    const size_t spec_bytes = (size_t)B * (size_t)n * sizeof(float), rec_bytes = (size_t)B * sizeof(sdrg_frame_record);
    size_t pcm_bytes = 0;
    SsbParams sp;
    if (do_ssb) {
        // frame size and PCM length this call will use (sampCount freezes at the first SSB call, :224-227)
        const int64_t samp = ssb_frozen_or(e);
        const int plen = ssb_pcm_len(samp, (uint32_t)e->cfg.sample_rate, e->fir_taps);
        if (!pcm && plen > 0) return fail(SDRG_E_INVALID, "null pcm with SSB stage");
        pcm_bytes = (size_t)B * (size_t)(plen > 0 ? plen : 0) * sizeof(int16_t);
        int32_t rc = ensure_device(&e->d_ssb_scratch, &e->ssb_scratch_elems, (size_t)B * ((size_t)samp + (size_t)plen));
        if (rc) return rc;
    }
    if (do_spec) {
        int32_t rc = upload_twiddles(e, n);
        if (rc) return rc;
        rc = ensure_device(&e->d_fft_scratch, &e->fft_scratch_elems, spectrum_scratch_floats(n, B));
        if (rc) return rc;
    }

    StatsGeometry geo{};
    if (do_stats) {
        if (e->fft_fs == 0) return fail(SDRG_E_INVALID, "the statistics' sample rate is 0");
        geo = stats_geometry(e->fft_fs, e->fft_fc, n, e->fft_focus);
        geo.cf_changed = e->cf_changed_pending ? 1 : 0;
        int32_t rc = ensure_device(&e->d_pool, &e->pool_elems, stats_global_pool_floats(geo, B));
        if (rc) return rc;
    }

    // last of the checks and allocations: the SSB control statics of this call (committed at the end)
    SsbControl ssb_next = e->ssb;
    uint32_t nco_next = e->nco_phase;
    if (do_ssb) {
        int32_t rc = prepare_ssb(e, ssb_next, nco_next, &sp);
        if (rc) return rc;
    }

    const bool prof = e->profiling;
    const int64_t seq = e->calls_total++;
    EvSet *ev = nullptr;
    if (prof) {
        const int slot = e->ring_next;
        if (e->ring[slot].pending) {
            int32_t rc = fold_slot(e, slot);
            if (rc) return rc;
        }
        // the next slot's call measures its pipelined SSB interval from this slot's end marker, about to be reused
        const int nx = (slot + 1) % sdrg_engine::RING;
        if (e->ring[nx].pending) {
            int32_t rc = fold_slot(e, nx);
            if (rc) return rc;
        }
        ev = &e->ring[slot];
        ev->has_spec = do_spec;
        ev->has_stats = do_stats;
        ev->has_ssb = do_ssb;
        // the SSB start marker sits on the SSB stream between the fork and the pipeline; pipelined, that stream is
        // the step's critical path, so a call carries one only when its SSB time cannot be measured from the previous
        // call's SSB end marker to its own (fold_slot): the previous call (seq - 1, every enqueue counts) was not a
        // profiled SSB call of this timing window
        const EvSet &pv = e->ring[(slot + sdrg_engine::RING - 1) % sdrg_engine::RING];
        const bool chained = pv.seq == seq - 1 && pv.has_ssb && seq > e->seq_reset;
        ev->ssb_timed = do_ssb && (!(e->pipelined && !join) || !chained);
        ev->seq = seq;
        // a joined call's end marker follows the wait for the SSB stream, and asynchronous statistics end on a
        // stream of their own: the statistics get a marker of their own
        ev->stats_marked = do_stats && (!(e->pipelined && !join) || e->stats_async);
    }
    // Markers: every event recorded between two kernels of a stream costs that stream a gap (several us
    // measured), so a call records at most one at its start on the main stream (the SSB fork and the timing
    // origin), one after the spectrum (timing only), and one at the end of each stream's work (input release,
    // join, timing).  Profiling uses the ring's timing events for these; otherwise untimed ones.
    hipEvent_t mk_start = prof ? ev->t0 : e->ev_fork;
    hipEvent_t mk_main_end = prof ? ev->end : e->ev_in_main;
    hipEvent_t mk_ssb_end = prof ? ev->ssb1 : e->ev_in_ssb;
    // The spectrum kernel runs alone on the whole chip first (it is HBM-bound and persistent, two
    // workgroups per CU); the SSB pipeline (latency-bound, one workgroup per CU) then runs beside the
    // statistics kernel on a forked stream.  Measured: the same step time as running the spectrum beside
    // the SSB pipeline, with the spectrum kernel's HBM rate not diluted by the SSB workgroups.
    // Pipelined (sdrg_engine_set_pipelining): the SSB stream forks at the start of the call and is not
    // joined at its end, so this call's SSB pipeline and the next call's spectrum share the chip as the
    // other's workgroups retire (steady state measured in tools/overlap_lab.py).
    const bool early_fork = e->pipelined && !join;
    // the fork: the SSB stage waits for what the caller enqueued on the main stream before this call (its
    // producer work on iq) -- unless the caller declared its inputs complete at call time
    // (SDRG_PIPELINE_INPUTS_READY), which saves the SSB stream a cross-stream wait per call (measured ~20 us)
    const bool fork_wait = do_ssb && early_fork && !e->inputs_ready;
    if (prof || fork_wait) HIP_TRY(hipEventRecord(mk_start, e->s_main));
    if (fork_wait) HIP_TRY(hipStreamWaitEvent(e->s_ssb, mk_start, 0));
    // the spectrum / statistics stream: s_main, or the CU-split stream forked from it
    const bool split = e->s_spec && (do_spec || do_stats);
    hipStream_t sm = split ? e->s_spec : e->s_main;
    if (split) {
        HIP_TRY(hipEventRecord(e->ev_fork_spec, e->s_main));
        HIP_TRY(hipStreamWaitEvent(e->s_spec, e->ev_fork_spec, 0));
    }
    // asynchronous statistics (SDRG_PIPELINE_STATS_ASYNC): the statistics of earlier calls may still read their
    // spectra on s_stats.  The host waits for the call two before; a spectrum that overwrites the buffer the
    // previous call's statistics read waits for them on the GPU.
    const bool async = e->stats_async && early_fork && do_stats && do_spec && (!split || e->lab_stats_cus);
    if (e->stats_async && do_spec) {
        const int64_t c = e->sa_calls;
        if (c >= 2 && e->sa_live[(c - 2) % sdrg_engine::SA_RING])
            HIP_TRY(hipEventSynchronize(e->ev_stats_end[(c - 2) % sdrg_engine::SA_RING]));
        const int pv = (int)((c + sdrg_engine::SA_RING - 1) % sdrg_engine::SA_RING);
        if (c >= 1 && e->sa_live[pv] && (e->sa_spec[pv] == spec || !async))
            HIP_TRY(hipStreamWaitEvent(sm, e->ev_stats_end[pv], 0));
    }
    if (hipEvent_t g = do_spec ? e->gathering(spec, spec_bytes) : nullptr) HIP_TRY(hipStreamWaitEvent(sm, g, 0));  // being gathered
    auto enqueue_spectrum = [&]() -> int32_t {
        if (do_spec) {
            HIP_TRY(launch_spectrum(iq, fmt, n, B, e->d_twiddles, spec, e->d_fft_scratch, sm, do_ssb && early_fork && !split,
                                    split ? e->spec_cus : 0, do_stats && stats_uses_wide(geo)));
            if (prof) HIP_TRY(hipEventRecord(ev->spec, sm));
        }
        return SDRG_OK;
    };
    // host launch order (lab SDRG_SSB_FIRST=1: a forked SSB stage is enqueued before the spectrum, so on an idle chip
    // its workgroups are placed first)
    const bool ssb_first = e->lab_ssb_first && do_ssb && early_fork;
    if (!ssb_first)
        if (int32_t rc = enqueue_spectrum()) return rc;
    if (do_ssb) {  // fork
        if (!early_fork) {
            HIP_TRY(hipEventRecord(e->ev_fork, e->s_main));
            HIP_TRY(hipStreamWaitEvent(e->s_ssb, e->ev_fork, 0));
        }
        if (hipEvent_t g = e->gathering(pcm, pcm_bytes)) HIP_TRY(hipStreamWaitEvent(e->s_ssb, g, 0));  // still being gathered
        if (prof && ev->ssb_timed) HIP_TRY(hipEventRecord(ev->ssb0, e->s_ssb));
        // AudioPulseDetector::process(pcm) after processSSB_opt (ssb_processor.cpp:109): its per-sample front
        // end runs inside the SSB kernel on the PCM it produces, the detector right after
        AudioFront af;
        const int ap_set = (int)(e->ap_calls % sdrg_pulse_bank::NEW_SETS);
        if (do_ap) {
            if (e->ap_live[ap_set]) HIP_TRY(hipEventSynchronize(e->ev_ap_end[ap_set]));
            int32_t rc = pulse_bank_audio_front(&e->audio_bank, sp.pcm_len, &af, e->s_ssb, ap_set);
            if (rc) return rc;
        }
        // the SSB stream's end marker: input release (the SSB pipeline, an iq reader, is done), join, timing, and
        // the audio detector's start -- completed by the pipeline kernel's own launch where launch_ssb can
        bool end_recorded = false;
        HIP_TRY(launch_ssb(iq, fmt, B, sp, e->d_taps, e->d_chunk_table, e->d_ssb, e->d_ssb_scratch, pcm,
                           do_ap ? &af : nullptr, e->s_ssb, mk_ssb_end, &end_recorded));
        if (!end_recorded) HIP_TRY(hipEventRecord(mk_ssb_end, e->s_ssb));
        if (do_ap) {
            HIP_TRY(hipStreamWaitEvent(e->s_ap, mk_ssb_end, 0));
            int32_t rc = pulse_bank_audio_detect(&e->audio_bank, e->audio_bank.d_out, e->s_ap, ap_set);
            if (rc) return rc;
            HIP_TRY(hipEventRecord(e->ev_ap_end[ap_set], e->s_ap));
            e->ap_live[ap_set] = true;
            e->last_ap_end = e->ev_ap_end[ap_set];
            e->ap_calls++;
        }
    }
    if (ssb_first)
        if (int32_t rc = enqueue_spectrum()) return rc;
    if (do_stats) {
        hipStream_t st = sm;
        if (async) {  // after this call's spectrum, beside the next call's
            HIP_TRY(hipEventRecord(e->ev_spec_done, sm));
            HIP_TRY(hipStreamWaitEvent(e->s_stats, e->ev_spec_done, 0));
            st = e->s_stats;
        }
        if (hipEvent_t g = e->gathering(recs, rec_bytes)) HIP_TRY(hipStreamWaitEvent(st, g, 0));  // still being gathered
        HIP_TRY(launch_stats(spec, B, geo, now_ms, e->d_stats, recs, e->d_pool, st));
        if (do_sp) {  // spectralPulseDetector.process(best1kHzSnrSigma, best1kHzCenterFreqHz) (:477-479)
            int32_t rc = pulse_bank_spectral(&e->spec_bank, &recs->best1khz_snr_sigma, &recs->best1khz_center_freq_hz,
                                             (int)sizeof(sdrg_frame_record), e->spec_bank.d_out, st);
            if (rc) return rc;
        }
        if (prof && ev->stats_marked) HIP_TRY(hipEventRecord(ev->stats, st));
        if (async) {
            const int k = (int)(e->sa_calls % sdrg_engine::SA_RING);
            HIP_TRY(hipEventRecord(e->ev_stats_end[k], st));
            e->sa_spec[k] = spec;
            e->sa_live[k] = true;
            e->sa_calls++;
            e->last_stats_end = e->ev_stats_end[k];
        }
    }
    // the main stream's end marker: input release (the spectrum reads iq), timing; joined calls place it after
    // the join, so total_ms spans both streams
    if (split) {
        HIP_TRY(hipEventRecord(e->ev_join_spec, e->s_spec));
        HIP_TRY(hipStreamWaitEvent(e->s_main, e->ev_join_spec, 0));
    }
    if (do_ssb && !early_fork) {  // join
        HIP_TRY(hipStreamWaitEvent(e->s_main, mk_ssb_end, 0));
        if (do_ap) HIP_TRY(hipStreamWaitEvent(e->s_main, e->last_ap_end, 0));
    }
    if (do_spec || prof) HIP_TRY(hipEventRecord(mk_main_end, e->s_main));
    if (prof) {
        ev->pending = true;
        e->ring_last = e->ring_next;
        e->ring_next = (e->ring_next + 1) % sdrg_engine::RING;
    }
    // every launch of the call is enqueued: commit its host-side state
    if (do_ssb) {
        e->ssb = ssb_next;
        e->nco_phase = nco_next;
    }
    if (do_stats) e->cf_changed_pending = false;
    // a gathered range this call wrote whole was waited for on a stream ordered after the gathers: no longer pending
    // (ranges it wrote only in part, and the other gathered ranges, stay pending until a call writes them whole)
    const std::pair<const void *, size_t> written[] = {{do_spec ? (const void *)spec : nullptr, spec_bytes},
                                                       {do_stats ? (const void *)recs : nullptr, rec_bytes},
                                                       {do_ssb ? (const void *)pcm : nullptr, pcm_bytes}};
    for (const auto &w : written)
        if (w.first) {
            const uintptr_t lo = reinterpret_cast<uintptr_t>(w.first), hi = lo + w.second;
            e->g_bufs.erase(std::remove_if(e->g_bufs.begin(), e->g_bufs.end(),
                                           [lo, hi](const sdrg_engine::GBuf &g) { return lo <= g.lo && g.hi <= hi; }),
                            e->g_bufs.end());
        }
    if (do_spec) e->last_in_main = mk_main_end;
    if (do_ssb) e->last_in_ssb = mk_ssb_end;
    if (do_spec || do_stats) e->last_async_stats = do_stats && async;
    return SDRG_OK;
}

void dispatch_callbacks(sdrg_engine *e, int32_t stages, int pcm_len) {
    // soapyCallback order (sdr-bridge-java-soapy.cpp:458-475), then the SSB worker's pcm callback
    const sdrg_callbacks &c = e->cbs;
    const int n = e->cfg.samples_per_reading;
    for (int s = 0; s < e->n_streams; s++) {
        if (stages & SDRG_STAGE_STATS) {
            const sdrg_frame_record &r = e->h_rec[s];
            if (c.fft) c.fft(c.user, s, e->h_spec.data() + (size_t)s * n, n);
            if (c.detection_flag) c.detection_flag(c.user, s, r.detection_flag);
            if (c.mean_snr) c.mean_snr(c.user, s, r.mean_snr_db);
            if (c.mean_snr_sigma) c.mean_snr_sigma(c.user, s, r.mean_snr_sigma);
            if (c.peak_frequency) c.peak_frequency(c.user, s, r.tracking_frequency);
            if (c.peak_above_noise_mean) c.peak_above_noise_mean(c.user, s, r.peak_above_noise_mean_db);
            if (c.max_bin) c.max_bin(c.user, s, r.max_bin_snr_db, r.max_bin_snr_sigma);
            if (c.best1khz) c.best1khz(c.user, s, r.best1khz_snr_db, r.best1khz_snr_sigma);
            if (c.noise_level) c.noise_level(c.user, s, r.per_bin_mean);
            if ((stages & SDRG_STAGE_SPECTRAL_PULSE) && c.spectral_pulse) {
                const sdrg_pulse_output &o = e->h_pspec[s];
                c.spectral_pulse(c.user, s, o.input, o.live_etat, o.est_freq_hz_rounded);
            }
        }
        if ((stages & SDRG_STAGE_SSB) && c.pcm && pcm_len > 0)
            c.pcm(c.user, s, e->h_pcm.data() + (size_t)s * pcm_len, pcm_len);
        if ((stages & SDRG_STAGE_AUDIO_PULSE) && c.audio_pulse) {  // every frame (ssb_processor.cpp:109-113)
            const sdrg_pulse_output &o = e->h_paudio[s];
            c.audio_pulse(c.user, s, o.strength, o.live_etat);
        }
    }
}

}  // namespace

extern "C" {

int32_t sdrg_abi_version(void) { return SDRG_ABI_VERSION; }

const char *sdrg_last_error(void) { return g_last_error.c_str(); }

int32_t sdrg_ssb_pcm_len(int32_t n, int64_t sample_rate) {
    if (n <= 0) return 0;
    return ssb_pcm_len(n, (uint32_t)sample_rate);
}

int32_t sdrg_host_alloc(size_t bytes, void **out) {
    if (!out) return fail(SDRG_E_INVALID, "null out");
    *out = nullptr;
    if (bytes == 0) return fail(SDRG_E_INVALID, "zero-byte host allocation");
    if (hipHostMalloc(out, bytes, hipHostMallocDefault) != hipSuccess) {
        *out = nullptr;
        return fail(SDRG_E_HIP, "hipHostMalloc of %zu bytes failed", bytes);
    }
    return SDRG_OK;
}

int32_t sdrg_host_free(void *p) {
    if (p) HIP_TRY(hipHostFree(p));
    return SDRG_OK;
}

int32_t sdrg_focus_window(int64_t sample_rate, int32_t n, int32_t focus_khz, int32_t *first_bin, int32_t *n_bins) {
    if (!first_bin || !n_bins) return fail(SDRG_E_INVALID, "null output");
    if (n <= 0 || (uint32_t)sample_rate == 0 || focus_khz < 0) return fail(SDRG_E_INVALID, "bad geometry arguments");
    const StatsGeometry g = stats_geometry((uint32_t)sample_rate, 0, n, focus_khz);
    *first_bin = g.focus_lo;
    *n_bins = g.focus_len > 0 ? g.focus_len : 0;
    return SDRG_OK;
}

int32_t sdrg_ssb_design(int32_t samp_count, int64_t sample_rate, int32_t sound_mode, float *lpf, float *hp,
                        float *bp, float *taps, int32_t *n_taps) {
    if (samp_count <= 0 || (uint32_t)sample_rate == 0) return fail(SDRG_E_INVALID, "bad samp_count/sample_rate");
    SsbControl c;
    if (sound_mode == 2 || sound_mode == 0) {
        c.lowpass_bd = 2200.0f;
        c.lowpass_q = 1.2f;
    }
    const uint32_t fs = (uint32_t)sample_rate;
    if (lpf) design_lowpass((float)fs, c.lowpass_bd, c.lowpass_q, lpf);
    if (hp) design_highpass(48000.0f, 1200.0f, 0.7f, hp);
    if (bp) design_bandpass(48000.0f, 2400.0f, 0.6f, bp);
    if (taps) {
        const int nt = design_fir(samp_count, ssb_decim(fs), 0.45f, taps);
        if (n_taps) *n_taps = nt;
    }
    return SDRG_OK;
}

// Lab (SDRG_QUEUES = "dedicated_mask[,eager]"): HIP maps streams onto GPU_MAX_HW_QUEUES hardware queues, shared
// round-robin by creation order, so streams another library creates (RCCL's, at communicator init) change which engine
// streams share a queue.  dedicated_mask bit 1 main, 2 SSB, 4 statistics, 8 audio detector, 16 gathers: that stream is
// created with a full CU mask, which gives it a hardware queue of its own; eager: the statistics and gather streams are
// created with the engine instead of at first use.
struct QueuePlan {
    int dedicated = 0;
    bool eager = false;
};
static QueuePlan queue_plan() {
    static const QueuePlan q = [] {
        QueuePlan r;
        if (const char *v = lab_getenv("SDRG_QUEUES")) {
            int eg = 0;
            if (sscanf(v, "%d,%d", &r.dedicated, &eg) >= 1) r.eager = eg != 0;
        }
        return r;
    }();
    return q;
}
static hipError_t create_engine_stream(hipStream_t *s, int role_bit, int device, int prio = 0) {
    if (queue_plan().dedicated & role_bit) {
        int ncu = 0;
        hipError_t e = hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device);
        if (e != hipSuccess) return e;
        std::vector<uint32_t> m((ncu + 31) / 32, 0u);
        for (int i = 0; i < ncu; i++) m[i / 32] |= 1u << (i % 32);
        return hipExtStreamCreateWithCUMask(s, (uint32_t)m.size(), m.data());
    }
    return prio ? hipStreamCreateWithPriority(s, hipStreamNonBlocking, prio) : hipStreamCreateWithFlags(s, hipStreamNonBlocking);
}

int32_t sdrg_engine_create(const sdrg_config *cfg, int32_t n_streams, int32_t device, sdrg_engine **out) {
    if (!out) return fail(SDRG_E_INVALID, "null out");
    *out = nullptr;
    int32_t rc = validate_config(cfg);
    if (rc) return rc;
    if (n_streams <= 0) return fail(SDRG_E_INVALID, "n_streams must be > 0");
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return fail(SDRG_E_NODEVICE, "no HIP device");
    if (device < 0 || device >= count) return fail(SDRG_E_INVALID, "device %d out of range [0, %d)", device, count);
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, device));
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(SDRG_E_NODEVICE, "device %d is %s, this build targets gfx950", device, prop.gcnArchName);
    DeviceScope dscope(device);
    HIP_TRY(dscope.error());
    sdrg_engine *e = new sdrg_engine();
    e->cfg = *cfg;
    e->spec_pulse_cfg = spectral_pulse_cfg_for(*cfg);
    sdrg_pulse_config_default(SDRG_PULSE_AUDIO, &e->audio_pulse_cfg);
    e->n_streams = n_streams;
    e->device = device;
    auto cleanup = [&](int32_t code) {
        sdrg_engine_destroy(e);
        return code;
    };
    // stream priorities (lab: SDRG_STREAM_PRIO = "main,ssb" in hipDeviceGetStreamPriorityRange units; default
    // both normal)
    int prio_main = 0, prio_ssb = 0;
    if (const char *v = lab_getenv("SDRG_STREAM_PRIO")) {
        if (sscanf(v, "%d,%d", &prio_main, &prio_ssb) != 2) prio_main = prio_ssb = 0;
    }
    if (create_engine_stream(&e->s_own, 1, device, prio_main) != hipSuccess ||
        create_engine_stream(&e->s_ssb, 2, device, prio_ssb) != hipSuccess)
        return cleanup(fail(SDRG_E_HIP, "hipStreamCreate failed"));
    e->s_main = e->s_own;
    // lab: SDRG_CU_SPLIT = 1 (SSB on even CU-mask bits, spectrum/statistics on odd) or 2 (low / high half): the
    // SSB stream and the spectrum / statistics stream on disjoint CUs.  (32-stream SSB workgroups on half the CUs
    // with the spectrum on the other half measured slower than co-residency: DESIGN.md 3.3.)
    if (const char *v = lab_getenv("SDRG_CU_SPLIT")) {
        const int mode = atoi(v);
        const int ncu = prop.multiProcessorCount;
        if ((mode == 1 || mode == 2) && ncu >= 2) {
            std::vector<uint32_t> ma((ncu + 31) / 32, 0u), mb((ncu + 31) / 32, 0u);
            for (int i = 0; i < ncu; i++) {
                const bool a = mode == 1 ? (i % 2 == 0) : (i < ncu / 2);
                (a ? ma : mb)[i / 32] |= 1u << (i % 32);
            }
            if (e->s_ssb) (void)hipStreamDestroy(e->s_ssb);
            e->s_ssb = nullptr;
            if (hipExtStreamCreateWithCUMask(&e->s_ssb, (uint32_t)ma.size(), ma.data()) != hipSuccess ||
                hipExtStreamCreateWithCUMask(&e->s_spec, (uint32_t)mb.size(), mb.data()) != hipSuccess ||
                hipEventCreateWithFlags(&e->ev_fork_spec, hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&e->ev_join_spec, hipEventDisableTiming) != hipSuccess)
                return cleanup(fail(SDRG_E_HIP, "CU-masked stream creation failed"));
            e->spec_cus = ncu - ncu / 2;
        }
    }
    configure_fft(e);
    // stream-to-stream ordering events on one device: no system-scope fence needed (lab: SDRG_EVENT_FENCE=1
    // restores the default system-scope release/acquire)
    static const unsigned ev_flags = [] {
        const char *v = lab_getenv("SDRG_EVENT_FENCE");
        return (v && atoi(v) == 1) ? (unsigned)hipEventDisableTiming
                                   : (unsigned)(hipEventDisableTiming | hipEventDisableSystemFence);
    }();
    if (create_engine_stream(&e->s_ap, 8, device) != hipSuccess)
        return cleanup(fail(SDRG_E_HIP, "hipStreamCreate failed"));
    // the statistics stream is created with the engine's other streams: HIP shares GPU_MAX_HW_QUEUES hardware queues
    // among a process's streams by creation order, and created later (after another library's streams, e.g. RCCL's at
    // communicator init) it landed on the main stream's queue, where the asynchronous statistics ran in line with the
    // spectrum (rocprofv3 r5p: --process-group 0.3136 vs 0.3029 ms per step)
    if (create_engine_stream(&e->s_stats, 4, device) != hipSuccess) return cleanup(fail(SDRG_E_HIP, "hipStreamCreate failed"));
    if (const char *v = lab_getenv("SDRG_GATHER_STREAM"))
        if (atoi(v) == 1 && create_engine_stream(&e->s_gather, 16, device) != hipSuccess)
            return cleanup(fail(SDRG_E_HIP, "hipStreamCreate failed"));
    if (const char *v = lab_getenv("SDRG_SSB_FIRST")) e->lab_ssb_first = atoi(v) == 1;
    // lab: SDRG_STATS_CUS = k: the asynchronous statistics on every (ncu / k)-th CU (k CUs), the spectrum on the others
    // (a CU partition for the FFT + statistics schedule with no SSB stage: each kernel on CUs of its own)
    if (const char *v = lab_getenv("SDRG_STATS_CUS")) {
        const int k = atoi(v), ncu = prop.multiProcessorCount;
        if (k > 0 && k < ncu && !e->s_spec) {
            const int stride = ncu / k;
            std::vector<uint32_t> ms((ncu + 31) / 32, 0u), mf((ncu + 31) / 32, 0u);
            int taken = 0;
            for (int i = 0; i < ncu; i++) {
                const bool st = (i % stride == 0) && taken < k;
                taken += st;
                (st ? ms : mf)[i / 32] |= 1u << (i % 32);
            }
            (void)hipStreamDestroy(e->s_stats);
            e->s_stats = nullptr;
            if (hipExtStreamCreateWithCUMask(&e->s_stats, (uint32_t)ms.size(), ms.data()) != hipSuccess ||
                hipExtStreamCreateWithCUMask(&e->s_spec, (uint32_t)mf.size(), mf.data()) != hipSuccess ||
                hipEventCreateWithFlags(&e->ev_fork_spec, hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&e->ev_join_spec, hipEventDisableTiming) != hipSuccess)
                return cleanup(fail(SDRG_E_HIP, "CU-masked stream creation failed"));
            e->spec_cus = ncu - taken;
            e->lab_stats_cus = true;
        }
    }
    hipEvent_t *evs[] = {&e->ev_fork, &e->ev_join, &e->ev_in_main, &e->ev_in_ssb, &e->ev_ap_end[0], &e->ev_ap_end[1],
                         &e->ev_ap_end[2]};
    static_assert(sdrg_pulse_bank::NEW_SETS == 3, "ev_ap_end creation");
    for (auto p : evs)
        if (hipEventCreateWithFlags(p, ev_flags) != hipSuccess)
            return cleanup(fail(SDRG_E_HIP, "hipEventCreate failed"));
    rc = alloc_state(e);
    if (rc) return cleanup(rc);
    *out = e;
    return SDRG_OK;
}

int32_t sdrg_engine_destroy(sdrg_engine *e) {
    if (!e) return SDRG_OK;
    DeviceScope dscope(e->device);
    // the caller's stream (sdrg_engine_set_stream) must outlive the engine: synchronise it while it is set
    if (e->s_main) (void)hipStreamSynchronize(e->s_main);
    if (e->s_ssb) (void)hipStreamSynchronize(e->s_ssb);
    if (e->s_stats) (void)hipStreamSynchronize(e->s_stats);
    if (e->s_ap) (void)hipStreamSynchronize(e->s_ap);
    e->spec_bank.last_stream = e->audio_bank.last_stream = nullptr;  // drained above
    e->spec_bank.detect_stream = e->audio_bank.detect_stream = nullptr;
    void *bufs[] = {e->d_stats, e->d_ssb, e->d_twiddles, e->d_taps, e->d_nco_tab, e->d_chunk_table, e->d_ssb_scratch,
                    e->d_spec_scratch, e->d_fft_scratch, e->d_pool, e->d_rec_scratch, e->d_iq_stage, e->d_spec_stage,
                    e->d_ss_stage, e->d_rec_stage, e->d_pcm_stage, e->d_focus_stage};
    for (void *b : bufs)
        if (b) (void)hipFree(b);
    if (e->s_spec) (void)hipStreamSynchronize(e->s_spec);
    for (hipEvent_t ev : e->ev_stats_end)
        if (ev) (void)hipEventDestroy(ev);
    if (e->s_gather) (void)hipStreamSynchronize(e->s_gather);
    hipEvent_t evs[] = {e->ev_fork, e->ev_join, e->ev_in_main, e->ev_in_ssb, e->ev_fork_spec, e->ev_join_spec,
                        e->ev_spec_done, e->ev_ap_end[0], e->ev_ap_end[1], e->ev_ap_end[2]};
    for (hipEvent_t ev : evs)
        if (ev) (void)hipEventDestroy(ev);
    for (hipEvent_t ev : e->ev_g)  // ev_gather is one of these
        if (ev) (void)hipEventDestroy(ev);
    for (auto &r : e->ring) {
        hipEvent_t rev[] = {r.t0, r.spec, r.stats, r.ssb0, r.ssb1, r.end};
        for (hipEvent_t ev : rev)
            if (ev) (void)hipEventDestroy(ev);
    }
    pulse_bank_release(&e->spec_bank);  // also what a failed lazy init left behind (null-safe)
    pulse_bank_release(&e->audio_bank);
    if (e->s_own) (void)hipStreamDestroy(e->s_own);
    if (e->s_ssb) (void)hipStreamDestroy(e->s_ssb);
    if (e->s_spec) (void)hipStreamDestroy(e->s_spec);
    if (e->s_stats) (void)hipStreamDestroy(e->s_stats);
    if (e->s_ap) (void)hipStreamDestroy(e->s_ap);
    if (e->s_gather) (void)hipStreamDestroy(e->s_gather);
    delete e;
    return SDRG_OK;
}

int32_t sdrg_engine_apply_config(sdrg_engine *e, const sdrg_config *cfg) {
    if (!e) return fail(SDRG_E_INVALID, "null engine");
    int32_t rc = validate_config(cfg);
    if (rc) return rc;
    e->cfg = *cfg;  // applied at the next process call (frame boundary)
    configure_fft(e);  // fftProcessor.configure (:1123-1128)
    e->spec_pulse_cfg = spectral_pulse_cfg_for(*cfg);
    if (e->spec_bank_live) return pulse_bank_configure(&e->spec_bank, &e->spec_pulse_cfg);
    return SDRG_OK;
}

int32_t sdrg_engine_set_frequency(sdrg_engine *e, int64_t center_frequency) {
    if (!e) return fail(SDRG_E_INVALID, "null engine");
    e->cfg.center_frequency = center_frequency;
    configure_fft(e);              // :896-901
    e->cf_changed_pending = true;  // :907 isCenterFrequencyChanged = true
    return SDRG_OK;
}

int32_t sdrg_engine_set_sample_rate(sdrg_engine *e, int64_t sample_rate) {
    if (!e) return fail(SDRG_E_INVALID, "null engine");
    if ((uint32_t)sample_rate == 0) return fail(SDRG_E_INVALID, "sample_rate must be > 0");
    e->cfg.sample_rate = sample_rate;  // BridgeConfig only (:931-953): the SSB sees it at the next frame
    return SDRG_OK;
}

int32_t sdrg_engine_set_samples_per_reading(sdrg_engine *e, int32_t n) {
    if (!e) return fail(SDRG_E_INVALID, "null engine");
    if (n < 1 || n > (1 << 20)) return fail(SDRG_E_UNSUPPORTED, "samples_per_reading %d outside [1, 2^20]", n);
    e->cfg.samples_per_reading = n;  // BridgeConfig only (:1015-1021): the frames are cut at n from now on
    return SDRG_OK;
}

int32_t sdrg_engine_input_released(const sdrg_engine *e, int32_t *released) {
    if (!e || !released) return fail(SDRG_E_INVALID, "null argument");
    *released = 1;
    hipEvent_t evs[] = {e->last_in_main, e->last_in_ssb};
    for (hipEvent_t ev : evs) {
        if (!ev) continue;
        const hipError_t q = hipEventQuery(ev);
        if (q == hipErrorNotReady) {
            *released = 0;
        } else if (q != hipSuccess) {
            return fail(SDRG_E_HIP, "hipEventQuery: %s", hipGetErrorString(q));
        }
    }
    return SDRG_OK;
}

int32_t sdrg_engine_wait_input_released(sdrg_engine *e, void *hip_stream) {
    if (!e) return fail(SDRG_E_INVALID, "null engine");
    DeviceScope dscope(e->device);
    HIP_TRY(dscope.error());
    hipStream_t s = hip_stream ? static_cast<hipStream_t>(hip_stream) : e->s_main;
    if (e->last_in_main && s != e->s_main) HIP_TRY(hipStreamWaitEvent(s, e->last_in_main, 0));
    if (e->last_in_ssb) HIP_TRY(hipStreamWaitEvent(s, e->last_in_ssb, 0));
    return SDRG_OK;
}

int32_t sdrg_engine_wait_outputs(sdrg_engine *e, void *hip_stream) {
    if (!e) return fail(SDRG_E_INVALID, "null engine");
    DeviceScope dscope(e->device);
    HIP_TRY(dscope.error());
    hipStream_t s = hip_stream ? static_cast<hipStream_t>(hip_stream) : e->s_main;
    if (e->last_in_main && s != e->s_main) HIP_TRY(hipStreamWaitEvent(s, e->last_in_main, 0));  // spectra
    if (e->last_in_ssb) HIP_TRY(hipStreamWaitEvent(s, e->last_in_ssb, 0));                    // PCM
    if (e->last_ap_end) HIP_TRY(hipStreamWaitEvent(s, e->last_ap_end, 0));                    // audio pulse
    if (e->stats_async && e->last_stats_end) HIP_TRY(hipStreamWaitEvent(s, e->last_stats_end, 0));  // records
    if (e->ev_gather) HIP_TRY(hipStreamWaitEvent(s, e->ev_gather, 0));  // the gathered outputs on the root
    return SDRG_OK;
}

int32_t sdrg_engine_set_frequency_focus_range(sdrg_engine *e, int32_t khz) {
    if (!e) return fail(SDRG_E_INVALID, "null engine");
    if (khz < 0) return fail(SDRG_E_INVALID, "focus range must be >= 0");
    e->cfg.freq_focus_range_khz = khz;
    configure_fft(e);  // :1031-1036
    return SDRG_OK;
}

int32_t sdrg_engine_set_sound_mode(sdrg_engine *e, int32_t mode) {
    if (!e) return fail(SDRG_E_INVALID, "null engine");
    e->cfg.sound_mode = mode;
    return SDRG_OK;
}

int32_t sdrg_engine_set_upper_sideband(sdrg_engine *e, int32_t upper) {
    if (!e) return fail(SDRG_E_INVALID, "null engine");
    e->upper = upper ? 1 : 0;
    return SDRG_OK;
}

int32_t sdrg_engine_set_ssb_variant(sdrg_engine *e, double nco_hz, int32_t fir_taps) {
    if (!e) return fail(SDRG_E_INVALID, "null engine");
    if (fir_taps != 0 && (fir_taps < 3 || fir_taps > 255 || (fir_taps & 1) == 0))
        return fail(SDRG_E_INVALID, "fir_taps must be 0 or odd in [3, 255], got %d", fir_taps);
    if (!std::isfinite(nco_hz)) return fail(SDRG_E_INVALID, "nco_hz must be finite");
    DeviceScope dscope(e->device);
    HIP_TRY(dscope.error());
    HIP_TRY(hipStreamSynchronize(e->s_ssb));  // in-flight SSB kernels read the taps being replaced
    e->nco_hz = nco_hz;
    e->fir_taps = fir_taps;
    e->nco_phase = 0;
    return SDRG_OK;
}

int32_t sdrg_engine_get_ssb_variant(const sdrg_engine *e, double *nco_hz, int32_t *fir_taps,
                                    uint32_t *nco_increment_out, uint32_t *nco_phase) {
    if (!e) return fail(SDRG_E_INVALID, "null engine");
    if (nco_hz) *nco_hz = e->nco_hz;
    if (fir_taps) *fir_taps = ssb_taps_for(ssb_frozen_or(e), e->fir_taps);
    if (nco_increment_out) *nco_increment_out = e->nco_hz != 0.0 ? nco_increment(e->nco_hz, (uint32_t)e->cfg.sample_rate) : 0;
    if (nco_phase) *nco_phase = e->nco_phase;
    return SDRG_OK;
}

int32_t sdrg_engine_get_config(const sdrg_engine *e, sdrg_config *out) {
    if (!e || !out) return fail(SDRG_E_INVALID, "null argument");
    *out = e->cfg;
    return SDRG_OK;
}

int32_t sdrg_engine_n_streams(const sdrg_engine *e) { return e ? e->n_streams : 0; }

int32_t sdrg_engine_pcm_len(const sdrg_engine *e) {
    if (!e) return 0;
    return ssb_pcm_len(ssb_frozen_or(e), (uint32_t)e->cfg.sample_rate, e->fir_taps);
}

int32_t sdrg_engine_reset_state(sdrg_engine *e) {
    if (!e) return fail(SDRG_E_INVALID, "null engine");
    DeviceScope dscope(e->device);
    HIP_TRY(dscope.error());
    HIP_TRY(hipStreamSynchronize(e->s_main));
    HIP_TRY(hipStreamSynchronize(e->s_ssb));
    if (e->s_stats) HIP_TRY(hipStreamSynchronize(e->s_stats));
    HIP_TRY(hipStreamSynchronize(e->s_ap));
    HIP_TRY(memset_sync(e->d_stats, 0, sizeof(StatsState) * (size_t)e->n_streams));
    HIP_TRY(memset_sync(e->d_ssb, 0, sizeof(SsbStreamState) * (size_t)e->n_streams));
    e->ssb = SsbControl{};
    e->nco_phase = 0;
    e->cf_changed_pending = false;
    e->spec_bank.reset_pending = true;
    e->audio_bank.reset_pending = true;
    return SDRG_OK;
}

int32_t sdrg_engine_set_pipelining(sdrg_engine *e, int32_t on) {
    if (!e) return fail(SDRG_E_INVALID, "null engine");
    DeviceScope dscope(e->device);
    HIP_TRY(dscope.error());
    const int mode = on & ~SDRG_PIPELINE_STATS_ASYNC;
    const bool async = (on & SDRG_PIPELINE_STATS_ASYNC) != 0;
    if ((mode != SDRG_PIPELINE_OFF && mode != SDRG_PIPELINE_ON && mode != SDRG_PIPELINE_INPUTS_READY) ||
        (async && mode == SDRG_PIPELINE_OFF))
        return fail(SDRG_E_INVALID, "pipelining mode must be 0, 1 or 2 (1 or 2 may add SDRG_PIPELINE_STATS_ASYNC), got %d",
                    on);
    if (e->pipelined && !mode) {  // re-join what is in flight so later work on s_main follows it
        HIP_TRY(hipEventRecord(e->ev_join, e->s_ssb));
        HIP_TRY(hipStreamWaitEvent(e->s_main, e->ev_join, 0));
        if (e->last_ap_end) HIP_TRY(hipStreamWaitEvent(e->s_main, e->last_ap_end, 0));
    }
    if (e->stats_async && !async && e->last_stats_end)  // the asynchronous statistics in flight, likewise
        HIP_TRY(hipStreamWaitEvent(e->s_main, e->last_stats_end, 0));
    if (async) {  // created lazily, each handle on its own: a failed earlier attempt leaves no null behind in use
        const unsigned fl = hipEventDisableTiming | hipEventDisableSystemFence;
        if (!e->s_stats) HIP_TRY(create_engine_stream(&e->s_stats, 4, e->device));
        if (!e->ev_spec_done) HIP_TRY(hipEventCreateWithFlags(&e->ev_spec_done, fl));
        for (hipEvent_t &ev : e->ev_stats_end)
            if (!ev) HIP_TRY(hipEventCreateWithFlags(&ev, fl));
    }
    e->pipelined = mode != SDRG_PIPELINE_OFF;
    e->inputs_ready = mode == SDRG_PIPELINE_INPUTS_READY;
    e->stats_async = async;
    return SDRG_OK;
}

int32_t sdrg_engine_set_stream(sdrg_engine *e, void *hip_stream) {
    if (!e) return fail(SDRG_E_INVALID, "null engine");
    DeviceScope dscope(e->device);
    HIP_TRY(dscope.error());
    HIP_TRY(hipStreamSynchronize(e->s_main));  // work already enqueued stays ordered before the switch
    e->s_main = hip_stream ? static_cast<hipStream_t>(hip_stream) : e->s_own;
    return SDRG_OK;
}

int32_t sdrg_engine_set_spectral_pulse_config(sdrg_engine *e, const sdrg_pulse_config *cfg) {
    if (!e) return fail(SDRG_E_INVALID, "null engine");
    int32_t rc = pulse_config_check(SDRG_PULSE_SPECTRAL, cfg);
    if (rc) return rc;
    e->spec_pulse_cfg = *cfg;
    if (e->spec_bank_live) return pulse_bank_configure(&e->spec_bank, cfg);
    return SDRG_OK;
}

int32_t sdrg_engine_set_audio_pulse_config(sdrg_engine *e, const sdrg_pulse_config *cfg) {
    if (!e) return fail(SDRG_E_INVALID, "null engine");
    int32_t rc = pulse_config_check(SDRG_PULSE_AUDIO, cfg);
    if (rc) return rc;
    e->audio_pulse_cfg = *cfg;
    if (e->audio_bank_live) return pulse_bank_configure(&e->audio_bank, cfg);
    return SDRG_OK;
}

int32_t sdrg_engine_pulse_outputs(const sdrg_engine *e, const sdrg_pulse_output **spectral,
                                  const sdrg_pulse_output **audio) {
    if (!e) return fail(SDRG_E_INVALID, "null engine");
    if (spectral) *spectral = e->spec_bank_live ? e->spec_bank.d_out : nullptr;
    if (audio) *audio = e->audio_bank_live ? e->audio_bank.d_out : nullptr;
    return SDRG_OK;
}

int32_t sdrg_engine_get_pulse_outputs(sdrg_engine *e, sdrg_pulse_output *spectral, sdrg_pulse_output *audio) {
    if (!e) return fail(SDRG_E_INVALID, "null engine");
    DeviceScope dscope(e->device);
    HIP_TRY(dscope.error());
    HIP_TRY(hipStreamSynchronize(e->s_main));
    HIP_TRY(hipStreamSynchronize(e->s_ssb));
    if (e->s_stats) HIP_TRY(hipStreamSynchronize(e->s_stats));
    HIP_TRY(hipStreamSynchronize(e->s_ap));
    const size_t bytes = sizeof(sdrg_pulse_output) * (size_t)e->n_streams;
    if (spectral) {
        if (!e->spec_bank_live) return fail(SDRG_E_INVALID, "the spectral pulse stage has not run");
        HIP_TRY(hipMemcpy(spectral, e->spec_bank.d_out, bytes, hipMemcpyDeviceToHost));
    }
    if (audio) {
        if (!e->audio_bank_live) return fail(SDRG_E_INVALID, "the audio pulse stage has not run");
        HIP_TRY(hipMemcpy(audio, e->audio_bank.d_out, bytes, hipMemcpyDeviceToHost));
    }
    return SDRG_OK;
}

int32_t sdrg_engine_process_device(sdrg_engine *e, const void *iq, int32_t format, int32_t stages, float *spectra,
                                   sdrg_frame_record *records, int16_t *pcm, int64_t now_ms) {
    if (!e) return fail(SDRG_E_INVALID, "null engine");
    DeviceScope dscope(e->device);
    HIP_TRY(dscope.error());
    return enqueue(e, iq, format, stages, spectra, records, pcm, now_ms, false);
}

// evaluateSignalStrength (fft_process.cpp:122-379) on spectra the caller supplies: the FFTProcessor's
// power_shifted member in, the getters' values out, the stream state (tracking latch, detection ring, stale
// outputs) carried exactly as a process() call carries it.  Ordered on the main stream.
static int32_t signal_strength(sdrg_engine *e, const float *spectra, sdrg_frame_record *records, int64_t now_ms) {
    const int n = e->cfg.samples_per_reading, B = e->n_streams;
    if (e->fft_fs == 0) return fail(SDRG_E_INVALID, "the statistics' sample rate is 0");
    StatsGeometry geo = stats_geometry(e->fft_fs, e->fft_fc, n, e->fft_focus);
    geo.cf_changed = e->cf_changed_pending ? 1 : 0;
    int32_t rc = ensure_device(&e->d_pool, &e->pool_elems, stats_global_pool_floats(geo, B));
    if (rc) return rc;
    // asynchronous statistics of an earlier pipelined call (SDRG_PIPELINE_STATS_ASYNC) may still run on s_stats and
    // read / write the same stream state (d_stats) and pool scratch: this launch follows them
    if (e->stats_async && e->last_stats_end) HIP_TRY(hipStreamWaitEvent(e->s_main, e->last_stats_end, 0));
    HIP_TRY(launch_stats(spectra, B, geo, now_ms, e->d_stats, records, e->d_pool, e->s_main));
    e->cf_changed_pending = false;
    return SDRG_OK;
}

int32_t sdrg_engine_signal_strength_device(sdrg_engine *e, const float *spectra, sdrg_frame_record *records,
                                           int64_t now_ms) {
    if (!e) return fail(SDRG_E_INVALID, "null engine");
    if (!spectra || !records) return fail(SDRG_E_INVALID, "null spectra or records");
    DeviceScope dscope(e->device);
    HIP_TRY(dscope.error());
    return signal_strength(e, spectra, records, now_ms);
}

int32_t sdrg_engine_signal_strength_host(sdrg_engine *e, const float *spectra, sdrg_frame_record *records,
                                         int64_t now_ms) {
    if (!e) return fail(SDRG_E_INVALID, "null engine");
    if (!spectra || !records) return fail(SDRG_E_INVALID, "null spectra or records");
    DeviceScope dscope(e->device);
    HIP_TRY(dscope.error());
    const int n = e->cfg.samples_per_reading, B = e->n_streams;
    // a staging buffer of its own: process_host's d_spec_stage carries each stream's never-written bin N-1 for odd N
    // (fft_process.cpp:92-97), which the caller's spectra must not replace
    int32_t rc = ensure_device(&e->d_ss_stage, &e->ss_stage_elems, (size_t)B * n);
    if (rc) return rc;
    if (!e->d_rec_stage)
        HIP_TRY(hipMalloc(reinterpret_cast<void **>(&e->d_rec_stage), sizeof(sdrg_frame_record) * (size_t)B));
    HIP_TRY(hipMemcpyAsync(e->d_ss_stage, spectra, sizeof(float) * (size_t)B * n, hipMemcpyHostToDevice, e->s_main));
    rc = signal_strength(e, e->d_ss_stage, e->d_rec_stage, now_ms);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(records, e->d_rec_stage, sizeof(sdrg_frame_record) * (size_t)B, hipMemcpyDeviceToHost,
                           e->s_main));
    HIP_TRY(hipStreamSynchronize(e->s_main));
    return SDRG_OK;
}

int32_t sdrg_engine_synchronize(sdrg_engine *e) {
    if (!e) return fail(SDRG_E_INVALID, "null engine");
    HIP_TRY(hipStreamSynchronize(e->s_main));
    HIP_TRY(hipStreamSynchronize(e->s_ssb));  // not joined into s_main when pipelined
    if (e->s_stats) HIP_TRY(hipStreamSynchronize(e->s_stats));  // SDRG_PIPELINE_STATS_ASYNC
    HIP_TRY(hipStreamSynchronize(e->s_ap));                      // the audio pulse detector
    if (e->s_gather) HIP_TRY(hipStreamSynchronize(e->s_gather));
    static const bool stamps = [] {
        const char *v = lab_getenv("SDRG_PIPE_STAMPS");
        return v && v[0] == '1';
    }();
    if (stamps) ssb_report_stamps();
    return SDRG_OK;
}

int32_t sdrg_engine_process_host(sdrg_engine *e, const void *iq, int32_t format, int32_t stages, float *spectra,
                                 sdrg_frame_record *records, int16_t *pcm, int64_t now_ms) {
    if (!e) return fail(SDRG_E_INVALID, "null engine");
    if (!iq) return fail(SDRG_E_INVALID, "null iq");
    const int bps = bytes_per_sample(format);
    if (!bps) return fail(SDRG_E_INVALID, "unknown iq format %d", format);
    DeviceScope dscope(e->device);
    HIP_TRY(dscope.error());
    const int n = e->cfg.samples_per_reading;
    const int B = e->n_streams;
    const size_t iq_bytes = (size_t)B * n * bps;
    if (e->iq_stage_bytes < iq_bytes) {
        size_t have = e->iq_stage_bytes;
        char *p = static_cast<char *>(e->d_iq_stage);
        int32_t rc = ensure_device(&p, &have, iq_bytes);
        if (rc) return rc;
        e->d_iq_stage = p;
        e->iq_stage_bytes = have;
    }
    const bool want_cb = e->has_cbs;
    const bool do_spec = stages & SDRG_STAGE_SPECTRUM, do_stats = stages & SDRG_STAGE_STATS,
               do_ssb = stages & SDRG_STAGE_SSB;
    if (do_spec) {
        int32_t rc = ensure_device(&e->d_spec_stage, &e->spec_stage_elems, (size_t)B * n, true);  // see enqueue
        if (rc) return rc;
    }
    if (do_stats && !e->d_rec_stage)
        HIP_TRY(hipMalloc(reinterpret_cast<void **>(&e->d_rec_stage), sizeof(sdrg_frame_record) * (size_t)B));
    int pcm_len = 0;
    if (do_ssb) {
        // pcm length is known before the call: frozen (or about-to-be frozen) size and current fs
        pcm_len = ssb_pcm_len(ssb_frozen_or(e), (uint32_t)e->cfg.sample_rate, e->fir_taps);
        int32_t rc = ensure_device(&e->d_pcm_stage, &e->pcm_stage_elems, (size_t)B * (pcm_len > 0 ? pcm_len : 1));
        if (rc) return rc;
    }
    HIP_TRY(hipMemcpyAsync(e->d_iq_stage, iq, iq_bytes, hipMemcpyHostToDevice, e->s_main));
    int32_t rc = enqueue(e, e->d_iq_stage, format, stages, do_spec ? e->d_spec_stage : nullptr,
                         do_stats ? e->d_rec_stage : nullptr, do_ssb ? e->d_pcm_stage : nullptr, now_ms, true);
    if (rc) return rc;
    float *h_spec = spectra;
    sdrg_frame_record *h_rec = records;
    int16_t *h_pcm = pcm;
    if (want_cb) {
        if ((do_spec && !e->h_spec.resize((size_t)B * n)) || (do_stats && !e->h_rec.resize(B)) ||
            (do_ssb && !e->h_pcm.resize((size_t)B * std::max(pcm_len, 1))) ||
            ((stages & SDRG_STAGE_SPECTRAL_PULSE) && !e->h_pspec.resize(B)) ||
            ((stages & SDRG_STAGE_AUDIO_PULSE) && !e->h_paudio.resize(B)))
            return fail(SDRG_E_HIP, "hipHostMalloc failed for the callback copies");
        if (do_spec && !h_spec) h_spec = e->h_spec.data();
        if (do_stats && !h_rec) h_rec = e->h_rec.data();
        if (do_ssb && !h_pcm) h_pcm = e->h_pcm.data();
    }
    if (do_spec && h_spec)
        HIP_TRY(hipMemcpyAsync(h_spec, e->d_spec_stage, sizeof(float) * (size_t)B * n, hipMemcpyDeviceToHost, e->s_main));
    if (do_stats && h_rec)
        HIP_TRY(hipMemcpyAsync(h_rec, e->d_rec_stage, sizeof(sdrg_frame_record) * (size_t)B, hipMemcpyDeviceToHost,
                               e->s_main));
    if (do_ssb && h_pcm && pcm_len > 0)
        HIP_TRY(hipMemcpyAsync(h_pcm, e->d_pcm_stage, sizeof(int16_t) * (size_t)B * pcm_len, hipMemcpyDeviceToHost,
                               e->s_main));
    if (want_cb && (stages & SDRG_STAGE_SPECTRAL_PULSE)) {
        HIP_TRY(hipMemcpyAsync(e->h_pspec.data(), e->spec_bank.d_out, sizeof(sdrg_pulse_output) * (size_t)B,
                               hipMemcpyDeviceToHost, e->s_main));
    }
    if (want_cb && (stages & SDRG_STAGE_AUDIO_PULSE)) {
        HIP_TRY(hipMemcpyAsync(e->h_paudio.data(), e->audio_bank.d_out, sizeof(sdrg_pulse_output) * (size_t)B,
                               hipMemcpyDeviceToHost, e->s_main));
    }
    HIP_TRY(hipStreamSynchronize(e->s_main));
    if (want_cb) {
        // callbacks read the engine-owned host copies; make sure they hold this call's data
        if (do_spec && h_spec != e->h_spec.data()) e->h_spec.assign(h_spec, h_spec + (size_t)B * n);
        if (do_stats && h_rec != e->h_rec.data()) e->h_rec.assign(h_rec, h_rec + B);
        if (do_ssb && h_pcm != e->h_pcm.data() && pcm_len > 0) e->h_pcm.assign(h_pcm, h_pcm + (size_t)B * pcm_len);
        dispatch_callbacks(e, stages, pcm_len);
    }
    return SDRG_OK;
}

int32_t sdrg_engine_set_callbacks(sdrg_engine *e, const sdrg_callbacks *cbs) {
    if (!e) return fail(SDRG_E_INVALID, "null engine");
    if (cbs) {
        e->cbs = *cbs;
        e->has_cbs = true;
    } else {
        e->cbs = sdrg_callbacks{};
        e->has_cbs = false;
    }
    return SDRG_OK;
}

int32_t sdrg_engine_set_profiling(sdrg_engine *e, int32_t enabled) {
    if (!e) return fail(SDRG_E_INVALID, "null engine");
    DeviceScope dscope(e->device);
    HIP_TRY(dscope.error());
    if (enabled && !e->ring_created) {
        for (auto &r : e->ring) {
            // timing only: no system-scope fence (its cache writeback would widen the gaps it measures)
            hipEvent_t *rev[] = {&r.t0, &r.spec, &r.stats, &r.ssb0, &r.ssb1, &r.end};
            for (hipEvent_t *p : rev) HIP_TRY(hipEventCreateWithFlags(p, hipEventDisableSystemFence));
        }
        e->ring_created = true;
    }
    // calls made while profiling was off break the chain of SSB end markers (their seqs are not profiled), so the first
    // profiled call after re-enabling takes a start marker of its own (enqueue's `chained`)
    e->profiling = enabled != 0;
    return SDRG_OK;
}

int32_t sdrg_engine_get_timings(const sdrg_engine *ce, sdrg_timings *out) {
    if (!ce || !out) return fail(SDRG_E_INVALID, "null argument");
    sdrg_engine *e = const_cast<sdrg_engine *>(ce);
    if (e->ring_last < 0) return fail(SDRG_E_INVALID, "no profiled call yet");
    int32_t rc = fold_slot(e, e->ring_last);
    if (rc) return rc;
    *out = e->last_timings;
    return SDRG_OK;
}

int32_t sdrg_engine_get_timing_stats(const sdrg_engine *ce, sdrg_timings *mean, int32_t *count) {
    if (!ce || !mean) return fail(SDRG_E_INVALID, "null argument");
    sdrg_engine *e = const_cast<sdrg_engine *>(ce);
    int32_t rc = fold_all(e);
    if (rc) return rc;
    const double k = e->n_acc > 0 ? 1.0 / e->n_acc : 0.0;
    mean->spectrum_ms = (float)(e->sum_spec * k);
    mean->stats_ms = (float)(e->sum_stats * k);
    mean->ssb_ms = (float)(e->n_ssb > 0 ? e->sum_ssb / e->n_ssb : 0.0);
    mean->total_ms = (float)(e->sum_total * k);
    if (count) *count = e->n_acc;
    return SDRG_OK;
}

// Multi-GPU gather (include/sdrg.h; dist.cpp holds RCCL).  A gather runs on the stream that produced what it reads, in
// order behind it and with no cross-stream wait: the statistics stream when the last call ran its statistics there
// (records, and the spectra its statistics already waited for), else the main stream; with PCM, the audio detector's
// stream, which follows the SSB stream's end marker, waiting for the main or statistics stream's last marker.  (On a
// stream of its own the gather's waits shared a hardware queue with the engine's streams: HIP maps a process's streams
// onto GPU_MAX_HW_QUEUES queues, and a wait blocks the whole queue.)  A later call that writes a buffer a gather reads
// waits for that gather's event first (enqueue).
int32_t sdrg_engine_gather(sdrg_engine *e, sdrg_dist *d, int32_t root, const sdrg_gather_buffers *b) {
    if (!e || !d || !b) return fail(SDRG_E_INVALID, "null argument");
    if (dist_device(d) != e->device)
        return fail(SDRG_E_INVALID, "communicator on device %d, engine on device %d", dist_device(d), e->device);
    if (root < 0 || root >= dist_world(d)) return fail(SDRG_E_INVALID, "root %d outside [0, %d)", root, dist_world(d));
    DeviceScope dscope(e->device);
    HIP_TRY(dscope.error());
    const bool at_root = dist_rank(d) == root;
    const size_t B = (size_t)e->n_streams;
    const int n = e->cfg.samples_per_reading;
    const int plen = ssb_pcm_len(ssb_frozen_or(e), (uint32_t)e->cfg.sample_rate, e->fir_taps);
    const bool g_rec = b->records, g_foc = b->focus_spectra, g_spec = b->spectra, g_pcm = b->pcm && plen > 0;
    if ((g_rec && at_root && !b->records_out) || (g_foc && at_root && !b->focus_out) ||
        (g_spec && at_root && !b->spectra_out) || (g_pcm && at_root && !b->pcm_out))
        return fail(SDRG_E_INVALID, "null output buffer on the root");
    StatsGeometry geo{};
    if (g_foc) {
        geo = stats_geometry(e->fft_fs, e->fft_fc, n, e->fft_focus);
        if (geo.focus_len <= 0) return fail(SDRG_E_INVALID, "the focus window is empty (focus wider than the band)");
        int32_t rc = ensure_device(&e->d_focus_stage, &e->focus_stage_elems, B * (size_t)geo.focus_len);
        if (rc) return rc;
    }
    if (!(g_rec || g_foc || g_spec || g_pcm)) return SDRG_OK;
    const int slot = (int)(e->g_calls % sdrg_engine::GRING);
    if (!e->ev_g[slot]) HIP_TRY(hipEventCreateWithFlags(&e->ev_g[slot], hipEventDisableTiming | hipEventDisableSystemFence));
    const bool on_stats = !g_pcm && e->last_async_stats && !e->s_gather;
    hipStream_t s = e->s_gather ? e->s_gather : g_pcm ? e->s_ap : on_stats ? e->s_stats : e->s_main;
    if (e->s_gather) {  // lab: waits for every producer
        if ((g_rec || g_foc || g_spec) && e->last_in_main) HIP_TRY(hipStreamWaitEvent(s, e->last_in_main, 0));
        if (g_rec && e->last_stats_end) HIP_TRY(hipStreamWaitEvent(s, e->last_stats_end, 0));
        if (g_pcm && e->last_in_ssb) HIP_TRY(hipStreamWaitEvent(s, e->last_in_ssb, 0));
    } else if (g_pcm) {
        if ((g_rec || g_foc || g_spec) && e->last_in_main) HIP_TRY(hipStreamWaitEvent(s, e->last_in_main, 0));
        if (g_rec && e->last_stats_end) HIP_TRY(hipStreamWaitEvent(s, e->last_stats_end, 0));  // any async records
        if (e->last_in_ssb) HIP_TRY(hipStreamWaitEvent(s, e->last_in_ssb, 0));
    }
    // records an earlier call's asynchronous statistics wrote (the last call ran no statistics there)
    if (!e->s_gather && !g_pcm && !on_stats && g_rec && e->last_stats_end)
        HIP_TRY(hipStreamWaitEvent(s, e->last_stats_end, 0));
    // the focus staging buffer and RCCL's issue order: a gather follows the previous one even on another stream
    if (e->ev_gather && s != e->s_last_gather) HIP_TRY(hipStreamWaitEvent(s, e->ev_gather, 0));
    e->s_last_gather = s;
    GatherItem items[4];
    int k = 0;
    if (g_rec) items[k++] = {b->records, b->records_out, B * sizeof(sdrg_frame_record)};
    if (g_foc) {
        HIP_TRY(launch_focus_pack(b->focus_spectra, (int)B, n, geo.focus_lo, geo.focus_len, e->d_focus_stage, s));
        items[k++] = {e->d_focus_stage, b->focus_out, B * (size_t)geo.focus_len * sizeof(float)};
    }
    if (g_spec) items[k++] = {b->spectra, b->spectra_out, B * (size_t)n * sizeof(float)};
    if (g_pcm) items[k++] = {b->pcm, b->pcm_out, B * (size_t)plen * sizeof(int16_t)};
    int32_t rc = dist_gather(d, items, k, root, s);
    if (rc) return rc;
    HIP_TRY(hipEventRecord(e->ev_g[slot], s));
    e->ev_gather = e->ev_g[slot];
    e->g_calls++;
    // the buffers this gather reads, mapped to its slot; a slot re-recorded by a later gather still covers this one
    // (gathers follow each other)
    const std::pair<const void *, size_t> read[] = {
        {g_rec ? (const void *)b->records : nullptr, B * sizeof(sdrg_frame_record)},
        {g_foc ? (const void *)b->focus_spectra : nullptr, B * (size_t)n * sizeof(float)},
        {g_spec ? (const void *)b->spectra : nullptr, B * (size_t)n * sizeof(float)},
        {g_pcm ? (const void *)b->pcm : nullptr, B * (size_t)plen * sizeof(int16_t)}};
    for (const auto &r : read) {
        if (!r.first || !r.second) continue;
        const uintptr_t lo = reinterpret_cast<uintptr_t>(r.first), hi = lo + r.second;
        bool found = false;
        for (sdrg_engine::GBuf &g : e->g_bufs)
            if (g.lo == lo && g.hi == hi) g.slot = slot, g.seq = e->g_calls - 1, found = true;
        if (!found) e->g_bufs.push_back({lo, hi, slot, e->g_calls - 1});
    }
    return SDRG_OK;
}

int32_t sdrg_engine_gather_records(sdrg_engine *e, sdrg_dist *d, int32_t root, const sdrg_frame_record *records,
                                   sdrg_frame_record *records_out) {
    if (!records) return fail(SDRG_E_INVALID, "null records");
    sdrg_gather_buffers b{};
    b.records = records;
    b.records_out = records_out;
    return sdrg_engine_gather(e, d, root, &b);
}

int32_t sdrg_engine_gather_focus(sdrg_engine *e, sdrg_dist *d, int32_t root, const float *spectra, float *focus_out) {
    if (!spectra) return fail(SDRG_E_INVALID, "null spectra");
    sdrg_gather_buffers b{};
    b.focus_spectra = spectra;
    b.focus_out = focus_out;
    return sdrg_engine_gather(e, d, root, &b);
}

int32_t sdrg_engine_gather_spectra(sdrg_engine *e, sdrg_dist *d, int32_t root, const float *spectra,
                                   float *spectra_out) {
    if (!spectra) return fail(SDRG_E_INVALID, "null spectra");
    sdrg_gather_buffers b{};
    b.spectra = spectra;
    b.spectra_out = spectra_out;
    return sdrg_engine_gather(e, d, root, &b);
}

int32_t sdrg_engine_gather_pcm(sdrg_engine *e, sdrg_dist *d, int32_t root, const int16_t *pcm, int16_t *pcm_out) {
    if (!pcm) return fail(SDRG_E_INVALID, "null pcm");
    sdrg_gather_buffers b{};
    b.pcm = pcm;
    b.pcm_out = pcm_out;
    return sdrg_engine_gather(e, d, root, &b);
}

int32_t sdrg_engine_reset_timing_stats(sdrg_engine *e) {
    if (!e) return fail(SDRG_E_INVALID, "null engine");
    int32_t rc = fold_all(e);
    if (rc) return rc;
    e->sum_spec = e->sum_stats = e->sum_ssb = e->sum_total = 0;
    e->n_acc = e->n_ssb = 0;
    // a pipelined call's SSB interval starts at the previous call's end marker: the window's first call has none
    e->seq_reset = e->calls_total;
    return SDRG_OK;
}

}  // extern "C"

// pulse.hip — the beacon pulse detectors, one wavefront per stream per frame.
//
// Replaces, for a batch of independent streams,
//   SpectralPulseDetector::process(snrSigma, freqHz)   src/dsp/spectral_pulse_detector.cpp:10-143
//   AudioPulseDetector::process(pcm)                   src/ssb/audio_pulse_detector.cpp:92-237
// plus their liveEtat / toLevel / estimatedFreqHz getters (spectral :147-170, audio :241-256).
//
// The detectors are serial state machines over an energy sequence (one value per FFT frame, or one RMS
// value per 10 ms of audio).  Per stream the state sits in HBM (PulseStreamState + rings, sdrg_types.h)
// and a wavefront advances it by one call's worth of input.  The scalar state machine runs uniformly in
// every lane in the reference's float operation order (FP contraction off, IEEE division and sqrt); the
// lanes only split the order-free work: the local-maximum test over the +-idx_z window (any neighbour >=),
// the live-state sum (integer-valued floats, exact in any order) and the ROI trim search.  The two
// order-sensitive sums (the audio noise reference and the double-precision frequency regression) are
// loaded across lanes and then accumulated sequentially through readlane.  The audio front end
// (band-pass biquads, per-frame RMS, energy low-pass) is a first-order recurrence per sample and runs
// one lane per stream in its own kernel, ahead of the audio detector kernel.
//
// Ring writes are made by lane 0 and read back by the whole wave after __syncthreads() (one-wave
// workgroups: a waitcnt plus a trivial barrier).
#include "pulse_front.h"
#include "sdrg_internal.h"

#pragma clang fp contract(off)

namespace sdrg {
namespace {

constexpr int WAVE = 64;

struct Rings {
    float *e, *f;   // eBuf_, freqBuf_ (f unused for audio)
    float *rt;      // rois_[k].t
    int *re;        // rois_[k].etat
    float *ft, *ff; // freqHistory_ (t, freqHz), PULSE_FH_SLOTS slots
};

// Field-wise copies of the detector part of the state: whole-struct copies of the register-resident state
// leave parts of it in scratch.
#define SDRG_PULSE_FIELDS(X)                                                                                  \
    X(ols_a) X(ols_b) X(head) X(n) X(t0) X(last_scan) X(t_last_roi) X(locked) X(t_target) X(live_etat)        \
    X(last_snr) X(level) X(roi_head) X(n_rois) X(n_last3) X(n_hist) X(last3[0]) X(last3[1]) X(last3[2])        \
    X(hist_dts[0]) X(hist_dts[1]) X(hist_dts[2]) X(hist_dts[3]) X(hist_dts[4]) X(hist_n[0]) X(hist_n[1])        \
    X(hist_n[2]) X(hist_n[3]) X(hist_n[4]) X(fh_head) X(n_fh) X(ols_mode) X(ols_mean) X(overflow)
// (the audio front-end fields band_z / low_z / frame_count / frame_acc belong to audio_front_kernel)

__device__ __forceinline__ void load_state(PulseStreamState &s, const PulseStreamState *__restrict__ g) {
#define SDRG_LD(f) s.f = g->f;
    SDRG_PULSE_FIELDS(SDRG_LD)
#undef SDRG_LD
}

__device__ __forceinline__ void store_state(PulseStreamState *__restrict__ g, const PulseStreamState &s) {
#define SDRG_ST(f) g->f = s.f;
    SDRG_PULSE_FIELDS(SDRG_ST)
#undef SDRG_ST
}

__device__ __forceinline__ float bcast(float v, int k) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), k));
}

__device__ __forceinline__ uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }

__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
    for (int off = WAVE / 2; off > 0; off >>= 1) v += __shfl_xor(v, off, WAVE);
    return v;
}

// bounded deque push_back + pop_front when over N, on a register array (constant indices only)
template <int N, typename T>
__device__ __forceinline__ void push_bounded(T (&a)[N], int &n, T v) {
    if (n == N) {
#pragma unroll
        for (int k = 0; k + 1 < N; k++) a[k] = a[k + 1];
        n = N - 1;
    }
#pragma unroll
    for (int k = 0; k < N; k++) a[k] = (k == n) ? v : a[k];
    n++;
}

template <bool AUDIO>
struct Detector {
    const PulseParams &p;
    PulseStreamState &s;
    Rings r;
    int lane;

    __device__ float E(int j) const { return r.e[(s.head + (uint32_t)j) & (uint32_t)p.cap_mask]; }
    __device__ float time_of(int i) const { return s.t0 + (float)i / p.fs_energy; }  // timeOfIdx

    __device__ bool last3_locked() const {
        if (s.n_last3 != 3) return false;
        float mn = s.last3[0], mx = s.last3[0];
#pragma unroll
        for (int k = 1; k < 3; k++) {
            if (s.last3[k] < mn) mn = s.last3[k];
            if (mx < s.last3[k]) mx = s.last3[k];
        }
        return mx - mn < p.dt_tol_s;
    }

    // noiseRef (audio_pulse_detector.cpp:78-90): sequential float mean of eBuf_[far, near)
    __device__ float noise_ref(int i) const {
        int lo = i - p.noise_far, hi = i - p.noise_near;
        if (hi <= 0 || lo >= hi) return -1.f;
        lo = max(lo, 0);
        hi = min(hi, s.n);
        if (lo >= hi) return -1.f;
        float acc = 0.f;
        for (int b = lo; b < hi; b += WAVE) {
            const int j = b + lane;
            const float v = j < hi ? E(j) : 0.f;
            const int cnt = min(WAVE, hi - b);
            for (int k = 0; k < cnt; k++) acc += bcast(v, k);
        }
        return acc / (float)(hi - lo);
    }

    // estimatedFreqHz's regression (spectral_pulse_detector.cpp:148-170), refreshed when freqHistory_ changes
    __device__ void refresh_regression() {
        const int nh = s.n_fh;
        if (nh < 2) {
            s.ols_mode = 0;
            return;
        }
        float tl = 0.f, fl = 0.f;
        if (lane < nh) {
            const int slot = (s.fh_head + lane) & (PULSE_FH_SLOTS - 1);
            tl = r.ft[slot];
            fl = r.ff[slot];
        }
        double st = 0, sf = 0, stt = 0, stf = 0;
        for (int k = 0; k < nh; k++) {
            const float t = bcast(tl, k), f = bcast(fl, k);
            st += (double)t;
            sf += (double)f;
            stt += (double)(t * t);  // float products, as in the reference
            stf += (double)(t * f);
        }
        const double den = (double)nh * stt - st * st;
        if (fabs(den) < 1e-9) {
            s.ols_mode = 1;
            s.ols_mean = (float)(sf / (double)nh);
        } else {
            const double a = ((double)nh * stf - st * sf) / den;
            s.ols_a = a;
            s.ols_b = (sf - a * st) / (double)nh;
            s.ols_mode = 2;
        }
    }

    __device__ float est_freq() const {
        if (s.ols_mode == 1) return s.ols_mean;
        if (s.ols_mode == 2) return (float)(s.ols_a * (double)time_of(s.n - 1) + s.ols_b);
        return 0.f;
    }

    // detectRois (spectral :46-143, audio :132-237)
    __device__ void detect_rois() {
        const uint32_t mask = (uint32_t)p.cap_mask;
        const float z_s = s.locked ? 0.75f * s.t_target : p.z_default_s;
        const int idx_z = max(1, (int)(z_s * p.fs_energy));
        const int safe = s.n - idx_z;
        if (safe <= idx_z) return;
        for (int i = max(idx_z, s.last_scan); i < safe; i++) {
            const float val = E(i);
            bool beaten = false;  // some j != i in [i - idx_z, i + idx_z] with eBuf_[j] >= val
            for (int b = i - idx_z; b <= i + idx_z; b += WAVE) {
                const int j = b + lane;
                const bool ge = j <= i + idx_z && j != i && E(j) >= val;
                if (ballot(ge)) {
                    beaten = true;
                    break;
                }
            }
            if (beaten) continue;

            float snr = val;
            if constexpr (AUDIO) {
                const float noise = noise_ref(i);
                if (noise <= 0.f) continue;
                snr = val / noise;
            }
            if (snr < p.snr_min) continue;

            const float t_roi = time_of(i);
            const float dt = (s.t_last_roi >= 0.f) ? t_roi - s.t_last_roi : 0.f;
            int n_cyc = 1;
            float norm_dt = dt;
            if (dt > 0.f) {
                n_cyc = max(1, (int)roundf(dt / s.t_target));
                if (n_cyc > 1 && fabsf(dt - (float)n_cyc * s.t_target) > p.dt_tol_s) n_cyc = 1;
                norm_dt = dt / (float)n_cyc;
            }
            const bool in_rhythm = (dt > 0.f) && (fabsf(norm_dt - s.t_target) < p.dt_tol_s);
            if (!(snr >= p.snr_strong || (snr >= p.snr_rhythm && in_rhythm))) continue;

            if (dt > 0.f) {  // phase lock (:86-102)
                push_bounded(s.last3, s.n_last3, norm_dt);
                if (last3_locked()) {
                    s.locked = 1;
                    s.t_target = (s.last3[0] + s.last3[1] + s.last3[2]) / 3.f;
                }
                int nh = s.n_hist;
                push_bounded(s.hist_dts, nh, norm_dt);
                nh = s.n_hist;
                push_bounded(s.hist_n, nh, n_cyc);
                s.n_hist = nh;
            }
            int base;
            if constexpr (AUDIO)  // fixed thresholds (audio_pulse_detector.cpp:194-198)
                base = (snr >= 2.0f) ? 5 : (snr >= 1.5f) ? 4 : (snr >= 1.2f) ? 3 : (snr >= 1.1f) ? 2 : 1;
            else  // spectral_pulse_detector.cpp:106-110
                base = (snr >= p.snr_strong) ? 5 : (snr >= 3.0f) ? 4 : (snr >= p.snr_rhythm) ? 3 : (snr >= 2.0f) ? 2 : 1;
            const int pen_rhythm = (dt > 0.f && !in_rhythm) ? 2 : 0;
            int pen_conf = 0;
            if (s.n_hist >= 4) {
                float disp = 0.f;
#pragma unroll
                for (int j = 1; j < 5; j++)
                    if (j < s.n_hist) disp += fabsf(s.hist_dts[j] - s.hist_dts[j - 1]);
                int sum_n = 0;
#pragma unroll
                for (int j = 0; j < 5; j++)
                    if (j < s.n_hist) sum_n += s.hist_n[j];
                if (disp > p.dispersion_max || sum_n > p.sum_n_max) pen_conf = 2;
            }
            if (last3_locked()) pen_conf = 0;
            const int etat = max(0, base - pen_rhythm - pen_conf);

            // rois_.push_back, freqHistory_.push_back (lane 0 writes, the wave reads after the barrier)
            if (s.n_rois == (int)mask + 1) {  // cannot happen within the documented bound; keep the newest
                s.roi_head++;
                s.n_rois--;
                s.overflow++;
            }
            const uint32_t rslot = (s.roi_head + (uint32_t)s.n_rois) & mask;
            s.n_rois++;
            s.t_last_roi = t_roi;
            s.last_snr = snr;
            float fi = 0.f;
            int fslot = 0;
            if constexpr (!AUDIO) {
                fi = r.f[(s.head + (uint32_t)i) & mask];  // freqBuf_[i]
                if (s.n_fh == 30) {
                    s.fh_head = (s.fh_head + 1) & (PULSE_FH_SLOTS - 1);
                    s.n_fh--;
                }
                fslot = (s.fh_head + s.n_fh) & (PULSE_FH_SLOTS - 1);
                s.n_fh++;
            }
            if (lane == 0) {
                r.rt[rslot] = t_roi;
                r.re[rslot] = etat;
                if constexpr (!AUDIO) {
                    r.ft[fslot] = t_roi;
                    r.ff[fslot] = fi;
                }
            }
            __syncthreads();
            if constexpr (!AUDIO) refresh_regression();

            // trim ROIs older than 20 s: pop while front.t < cutoff (the new ROI itself always stays)
            const float cutoff = t_roi - 20.f;
            const int older = s.n_rois - 1;
            int drop = older;
            for (int b = 0; b < older; b += WAVE) {
                const int j = b + lane;
                const bool keep = j < older && !(r.rt[(s.roi_head + (uint32_t)j) & mask] < cutoff);
                const uint64_t m = ballot(keep);
                if (m) {
                    drop = b + (int)__builtin_ctzll(m);
                    break;
                }
            }
            s.roi_head += (uint32_t)drop;
            s.n_rois -= drop;

            i += idx_z;
            s.last_scan = i + 1;
        }
        s.last_scan = max(s.last_scan, safe);
    }

    // computeLiveEtat + toLevel
    __device__ void update_live() {
        int live = 0;
        if (s.n_rois > 0) {
            const float now = time_of(s.n - 1);
            const float start = now - p.live_window_t * s.t_target;
            int sum = 0;
            for (int b = 0; b < s.n_rois; b += WAVE) {
                const int j = b + lane;
                if (j < s.n_rois) {
                    const uint32_t slot = (s.roi_head + (uint32_t)j) & (uint32_t)p.cap_mask;
                    if (r.rt[slot] >= start) sum += r.re[slot];
                }
            }
            // the reference sums the etats as floats in order: integer partial sums < 2^24 are exact
            const float total = (float)wave_sum(sum);
            live = min(5, (int)floorf(total / p.live_divisor));
        }
        s.live_etat = live;
        s.level = live >= 5 ? 3 : live >= 3 ? 2 : live >= 1 ? 1 : 0;
    }

    // onEnergyFrame (spectral :27-42, audio :113-128)
    __device__ void energy_frame(float v, float fv) {
        if (s.n == 0) s.t0 = 0.f;
        const uint32_t slot = (s.head + (uint32_t)s.n) & (uint32_t)p.cap_mask;
        if (lane == 0) {
            r.e[slot] = v;
            if constexpr (!AUDIO) r.f[slot] = fv;
        }
        s.n++;
        while (s.n > p.max_buf) {
            s.head++;
            s.n--;
            s.t0 += p.inv_fs;
            if (s.last_scan > 0) s.last_scan--;
        }
        __syncthreads();
        detect_rois();
        __syncthreads();
        update_live();
    }
};

__device__ __forceinline__ Rings stream_rings(int stream, int cap, float *ebuf, float *fbuf, float *roi_t, int *roi_etat,
                                              float *fh) {
    const size_t o = (size_t)stream * (size_t)cap;
    Rings r;
    r.e = ebuf + o;
    r.f = fbuf ? fbuf + o : nullptr;
    r.rt = roi_t + o;
    r.re = roi_etat + o;
    r.ft = fh ? fh + (size_t)stream * 2 * PULSE_FH_SLOTS : nullptr;
    r.ff = r.ft ? r.ft + PULSE_FH_SLOTS : nullptr;
    return r;
}

__device__ __forceinline__ void write_output(const PulseStreamState &s, float input, float est, sdrg_pulse_output *o) {
    sdrg_pulse_output w;
    w.strength = s.last_snr;
    w.live_etat = s.live_etat;
    w.level = s.level;
    w.locked = s.locked;
    w.period_s = s.t_target;
    w.est_freq_hz = est;
    w.est_freq_hz_rounded = (int64_t)roundf(est);  // std::llround of a float (half away from zero)
    w.input = input;
    w.n_energy = s.n;
    w.n_rois = s.n_rois;
    w.overflow = s.overflow;
    *o = w;
}

__global__ __launch_bounds__(WAVE) void spectral_pulse_kernel(PulseParams p, PulseStreamState *__restrict__ states,
                                                              float *ebuf, float *fbuf, float *roi_t, int *roi_etat,
                                                              float *fh, const float *snr_sigma, const float *freq_hz,
                                                              int stride_bytes, sdrg_pulse_output *__restrict__ out) {
    const int stream = blockIdx.x;
    const int lane = threadIdx.x;
    PulseStreamState s;
    load_state(s, states + stream);
    Detector<false> d{p, s, stream_rings(stream, p.cap_mask + 1, ebuf, fbuf, roi_t, roi_etat, fh), lane};
    const size_t off = (size_t)stream * (size_t)stride_bytes;
    const float v = *reinterpret_cast<const float *>(reinterpret_cast<const char *>(snr_sigma) + off);
    const float fv = *reinterpret_cast<const float *>(reinterpret_cast<const char *>(freq_hz) + off);
    d.energy_frame(v, fv);
    if (lane == 0) {
        write_output(s, v, d.est_freq(), out + stream);
        store_state(states + stream, s);
    }
}

// Standalone audio front end (the bank's own calls, and the SSB reference-kernel path; the pipelined SSB kernel
// runs the same front_sample() on the PCM it produces), one LANE per stream: the SIMD runs 64 streams'
// recurrences side by side.  Each 64-sample column of the 64 streams' blocks is read with 64 independent
// loads (lane = sample, one row per load), kept in registers while the previous column is processed from
// LDS, then transposed through LDS so each lane walks its own row.
constexpr int FT = 64;  // samples per column

template <int FMT>
__global__ __launch_bounds__(WAVE) void audio_front_kernel(AudioFront a, const void *audio, int n_samples, int stride,
                                                           int n_streams) {
    __shared__ float tile[2][WAVE][FT + 1];
    const int lane = threadIdx.x;
    const int s0 = blockIdx.x * WAVE;
    const int stream = s0 + lane;
    const bool live = stream < n_streams;
    const int rows = min(WAVE, n_streams - s0);
    FrontState f{};
    if (live) f = front_load(a.state + stream);
    float *my_new = a.new_e + (size_t)(live ? stream : 0) * (size_t)a.max_new;
    int np = 0;
    float v[WAVE];
    auto load_col = [&](int c0) {
#pragma unroll
        for (int r = 0; r < WAVE; r++) {
            const size_t o = (size_t)(s0 + r) * (size_t)stride + (size_t)(c0 + lane);
            float x = 0.f;
            if (r < rows && c0 + lane < n_samples) {
                if constexpr (FMT == 0) x = (float)reinterpret_cast<const int16_t *>(audio)[o] * PCM_TO_FLOAT;
                else x = reinterpret_cast<const float *>(audio)[o];
            }
            v[r] = x;
        }
    };
    if (n_samples > 0) load_col(0);
    int buf = 0;
    for (int c0 = 0; c0 < n_samples; c0 += FT, buf ^= 1) {
#pragma unroll
        for (int r = 0; r < WAVE; r++) tile[buf][r][lane] = v[r];
        __syncthreads();
        if (c0 + FT < n_samples) load_col(c0 + FT);  // in flight while this column is processed
        const int cn = min(FT, n_samples - c0);
        if (live)
            for (int k = 0; k < cn; k++) front_sample(a, f, tile[buf][lane][k], my_new, np);
    }
    if (live) {
        front_store(a.state + stream, f);
        a.new_count[stream] = np;
    }
}

// Audio detector, one wavefront per stream: onEnergyFrame for each energy value the front end produced.
__global__ __launch_bounds__(WAVE) void audio_pulse_kernel(PulseParams p, PulseStreamState *__restrict__ states,
                                                           float *ebuf, float *roi_t, int *roi_etat,
                                                           const float *__restrict__ new_e, int max_new,
                                                           const int *__restrict__ new_count,
                                                           sdrg_pulse_output *__restrict__ out) {
    const int stream = blockIdx.x;
    const int lane = threadIdx.x;
    PulseStreamState s;
    load_state(s, states + stream);
    Detector<true> d{p, s, stream_rings(stream, p.cap_mask + 1, ebuf, nullptr, roi_t, roi_etat, nullptr), lane};
    const int np = new_count[stream];
    const float *e = new_e + (size_t)stream * (size_t)max_new;
    for (int q = 0; q < np; q++) d.energy_frame(e[q], 0.f);
    if (lane == 0) {
        write_output(s, s.last_snr, 0.f, out + stream);
        store_state(states + stream, s);
    }
}

// AudioPulseDetector(cfg) / reset(): fresh detector state
__global__ void pulse_reset_kernel(PulseStreamState *states, int n_streams, float t_target_init) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_streams) return;
    PulseStreamState s;
    memset(&s, 0, sizeof(s));
    s.t_last_roi = -1.f;
    s.t_target = t_target_init;
    states[i] = s;
}

}  // namespace

hipError_t launch_pulse_reset(PulseStreamState *states, int n_streams, float t_target_init, hipStream_t stream) {
    if (n_streams <= 0) return hipSuccess;
    hipLaunchKernelGGL(pulse_reset_kernel, dim3((n_streams + 255) / 256), dim3(256), 0, stream, states, n_streams,
                       t_target_init);
    return hipGetLastError();
}

hipError_t launch_spectral_pulse(const PulseParams &p, int n_streams, PulseStreamState *states, float *ebuf,
                                 float *fbuf, float *roi_t, int *roi_etat, float *fh, const float *snr_sigma,
                                 const float *freq_hz, int stride_bytes, sdrg_pulse_output *out, hipStream_t stream) {
    if (n_streams <= 0) return hipSuccess;
    hipLaunchKernelGGL(spectral_pulse_kernel, dim3(n_streams), dim3(WAVE), 0, stream, p, states, ebuf, fbuf, roi_t,
                       roi_etat, fh, snr_sigma, freq_hz, stride_bytes, out);
    return hipGetLastError();
}

hipError_t launch_audio_front(const AudioFront &a, const void *audio, int fmt, int n_samples, int stride, int n_streams,
                              hipStream_t stream) {
    if (n_streams <= 0) return hipSuccess;
    const dim3 grid((n_streams + WAVE - 1) / WAVE);
    if (fmt == 0)
        hipLaunchKernelGGL(audio_front_kernel<0>, grid, dim3(WAVE), 0, stream, a, audio, n_samples, stride, n_streams);
    else
        hipLaunchKernelGGL(audio_front_kernel<1>, grid, dim3(WAVE), 0, stream, a, audio, n_samples, stride, n_streams);
    return hipGetLastError();
}

hipError_t launch_audio_detect(const PulseParams &p, int n_streams, PulseStreamState *states, float *ebuf, float *roi_t,
                               int *roi_etat, const float *new_e, int max_new, const int *new_count,
                               sdrg_pulse_output *out, hipStream_t stream) {
    if (n_streams <= 0) return hipSuccess;
    hipLaunchKernelGGL(audio_pulse_kernel, dim3(n_streams), dim3(WAVE), 0, stream, p, states, ebuf, roi_t, roi_etat,
                       new_e, max_new, new_count, out);
    return hipGetLastError();
}

}  // namespace sdrg

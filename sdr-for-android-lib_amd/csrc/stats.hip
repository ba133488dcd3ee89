// stats.hip — per-frame signal-strength statistics, frequency tracking and detection flag.
//
// Replaces FFTProcessor::evaluateSignalStrength (src/dsp/fft_process.cpp:122-379) for a batch of frames,
// one wavefront per frame, reading the fftshifted power spectrum the spectrum kernel wrote and updating
// the stream's FFTProcessor state (StatsState) in HBM.
//
// The reference's float expressions are kept in their order, with FP contraction off, so the statistics
// follow it to libm rounding: the sequential running sums (best1kHzMean, the best-start scan) are
// replayed sequentially by one lane per window because their drift is part of the reference result
// (fft_process.cpp:163-180, :313-319); the focus peak is the FIRST maximum of the dB values (strict >,
// seeded at -130 dB), found by a wave reduction that prefers the lower index on ties; the MAD medians
// are exact k-th-element radix selects instead of std::sort.  Only the trip-wise order-free parts
// (dB conversions, the pooled-gap selection) run across lanes.
#include "sdrg_internal.h"

#pragma clang fp contract(off)

namespace sdrg {
namespace {

constexpr int WAVE = 64;
constexpr int STAGE_MAX = 8192;  // bins staged into LDS for the window scans (32 KiB)
constexpr int MAX_POOL = 16384;  // pooled-bin bound: N/4 at N = 65536 (the widest nBottom case, see engine.cpp)

__device__ __forceinline__ float db_of(float p) { return 10.0f * log10f(p / 1.0f + 1e-20f); }  // refPower = 1

struct WinScan {
    float sum;       // sequential sum over [lo, hi]
    float best1k;    // best1kHzMean(lo, hi)
    int best_start;  // first start maximising the raw running sum (focus scan, :311-320)
};

// One lane replays the reference's sequential loops over P[lo..hi] (P: staged LDS copy or HBM).
__device__ __forceinline__ WinScan scan_window(const float *__restrict__ P, int lo, int hi, int w) {
    WinScan r;
    float s = 0.0f;
#pragma unroll 8
    for (int i = lo; i <= hi; i++) s += P[i];
    r.sum = s;
    const int len = hi - lo + 1;
    r.best_start = lo;
    if (len <= 0) {
        r.best1k = 0.0f;
    } else if (len < w) {
        r.best1k = s / len;
    } else {
        float rs = 0.0f;
#pragma unroll 8
        for (int i = lo; i < lo + w; i++) rs += P[i];
        float bv = rs;
#pragma unroll 4
        for (int st = lo + 1; st + w - 1 <= hi; st++) {
            rs += P[st + w - 1] - P[st - 1];
            if (rs > bv) {
                bv = rs;
                r.best_start = st;
            }
        }
        // the reference keeps best = max over st of rs/w (:171-178); x -> RN(x / w) is monotone for w > 0,
        // so that maximum is exactly RN(max rs / w): one division instead of one per step
        r.best1k = bv / w;
    }
    return r;
}

// The same sequential loops for up to 11 windows whose bins do not fit the LDS stage at once (e.g. N = 65536
// with a 200 kHz focus: three windows of 13107 bins).  All 64 lanes copy the next chunk of every window
// (plus the w bins before it, which the sliding scan subtracts) from HBM into LDS, coalesced; then lane j
// runs window j's plain sum and lane 32 + j its best-1-kHz sliding scan over that chunk, the two sequential
// chains of a window on two lanes, in the reference's element order.  Without the staging each dependent
// step of those chains waited on an HBM load.  Lane j (j < nwin) returns window j's WinScan.
__device__ WinScan scan_windows_chunked(const float *__restrict__ P, float *buf, int buf_floats, int nwin,
                                        const int *wlo, const int *whi, int w) {
    const int lane = threadIdx.x;
    const int row = buf_floats / nwin;        // floats per window row: w history bins + SC new ones
    const int SC = row - w;                   // > 0: checked by the caller
    const int j = lane & 31;
    const bool sum_lane = lane < nwin, scan_lane = lane >= 32 && j < nwin;
    const int my_lo = (j < nwin) ? wlo[j] : 0, my_len = (j < nwin) ? whi[j] - wlo[j] + 1 : 0;
    int max_len = 0;
    for (int q = 0; q < nwin; q++) max_len = max(max_len, whi[q] - wlo[q] + 1);
    float s = 0.0f, rs = 0.0f, bv = 0.0f;
    int best_start = my_lo;
    const float *mine = buf + j * row + w;  // mine[e - c0] = P[lo + e], e in [c0 - w, c0 + SC)
    for (int c0 = 0; c0 < max_len; c0 += SC) {
        for (int q = 0; q < nwin; q++) {
            const int lo = wlo[q], len = whi[q] - wlo[q] + 1;
            const int t0 = max(c0 - w, 0), t1 = min(c0 + SC, len);  // elements of window q this chunk needs
#pragma unroll 16  // 16 loads in flight per lane: a rolled loop would wait out HBM latency per 256 B
            for (int t = t0 + lane; t < t1; t += WAVE) buf[q * row + w + (t - c0)] = P[lo + t];
        }
        __syncthreads();
        const int end = min(c0 + SC, my_len);
        if (sum_lane) {
#pragma unroll 8
            for (int e = c0; e < end; e++) s += mine[e - c0];
        } else if (scan_lane && my_len >= w) {
            int e = c0;
            for (; e < end && e < w; e++) {  // the first window's sum (:171-172)
                rs += mine[e - c0];
                if (e == w - 1) bv = rs;
            }
#pragma unroll 4
            for (; e < end; e++) {  // slide: start st = lo + e - w + 1 (:173-178)
                rs += mine[e - c0] - mine[e - c0 - w];
                if (rs > bv) {
                    bv = rs;
                    best_start = my_lo + e - w + 1;
                }
            }
        }
        __syncthreads();
    }
    const float bv_scan = __shfl(bv, (lane & 31) + 32);
    const int bs_scan = __shfl(best_start, (lane & 31) + 32);
    WinScan r;
    r.sum = s;
    r.best_start = my_lo;
    if (my_len <= 0) {
        r.best1k = 0.0f;
    } else if (my_len < w) {
        r.best1k = s / my_len;
    } else {
        r.best1k = bv_scan / w;  // as scan_window: RN(max rs / w)
        r.best_start = bs_scan;
    }
    return r;
}

__device__ __forceinline__ float fmax_ref(float a, float b) { return (a < b) ? b : a; }  // std::max

// Ascending sort of 10 (key, index) pairs by (key, index): odd-even transposition network, registers only.
__device__ __forceinline__ void sort_pairs10(float (&k)[10], int (&ix)[10]) {
#pragma unroll
    for (int round = 0; round < 10; round++) {
#pragma unroll
        for (int i = round & 1; i + 1 < 10; i += 2) {
            const bool sw = (k[i + 1] < k[i]) || (k[i + 1] == k[i] && ix[i + 1] < ix[i]);
            const float ka = sw ? k[i + 1] : k[i], kb = sw ? k[i] : k[i + 1];
            const int ia = sw ? ix[i + 1] : ix[i], ib = sw ? ix[i] : ix[i + 1];
            k[i] = ka; k[i + 1] = kb; ix[i] = ia; ix[i + 1] = ib;
        }
    }
}

// k-th smallest (k < 4) of 4 floats (the reference sorts then indexes: same value).
__device__ __forceinline__ float kth_of4(float (&g)[4], int k) {
#pragma unroll
    for (int round = 0; round < 4; round++) {
#pragma unroll
        for (int i = round & 1; i + 1 < 4; i += 2) {
            const float a = fminf(g[i], g[i + 1]), b = fmaxf(g[i], g[i + 1]);
            g[i] = a;
            g[i + 1] = b;
        }
    }
    // selects, not an indexed load (the compiler would place g in scratch to index it)
    float r = g[0];
    asm volatile("" : "+v"(r));
    r = (k == 1) ? g[1] : r;
    asm volatile("" : "+v"(r));
    r = (k == 2) ? g[2] : r;
    asm volatile("" : "+v"(r));
    r = (k == 3) ? g[3] : r;
    return r;
}

// k-th smallest (0-based) of non-negative floats in vals[0..cnt) by 4 x 8-bit radix select (one wave).
// Per digit: an LDS histogram (atomics), then a wave-parallel prefix scan (4 bins per lane) locates the
// bucket holding the k-th element.  Same element as the reference's std::sort + gaps[k].
__device__ float kth_smallest(const float *vals, int cnt, int k, int *hist, int *) {
    const int lane = threadIdx.x;
    uint32_t prefix = 0, mask = 0;
    for (int shift = 24; shift >= 0; shift -= 8) {
        *reinterpret_cast<int4 *>(&hist[4 * lane]) = make_int4(0, 0, 0, 0);
        __syncthreads();
        for (int q = lane; q < cnt; q += WAVE) {
            const uint32_t b = __float_as_uint(vals[q]);
            if ((b & mask) == prefix) atomicAdd(&hist[(b >> shift) & 0xff], 1);
        }
        __syncthreads();
        const int4 h = *reinterpret_cast<const int4 *>(&hist[4 * lane]);
        const int own = h.x + h.y + h.z + h.w;
        int incl = own;
#pragma unroll
        for (int off = 1; off < WAVE; off <<= 1) {
            const int v = __shfl_up(incl, off);
            if (lane >= off) incl += v;
        }
        const unsigned long long over = __ballot(incl > k);  // non-empty: k < number of candidates
        const int L = __ffsll((long long)over) - 1;
        int d = 0, acc = incl - own;
        if (lane == L) {
            const int hv[4] = {h.x, h.y, h.z, h.w};
            int j = 3;  // the lane's last bin unless an earlier one already passes k
#pragma unroll
            for (int t = 2; t >= 0; t--) {
                int before = acc;
#pragma unroll
                for (int u = 0; u < t; u++) before += hv[u];
                if (before + hv[t] > k) j = t;
            }
#pragma unroll
            for (int u = 0; u < 3; u++)
                if (u < j) acc += hv[u];
            d = 4 * L + j;
        }
        d = __shfl(d, L);
        acc = __shfl(acc, L);
        k -= acc;
        prefix |= (uint32_t)d << shift;
        mask |= 0xffu << shift;
        __syncthreads();
    }
    return __uint_as_float(prefix);
}

__global__ __launch_bounds__(WAVE) void stats_kernel(const float *__restrict__ spectra, StatsGeometry g,
                                                     int64_t now_ms, StatsState *__restrict__ state,
                                                     sdrg_frame_record *__restrict__ records, float *gpool,
                                                     int gpool_stride) {
    // one dynamic LDS area, used twice: first the staged bins of the window scans, then (after a barrier)
    // the pooled dB values / gaps of the MAD median -- unless the pool exceeds MAX_POOL bins (wide focus at
    // N > 65536), which then lives in this frame's slice of the global scratch gpool
    extern __shared__ __attribute__((aligned(16))) float dyn[];
    float *pool = gpool ? gpool + (size_t)blockIdx.x * gpool_stride : dyn;
    float *stage = dyn;
    __shared__ __attribute__((aligned(16))) int hist[256];
    __shared__ int sh_int[2];
    __shared__ int sh_nbottom, sh_best_start;
    __shared__ float w_mean_db[10], w_best1k_db[10];
    __shared__ int w_lo[10], w_hi[10], order[10];
    __shared__ float sh_f[4];
    __shared__ int sh_geo_lo[11], sh_geo_hi[11];  // the reference windows, then the focus window (index n_ref)

    const int lane = threadIdx.x;
    const size_t frame = blockIdx.x;
    // the window bounds are indexed by lane below: copy them out of the kernel arguments with constant
    // indices (a lane-indexed kernarg array would be copied to scratch)
#pragma unroll
    for (int i = 0; i < 10; i++) {
        if (lane == i) {
            sh_geo_lo[i] = g.win_lo[i];
            sh_geo_hi[i] = g.win_hi[i];
        }
    }
    const float *P = spectra + frame * (size_t)g.n;
    StatsState st = state[frame];
    if (g.cf_changed) st.center_frequency_changed = 1;  // sdr_bridge_internal::isCenterFrequencyChanged
    sdrg_frame_record rec;
    __builtin_memset(&rec, 0, sizeof(rec));  // tail padding included: records compare and gather as bytes
    rec.peak_bin = -1;
    rec.abs_peak_db = -130.0f;
    rec.signal_power_db = 0.0f;
    rec.valid = 0;
    rec.n_ref_windows = 0;

    if (g.focus_len > 0) {
        // ---- 6.2 focus peak: first maximum of dB, seeded at -130 (fft_process.cpp:142-154) ----
        float best = -130.0f;
        int bidx = 0x7fffffff;
#pragma unroll 8  // loads in flight (13107-bin focus windows at N = 65536 / 200 kHz)
        for (int i = g.focus_lo + lane; i <= g.focus_hi; i += WAVE) {
            const float d = db_of(P[i]);
            if (d > best) {
                best = d;
                bidx = i;
            }
        }
        for (int off = WAVE / 2; off > 0; off >>= 1) {
            const float ob = __shfl_xor(best, off);
            const int oi = __shfl_xor(bidx, off);
            if (ob > best || (ob == best && oi < bidx)) {
                best = ob;
                bidx = oi;
            }
        }
        const float abs_peak_db = best;
        const int peak_bin = (bidx == 0x7fffffff) ? g.focus_lo : bidx;

        // ---- 6.2 focus sum + 6.3 reference windows: one lane per window (reference order), lane n_ref
        //      takes the focus window; all of them run the same sequential scan in lockstep ----
        const int w1k = g.win_bins_1k;
        const int n_ref = g.n_ref;
        // stage the bins every window touches into LDS (coalesced) when they fit, so the sequential
        // per-lane scans below read LDS instead of waiting on HBM for every element
        const bool staged = g.span_len > 0 && g.span_len <= STAGE_MAX;
        if (staged) {
#pragma unroll 16
            for (int i = lane; i < g.span_len; i += WAVE) stage[i] = P[g.span_lo + i];
            __syncthreads();
        }
        if (lane == 0) {
            sh_geo_lo[n_ref] = g.focus_lo;
            sh_geo_hi[n_ref] = g.focus_hi;
        }
        __syncthreads();
        // windows too wide to stage together: chunked through the same LDS area (all lanes take part)
        const bool chunked = !staged && STAGE_MAX / (n_ref + 1) - w1k >= 64;
        WinScan wsc{};
        if (chunked) wsc = scan_windows_chunked(P, stage, STAGE_MAX, n_ref + 1, sh_geo_lo, sh_geo_hi, w1k);
        if (lane <= n_ref) {
            const bool is_focus = (lane == n_ref);
            const int lo = sh_geo_lo[lane];
            const int hi = sh_geo_hi[lane];
            const WinScan ws = chunked ? wsc : staged ? scan_window(stage - g.span_lo, lo, hi, w1k) : scan_window(P, lo, hi, w1k);
            const int n = hi - lo + 1;
            if (is_focus) {
                sh_f[0] = db_of(ws.sum / n);  // signalPowerDb (:155)
                sh_f[1] = ws.best1k;          // focusBest1kLinear (:302)
                sh_best_start = ws.best_start;
            } else {
                w_mean_db[lane] = db_of(ws.sum / n);
                w_best1k_db[lane] = db_of(ws.best1k);
                w_lo[lane] = lo;
                w_hi[lane] = hi;
            }
        }
        __syncthreads();
        const float signal_power_db = sh_f[0];
        const int valid = (n_ref >= 2);
        rec.peak_bin = peak_bin;
        rec.abs_peak_db = abs_peak_db;
        rec.signal_power_db = signal_power_db;
        rec.valid = valid;
        rec.n_ref_windows = n_ref;

        if (!valid) {
            st.mean_snr_db = st.mean_snr_sigma = 0.0f;
            st.peak_above_noise_mean_db = st.max_bin_snr_db = st.max_bin_snr_sigma = 0.0f;
            st.best1khz_snr_db = st.best1khz_snr_sigma = 0.0f;
        } else {
            int n_bottom = 1;
            if (lane == 0) {
                // std::sort of <= 16 elements in libstdc++ is a (stable) insertion sort: the same order is a
                // sort by (meanDb, window index), done here by a network on registers
                float key[10];
                int ix[10];
#pragma unroll
                for (int i = 0; i < 10; i++) {
                    key[i] = (i < n_ref) ? w_mean_db[i] : INFINITY;
                    ix[i] = i;
                }
                sort_pairs10(key, ix);
#pragma unroll
                for (int i = 0; i < 10; i++)
                    if (i < n_ref) order[i] = ix[i];
                const int nb0 = (int)(n_ref * 0.4f);
                n_bottom = nb0 > 1 ? nb0 : 1;  // <= 4 (n_ref <= 10)
                // 6.4a (:235-247)
                float mean = 0.0f;
#pragma unroll
                for (int i = 0; i < 4; i++)
                    if (i < n_bottom) mean += key[i];
                mean /= n_bottom;
                float gp[4];
#pragma unroll
                for (int i = 0; i < 4; i++) gp[i] = (i < n_bottom) ? fabsf(key[i] - mean) : INFINITY;
                const float sigma = fmax_ref(1.4816f * kth_of4(gp, n_bottom / 2), 0.5f);
                const float snr_db = signal_power_db - mean;
                st.mean_snr_db = snr_db;
                st.mean_snr_sigma = snr_db / sigma;
                sh_nbottom = n_bottom;
            }
            __syncthreads();
            n_bottom = sh_nbottom;

            // ---- 6.4b pooled per-bin dB of the bottom windows, sorted-window order (:252-269) ----
            int cnt = 0;
            for (int j = 0; j < n_bottom; j++) {
                const int lo = w_lo[order[j]], hi = w_hi[order[j]];
#pragma unroll 8
                for (int i = lo + lane; i <= hi; i += WAVE) {
                    const int q = cnt + (i - lo);
                    if (q < g.max_pool) pool[q] = db_of(P[i]);
                }
                cnt += hi - lo + 1;
            }
            if (cnt > g.max_pool) cnt = g.max_pool;  // host sizes max_pool from the geometry
            __syncthreads();
            if (lane == 0) {
                // sequential sum in pool order (:259-263); 16 values per step read with 4 ds_read_b128
                float m = 0.0f;
                int q = 0;
                for (; q + 16 <= cnt; q += 16) {
                    float4 b[4];
#pragma unroll
                    for (int u = 0; u < 4; u++) b[u] = *reinterpret_cast<const float4 *>(&pool[q + 4 * u]);
#pragma unroll
                    for (int u = 0; u < 4; u++) {
                        m += b[u].x;
                        m += b[u].y;
                        m += b[u].z;
                        m += b[u].w;
                    }
                }
                for (; q < cnt; q++) m += pool[q];
                m /= (float)cnt;
                sh_f[2] = m;
            }
            __syncthreads();
            const float per_bin_mean = sh_f[2];
            for (int q = lane; q < cnt; q += WAVE) pool[q] = fabsf(pool[q] - per_bin_mean);
            __syncthreads();
            const float med = kth_smallest(pool, cnt, cnt / 2, hist, sh_int);
            const float sigma_bin = (cnt > 0) ? fmax_ref(1.4816f * med, 1.0f) : 1.0f;
            if (cnt > 0) st.per_bin_mean = per_bin_mean;
            const float pbm = (cnt > 0) ? per_bin_mean : 0.0f;

            if (lane == 0) {
                st.peak_above_noise_mean_db = abs_peak_db - pbm;  // :274
                // 6.4c (:281-288)
                const float logN = logf((float)g.focus_len);
                const float sqrt2logN = sqrtf(2.0f * logN);
                const float gumbel_loc = pbm + sigma_bin * sqrt2logN;
                const float gumbel_sig = fmax_ref(sigma_bin * 3.14159f / (sqrtf(6.0f) * sqrt2logN), 0.5f);
                st.max_bin_snr_db = abs_peak_db - gumbel_loc;
                st.max_bin_snr_sigma = st.max_bin_snr_db / gumbel_sig;
                // 6.4d (:292-327)
                float mean1k = 0.0f;
                for (int i = 0; i < n_bottom; i++) mean1k += w_best1k_db[order[i]];
                mean1k /= n_bottom;
                float g1k[4];
#pragma unroll
                for (int i = 0; i < 4; i++) g1k[i] = (i < n_bottom) ? fabsf(w_best1k_db[order[i]] - mean1k) : INFINITY;
                const float sigma_floor_1k = sigma_bin / sqrtf((float)w1k);
                float sigma1k = 1.4816f * kth_of4(g1k, n_bottom / 2);
                if (sigma1k < sigma_floor_1k) sigma1k = sigma_floor_1k;
                if (sigma1k < 0.5f) sigma1k = 0.5f;
                const float focus_best1k_linear = sh_f[1];
                if (focus_best1k_linear > 0.0f) {
                    const float focus_best1k_db = db_of(focus_best1k_linear);
                    st.best1khz_snr_db = focus_best1k_db - mean1k;
                    st.best1khz_snr_sigma = st.best1khz_snr_db / sigma1k;
                    const int best_start = sh_best_start;
                    st.best1khz_center_freq_hz = (best_start + w1k / 2) * g.freq_per_bin + g.cf_minus_nyq;
                } else {
                    st.best1khz_snr_db = st.best1khz_snr_sigma = 0.0f;
                }
            }
        }

        if (lane == 0) {
            // ---- 6.5 frequency tracking (:333-361), clock injected ----
            if (st.tracking_frequency == 0.0f) st.tracking_frequency = g.cf_float;
            if (st.center_frequency_changed) {
                st.tracking_frequency = g.cf_float;
                st.center_frequency_changed = 0;
            }
            if (!st.max_peak_set) {
                st.max_peak_db = -130.0f;
                st.max_peak_freq = g.cf_float;
                st.max_peak_set = 1;
            }
            if (valid && abs_peak_db > st.max_peak_db) {
                st.max_peak_db = abs_peak_db;
                st.max_peak_freq = peak_bin * g.freq_per_bin + g.cf_u32_minus_nyq;
                st.time_last_max_peak_ms = now_ms;
            }
            const int64_t ms_since = now_ms - st.time_last_max_peak_ms;
            if (st.time_last_update_ms < st.time_last_max_peak_ms && ms_since > 300) {
                st.tracking_frequency = st.max_peak_freq;
                st.time_last_update_ms = now_ms;
                st.max_peak_db = -130.0f;
            }
            // ---- 6.6 detection (:365-378) ----
            const bool above = valid && (st.mean_snr_sigma >= 4.0f);
            if (above) {
                if (st.peak_confirmed < 1) st.peak_confirmed++;
            } else {
                st.peak_confirmed = 0;
            }
            const int flag = (above && st.peak_confirmed >= 1) ? 3 : 0;
            // det_buf[det_idx] = flag with constant indices (no private-memory indexing)
            const int d0 = (st.det_idx == 0) ? flag : st.det_buf[0];
            const int d1 = (st.det_idx == 1) ? flag : st.det_buf[1];
            const int d2 = (st.det_idx == 2) ? flag : st.det_buf[2];
            st.det_buf[0] = d0;
            st.det_buf[1] = d1;
            st.det_buf[2] = d2;
            st.det_idx = (st.det_idx + 1) % 3;
            int m = d0;
            if (d1 > m) m = d1;
            if (d2 > m) m = d2;
            st.detection_flag_sent = m;
        }
    }

    if (lane == 0) {
        rec.tracking_frequency = (int64_t)roundf(st.tracking_frequency);
        rec.mean_snr_db = st.mean_snr_db;
        rec.mean_snr_sigma = st.mean_snr_sigma;
        rec.peak_above_noise_mean_db = st.peak_above_noise_mean_db;
        rec.max_bin_snr_db = st.max_bin_snr_db;
        rec.max_bin_snr_sigma = st.max_bin_snr_sigma;
        rec.best1khz_snr_db = st.best1khz_snr_db;
        rec.best1khz_snr_sigma = st.best1khz_snr_sigma;
        rec.best1khz_center_freq_hz = st.best1khz_center_freq_hz;
        rec.per_bin_mean = st.per_bin_mean;
        rec.detection_flag = st.detection_flag_sent;
        if (records) records[frame] = rec;
        state[frame] = st;
    }
}

}  // namespace

size_t stats_global_pool_floats(const StatsGeometry &geo, int n_frames) {
    return geo.max_pool > MAX_POOL ? (size_t)n_frames * (size_t)((geo.max_pool + 3) & ~3) : 0;
}

hipError_t launch_stats(const float *spectra, int n_frames, const StatsGeometry &geo, int64_t now_ms,
                        StatsState *state, sdrg_frame_record *records, float *gpool, hipStream_t stream) {
    if (n_frames <= 0) return hipSuccess;
    const bool global_pool = geo.max_pool > MAX_POOL;
    if (global_pool && !gpool) return hipErrorInvalidValue;
    // the stage area (the staged span, or STAGE_MAX floats for the chunked window scans), reused for the pool
    const int staged = (geo.span_len > 0 && geo.span_len <= STAGE_MAX) ? geo.span_len : STAGE_MAX;
    const int pool = global_pool ? 0 : (geo.max_pool + 3) & ~3;
    const size_t lds = sizeof(float) * (size_t)((pool > staged ? pool : staged) + 4);
    hipError_t e = ensure_dynamic_lds(reinterpret_cast<const void *>(stats_kernel), (MAX_POOL + STAGE_MAX + 8) * 4);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(stats_kernel, dim3(n_frames), dim3(WAVE), lds, stream, spectra, geo, now_ms, state, records,
                       global_pool ? gpool : nullptr, (geo.max_pool + 3) & ~3);
    return hipGetLastError();
}

}  // namespace sdrg

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
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <type_traits>
#include <vector>

#include "glibc_logf.h"
#include "sdrg_internal.h"

#pragma clang fp contract(off)

namespace sdrg {
namespace {

constexpr int WAVE = 64;
constexpr int STAGE_MAX = 8192;  // bins staged into LDS for the window scans (32 KiB)

// Diagnostic build only (-DSDRG_STATS_STAMPS=1, tools/build_variant.sh): s_memtime at phase boundaries per frame
#ifndef SDRG_STATS_STAMPS
#define SDRG_STATS_STAMPS 0
#endif
constexpr int STAMP_PHASES = 12;


__device__ unsigned long long g_stats_stamps[STAMP_PHASES * 8192];
#define STATS_STAMP(k)                                                                                        \
    do {                                                                                                      \
        if (SDRG_STATS_STAMPS && threadIdx.x == 0 && blockIdx.x < 8192)                                       \
            g_stats_stamps[blockIdx.x * STAMP_PHASES + (k)] = __builtin_amdgcn_s_memtime();                   \
    } while (0)

// glibc's logf table, copied into LDS by every kernel of this file before its first barrier (load_logf_tab): the
// dB values are the reference's `10.0f * log10f(p / refPower + 1e-20f)` with glibc's log10f (glibc_logf.h), so
// every dB, the peak index, the window order and the pooled gaps equal the reference's x86-64 build bit for bit
__shared__ glibc::LogfEntry s_logf_tab[16];
__device__ __forceinline__ void load_logf_tab() {
    if (threadIdx.x < 16) s_logf_tab[threadIdx.x] = glibc::logf_table()[threadIdx.x];
}
__device__ __forceinline__ float db_of(float p) {  // refPower = 1
    return 10.0f * glibc::log10f_fast(p / 1.0f + 1e-20f, s_logf_tab);
}

// The same dB through the folded table (glibc_logf.h, log10f_posnormal_fold: the same bits, one conversion and one
// f64 fma fewer per log): the wide kernels' per-bin logs (their producers and pooled gaps).  Loaded beside s_logf_tab
// by load_logf_fold in those kernels only (the narrow kernel's LDS stays as it was: it shares CUs with the SSB
// pipeline and the spectrum).
__shared__ glibc::LogfFold s_logf_fold[glibc::LOGF_FOLD_N];
__device__ __forceinline__ void load_logf_fold() {
    if (threadIdx.x < glibc::LOGF_FOLD_N) s_logf_fold[threadIdx.x] = glibc::logf_fold_entry(threadIdx.x, glibc::logf_table());
}
__device__ __forceinline__ float db_fold(float p) {  // refPower = 1
    return 10.0f * glibc::log10f_fast_fold(p / 1.0f + 1e-20f, s_logf_fold);
}

struct WinScan {
    float sum;       // sequential sum over [lo, hi]
    float best1k;    // best1kHzMean(lo, hi)
    int best_start;  // first start maximising the raw running sum (focus scan, :311-320)
};

// One lane replays the reference's sequential loops over the window P[lo..hi], staged in LDS at W (W[i - lo]).
// (The window's own base pointer, not a virtual P: LDS pointers must stay inside the allocation.)  The window
// sum (:190-193) and the best-1-kHz scan (:171-178) run in one loop: the scan's first window sum is the window
// sum's first w terms in the same order (the same float), and after it the two chains are independent, so
// they overlap instead of running one after the other.
__device__ __forceinline__ WinScan scan_window(const float *__restrict__ W, int lo, int hi, int w) {
    WinScan r;
    const int len = hi - lo + 1;
    r.best_start = lo;
    float s = 0.0f;
    int i = 0;
    const int head = len < w ? len : w;
#pragma unroll 8
    for (; i < head; i++) s += W[i];
    if (len <= 0) {
        r.sum = s;
        r.best1k = 0.0f;
        return r;
    }
    if (len < w) {
        r.sum = s;
        r.best1k = s / len;
        return r;
    }
    float rs = s, bv = s;
#pragma unroll 8
    for (; i < len; i++) {
        const float x = W[i];
        s += x;
        rs += x - W[i - w];
        if (rs > bv) {
            bv = rs;
            r.best_start = lo + i - w + 1;
        }
    }
    r.sum = s;
    // the reference keeps best = max over st of rs/w (:171-178); x -> RN(x / w) is monotone for w > 0,
    // so that maximum is exactly RN(max rs / w): one division instead of one per step
    r.best1k = bv / w;
    return r;
}

// Wide windows: the same sequential loops for up to 11 windows whose bins do not fit the LDS stage (e.g.
// N = 65536 with a 200 kHz focus: three windows of 13107 bins).  One 256-thread workgroup per frame.  Four such
// workgroups share a CU and the chains are one lane per window, so the kernel is bound by the CU's VALU issue:
// the design spends as few wave-instructions per bin as the reference's float order allows.
//   waves 2-3 (producers) stream chunk c of every window from HBM into one slot of an LDS ring: the bins x,
//            the running-sum terms (x for the first w bins, then the sliding difference x[e] - x[e-w], the
//            reference's `P[st+w-1] - P[st-1]`, :173-175, an order-free subtraction) and, when want_db, the
//            bins' dB values; on the way they evaluate the focus window's dB values for its first maximum
//            (fft_process.cpp:146-154).  Bins past a window's end are zeros (adding +0 changes no sum);
//   wave 0   (chains) consumes chunk c - 1: every lane runs the same plain sequential sum over its row, 4 bins
//            per ds_read_b128, writing its running values back: lane j sums window j's bins (the window sum
//            s, :190-193, :149 for the focus), lane 16 + j its running-sum terms (rs, the best-1-kHz running
//            sum, :171-178, :313-319, into the rs ring), lane 32 + j its dB values (want_db: the pooled-bin
//            mean's sum, :259-263, when window j turns out to be the only bottom window);
//   wave 1   (records) consumes chunk c - 2's running sums rs, lane-parallel: the chunk's first maximum over
//            the bins e >= w - 1, kept when it exceeds the maximum so far -- the reference's last strict
//            `rs > bv` record (bv starts at the first window's sum, bin w - 1), whose start is bestStart.
// One barrier per chunk.
constexpr int WIDE_WG = 256;
#ifndef SDRG_WIDE_RING  // lab: the ring's floats (a smaller ring leaves LDS to the four-step kernels running beside it)
#define SDRG_WIDE_RING 9216
#endif
constexpr int RING_FLOATS = SDRG_WIDE_RING;  // 36 KiB at most: (2 slots x 3 rows + 2 rs rows) x windows x (SC + 4)

struct WideScan {
    float sum[11], bv[11], dsum[11];
    int best_e[11];
    float peak_db;
    int peak_idx;
};

// SDRG_WIDE_DBPOOL: where the pooled-gap pass (one bottom window) gets the bottom window's dB values -- 0: evaluates
// its 13107 logs again; 1 (lab): the producers also store every reference bin's dB value to the frame's pool scratch
// (their stores then share vmcnt with the next chunk's loads: slower); 2 (product): the record wave copies the dB rows
// of the ring to the pool scratch (it issues no loads).  Measured at 65536 / 200 kHz: pool phase 56k -> 6.7k cycles per
// frame, configs[4] 200 kHz step 0.5135 -> 0.4955 ms (tools/gpu_wide_db2.sh).
#ifndef SDRG_WIDE_DBPOOL
#define SDRG_WIDE_DBPOOL 2
#endif
// The wide scans' per-chunk barrier orders LDS only (s_waitcnt lgkmcnt(0); s_barrier), so the producers' loads of the
// next chunk stay in flight across it; __syncthreads() would wait for them (vmcnt(0)) at every chunk.  Nothing global is
// exchanged between the waves inside the scan (the pool copies are read after it, behind a __syncthreads).
__device__ __forceinline__ void wide_chunk_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// The focus peak of fft_process.cpp:142-154 (first strict maximum of the dB values, seeded at -130) from the largest
// focus power pmax = out.peak_db (on entry), by monotonicity: dB(p) = 10 log10f(p + 1e-20) never decreases with p
// (glibc's log10f is monotone: checked over every float, tests/test_libm_exact.py), so the bins whose dB equals the
// maximum d* = dB(pmax) are exactly those with p >= p_lo, the smallest float whose dB is d*; the peak is the first of
// them.  p_lo: the WG threads test pmax's 256 float neighbours below it, then (only when all of them share d*, e.g.
// powers where the 1e-20 dominates) one thread bisects the float bit patterns below.  Every thread calls this.
template <int WG>
__device__ __forceinline__ void focus_peak_monotone(const float *__restrict__ P, int flo, int flen, WideScan &out) {
    __shared__ int s_t, s_plo, s_first;
    const int tid = threadIdx.x;
    const float pm = out.peak_db;
    const float ds = db_of(pm);
    if (tid == 0) {
        s_t = WG;
        s_first = 0x7fffffff;
    }
    __syncthreads();
    const int bm = __float_as_int(pm);
    const int b = bm - tid;
    if (ds > -130.0f && b >= 0 && db_of(__int_as_float(b)) != ds) atomicMin(&s_t, tid);
    __syncthreads();
    if (tid == 0 && ds > -130.0f) {
        const int T = s_t;
        int plo = bm - (T - 1);
        if (T == WG) {  // every tested neighbour shares d*: bisect [0, bm - WG + 1]
            int lo = 0, hi = bm - (WG - 1);
            if (hi <= 0) {
                lo = 0;
            } else {
                while (lo < hi) {
                    const int mid = lo + ((hi - lo) >> 1);
                    if (db_of(__int_as_float(mid)) == ds) hi = mid;
                    else lo = mid + 1;
                }
            }
            plo = lo;
        }
        s_plo = plo < 0 ? 0 : plo;
    }
    __syncthreads();
    if (ds > -130.0f) {
        const float plo = __int_as_float(s_plo);
        for (int i = tid; i < flen; i += WG)
            if (P[flo + i] >= plo) {
                atomicMin(&s_first, i);
                break;
            }
    }
    __syncthreads();
    if (tid == 0) {
        const bool hit = ds > -130.0f && s_first != 0x7fffffff;
        out.peak_db = hit ? ds : -130.0f;
        out.peak_idx = hit ? flo + s_first : flo;
    }
    __syncthreads();
}

template <bool want_db>
__device__ __forceinline__ void scan_wide(const float *__restrict__ P, float *ring, int nwin, const int *wlo, const int *whi, int w,
                          int role, float *__restrict__ dbp, int wst, WideScan &out) {
    // roles: 0 chains, 1 records, 2-3 producers (role = wave index)
    const int lane = threadIdx.x & 63;
    const int fq = nwin - 1;
    // SC = 2^lg bins per window per chunk, the largest that fits; rows are RS = SC + 4 floats apart, so the chain
    // lanes' float4 accesses (one row each, same bin) fall in different LDS banks
    int lg = 6;
    while (8 * nwin * ((2 << lg) + 4) <= RING_FLOATS && lg < 12) lg++;
    const int SC = 1 << lg, RS = SC + 4, slot_floats = 3 * RS * nwin;
    float *rsring = ring + 2 * slot_floats;  // [2][nwin] rows
    int max_len = 0;
    for (int q = 0; q < nwin; q++) max_len = max(max_len, whi[q] - wlo[q] + 1);
    const int nch = (max_len + SC - 1) >> lg;

    // chain lanes (wave 0): group 0 window sums, group 1 running sums, group 2 dB sums
    const int grp = lane >> 4, j = lane & 15;
    const bool chain = role == 0 && j < nwin && (grp < 2 || (grp == 2 && want_db && j < nwin - 1));
    float acc = 0.0f;
    // records (wave 1): the reference's strict `rs > bv` records over the bins e >= w - 1, bv starting at the
    // first window's sum, end at the FIRST bin holding the maximum of rs over those bins: an order-free first
    // arg-max.  G lanes per window each keep the first maximum of their bins; one reduction at the end.  Bins
    // past the window's end hold its last running sum again, so they can only tie with a lower real bin.
    const int G = WAVE / nwin, rq = min(lane / G, fq), rk = lane - rq * G;
    const bool rec_lane = role == 1 && lane < G * nwin;
    float rm = -INFINITY;
    int ri = 0x7fffffff;
    float pk = -130.0f;
    int pki = 0x7fffffff;

    // producers: PG threads per window, thread k of window pq's group handles bins k, k + PG, ... of each chunk.
    // The bins (and the bins w before them) of chunk c + 1 are fetched into registers before the barrier that
    // ends chunk c, so their HBM latency overlaps the consumers' work instead of following it.
    constexpr int PTHREADS = WIDE_WG - 128;
    constexpr int PR = 9;  // >= SC / PG for every nwin <= 11 (SC from the ring size above)
    const int pw = role >= 2 ? ((role - 2) << 6) | lane : 0;
    const int PG = PTHREADS / nwin;
    const int pq = min(pw / PG, fq);
    const int pk0 = pw - pq * PG;
    const bool prod = role >= 2 && pw < PG * nwin;
    const int plo = wlo[pq], plen = whi[pq] - plo + 1;
    const float *Pq = P + plo;
    float va[PR], vb[PR];
    auto fetch = [&](int c) {
        const int c0 = c << lg;
#pragma unroll
        for (int k = 0; k < PR; k++) {
            const int t = pk0 + PG * k, e = c0 + t;
            const bool ok = t < SC && e < plen;
            va[k] = ok ? Pq[e] : 0.0f;
            vb[k] = (ok && e >= w) ? Pq[e - w] : 0.0f;
        }
    };
    auto store = [&](int c) {
        const int c0 = c << lg;
        float *row = ring + (c & 1) * slot_floats + pq * 3 * RS;
#pragma unroll
        for (int k = 0; k < PR; k++) {
            const int t = pk0 + PG * k, e = c0 + t;
            if (t < SC) {
                const bool in = e < plen;
                const float v = va[k];
                row[t] = v;
                row[RS + t] = (e >= w) ? v - vb[k] : v;
                const float d = db_fold(v);
                if (want_db) row[2 * RS + t] = in ? d : 0.0f;
                // SDRG_WIDE_DBPOOL: the reference windows' dB values also go to the frame's pool scratch, where the
                // pooled-gap pass reads the bottom window's instead of evaluating its logs again
                if (SDRG_WIDE_DBPOOL == 1 && want_db && in && pq < fq) dbp[pq * wst + e] = d;
                // a thread sees its focus bins in increasing order: strict > keeps its first maximum
                if (in && pq == fq && d > pk) {
                    pk = d;
                    pki = plo + e;
                }
            }
            __builtin_amdgcn_sched_barrier(0);  // one bin's log10 at a time: interleaved they would hold ~70 VGPRs
        }
    };
    if (prod && nch > 0) fetch(0);

    unsigned long long busy = 0;
    for (int c = 0; c <= nch + 1; c++) {
        const unsigned long long t_in = SDRG_STATS_STAMPS ? __builtin_amdgcn_s_memtime() : 0;
        if (role >= 2) {
            if (prod && c < nch) {
                store(c);
                if (c + 1 < nch) fetch(c + 1);
            }
        } else if (role == 0) {
            if (c >= 1 && c <= nch && chain) {
                const int cj = j, cg = grp;
                const float *slot = ring + ((c - 1) & 1) * slot_floats;
                const float *src = slot + (cj * 3 + cg) * RS;  // x, rs terms, dB rows
                // running values: the rs lanes' go to the rs ring (the record wave reads them); the window and dB
                // sums' are never read and go back over their own row -- with SDRG_WIDE_DBPOOL 2 the dB lanes' over
                // the window's bins row instead (beside its sum lane's, same addresses, bins already consumed), so the
                // dB row stays intact for the record wave's copy to the pool scratch
                float *dst = cg == 1 ? rsring + (((c - 1) & 1) * nwin + cj) * RS
                                     : const_cast<float *>(src) - ((SDRG_WIDE_DBPOOL == 2 && cg == 2) ? 2 * RS : 0);
                // 16 bins per half-step, the next half's four float4 read before this half's adds (two register
                // sets, no copies), so the LDS latency hides under 16 dependent adds
                float4 A[4], B[4];
                auto rd = [&](float4 (&X)[4], int u) {
#pragma unroll
                    for (int i = 0; i < 4; i++) X[i] = *reinterpret_cast<const float4 *>(src + u + 4 * i);
                };
                auto add = [&](float x) {
                    acc += x;
                    return acc;
                };
                auto sum16 = [&](const float4 (&X)[4], int u) {
                    float4 r[4];
#pragma unroll
                    for (int i = 0; i < 4; i++) {
                        r[i].x = add(X[i].x);
                        r[i].y = add(X[i].y);
                        r[i].z = add(X[i].z);
                        r[i].w = add(X[i].w);
                    }
#pragma unroll
                    for (int i = 0; i < 4; i++) *reinterpret_cast<float4 *>(dst + u + 4 * i) = r[i];
                };
                rd(A, 0);
                for (int t = 0; t < SC; t += 32) {  // SC >= 64, a multiple of 32
                    rd(B, t + 16);
                    sum16(A, t);
                    if (t + 32 < SC) rd(A, t + 32);
                    sum16(B, t + 16);
                }
            }
        } else {
            // SDRG_WIDE_DBPOOL 2: the record wave copies chunk c - 1's dB rows of the reference windows (the slot the
            // chain reads this iteration) to the frame's pool scratch; it issues no loads, so its stores never hold
            // up a vmcnt wait
            if (SDRG_WIDE_DBPOOL == 2 && want_db && role == 1 && c >= 1 && c <= nch) {
                const int c0 = (c - 1) << lg, q4 = SC >> 2;
                const float *slot = ring + ((c - 1) & 1) * slot_floats;
                for (int i = lane; i < fq * q4; i += WAVE) {
                    const int q = i / q4, t = (i - q * q4) << 2, e = c0 + t, len = whi[q] - wlo[q] + 1;
                    const float4 v = *reinterpret_cast<const float4 *>(slot + (q * 3 + 2) * RS + t);
                    float *o = dbp + q * wst + e;
                    if (e + 3 < len) {
                        o[0] = v.x;
                        o[1] = v.y;
                        o[2] = v.z;
                        o[3] = v.w;
                    } else {
                        if (e < len) o[0] = v.x;
                        if (e + 1 < len) o[1] = v.y;
                        if (e + 2 < len) o[2] = v.z;
                    }
                }
            }
        }
        if (role == 1 && c >= 2 && rec_lane) {
            // chunk c - 2's running sums: lane k of window rq's group visits bins k, k + G, ... in increasing order
            const int c0 = (c - 2) << lg;
            const float *rsrow = rsring + ((c & 1) * nwin + rq) * RS;  // (c - 2) & 1
            if (c0 + SC > w - 1) {
                if (c0 >= w - 1) {
                    for (int t = rk; t < SC; t += G) {
                        const float v = rsrow[t];
                        const bool gt = v > rm;  // strict: the lane keeps its first maximum
                        rm = gt ? v : rm;
                        ri = gt ? c0 + t : ri;
                    }
                } else {
                    for (int t = rk; t < SC; t += G) {
                        const float v = rsrow[t];
                        const bool gt = c0 + t >= w - 1 && v > rm;
                        rm = gt ? v : rm;
                        ri = gt ? c0 + t : ri;
                    }
                }
            }
        }
        if (SDRG_STATS_STAMPS) busy += __builtin_amdgcn_s_memtime() - t_in;
        wide_chunk_barrier();
    }
    if (SDRG_STATS_STAMPS && lane == 0 && role <= 2 && blockIdx.x < 8192)
        g_stats_stamps[blockIdx.x * STAMP_PHASES + 6 + role] = busy;
    if (role >= 2) {  // first maximum over the producer threads (lower bin on ties)
        for (int off = WAVE / 2; off > 0; off >>= 1) {
            const float ob = __shfl_xor(pk, off);
            const int oi = __shfl_xor(pki, off);
            if (ob > pk || (ob == pk && oi < pki)) {
                pk = ob;
                pki = oi;
            }
        }
        if (role == 3 && lane == 0) {
            out.peak_db = pk;
            out.peak_idx = pki;
        }
    }
    if (role == 1) {  // first maximum per window over its lane group (lower bin on ties)
        for (int q = 0; q < nwin; q++) {
            float m = (rec_lane && rq == q) ? rm : -INFINITY;
            int mi = (rec_lane && rq == q) ? ri : 0x7fffffff;
            for (int off = WAVE / 2; off > 0; off >>= 1) {
                const float om = __shfl_xor(m, off);
                const int oi = __shfl_xor(mi, off);
                if (om > m || (om == m && oi < mi)) {
                    m = om;
                    mi = oi;
                }
            }
            if (lane == 0) {
                out.bv[q] = m;
                out.best_e[q] = mi;
            }
        }
    }
    if (chain && grp == 0) out.sum[j] = acc;
    if (chain && grp == 2) out.dsum[j] = acc;
    __syncthreads();
    if (role == 2 && lane == 0) {
        const bool other = pk > out.peak_db || (pk == out.peak_db && pki < out.peak_idx);
        if (other) {
            out.peak_db = pk;
            out.peak_idx = pki;
        }
        if (out.peak_idx == 0x7fffffff) out.peak_idx = wlo[fq];
    }
    __syncthreads();
}

__device__ __forceinline__ float fmax_ref(float a, float b) { return (a < b) ? b : a; }  // std::max

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

// ---- per-frame scalar parts, shared by the narrow and the wide kernel (one lane per frame) ----
__device__ __forceinline__ int n_bottom_of(int n_ref) {
    const int nb0 = (int)(n_ref * 0.4f);  // nBottom (:233), <= 4 (n_ref <= 10)
    return nb0 > 1 ? nb0 : 1;
}

// 6.4a (:235-247): mean SNR over the nBottom lowest windows (order: the windows sorted by mean dB)
__device__ __forceinline__ void mean_snr_6_4a(const float *w_mean_db, const int *order, int n_ref, float signal_power_db,
                                              StatsState &st) {
    const int n_bottom = n_bottom_of(n_ref);
    float key[4];
#pragma unroll
    for (int i = 0; i < 4; i++) key[i] = (i < n_ref) ? w_mean_db[order[i]] : INFINITY;
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
}

// 6.4b tail + 6.4c (:274, :281-288) + 6.4d (:292-327)
__device__ __forceinline__ void snr_6_4cd(const StatsGeometry &g, StatsState &st, float abs_peak_db, float pbm,
                                          float sigma_bin, int n_bottom, const float *w_best1k_db, const int *order,
                                          float focus_best1k_linear, int best_start) {
    const int w1k = g.win_bins_1k;
    st.peak_above_noise_mean_db = abs_peak_db - pbm;  // :274
    const float logN = g.log_focus_len;  // std::log(float(focusLen)) (:282), glibc logf on the host
    const float sqrt2logN = sqrtf(2.0f * logN);
    const float gumbel_loc = pbm + sigma_bin * sqrt2logN;
    const float gumbel_sig = fmax_ref(sigma_bin * 3.14159f / (sqrtf(6.0f) * sqrt2logN), 0.5f);
    st.max_bin_snr_db = abs_peak_db - gumbel_loc;
    st.max_bin_snr_sigma = st.max_bin_snr_db / gumbel_sig;
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
    // (:303-327; selects rather than a branch around the dB, which kept the state struct in scratch)
    const bool pos = focus_best1k_linear > 0.0f;
    const float focus_best1k_db = db_of(pos ? focus_best1k_linear : 1.0f);
    const float snr1k_db = focus_best1k_db - mean1k;
    st.best1khz_snr_db = pos ? snr1k_db : 0.0f;
    st.best1khz_snr_sigma = pos ? snr1k_db / sigma1k : 0.0f;
    if (pos) st.best1khz_center_freq_hz = (best_start + w1k / 2) * g.freq_per_bin + g.cf_minus_nyq;
}

// 6.5 frequency tracking (:333-361), clock injected; 6.6 detection (:365-378)
__device__ __forceinline__ void track_detect_6_5_6_6(const StatsGeometry &g, StatsState &st, int valid,
                                                     float abs_peak_db, int peak_bin, int64_t now_ms) {
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

__device__ __forceinline__ void finish_record(sdrg_frame_record &rec, const StatsState &st) {
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
}

// k-th smallest (0-based) of non-negative floats in vals[0..cnt) by an 8-bit-digit radix select (WG threads).
// Bits that every value shares (AND == OR, found by one pass) need no digit pass, so the first histogram splits on
// the highest bit where the values differ: the values are spread over the bins instead of all landing in the few
// bins of a common exponent (which serialised the LDS atomics: wide windows at N = 65536 pool 13107 values).
// Per digit: an LDS histogram (atomics), then a wave-parallel prefix scan (4 bins per lane, wave 0) locates the
// bucket holding the k-th element.  Same element as the reference's std::sort + gaps[k].
// visit(f) calls f(bits) once for every value this thread holds (an LDS/HBM array or registers).
template <int WG, class Visit>
__device__ __forceinline__ float kth_smallest(Visit visit, int k, int *hist, uint32_t *xch) {
    const int tid = threadIdx.x, lane = tid & (WAVE - 1), wave = tid / WAVE;
    constexpr int XB = 2 * (WG / WAVE) > 8 ? 2 * (WG / WAVE) : 8;  // xch: the waves' AND / OR, then [XB, XB + 1]
    uint32_t band = 0xffffffffu, bor = 0u;
    visit([&](uint32_t b) {
        band &= b;
        bor |= b;
    });
    for (int off = WAVE / 2; off > 0; off >>= 1) {
        band &= (uint32_t)__shfl_xor((int)band, off);
        bor |= (uint32_t)__shfl_xor((int)bor, off);
    }
    if constexpr (WG > WAVE) {
        if (lane == 0) {
            xch[2 * wave] = band;
            xch[2 * wave + 1] = bor;
        }
        __syncthreads();
#pragma unroll
        for (int v = 0; v < WG / WAVE; v++) {
            band &= xch[2 * v];
            bor |= xch[2 * v + 1];
        }
    }
    const uint32_t diff = band ^ bor;
    if (diff == 0) return __uint_as_float(band);  // every value equal
    int top = 31 - __clz(diff);                   // highest bit where the values differ
    uint32_t mask = top >= 31 ? 0u : ~((2u << top) - 1u);
    uint32_t prefix = band & mask;
    while (top >= 0) {
        const int lo = top >= 7 ? top - 7 : 0;
        const uint32_t dm = (1u << (top - lo + 1)) - 1u;
        for (int i = 4 * tid; i < 256; i += 4 * WG) *reinterpret_cast<int4 *>(&hist[i]) = make_int4(0, 0, 0, 0);
        __syncthreads();
        visit([&](uint32_t b) {
            if ((b & mask) == prefix) atomicAdd(&hist[(b >> lo) & dm], 1);
        });
        __syncthreads();
        if (wave == 0) {
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
            if (lane == L) {
                int acc = incl - own;
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
                xch[XB] = (uint32_t)(4 * L + j);
                xch[XB + 1] = (uint32_t)acc;
            }
        }
        __syncthreads();
        const uint32_t d = xch[XB];
        k -= (int)xch[XB + 1];
        prefix |= d << lo;
        mask |= dm << lo;
        top = lo - 1;
        __syncthreads();
    }
    return __uint_as_float(prefix);
}

template <int WG>
__device__ __forceinline__ float kth_smallest_of(const float *vals, int cnt, int k, int *hist, uint32_t *xch) {
    return kth_smallest<WG>(
        [&](auto f) {
            for (int q = threadIdx.x; q < cnt; q += WG) f(__float_as_uint(vals[q]));
        },
        k, hist, xch);
}

// the wide kernel's pool when it fits the threads' registers: value q = threadIdx.x + WIDE_WG * r of v[r]
constexpr int REG_POOL = 64;
constexpr int NARROW_REG_POOL = 24;  // the narrow kernel's pool in registers up to 24 x 64 values

extern "C" __device__ uint32_t __ockl_wfred_and_u32(uint32_t);
extern "C" __device__ uint32_t __ockl_wfred_or_u32(uint32_t);
extern "C" __device__ int __ockl_wfscan_add_i32(int, bool);

// k-th smallest (0-based) of the non-negative floats one wave holds (visit(f) calls f(bits) for each value
// this lane holds): the radix select of kth_smallest with the device library's DPP wave operations for the
// AND/OR reduction and the bucket scan (no LDS round trips), 4 histogram bins per lane.
template <class Visit>
__device__ float kth_smallest_wave(Visit visit, int k, int *hist, uint32_t *xch) {
    const int lane = threadIdx.x;
    uint32_t band = 0xffffffffu, bor = 0u;
    visit([&](uint32_t b) {
        band &= b;
        bor |= b;
    });
    band = __ockl_wfred_and_u32(band);
    bor = __ockl_wfred_or_u32(bor);
    const uint32_t diff = band ^ bor;
    if (diff == 0) return __uint_as_float(band);  // every value equal
    int top = 31 - __clz(diff);                   // highest bit where the values differ
    uint32_t mask = top >= 31 ? 0u : ~((2u << top) - 1u);
    uint32_t prefix = band & mask;
    while (top >= 0) {
        const int lo = top >= 7 ? top - 7 : 0;
        const uint32_t dm = (1u << (top - lo + 1)) - 1u;
        *reinterpret_cast<int4 *>(&hist[4 * lane]) = make_int4(0, 0, 0, 0);
        __syncthreads();
        visit([&](uint32_t b) {
            if ((b & mask) == prefix) atomicAdd(&hist[(b >> lo) & dm], 1);
        });
        __syncthreads();
        const int4 h = *reinterpret_cast<const int4 *>(&hist[4 * lane]);
        const int own = h.x + h.y + h.z + h.w;
        const int incl = __ockl_wfscan_add_i32(own, true);  // DPP inclusive scan
        const unsigned long long over = __ballot(incl > k);  // non-empty: k < number of candidates
        const int L = __ffsll((long long)over) - 1;
        if (lane == L) {
            int acc = incl - own;
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
            xch[0] = (uint32_t)(4 * L + j);
            xch[1] = (uint32_t)acc;
        }
        __syncthreads();
        k -= (int)xch[1];
        prefix |= xch[0] << lo;
        mask |= dm << lo;
        top = lo - 1;
        __syncthreads();
    }
    return __uint_as_float(prefix);
}

// Narrow statistics, one wave per frame.  Every window's bins are staged compactly into LDS (window q at
// sh_woff[q]) by buffer loads straight into LDS, all of the frame's loads in flight at once; the focus peak's dB
// values are evaluated from LDS right after (the other bins need no dB until the pool).  The reference's sequential sums run one lane per window
// (the window scans) or per frame (the pooled mean, the scalar tail); the order-free work (copy, dB, pooled
// gaps, select) runs across the lanes.  LDS per frame: the staged bins, over which the pool is laid out in
// order once the scans are done (R > 0: pool values <= R per lane, held in registers for the select), or, for
// pools beyond 24 x 64 values (R == 0), a pool region after them.  Small on purpose: beside the SSB pipeline
// (84.5 KiB of LDS per CU) the frames that fit at once set the kernel's time.
// Registers for eight waves per SIMD (<= 64 VGPRs; the 24-register pool variant six): the statistics of a pipelined
// call then fit beside the next call's spectrum on every SIMD (its four waves hold 112 VGPRs each) instead of waiting
// for its workgroups to retire.
// Measured (tools/gpu_r4n.sh, alternating, one box): alone 27.2 vs 26.7 us per 4096 frames; the c3 step with the
// statistics on their own stream 0.3077-0.3088 ms against 0.3121-0.3124 (76 VGPRs) and 0.3141 on the main stream.
// Round 6 (tools/gpu_r6u.sh, alternating, one box): the staging copy as LDS-direct buffer loads, one instruction per
// 64 bins of a window, instead of 8 register loads per lane in flight behind a 10-step window search per bin (50
// VGPRs instead of 64, no second HBM round trip): alone 27.0 -> 26.6 us per 4096 x 16384 / 5 kHz and 47.0 -> 41.6 us
// per 1024 x 65536 / 5 kHz; the configs[4] 5 kHz line 207.9 / 208.0 -> 216.6 / 216.5 G; bit-exact.

#ifndef SDRG_NARROW_WPE  // lab: waves per SIMD the narrow kernel is compiled for
#define SDRG_NARROW_WPE 8
#endif
template <int R>
__global__ __launch_bounds__(WAVE) __attribute__((amdgpu_waves_per_eu(R > 8 ? 6 : SDRG_NARROW_WPE))) void stats_narrow_kernel(
    const float *__restrict__ spectra, StatsGeometry g, int64_t now_ms, StatsState *__restrict__ state,
    sdrg_frame_record *__restrict__ records) {
    extern __shared__ __attribute__((aligned(16))) float stage[];
    __shared__ int sh_woff[12];
    __shared__ int sh_geo_lo[11], sh_geo_hi[11];  // the reference windows, then the focus window (index n_ref)
    __shared__ __attribute__((aligned(16))) int hist[256];
    __shared__ uint32_t sh_xch[2];
    __shared__ float w_mean_db[10], w_best1k_db[10];
    __shared__ int order[10];
    __shared__ float sh_f[4];
    __shared__ int sh_best_start;

    const int lane = threadIdx.x;
    const size_t frame = blockIdx.x;
    const int n_ref = g.n_ref;
    load_logf_tab();
#pragma unroll
    for (int i = 0; i < 10; i++) {  // constant kernarg indices (a lane-indexed kernarg array would go to scratch)
        if (lane == i) {
            sh_geo_lo[i] = g.win_lo[i];
            sh_geo_hi[i] = g.win_hi[i];
        }
    }
    if (lane == 0) {
        sh_geo_lo[n_ref] = g.focus_lo;
        sh_geo_hi[n_ref] = g.focus_hi;
        int o = 0;
        for (int q = 0; q <= n_ref; q++) {
            sh_woff[q] = o;
            o += max(0, (q < n_ref ? g.win_hi[q] - g.win_lo[q] : g.focus_hi - g.focus_lo) + 1);
        }
        sh_woff[n_ref + 1] = o;
    }
    __syncthreads();
    const int stage_total = sh_woff[n_ref + 1], stage_pad = (stage_total + 3) & ~3;
    const float *P = spectra + frame * (size_t)g.n;
    StatsState st = state[frame];
    if (g.cf_changed) st.center_frequency_changed = 1;  // sdr_bridge_internal::isCenterFrequencyChanged
    sdrg_frame_record rec;
    __builtin_memset(&rec, 0, sizeof(rec));  // tail padding included: records compare and gather as bytes
    rec.peak_bin = -1;
    rec.abs_peak_db = -130.0f;

    if (g.focus_len > 0 && stage_total <= STAGE_MAX) {
        const int w1k = g.win_bins_1k;
        STATS_STAMP(0);
        // ---- staging + 6.2 focus peak: first maximum of dB, seeded at -130 (fft_process.cpp:142-154) ----
        float best = -130.0f;
        int bidx = 0x7fffffff;
        {
            // window q's bins straight into stage[woff[q] ..] by buffer loads to LDS (no registers, no per-bin
            // window search): 64 bins per instruction, the window's offset in the scalar offset, every load of the
            // frame in flight at once; then the focus bins' dB from LDS (a lane sees its focus bins in increasing
            // order, strict > keeps each lane's first maximum; the reduction below takes the lower bin on ties, so
            // the result does not depend on which lane holds which bin)
            const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(P), (short)0,
                                                                                 g.n * 4, 0x00020000);
            for (int q = 0; q <= n_ref; q++) {
                const int lo = __builtin_amdgcn_readfirstlane(sh_geo_lo[q]);
                const int len = __builtin_amdgcn_readfirstlane(sh_geo_hi[q]) - lo + 1;
                const int wo = __builtin_amdgcn_readfirstlane(sh_woff[q]);
                for (int j0 = 0; j0 < len; j0 += WAVE)
                    if (j0 + lane < len)
                        __builtin_amdgcn_raw_ptr_buffer_load_lds(prs, (__attribute__((address_space(3))) void *)&stage[wo + j0],
                                                                 4, lane * 4, (lo + j0) * 4, 0, 0);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the LDS writes of this wave's loads are done
            const int foff = sh_woff[n_ref];
            for (int i = foff + lane; i < stage_total; i += WAVE) {
                const float d = db_of(stage[i]);
                if (d > best) {
                    best = d;
                    bidx = g.focus_lo + (i - foff);
                }
            }
            for (int off = WAVE / 2; off > 0; off >>= 1) {  // first maximum over the lanes (lower bin on ties)
                const float ob = __shfl_xor(best, off);
                const int oi = __shfl_xor(bidx, off);
                if (ob > best || (ob == best && oi < bidx)) {
                    best = ob;
                    bidx = oi;
                }
            }
        }
        __syncthreads();
        if (SDRG_STATS_STAMPS && threadIdx.x == 0 && blockIdx.x < 8192)  // slot 6: the staging copy's cycles
            g_stats_stamps[blockIdx.x * STAMP_PHASES + 6] = __builtin_amdgcn_s_memtime() - g_stats_stamps[blockIdx.x * STAMP_PHASES];
        const float abs_peak_db = best;
        const int peak_bin = (bidx == 0x7fffffff) ? g.focus_lo : bidx;

        // ---- 6.2 focus sum + 6.3 reference windows: lane q scans window q (the focus is window n_ref) ----
        if (lane <= n_ref) {
            const int lo = sh_geo_lo[lane], hi = sh_geo_hi[lane], n = hi - lo + 1;
            const WinScan ws = scan_window(stage + sh_woff[lane], lo, hi, w1k);
            if (lane == n_ref) {
                sh_f[0] = db_of(ws.sum / n);  // signalPowerDb (:155)
                sh_f[1] = ws.best1k;          // focusBest1kLinear (:302)
                sh_best_start = ws.best_start;
            } else {
                w_mean_db[lane] = db_of(ws.sum / n);
                w_best1k_db[lane] = db_of(ws.best1k);
            }
        }
        __syncthreads();
        STATS_STAMP(1);
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
            // std::sort of <= 16 elements in libstdc++ is a (stable) insertion sort: the same order is a sort by
            // (meanDb, window index); lane i places window i at its rank
            if (lane < n_ref) {
                const float ki = w_mean_db[lane];
                int rank = 0;
                for (int k = 0; k < n_ref; k++) {
                    const float kk = w_mean_db[k];
                    rank += (kk < ki || (kk == ki && k < lane)) ? 1 : 0;
                }
                order[rank] = lane;
            }
            __syncthreads();
            const int n_bottom = n_bottom_of(n_ref);
            if (lane == 0) mean_snr_6_4a(w_mean_db, order, n_ref, signal_power_db, st);
            STATS_STAMP(2);

            // ---- 6.4b pooled per-bin dB of the bottom windows, sorted-window order (:252-269) ----
            // pool value q lies in bottom window j (cum[j] <= q < cum[j + 1]) at staged bin q + basej[j]
            int cum[5], basej[4];
            cum[0] = 0;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const bool in = j < n_bottom;
                const int wj = in ? order[j] : 0;
                cum[j + 1] = cum[j] + (in ? sh_geo_hi[wj] - sh_geo_lo[wj] + 1 : 0);
                basej[j] = (in ? sh_woff[wj] : 0) - cum[j];
            }
            const int cnt = cum[4];
            // as a sum of steps (a select chain over basej[] becomes an indexed load from scratch)
            const int d1 = basej[1] - basej[0], d2 = basej[2] - basej[1], d3 = basej[3] - basej[2];
            auto staged_of = [&](int q) {
                return q + basej[0] + (q >= cum[1] ? d1 : 0) + (q >= cum[2] ? d2 : 0) + (q >= cum[3] ? d3 : 0);
            };
            // the pool in order (zero tail up to a 16-value block), for lane 0's float4 reads: over the staged
            // bins once every lane has read them (R > 0), or in its own region after them (R == 0)
            float *pl = R > 0 ? stage : stage + stage_pad;
            float v[R > 0 ? R : 1];
            if constexpr (R > 0) {
#pragma unroll
                for (int r = 0; r < R; r++) {
                    const int q = lane + WAVE * r;
                    v[r] = 0.0f;
                    if (q < cnt) v[r] = db_of(stage[staged_of(q)]);
                }
                __syncthreads();
#pragma unroll
                for (int r = 0; r < R; r++) {
                    const int q = lane + WAVE * r;
                    if (q < ((cnt + 15) & ~15)) pl[q] = v[r];
                }
            } else {
                for (int q = lane; q < ((cnt + 15) & ~15); q += WAVE) pl[q] = q < cnt ? db_of(stage[staged_of(q)]) : 0.0f;
            }
            __syncthreads();
            if (lane == 0) {
                // the sequential sum (:259-263), 16 values per block read as four float4 one block ahead; the
                // zero tail is not added
                float m = 0.0f;
                float4 A[4], B[4];
                auto rd = [&](float4 (&X)[4], int u) {
#pragma unroll
                    for (int i = 0; i < 4; i++) X[i] = *reinterpret_cast<const float4 *>(pl + u + 4 * i);
                };
                auto add16 = [&](const float4 (&X)[4], int n) {
                    const float x[16] = {X[0].x, X[0].y, X[0].z, X[0].w, X[1].x, X[1].y, X[1].z, X[1].w,
                                         X[2].x, X[2].y, X[2].z, X[2].w, X[3].x, X[3].y, X[3].z, X[3].w};
                    if (n >= 16) {
#pragma unroll
                        for (int i = 0; i < 16; i++) m += x[i];
                    } else {
#pragma unroll
                        for (int i = 0; i < 16; i++)
                            if (i < n) m += x[i];
                    }
                };
                rd(A, 0);
                for (int q = 0; q < cnt; q += 32) {
                    if (q + 16 < cnt) rd(B, q + 16);
                    add16(A, cnt - q);
                    if (q + 16 >= cnt) break;
                    if (q + 32 < cnt) rd(A, q + 32);
                    add16(B, cnt - q - 16);
                }
                sh_f[2] = m / (float)cnt;
            }
            __syncthreads();
            const float per_bin_mean = sh_f[2];
            STATS_STAMP(3);
            float med;
            if constexpr (R > 0) {
#pragma unroll
                for (int r = 0; r < R; r++) v[r] = fabsf(v[r] - per_bin_mean);
                med = kth_smallest_wave(
                    [&](auto f) {
#pragma unroll
                        for (int r = 0; r < R; r++)
                            if (lane + WAVE * r < cnt) f(__float_as_uint(v[r]));
                    },
                    cnt / 2, hist, sh_xch);
            } else {
                med = kth_smallest_wave(
                    [&](auto f) {
                        for (int q = lane; q < cnt; q += WAVE) f(__float_as_uint(fabsf(pl[q] - per_bin_mean)));
                    },
                    cnt / 2, hist, sh_xch);
            }
            STATS_STAMP(4);
            const float sigma_bin = (cnt > 0) ? fmax_ref(1.4816f * med, 1.0f) : 1.0f;
            if (cnt > 0) st.per_bin_mean = per_bin_mean;
            const float pbm = (cnt > 0) ? per_bin_mean : 0.0f;
            if (lane == 0)
                snr_6_4cd(g, st, abs_peak_db, pbm, sigma_bin, n_bottom, w_best1k_db, order, sh_f[1], sh_best_start);
        }
        STATS_STAMP(5);
        if (lane == 0) track_detect_6_5_6_6(g, st, valid, abs_peak_db, peak_bin, now_ms);
    }
    if (lane == 0) {
        finish_record(rec, st);
        if (records) records[frame] = rec;
        state[frame] = st;
    }
}

// Wide statistics: windows too wide to stage together (BASELINE configs[4]: 65536 bins at a 200 kHz focus),
// one WIDE_WG-thread workgroup per frame; the window scans in scan_wide, the pool in the frame's slice of the
// global scratch gpool (or in registers when it fits).
__global__ __launch_bounds__(WIDE_WG) __attribute__((amdgpu_waves_per_eu(4))) void stats_wide_kernel(
    const float *__restrict__ spectra, StatsGeometry g, int64_t now_ms, StatsState *__restrict__ state,
    sdrg_frame_record *__restrict__ records, float *gpool, int gpool_stride) {
    constexpr int WG = WIDE_WG;
    extern __shared__ __attribute__((aligned(16))) float dyn[];  // scan_wide's ring
    __shared__ __attribute__((aligned(16))) int hist[256];
    __shared__ uint32_t sh_xch[10];
    __shared__ WideScan sh_wide;
    __shared__ int sh_best_start;
    __shared__ float w_mean_db[10], w_best1k_db[10], w_dsum[10];
    __shared__ int w_lo[10], w_hi[10], order[10];
    __shared__ float sh_f[4];
    __shared__ int sh_geo_lo[11], sh_geo_hi[11];  // the reference windows, then the focus window (index n_ref)

    const int lane = threadIdx.x;
    const size_t frame = blockIdx.x;
    const int n_ref = g.n_ref;
    load_logf_tab();
    load_logf_fold();
    // the window bounds are indexed by thread below: copy them out of the kernel arguments with constant
    // indices (a thread-indexed kernarg array would be copied to scratch)
#pragma unroll
    for (int i = 0; i < 10; i++) {
        if (lane == i) {
            sh_geo_lo[i] = g.win_lo[i];
            sh_geo_hi[i] = g.win_hi[i];
        }
    }
    if (lane == 0) {
        sh_geo_lo[n_ref] = g.focus_lo;
        sh_geo_hi[n_ref] = g.focus_hi;
    }
    __syncthreads();
    const int role = threadIdx.x >> 6;  // scan_wide's roles by wave
    const float *P = spectra + frame * (size_t)g.n;
    float *pool = gpool + frame * (size_t)gpool_stride;
    StatsState st = state[frame];
    if (g.cf_changed) st.center_frequency_changed = 1;  // sdr_bridge_internal::isCenterFrequencyChanged
    sdrg_frame_record rec;
    __builtin_memset(&rec, 0, sizeof(rec));  // tail padding included: records compare and gather as bytes
    rec.peak_bin = -1;
    rec.abs_peak_db = -130.0f;

    if (g.focus_len > 0) {
        const int w1k = g.win_bins_1k;
        const int n_bottom = n_bottom_of(n_ref);
        const bool spec_pool = n_ref >= 2 && n_bottom == 1;  // pooled-bin sum = one window's dB sum
        STATS_STAMP(0);
        const int wst = (g.max_pool + 3) & ~3;  // SDRG_WIDE_DBPOOL: window q's dB values at pool + q * wst
        if (spec_pool)
            scan_wide<true>(P, dyn, n_ref + 1, sh_geo_lo, sh_geo_hi, w1k, role, pool, wst, sh_wide);
        else
            scan_wide<false>(P, dyn, n_ref + 1, sh_geo_lo, sh_geo_hi, w1k, role, pool, wst, sh_wide);
        STATS_STAMP(1);
        const float abs_peak_db = sh_wide.peak_db;  // 6.2 focus peak (fft_process.cpp:142-154)
        const int peak_bin = sh_wide.peak_idx;
        if (lane < n_ref) w_dsum[lane] = sh_wide.dsum[lane];
        // ---- 6.2 focus sum + 6.3 reference windows ----
        if (lane <= n_ref) {
            const int lo = sh_geo_lo[lane], hi = sh_geo_hi[lane], n = hi - lo + 1;
            WinScan ws;
            ws.sum = sh_wide.sum[lane];
            ws.best_start = lo;
            if (n <= 0) {
                ws.best1k = 0.0f;
            } else if (n < w1k) {
                ws.best1k = ws.sum / n;
            } else {
                ws.best1k = sh_wide.bv[lane] / w1k;  // as scan_window: RN(max rs / w)
                ws.best_start = lo + sh_wide.best_e[lane] - w1k + 1;
            }
            if (lane == n_ref) {
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
            // std::sort of <= 16 elements in libstdc++ is a (stable) insertion sort: the same order is a sort by
            // (meanDb, window index); thread i places window i at its rank
            if (lane < n_ref) {
                const float ki = w_mean_db[lane];
                int rank = 0;
                for (int k = 0; k < n_ref; k++) {
                    const float kk = w_mean_db[k];
                    rank += (kk < ki || (kk == ki && k < lane)) ? 1 : 0;
                }
                order[rank] = lane;
            }
            __syncthreads();
            if (lane == 0) mean_snr_6_4a(w_mean_db, order, n_ref, signal_power_db, st);
            STATS_STAMP(2);
            // ---- 6.4b pooled per-bin dB of the bottom windows, sorted-window order (:252-269) ----
            int cnt = 0;
            float med = 0.0f, per_bin_mean = 0.0f;
            if (spec_pool) {
                // one bottom window: its dB sum came out of the wide scan (same values, same order, from 0); the
                // pool holds the |dB - mean| gaps directly
                const int wb = order[0];
                const int lo = w_lo[wb], hi = w_hi[wb];
                cnt = hi - lo + 1;
                per_bin_mean = w_dsum[wb] / (float)cnt;
                const float m = per_bin_mean;
                if (cnt <= REG_POOL * WG) {
                    // gaps in registers: the select's passes read no memory
                    float v[REG_POOL];
                    if constexpr (SDRG_WIDE_DBPOOL) {  // the scan's dB values of window wb
                        const float *gd = pool + wb * wst;
#pragma unroll
                        for (int r = 0; r < REG_POOL; r++) {
                            const int q = lane + WG * r;
                            v[r] = q < cnt ? gd[q] : m;
                        }
#pragma unroll
                        for (int r = 0; r < REG_POOL; r++) v[r] = fabsf(v[r] - m);
                    } else {
#pragma unroll
                        for (int r = 0; r < REG_POOL; r++) {
                            const int q = lane + WG * r;
                            v[r] = q < cnt ? P[lo + q] : 0.0f;
                        }
#pragma unroll
                        for (int r = 0; r < REG_POOL; r++) {
                            v[r] = fabsf(db_fold(v[r]) - m);
                            __builtin_amdgcn_sched_barrier(0);  // one log10 at a time (register pressure)
                        }
                    }
                    STATS_STAMP(3);
                    med = kth_smallest<WG>(
                        [&](auto f) {
#pragma unroll
                            for (int r = 0; r < REG_POOL; r++)
                                if (lane + WG * r < cnt) f(__float_as_uint(v[r]));
                        },
                        cnt / 2, hist, sh_xch);
                } else {
#pragma unroll 4
                    for (int i = lo + lane; i <= hi; i += WG) pool[i - lo] = fabsf(db_fold(P[i]) - m);
                    __syncthreads();
                    STATS_STAMP(3);
                    med = kth_smallest_of<WG>(pool, cnt, cnt / 2, hist, sh_xch);
                }
            } else {
                // several bottom windows: pooled in HBM scratch, summed in order by one thread
                for (int j = 0; j < n_bottom; j++) {
                    const int wj = order[j], len = w_hi[wj] - w_lo[wj] + 1;
                    const float *src = P + w_lo[wj];
#pragma unroll 8
                    for (int i = lane; i < len; i += WG) {
                        const int q = cnt + i;
                        if (q < g.max_pool) pool[q] = db_fold(src[i]);
                    }
                    cnt += len;
                }
                if (cnt > g.max_pool) cnt = g.max_pool;  // host sizes max_pool from the geometry
                __syncthreads();
                if (lane == 0) {
                    float m = 0.0f;
#pragma unroll 8
                    for (int q = 0; q < cnt; q++) m += pool[q];
                    sh_f[2] = m / (float)cnt;
                }
                __syncthreads();
                per_bin_mean = sh_f[2];
                for (int q = lane; q < cnt; q += WG) pool[q] = fabsf(pool[q] - per_bin_mean);
                __syncthreads();
                STATS_STAMP(3);
                med = kth_smallest_of<WG>(pool, cnt, cnt / 2, hist, sh_xch);
            }
            STATS_STAMP(4);
            const float sigma_bin = (cnt > 0) ? fmax_ref(1.4816f * med, 1.0f) : 1.0f;
            if (cnt > 0) st.per_bin_mean = per_bin_mean;
            const float pbm = (cnt > 0) ? per_bin_mean : 0.0f;
            if (lane == 0)
                snr_6_4cd(g, st, abs_peak_db, pbm, sigma_bin, n_bottom, w_best1k_db, order, sh_f[1], sh_best_start);
        }
        STATS_STAMP(5);
        if (lane == 0) track_detect_6_5_6_6(g, st, valid, abs_peak_db, peak_bin, now_ms);
    }
    if (lane == 0) {
        finish_record(rec, st);
        if (records) records[frame] = rec;
        state[frame] = st;
    }
}


// ------------------------------------------------------------------------------------------------
// Wide statistics, four frames per workgroup (stats_wide_multi_kernel), for the geometries whose pooled gaps are one
// bottom window (n_ref 2..4) or none (n_ref < 2) -- BASELINE configs[4]: 65536 bins, 200 kHz focus, two reference
// windows of 13107 bins.  The single-frame kernel above spends most of its VALU on glibc-exact log10s (~30 VALU each,
// nine of them f64): every focus bin's (the focus peak), every reference bin's (the pooled mean's dB sums) and, for
// the pool, the bottom window's again or through HBM scratch.  This kernel evaluates only the logs the reference's
// results depend on bin by bin:
//   * the focus peak from powers alone: dB(p) = 10 log10f(p + 1e-20) never decreases with p (glibc's log10f is
//     monotone, checked over every float: tests/test_libm_exact.py), so the first maximum of the dB values is the
//     first focus bin whose power reaches p_lo, the smallest float with the dB of the largest power M.  During the
//     scan each producer lane keeps its largest power and up to MW_K candidate bins (index order) whose power came
//     within MW_DELTA of its running maximum; after it, p_lo is found among the 256 floats below M, and the peak is
//     the first candidate >= p_lo.  A frame whose candidates overflowed, or whose p_lo is not within MW_DELTA / 2
//     of M (powers where the 1e-20 dominates), re-scans its focus window for the first bin >= p_lo instead;
//   * the reference windows' dB values for their dB sums in the scan (the chain wave), as scan_wide;
//   * the bottom window's pooled gaps again after the scan, in parallel, into registers: nothing per bin goes to
//     HBM, and the pool costs one more read of that window (MALL-resident: the scan read it just before).
// ONE chain wave runs the sequential sums of the four frames side by side (16 lanes per frame: window sums, running
// sums, dB sums), one record wave takes the strict `rs > bv` records of all four, and the producer waves stream every
// window of every frame into the four rings (three lanes on a reference window per lane on the focus: its bins carry
// no log).  Sums, records and peaks are the reference's, in its order; results cross lanes through LDS keys (value,
// then the lower index) so that one atomic max picks the same element as scan_wide's shuffle reductions.  Each frame's
// tail (6.2-6.6) runs on wave f, its pooled median on MW_T / 4 threads (four radix selects at once).  One 1024-thread
// workgroup per CU: 1024 frames fill the chip once.
#ifndef SDRG_MW_T  // threads per multi-frame workgroup
#define SDRG_MW_T 1024
#endif
constexpr int MW_T = SDRG_MW_T;
// lab: SDRG_MW_STAMPS=1 records s_memtime per workgroup at the phase boundaries (and each scan role's busy cycles)
#ifndef SDRG_MW_STAMPS
#define SDRG_MW_STAMPS 0
#endif
#define MW_STAMP(k)                                                                                            \
    do {                                                                                                       \
        if (SDRG_MW_STAMPS && threadIdx.x == 0 && blockIdx.x < 8192)                                           \
            g_stats_stamps[blockIdx.x * STAMP_PHASES + (k)] = __builtin_amdgcn_s_memtime();                    \
    } while (0)
constexpr int MW_F = 4;                     // frames per workgroup
#ifndef SDRG_MW_WREF  // producer lanes per reference-window lane per focus lane (a reference bin carries a log10)
#define SDRG_MW_WREF 2
#endif
#ifndef SDRG_MW_ILP  // 1: the reference producers' log10s of several bins interleave (no scheduling barrier)
#define SDRG_MW_ILP 1
#endif
// The pooled gaps' dB values: 0 = evaluated again after the scan (13107 glibc-exact log10s per frame
// at 65536 / 200 kHz, the "pool logs" phase); 1 = the record waves copy every reference window's dB row of the chunk the
// chain is reading from the LDS ring to a per-frame HBM scratch during the scan (they issue no loads, so their stores
// hold up no wait), and the pool phase loads the bottom window's values from it (the same floats: the producers'
// db_fold), past L1 (sc1)
// Measured (r6m, alternating, one box): the kernel alone at 1024 x 65536 / 200 kHz 183.8 / 184.6 -> 173.3 / 176.0 us,
// the configs[4] 200 kHz line 137.3 / 137.4 -> 141.1 / 140.8 G; the statistics GPU tests bit-exact (105 passed).
#ifndef SDRG_MW_DBPOOL
#define SDRG_MW_DBPOOL 1
#endif
constexpr int MW_RECW = MW_F;  // record waves: one per frame
constexpr int MW_P0 = 1 + MW_RECW;          // first producer wave
constexpr int MW_PROD = MW_T - 64 * MW_P0;  // producer lanes
constexpr int MW_PR = 12;                   // bins per producer lane per chunk at most (the host sizes SC for it)
constexpr int MW_RING_FLOATS = 28672;       // 112 KiB of rings at most
constexpr int MW_POOL = 13312;              // pooled gaps per frame held in registers
constexpr int MW_K = 4;                     // focus candidates per producer lane
constexpr float MW_DELTA = 1e-4f;           // candidates: power >= running maximum x (1 - MW_DELTA)

// float -> uint32 with the float order (-0 taken as +0, as a float compare does); NaN never reaches it
__device__ __forceinline__ uint32_t ord_f(float x) {
    const uint32_t b = __float_as_uint(x + 0.0f);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float unord_f(uint32_t o) {
    return __uint_as_float((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o);
}
// key of (value, index): a larger value wins, then the lower index (scan_wide's `om > m || (om == m && oi < mi)`)
__device__ __forceinline__ unsigned long long vi_key(float v, int i) {
    return ((unsigned long long)ord_f(v) << 32) | (unsigned long long)(0xffffffffu - (uint32_t)i);
}

// producer lanes per focus item and per reference item: a reference bin costs about three times a focus bin (its
// log10), so reference windows get three times the lanes; without dB sums, equal shares
__host__ __device__ inline void mw_lanes(int n_ref, bool want_db, int *pgf, int *pgr) {
    const int fq = n_ref, nwin = n_ref + 1;
    if (want_db && fq > 0) {
        *pgf = MW_PROD / (SDRG_MW_WREF * MW_F * fq + MW_F);
        *pgr = (MW_PROD - MW_F * *pgf) / (MW_F * fq);
    } else {
        *pgf = *pgr = MW_PROD / (MW_F * nwin);
    }
}

template <bool want_db>
__global__ __launch_bounds__(MW_T) __attribute__((amdgpu_waves_per_eu(MW_T / 256))) void stats_wide_multi_kernel(
    const float *__restrict__ spectra, int n_frames, StatsGeometry g, int64_t now_ms, StatsState *__restrict__ state,
    sdrg_frame_record *__restrict__ records, int lg, float *__restrict__ gdb, int wst) {
    constexpr int F = MW_F, GT = MW_T / F, REG = (MW_POOL + GT - 1) / GT, LPFR = WAVE / F, GW = GT / WAVE;
    // SDRG_MW_DBPOOL: frame f's reference window q's dB values at gdb[((f0 + f) * n_ref + q) * wst + e]
    extern __shared__ __attribute__((aligned(16))) float ring[];
    __shared__ __attribute__((aligned(16))) int hist[F][256];
    __shared__ uint32_t sxch[F][2];
    __shared__ uint32_t sband[MW_T / WAVE][2];
    __shared__ int s_wt[MW_T / WAVE];
    __shared__ unsigned long long s_rec[F][11];
    __shared__ uint32_t s_pmax[F];
    __shared__ int s_ovf[F], s_t[F], s_first[F];
    __shared__ float s_sum[F][11], s_dsum[F][11], s_med[F], s_plo[F];
    __shared__ float w_mean_db[F][10], w_best1k_db[F][10], sh_f[F][2];
    __shared__ int order[F][10], sh_best_start[F];
    __shared__ int sh_geo_lo[11], sh_geo_hi[11];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int n_ref = g.n_ref, nwin = n_ref + 1, fq = n_ref;
    const int f0 = blockIdx.x * F;
    load_logf_tab();
    load_logf_fold();
#pragma unroll
    for (int i = 0; i < 10; i++) {
        if (tid == i) {
            sh_geo_lo[i] = g.win_lo[i];
            sh_geo_hi[i] = g.win_hi[i];
        }
    }
    if (tid == 0) {
        sh_geo_lo[n_ref] = g.focus_lo;
        sh_geo_hi[n_ref] = g.focus_hi;
    }
    if (tid < F) {
        s_pmax[tid] = 0u;  // below every ordered float: no focus bin
        s_ovf[tid] = 0;
        s_t[tid] = 256;
        s_first[tid] = 0x7fffffff;
    }
    if (tid < F * 11) s_rec[tid / 11][tid % 11] = 0ull;
    __syncthreads();
    MW_STAMP(0);

    const int SC = 1 << lg, RS = SC + 4, slot_floats = 3 * RS * nwin, frame_floats = 8 * RS * nwin;
    int max_len = 0;
    for (int q = 0; q < nwin; q++) max_len = max(max_len, sh_geo_hi[q] - sh_geo_lo[q] + 1);
    const int nch = (max_len + SC - 1) >> lg;
    const int w = g.win_bins_1k;
    auto frame_of = [&](int f) { return min(f0 + f, n_frames - 1); };  // loads of a missing frame: a real one
    auto frame_ptr = [&](int f) { return spectra + (size_t)frame_of(f) * (size_t)g.n; };

    // ---- chain wave: lane = LPFR x frame + j; j < nwin window sums, then running sums, then dB sums ----
    const int cf = lane / LPFR, cjj = lane - cf * LPFR;
    int cg = 3, cj = 0;
    if (cjj < nwin) cg = 0, cj = cjj;
    else if (cjj < 2 * nwin) cg = 1, cj = cjj - nwin;
    else if (want_db && cjj < 3 * nwin - 1) cg = 2, cj = cjj - 2 * nwin;
    const bool chain = wave == 0 && cg < 3;
    float acc = 0.0f;
    // ---- record waves: wave 1 + f for frame f, G lanes per window ----
    const int G = WAVE / nwin, ritem = lane / G, rq = ritem % nwin, rk = lane - ritem * G;
    const int rwave = wave >= 1 && wave <= MW_RECW ? wave - 1 : -1;  // record wave index
    const int rf = rwave;
    const bool rec_lane = rwave >= 0 && ritem < nwin;
    float rm = -INFINITY;
    int ri = 0x7fffffff;
    // ---- producers: the F focus items first (pgf lanes each), then the F x fq reference items (pgr lanes each) ----
    int pgf, pgr;
    mw_lanes(n_ref, want_db, &pgf, &pgr);
    // producer ordinal: the waves that are neither the chain nor a record wave, in order
    const int pwave = wave - MW_P0;
    const bool is_prod_wave = wave != 0 && rwave < 0;
    const int pw = pwave * 64 + lane;
    int pf = 0, pq = 0, pk0 = 0, PGc = 1;
    bool prod = false;
    if (is_prod_wave) {
        if (want_db) {
            if (pw < F * pgf) {
                pf = pw / pgf, pq = fq, pk0 = pw - pf * pgf, PGc = pgf, prod = true;
            } else if (fq > 0) {
                const int r = pw - F * pgf, it = r / pgr;
                pf = it / fq, pq = it - pf * fq, pk0 = r - it * pgr, PGc = pgr, prod = it < F * fq;
            }
        } else {
            const int it = pw / pgf;
            pf = it / nwin, pq = it - pf * nwin, pk0 = pw - it * pgf, PGc = pgf, prod = it < F * nwin;
        }
    }
    const bool foc_lane = prod && pq == fq;
    const int plo = sh_geo_lo[prod ? pq : 0], plen = sh_geo_hi[prod ? pq : 0] - plo + 1;
    const float *Pq = frame_ptr(prod ? pf : 0) + plo;
    float va[MW_PR], vb[MW_PR];
    // focus candidates: the lane's running maximum cm, up to MW_K bins (index order) that came within MW_DELTA of it
    float cm = -INFINITY, cv[MW_K];
    int ci[MW_K], nc = 0;
    bool ovf = false;
#pragma unroll
    for (int j = 0; j < MW_K; j++) {
        cv[j] = 0.0f;
        ci[j] = 0x7fffffff;
    }
    // (the slots t >= SC are masked, not branched over: branches around each bin's log10 cost the producers 70 % more
    // time, tools/gpu_r4g.sh)
    auto fetch = [&](int c) {
        const int c0 = c << lg;
#pragma unroll
        for (int k = 0; k < MW_PR; k++) {
            const int t = pk0 + PGc * k, e = c0 + t;
            const bool ok = t < SC && e < plen;
            va[k] = ok ? Pq[e] : 0.0f;
            vb[k] = (ok && e >= w) ? Pq[e - w] : 0.0f;
        }
    };
    auto store = [&](int c) {
        const int c0 = c << lg;
        float *row = ring + pf * frame_floats + (c & 1) * slot_floats + pq * 3 * RS;
#pragma unroll
        for (int k = 0; k < MW_PR; k++) {
            const int t = pk0 + PGc * k, e = c0 + t;
            if (t < SC) {
                const bool in = e < plen;
                const float v = va[k];
                row[t] = v;
                row[RS + t] = (e >= w) ? v - vb[k] : v;
                if (foc_lane) {
                    if (in) {
                        // a lane sees its focus bins in increasing order.  A new maximum more than MW_DELTA above the
                        // last drops every candidate (all are then below any p_lo the check below accepts)
                        if (v > cm) {
                            if (v * (1.0f - MW_DELTA) > cm) nc = 0;
                            cm = v;
                        }
                        if (v >= cm * (1.0f - MW_DELTA)) {
#pragma unroll
                            for (int j = 0; j < MW_K; j++) {
                                cv[j] = (nc == j) ? v : cv[j];
                                ci[j] = (nc == j) ? plo + e : ci[j];
                            }
                            ovf = ovf || nc == MW_K;
                            nc = min(nc + 1, MW_K);
                        }
                    }
                } else if (want_db) {
                    row[2 * RS + t] = in ? db_fold(v) : 0.0f;
                }
            }
            if (!SDRG_MW_ILP) __builtin_amdgcn_sched_barrier(0);  // one bin's log10 at a time
        }
    };
    if (prod && nch > 0) fetch(0);

    unsigned long long busy = 0;
    for (int c = 0; c <= nch + 1; c++) {
        const unsigned long long t_in = SDRG_MW_STAMPS ? __builtin_amdgcn_s_memtime() : 0;
        if (is_prod_wave) {
            if (prod && c < nch) {
                store(c);
                if (c + 1 < nch) fetch(c + 1);
            }
        } else if (wave == 0) {
            if (c >= 1 && c <= nch && chain) {
                const float *slot = ring + cf * frame_floats + ((c - 1) & 1) * slot_floats;
                const float *src = slot + (cj * 3 + cg) * RS;  // x, rs terms, dB rows
                float *rsring = ring + cf * frame_floats + 2 * slot_floats;
                // running values: the rs lanes' go to the rs ring (the record wave reads them); the window and dB
                // sums' are never read and go back over the consumed bins row
                float *dst = cg == 1 ? rsring + (((c - 1) & 1) * nwin + cj) * RS : const_cast<float *>(slot + cj * 3 * RS);
                float4 A[4], B[4];
                auto rd = [&](float4 (&X)[4], int u) {
#pragma unroll
                    for (int i = 0; i < 4; i++) X[i] = *reinterpret_cast<const float4 *>(src + u + 4 * i);
                };
                auto sum16 = [&](const float4 (&X)[4], int u) {
                    float4 r[4];
#pragma unroll
                    for (int i = 0; i < 4; i++) {
                        acc += X[i].x;
                        r[i].x = acc;
                        acc += X[i].y;
                        r[i].y = acc;
                        acc += X[i].z;
                        r[i].z = acc;
                        acc += X[i].w;
                        r[i].w = acc;
                    }
#pragma unroll
                    for (int i = 0; i < 4; i++) *reinterpret_cast<float4 *>(dst + u + 4 * i) = r[i];
                };
                rd(A, 0);
                for (int t = 0; t < SC; t += 32) {  // SC >= 64, a multiple of 32
                    rd(B, t + 16);
                    sum16(A, t);
                    if (t + 32 < SC) rd(A, t + 32);
                    sum16(B, t + 16);
                }
            }
        } else if (rwave >= 0) {
            if (SDRG_MW_DBPOOL && want_db && c >= 1 && c <= nch) {
                // chunk c - 1's reference dB rows of this wave's frame (stable in the ring until the producers' store of
                // chunk c + 1) to the frame's HBM scratch, 16 bytes per lane and store
                const int c0 = (c - 1) << lg;
                const float *rows = ring + rf * frame_floats + ((c - 1) & 1) * slot_floats + 2 * RS;
                float *fdb = gdb + (size_t)(f0 + rf) * (size_t)fq * (size_t)wst;
                for (int i4 = lane; i4 < (fq << lg) / 4; i4 += WAVE) {
                    const int q = (4 * i4) >> lg, t = (4 * i4) & (SC - 1), e = c0 + t;
                    if (e < sh_geo_hi[q] - sh_geo_lo[q] + 1)
                        *reinterpret_cast<float4 *>(fdb + q * wst + e) = *reinterpret_cast<const float4 *>(rows + q * 3 * RS + t);
                }
            }
            if (rec_lane && c >= 2) {
            // chunk c - 2's running sums: lane k of the group visits bins k, k + G, ... in increasing order
            const int c0 = (c - 2) << lg;
            const float *rsrow = ring + rf * frame_floats + 2 * slot_floats + ((c & 1) * nwin + rq) * RS;
            if (c0 + SC > w - 1) {
                for (int t = rk; t < SC; t += G) {
                    const float v = rsrow[t];
                    const bool gt = c0 + t >= w - 1 && v > rm;  // strict: the lane keeps its first maximum
                    rm = gt ? v : rm;
                    ri = gt ? c0 + t : ri;
                }
            }
            }
        }
        if (SDRG_MW_STAMPS) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            busy += __builtin_amdgcn_s_memtime() - t_in;
        }
        wide_chunk_barrier();
    }
    if (SDRG_MW_STAMPS && lane == 0 && blockIdx.x < 8192) {  // chain, a record wave, a focus and a reference producer
        const int slot = wave == 0 ? 7 : rwave == 0 ? 8 : (is_prod_wave && pwave == 0) ? 9 : wave == MW_T / 64 - 1 ? 10 : -1;
        if (slot > 0) g_stats_stamps[blockIdx.x * STAMP_PHASES + slot] = busy;
    }
    // the dB scratch: every store done before the barrier below, after which other waves load it
    if (SDRG_MW_DBPOOL && want_db && rwave >= 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // ---- per-frame results through LDS ----
    if (foc_lane && cm > -INFINITY) atomicMax(&s_pmax[pf], ord_f(cm));
    if (foc_lane && ovf) atomicOr(&s_ovf[pf], 1);
    if (rec_lane) atomicMax(&s_rec[rf][rq], vi_key(rm, ri));
    if (chain && cg == 0) s_sum[cf][cj] = acc;
    if (chain && cg == 2) s_dsum[cf][cj] = acc;
    __syncthreads();
    MW_STAMP(1);

    // ---- 6.2 focus peak (:142-154): p_lo among the 256 floats below each frame's largest focus power ----
    const int sf = tid / GT, stid = tid - sf * GT;  // the frame this thread works for in the group phases
    const int flo = sh_geo_lo[fq], flen = sh_geo_hi[fq] - flo + 1;
    const uint32_t om = s_pmax[sf];
    const float M = om ? unord_f(om) : 0.0f;
    const float ds = om ? db_of(M) : -130.0f;
    const int bm = __float_as_int(M);
    for (int t = stid; t < 256; t += GT) {
        const int b = bm - t;
        if (ds > -130.0f && b >= 0 && db_of(__int_as_float(b)) != ds) atomicMin(&s_t[sf], t);
    }
    __syncthreads();
    if (stid == 0 && ds > -130.0f) {
        const int T = s_t[sf];
        int plo_b = bm - (T - 1);
        if (T == 256) {  // every tested neighbour shares the maximum's dB (the 1e-20 floor): bisect below them
            int lo = 0, hi = bm - 255;
            if (hi <= 0) {
                lo = 0;
            } else {
                while (lo < hi) {
                    const int mid = lo + ((hi - lo) >> 1);
                    if (db_of(__int_as_float(mid)) == ds) hi = mid;
                    else lo = mid + 1;
                }
            }
            plo_b = lo;
        }
        const float pl = __int_as_float(plo_b < 0 ? 0 : plo_b);
        s_plo[sf] = pl;
        // the candidates hold every bin >= p_lo when p_lo is within MW_DELTA / 2 of M and no lane overflowed
        if (s_ovf[sf] || !(pl >= M * (1.0f - 0.5f * MW_DELTA))) s_ovf[sf] = 2;
    }
    __syncthreads();
    if (ds > -130.0f) {
        const float pl = s_plo[sf];
        if (s_ovf[sf]) {  // the frame's focus window, read again: the first bin >= p_lo
            const float *Pf = frame_ptr(sf) + flo;
            for (int i = stid; i < flen; i += GT)
                if (Pf[i] >= pl) {
                    atomicMin(&s_first[sf], flo + i);
                    break;
                }
        }
    }
    if (foc_lane) {  // the lane's first candidate >= p_lo (every candidate frame's threads: only where no re-scan ran)
        const float pl = s_plo[pf];
        const uint32_t omf = s_pmax[pf];
        if (omf && !s_ovf[pf] && db_of(unord_f(omf)) > -130.0f) {
            int first = 0x7fffffff;
#pragma unroll
            for (int j = MW_K - 1; j >= 0; j--)
                if (j < nc && cv[j] >= pl) first = ci[j];
            if (first != 0x7fffffff) atomicMin(&s_first[pf], first);
        }
    }
    __syncthreads();
    MW_STAMP(2);

    // ---- each frame's tail on wave f (6.2 focus sum, 6.3 reference windows, sort, 6.4a) ----
    const bool tw = wave < F;
    const int tf = tw ? wave : 0;
    const uint32_t omt = s_pmax[tf];
    const float ds_t = omt ? db_of(unord_f(omt)) : -130.0f;
    const bool hit = ds_t > -130.0f && s_first[tf] != 0x7fffffff;
    const float abs_peak_db = hit ? ds_t : -130.0f;
    const int peak_bin = hit ? s_first[tf] : flo;
    if (tw && lane <= n_ref) {
        const int lo = sh_geo_lo[lane], hi = sh_geo_hi[lane], n = hi - lo + 1;
        const unsigned long long rkey = s_rec[tf][lane];
        WinScan ws;
        ws.sum = s_sum[tf][lane];
        ws.best_start = lo;
        if (n <= 0) {
            ws.best1k = 0.0f;
        } else if (n < w) {
            ws.best1k = ws.sum / n;
        } else {
            ws.best1k = unord_f((uint32_t)(rkey >> 32)) / w;  // as scan_window: RN(max rs / w)
            ws.best_start = lo + (int)(0xffffffffu - (uint32_t)rkey) - w + 1;
        }
        if (lane == n_ref) {
            sh_f[tf][0] = db_of(ws.sum / n);  // signalPowerDb (:155)
            sh_f[tf][1] = ws.best1k;          // focusBest1kLinear (:302)
            sh_best_start[tf] = ws.best_start;
        } else {
            w_mean_db[tf][lane] = db_of(ws.sum / n);
            w_best1k_db[tf][lane] = db_of(ws.best1k);
        }
    }
    __syncthreads();
    const int valid = (n_ref >= 2);
    if (valid && tw && lane < n_ref) {  // libstdc++'s insertion sort for <= 16 elements: (meanDb, index) order
        const float ki = w_mean_db[tf][lane];
        int rank = 0;
        for (int k = 0; k < n_ref; k++) {
            const float kk = w_mean_db[tf][k];
            rank += (kk < ki || (kk == ki && k < lane)) ? 1 : 0;
        }
        order[tf][rank] = lane;
    }
    __syncthreads();
    const float signal_power_db = sh_f[tf][0];
    MW_STAMP(3);

    // ---- 6.4b: the bottom window's pooled gaps |dB - mean| (:252-269), evaluated again into registers, and their
    //      median: four radix selects at once, GT threads per frame ----
    if (want_db && valid) {
        const int wb = order[sf][0];
        const int lo = sh_geo_lo[wb], cnt = sh_geo_hi[wb] - lo + 1;
        const float m = s_dsum[sf][wb] / (float)cnt;
        float v[REG];
        // slots past the window hold all-ones bits: a gap is never negative (bit 31 clear), so bit 31 is never a
        // differing bit of the real values and the select's prefix never matches them (no per-slot masks to keep)
        if constexpr (SDRG_MW_DBPOOL) {
            const float *Dw = gdb + ((size_t)(f0 + sf) * (size_t)fq + (size_t)wb) * (size_t)wst;
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(Dw), (short)0, cnt * 4, 0x00020000);
#pragma unroll
            for (int r = 0; r < REG; r++)  // out-of-range offsets read 0 from the buffer resource
                v[r] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, (stid + GT * r) * 4, 0, 16));
#pragma unroll
            for (int r = 0; r < REG; r++) v[r] = stid + GT * r < cnt ? fabsf(v[r] - m) : __uint_as_float(0xffffffffu);
        } else {
            const float *Pw = frame_ptr(sf) + lo;
#pragma unroll
            for (int r = 0; r < REG; r++) {
                const int q = stid + GT * r;
                v[r] = q < cnt ? Pw[q] : 0.0f;
            }
#pragma unroll
            for (int r = 0; r < REG; r++) {
                v[r] = stid + GT * r < cnt ? fabsf(db_fold(v[r]) - m) : __uint_as_float(0xffffffffu);
                if (!SDRG_MW_ILP) __builtin_amdgcn_sched_barrier(0);  // one log10 at a time
            }
        }
        MW_STAMP(4);
        uint32_t band = 0xffffffffu, bor = 0u;
#pragma unroll
        for (int r = 0; r < REG; r++) {
            const uint32_t b = __float_as_uint(v[r]);
            band &= b;
            bor |= b == 0xffffffffu ? 0u : b;
        }
        for (int off = WAVE / 2; off > 0; off >>= 1) {
            band &= (uint32_t)__shfl_xor((int)band, off);
            bor |= (uint32_t)__shfl_xor((int)bor, off);
        }
        if (lane == 0) {
            sband[wave][0] = band;
            sband[wave][1] = bor;
        }
        __syncthreads();
        for (int u = sf * GW; u < (sf + 1) * GW; u++) {
            band &= sband[u][0];
            bor |= sband[u][1];
        }
        const uint32_t diff = band ^ bor;
        int top = diff ? 31 - __clz(diff) : -1;  // highest bit where the frame's values differ (-1: all equal)
        uint32_t mask = top >= 31 ? 0u : ~((2u << top) - 1u);
        uint32_t prefix = band & mask;
        int k = cnt / 2;
        {
            // the first digit 12 bits wide, its 4096-bin histogram per frame over the (now idle) rings: the top
            // differing bits of the gaps are mostly exponent bits, which 8-bit digits leave in a few bins, and every
            // lane adding to the same bin serialises the atomics
            int *h1 = reinterpret_cast<int *>(ring) + sf * 4096;
            const bool act = top >= 0;
            const int dlo = top >= 11 ? top - 11 : 0;
            const uint32_t dm = act ? (1u << (top - dlo + 1)) - 1u : 0u;
#pragma unroll
            for (int i = 0; i < 4096 / (4 * GT); i++)
                *reinterpret_cast<int4 *>(&h1[4 * (stid + GT * i)]) = make_int4(0, 0, 0, 0);
            __syncthreads();
            if (act) {
#pragma unroll
                for (int r = 0; r < REG; r++) {
                    const uint32_t b = __float_as_uint(v[r]);
                    if ((b & mask) == prefix) atomicAdd(&h1[(b >> dlo) & dm], 1);
                }
            }
            __syncthreads();
            // bins [16 stid, 16 stid + 16) per thread: their sum, the frame's inclusive prefix over its GT threads
            constexpr int BPT = 4096 / GT;
            int own = 0;
            if (act) {
#pragma unroll
                for (int i = 0; i < BPT; i += 4) {
                    const int4 h = *reinterpret_cast<const int4 *>(&h1[BPT * stid + i]);
                    own += h.x + h.y + h.z + h.w;
                }
            }
            int incl = own;
#pragma unroll
            for (int off = 1; off < WAVE; off <<= 1) {
                const int t = __shfl_up(incl, off);
                if (lane >= off) incl += t;
            }
            if (lane == WAVE - 1) s_wt[wave] = incl;
            __syncthreads();
            for (int u = sf * GW; u < wave; u++) incl += s_wt[u];
            const int excl = incl - own;
            if (act && excl <= k && k < incl) {  // this thread's bins hold the k-th value
                int a = excl, j = 0;
                for (; j < BPT; j++) {
                    const int hv = h1[BPT * stid + j];
                    if (a + hv > k) break;
                    a += hv;
                }
                sxch[sf][0] = (uint32_t)(BPT * stid + j);
                sxch[sf][1] = (uint32_t)a;
            }
            __syncthreads();
            if (act) {
                k -= (int)sxch[sf][1];
                prefix |= sxch[sf][0] << dlo;
                mask |= dm << dlo;
                top = dlo - 1;
            }
        }
        for (int pass = 0; pass < 3; pass++) {  // then 8-bit digits: 12 + 3 x 8 bits cover 32
            const bool act = top >= 0;
            const int dlo = top >= 7 ? top - 7 : 0;
            const uint32_t dm = act ? (1u << (top - dlo + 1)) - 1u : 0u;
            if (stid < 64) *reinterpret_cast<int4 *>(&hist[sf][4 * stid]) = make_int4(0, 0, 0, 0);
            __syncthreads();
            if (act) {
#pragma unroll
                for (int r = 0; r < REG; r++) {
                    const uint32_t b = __float_as_uint(v[r]);
                    if ((b & mask) == prefix) atomicAdd(&hist[sf][(b >> dlo) & dm], 1);
                }
            }
            __syncthreads();
            if (act && stid < 64) {  // the frame's first wave locates the bucket holding the k-th value
                const int4 h = *reinterpret_cast<const int4 *>(&hist[sf][4 * stid]);
                const int own = h.x + h.y + h.z + h.w;
                int incl = own;
#pragma unroll
                for (int off = 1; off < WAVE; off <<= 1) {
                    const int t = __shfl_up(incl, off);
                    if (lane >= off) incl += t;
                }
                const unsigned long long over = __ballot(incl > k);
                const int L = __ffsll((long long)over) - 1;
                if (lane == L) {
                    int a = incl - own;
                    const int hv[4] = {h.x, h.y, h.z, h.w};
                    int j = 3;
#pragma unroll
                    for (int t = 2; t >= 0; t--) {
                        int before = a;
#pragma unroll
                        for (int u = 0; u < t; u++) before += hv[u];
                        if (before + hv[t] > k) j = t;
                    }
#pragma unroll
                    for (int u = 0; u < 3; u++)
                        if (u < j) a += hv[u];
                    sxch[sf][0] = (uint32_t)(4 * L + j);
                    sxch[sf][1] = (uint32_t)a;
                }
            }
            __syncthreads();
            if (act) {
                k -= (int)sxch[sf][1];
                prefix |= sxch[sf][0] << dlo;
                mask |= dm << dlo;
                top = dlo - 1;
            }
        }
        if (stid == 0) s_med[sf] = __uint_as_float(diff ? prefix : band);
        __syncthreads();
        MW_STAMP(5);
    }
    // ---- 6.4c/d, 6.5, 6.6 and the record: lane 0 of wave f ----
    if (tw && lane == 0 && f0 + tf < n_frames) {
        // the stream state only now: held in registers across the pool phase it would crowd out the pooled gaps
        StatsState st = state[f0 + tf];
        if (g.cf_changed) st.center_frequency_changed = 1;  // sdr_bridge_internal::isCenterFrequencyChanged
        if (valid) mean_snr_6_4a(w_mean_db[tf], order[tf], n_ref, signal_power_db, st);  // 6.4a (:235-247)
        sdrg_frame_record rec;
        __builtin_memset(&rec, 0, sizeof(rec));  // tail padding included: records compare and gather as bytes
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
            const int n_bottom = 1;  // want_db: n_ref in 2..4 (nBottom = max(1, int(0.4 n_ref)), :233)
            const int wb = order[tf][0];
            const int cnt = sh_geo_hi[wb] - sh_geo_lo[wb] + 1;
            const float per_bin_mean = s_dsum[tf][wb] / (float)cnt;
            const float med = s_med[tf];
            const float sigma_bin = (cnt > 0) ? fmax_ref(1.4816f * med, 1.0f) : 1.0f;
            if (cnt > 0) st.per_bin_mean = per_bin_mean;
            const float pbm = (cnt > 0) ? per_bin_mean : 0.0f;
            snr_6_4cd(g, st, abs_peak_db, pbm, sigma_bin, n_bottom, w_best1k_db[tf], order[tf], sh_f[tf][1],
                      sh_best_start[tf]);
        }
        track_detect_6_5_6_6(g, st, valid, abs_peak_db, peak_bin, now_ms);
        finish_record(rec, st);
        if (records) records[f0 + tf] = rec;
        state[f0 + tf] = st;
    }
    if (SDRG_MW_STAMPS) {
        __syncthreads();
        MW_STAMP(6);
    }
}

}  // namespace

// spans beyond the LDS stage take the wide kernel (scan_wide), whose pool is in HBM scratch (the radix select's
// passes then read it from L2/MALL; LDS keeps the ring small enough for four frames per CU)
// bins the narrow kernel stages: every reference window and the focus window
static int stage_bins(const StatsGeometry &geo) {
    int o = std::max(0, geo.focus_hi - geo.focus_lo + 1);  // as the kernel's sh_woff
    for (int q = 0; q < geo.n_ref && q < 10; q++) o += std::max(0, geo.win_hi[q] - geo.win_lo[q] + 1);
    return o;
}
static bool wide_for(const StatsGeometry &geo) { return stage_bins(geo) > STAGE_MAX; }
static bool multi_runs(const StatsGeometry &geo);
// the single-frame wide kernel's pool scratch (the multi-frame kernel keeps its pool in registers)
static bool global_pool_for(const StatsGeometry &geo) { return wide_for(geo) && !multi_runs(geo); }
bool stats_uses_wide(const StatsGeometry &geo) { return wide_for(geo); }
// floats of pool scratch per frame: the pooled bins, or (SDRG_WIDE_DBPOOL, one bottom window) every reference window's
// dB values, window q at q * wst
static int pool_stride_for(const StatsGeometry &geo) {
    const int wst = (geo.max_pool + 3) & ~3;
    const int nb0 = (int)(geo.n_ref * 0.4f);
    const bool spec_pool = geo.n_ref >= 2 && (nb0 > 1 ? nb0 : 1) == 1;
    return (SDRG_WIDE_DBPOOL && spec_pool) ? geo.n_ref * wst : wst;
}

// The multi-frame wide kernel's plan (stats_wide_multi_kernel): ok when the pool is one bottom window (n_ref 2..4)
// or there is none (n_ref < 2), the pooled gaps fit the registers and the chains fit 16 lanes per frame; the
// chunk's bins per window 2^lg from the ring budget and the producer lanes; want_db: the dB sums and the pool.
struct MultiPlan {
    bool ok = false, want_db = false;
    int lg = 0;
};
static MultiPlan multi_for(const StatsGeometry &geo) {
    MultiPlan mp;
    const int nwin = geo.n_ref + 1;
    const int nb0 = (int)(geo.n_ref * 0.4f);
    const bool spec_pool = geo.n_ref >= 2 && (nb0 > 1 ? nb0 : 1) == 1;
    if (geo.focus_len <= 0 || geo.n_ref > 10 || (geo.n_ref >= 2 && !spec_pool) || geo.max_pool > MW_POOL) return mp;
    const int chains = 2 * nwin + (spec_pool ? nwin - 1 : 0);
    if (chains > WAVE / MW_F || WAVE / (MW_F * nwin) < 1) return mp;
    int pgf, pgr;
    mw_lanes(geo.n_ref, spec_pool, &pgf, &pgr);
    if (pgf < 1 || pgr < 1) return mp;
    const int pg = pgf < pgr ? pgf : pgr;
    for (int l = 6; l <= 10; l++)
        if (MW_F * nwin * 8 * ((1 << l) + 4) <= MW_RING_FLOATS && (1 << l) <= MW_PR * pg) mp.lg = l;
    mp.ok = mp.lg > 0;
    mp.want_db = spec_pool;
    return mp;
}
static bool multi_runs(const StatsGeometry &geo) {
    return wide_for(geo) && multi_for(geo).ok && !(SDRG_STATS_STAMPS || lab_getenv("SDRG_WIDE_SINGLE"));
}
// SDRG_MW_DBPOOL: the multi-frame kernel's dB scratch, n_ref windows of wst floats per frame (frames rounded up to whole
// workgroups: a workgroup's missing frames write and read their own slots)
static int mw_db_stride(const StatsGeometry &geo) { return (geo.max_pool + 3) & ~3; }
static bool mw_dbpool_for(const StatsGeometry &geo) {
    return SDRG_MW_DBPOOL && multi_runs(geo) && multi_for(geo).want_db && geo.n_ref >= 1;
}

size_t stats_global_pool_floats(const StatsGeometry &geo, int n_frames) {
    if (mw_dbpool_for(geo))
        return (size_t)((n_frames + MW_F - 1) / MW_F * MW_F) * (size_t)geo.n_ref * (size_t)mw_db_stride(geo);
    return global_pool_for(geo) ? (size_t)n_frames * (size_t)pool_stride_for(geo) : 0;
}

hipError_t launch_stats(const float *spectra, int n_frames, const StatsGeometry &geo, int64_t now_ms,
                        StatsState *state, sdrg_frame_record *records, float *gpool, hipStream_t stream) {
    if (n_frames <= 0) return hipSuccess;
    const bool global_pool = global_pool_for(geo);
    if (global_pool && !gpool) return hipErrorInvalidValue;
    if (geo.n_ref > 10) return hipErrorInvalidValue;
    const int pool_stride = pool_stride_for(geo);
    if (multi_runs(geo)) {
        const MultiPlan mp = multi_for(geo);
        // the rings; after the scan the same LDS holds each frame's 4096-bin first-digit histogram of the select
        const size_t lds = std::max(sizeof(float) * (size_t)MW_F * (size_t)(8 * (4 + (1 << mp.lg)) * (geo.n_ref + 1)),
                                    sizeof(int) * (size_t)MW_F * 4096);
        const void *k = mp.want_db ? reinterpret_cast<const void *>(stats_wide_multi_kernel<true>)
                                   : reinterpret_cast<const void *>(stats_wide_multi_kernel<false>);
        hipError_t e = ensure_dynamic_lds(k, (int)lds);
        if (e != hipSuccess) return e;
        const dim3 grid((n_frames + MW_F - 1) / MW_F);
        const bool dbp = mw_dbpool_for(geo);
        if (dbp && !gpool) return hipErrorInvalidValue;
        if (mp.want_db)
            hipLaunchKernelGGL(stats_wide_multi_kernel<true>, grid, dim3(MW_T), lds, stream, spectra, n_frames, geo, now_ms,
                               state, records, mp.lg, dbp ? gpool : nullptr, mw_db_stride(geo));
        else
            hipLaunchKernelGGL(stats_wide_multi_kernel<false>, grid, dim3(MW_T), lds, stream, spectra, n_frames, geo, now_ms,
                               state, records, mp.lg, nullptr, 0);
        if (SDRG_MW_STAMPS) {  // lab: mean cycles per phase over the workgroups of this call
            std::vector<unsigned long long> h((size_t)STAMP_PHASES * 8192);
            if (hipStreamSynchronize(stream) == hipSuccess &&
                hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(g_stats_stamps), h.size() * 8) == hipSuccess) {
                const int nw = std::min((int)grid.x, 8192);
                double d[10] = {};
                for (int b = 0; b < nw; b++) {
                    const unsigned long long *t = &h[(size_t)b * STAMP_PHASES];
                    for (int k = 0; k < 6; k++) d[k] += (double)(t[k + 1] - t[k]);
                    for (int k = 0; k < 4; k++) d[6 + k] += (double)t[7 + k];
                }
                fprintf(stderr, "[mw stamps] cycles/workgroup: scan %.0f (busy: chain %.0f, records %.0f, first producer %.0f, "
                                "last producer %.0f) | peak %.0f | tail %.0f | pool logs %.0f | select %.0f | end %.0f\n",
                        d[0] / nw, d[6] / nw, d[7] / nw, d[8] / nw, d[9] / nw, d[1] / nw, d[2] / nw, d[3] / nw, d[4] / nw,
                        d[5] / nw);
            }
        }
    } else if (wide_for(geo)) {
        size_t lds = sizeof(float) * (size_t)RING_FLOATS;
        if (SDRG_STATS_STAMPS && lab_getenv("SDRG_STATS_LDS_KB")) {  // diagnostic: fewer frames per CU
            lds = (size_t)atoi(lab_getenv("SDRG_STATS_LDS_KB")) * 1024;
            hipError_t e = ensure_dynamic_lds(reinterpret_cast<const void *>(stats_wide_kernel), (int)lds);
            if (e != hipSuccess) return e;
        }
        hipLaunchKernelGGL(stats_wide_kernel, dim3(n_frames), dim3(WIDE_WG), lds, stream, spectra, geo, now_ms, state,
                           records, gpool, pool_stride);
    } else {
        // the staged windows' bins, over which the pool is laid out in order (R > 0), or followed by a pool
        // region (R == 0: pools beyond 24 x 64 values); + a 16-value zero tail
        const int staged = (stage_bins(geo) + 3) & ~3, pool16 = (geo.max_pool + 15) & ~15;
        const int R = pool16 <= 8 * WAVE ? 8 : pool16 <= NARROW_REG_POOL * WAVE ? NARROW_REG_POOL : 0;
        const size_t lds = sizeof(float) * (size_t)(R > 0 ? std::max(staged, pool16) + 16 : staged + pool16 + 16);
        const void *k = R == 8 ? reinterpret_cast<const void *>(stats_narrow_kernel<8>)
                      : R > 0 ? reinterpret_cast<const void *>(stats_narrow_kernel<NARROW_REG_POOL>)
                              : reinterpret_cast<const void *>(stats_narrow_kernel<0>);
        hipError_t e = ensure_dynamic_lds(k, (int)lds);
        if (e != hipSuccess) return e;
        if (R == 8)
            hipLaunchKernelGGL(stats_narrow_kernel<8>, dim3(n_frames), dim3(WAVE), lds, stream, spectra, geo, now_ms,
                               state, records);
        else if (R > 0)
            hipLaunchKernelGGL(stats_narrow_kernel<NARROW_REG_POOL>, dim3(n_frames), dim3(WAVE), lds, stream, spectra,
                               geo, now_ms, state, records);
        else
            hipLaunchKernelGGL(stats_narrow_kernel<0>, dim3(n_frames), dim3(WAVE), lds, stream, spectra, geo, now_ms,
                               state, records);
    }
    if (SDRG_STATS_STAMPS) {  // diagnostic build: mean cycles per phase over the frames of this call
        std::vector<unsigned long long> h((size_t)STAMP_PHASES * 8192);
        if (hipStreamSynchronize(stream) == hipSuccess &&
            hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(g_stats_stamps), h.size() * 8) == hipSuccess) {
            const int nf = n_frames < 8192 ? n_frames : 8192;
            double d[8] = {0, 0, 0, 0, 0, 0, 0, 0};
            for (int f = 0; f < nf; f++) {
                const unsigned long long *t = &h[(size_t)f * STAMP_PHASES];
                for (int k = 0; k < 5; k++) d[k] += (double)(t[k + 1] - t[k]);
                d[5] += (double)t[6];
                d[6] += (double)t[7];
                d[7] += (double)t[8];
            }
            fprintf(stderr, "[stats stamps] cycles/frame: scans %.0f (wide busy: chain wave / record wave / producers; narrow: "
                            "staging copy first: %.0f %.0f %.0f) | "
                            "sort+6.4a %.0f | pool %.0f | select %.0f | tail %.0f\n", d[0] / nf, d[5] / nf, d[6] / nf,
                    d[7] / nf, d[1] / nf, d[2] / nf, d[3] / nf, d[4] / nf);
        }
    }
    return hipGetLastError();
}

}  // namespace sdrg

// fftany.hip — the spectrum (IQ unpack -> forward DFT -> |X|^2 -> fftshift) for ANY frame size the reference
// accepts: fftwf_plan_dft_1d(sampCount, ...) plans every N >= 1 (src/dsp/fft_process.cpp:77-79; SDRConfig only
// recommends multiples of 512, SDRBridge.kt:25-26).  The power-of-two sizes 64 .. 65536 keep their dedicated
// kernels (spectrum.hip); every other N runs here:
//
//   * N <= 16384 whose prime factors are all <= 13: one workgroup holds C whole frames in LDS and runs a
//     mixed-radix Stockham FFT (radices 16, 8, 4, 2, 3, 5, 7, 11, 13; register codelets, runtime pass plan).
//   * larger 13-smooth N = N1 x N2 (both <= 16384): two-kernel four-step through an HBM scratch, the column
//     kernel applying W_N^(n2 k1), frames in waves so the scratch stays small.
//   * any other N (a prime factor > 13): Bluestein's chirp-z, X_k = b*_k sum_n (x_n b*_n) b_(k-n),
//     b_m = exp(i pi m^2 / N), as two forward FFTs of a power-of-two M >= 2N - 1 with the chirp's transform
//     B^ (pre-scaled by 1/M) applied in between: |X_k|^2 = |FFT_M(conj(FFT_M(a) . B^))_k|^2 (|b_k| = 1).
//     M <= 16384 (N <= 8192) stays inside one workgroup; larger M uses the four-step kernels twice.
//     The chirp angle uses m^2 mod 2N in exact integer arithmetic, and B^ is computed on the host in double.
//
// The fftshift follows the reference's loop exactly (fft_process.cpp:92-97), including odd N: with half =
// floor(N/2), ps[i] = p[i + half] and ps[i + half] = p[i] for i < half, so p[N-1] is dropped and ps[N-1] is never
// written (the reference keeps whatever its vector held there; the engine leaves that element of the output
// buffer untouched).  Data layout and what bounds these kernels: DESIGN.md section 3.1a.
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <complex>
#include <mutex>
#include <vector>

#include "fftany.h"
#include "sdrg_internal.h"

namespace sdrg {
namespace {

#include "fft_codelets.h"

constexpr int TILE_MAX = 16384;   // complex values one workgroup holds in LDS (128 KiB)
constexpr int TILE_TARGET = 8192; // preferred tile (64 KiB: two workgroups per CU)
constexpr int TW_LO = 64;         // two-level twiddle tables in LDS: W_L^m = hi[m / 64] * lo[m % 64]

// ------------------------------------------------------------------------------------------------
// compile-time cos/sin (double Taylor series after reduction to [-pi/4, pi/4]) for the odd-radix codelets
// ------------------------------------------------------------------------------------------------
constexpr double kPi = 3.14159265358979323846264338327950288;
constexpr double ct_sin_small(double x) {  // |x| <= pi/4
    double term = x, sum = x;
    for (int k = 1; k < 14; k++) {
        term *= -x * x / ((2.0 * k) * (2.0 * k + 1.0));
        sum += term;
    }
    return sum;
}
constexpr double ct_cos_small(double x) {
    double term = 1.0, sum = 1.0;
    for (int k = 1; k < 14; k++) {
        term *= -x * x / ((2.0 * k - 1.0) * (2.0 * k));
        sum += term;
    }
    return sum;
}
// cos(2 pi a / R) for integer a: the angle is A + r with A = q pi/4 + pi/8 (q = its octant) and |r| <= pi/8;
// cos A and sin A come from the exact octant values and cos / sin(pi/8)
constexpr double ct_cos_frac(long a, long R) {
    a %= R;
    if (a < 0) a += R;
    const double t = (double)a / (double)R;  // turns in [0, 1)
    const int q = (int)(t * 8.0);
    const double r = (t - (q + 0.5) / 8.0) * 2.0 * kPi;
    const double h = 0.70710678118654752440084436210484903928;
    const double cb[8] = {1, h, 0, -h, -1, -h, 0, h}, sb[8] = {0, h, 1, h, 0, -h, -1, -h};
    const double cc = ct_cos_small(kPi / 8.0), sc = ct_sin_small(kPi / 8.0);
    const double cA = cb[q] * cc - sb[q] * sc, sA = sb[q] * cc + cb[q] * sc;
    return cA * ct_cos_small(r) - sA * ct_sin_small(r);
}
constexpr double ct_sin_frac(long a, long R) { return ct_cos_frac(a * 4 - R, 4 * R); }  // sin x = cos(x - pi/2)

// forward codelet constants of an odd radix R: C[a] = cos(2 pi a / R), S[a] = sin(2 pi a / R)
template <int R>
struct OddTw {
    float c[R], s[R];
    constexpr OddTw() : c(), s() {
        for (int a = 0; a < R; a++) {
            c[a] = (float)ct_cos_frac(a, R);
            s[a] = (float)ct_sin_frac(a, R);
        }
    }
};
template <int R>
struct OddTwHolder {
    static constexpr OddTw<R> v{};
};

// DFT of an odd prime radix: X_k = sum_n x_n W^(nk), W = exp(-2 pi i / R), with the symmetric pairs
// a_n = x_n + x_(R-n), d_n = x_n - x_(R-n): X_k = P_k + Q_k, X_(R-k) = P_k - Q_k,
// P_k = x_0 + sum a_n cos(2 pi n k / R), Q_k = -i sum d_n sin(2 pi n k / R).
template <int R>
__device__ __forceinline__ void dft_odd(f2 (&x)[R]) {
    constexpr int H = (R - 1) / 2;
    f2 a[H + 1], d[H + 1];
    f2 sum = x[0];
#pragma unroll
    for (int n = 1; n <= H; n++) {
        a[n] = x[n] + x[R - n];
        d[n] = x[n] - x[R - n];
        sum += a[n];
    }
    f2 out[R];
    out[0] = sum;
#pragma unroll
    for (int k = 1; k <= H; k++) {
        f2 P = x[0];
        float qr = 0.0f, qi = 0.0f;  // Q_k = -i sum d_n s  ->  (sum d.y s, -sum d.x s)
#pragma unroll
        for (int n = 1; n <= H; n++) {
            const int m = (n * k) % R;
            const float c = OddTwHolder<R>::v.c[m], s = OddTwHolder<R>::v.s[m];
            P += a[n] * f2{c, c};
            qr += d[n].y * s;
            qi -= d[n].x * s;
        }
        out[k] = P + f2{qr, qi};
        out[R - k] = P - f2{qr, qi};
    }
#pragma unroll
    for (int k = 0; k < R; k++) x[k] = out[k];
}

template <int R>
__device__ __forceinline__ void dft_any(f2 (&x)[R]) {
    if constexpr ((R & (R - 1)) == 0) {
        dft<R>(x);
    } else {
        dft_odd<R>(x);
    }
}

__device__ __forceinline__ f2 cmul(f2 a, f2 b) { return f2{a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x}; }
__device__ __forceinline__ f2 conj2(f2 a) { return f2{a.x, -a.y}; }

template <int FMT>
__device__ __forceinline__ f2 load_sample_any(const void *frame, int64_t e) {
    if constexpr (FMT == SDRG_IQ_CS8) {
        const uint16_t v = reinterpret_cast<const uint16_t *>(frame)[e];
        return f2{(float)(int8_t)(v & 0xff), (float)(int8_t)(v >> 8)} * (1.0f / 128.0f);
    } else if constexpr (FMT == SDRG_IQ_CU8) {
        const uint16_t v = reinterpret_cast<const uint16_t *>(frame)[e];
        return (f2{(float)(v & 0xff), (float)(v >> 8)} - 127.4f) * (1.0f / 128.0f);
    } else if constexpr (FMT == SDRG_IQ_CS16) {
        const uint32_t v = reinterpret_cast<const uint32_t *>(frame)[e];
        return f2{(float)(int16_t)(v & 0xffff), (float)(int16_t)(v >> 16)} * (1.0f / 32768.0f);
    } else {
        return reinterpret_cast<const f2 *>(frame)[e];
    }
}
template <int FMT>
constexpr int bps_any() {
    return FMT == SDRG_IQ_CF32 ? 8 : FMT == SDRG_IQ_CS16 ? 4 : 2;
}
constexpr int FMT_CPLX = 100;  // input is a complex float scratch (four-step row kernels, Bluestein pass 2)

// ------------------------------------------------------------------------------------------------
// One Stockham pass of radix R over C sequences of length L held in LDS (sequence c at lds + c * L):
// butterfly j of a sequence: x[r] = A[j + r L/R] * w^(r k), k = j mod NS, w = exp(-2 pi i / (NS R));
// X = DFT_R(x); B[(j / NS) NS R + k + r NS] = X[r].  In place: every thread reads its butterflies into
// registers, then a barrier, then the writes.  A thread holds at most ceil(16 / R) butterflies (tile sizes
// keep C L <= 16 T).
// ------------------------------------------------------------------------------------------------
template <int R>
__device__ __forceinline__ void tile_pass(f2 *lds, int C, int L, int NS, const f2 *thi, const f2 *tlo) {
    constexpr int NBM = (16 + R - 1) / R;
    const int T = blockDim.x;
    const int LR = L / R;
    const int total = C * LR;
    const int stw = L / (NS * R);
    f2 x[NBM][R];
    int cc[NBM], jj[NBM];
#pragma unroll
    for (int b = 0; b < NBM; b++) {
        const int bf = threadIdx.x + b * T;
        cc[b] = -1;
        if (bf < total) {
            const int c = bf / LR, j = bf - c * LR;
            cc[b] = c;
            jj[b] = j;
            const f2 *src = lds + (size_t)c * L + j;
#pragma unroll
            for (int r = 0; r < R; r++) x[b][r] = src[r * LR];
        }
    }
    __syncthreads();
#pragma unroll
    for (int b = 0; b < NBM; b++) {
        if (cc[b] < 0) continue;
        const int j = jj[b];
        const int blk = j / NS, k = j - blk * NS;
        if (NS > 1) {
#pragma unroll
            for (int r = 1; r < R; r++) {
                const int m = stw * r * k;  // < L
                x[b][r] = cmul(x[b][r], cmul(thi[m / TW_LO], tlo[m % TW_LO]));
            }
        }
        dft_any<R>(x[b]);
        f2 *dst = lds + (size_t)cc[b] * L + blk * NS * R + k;
#pragma unroll
        for (int r = 0; r < R; r++) dst[r * NS] = x[b][r];
    }
    __syncthreads();
}

__device__ void tile_fft(f2 *lds, int C, const FftPassPlan &p, const f2 *thi, const f2 *tlo) {
    for (int q = 0; q < p.n_pass; q++) {
        const int R = p.radix[q], NS = p.ns[q];
        switch (R) {
        case 2: tile_pass<2>(lds, C, p.L, NS, thi, tlo); break;
        case 3: tile_pass<3>(lds, C, p.L, NS, thi, tlo); break;
        case 4: tile_pass<4>(lds, C, p.L, NS, thi, tlo); break;
        case 5: tile_pass<5>(lds, C, p.L, NS, thi, tlo); break;
        case 7: tile_pass<7>(lds, C, p.L, NS, thi, tlo); break;
        case 8: tile_pass<8>(lds, C, p.L, NS, thi, tlo); break;
        case 11: tile_pass<11>(lds, C, p.L, NS, thi, tlo); break;
        case 13: tile_pass<13>(lds, C, p.L, NS, thi, tlo); break;
        case 16: tile_pass<16>(lds, C, p.L, NS, thi, tlo); break;
        default: break;  // the host plans only these radices
        }
    }
}

// copy the sequence length's two-level twiddle tables into LDS (after the data area)
__device__ __forceinline__ void load_tw(f2 *thi, f2 *tlo, const f2 *g_hi, const f2 *g_lo, int n_hi) {
    for (int i = threadIdx.x; i < n_hi; i += blockDim.x) thi[i] = g_hi[i];
    for (int i = threadIdx.x; i < TW_LO; i += blockDim.x) tlo[i] = g_lo[i];
}

// the reference's fftshift (fft_process.cpp:92-97): bin k of the FFT -> index in power_shifted, or -1 for the
// element the loop drops (k = N - 1 when N is odd)
__device__ __forceinline__ int shift_index(int k, int N) {
    const int half = N >> 1;
    if (k < half) return k + half;
    if (k < 2 * half) return k - half;
    return -1;
}

// ------------------------------------------------------------------------------------------------
// Single-level kernel: C frames per workgroup, the whole L-point transform in LDS.
// BLUE: Bluestein with L = M: a_n = x_n conj(b_n) (n < N, 0 above), FFT, * B^ (1/M folded in), conj, FFT,
// |.|^2 of the first N bins.  Otherwise L = N.
// ------------------------------------------------------------------------------------------------
template <int FMT, bool BLUE>
__global__ __launch_bounds__(1024) void fft1_kernel(const void *__restrict__ iq, float *__restrict__ spectra, int n_frames,
                                                    int N, int C, FftPassPlan plan, const f2 *__restrict__ g_hi,
                                                    const f2 *__restrict__ g_lo, int n_hi,
                                                    const f2 *__restrict__ chirp, const f2 *__restrict__ bhat) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int L = plan.L;
    f2 *lds = reinterpret_cast<f2 *>(smem);
    f2 *thi = lds + (size_t)C * L;
    f2 *tlo = thi + n_hi;
    load_tw(thi, tlo, g_hi, g_lo, n_hi);
    const int f0 = blockIdx.x * C;
    const int nc = min(C, n_frames - f0);
    constexpr int BPS = bps_any<FMT>();
    const char *src = reinterpret_cast<const char *>(iq) + (size_t)f0 * N * BPS;
    for (int e = threadIdx.x; e < C * L; e += blockDim.x) {
        const int c = e / L, n = e - c * L;
        f2 v = f2{0.0f, 0.0f};
        if (c < nc && n < N) {
            v = load_sample_any<FMT>(src + (size_t)c * N * BPS, n);
            if constexpr (BLUE) v = cmul(v, conj2(chirp[n]));
        }
        lds[e] = v;
    }
    __syncthreads();
    tile_fft(lds, C, plan, thi, tlo);
    if constexpr (BLUE) {
        for (int e = threadIdx.x; e < C * L; e += blockDim.x) {
            const int n = e - (e / L) * L;
            lds[e] = conj2(cmul(lds[e], bhat[n]));
        }
        __syncthreads();
        tile_fft(lds, C, plan, thi, tlo);
    }
    float *out = spectra + (size_t)f0 * N;
    for (int e = threadIdx.x; e < C * N; e += blockDim.x) {
        const int c = e / N, k = e - c * N;
        if (c >= nc) break;
        const int o = shift_index(k, N);
        if (o < 0) continue;
        const f2 v = lds[(size_t)c * L + k];
        out[(size_t)c * N + o] = v.x * v.x + v.y * v.y;
    }
}

// ------------------------------------------------------------------------------------------------
// Four-step kernels for an M-point transform, M = N1 N2, n = N2 n1 + n2, k = k1 + N1 k2.
//   A (columns): C columns n2 per workgroup; Y[k1 N2 + n2] = W_M^(n2 k1) DFT_N1 over n1 of in[N2 n1 + n2].
//     Input: raw frame samples (FMT) with, for Bluestein, a_n = x_n conj(b_n) for n < Nin and 0 above;
//     or a complex scratch (FMT_CPLX).
//   B (rows): C rows k1 per workgroup; X[k1 + N1 k2] = DFT_N2 over n2 of Y[k1 N2 + n2].  Output: |X_k|^2 at the
//     fftshifted index of the first Nout bins (POWER), or Z_k = conj(X_k B^_k) into a complex scratch (BLUE_MID).
// Frames: blockIdx.y (a wave of frames; in/out pointers are the wave's first frame).
// ------------------------------------------------------------------------------------------------
template <int FMT, bool BLUE>
__global__ __launch_bounds__(1024) void fft4a_kernel(const void *__restrict__ in, f2 *__restrict__ Y, int Nin, int N1,
                                                     int N2, int C, FftPassPlan plan, const f2 *__restrict__ g_hi,
                                                     const f2 *__restrict__ g_lo, int n_hi, const f2 *__restrict__ m_hi,
                                                     const f2 *__restrict__ m_lo, const f2 *__restrict__ chirp) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    f2 *lds = reinterpret_cast<f2 *>(smem);
    f2 *thi = lds + (size_t)C * N1;
    f2 *tlo = thi + n_hi;
    load_tw(thi, tlo, g_hi, g_lo, n_hi);
    const int M = N1 * N2;
    const int c0 = blockIdx.x * C;
    const int nc = min(C, N2 - c0);
    const size_t frame = blockIdx.y;
    // load: consecutive threads take consecutive columns of one row (coalesced runs of C samples)
    for (int e = threadIdx.x; e < C * N1; e += blockDim.x) {
        const int n1 = e / C, c = e - n1 * C;
        f2 v = f2{0.0f, 0.0f};
        if (c < nc) {
            const int n = N2 * n1 + c0 + c;
            if constexpr (FMT == FMT_CPLX) {
                v = reinterpret_cast<const f2 *>(in)[frame * (size_t)M + n];
            } else {
                if (n < Nin) {
                    v = load_sample_any<FMT>(reinterpret_cast<const char *>(in) + frame * (size_t)Nin * bps_any<FMT>(), n);
                    if constexpr (BLUE) v = cmul(v, conj2(chirp[n]));
                }
            }
        }
        lds[(size_t)c * N1 + n1] = v;
    }
    __syncthreads();
    tile_fft(lds, C, plan, thi, tlo);
    f2 *y = Y + frame * (size_t)M;
    for (int e = threadIdx.x; e < C * N1; e += blockDim.x) {
        const int k1 = e / C, c = e - k1 * C;
        if (c >= nc) continue;
        const int n2 = c0 + c;
        const int m = n2 * k1;  // < M <= 2^21
        const f2 w = cmul(m_hi[m >> 10], m_lo[m & 1023]);
        y[(size_t)k1 * N2 + n2] = cmul(lds[(size_t)c * N1 + k1], w);
    }
}

template <bool BLUE_MID>
__global__ __launch_bounds__(1024) void fft4b_kernel(const f2 *__restrict__ Y, void *__restrict__ out, int Nout, int N1,
                                                     int N2, int C, FftPassPlan plan, const f2 *__restrict__ g_hi,
                                                     const f2 *__restrict__ g_lo, int n_hi, const f2 *__restrict__ bhat) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    f2 *lds = reinterpret_cast<f2 *>(smem);
    f2 *thi = lds + (size_t)C * N2;
    f2 *tlo = thi + n_hi;
    load_tw(thi, tlo, g_hi, g_lo, n_hi);
    const int M = N1 * N2;
    const int r0 = blockIdx.x * C;
    const int nr = min(C, N1 - r0);
    const size_t frame = blockIdx.y;
    const f2 *y = Y + frame * (size_t)M + (size_t)r0 * N2;
    for (int e = threadIdx.x; e < C * N2; e += blockDim.x) lds[e] = (e < nr * N2) ? y[e] : f2{0.0f, 0.0f};
    __syncthreads();
    tile_fft(lds, C, plan, thi, tlo);
    // store: consecutive threads take consecutive rows k1 of one k2 (runs of C consecutive outputs k)
    for (int e = threadIdx.x; e < C * N2; e += blockDim.x) {
        const int k2 = e / C, c = e - k2 * C;
        if (c >= nr) continue;
        const int k = r0 + c + N1 * k2;
        const f2 v = lds[(size_t)c * N2 + k2];
        if constexpr (BLUE_MID) {
            reinterpret_cast<f2 *>(out)[frame * (size_t)M + k] = conj2(cmul(v, bhat[k]));
        } else {
            if (k >= Nout) continue;
            const int o = shift_index(k, Nout);
            if (o >= 0) reinterpret_cast<float *>(out)[frame * (size_t)Nout + o] = v.x * v.x + v.y * v.y;
        }
    }
}

// ------------------------------------------------------------------------------------------------
// Host planning
// ------------------------------------------------------------------------------------------------
bool smooth13(int64_t n) {
    for (int p : {2, 3, 5, 7, 11, 13})
        while (n % p == 0) n /= p;
    return n == 1;
}

FftPassPlan pass_plan(int L) {
    FftPassPlan p{};
    p.L = L;
    int rest = L, ns = 1;
    auto add = [&](int r) {
        p.radix[p.n_pass] = r;
        p.ns[p.n_pass] = ns;
        p.n_pass++;
        ns *= r;
        rest /= r;
    };
    while (rest % 16 == 0) add(16);
    if (rest % 8 == 0) add(8);
    if (rest % 4 == 0) add(4);
    if (rest % 2 == 0) add(2);
    for (int r : {3, 5, 7, 11, 13})
        while (rest % r == 0) add(r);
    return p;
}

int threads_for(int elems) {
    int t = (elems + 15) / 16;
    t = (t + 63) / 64 * 64;
    return std::min(1024, std::max(64, t));
}

// W_L^m tables: hi[a] = W_L^(64 a), a < ceil(L/64); lo[b] = W_L^b, b < 64 (double, rounded once)
void fill_two_level(int L, int step, std::vector<std::complex<float>> &hi, std::vector<std::complex<float>> &lo) {
    const int nh = (L + step - 1) / step;
    hi.resize(nh);
    lo.resize(step);
    for (int a = 0; a < nh; a++) {
        const double t = -2.0 * M_PI * (double)((int64_t)a * step % L) / L;
        hi[a] = {(float)cos(t), (float)sin(t)};
    }
    for (int b = 0; b < step; b++) {
        const double t = -2.0 * M_PI * (double)(b % L) / L;
        lo[b] = {(float)cos(t), (float)sin(t)};
    }
}

// in-place iterative radix-2 DFT in double (host, power-of-two m): for B^ = FFT_M(b~)
void fft_double(std::vector<std::complex<double>> &a) {
    const size_t n = a.size();
    for (size_t i = 1, j = 0; i < n; i++) {
        size_t bit = n >> 1;
        for (; j & bit; bit >>= 1) j ^= bit;
        j ^= bit;
        if (i < j) std::swap(a[i], a[j]);
    }
    std::vector<std::complex<double>> w(n / 2);  // W_n^k, each computed directly in double
    for (size_t k = 0; k < n / 2; k++) {
        const double ang = -2.0 * M_PI * (double)k / (double)n;
        w[k] = {cos(ang), sin(ang)};
    }
    for (size_t len = 2; len <= n; len <<= 1) {
        const size_t step = n / len;
        for (size_t i = 0; i < n; i += len)
            for (size_t k = 0; k < len / 2; k++) {
                const std::complex<double> u = a[i + k], v = a[i + k + len / 2] * w[k * step];
                a[i + k] = u + v;
                a[i + k + len / 2] = u - v;
            }
    }
}

}  // namespace

AnyPlan any_plan(int n) {
    AnyPlan P{};
    P.n = n;
    if (smooth13(n) && n <= TILE_MAX) {
        P.mode = AnyPlan::ONE;
        P.m = n;
        return P;
    }
    if (smooth13(n)) {
        // N = N1 N2 with N1 <= N2 <= TILE_MAX, N1 the largest divisor <= sqrt(N)
        int best = 0;
        for (int d = 1; (int64_t)d * d <= n; d++)
            if (n % d == 0 && n / d <= TILE_MAX) best = d;
        if (best > 0) {
            P.mode = AnyPlan::FOUR;
            P.m = n;
            P.n1 = best;
            P.n2 = n / best;
            return P;
        }
    }
    // Bluestein over the power of two M >= 2N - 1
    int64_t m = 1;
    while (m < 2 * (int64_t)n - 1) m <<= 1;
    P.m = (int)m;
    if (m <= TILE_MAX) {
        P.mode = AnyPlan::BLUE_ONE;
    } else {
        P.mode = AnyPlan::BLUE_FOUR;
        int lg = 0;
        while ((1LL << lg) < m) lg++;
        P.n1 = 1 << (lg / 2);
        P.n2 = (int)(m / P.n1);
    }
    return P;
}

// Table layout (complex floats, in this order): for each sequence length the kernels use (L1 = m or n1, then
// L2 = n2 for the four-step modes) hi[ceil(L/64)] + lo[64]; four-step modes: W_M hi[ceil(M/1024)] + lo[1024];
// Bluestein: chirp b_n (n < N) then B^_k / M (k < M).
size_t any_table_floats(const AnyPlan &P) {
    auto tl = [](int L) { return (size_t)((L + TW_LO - 1) / TW_LO + TW_LO); };
    size_t c = 0;
    const bool four = P.mode == AnyPlan::FOUR || P.mode == AnyPlan::BLUE_FOUR;
    c += tl(four ? P.n1 : P.m);
    if (four) c += tl(P.n2) + (size_t)((P.m + 1023) / 1024 + 1024);
    if (P.mode == AnyPlan::BLUE_ONE || P.mode == AnyPlan::BLUE_FOUR) c += (size_t)P.n + (size_t)P.m;
    return 2 * c;
}

void any_fill_tables(const AnyPlan &P, float *out) {
    std::vector<std::complex<float>> all, hi, lo;
    const bool four = P.mode == AnyPlan::FOUR || P.mode == AnyPlan::BLUE_FOUR;
    auto put = [&](int L, int step) {
        fill_two_level(L, step, hi, lo);
        all.insert(all.end(), hi.begin(), hi.end());
        all.insert(all.end(), lo.begin(), lo.end());
    };
    put(four ? P.n1 : P.m, TW_LO);
    if (four) {
        put(P.n2, TW_LO);
        put(P.m, 1024);
    }
    if (P.mode == AnyPlan::BLUE_ONE || P.mode == AnyPlan::BLUE_FOUR) {
        const int64_t N = P.n, M = P.m;
        std::vector<std::complex<double>> b(N), bt(M, 0.0);
        for (int64_t k = 0; k < N; k++) {
            const int64_t q = (k * k) % (2 * N);  // exact: b_k = exp(i pi k^2 / N) has period 2N in k^2
            const double t = M_PI * (double)q / (double)N;
            b[k] = {cos(t), sin(t)};
        }
        for (int64_t k = 0; k < N; k++) all.push_back({(float)b[k].real(), (float)b[k].imag()});
        bt[0] = b[0];
        for (int64_t k = 1; k < N; k++) bt[k] = bt[M - k] = b[k];
        fft_double(bt);
        for (int64_t k = 0; k < M; k++) all.push_back({(float)(bt[k].real() / M), (float)(bt[k].imag() / M)});
    }
    memcpy(out, all.data(), all.size() * sizeof(std::complex<float>));
}

size_t any_scratch_floats(const AnyPlan &P, int n_frames) {
    if (P.mode == AnyPlan::ONE || P.mode == AnyPlan::BLUE_ONE) return 0;
    const int wave = any_wave_frames(P, n_frames);
    const size_t per = (size_t)P.m * 2;  // one complex M-point intermediate
    return (size_t)wave * per * (P.mode == AnyPlan::BLUE_FOUR ? 2 : 1);
}

int any_wave_frames(const AnyPlan &P, int n_frames) {
    // frames in flight per four-step wave: the intermediate(s) of a wave ~128 MiB (inside the Infinity Cache)
    const size_t per = (size_t)P.m * 8 * (P.mode == AnyPlan::BLUE_FOUR ? 2 : 1);
    const int w = (int)std::max<size_t>(1, ((size_t)128 << 20) / per);
    return std::min(w, std::max(1, n_frames));
}

namespace {

template <class K>
hipError_t lds_launch_attr(K k, size_t bytes) {
    return ensure_dynamic_lds(reinterpret_cast<const void *>(k), (int)bytes);
}

size_t tile_lds(int C, int L) { return ((size_t)C * L + (size_t)(L + TW_LO - 1) / TW_LO + TW_LO) * sizeof(f2); }

template <int FMT>
hipError_t launch_any_fmt(const AnyPlan &P, const void *iq, int n_frames, const float *tables, float *spectra,
                          float *scratch, hipStream_t s) {
    const f2 *t = reinterpret_cast<const f2 *>(tables);
    const bool four = P.mode == AnyPlan::FOUR || P.mode == AnyPlan::BLUE_FOUR;
    const int L1 = four ? P.n1 : P.m;
    const int nh1 = (L1 + TW_LO - 1) / TW_LO;
    const f2 *hi1 = t, *lo1 = hi1 + nh1;
    const f2 *p = lo1 + TW_LO;
    const f2 *hi2 = nullptr, *lo2 = nullptr, *mhi = nullptr, *mlo = nullptr, *chirp = nullptr, *bhat = nullptr;
    int nh2 = 0;
    if (four) {
        nh2 = (P.n2 + TW_LO - 1) / TW_LO;
        hi2 = p;
        lo2 = hi2 + nh2;
        p = lo2 + TW_LO;
        mhi = p;
        mlo = mhi + (P.m + 1023) / 1024;
        p = mlo + 1024;
    }
    if (P.mode == AnyPlan::BLUE_ONE || P.mode == AnyPlan::BLUE_FOUR) {
        chirp = p;
        bhat = chirp + P.n;
    }
    hipError_t e;
    if (!four) {
        const FftPassPlan pl = pass_plan(P.m);
        const int C = std::max(1, std::min(n_frames, TILE_TARGET / P.m));
        const int T = threads_for(C * P.m);
        const size_t lds = tile_lds(C, P.m);
        const int grid = (n_frames + C - 1) / C;
        if (P.mode == AnyPlan::ONE) {
            auto k = fft1_kernel<FMT, false>;
            if ((e = lds_launch_attr(k, lds)) != hipSuccess) return e;
            hipLaunchKernelGGL(k, dim3(grid), dim3(T), lds, s, iq, spectra, n_frames, P.n, C, pl, hi1, lo1, nh1,
                               chirp, bhat);
        } else {
            auto k = fft1_kernel<FMT, true>;
            if ((e = lds_launch_attr(k, lds)) != hipSuccess) return e;
            hipLaunchKernelGGL(k, dim3(grid), dim3(T), lds, s, iq, spectra, n_frames, P.n, C, pl, hi1, lo1, nh1,
                               chirp, bhat);
        }
        return hipGetLastError();
    }
    const FftPassPlan pa = pass_plan(P.n1), pb = pass_plan(P.n2);
    const int CA = std::max(1, std::min(P.n2, TILE_TARGET / P.n1));
    const int CB = std::max(1, std::min(P.n1, TILE_TARGET / P.n2));
    const int TA = threads_for(CA * P.n1), TB = threads_for(CB * P.n2);
    const size_t ldsA = tile_lds(CA, P.n1), ldsB = tile_lds(CB, P.n2);
    const int gA = (P.n2 + CA - 1) / CA, gB = (P.n1 + CB - 1) / CB;
    const int wave = any_wave_frames(P, n_frames);
    f2 *Y = reinterpret_cast<f2 *>(scratch);
    f2 *Z = Y + (size_t)wave * P.m;
    constexpr int BPS = bps_any<FMT>();
    if (P.mode == AnyPlan::FOUR) {
        auto ka = fft4a_kernel<FMT, false>;
        auto kb = fft4b_kernel<false>;
        if ((e = lds_launch_attr(ka, ldsA)) != hipSuccess || (e = lds_launch_attr(kb, ldsB)) != hipSuccess) return e;
        for (int f0 = 0; f0 < n_frames; f0 += wave) {
            const int nf = std::min(wave, n_frames - f0);
            const char *src = reinterpret_cast<const char *>(iq) + (size_t)f0 * P.n * BPS;
            hipLaunchKernelGGL(ka, dim3(gA, nf), dim3(TA), ldsA, s, src, Y, P.n, P.n1, P.n2, CA, pa, hi1, lo1, nh1, mhi,
                               mlo, chirp);
            hipLaunchKernelGGL(kb, dim3(gB, nf), dim3(TB), ldsB, s, Y, (void *)(spectra + (size_t)f0 * P.n), P.n, P.n1,
                               P.n2, CB, pb, hi2, lo2, nh2, bhat);
        }
        return hipGetLastError();
    }
    // Bluestein through two four-step transforms of M points
    auto ka1 = fft4a_kernel<FMT, true>;
    auto ka2 = fft4a_kernel<FMT_CPLX, false>;
    auto kb1 = fft4b_kernel<true>;
    auto kb2 = fft4b_kernel<false>;
    if ((e = lds_launch_attr(ka1, ldsA)) != hipSuccess || (e = lds_launch_attr(ka2, ldsA)) != hipSuccess ||
        (e = lds_launch_attr(kb1, ldsB)) != hipSuccess || (e = lds_launch_attr(kb2, ldsB)) != hipSuccess)
        return e;
    for (int f0 = 0; f0 < n_frames; f0 += wave) {
        const int nf = std::min(wave, n_frames - f0);
        const char *src = reinterpret_cast<const char *>(iq) + (size_t)f0 * P.n * BPS;
        hipLaunchKernelGGL(ka1, dim3(gA, nf), dim3(TA), ldsA, s, src, Y, P.n, P.n1, P.n2, CA, pa, hi1, lo1, nh1, mhi, mlo,
                           chirp);
        hipLaunchKernelGGL(kb1, dim3(gB, nf), dim3(TB), ldsB, s, Y, (void *)Z, P.m, P.n1, P.n2, CB, pb, hi2, lo2, nh2, bhat);
        hipLaunchKernelGGL(ka2, dim3(gA, nf), dim3(TA), ldsA, s, (const void *)Z, Y, P.m, P.n1, P.n2, CA, pa, hi1, lo1,
                           nh1, mhi, mlo, chirp);
        hipLaunchKernelGGL(kb2, dim3(gB, nf), dim3(TB), ldsB, s, Y, (void *)(spectra + (size_t)f0 * P.n), P.n, P.n1,
                           P.n2, CB, pb, hi2, lo2, nh2, bhat);
    }
    return hipGetLastError();
}

}  // namespace

hipError_t launch_spectrum_any(const AnyPlan &P, const void *iq, int fmt, int n_frames, const float *tables,
                               float *spectra, float *scratch, hipStream_t s) {
    if (n_frames <= 0) return hipSuccess;
    switch (fmt) {
    case SDRG_IQ_CS8: return launch_any_fmt<SDRG_IQ_CS8>(P, iq, n_frames, tables, spectra, scratch, s);
    case SDRG_IQ_CU8: return launch_any_fmt<SDRG_IQ_CU8>(P, iq, n_frames, tables, spectra, scratch, s);
    case SDRG_IQ_CS16: return launch_any_fmt<SDRG_IQ_CS16>(P, iq, n_frames, tables, spectra, scratch, s);
    case SDRG_IQ_CF32: return launch_any_fmt<SDRG_IQ_CF32>(P, iq, n_frames, tables, spectra, scratch, s);
    default: return hipErrorInvalidValue;
    }
}

}  // namespace sdrg

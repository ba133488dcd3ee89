// spectrum.hip — fused IQ unpack -> N-point forward FFT -> |X|^2 -> fftshift, one frame per workgroup.
//
// Replaces FFTProcessor::process steps 1-4 (src/dsp/fft_process.cpp:42-97): copy into the FFTW buffer,
// fftwf_plan_dft_1d(N, FORWARD, ESTIMATE) + execute (unnormalised, no window), power = re^2 + im^2,
// fftshift.  The unused 10-frame ring buffer (:62-73) has no observable output and is not kept.
//
// Design (gfx950): Stockham autosort FFT with radix-32 register butterflies (N = 16384: 3 passes =
// 32 * 32 * 16, two exchanges).  Each thread owns E = 32 complex values (T = N/32 threads, 512 at
// N = 16384).  Between passes the values move through an LDS buffer of HALF the frame (66 KiB) in two
// phases, so two frames' workgroups fit a CU beside the SSB pipeline's workgroup.  Pass 0 reads the raw
// int8/uint8/int16/float samples straight from HBM (coalesced across lanes) and converts them in
// registers; the last pass writes |X|^2 straight to HBM at the fftshifted index (coalesced).  Twiddles
// come from two small factored tables (L1-resident).  Complex arithmetic is written on
// 2-wide float vectors so it maps onto v_pk_{add,mul,fma}_f32.  HBM traffic = bytes in + 4 B out per
// sample (6 B/sample for CS8), the algorithmic minimum.
#include <math.h>
#include <string.h>

#include <type_traits>
#include <vector>

#include "sdrg_internal.h"

namespace sdrg {
namespace {

typedef float f2 __attribute__((ext_vector_type(2)));

constexpr int E = 32;  // complex values per thread

// exp(-2 pi i k / 32), k in [0, 16)
__device__ constexpr float W32_RE[16] = {1.0f, 0.980785251f, 0.923879504f, 0.831469595f, 0.707106769f,
                                         0.555570245f, 0.382683426f, 0.195090324f, 0.0f, -0.195090324f,
                                         -0.382683426f, -0.555570245f, -0.707106769f, -0.831469595f,
                                         -0.923879504f, -0.980785251f};
__device__ constexpr float W32_IM[16] = {-0.0f, -0.195090324f, -0.382683426f, -0.555570245f, -0.707106769f,
                                         -0.831469595f, -0.923879504f, -0.980785251f, -1.0f, -0.980785251f,
                                         -0.923879504f, -0.831469595f, -0.707106769f, -0.555570245f,
                                         -0.382683426f, -0.195090324f};

__device__ __forceinline__ f2 cmul(f2 a, f2 w) {
    // (a.x w.x - a.y w.y, a.x w.y + a.y w.x)
    f2 r = a.xx * w;
    f2 wr = {-w.y, w.x};
    return r + a.yy * wr;
}

// multiply by W32^t (t compile-time after unrolling)
__device__ __forceinline__ f2 twiddle32(f2 a, int t) {
    if (t == 0) return a;
    if (t == 8) return f2{a.y, -a.x};  // * (-i)
    return cmul(a, f2{W32_RE[t], W32_IM[t]});
}

template <int R>
__device__ __forceinline__ constexpr int bitrev(int i) {
    int r = 0;
    for (int b = 1; b < R; b <<= 1) {
        r = (r << 1) | (i & 1);
        i >>= 1;
    }
    return r;
}

// In-register DFT of R points (R | 32), natural order in and out (radix-2 DIT).
template <int R>
__device__ __forceinline__ void dft(f2 (&v)[R]) {
#pragma unroll
    for (int i = 0; i < R; ++i) {
        const int j = bitrev<R>(i);
        if (j > i) {
            f2 t = v[i];
            v[i] = v[j];
            v[j] = t;
        }
    }
#pragma unroll
    for (int len = 2; len <= R; len <<= 1) {
#pragma unroll
        for (int base = 0; base < R; base += len) {
#pragma unroll
            for (int k = 0; k < len / 2; ++k) {
                const f2 b = twiddle32(v[base + k + len / 2], k * (32 / len));
                const f2 a = v[base + k];
                v[base + k] = a + b;
                v[base + k + len / 2] = a - b;
            }
        }
    }
}

__device__ __forceinline__ int lds_idx(int e) { return e + (e >> 5); }  // one pad slot per 32 values

template <int FMT>
__device__ __forceinline__ f2 load_sample(const void *frame, int e) {
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
constexpr int bytes_per_sample() {
    return FMT == SDRG_IQ_CF32 ? 8 : FMT == SDRG_IQ_CS16 ? 4 : 2;
}

template <int LOG2N>
struct Plan {
    static constexpr int N = 1 << LOG2N;
    static constexpr int T = N / E;
    static constexpr int NP = (LOG2N + 4) / 5;  // passes: radix 32 ..., last = remainder
    static constexpr int RLAST = (LOG2N % 5 == 0) ? 32 : (1 << (LOG2N % 5));
    static constexpr int HALF = N / 2;
    static constexpr int LDS_BYTES = (HALF + HALF / 32) * 8;  // half the frame + pad (66 KiB at 16384)
    template <int P>
    static constexpr int radix() { return P == NP - 1 ? RLAST : 32; }
    static constexpr int radix_of(int p) { return p == NP - 1 ? RLAST : 32; }
    static constexpr int ns_of(int p) {
        int s = 1;
        for (int i = 0; i < p; i++) s *= radix_of(i);
        return s;
    }
    // per-pass twiddle table of pass p >= 1: [R/2 pairs][NS] of float4 (w^(r k), w^((r+1) k)), r = 2q+1,
    // w = exp(-2 pi i / (NS R)); offset in float4 units from the start of the pass tables
    static constexpr int tw_off(int p) {
        int o = 0;
        for (int i = 1; i < p; i++) o += (radix_of(i) / 2) * ns_of(i);
        return o;
    }
    template <int P>
    static constexpr int ns() { return ns_of(P); }
    template <int P>
    static constexpr int tw_offset() { return tw_off(P); }
    static constexpr int TW_F4 = tw_off(NP);
};

// Butterfly handled as block b by this thread.  The last pass pairs consecutive butterflies (j = 2t + b)
// when a thread holds two, so its |X|^2 stores are 8 bytes wide; every other pass uses j = t + b T.
template <int LOG2N, int R, bool LAST = false>
__device__ __forceinline__ int bfly_j(int b) {
    constexpr int N = 1 << LOG2N, T = N / E, NB = E / R;
    if constexpr (LAST && NB == 2) return 2 * (int)threadIdx.x + b;
    return (int)threadIdx.x + b * T;
}

template <int LOG2N, int R>
__device__ __forceinline__ int last_j(int b) { return bfly_j<LOG2N, R, true>(b); }

// Stockham pass P (radix R, NS = product of the previous radices) on the E values a thread holds as
// v[b*R + r] for butterflies j = t + b*T:
//   x[r] = A[j + r N/R] * w^(r k), k = j mod NS, w = exp(-2 pi i/(NS R));  X = DFT_R(x);
//   B[(j/NS) NS R + k + r NS] = X[r]
template <int LOG2N, int R, int NS, bool LAST>
__device__ __forceinline__ void pass_compute(f2 (&v)[E], const float4 *__restrict__ tw) {
    constexpr int NB = E / R;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        const int j = bfly_j<LOG2N, R, LAST>(b);
        f2 x[R];
#pragma unroll
        for (int r = 0; r < R; ++r) x[r] = v[b * R + r];
        if constexpr (NS > 1) {
            // this pass's table, laid out [pair][k]: lanes (consecutive k) read consecutive 16 B
            const int k = j & (NS - 1);
#pragma unroll
            for (int q = 0; q < R / 2; ++q) {
#ifdef SDRG_DIAG_NO_TWIDDLE  // diagnostic builds only (wrong results): time the pass without twiddle loads
                const float4 w = make_float4(1.0f, (float)k * 1e-30f, 1.0f, 0.0f);
#else
                const float4 w = tw[q * NS + k];
#endif
                x[2 * q + 1] = cmul(x[2 * q + 1], f2{w.x, w.y});
                if (2 * q + 2 < R) x[2 * q + 2] = cmul(x[2 * q + 2], f2{w.z, w.w});
            }
        }
        dft<R>(x);
#pragma unroll
        for (int r = 0; r < R; ++r) v[b * R + r] = x[r];
    }
}

// Exchange pass P's outputs (radix R, NS) into pass P+1's inputs (radix R2) through an LDS buffer that
// holds HALF the frame: phase h moves the outputs whose position lies in half h.  A reader's element
// e = j' + r' N/R2 is in half 0 iff r' < R2/2 (compile-time), so every phase reads exactly half of each
// thread's next inputs; a writer's outputs all fall in one half when NB = 1, so in phase 0 the waves of
// the lower half of the threads empty their registers while the upper half still hold theirs (48 live
// complex values at most).
template <int LOG2N, int R, int NS, int R2, bool NEXT_LAST>
__device__ __forceinline__ void exchange(f2 *lds, f2 (&v)[E]) {
    constexpr int N = 1 << LOG2N;
    constexpr int T = N / E;
    constexpr int NB = E / R, NB2 = E / R2;
    constexpr int HALF = N / 2;
    f2 nxt[E];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            const int j = threadIdx.x + b * T;
            const int base = (j / NS) * NS * R + (j & (NS - 1));
            if ((base >= HALF) == (h == 1)) {  // all R outputs of a butterfly share the half (NS R <= HALF)
#pragma unroll
                for (int r = 0; r < R; ++r) lds[lds_idx(base + r * NS - h * HALF)] = v[b * R + r];
            }
        }
        __syncthreads();
#pragma unroll
        for (int b = 0; b < NB2; ++b) {
            const int j = bfly_j<LOG2N, R2, NEXT_LAST>(b);
#pragma unroll
            for (int r = h * (R2 / 2); r < (h + 1) * (R2 / 2); ++r) nxt[b * R2 + r] = lds[lds_idx(j + r * (N / R2) - h * HALF)];
        }
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < E; ++i) v[i] = nxt[i];
}

template <int LOG2N, int P, int NS>
__device__ __forceinline__ void run_passes(f2 *lds, f2 (&v)[E], float *out, const float4 *tw) {
    using PL = Plan<LOG2N>;
    constexpr int N = 1 << LOG2N;
    constexpr int R = PL::template radix<P>();
    pass_compute<LOG2N, R, NS, P == PL::NP - 1>(v, tw + (P >= 1 ? PL::template tw_offset<P>() : 0));
    if constexpr (P == PL::NP - 1) {
        // last pass: output positions j + r N/R; |X|^2 at the fftshifted index (fft_process.cpp:83-97)
        constexpr int NB = E / R;
        if constexpr (NB == 2) {
            // this thread's two butterflies are j = 2t, 2t+1 (see last_j): one 8-byte store per r
            const int j = 2 * threadIdx.x;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const f2 x0 = v[r], x1 = v[R + r];
                *reinterpret_cast<float2 *>(&out[(j + r * (N / R) + N / 2) & (N - 1)]) =
                    make_float2(x0.x * x0.x + x0.y * x0.y, x1.x * x1.x + x1.y * x1.y);
            }
        } else {
#pragma unroll
            for (int b = 0; b < NB; ++b) {
                const int j = last_j<LOG2N, R>(b);
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const f2 x = v[b * R + r];
                    out[(j + r * (N / R) + N / 2) & (N - 1)] = x.x * x.x + x.y * x.y;
                }
            }
        }
    } else {
        constexpr int R2 = PL::template radix<P + 1>();
        exchange<LOG2N, R, NS, R2, P + 1 == PL::NP - 1>(lds, v);
        run_passes<LOG2N, P + 1, NS * R>(lds, v, out, tw);
    }
}

template <int LOG2N, int FMT>
__global__ __launch_bounds__(Plan<LOG2N>::T, 2) void spectrum_kernel(const void *__restrict__ iq,
                                                                     float *__restrict__ spectra,
                                                                     const float4 *__restrict__ tw) {
    using PL = Plan<LOG2N>;
    constexpr int N = PL::N, T = PL::T, R0 = PL::template radix<0>(), NB0 = E / R0;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    f2 *lds = reinterpret_cast<f2 *>(smem);
    const size_t frame = blockIdx.x;
    const void *src = reinterpret_cast<const char *>(iq) + frame * (size_t)N * bytes_per_sample<FMT>();
    f2 v[E];
    constexpr int BYTES = N * bytes_per_sample<FMT>();
    constexpr int WAVES = T / 64;
    // measured (tools/gpu_variants.sh): staging the raw frame through LDS by LDS-DMA is slower than the
    // direct strided loads at N = 16384 (0.157 vs 0.148 ms per 4096 frames); kept as a build option
#ifdef SDRG_SPEC_DMA
    constexpr bool DMA = FMT != SDRG_IQ_CF32 && WAVES >= 1 && BYTES <= PL::LDS_BYTES && BYTES % (WAVES * 1024) == 0;
#else
    constexpr bool DMA = false;
#endif
    if constexpr (DMA) {
        // the raw frame (32 KiB CS8, 64 KiB CS16) lands in the exchange buffer by LDS-DMA, 16 B per lane and
        // 1 KiB per wave instruction, then each thread picks its strided samples out of LDS
        const int wave = threadIdx.x / 64, lane = threadIdx.x % 64;
#pragma unroll
        for (int q = 0; q < BYTES / (WAVES * 1024); q++) {
            const int piece = wave + q * WAVES;
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void *)(reinterpret_cast<const char *>(src) + piece * 1024 + lane * 16),
                (__attribute__((address_space(3))) void *)(smem + piece * 1024), 16, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
#pragma unroll
        for (int b = 0; b < NB0; ++b) {
            const int j = threadIdx.x + b * T;
#pragma unroll
            for (int r = 0; r < R0; ++r) v[b * R0 + r] = load_sample<FMT>(smem, j + r * (N / R0));
        }
        __syncthreads();  // the first exchange overwrites the raw bytes
    } else {
#pragma unroll
        for (int b = 0; b < NB0; ++b) {
            const int j = threadIdx.x + b * T;
#pragma unroll
            for (int r = 0; r < R0; ++r) v[b * R0 + r] = load_sample<FMT>(src, j + r * (N / R0));
        }
    }
    run_passes<LOG2N, 0, 1>(lds, v, spectra + frame * (size_t)N, tw);
}

template <int LOG2N, int FMT>
hipError_t launch_t(const void *iq, int n_frames, const float *tw, float *spectra, hipStream_t s) {
    using PL = Plan<LOG2N>;
    auto k = spectrum_kernel<LOG2N, FMT>;
    static bool attr_set = false;
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(k),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, PL::LDS_BYTES);
        if (e != hipSuccess) return e;
        attr_set = true;
    }
    // the per-pass tables follow the full W_N table (layout of spectrum_fill_twiddles)
    const float4 *pass_tw = reinterpret_cast<const float4 *>(tw + 2 * (size_t)PL::N);
    hipLaunchKernelGGL(k, dim3(n_frames), dim3(PL::T), PL::LDS_BYTES, s, iq, spectra, pass_tw);
    return hipGetLastError();
}

template <int LOG2N>
hipError_t launch_n(const void *iq, int fmt, int n_frames, const float *tw, float *spectra, hipStream_t s) {
    switch (fmt) {
    case SDRG_IQ_CS8: return launch_t<LOG2N, SDRG_IQ_CS8>(iq, n_frames, tw, spectra, s);
    case SDRG_IQ_CU8: return launch_t<LOG2N, SDRG_IQ_CU8>(iq, n_frames, tw, spectra, s);
    case SDRG_IQ_CS16: return launch_t<LOG2N, SDRG_IQ_CS16>(iq, n_frames, tw, spectra, s);
    case SDRG_IQ_CF32: return launch_t<LOG2N, SDRG_IQ_CF32>(iq, n_frames, tw, spectra, s);
    default: return hipErrorInvalidValue;
    }
}

// ================================================================================================
// N = 32768 / 65536: the frame (256 / 512 KiB as complex float) does not fit in LDS (160 KiB), so the
// transform is a two-kernel four-step FFT, N = N1 * N2 with n = N2 n1 + n2 and k = k1 + N1 k2:
//   kernel A (column tiles): Y[k1][n2] = W_N^(n2 k1) * DFT_N1 over n1 of x[N2 n1 + n2]   (reads raw IQ)
//   kernel B (row tiles)   : X[k1 + N1 k2] = DFT_N2 over n2 of Y[k1][n2]; writes |X|^2 fftshifted
// Each tile runs a Stockham FFT in LDS with 16 values per thread.  Frames go through in waves whose
// intermediate Y (8 B/sample) stays inside the 256 MiB Infinity Cache between the two kernels.
// ================================================================================================
constexpr int TILE_T = 256;  // threads per tile workgroup

template <int L>
struct TilePlan {
    static constexpr int C = 16 * TILE_T / L;  // columns (rows) per tile so that C*L = 16*T
    static constexpr int LP = L + 1;           // padded column length in LDS
    static constexpr int RA = (L == 256) ? 16 : (L == 128) ? 8 : 0;
    static constexpr int RB = 16;
};

// One Stockham pass over every column of an LDS tile [C][LP]; FIRST reads through load(c, e),
// LAST writes through store(c, k, v).
template <int N, int L, int R, int NS, bool FIRST, bool LAST, class Load, class Store>
__device__ __forceinline__ void tile_pass(f2 *lds, const f2 *__restrict__ tw, Load load, Store store) {
    using TP = TilePlan<L>;
    constexpr int C = TP::C;
    constexpr int NB = (C * L / R) / TILE_T;
    static_assert(NB >= 1, "tile too small for radix");
    const int c = threadIdx.x % C, jj = threadIdx.x / C;
    f2 x[NB][R];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        const int j = jj + b * (TILE_T / C);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int e = j + r * (L / R);
            if constexpr (FIRST)
                x[b][r] = load(c, e);
            else
                x[b][r] = lds[c * TP::LP + e];
        }
    }
    if constexpr (!FIRST) __syncthreads();
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        const int j = jj + b * (TILE_T / C);
        if constexpr (NS > 1) {
            const int k = j & (NS - 1);
#pragma unroll
            for (int r = 1; r < R; ++r) x[b][r] = cmul(x[b][r], tw[(r * k) * (N / (NS * R))]);
        }
        dft<R>(x[b]);
        if constexpr (LAST) {
#pragma unroll
            for (int r = 0; r < R; ++r) store(c, j + r * (L / R), x[b][r]);
        } else {
            const int base = (j / NS) * NS * R + (j & (NS - 1));
#pragma unroll
            for (int r = 0; r < R; ++r) lds[c * TP::LP + base + r * NS] = x[b][r];
        }
    }
    if constexpr (!LAST) __syncthreads();
}

template <int LOG2N1, int LOG2N2, int FMT>
__global__ __launch_bounds__(TILE_T) void four_step_a(const void *__restrict__ iq, f2 *__restrict__ Y,
                                                       const f2 *__restrict__ tw) {
    constexpr int N1 = 1 << LOG2N1, N2 = 1 << LOG2N2, N = N1 * N2;
    using TP = TilePlan<N1>;
    __shared__ __attribute__((aligned(16))) f2 lds[TP::C * TP::LP];
    const size_t frame = blockIdx.y;
    const int c0 = blockIdx.x * TP::C;
    const void *src = reinterpret_cast<const char *>(iq) + frame * (size_t)N * bytes_per_sample<FMT>();
    f2 *y = Y + frame * (size_t)N;
    auto load = [&](int c, int n1) { return load_sample<FMT>(src, N2 * n1 + c0 + c); };
    auto none = [](int, int, f2) {};
    auto store = [&](int c, int k1, f2 v) {
        const int n2 = c0 + c;
        y[k1 * N2 + n2] = cmul(v, tw[(n2 * k1) & (N - 1)]);
    };
    auto noload = [](int, int) { return f2{0.0f, 0.0f}; };
    tile_pass<N, N1, TP::RA, 1, true, false>(lds, tw, load, none);
    tile_pass<N, N1, TP::RB, TP::RA, false, true>(lds, tw, noload, store);
}

template <int LOG2N1, int LOG2N2>
__global__ __launch_bounds__(TILE_T) void four_step_b(const f2 *__restrict__ Y, float *__restrict__ spectra,
                                                       const f2 *__restrict__ tw) {
    constexpr int N1 = 1 << LOG2N1, N2 = 1 << LOG2N2, N = N1 * N2;
    using TP = TilePlan<N2>;
    __shared__ __attribute__((aligned(16))) f2 lds[TP::C * TP::LP];
    const size_t frame = blockIdx.y;
    const int r0 = blockIdx.x * TP::C;
    const f2 *y = Y + frame * (size_t)N + (size_t)r0 * N2;
    float *out = spectra + frame * (size_t)N;
    // stage the C rows coalesced
#pragma unroll
    for (int i = 0; i < TP::C * N2 / TILE_T; ++i) {
        const int e = threadIdx.x + i * TILE_T;
        lds[(e / N2) * TP::LP + (e % N2)] = y[e];
    }
    __syncthreads();
    auto noload = [](int, int) { return f2{0.0f, 0.0f}; };
    auto none = [](int, int, f2) {};
    auto store = [&](int rho, int k2, f2 v) {
        const int k = r0 + rho + N1 * k2;
        out[(k + N / 2) & (N - 1)] = v.x * v.x + v.y * v.y;
    };
    tile_pass<N, N2, TP::RA, 1, false, false>(lds, tw, noload, none);
    tile_pass<N, N2, TP::RB, TP::RA, false, true>(lds, tw, noload, store);
}

template <int LOG2N1, int LOG2N2, int FMT>
hipError_t launch_four_step(const void *iq, int n_frames, const float *twf, float *spectra, float *scratch,
                            int wave, hipStream_t s) {
    constexpr int N1 = 1 << LOG2N1, N2 = 1 << LOG2N2, N = N1 * N2;
    const f2 *tw = reinterpret_cast<const f2 *>(twf);
    f2 *Y = reinterpret_cast<f2 *>(scratch);
    for (int f0 = 0; f0 < n_frames; f0 += wave) {
        const int nf = (n_frames - f0) < wave ? (n_frames - f0) : wave;
        const char *src = reinterpret_cast<const char *>(iq) + (size_t)f0 * N * bytes_per_sample<FMT>();
        hipLaunchKernelGGL((four_step_a<LOG2N1, LOG2N2, FMT>), dim3(N2 / TilePlan<N1>::C, nf), dim3(TILE_T), 0, s,
                           src, Y, tw);
        hipLaunchKernelGGL((four_step_b<LOG2N1, LOG2N2>), dim3(N1 / TilePlan<N2>::C, nf), dim3(TILE_T), 0, s, Y,
                           spectra + (size_t)f0 * N, tw);
    }
    return hipGetLastError();
}

template <int LOG2N1, int LOG2N2>
hipError_t launch_four_step_fmt(const void *iq, int fmt, int n_frames, const float *tw, float *spectra,
                                float *scratch, int wave, hipStream_t s) {
    switch (fmt) {
    case SDRG_IQ_CS8: return launch_four_step<LOG2N1, LOG2N2, SDRG_IQ_CS8>(iq, n_frames, tw, spectra, scratch, wave, s);
    case SDRG_IQ_CU8: return launch_four_step<LOG2N1, LOG2N2, SDRG_IQ_CU8>(iq, n_frames, tw, spectra, scratch, wave, s);
    case SDRG_IQ_CS16: return launch_four_step<LOG2N1, LOG2N2, SDRG_IQ_CS16>(iq, n_frames, tw, spectra, scratch, wave, s);
    case SDRG_IQ_CF32: return launch_four_step<LOG2N1, LOG2N2, SDRG_IQ_CF32>(iq, n_frames, tw, spectra, scratch, wave, s);
    default: return hipErrorInvalidValue;
    }
}

}  // namespace

template <int LOG2N>
static void fill_pass_tables(std::vector<float> &tw, size_t at) {
    using PL = Plan<LOG2N>;
    auto fill = [&](auto pc) {
        constexpr int P = decltype(pc)::value;
        if constexpr (P >= 1 && P < PL::NP) {
            constexpr int R = PL::template radix<P>(), NS = PL::template ns<P>();
            const size_t base = at + 4 * (size_t)PL::template tw_offset<P>();
            for (int q = 0; q < R / 2; q++)
                for (int k = 0; k < NS; k++)
                    for (int h = 0; h < 2; h++) {
                        const int r = 2 * q + 1 + h;
                        const double a = -2.0 * M_PI * (double)((long long)r * k % (NS * R)) / (double)(NS * R);
                        const size_t o = base + 4 * ((size_t)q * NS + k) + 2 * h;
                        tw[o] = (r < R) ? (float)cos(a) : 0.0f;
                        tw[o + 1] = (r < R) ? (float)sin(a) : 0.0f;
                    }
        }
    };
    fill(std::integral_constant<int, 1>{});
    fill(std::integral_constant<int, 2>{});
    fill(std::integral_constant<int, 3>{});
}

size_t spectrum_twiddle_floats(int n) {
    size_t pass = 0;
    switch (n) {
#define SDRG_TW_CASE(L) \
    case 1 << L: pass = 4 * (size_t)Plan<L>::TW_F4; break;
        SDRG_TW_CASE(6) SDRG_TW_CASE(7) SDRG_TW_CASE(8) SDRG_TW_CASE(9) SDRG_TW_CASE(10) SDRG_TW_CASE(11)
        SDRG_TW_CASE(12) SDRG_TW_CASE(13) SDRG_TW_CASE(14)
#undef SDRG_TW_CASE
    default: break;
    }
    return 2 * (size_t)n + pass;
}

// Layout: the full table W_N^m (m < N, the four-step kernels), then for N <= 16384 the LDS kernel's
// per-pass tables.  Every entry is exp(-2 pi i m / M) evaluated in double and rounded once to float.
void spectrum_fill_twiddles(int n, float *out) {
    std::vector<float> tw(spectrum_twiddle_floats(n));
    for (int m = 0; m < n; m++) {
        const double a = -2.0 * M_PI * m / (double)n;
        tw[2 * (size_t)m] = (float)cos(a);
        tw[2 * (size_t)m + 1] = (float)sin(a);
    }
    switch (n) {
#define SDRG_TW_CASE(L) \
    case 1 << L: fill_pass_tables<L>(tw, 2 * (size_t)n); break;
        SDRG_TW_CASE(6) SDRG_TW_CASE(7) SDRG_TW_CASE(8) SDRG_TW_CASE(9) SDRG_TW_CASE(10) SDRG_TW_CASE(11)
        SDRG_TW_CASE(12) SDRG_TW_CASE(13) SDRG_TW_CASE(14)
#undef SDRG_TW_CASE
    default: break;
    }
    memcpy(out, tw.data(), tw.size() * sizeof(float));
}

bool spectrum_supported(int n) {
    return n >= 64 && n <= 65536 && (n & (n - 1)) == 0;
}

size_t spectrum_scratch_floats(int n, int n_frames) {
    if (n <= 16384) return 0;
    const int wave = n_frames < SPECTRUM_WAVE_FRAMES ? n_frames : SPECTRUM_WAVE_FRAMES;
    return (size_t)wave * n * 2;
}

hipError_t launch_spectrum(const void *iq, int fmt, int n, int n_frames, const float *twiddles, float *spectra,
                           float *scratch, hipStream_t stream) {
    if (n_frames <= 0) return hipSuccess;
    switch (n) {
    case 32768: return launch_four_step_fmt<7, 8>(iq, fmt, n_frames, twiddles, spectra, scratch, SPECTRUM_WAVE_FRAMES, stream);
    case 65536: return launch_four_step_fmt<8, 8>(iq, fmt, n_frames, twiddles, spectra, scratch, SPECTRUM_WAVE_FRAMES, stream);
    case 64: return launch_n<6>(iq, fmt, n_frames, twiddles, spectra, stream);
    case 128: return launch_n<7>(iq, fmt, n_frames, twiddles, spectra, stream);
    case 256: return launch_n<8>(iq, fmt, n_frames, twiddles, spectra, stream);
    case 512: return launch_n<9>(iq, fmt, n_frames, twiddles, spectra, stream);
    case 1024: return launch_n<10>(iq, fmt, n_frames, twiddles, spectra, stream);
    case 2048: return launch_n<11>(iq, fmt, n_frames, twiddles, spectra, stream);
    case 4096: return launch_n<12>(iq, fmt, n_frames, twiddles, spectra, stream);
    case 8192: return launch_n<13>(iq, fmt, n_frames, twiddles, spectra, stream);
    case 16384: return launch_n<14>(iq, fmt, n_frames, twiddles, spectra, stream);
    default: return hipErrorInvalidValue;
    }
}

}  // namespace sdrg

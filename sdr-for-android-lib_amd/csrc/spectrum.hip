// spectrum.hip — fused IQ unpack -> N-point forward FFT -> |X|^2 -> fftshift, one frame per workgroup.
//
// Replaces FFTProcessor::process steps 1-4 (src/dsp/fft_process.cpp:42-97): copy into the FFTW buffer,
// fftwf_plan_dft_1d(N, FORWARD, ESTIMATE) + execute (unnormalised, no window), power = re^2 + im^2,
// fftshift.  The unused 10-frame ring buffer (:62-73) has no observable output and is not kept.
//
// Design (gfx950): Stockham autosort FFT with radix-32 register butterflies, the frame resident in LDS
// between passes (N = 16384: 3 passes = 32 * 32 * 16, two LDS exchanges).  Each thread owns E = 32
// complex values (T = N/32 threads, 512 at N = 16384).  Pass 0 reads the raw int8/uint8/int16/float
// samples straight from HBM (coalesced across lanes) and converts them in registers; the last pass
// writes |X|^2 straight to HBM at the fftshifted index (coalesced).  Complex arithmetic is written on
// 2-wide float vectors so it maps onto v_pk_{add,mul,fma}_f32.  HBM traffic = bytes in + 4 B out per
// sample (6 B/sample for CS8), the algorithmic minimum.
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

// One Stockham pass: radix R, Ns = product of the previous radices.
//   j in [0, N/R): k = j mod Ns; x[r] = A[j + r N/R] * w^(r k), w = exp(-2 pi i/(Ns R)); X = DFT_R(x);
//   B[(j/Ns) Ns R + k + r Ns] = X[r]
template <int LOG2N, int R, int NS, bool FIRST, bool LAST, int FMT>
__device__ __forceinline__ void stockham_pass(f2 *lds, const void *frame, float *out, const f2 *__restrict__ tw) {
    constexpr int N = 1 << LOG2N;
    constexpr int T = N / E;
    constexpr int NB = E / R;  // butterflies per thread in this pass
    const int t = threadIdx.x;
    f2 x[NB][R];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        const int j = t + b * T;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int e = j + r * (N / R);
            if constexpr (FIRST)
                x[b][r] = load_sample<FMT>(frame, e);
            else
                x[b][r] = lds[lds_idx(e)];
        }
    }
    if constexpr (!FIRST) __syncthreads();  // every read of this pass done before anyone overwrites
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        const int j = t + b * T;
        if constexpr (NS > 1) {
            const int k = j & (NS - 1);
#pragma unroll
            for (int r = 1; r < R; ++r) x[b][r] = cmul(x[b][r], tw[(r * k) * (N / (NS * R))]);
        }
        dft<R>(x[b]);
        if constexpr (LAST) {
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int o = j + r * (N / R);
                const f2 v = x[b][r];
                out[(o + N / 2) & (N - 1)] = v.x * v.x + v.y * v.y;
            }
        } else {
            const int base = (j / NS) * NS * R + (j & (NS - 1));
#pragma unroll
            for (int r = 0; r < R; ++r) lds[lds_idx(base + r * NS)] = x[b][r];
        }
    }
    if constexpr (!LAST) __syncthreads();
}

template <int LOG2N>
struct Plan {
    static constexpr int N = 1 << LOG2N;
    static constexpr int T = N / E;
    static constexpr int NP = (LOG2N + 4) / 5;                   // passes
    static constexpr int RLAST = (LOG2N % 5 == 0) ? 32 : (1 << (LOG2N % 5));
    static constexpr int LDS_BYTES = (N + N / 32) * 8;
};

template <int LOG2N, int P, int NS, int FMT>
__device__ __forceinline__ void run_passes(f2 *lds, const void *frame, float *out, const f2 *tw) {
    using PL = Plan<LOG2N>;
    if constexpr (P < PL::NP) {
        constexpr bool LAST = (P == PL::NP - 1);
        constexpr int R = LAST ? PL::RLAST : 32;
        stockham_pass<LOG2N, R, NS, P == 0, LAST, FMT>(lds, frame, out, tw);
        run_passes<LOG2N, P + 1, NS * R, FMT>(lds, frame, out, tw);
    }
}

template <int LOG2N, int FMT>
__global__ __launch_bounds__(Plan<LOG2N>::T) void spectrum_kernel(const void *__restrict__ iq,
                                                                  float *__restrict__ spectra,
                                                                  const f2 *__restrict__ tw) {
    using PL = Plan<LOG2N>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    f2 *lds = reinterpret_cast<f2 *>(smem);
    const size_t frame = blockIdx.x;
    const void *src = reinterpret_cast<const char *>(iq) + frame * (size_t)PL::N * bytes_per_sample<FMT>();
    float *dst = spectra + frame * (size_t)PL::N;
    run_passes<LOG2N, 0, 1, FMT>(lds, src, dst, tw);
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
    hipLaunchKernelGGL(k, dim3(n_frames), dim3(PL::T), PL::LDS_BYTES, s, iq, spectra,
                       reinterpret_cast<const f2 *>(tw));
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

}  // namespace

bool spectrum_supported(int n) {
    return n >= 64 && n <= 16384 && (n & (n - 1)) == 0;
}

hipError_t launch_spectrum(const void *iq, int fmt, int n, int n_frames, const float *twiddles, float *spectra,
                           hipStream_t stream) {
    if (n_frames <= 0) return hipSuccess;
    switch (n) {
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

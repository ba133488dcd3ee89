// spectrum.hip — fused IQ unpack -> N-point forward FFT -> |X|^2 -> fftshift for a batch of frames.
//
// Replaces FFTProcessor::process steps 1-4 (src/dsp/fft_process.cpp:42-97): copy into the FFTW buffer,
// fftwf_plan_dft_1d(N, FORWARD, ESTIMATE) + execute (unnormalised, no window), power = re^2 + im^2,
// fftshift.  The unused 10-frame ring buffer (:62-73) has no observable output and is not kept.
//
// Design (gfx950):
//   * Stockham autosort FFT with radix-32 register butterflies: each thread owns E = 32 complex values
//     (T = N/32 threads per frame); N = 16384 is 32 x 32 x 16 (3 passes, two LDS exchanges).
//   * Codelets are written against gfx950's packed f32 ops (v_pk_add/mul/fma_f32, 2 lanes = one complex
//     number): the -i and (+-1-i)/sqrt2 twiddles cost no multiply (op_sel swaps and neg modifiers), a
//     general twiddled butterfly is three packed ops (x = a + bW by two fmas, y = 2a - x).
//   * int8/int16 samples are converted unscaled (one SDWA sign-extending convert per component) and the
//     format's power-of-two scale is applied once to |X|^2: scaling by a power of two commutes exactly with
//     every rounding step, so this equals scaling the input.  CU8 subtracts its 127.4 offset on input.
//   * Pass 0 reads the raw samples straight from HBM (coalesced 128-B rows per wave instruction), the last
//     pass writes |X|^2 straight to HBM at the fftshifted index (512-B rows): HBM traffic = bytes in +
//     4 B out per sample (6 B/sample for CS8), the algorithmic minimum.
//   * N = 16384 (the benchmark size) has its own persistent kernel (two 512-thread workgroups per CU looping
//     over frames, twiddles in LDS, the next frame's raw samples loaded before this frame's stores).
//   * N = 32768 / 65536 do not fit a CU's LDS and run as a two-kernel four-step FFT.
// MFMA is not used: there is no dense contraction on this path.
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <type_traits>
#include <vector>

#include "fftany.h"
#include "sdrg_internal.h"

namespace sdrg {
namespace {

#include "fft_codelets.h"

constexpr int E = 32;  // complex values per thread

// ------------------------------------------------------------------------------------------------
// Samples
// ------------------------------------------------------------------------------------------------
// Sample e of a frame with the format's scale (four-step kernels).
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

// Unscaled sample from its raw 16-bit (CS8/CU8) or 32-bit (CS16) word; the power-of-two scale goes on |X|^2.
template <int FMT>
__device__ __forceinline__ f2 convert_raw(uint32_t v) {
    f2 r;
    if constexpr (FMT == SDRG_IQ_CS8) {
        asm("v_cvt_f32_i32_sdwa %0, sext(%1) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0" : "=v"(r.x) : "v"(v));
        asm("v_cvt_f32_i32_sdwa %0, sext(%1) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1" : "=v"(r.y) : "v"(v));
    } else if constexpr (FMT == SDRG_IQ_CU8) {
        // (v - 127.4f) * (1/128): the subtraction here (not a power of two), the 1/128 on |X|^2
        r = f2{(float)(v & 0xffu), (float)((v >> 8) & 0xffu)} - f2{127.4f, 127.4f};
    } else {
        asm("v_cvt_f32_i32_sdwa %0, sext(%1) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_0" : "=v"(r.x) : "v"(v));
        asm("v_cvt_f32_i32_sdwa %0, sext(%1) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1" : "=v"(r.y) : "v"(v));
    }
    return r;
}

// buffer resource over one frame: per-lane offset in a VGPR, per-element offset as a scalar
__device__ __forceinline__ __amdgpu_buffer_rsrc_t frame_rsrc(const void *base, int bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, bytes, 0x00020000);
}

template <int FMT>
__device__ __forceinline__ uint32_t load_raw_word(__amdgpu_buffer_rsrc_t rs, int voff, int soff) {
    if constexpr (bytes_per_sample<FMT>() == 2) return __builtin_amdgcn_raw_buffer_load_b16(rs, voff, soff, 0);
    else return __builtin_amdgcn_raw_buffer_load_b32(rs, voff, soff, 0);
}

template <int FMT>
__device__ __forceinline__ f2 load_unscaled(__amdgpu_buffer_rsrc_t rs, int voff, int soff) {
    if constexpr (FMT == SDRG_IQ_CF32) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b64(rs, voff, soff, 0);
        return f2{__uint_as_float(v[0]), __uint_as_float(v[1])};
    } else {
        return convert_raw<FMT>(load_raw_word<FMT>(rs, voff, soff));
    }
}

// |X|^2 scale of a format: (2^-7)^2 for 8-bit, (2^-15)^2 for 16-bit, 1 for float
template <int FMT>
constexpr float power_scale() {
    return FMT == SDRG_IQ_CF32 ? 1.0f : FMT == SDRG_IQ_CS16 ? 1.0f / 1073741824.0f : 1.0f / 16384.0f;
}

// ------------------------------------------------------------------------------------------------
// Generic LDS kernel (N = 64 .. 8192): one frame per workgroup of T = N/32 threads
// ------------------------------------------------------------------------------------------------
template <int LOG2N>
struct Plan {
    static constexpr int N = 1 << LOG2N;
    static constexpr int T = N / E;
    static constexpr int NP = (LOG2N + 4) / 5;  // passes: radix 32 ..., last = remainder
    static constexpr int RLAST = (LOG2N % 5 == 0) ? 32 : (1 << (LOG2N % 5));
    static constexpr int HALF = N / 2;
    static constexpr int LDS_BYTES = (HALF + HALF / 32) * 8;  // half the frame + pad
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

// LDS slot of element A + c (A per thread, c compile-time) with one pad slot per 32 values: when
// (A mod 32) + (c mod 32) < 32, (A + c) + ((A + c) >> 5) = pad_base(A) + pad_off(c).
__device__ __forceinline__ int pad_base(int a) { return a + (a >> 5); }
constexpr int pad_off(int c) { return c + c / 32; }

// Stockham pass (radix R, NS = product of the previous radices) on the E values a thread holds as
// v[b*R + r] for butterflies j:  x[r] = A[j + r N/R] * w^(r k), k = j mod NS, w = exp(-2 pi i/(NS R));
// X = DFT_R(x);  B[(j/NS) NS R + k + r NS] = X[r]
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
            const int k = j & (NS - 1);  // this pass's table, [pair][k]: lanes read consecutive 16 B
#pragma unroll
            for (int q = 0; q < R / 2; ++q) {
                const float4 w = tw[q * NS + k];
                x[2 * q + 1] = cmul_v(x[2 * q + 1], f2{w.x, w.y});
                if (2 * q + 2 < R) x[2 * q + 2] = cmul_v(x[2 * q + 2], f2{w.z, w.w});
            }
        }
        dft<R>(x);
#pragma unroll
        for (int r = 0; r < R; ++r) v[b * R + r] = x[r];
    }
}

// Exchange pass outputs (radix R, NS) into next-pass inputs (radix R2) through an LDS buffer holding HALF
// the frame: phase h moves the elements whose position lies in half h.  A reader's element j + r N/R2 is
// in half 0 iff r < R2/2 (compile-time); a writer's R outputs share one half (NS R <= N/2), so in phase 0
// the waves of the lower half empty their registers while the upper half still hold theirs.
template <int LOG2N, int R, int NS, int R2, bool NEXT_LAST>
__device__ __forceinline__ void exchange(f2 *lds, f2 (&v)[E]) {
    constexpr int N = 1 << LOG2N;
    constexpr int T = N / E;
    constexpr int NB = E / R, NB2 = E / R2;
    constexpr int HALF = N / 2;
    static_assert(N / R2 >= 32, "reader offsets must be multiples of 32");
    f2 nxt[E];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            const int j = threadIdx.x + b * T;
            const int base = (j / NS) * NS * R + (j & (NS - 1));
            if ((base >= HALF) == (h == 1)) {
                const int pb = pad_base(base - h * HALF);
#pragma unroll
                for (int r = 0; r < R; ++r) lds[pb + pad_off(r * NS)] = v[b * R + r];
            }
        }
        __syncthreads();
#pragma unroll
        for (int b = 0; b < NB2; ++b) {
            const int j = bfly_j<LOG2N, R2, NEXT_LAST>(b);
            const int pj = pad_base(j);
#pragma unroll
            for (int r = h * (R2 / 2); r < (h + 1) * (R2 / 2); ++r) nxt[b * R2 + r] = lds[pj + pad_off(r * (N / R2) - h * HALF)];
        }
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < E; ++i) v[i] = nxt[i];
}

template <int LOG2N, int FMT, int P, int NS>
__device__ __forceinline__ void run_passes(f2 *lds, f2 (&v)[E], float *out, const float4 *tw) {
    using PL = Plan<LOG2N>;
    constexpr int N = 1 << LOG2N;
    constexpr int R = PL::template radix<P>();
    pass_compute<LOG2N, R, NS, P == PL::NP - 1>(v, tw + (P >= 1 ? PL::template tw_offset<P>() : 0));
    if constexpr (P == PL::NP - 1) {
        // last pass: output positions j + r N/R; |X|^2 at the fftshifted index (fft_process.cpp:83-97)
        constexpr int NB = E / R;
        constexpr float S = power_scale<FMT>();
        if constexpr (NB == 2) {
            float *o = out + 2 * threadIdx.x;  // j = 2t, 2t+1 < N/R: the fftshifted index is j + const
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const f2 x0 = v[r], x1 = v[R + r];
                *reinterpret_cast<float2 *>(o + ((r * (N / R) + N / 2) & (N - 1))) =
                    make_float2((x0.x * x0.x + x0.y * x0.y) * S, (x1.x * x1.x + x1.y * x1.y) * S);
            }
        } else {
#pragma unroll
            for (int b = 0; b < NB; ++b) {
                const int j = bfly_j<LOG2N, R, true>(b);
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const f2 x = v[b * R + r];
                    out[(j + r * (N / R) + N / 2) & (N - 1)] = (x.x * x.x + x.y * x.y) * S;
                }
            }
        }
    } else {
        constexpr int R2 = PL::template radix<P + 1>();
        exchange<LOG2N, R, NS, R2, P + 1 == PL::NP - 1>(lds, v);
        run_passes<LOG2N, FMT, P + 1, NS * R>(lds, v, out, tw);
    }
}

template <int LOG2N, int FMT>
__global__ __launch_bounds__(Plan<LOG2N>::T) void spectrum_kernel(const void *__restrict__ iq, float *__restrict__ spectra,
                                                                  const float4 *__restrict__ tw) {
    using PL = Plan<LOG2N>;
    constexpr int N = PL::N, T = PL::T, R0 = PL::template radix<0>(), NB0 = E / R0;
    constexpr int BPS = bytes_per_sample<FMT>();
    extern __shared__ __attribute__((aligned(16))) char smem[];
    f2 *lds = reinterpret_cast<f2 *>(smem);
    const size_t frame = blockIdx.x;
    const __amdgpu_buffer_rsrc_t rs = frame_rsrc(reinterpret_cast<const char *>(iq) + frame * (size_t)N * BPS, N * BPS);
    f2 v[E];
#pragma unroll
    for (int b = 0; b < NB0; ++b) {
        const int voff = (threadIdx.x + b * T) * BPS;
#pragma unroll
        for (int r = 0; r < R0; ++r) v[b * R0 + r] = load_unscaled<FMT>(rs, voff, r * (N / R0) * BPS);
    }
    run_passes<LOG2N, FMT, 0, 1>(lds, v, spectra + frame * (size_t)N, tw);
}

template <int LOG2N, int FMT>
hipError_t launch_t(const void *iq, int n_frames, const float *tw, float *spectra, hipStream_t s) {
    using PL = Plan<LOG2N>;
    auto k = spectrum_kernel<LOG2N, FMT>;
    hipError_t e = ensure_dynamic_lds(reinterpret_cast<const void *>(k), PL::LDS_BYTES);
    if (e != hipSuccess) return e;
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
// N = 16384, the benchmark size: persistent kernel, two 512-thread workgroups per CU (4 waves per SIMD),
// each looping over frames blockIdx.x, + gridDim.x, ...  Stockham plan 32 x 32 x 16 with the twiddles in LDS:
//   pass 1 twiddle w_1024^(r k), k = j mod 32 : P1[r][k]  (8 KiB table)
//   pass 2 twiddle w_16384^(r j), j = 2t + b  : (w^j)^r, w^j = P1[2][j / 32] * A2[j mod 32]  (w_16384^(32 k) =
//     w_1024^(2 k)); the 15 powers by repeated products (error ~r ulp, far inside the parity bound): 2 LDS reads
//     and 30 complex multiplies per thread instead of 30 table reads + 30 multiplies to compose factors.
// The next frame's raw samples are loaded into registers before this frame's |X|^2 stores, so the in-order
// vmcnt wait at the top of the next iteration does not also wait for the stores; the stores are
// non-temporal (the spectra are written once, not re-read by this kernel).  LDS per workgroup: 66 KiB
// half-frame exchange + 8.25 KiB tables.
// Measured (tools/fftlab, 4096 CS8 frames, tools/fftlab/run_variants.sh): ~107 us; the composed-factor
// twiddles with plain stores ~126 us, the generic kernel at this size 137-150 us.
// ================================================================================================
namespace k16 {

// Lab-only ablations (tools/fftlab builds with -DSDRG_K16_ABLATE=mask; results are wrong when set):
// 1 pass-1 twiddles off, 2 pass-2 twiddles off, 4 exchanges off, 8 DFTs off, 16 stores off
#ifndef SDRG_K16_ABLATE
#define SDRG_K16_ABLATE 0
#endif
constexpr int ABL = SDRG_K16_ABLATE;
// the |X|^2 stores' cache policy (buffer-store aux bits, gfx950: 1 sc0, 2 nt, 16 sc1)
#ifndef SDRG_K16_STORE_AUX
#define SDRG_K16_STORE_AUX 2
#endif
constexpr int K16_STORE_AUX = SDRG_K16_STORE_AUX;

constexpr int LOG2N = 14, N = 1 << LOG2N, T = N / E, HALF = N / 2;
constexpr int XCH_F2 = HALF;              // half-frame exchange buffer, f2 slots (XOR-swizzled, no padding)
constexpr int P1_F2 = 32 * 32;            // P1[r][k] = w_1024^(r k), r, k < 32
constexpr int A2_F4 = 16;                 // A2[m] = (w_16384^(2m), w_16384^(2m+1)), m < 16
constexpr int TAB_FLOATS = 2 * P1_F2 + 4 * A2_F4;
constexpr int LDS_BYTES = XCH_F2 * 8 + P1_F2 * 8 + A2_F4 * 16;
static_assert(2 * LDS_BYTES <= 160 * 1024, "two workgroups per CU");

typedef float f2s __attribute__((ext_vector_type(2)));

// The exchanges move half a frame at a time through XCH_F2 slots.  Slot s of a half is stored at
// s ^ (2 ((s >> 5) & 15)): the XOR permutes 16-byte units inside each 256-byte row, so every access pattern
// below -- a thread's 32 consecutive slots written as float4 pairs, 16 lanes reading consecutive slots, and
// 16 lanes reading float4 pairs 2t, 2t + 1 -- spreads a wave's 16-lane groups over all 16 bank groups, and
// a pair stays 16-byte aligned and adjacent, so half the exchange traffic moves as ds_read/write_b128.
__device__ __forceinline__ float4 pair4(f2 a, f2 b) { return make_float4(a.x, a.y, b.x, b.y); }

// pass-0 outputs (radix 32, NS = 1: thread t writes slots 32 t + r) -> pass-1 inputs (thread t reads t + 512 r)
__device__ __forceinline__ void exch1(f2 *lds, f2 (&v)[E]) {
    const int t = threadIdx.x;
    char *lb = reinterpret_cast<char *>(lds);
    f2 nxt[E];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        if ((t >= T / 2) == (h == 1)) {
            const int tp = t - h * (T / 2);
            // the row's LDS byte address with the buffer's base in it: the base is 256-byte aligned (the dynamic
            // allocation starts the kernel's LDS), so the XOR of the unit index touches the row offset only, and
            // each write costs one v_xor (the compiler's form also added the base, a relocation literal, per write)
            uint32_t row = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char *)lb + 256 * tp + ((tp & 15) << 4);
            asm volatile("" : "+v"(row));
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                typedef float v4f __attribute__((ext_vector_type(4)));
                const v4f x = {v[2 * q].x, v[2 * q].y, v[2 * q + 1].x, v[2 * q + 1].y};
                asm volatile("ds_write_b128 %0, %1" ::"v"(row ^ (q << 4)), "v"(x) : "memory");
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the asm writes
        __syncthreads();
        const f2 *rb = lds + (t ^ (2 * ((t >> 5) & 15)));
#pragma unroll
        for (int r = 0; r < 16; ++r) nxt[16 * h + r] = rb[512 * r];
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < E; ++i) v[i] = nxt[i];
}

// pass-1 outputs (radix 32, NS = 32: slots (t / 32) 1024 + t mod 32 + 32 r) -> pass-2 inputs (radix 16, butterflies
// 2t and 2t + 1: slots 2t + b + 1024 r, read as float4 pairs), in a linear layout (no XOR): a
// half-wave's writes of one r are 32 consecutive slots (256 B, every bank once) and a wave's float4 reads 1 KiB of
// consecutive slots, so neither side conflicts, and every access is the thread's base plus a constant offset (no
// address VALU; the XOR layout, shared with exch1's, cost one v_xor per write)
__device__ __forceinline__ void exch2(f2 *lds, f2 (&v)[E]) {
    const int t = threadIdx.x;
    f2 nxt[E];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        if (((t >> 5) >= 8) == (h == 1)) {
            int row = ((t >> 5) - 8 * h) * 1024 + (t & 31);
            asm volatile("" : "+v"(row));  // as in exch1
#pragma unroll
            for (int r = 0; r < 32; ++r) lds[row + 32 * r] = v[r];
        }
        __syncthreads();
        const float4 *rb = reinterpret_cast<const float4 *>(lds + 2 * t);
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const float4 p = rb[512 * r];  // slots 2t, 2t + 1 of row 1024 r
            nxt[8 * h + r] = f2{p.x, p.y};
            nxt[16 + 8 * h + r] = f2{p.z, p.w};
        }
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < E; ++i) v[i] = nxt[i];
}

// raw samples x[t + 512 r] of frame f into registers (zero-extended 16/32-bit words); live = false gives a
// zero-sized resource, so the loads return 0 without touching memory
template <int FMT>
__device__ __forceinline__ void issue_raw(const void *iq, int f, int t, uint32_t (&raw)[E], bool live = true) {
    constexpr int BPS = bytes_per_sample<FMT>();
    const __amdgpu_buffer_rsrc_t rs =
        frame_rsrc(reinterpret_cast<const char *>(iq) + (size_t)f * N * BPS, live ? N * BPS : 0);
#pragma unroll
    for (int r = 0; r < E; ++r) raw[r] = load_raw_word<FMT>(rs, t * BPS, r * (N / 32) * BPS);
}

template <int FMT>
__device__ __forceinline__ void spectrum16k_body(const void *__restrict__ iq, float *__restrict__ spectra,
                                                 const float *__restrict__ tabs, int n_frames) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int XB = XCH_F2 * 8;  // exchange buffer bytes
    f2 *xch = reinterpret_cast<f2 *>(smem);
    f2 *p1 = reinterpret_cast<f2 *>(smem + XB);
    float4 *a2 = reinterpret_cast<float4 *>(smem + XB + P1_F2 * 8);
    const int t = threadIdx.x;
    const int src = t;  // pass 0 reads x[src + 512 r]
    for (int i = t; i < P1_F2; i += T) p1[i] = reinterpret_cast<const f2 *>(tabs)[i];
    for (int i = t; i < A2_F4; i += T) a2[i] = reinterpret_cast<const float4 *>(tabs + 2 * P1_F2)[i];
    __syncthreads();
    constexpr int BPS = bytes_per_sample<FMT>();
    const f2 *p1_row = p1 + (t & 31);  // pass 1: P1[r][k], k = t mod 32

    constexpr bool STAGE = FMT != SDRG_IQ_CF32;  // CF32 (8 B/sample) loads at the top of the iteration
    uint32_t raw[E];
    if constexpr (STAGE) {
        issue_raw<FMT>(iq, (int)blockIdx.x < n_frames ? blockIdx.x : 0, src, raw, (int)blockIdx.x < n_frames);
        // opaque words into the frame loop: with the loop's own loads zero-extended too, the compiler would hoist the
        // zero-extension behind the loop's phi and spend a v_and per word per frame on it (once here, before the loop)
#pragma unroll
        for (int r = 0; r < E; ++r) asm volatile("; raw word %0" : "+v"(raw[r]));
    }

    for (int frame = blockIdx.x; frame < n_frames; frame += gridDim.x) {
        f2 v[E];
        // ---- pass 0: radix 32 over x[t + 512 r] (no twiddles) ----
        if constexpr (STAGE) {
#pragma unroll
            for (int r = 0; r < E; ++r) v[r] = convert_raw<FMT>(raw[r]);
        } else {
            const __amdgpu_buffer_rsrc_t rs = frame_rsrc(reinterpret_cast<const char *>(iq) + (size_t)frame * N * BPS, N * BPS);
#pragma unroll
            for (int r = 0; r < E; ++r) v[r] = load_unscaled<FMT>(rs, src * BPS, r * (N / 32) * BPS);
        }
        const int next = frame + gridDim.x;
        if constexpr (!(ABL & 8)) dft<32>(v);
        if constexpr (!(ABL & 4)) {
            exch1(xch, v);
        }
        // ---- pass 1: radix 32, NS = 32 ----
        if constexpr (!(ABL & 1)) {
#pragma unroll
            for (int r = 1; r < 32; ++r) v[r] = cmul_v(v[r], p1_row[r * 32]);
        }
        if constexpr (!(ABL & 8)) dft<32>(v);
        if constexpr (!(ABL & 4)) {
            exch2(xch, v);
        }
        // ---- pass 2: radix 16, NS = 1024, butterflies j = 2t + b held as v[16 b + r] ----
        if constexpr (!(ABL & 2)) {
            f2 wa, wb;  // w_16384^j for j = 2t, 2t + 1
            {
                const f2 bw = p1[2 * 32 + (t >> 4)];
                const float4 aw = a2[t & 15];
                wa = cmul_v(bw, f2{aw.x, aw.y});
                wb = cmul_v(bw, f2{aw.z, aw.w});
            }
            // the input scale (a power of two, sqrt of power_scale) rides on the pass-2 twiddles and on the two
            // untwiddled rows: every product scales exactly, so |X|^2 comes out scaled by S with the same bits
            // as scaling it afterwards, and the 16 per-output multiplies go
            constexpr float SS = FMT == SDRG_IQ_CF32 ? 1.0f : FMT == SDRG_IQ_CS16 ? 1.0f / 32768.0f : 1.0f / 128.0f;
            static_assert(SS * SS == power_scale<FMT>(), "scale split");
            f2 pa = wa, pb = wb;
            if constexpr (SS != 1.0f) {
                pa = wa * SS;
                pb = wb * SS;
                v[0] = v[0] * SS;
                v[16] = v[16] * SS;
            }
#pragma unroll
            for (int r = 1; r < 16; ++r) {
                if (r > 1) {
                    pa = cmul_v(pa, wa);
                    pb = cmul_v(pb, wb);
                }
                v[r] = cmul_v(v[r], pa);
                v[16 + r] = cmul_v(v[16 + r], pb);
            }
        }
        f2 x0[16], x1[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) { x0[r] = v[r]; x1[r] = v[16 + r]; }
        if constexpr (!(ABL & 8)) {
            dft<16>(x0);
            dft<16>(x1);
        }
        // ---- |X|^2 at the fftshifted index: outputs j + 1024 r, j = 2t, 2t + 1 ----
        f2s pw[16];
        // one v_mul + one v_fma per output (im^2, then re^2 + that: the contraction the packed form compiled to),
        // written straight into the store pair: the packed form needed three moves per pair to transpose the two
        // butterflies' (re, im) into (re0, re1), (im0, im1)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            float q0, q1, p0, p1;
            asm("v_mul_f32 %0, %1, %1" : "=v"(q0) : "v"(x0[r].y));
            asm("v_mul_f32 %0, %1, %1" : "=v"(q1) : "v"(x1[r].y));
            asm("v_fma_f32 %0, %1, %1, %2" : "=v"(p0) : "v"(x0[r].x), "v"(q0));
            asm("v_fma_f32 %0, %1, %1, %2" : "=v"(p1) : "v"(x1[r].x), "v"(q1));
            pw[r] = f2s{p0, p1};
        }
        if constexpr (STAGE) issue_raw<FMT>(iq, next < n_frames ? next : frame, src, raw, next < n_frames);
        float *o = spectra + (size_t)frame * N + 2 * t;
        if constexpr (ABL & 16) {  // keep the values live without the stores
            float acc = 0.f;
#pragma unroll
            for (int r = 0; r < 16; ++r) acc += pw[r].x + pw[r].y;
            if (acc == 1.2345f) o[0] = acc;
        } else {
            // buffer stores: the fftshifted row offsets are scalar constants, so no 64-bit address adds per store
            const __amdgpu_buffer_rsrc_t os = frame_rsrc(spectra + (size_t)frame * N, N * 4);
            typedef unsigned u2 __attribute__((ext_vector_type(2)));
#pragma unroll
            for (int r = 0; r < 16; ++r)
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, pw[r]), os, 8 * t,
                                                      4 * ((r * 1024 + N / 2) & (N - 1)), K16_STORE_AUX);
        }
    }
}

// __launch_bounds__(512, 4): four waves per SIMD = two workgroups per CU, so at most 128 VGPRs
template <int FMT>
__global__ __launch_bounds__(T, 4) void spectrum16k_kernel(const void *__restrict__ iq, float *__restrict__ spectra,
                                                           const float *__restrict__ tabs, int n_frames) {
    spectrum16k_body<FMT>(iq, spectra, tabs, n_frames);
}

// the two LDS tables, laid out as the kernel reads them (exp evaluated in double, rounded once)
void fill_tables(float *out) {
    for (int r = 0; r < 32; r++)
        for (int k = 0; k < 32; k++) {
            const double a = -2.0 * M_PI * (double)(r * k) / 1024.0;
            out[2 * (r * 32 + k)] = (float)cos(a);
            out[2 * (r * 32 + k) + 1] = (float)sin(a);
        }
    float *a2 = out + 2 * P1_F2;
    for (int m = 0; m < 16; m++)
        for (int b = 0; b < 2; b++) {
            const double a = -2.0 * M_PI * (double)(2 * m + b) / 16384.0;
            a2[4 * m + 2 * b] = (float)cos(a);
            a2[4 * m + 2 * b + 1] = (float)sin(a);
        }
}

int device_cus() {
    static const int cus = [] {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            n = 256;
        return n > 0 ? n : 256;
    }();
    return cus;
}

// wg_per_cu: persistent workgroups per CU (2 alone; 1 when the SSB pipeline shares the CUs, see launch_spectrum)
template <int FMT>
hipError_t launch(const void *iq, int n_frames, const float *tabs, float *spectra, hipStream_t s, int wg_per_cu = 2,
                  int n_cus = 0) {
    auto k = spectrum16k_kernel<FMT>;
    const int lds = LDS_BYTES;
    hipError_t e = ensure_dynamic_lds(reinterpret_cast<const void *>(k), lds);
    if (e != hipSuccess) return e;
    static const int max_grid = [] {  // lab override (SDRG_SPECTRUM_GRID): persistent workgroups
        const char *v = lab_getenv("SDRG_SPECTRUM_GRID");
        const int g = v ? atoi(v) : 0;
        return g > 0 ? g : 0;
    }();
    const int cap = max_grid > 0 ? max_grid : (wg_per_cu == 2 ? 2 : 1) * (n_cus > 0 ? n_cus : device_cus());
    const int grid = n_frames < cap ? n_frames : cap;
    hipLaunchKernelGGL(k, dim3(grid), dim3(T), lds, s, iq, spectra, tabs, n_frames);
    return hipGetLastError();
}

hipError_t launch_fmt(const void *iq, int fmt, int n_frames, const float *tabs, float *spectra, hipStream_t s,
                      int wg_per_cu, int n_cus) {
    switch (fmt) {
    case SDRG_IQ_CS8: return launch<SDRG_IQ_CS8>(iq, n_frames, tabs, spectra, s, wg_per_cu, n_cus);
    case SDRG_IQ_CU8: return launch<SDRG_IQ_CU8>(iq, n_frames, tabs, spectra, s, wg_per_cu, n_cus);
    case SDRG_IQ_CS16: return launch<SDRG_IQ_CS16>(iq, n_frames, tabs, spectra, s, wg_per_cu, n_cus);
    case SDRG_IQ_CF32: return launch<SDRG_IQ_CF32>(iq, n_frames, tabs, spectra, s, wg_per_cu, n_cus);
    default: return hipErrorInvalidValue;
    }
}

}  // namespace k16

// ================================================================================================
// N = 32768 / 65536: the frame (256 / 512 KiB as complex float) does not fit in LDS (160 KiB), so the
// transform is a two-kernel four-step FFT, N = N1 * N2 with n = N2 n1 + n2 and k = k1 + N1 k2:
//   kernel A (column tiles): Y[k1][n2] = W_N^(n2 k1) * DFT_N1 over n1 of x[N2 n1 + n2]   (reads raw IQ)
//   kernel B (row tiles)   : X[k1 + N1 k2] = DFT_N2 over n2 of Y[k1][n2]; writes |X|^2 fftshifted
// Each tile runs a Stockham FFT in LDS with 16 values per thread.  Frames go through in waves whose
// intermediate Y (8 B/sample) stays inside the 256 MiB Infinity Cache between the two kernels.
// ================================================================================================
#ifndef SDRG_TILE_A
#define SDRG_TILE_A 512
#endif
constexpr int TILE_A = SDRG_TILE_A;  // threads per kernel-A tile: 32 columns = 128-B rows of CS16 input
constexpr int TILE_B = 256;          // threads per kernel-B tile

template <int L, int TILE_T>
struct TilePlan {
    static constexpr int C = 16 * TILE_T / L;  // columns (rows) per tile so that C*L = 16*T
    static constexpr int LP = L + 1;           // padded column length in LDS
    static constexpr int RA = (L == 256) ? 16 : (L == 128) ? 8 : 0;
    static constexpr int RB = 16;
};

// Twiddles of the four-step kernels from two LDS tables: W_N^m = hi[m >> 8] * lo[m & 255], hi[a] = W_N^(256 a),
// lo[b] = W_N^b (both copied from the full W_N table at kernel start).  Reading W_N^m straight from the
// 512 KiB global table touched one cache line per lane per load (strided m), which bounded kernel A by L2
// line traffic; the LDS product costs one complex multiply.  S: compile-time stride of m (m = i S); when S
// is a multiple of 256 the lo factor is W^0 = 1 and one lookup suffices.
template <int S>
__device__ __forceinline__ f2 tw_lds(const f2 *t_hi, const f2 *t_lo, int i) {
    if constexpr (S % 256 == 0) {
        return t_hi[i * (S / 256)];
    } else {
        const int m = i * S;
        return cmul_v(t_hi[m >> 8], t_lo[m & 255]);
    }
}

template <int N>
__device__ __forceinline__ void load_tw_tables(const f2 *__restrict__ tw, f2 *t_hi, f2 *t_lo) {
    for (int i = threadIdx.x; i < N / 256; i += blockDim.x) t_hi[i] = tw[256 * i];
    for (int i = threadIdx.x; i < 256; i += blockDim.x) t_lo[i] = tw[i];
}

// One Stockham pass over every column of an LDS tile [C][LP]; FIRST reads through load(c, e),
// LAST writes through store(c, k, v).
template <int N, int L, int R, int NS, bool FIRST, bool LAST, int TILE_T, class Load, class Store>
__device__ __forceinline__ void tile_pass(f2 *lds, const f2 *t_hi, const f2 *t_lo, Load load, Store store) {
    using TP = TilePlan<L, TILE_T>;
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
            for (int r = 1; r < R; ++r) x[b][r] = cmul_v(x[b][r], tw_lds<N / (NS * R)>(t_hi, t_lo, r * k));
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
__global__ __launch_bounds__(TILE_A) void four_step_a(const void *__restrict__ iq, f2 *__restrict__ Y,
                                                       const f2 *__restrict__ tw, int hi) {
    if (hi) __builtin_amdgcn_s_setprio(1);  // see launch_four_step
    constexpr int N1 = 1 << LOG2N1, N2 = 1 << LOG2N2, N = N1 * N2;
    using TP = TilePlan<N1, TILE_A>;
    __shared__ __attribute__((aligned(16))) f2 lds[TP::C * TP::LP];
    __shared__ f2 t_hi[N / 256], t_lo[256];
    load_tw_tables<N>(tw, t_hi, t_lo);
    __syncthreads();
    const size_t frame = blockIdx.y;
    const int c0 = blockIdx.x * TP::C;
    const void *src = reinterpret_cast<const char *>(iq) + frame * (size_t)N * bytes_per_sample<FMT>();
    f2 *y = Y + frame * (size_t)N;
    auto load = [&](int c, int n1) { return load_sample<FMT>(src, N2 * n1 + c0 + c); };
    auto none = [](int, int, f2) {};
    auto store = [&](int c, int k1, f2 v) {
        const int n2 = c0 + c;
        y[k1 * N2 + n2] = cmul_v(v, tw_lds<1>(t_hi, t_lo, (n2 * k1) & (N - 1)));
    };
    auto noload = [](int, int) { return f2{0.0f, 0.0f}; };
    tile_pass<N, N1, TP::RA, 1, true, false, TILE_A>(lds, t_hi, t_lo, load, none);
    tile_pass<N, N1, TP::RB, TP::RA, false, true, TILE_A>(lds, t_hi, t_lo, noload, store);
}

template <int LOG2N1, int LOG2N2>
__global__ __launch_bounds__(TILE_B) void four_step_b(const f2 *__restrict__ Y, float *__restrict__ spectra,
                                                       const f2 *__restrict__ tw, int hi) {
    if (hi) __builtin_amdgcn_s_setprio(1);
    constexpr int N1 = 1 << LOG2N1, N2 = 1 << LOG2N2, N = N1 * N2;
    using TP = TilePlan<N2, TILE_B>;
    __shared__ __attribute__((aligned(16))) f2 lds[TP::C * TP::LP];
    __shared__ f2 t_hi[N / 256], t_lo[256];
    load_tw_tables<N>(tw, t_hi, t_lo);  // visible after the staging barrier below
    const size_t frame = blockIdx.y;
    const int r0 = blockIdx.x * TP::C;
    const f2 *y = Y + frame * (size_t)N + (size_t)r0 * N2;
    float *out = spectra + frame * (size_t)N;
    // stage the C rows coalesced
#pragma unroll
    for (int i = 0; i < TP::C * N2 / TILE_B; ++i) {
        const int e = threadIdx.x + i * TILE_B;
        lds[(e / N2) * TP::LP + (e % N2)] = y[e];
    }
    __syncthreads();
    auto noload = [](int, int) { return f2{0.0f, 0.0f}; };
    auto none = [](int, int, f2) {};
    auto store = [&](int rho, int k2, f2 v) {
        const int k = r0 + rho + N1 * k2;
        out[(k + N / 2) & (N - 1)] = v.x * v.x + v.y * v.y;
    };
    tile_pass<N, N2, TP::RA, 1, false, false, TILE_B>(lds, t_hi, t_lo, noload, none);
    tile_pass<N, N2, TP::RB, TP::RA, false, true, TILE_B>(lds, t_hi, t_lo, noload, store);
}

// Persistent forms of the two four-step kernels: a grid of a few workgroups per CU loops over the wave's tiles, loads
// the twiddle tables once, and fetches the NEXT tile's inputs into registers (raw 8/16-bit words for kernel A, the
// staged rows for kernel B) before running this tile's FFT, so HBM / Infinity Cache latency overlaps the LDS passes
// instead of following them.  Same arithmetic as four_step_a / four_step_b (the same bits).  Measured at 1024 x
// 65536 CS16 (tools/gpu_four_persist.sh): A 42.6 -> 40.7 us, B 32.4 -> 33.1 us per 256-frame wave, the configs[4]
// 5 kHz step 0.320 -> 0.312 ms; beside the wide statistics kernel (200 kHz focus, asynchronous statistics) they are
// 1 % slower than the one-tile-per-workgroup kernels, so launch_spectrum takes those there (persistent = false).
template <int FMT>
__device__ __forceinline__ f2 convert_scaled(uint32_t v) {  // load_sample's value from its raw word
    if constexpr (FMT == SDRG_IQ_CS8) {
        return f2{(float)(int8_t)(v & 0xff), (float)(int8_t)((v >> 8) & 0xff)} * (1.0f / 128.0f);
    } else if constexpr (FMT == SDRG_IQ_CU8) {
        return (f2{(float)(v & 0xff), (float)((v >> 8) & 0xff)} - 127.4f) * (1.0f / 128.0f);
    } else {
        return f2{(float)(int16_t)(v & 0xffff), (float)(int16_t)(v >> 16)} * (1.0f / 32768.0f);
    }
}

template <int LOG2N1, int LOG2N2, int FMT>
__global__ __launch_bounds__(TILE_A) void four_step_a_p(const void *__restrict__ iq, f2 *__restrict__ Y,
                                                         const f2 *__restrict__ tw, int n_frames, int hi) {
    if (hi) __builtin_amdgcn_s_setprio(1);
    constexpr int N1 = 1 << LOG2N1, N2 = 1 << LOG2N2, N = N1 * N2;
    using TP = TilePlan<N1, TILE_A>;
    constexpr int C = TP::C, R = TP::RA, TPF = N2 / C, NB = (C * N1 / R) / TILE_A, JS = TILE_A / C;
    constexpr int BPS = bytes_per_sample<FMT>();
    __shared__ __attribute__((aligned(16))) f2 lds[C * TP::LP];
    __shared__ f2 t_hi[N / 256], t_lo[256];
    load_tw_tables<N>(tw, t_hi, t_lo);
    __syncthreads();
    const int total = n_frames * TPF;
    const int c = threadIdx.x % C, jj = threadIdx.x / C;  // pass 1: column c, butterflies j = jj + b * JS
    constexpr bool RAW = FMT != SDRG_IQ_CF32;
    uint32_t raw[NB][R];
    auto issue = [&](int tile) {
        const int frame = tile / TPF, c0 = (tile % TPF) * C;
        const __amdgpu_buffer_rsrc_t rs =
            frame_rsrc(reinterpret_cast<const char *>(iq) + (size_t)frame * N * BPS, N * BPS);
#pragma unroll
        for (int b = 0; b < NB; b++)
#pragma unroll
            for (int r = 0; r < R; r++)
                raw[b][r] = load_raw_word<FMT>(rs, (c0 + c) * BPS, N2 * (jj + b * JS + r * (N1 / R)) * BPS);
    };
    int tile = blockIdx.x;
    if constexpr (RAW)
        if (tile < total) issue(tile);
    for (; tile < total; tile += gridDim.x) {
        const int frame = tile / TPF, c0 = (tile % TPF) * C;
        f2 x[NB][R];
        if constexpr (RAW) {
#pragma unroll
            for (int b = 0; b < NB; b++)
#pragma unroll
                for (int r = 0; r < R; r++) x[b][r] = convert_scaled<FMT>(raw[b][r]);
            if (tile + (int)gridDim.x < total) issue(tile + gridDim.x);
        } else {
            const f2 *src = reinterpret_cast<const f2 *>(iq) + (size_t)frame * N;
#pragma unroll
            for (int b = 0; b < NB; b++)
#pragma unroll
                for (int r = 0; r < R; r++) x[b][r] = src[N2 * (jj + b * JS + r * (N1 / R)) + c0 + c];
        }
        // pass 1 (NS = 1): DFT over n1, outputs to the column's LDS slots j * R + r
#pragma unroll
        for (int b = 0; b < NB; b++) {
            dft<R>(x[b]);
#pragma unroll
            for (int r = 0; r < R; r++) lds[c * TP::LP + (jj + b * JS) * R + r] = x[b][r];
        }
        __syncthreads();
        f2 *y = Y + (size_t)frame * N;
        auto noload = [](int, int) { return f2{0.0f, 0.0f}; };
        auto store = [&](int cc, int k1, f2 v) {
            const int n2 = c0 + cc;
            const f2 w = cmul_v(v, tw_lds<1>(t_hi, t_lo, (n2 * k1) & (N - 1)));
            y[k1 * N2 + n2] = w;
        };
        // pass 2 reads the tile, then a barrier (inside), so the next tile's pass-1 writes are safe
        tile_pass<N, N1, TP::RB, TP::RA, false, true, TILE_A>(lds, t_hi, t_lo, noload, store);
    }
}

template <int LOG2N1, int LOG2N2>
__global__ __launch_bounds__(TILE_B) void four_step_b_p(const f2 *__restrict__ Y, float *__restrict__ spectra,
                                                         const f2 *__restrict__ tw, int n_frames, int hi) {
    if (hi) __builtin_amdgcn_s_setprio(1);
    constexpr int N1 = 1 << LOG2N1, N2 = 1 << LOG2N2, N = N1 * N2;
    using TP = TilePlan<N2, TILE_B>;
    constexpr int C = TP::C, TPF = N1 / C, S = C * N2 / TILE_B;
    __shared__ __attribute__((aligned(16))) f2 lds[C * TP::LP];
    __shared__ f2 t_hi[N / 256], t_lo[256];
    load_tw_tables<N>(tw, t_hi, t_lo);  // visible after the first staging barrier
    const int total = n_frames * TPF;
    f2 stage[S];
    auto issue = [&](int tile) {
        const int frame = tile / TPF, r0 = (tile % TPF) * C;
        const f2 *y = Y + (size_t)frame * N + (size_t)r0 * N2;
#pragma unroll
        for (int i = 0; i < S; ++i) stage[i] = y[threadIdx.x + i * TILE_B];
    };
    int tile = blockIdx.x;
    if (tile < total) issue(tile);
    for (; tile < total; tile += gridDim.x) {
        const int frame = tile / TPF, r0 = (tile % TPF) * C;
#pragma unroll
        for (int i = 0; i < S; ++i) {
            const int e = threadIdx.x + i * TILE_B;
            lds[(e / N2) * TP::LP + (e % N2)] = stage[i];
        }
        if (tile + (int)gridDim.x < total) issue(tile + gridDim.x);
        __syncthreads();
        float *out = spectra + (size_t)frame * N;
        auto noload = [](int, int) { return f2{0.0f, 0.0f}; };
        auto none = [](int, int, f2) {};
        auto store = [&](int rho, int k2, f2 v) {
            const int k = r0 + rho + N1 * k2;
            out[(k + N / 2) & (N - 1)] = v.x * v.x + v.y * v.y;
        };
        tile_pass<N, N2, TP::RA, 1, false, false, TILE_B>(lds, t_hi, t_lo, noload, none);
        tile_pass<N, N2, TP::RB, TP::RA, false, true, TILE_B>(lds, t_hi, t_lo, noload, store);
    }
}

// hi: the waves run at issue priority 1, above statistics that run beside them on a stream of their own (configs[4]
// at 5 kHz: 0.3096-0.3113 vs 0.3127-0.3130 ms per step, 200 kHz unchanged, tools/gpu_r4y.sh); not beside the SSB
// pipeline, whose helper roles at priority 0 would yield to them
template <int LOG2N1, int LOG2N2, int FMT>
hipError_t launch_four_step(const void *iq, int n_frames, const float *twf, float *spectra, float *scratch,
                            int wave, hipStream_t s, bool persistent, bool hi_prio) {
    const int hi = hi_prio ? 1 : 0;
    constexpr int N1 = 1 << LOG2N1, N2 = 1 << LOG2N2, N = N1 * N2;
    const f2 *tw = reinterpret_cast<const f2 *>(twf);
    f2 *Y = reinterpret_cast<f2 *>(scratch);
    for (int f0 = 0; f0 < n_frames; f0 += wave) {
        const int nf = (n_frames - f0) < wave ? (n_frames - f0) : wave;
        const char *src = reinterpret_cast<const char *>(iq) + (size_t)f0 * N * bytes_per_sample<FMT>();
        if (persistent) {
            const int cus = k16::device_cus();
            const int ta = nf * (N2 / TilePlan<N1, TILE_A>::C), tb = nf * (N1 / TilePlan<N2, TILE_B>::C);
            const int ga = ta < 2 * cus ? ta : 2 * cus, gb = tb < 4 * cus ? tb : 4 * cus;
            hipLaunchKernelGGL((four_step_a_p<LOG2N1, LOG2N2, FMT>), dim3(ga), dim3(TILE_A), 0, s, src, Y, tw, nf, hi);
            hipLaunchKernelGGL((four_step_b_p<LOG2N1, LOG2N2>), dim3(gb), dim3(TILE_B), 0, s, Y, spectra + (size_t)f0 * N,
                               tw, nf, hi);
            continue;
        }
        hipLaunchKernelGGL((four_step_a<LOG2N1, LOG2N2, FMT>), dim3(N2 / TilePlan<N1, TILE_A>::C, nf), dim3(TILE_A), 0,
                           s, src, Y, tw, hi);
        hipLaunchKernelGGL((four_step_b<LOG2N1, LOG2N2>), dim3(N1 / TilePlan<N2, TILE_B>::C, nf), dim3(TILE_B), 0, s, Y,
                           spectra + (size_t)f0 * N, tw, hi);
    }
    return hipGetLastError();
}

template <int LOG2N1, int LOG2N2>
hipError_t launch_four_step_fmt(const void *iq, int fmt, int n_frames, const float *tw, float *spectra,
                                float *scratch, int wave, hipStream_t s, bool pe, bool hi) {
    switch (fmt) {
    case SDRG_IQ_CS8: return launch_four_step<LOG2N1, LOG2N2, SDRG_IQ_CS8>(iq, n_frames, tw, spectra, scratch, wave, s, pe, hi);
    case SDRG_IQ_CU8: return launch_four_step<LOG2N1, LOG2N2, SDRG_IQ_CU8>(iq, n_frames, tw, spectra, scratch, wave, s, pe, hi);
    case SDRG_IQ_CS16: return launch_four_step<LOG2N1, LOG2N2, SDRG_IQ_CS16>(iq, n_frames, tw, spectra, scratch, wave, s, pe, hi);
    case SDRG_IQ_CF32: return launch_four_step<LOG2N1, LOG2N2, SDRG_IQ_CF32>(iq, n_frames, tw, spectra, scratch, wave, s, pe, hi);
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

// Twiddle buffer layout: the full table W_N^m (m < N, four-step kernels), then for N <= 8192 the generic
// kernel's per-pass tables, or for N = 16384 the k16 kernel's LDS tables.  Every entry is exp(-2 pi i m / M)
// evaluated in double and rounded once to float.
size_t spectrum_k16_tables_offset() { return 2 * (size_t)16384; }

static bool pow2_kernels(int n) { return n >= 64 && n <= 65536 && (n & (n - 1)) == 0; }

size_t spectrum_twiddle_floats(int n) {
    if (!pow2_kernels(n)) return any_table_floats(any_plan(n));  // fftany.hip
    size_t pass = 0;
    if (n == 16384) return spectrum_k16_tables_offset() + k16::TAB_FLOATS;
    switch (n) {
#define SDRG_TW_CASE(L) \
    case 1 << L: pass = 4 * (size_t)Plan<L>::TW_F4; break;
        SDRG_TW_CASE(6) SDRG_TW_CASE(7) SDRG_TW_CASE(8) SDRG_TW_CASE(9) SDRG_TW_CASE(10) SDRG_TW_CASE(11)
        SDRG_TW_CASE(12) SDRG_TW_CASE(13)
#undef SDRG_TW_CASE
    default: break;
    }
    return 2 * (size_t)n + pass;
}

void spectrum_fill_twiddles(int n, float *out) {
    if (!pow2_kernels(n)) {
        any_fill_tables(any_plan(n), out);
        return;
    }
    std::vector<float> tw(spectrum_twiddle_floats(n));
    for (int m = 0; m < n; m++) {
        const double a = -2.0 * M_PI * m / (double)n;
        tw[2 * (size_t)m] = (float)cos(a);
        tw[2 * (size_t)m + 1] = (float)sin(a);
    }
    if (n == 16384) k16::fill_tables(tw.data() + spectrum_k16_tables_offset());
    switch (n) {
#define SDRG_TW_CASE(L) \
    case 1 << L: fill_pass_tables<L>(tw, 2 * (size_t)n); break;
        SDRG_TW_CASE(6) SDRG_TW_CASE(7) SDRG_TW_CASE(8) SDRG_TW_CASE(9) SDRG_TW_CASE(10) SDRG_TW_CASE(11)
        SDRG_TW_CASE(12) SDRG_TW_CASE(13)
#undef SDRG_TW_CASE
    default: break;
    }
    memcpy(out, tw.data(), tw.size() * sizeof(float));
}

bool spectrum_supported(int n) { return n >= 1 && n <= (1 << 20); }

size_t spectrum_scratch_floats(int n, int n_frames) {
    if (!pow2_kernels(n)) return any_scratch_floats(any_plan(n), n_frames);
    if (n <= 16384) return 0;
    const int wave = n_frames < spectrum_wave_frames(n) ? n_frames : spectrum_wave_frames(n);
    return (size_t)wave * n * 2;
}

hipError_t launch_spectrum(const void *iq, int fmt, int n, int n_frames, const float *twiddles, float *spectra,
                           float *scratch, hipStream_t stream, bool beside_ssb, int n_cus, bool beside_wide_stats) {
    if (n_frames <= 0) return hipSuccess;
    if (!pow2_kernels(n)) return launch_spectrum_any(any_plan(n), iq, fmt, n_frames, twiddles, spectra, scratch, stream);
    switch (n) {
    case 32768:
        return launch_four_step_fmt<7, 8>(iq, fmt, n_frames, twiddles, spectra, scratch, spectrum_wave_frames(n), stream,
                                          !beside_wide_stats, !beside_ssb);
    case 65536:
        return launch_four_step_fmt<8, 8>(iq, fmt, n_frames, twiddles, spectra, scratch, spectrum_wave_frames(n), stream,
                                          !beside_wide_stats, !beside_ssb);
    case 16384: return k16::launch_fmt(iq, fmt, n_frames, twiddles + spectrum_k16_tables_offset(), spectra, stream,
                                      beside_ssb ? 1 : 2, n_cus);
    case 64: return launch_n<6>(iq, fmt, n_frames, twiddles, spectra, stream);
    case 128: return launch_n<7>(iq, fmt, n_frames, twiddles, spectra, stream);
    case 256: return launch_n<8>(iq, fmt, n_frames, twiddles, spectra, stream);
    case 512: return launch_n<9>(iq, fmt, n_frames, twiddles, spectra, stream);
    case 1024: return launch_n<10>(iq, fmt, n_frames, twiddles, spectra, stream);
    case 2048: return launch_n<11>(iq, fmt, n_frames, twiddles, spectra, stream);
    case 4096: return launch_n<12>(iq, fmt, n_frames, twiddles, spectra, stream);
    case 8192: return launch_n<13>(iq, fmt, n_frames, twiddles, spectra, stream);
    default: return hipErrorInvalidValue;
    }
}

}  // namespace sdrg

// ssb_common.h — raw-IQ unpack, the NCO mix and LDS helpers shared by the SSB kernels (ssb.hip: the 16-stream
// pipeline and the lane-per-stream kernels).  Unpack conventions as
// include/sdrg.h: CS8 v/128, CU8 (v - 127.4)/128, CS16 v/32768, CF32 as is.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sdrg_types.h"

#pragma clang fp contract(off)

namespace sdrg {
namespace {

__device__ __forceinline__ float clamp_ref(float v, float lo, float hi) {  // std::clamp
    return (v < lo) ? lo : (hi < v) ? hi : v;
}

// Real parts (I) of 8 consecutive samples starting at sample n of a frame (n multiple of 8, all in range).
template <int FMT>
__device__ __forceinline__ void load_i8(const char *frame, int n, float (&x)[8]) {
    if constexpr (FMT == SDRG_IQ_CS8 || FMT == SDRG_IQ_CU8) {
        const uint4 v = *reinterpret_cast<const uint4 *>(frame + 2 * (size_t)n);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int q = 0; q < 4; q++) {
            if constexpr (FMT == SDRG_IQ_CS8) {
                x[2 * q] = (float)(int8_t)(w[q] & 0xff) * (1.0f / 128.0f);
                x[2 * q + 1] = (float)(int8_t)((w[q] >> 16) & 0xff) * (1.0f / 128.0f);
            } else {
                x[2 * q] = ((float)(w[q] & 0xff) - 127.4f) * (1.0f / 128.0f);
                x[2 * q + 1] = ((float)((w[q] >> 16) & 0xff) - 127.4f) * (1.0f / 128.0f);
            }
        }
    } else if constexpr (FMT == SDRG_IQ_CS16) {
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const uint4 v = *reinterpret_cast<const uint4 *>(frame + 4 * (size_t)(n + 4 * h));
            const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int q = 0; q < 4; q++) x[4 * h + q] = (float)(int16_t)(w[q] & 0xffff) * (1.0f / 32768.0f);
        }
    } else {
#pragma unroll
        for (int h = 0; h < 4; h++) {
            const float4 v = *reinterpret_cast<const float4 *>(frame + 8 * (size_t)(n + 2 * h));
            x[2 * h] = v.x;
            x[2 * h + 1] = v.z;
        }
    }
}

// I parts of 8 consecutive samples held in raw form in u[] (1, 2 or 4 uint4 by format).
// The integer formats' scale (and CU8's offset) run on sample pairs: one packed op per two samples, each lane
// rounding as the scalar expression of load_i8 / load_i1.
template <int FMT>
__device__ __forceinline__ void scale_pair(float a, float b, float &xa, float &xb) {
    typedef float f2_t __attribute__((ext_vector_type(2)));
    f2_t v = f2_t{a, b};
    if constexpr (FMT == SDRG_IQ_CU8) v = v - f2_t{127.4f, 127.4f};
    v = v * (FMT == SDRG_IQ_CS16 ? f2_t{1.0f / 32768.0f, 1.0f / 32768.0f} : f2_t{1.0f / 128.0f, 1.0f / 128.0f});
    xa = v.x;
    xb = v.y;
}

template <int FMT>
__device__ __forceinline__ void unpack_i8(const uint4 *u, float (&x)[8]) {
    if constexpr (FMT == SDRG_IQ_CS8 || FMT == SDRG_IQ_CU8) {
        const uint32_t w[4] = {u[0].x, u[0].y, u[0].z, u[0].w};
#pragma unroll
        for (int q = 0; q < 4; q++) {
            if constexpr (FMT == SDRG_IQ_CS8)
                scale_pair<FMT>((float)(int8_t)(w[q] & 0xff), (float)(int8_t)((w[q] >> 16) & 0xff), x[2 * q], x[2 * q + 1]);
            else
                scale_pair<FMT>((float)(w[q] & 0xff), (float)((w[q] >> 16) & 0xff), x[2 * q], x[2 * q + 1]);
        }
    } else if constexpr (FMT == SDRG_IQ_CS16) {
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const uint32_t w[4] = {u[h].x, u[h].y, u[h].z, u[h].w};
#pragma unroll
            for (int q = 0; q < 4; q += 2)
                scale_pair<FMT>((float)(int16_t)(w[q] & 0xffff), (float)(int16_t)(w[q + 1] & 0xffff), x[4 * h + q],
                                x[4 * h + q + 1]);
        }
    } else {
#pragma unroll
        for (int h = 0; h < 4; h++) {
            x[2 * h] = __uint_as_float(u[h].x);
            x[2 * h + 1] = __uint_as_float(u[h].z);
        }
    }
}

// Q parts of 8 consecutive samples held in raw form in u[] (the NCO variant's loader).
template <int FMT>
__device__ __forceinline__ void unpack_q8(const uint4 *u, float (&x)[8]) {
    if constexpr (FMT == SDRG_IQ_CS8 || FMT == SDRG_IQ_CU8) {
        const uint32_t w[4] = {u[0].x, u[0].y, u[0].z, u[0].w};
#pragma unroll
        for (int q = 0; q < 4; q++) {
            if constexpr (FMT == SDRG_IQ_CS8)
                scale_pair<FMT>((float)(int8_t)((w[q] >> 8) & 0xff), (float)(int8_t)(w[q] >> 24), x[2 * q], x[2 * q + 1]);
            else
                scale_pair<FMT>((float)((w[q] >> 8) & 0xff), (float)(w[q] >> 24), x[2 * q], x[2 * q + 1]);
        }
    } else if constexpr (FMT == SDRG_IQ_CS16) {
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const uint32_t w[4] = {u[h].x, u[h].y, u[h].z, u[h].w};
#pragma unroll
            for (int q = 0; q < 4; q += 2)
                scale_pair<FMT>((float)(int16_t)(w[q] >> 16), (float)(int16_t)(w[q + 1] >> 16), x[4 * h + q], x[4 * h + q + 1]);
        }
    } else {
#pragma unroll
        for (int h = 0; h < 4; h++) {
            x[2 * h] = __uint_as_float(u[h].y);
            x[2 * h + 1] = __uint_as_float(u[h].w);
        }
    }
}

template <int FMT>
__device__ __forceinline__ float load_i1(const char *frame, int n) {
    if constexpr (FMT == SDRG_IQ_CS8) return (float)(int8_t)frame[2 * (size_t)n] * (1.0f / 128.0f);
    else if constexpr (FMT == SDRG_IQ_CU8) return ((float)(uint8_t)frame[2 * (size_t)n] - 127.4f) * (1.0f / 128.0f);
    else if constexpr (FMT == SDRG_IQ_CS16)
        return (float)reinterpret_cast<const int16_t *>(frame)[2 * (size_t)n] * (1.0f / 32768.0f);
    else return reinterpret_cast<const float *>(frame)[2 * (size_t)n];
}

// Imaginary part (Q) of sample n, same unpack conventions as load_i1.
template <int FMT>
__device__ __forceinline__ float load_q1(const char *frame, int n) {
    if constexpr (FMT == SDRG_IQ_CS8) return (float)(int8_t)frame[2 * (size_t)n + 1] * (1.0f / 128.0f);
    else if constexpr (FMT == SDRG_IQ_CU8) return ((float)(uint8_t)frame[2 * (size_t)n + 1] - 127.4f) * (1.0f / 128.0f);
    else if constexpr (FMT == SDRG_IQ_CS16)
        return (float)reinterpret_cast<const int16_t *>(frame)[2 * (size_t)n + 1] * (1.0f / 32768.0f);
    else return reinterpret_cast<const float *>(frame)[2 * (size_t)n + 1];
}

// NCO variant: Re((xr + j xi) * w), w = e^{-j 2 pi ph / 2^32} = hi[ph >> 22] * lo[(ph >> 12) & 1023] with the
// tables of design.cpp nco_tables (tab = hi then lo, {re, im}); complex products in this fixed order,
// no contraction, so the CPU restatement (oracle/sdrg_oracle.c oracle_nco_mix) rounds identically.
__device__ __forceinline__ float nco_mix(const float *tab, uint32_t ph, float xr, float xi) {
    const float2 h = reinterpret_cast<const float2 *>(tab)[ph >> 22];
    const float2 l = reinterpret_cast<const float2 *>(tab)[1024 + ((ph >> 12) & 1023)];
    const float wr = h.x * l.x - h.y * l.y;
    const float wi = h.x * l.y + h.y * l.x;
    return xr * wr - xi * wi;
}

template <int FMT>
constexpr int bytes_per_sample() {
    return FMT == SDRG_IQ_CF32 ? 8 : FMT == SDRG_IQ_CS16 ? 4 : 2;
}

// LDS byte address of a pointer into the workgroup's LDS (for asm operands)
__device__ __forceinline__ uint32_t lds_addr(const float *p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) float *)p;
}

// Workgroup barrier that orders LDS only.  __syncthreads() is a workgroup release/acquire, which makes
// every wave drain ALL its outstanding memory operations (s_waitcnt vmcnt(0)) first - the loader's
// raw-IQ prefetch would then complete every chunk instead of several chunks ahead, and the pipeline
// would pay an HBM round trip per chunk.  Nothing global is exchanged between waves inside the loop.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

}  // namespace
}  // namespace sdrg

// gather.hip — the HBM streaming-copy probe (bench.py hbm_measured) and packing for the multi-GPU gather (dist.cpp, engine.cpp sdrg_engine_gather): each stream's
// focus-window slice of the fftshifted spectrum (the bins evaluateSignalStrength's focus window reads,
// src/dsp/fft_process.cpp:124-140) copied into a contiguous [stream][bin] block, so one ncclGather moves only
// the bins a consumer on the root rank looks at (81 of 16384 at 2 MHz / +-5 kHz) instead of the whole spectrum.
#include <algorithm>

#include "sdrg_internal.h"

namespace sdrg {
namespace {

// one workgroup of 256 threads per 4 streams (64 threads per row); nb <= a few thousand bins at most
__global__ __launch_bounds__(256) void focus_pack_kernel(const float *__restrict__ spectra, int n_streams, int n, int lo,
                                                         int nb, float *__restrict__ out) {
    const int s = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (s >= n_streams) return;
    const float *src = spectra + (size_t)s * n + lo;
    float *dst = out + (size_t)s * nb;
    for (int j = threadIdx.x & 63; j < nb; j += 64) dst[j] = src[j];
}

// The HBM bandwidth probe behind bench.py's hbm_measured (MI355X_MICROARCH.md: a float4 streaming copy measures 6.29 TB/s,
// a hipMemcpy D2D less): every thread moves UNROLL float4 per grid-stride step with nontemporal loads and stores, so
// the achievable read + write rate of a plain streaming pattern, not the copy engine's, is the roofline's basis.
constexpr int COPY_UNROLL = 4;
typedef float copy_v4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void stream_copy_kernel(const copy_v4 *__restrict__ src, copy_v4 *__restrict__ dst,
                                                          size_t n4) {
    const size_t stride = (size_t)gridDim.x * blockDim.x * COPY_UNROLL;
    for (size_t i = (size_t)blockIdx.x * blockDim.x * COPY_UNROLL + threadIdx.x; i < n4; i += stride) {
        copy_v4 v[COPY_UNROLL];
#pragma unroll
        for (int u = 0; u < COPY_UNROLL; u++) {
            const size_t j = i + (size_t)u * blockDim.x;
            if (j < n4) v[u] = __builtin_nontemporal_load(src + j);
        }
#pragma unroll
        for (int u = 0; u < COPY_UNROLL; u++) {
            const size_t j = i + (size_t)u * blockDim.x;
            if (j < n4) __builtin_nontemporal_store(v[u], dst + j);
        }
    }
}

}  // namespace

hipError_t measure_stream_copy(size_t bytes, int reps, double *gbs) {
    *gbs = 0.0;
    const size_t n4 = bytes / sizeof(float4);
    if (n4 == 0 || reps <= 0) return hipErrorInvalidValue;
    copy_v4 *a = nullptr, *b = nullptr;
    hipEvent_t t0 = nullptr, t1 = nullptr;
    hipError_t e = hipMalloc(reinterpret_cast<void **>(&a), n4 * sizeof(float4));
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void **>(&b), n4 * sizeof(float4));
    if (e == hipSuccess) e = hipMemset(a, 0, n4 * sizeof(float4));
    if (e == hipSuccess) e = hipEventCreate(&t0);
    if (e == hipSuccess) e = hipEventCreate(&t1);
    hipStream_t s = nullptr;
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    if (e == hipSuccess) {
        // 16 workgroups of 256 threads per CU (256 CUs), fewer when the buffer is small
        const size_t per_block = (size_t)256 * COPY_UNROLL;
        const unsigned grid = (unsigned)std::min<size_t>((n4 + per_block - 1) / per_block, (size_t)256 * 16);
        hipLaunchKernelGGL(stream_copy_kernel, dim3(grid), dim3(256), 0, s, a, b, n4);  // untimed first launch
        e = hipEventRecord(t0, s);
        for (int r = 0; r < reps && e == hipSuccess; r++)
            hipLaunchKernelGGL(stream_copy_kernel, dim3(grid), dim3(256), 0, s, a, b, n4);
        if (e == hipSuccess) e = hipGetLastError();
        if (e == hipSuccess) e = hipEventRecord(t1, s);
        if (e == hipSuccess) e = hipEventSynchronize(t1);
        float ms = 0.0f;
        if (e == hipSuccess) e = hipEventElapsedTime(&ms, t0, t1);
        if (e == hipSuccess && ms > 0.0f) *gbs = 2.0 * (double)(n4 * sizeof(float4)) * reps / (ms * 1e-3) / 1e9;
    }
    if (s) (void)hipStreamDestroy(s);
    if (t0) (void)hipEventDestroy(t0);
    if (t1) (void)hipEventDestroy(t1);
    if (a) (void)hipFree(a);
    if (b) (void)hipFree(b);
    return e;
}

hipError_t launch_focus_pack(const float *spectra, int n_streams, int n, int lo, int nb, float *out, hipStream_t stream) {
    if (n_streams <= 0 || nb <= 0) return hipSuccess;
    if (lo < 0 || lo + nb > n) return hipErrorInvalidValue;
    hipLaunchKernelGGL(focus_pack_kernel, dim3((n_streams + 3) / 4), dim3(256), 0, stream, spectra, n_streams, n, lo, nb,
                       out);
    return hipGetLastError();
}

}  // namespace sdrg

// gather.hip — packing for the multi-GPU gather (dist.cpp, engine.cpp sdrg_engine_gather): each stream's
// focus-window slice of the fftshifted spectrum (the bins evaluateSignalStrength's focus window reads,
// src/dsp/fft_process.cpp:124-140) copied into a contiguous [stream][bin] block, so one ncclGather moves only
// the bins a consumer on the root rank looks at (81 of 16384 at 2 MHz / +-5 kHz) instead of the whole spectrum.
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

}  // namespace

hipError_t launch_focus_pack(const float *spectra, int n_streams, int n, int lo, int nb, float *out, hipStream_t stream) {
    if (n_streams <= 0 || nb <= 0) return hipSuccess;
    if (lo < 0 || lo + nb > n) return hipErrorInvalidValue;
    hipLaunchKernelGGL(focus_pack_kernel, dim3((n_streams + 3) / 4), dim3(256), 0, stream, spectra, n_streams, n, lo, nb,
                       out);
    return hipGetLastError();
}

}  // namespace sdrg

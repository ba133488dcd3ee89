// Lab: calibrate rocprofv3 FETCH_SIZE for the statistics kernel's access pattern on gfx950.
// (1) stream1: 1 GiB read as 4 B per lane; (2) stream16: 1 GiB read as 16 B per lane;
// (3) windows: the c2 statistics windows (11 runs of 81-82 floats per 16384-float frame, 4096 frames, dword
//     loads, exactly 4096 x 901 x 4 B) from a cold 256 MiB spectra array (a 1 GiB write evicts it first).
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void stream1(const float *p, size_t n, float *out) {
    float s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += p[i];
    if (s == 1.2345f) out[0] = s;
}
__global__ void stream16(const float4 *p, size_t n4, float *out) {
    float s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
        const float4 v = p[i];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 1.2345f) out[0] = s;
}
__global__ void fill(float *p, size_t n, float v) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = v;
}
__constant__ int c_lo[11], c_len[11];
__global__ void windows(const float *spec, float *out) {
    const float *P = spec + (size_t)blockIdx.x * 16384;
    float s = 0;
    for (int q = 0; q < 11; q++)
        for (int i = threadIdx.x; i < c_len[q]; i += 64) s += P[c_lo[q] + i];
    if (s == 1.2345f) out[blockIdx.x] = s;
}
int main() {
    const size_t G = (size_t)1 << 28;  // floats: 1 GiB
    float *a, *b, *o;
    if (hipMalloc(&a, G * 4) || hipMalloc(&b, G * 4) || hipMalloc(&o, 1 << 20)) return 1;
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, a, G, 1.0f);
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, b, G, 2.0f);  // evicts a
    hipLaunchKernelGGL(stream1, dim3(4096), dim3(256), 0, 0, a, G, o);
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, b, G, 3.0f);
    hipLaunchKernelGGL(stream16, dim3(4096), dim3(256), 0, 0, reinterpret_cast<const float4 *>(a), G / 4, o);
    // c2 geometry (tests/golden/geometry.json): focus [8151, 8231], reference windows of 82 bins
    const int lo[11] = {8273, 8028, 8437, 7864, 8601, 7700, 8765, 7536, 8929, 7372, 8151};
    int len[11];
    for (int q = 0; q < 10; q++) len[q] = 82;
    len[10] = 81;
    hipMemcpyToSymbol(HIP_SYMBOL(c_lo), lo, sizeof(lo));
    hipMemcpyToSymbol(HIP_SYMBOL(c_len), len, sizeof(len));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, b, G, 4.0f);  // a's first 256 MiB evicted
    hipLaunchKernelGGL(windows, dim3(4096), dim3(64), 0, 0, a, o);
    if (hipDeviceSynchronize()) return 2;
    int tot = 0;
    for (int q = 0; q < 11; q++) tot += len[q];
    printf("stream1 %.1f MB, stream16 %.1f MB, windows %.2f MB (algorithmic)\n", G * 4 / 1e6, G * 4 / 1e6, 4096.0 * tot * 4 / 1e6);
    return 0;
}

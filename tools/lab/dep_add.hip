// Lab: cycles per dependent v_add_f32 for one wave, and with independent chains / co-resident waves.
#include <hip/hip_runtime.h>
#include <stdio.h>
template <int CH>
__global__ void chain(float *out, unsigned long long *cyc, int n, float d) {
    float a[CH];
#pragma unroll
    for (int c = 0; c < CH; c++) a[c] = threadIdx.x * 0.001f + c;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; i++) {
#pragma unroll
        for (int u = 0; u < 16; u++)
#pragma unroll
            for (int c = 0; c < CH; c++) a[c] += d;
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0;
#pragma unroll
    for (int c = 0; c < CH; c++) s += a[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x % 64 == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}
template <int CH>
void run(int blocks, int threads) {
    const int n = 4096;
    float *o; unsigned long long *c;
    hipMalloc(&o, blocks * threads * 4); hipMalloc(&c, blocks * threads / 64 * 8);
    hipLaunchKernelGGL(chain<CH>, dim3(blocks), dim3(threads), 0, 0, o, c, n, 1e-7f);
    hipDeviceSynchronize();
    hipLaunchKernelGGL(chain<CH>, dim3(blocks), dim3(threads), 0, 0, o, c, n, 1e-7f);
    hipDeviceSynchronize();
    unsigned long long h[4096];
    int nw = blocks * threads / 64; if (nw > 4096) nw = 4096;
    hipMemcpy(h, c, nw * 8, hipMemcpyDeviceToHost);
    double m = 0; for (int i = 0; i < nw; i++) m += h[i]; m /= nw;
    printf("chains/lane %d, %5d blocks x %4d threads: %.2f cycles per dependent step (%.2f per add instr)\n", CH, blocks,
           threads, m / (n * 16.0), m / (n * 16.0 * CH));
    hipFree(o); hipFree(c);
}
int main() {
    run<1>(1, 64); run<2>(1, 64); run<4>(1, 64); run<8>(1, 64);
    run<1>(1, 256); run<1>(1, 1024); run<1>(256, 256); run<1>(1024, 256); run<4>(1024, 256);
    return 0;
}

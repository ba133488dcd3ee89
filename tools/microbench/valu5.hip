// valu5.hip — per-sample latency of the SSB recurrences' instruction chains (one wave alone on its SIMD),
// with all 64 lanes active vs 16 (the pipeline's lane = stream layout of 16 streams per workgroup).
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f2v __attribute__((ext_vector_type(2)));

#pragma clang fp contract(off)

template <int MODE>
__device__ __forceinline__ float step(float z1, float &z2, float x, f2v c1, f2v c2, f2v keep, f2v rates) {
    if constexpr (MODE == 0) {  // LPF as in the pipeline: (((x + a1 z1) + a2 z2) - b1 z1) - b2 z2
        const f2v p1 = c1 * z1, p2 = c2 * z2;
        const float y = (((x + p1.x) + p2.x) - p1.y) - p2.y;
        z2 = z1;
        return y;
    } else if constexpr (MODE == 1) {  // LPF with negated b (all adds): c1 = {a1, -b1}, c2 = {a2, -b2}
        const f2v p1 = c1 * z1, p2 = c2 * z2;
        const float y = (((x + p1.x) + p2.x) + p1.y) + p2.y;
        z2 = z1;
        return y;
    } else if constexpr (MODE == 2) {  // LPF, scalar products
        const float y = (((x + c1.x * z1) + c2.x * z2) + c1.y * z1) + c2.y * z2;
        z2 = z1;
        return y;
    } else {  // AGC gain: cand = gain*keep + d*rates ; gain = d < gain ? cand.x : cand.y   (z1 = gain, x = d)
        const f2v cand = z1 * keep + x * rates;
        return (x < z1) ? cand.x : cand.y;
    }
}

template <int MODE>
__global__ void k(unsigned long long *out, const float *xs, int active) {
    float z1 = 0.1f, z2 = 0.2f;
    const f2v c1 = {1.99f, -0.9901f}, c2 = {-0.99f, 0.0001f}, keep = {0.994f, 0.99965f}, rates = {0.006f, 0.00035f};
    __syncthreads();
    unsigned long long dt = 0;
    if ((int)threadIdx.x < active) {
        float x[32];
        for (int i = 0; i < 32; i++) x[i] = xs[i + threadIdx.x];
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();
        for (int it = 0; it < 64; it++) {
#pragma unroll
            for (int i = 0; i < 32; i++) z1 = step<MODE>(z1, z2, x[i], c1, c2, keep, rates);
        }
        dt = __builtin_amdgcn_s_memtime() - t0;
    }
    if (threadIdx.x == 0) out[0] = dt;
    if (z1 == 12345.f) out[9] = 1;
}

template <int MODE>
void run(const char *name, unsigned long long *d, const float *xs, int active) {
    unsigned long long h[10];
    for (int r = 0; r < 3; r++) k<MODE><<<1, 64>>>(d, xs, active);
    if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return;
    printf("%-34s active %2d lanes: %6.2f cyc/sample\n", name, active, h[0] / (64.0 * 32));
}

int main() {
    unsigned long long *d;
    float *xs;
    if (hipMalloc(&d, 10 * sizeof(unsigned long long)) != hipSuccess || hipMalloc(&xs, 256 * 4) != hipSuccess) return 2;
    float h[256];
    for (int i = 0; i < 256; i++) h[i] = 0.01f * (i % 17) - 0.05f;
    if (hipMemcpy(xs, h, sizeof h, hipMemcpyHostToDevice) != hipSuccess) return 2;
    for (int act : {64, 16}) {
        run<0>("LPF sub (pipeline)", d, xs, act);
        run<1>("LPF add of negated products", d, xs, act);
        run<2>("LPF scalar products", d, xs, act);
        run<3>("AGC gain", d, xs, act);
    }
    return 0;
}

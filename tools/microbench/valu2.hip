// valu2.hip — how two waves share one SIMD: a workgroup of 8 waves (2 per SIMD); waves 0-3 run body A,
// waves 4-7 run body B (wave w and w+4 are expected on the same SIMD).  Prints per-wave cycles per instr.
#include <hip/hip_runtime.h>
#include <stdio.h>

#define R8(x) x x x x x x x x
#define R32(x) R8(x) R8(x) R8(x) R8(x)

template <int MODE>
__device__ void body(float &a, float &b, float &c, float &e, float &g) {
    if constexpr (MODE == 0) {  // dependent v_add chain
        R32(asm volatile("v_add_f32 %0, %0, %1" : "+v"(a) : "v"(b));)
    } else if constexpr (MODE == 1) {  // 4 independent streams
        R8(asm volatile("v_add_f32 %0, %0, %4\n v_add_f32 %1, %1, %4\n v_add_f32 %2, %2, %4\n v_add_f32 %3, %3, %4" : "+v"(a), "+v"(c), "+v"(e), "+v"(g) : "v"(b));)
    } else if constexpr (MODE == 2) {  // idle (s_sleep)
        R8(asm volatile("s_sleep 1");)
    } else if constexpr (MODE == 3) {  // 2 interleaved dependent chains
        R8(asm volatile("v_add_f32 %0, %0, %2\n v_add_f32 %1, %1, %2\n v_add_f32 %0, %0, %2\n v_add_f32 %1, %1, %2" : "+v"(a), "+v"(c) : "v"(b));)
    }
}

template <int A, int B>
__global__ void k(unsigned long long *out, float seed) {
    float a = seed, b = seed * 0.5f, c = seed * 0.25f, e = seed + 1, g = seed + 2;
    const int w = threadIdx.x >> 6;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < 512; i++) {
        if (w < 4) body<A>(a, b, c, e, g); else body<B>(a, b, c, e, g);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) out[w] = t1 - t0;
    if (a + c + e + g == 12345.f) out[9] = 1;
}

template <int A, int B>
void run(const char *name, unsigned long long *d) {
    unsigned long long h[10];
    k<A, B><<<1, 512>>>(d, 1.0f);
    k<A, B><<<1, 512>>>(d, 1.0f);
    if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return;
    printf("%-40s A(w0) %6.2f  B(w4) %6.2f cyc/instr\n", name, h[0] / (512.0 * 32), h[4] / (512.0 * 32));
}

int main() {
    unsigned long long *d;
    if (hipMalloc(&d, 10 * sizeof(unsigned long long)) != hipSuccess) return 2;
    run<0, 2>("dep | idle", d);
    run<0, 0>("dep | dep", d);
    run<0, 1>("dep | 4 indep", d);
    run<1, 1>("4 indep | 4 indep", d);
    run<1, 2>("4 indep | idle", d);
    run<3, 2>("2 interleaved dep | idle", d);
    run<3, 3>("2 interleaved dep | 2 interleaved dep", d);
    return 0;
}

// valu3.hip — dependent-chain latency of one wave alone on its SIMD, by EXEC width and instruction form.
// One workgroup of 64 threads; cycles per dependent instruction from s_memtime (= shader cycles).
#include <hip/hip_runtime.h>
#include <stdio.h>

#define R8(x) x x x x x x x x
#define R32(x) R8(x) R8(x) R8(x) R8(x)

template <int MODE>
__device__ __forceinline__ void body(float &a, float b) {
    if constexpr (MODE == 0) {  // dependent v_add_f32
        R32(asm volatile("v_add_f32 %0, %0, %1" : "+v"(a) : "v"(b));)
    } else if constexpr (MODE == 1) {  // dependent v_mul_f32
        R32(asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a) : "v"(b));)
    } else if constexpr (MODE == 2) {  // dependent v_add_f32 e64 (VOP3)
        R32(asm volatile("v_add_f32_e64 %0, %0, %1" : "+v"(a) : "v"(b));)
    } else if constexpr (MODE == 3) {  // dependent v_sub_f32
        R32(asm volatile("v_sub_f32 %0, %0, %1" : "+v"(a) : "v"(b));)
    } else if constexpr (MODE == 4) {  // dependent v_pk_add_f32 (both halves)
        R32(asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(*(double *)&a) : "v"(0.0));)
    } else if constexpr (MODE == 5) {  // dependent v_fma_f32
        R32(asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(a) : "v"(b));)
    } else if constexpr (MODE == 6) {  // dependent v_med3_f32
        R32(asm volatile("v_med3_f32 %0, %0, %1, 1.0" : "+v"(a) : "v"(b));)
    } else if constexpr (MODE == 7) {  // dependent v_cndmask via compare (2 instr per step)
        R32(asm volatile("v_cmp_lt_f32 vcc, %0, %1\n v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a) : "v"(b) : "vcc");)
    }
}

template <int MODE>
__global__ void k(unsigned long long *out, float seed, int active) {
    float a = seed, b = seed * 0.5f;
    __syncthreads();
    unsigned long long dt = 0;
    if ((int)threadIdx.x < active) {
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();
        for (int i = 0; i < 256; i++) body<MODE>(a, b);
        dt = __builtin_amdgcn_s_memtime() - t0;
    }
    if (threadIdx.x == 0) out[0] = dt;
    if (a == 12345.f) out[9] = 1;
}

template <int MODE>
void run(const char *name, unsigned long long *d, int active) {
    unsigned long long h[10];
    const int per = MODE == 7 ? 64 : 32;
    for (int r = 0; r < 3; r++) k<MODE><<<1, 64>>>(d, 1.0f, active);
    if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return;
    printf("%-28s active %2d lanes: %6.2f cyc/instr\n", name, active, h[0] / (256.0 * per));
}

int main() {
    unsigned long long *d;
    if (hipMalloc(&d, 10 * sizeof(unsigned long long)) != hipSuccess) return 2;
    for (int act : {64, 32, 16, 1}) {
        run<0>("v_add_f32 dep", d, act);
        run<1>("v_mul_f32 dep", d, act);
        run<2>("v_add_f32_e64 dep", d, act);
        run<3>("v_sub_f32 dep", d, act);
        run<4>("v_pk_add_f32 dep", d, act);
        run<5>("v_fma_f32 dep", d, act);
        run<6>("v_med3_f32 dep", d, act);
        run<7>("v_cmp+v_cndmask dep", d, act);
    }
    return 0;
}

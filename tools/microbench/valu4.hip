// valu4.hip — VALU THROUGHPUT per SIMD (independent instructions, W waves per SIMD): scalar vs packed f32.
// One workgroup of 4*W waves (W per SIMD); cycles per wave-instruction per SIMD from s_memtime.
#include <hip/hip_runtime.h>
#include <stdio.h>

#define R8(x) x x x x x x x x

template <int MODE>
__device__ __forceinline__ void body(float (&a)[8], float b) {
    if constexpr (MODE == 0) {  // 8 independent v_add_f32
        R8(asm volatile("v_add_f32 %0, %0, %8\n v_add_f32 %1, %1, %8\n v_add_f32 %2, %2, %8\n v_add_f32 %3, %3, %8\n"
                        "v_add_f32 %4, %4, %8\n v_add_f32 %5, %5, %8\n v_add_f32 %6, %6, %8\n v_add_f32 %7, %7, %8"
                        : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]) : "v"(b));)
    } else if constexpr (MODE == 1) {  // 8 independent v_fma_f32
        R8(asm volatile("v_fma_f32 %0, %0, %8, %8\n v_fma_f32 %1, %1, %8, %8\n v_fma_f32 %2, %2, %8, %8\n v_fma_f32 %3, %3, %8, %8\n"
                        "v_fma_f32 %4, %4, %8, %8\n v_fma_f32 %5, %5, %8, %8\n v_fma_f32 %6, %6, %8, %8\n v_fma_f32 %7, %7, %8, %8"
                        : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]) : "v"(b));)
    } else if constexpr (MODE == 2) {  // 4 independent v_pk_add_f32 (= 8 scalar adds)
        double *d = reinterpret_cast<double *>(a);
        R8(asm volatile("v_pk_add_f32 %0, %0, %4\n v_pk_add_f32 %1, %1, %4\n v_pk_add_f32 %2, %2, %4\n v_pk_add_f32 %3, %3, %4"
                        : "+v"(d[0]), "+v"(d[1]), "+v"(d[2]), "+v"(d[3]) : "v"(0.5));)
    } else if constexpr (MODE == 3) {  // 4 independent v_pk_fma_f32 (= 8 scalar fma)
        double *d = reinterpret_cast<double *>(a);
        R8(asm volatile("v_pk_fma_f32 %0, %0, %4, %4\n v_pk_fma_f32 %1, %1, %4, %4\n v_pk_fma_f32 %2, %2, %4, %4\n v_pk_fma_f32 %3, %3, %4, %4"
                        : "+v"(d[0]), "+v"(d[1]), "+v"(d[2]), "+v"(d[3]) : "v"(0.5));)
    } else if constexpr (MODE == 4) {  // 8 independent v_cvt_f32_i32 sdwa byte sext
        R8(asm volatile("v_cvt_f32_i32_sdwa %0, %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1\n v_cvt_f32_i32_sdwa %1, %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1\n"
                        "v_cvt_f32_i32_sdwa %2, %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1\n v_cvt_f32_i32_sdwa %3, %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1\n"
                        "v_cvt_f32_i32_sdwa %4, %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1\n v_cvt_f32_i32_sdwa %5, %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1\n"
                        "v_cvt_f32_i32_sdwa %6, %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1\n v_cvt_f32_i32_sdwa %7, %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1"
                        : "=v"(a[0]), "=v"(a[1]), "=v"(a[2]), "=v"(a[3]), "=v"(a[4]), "=v"(a[5]), "=v"(a[6]), "=v"(a[7]) : "v"(b));)
    } else if constexpr (MODE == 5) {  // 8 independent v_mov_b32
        R8(asm volatile("v_mov_b32 %0, %8\n v_mov_b32 %1, %8\n v_mov_b32 %2, %8\n v_mov_b32 %3, %8\n"
                        "v_mov_b32 %4, %8\n v_mov_b32 %5, %8\n v_mov_b32 %6, %8\n v_mov_b32 %7, %8"
                        : "=v"(a[0]), "=v"(a[1]), "=v"(a[2]), "=v"(a[3]), "=v"(a[4]), "=v"(a[5]), "=v"(a[6]), "=v"(a[7]) : "v"(b));)
    } else if constexpr (MODE == 6) {  // 4 independent v_pk_mul_f32
        double *d = reinterpret_cast<double *>(a);
        R8(asm volatile("v_pk_mul_f32 %0, %0, %4\n v_pk_mul_f32 %1, %1, %4\n v_pk_mul_f32 %2, %2, %4\n v_pk_mul_f32 %3, %3, %4"
                        : "+v"(d[0]), "+v"(d[1]), "+v"(d[2]), "+v"(d[3]) : "v"(0.5));)
    }
}

template <int MODE>
__global__ void k(unsigned long long *out, float seed) {
    float a[8];
    for (int i = 0; i < 8; i++) a[i] = seed + i;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < 128; i++) body<MODE>(a, seed);
    __syncthreads();
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) out[0] = t1 - t0;
    float s = 0;
    for (int i = 0; i < 8; i++) s += a[i];
    if (s == 12345.f) out[9] = 1;
}

template <int MODE>
void run(const char *name, unsigned long long *d, int wps) {
    unsigned long long h[10];
    const int instr = (MODE == 2 || MODE == 3 || MODE == 6) ? 32 : 64;  // wave-instructions per iteration
    for (int r = 0; r < 3; r++) k<MODE><<<1, 256 * wps>>>(d, 1.0f);
    if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return;
    const double per_simd = (double)instr * 128 * wps;  // wave-instructions per SIMD
    printf("%-22s waves/SIMD %d: %6.2f cyc per wave-instr per SIMD\n", name, wps, h[0] / per_simd);
}

int main() {
    unsigned long long *d;
    if (hipMalloc(&d, 10 * sizeof(unsigned long long)) != hipSuccess) return 2;
    for (int w : {1, 2, 4}) {
        run<0>("v_add_f32", d, w);
        run<1>("v_fma_f32", d, w);
        run<2>("v_pk_add_f32", d, w);
        run<3>("v_pk_fma_f32", d, w);
        run<6>("v_pk_mul_f32", d, w);
        run<4>("v_cvt_f32_i32 sdwa", d, w);
        run<5>("v_mov_b32", d, w);
    }
    return 0;
}

// Lab: dependent-chain latency (cycles per instruction of the chain) of the VALU forms the SSB recurrences use,
// one wave alone on the chip (s_memtime cycles).  Build: hipcc --offload-arch=gfx950 -O3 -o tools/lab/lat tools/lab/lat.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f2v __attribute__((ext_vector_type(2)));
constexpr int REP = 2048, U = 16;
__device__ __forceinline__ f2v mk(float x, float y) { f2v r; r.x = x; r.y = y; return r; }

#define CHAIN_KERNEL(NAME, DECL, BODY, OUT)                                              \
    __global__ void NAME(float *out, unsigned long long *cyc, float s) {                \
        DECL;                                                                            \
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();                      \
        for (int i = 0; i < REP; i++) {                                                  \
            _Pragma("unroll") for (int u = 0; u < U; u++) { BODY; }                      \
        }                                                                                \
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();                      \
        out[threadIdx.x] = OUT;                                                          \
        if (threadIdx.x == 0) cyc[0] = t1 - t0;                                          \
    }

CHAIN_KERNEL(k_add, float a = threadIdx.x * 1e-3f; float b = s,
             asm volatile("v_add_f32 %0, %0, %1" : "+v"(a) : "v"(b)), a)
CHAIN_KERNEL(k_mul, float a = threadIdx.x * 1e-3f; float b = s,
             asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a) : "v"(b)), a)
CHAIN_KERNEL(k_fma, float a = threadIdx.x * 1e-3f; float b = s; float c = s,
             asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c)), a)
CHAIN_KERNEL(k_pkmul, f2v a = mk(threadIdx.x * 1e-3f, 1.f); f2v b = mk(s, s),
             asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(a) : "v"(b)), a.x + a.y)
CHAIN_KERNEL(k_pkadd, f2v a = mk(threadIdx.x * 1e-3f, 1.f); f2v b = mk(s, s),
             asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(a) : "v"(b)), a.x + a.y)
// two scalar ops per step (mul then add): the non-packed equivalent
CHAIN_KERNEL(k_mul_then_add, float z = threadIdx.x * 1e-3f; float c = s; float p; float v = s,
             asm volatile("v_mul_f32 %1, %2, %0\n\tv_add_f32 %0, %1, %3" : "+v"(z), "=&v"(p) : "v"(c), "v"(v)), z)
// the AGC's select: compare against the chain value, then cndmask on vcc (2 instructions per step)
CHAIN_KERNEL(k_cmp_cnd, float g = threadIdx.x * 1e-3f; float d = s; float alt = 2 * s,
             asm volatile("v_cmp_lt_f32 vcc, %1, %0\n\tv_cndmask_b32 %0, %2, %0, vcc" : "+v"(g) : "v"(d), "v"(alt) : "vcc"), g)
// cndmask chained through its data operand only (vcc fixed)
CHAIN_KERNEL(k_cnd, float g = threadIdx.x * 1e-3f; float alt = 2 * s,
             asm volatile("v_cndmask_b32 %0, %1, %0, vcc" : "+v"(g) : "v"(alt) : "vcc"), g)
// v_max_f32 chain (a select-free alternative for ordered picks)
CHAIN_KERNEL(k_max, float g = threadIdx.x * 1e-3f; float alt = s,
             asm volatile("v_max_f32 %0, %0, %1" : "+v"(g) : "v"(alt)), g)
// register-reuse probes: the same dependent add chain written in place, ping-ponged between two registers, rotated
// over four, and with the constant operand in an SGPR
CHAIN_KERNEL(k_add_pp, float a = threadIdx.x * 1e-3f; float b = s; float t,
             asm volatile("v_add_f32 %1, %0, %2\n\tv_add_f32 %0, %1, %2" : "+v"(a), "=&v"(t) : "v"(b)), a)
CHAIN_KERNEL(k_add_rot4, float a = threadIdx.x * 1e-3f; float b = s; float r1; float r2; float r3,
             asm volatile("v_add_f32 %1, %0, %4\n\tv_add_f32 %2, %1, %4\n\tv_add_f32 %3, %2, %4\n\tv_add_f32 %0, %3, %4"
                          : "+v"(a), "=&v"(r1), "=&v"(r2), "=&v"(r3) : "v"(b)), a)
CHAIN_KERNEL(k_add_sgpr, float a = threadIdx.x * 1e-3f,
             asm volatile("v_add_f32 %0, %1, %0" : "+v"(a) : "s"(s)), a)
CHAIN_KERNEL(k_add_sgpr_pp, float a = threadIdx.x * 1e-3f; float t,
             asm volatile("v_add_f32 %1, %2, %0\n\tv_add_f32 %0, %2, %1" : "+v"(a), "=&v"(t) : "s"(s)), a)
// the LPF step as the compiler emits it (in-place accumulator) and renamed (a fresh register per add)
CHAIN_KERNEL(k_lpf_inplace, float z = threadIdx.x * 1e-3f; float v = s; float q1 = s; float q2 = s; float q3 = s; float acc,
             asm volatile("v_mul_f32 %1, %2, %0\n\tv_add_f32 %1, %3, %1\n\tv_add_f32 %1, %4, %1\n\tv_add_f32 %1, %5, %1\n\tv_add_f32 %0, %6, %1"
                          : "+v"(z), "=&v"(acc) : "v"(v), "v"(q1), "v"(q2), "v"(q3), "v"(v)), z)
CHAIN_KERNEL(k_lpf_renamed, float z = threadIdx.x * 1e-3f; float v = s; float q1 = s; float q2 = s; float q3 = s; float a1; float a2; float a3; float a4,
             asm volatile("v_mul_f32 %1, %5, %0\n\tv_add_f32 %2, %6, %1\n\tv_add_f32 %3, %7, %2\n\tv_add_f32 %4, %8, %3\n\tv_add_f32 %0, %5, %4"
                          : "+v"(z), "=&v"(a1), "=&v"(a2), "=&v"(a3), "=&v"(a4) : "v"(v), "v"(q1), "v"(q2), "v"(q3)), z)

template <class K>
void run(const char *name, K k, int insts_per_step, int threads) {
    float *o; unsigned long long *c, h = 0;
    hipMalloc(&o, 4096 * 4); hipMalloc(&c, 8);
    for (int w = 0; w < 2; w++) {
        hipLaunchKernelGGL(k, dim3(1), dim3(threads), 0, 0, o, c, 1.0000001f);
        hipDeviceSynchronize();
    }
    hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
    const double steps = (double)REP * U;
    printf("%-16s %4d thr: %6.2f cycles per chain step, %5.2f per instruction\n", name, threads, h / steps,
           h / steps / insts_per_step);
    hipFree(o); hipFree(c);
}
int main() {
    for (int thr : {64, 256}) {
        run("v_add_f32", k_add, 1, thr);
        run("v_mul_f32", k_mul, 1, thr);
        run("v_fma_f32", k_fma, 1, thr);
        run("v_pk_mul_f32", k_pkmul, 1, thr);
        run("v_pk_add_f32", k_pkadd, 1, thr);
        run("mul->add", k_mul_then_add, 2, thr);
        run("cmp->cndmask", k_cmp_cnd, 2, thr);
        run("cndmask", k_cnd, 1, thr);
        run("v_max_f32", k_max, 1, thr);
        run("add ping-pong", k_add_pp, 2, thr);
        run("add rotate-4", k_add_rot4, 4, thr);
        run("add sgpr", k_add_sgpr, 1, thr);
        run("add sgpr pp", k_add_sgpr_pp, 2, thr);
        run("lpf in-place", k_lpf_inplace, 5, thr);
        run("lpf renamed", k_lpf_renamed, 5, thr);
    }
    return 0;
}

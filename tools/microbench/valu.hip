// valu.hip — issue/latency cost of the VALU forms the SSB recurrences use, one wave per CU (s_memtime).
// Prints cycles per instruction for dependent chains and independent streams.
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f2v __attribute__((ext_vector_type(2)));
#define R8(x) x x x x x x x x
#define R32(x) R8(x) R8(x) R8(x) R8(x)

__global__ void bench(unsigned long long *out, float seed) {
    float a = seed, b = seed * 0.5f, c = seed * 0.25f, d = seed * 0.125f;
    float e = a + 1, f = b + 1, g = c + 1, h = d + 1;
    f2v pa = {a, b}, pb = {c, d}, pc = {e, f}, pd = {g, h};
    const int ITER = 256;
    unsigned long long t0, t1;
    int k = 0;
#define TIME(body)                                                   \
    t0 = __builtin_amdgcn_s_memtime();                               \
    for (int i = 0; i < ITER; i++) { body }                          \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");               \
    t1 = __builtin_amdgcn_s_memtime();                               \
    if (threadIdx.x == 0) out[blockIdx.x * 32 + k] = t1 - t0;        \
    k++;
    // 0: dependent v_add_f32
    TIME(R32(asm volatile("v_add_f32 %0, %0, %1" : "+v"(a) : "v"(b));))
    // 1: 4 independent v_add_f32 streams
    TIME(R8(asm volatile("v_add_f32 %0, %0, %4\n v_add_f32 %1, %1, %4\n v_add_f32 %2, %2, %4\n v_add_f32 %3, %3, %4" : "+v"(a), "+v"(c), "+v"(e), "+v"(g) : "v"(b));))
    // 2: dependent v_pk_add_f32
    TIME(R32(asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(pa) : "v"(pb));))
    // 3: 4 independent v_pk_add_f32
    TIME(R8(asm volatile("v_pk_add_f32 %0, %0, %4\n v_pk_add_f32 %1, %1, %4\n v_pk_add_f32 %2, %2, %4\n v_pk_add_f32 %3, %3, %4" : "+v"(pa), "+v"(pc), "+v"(pd), "+v"(pb) : "v"(pb));))
    // 4: dependent v_pk_mul_f32
    TIME(R32(asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(pa) : "v"(pb));))
    // 5: dependent v_mul_f32
    TIME(R32(asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a) : "v"(b));))
    // 6: v_cmp + v_cndmask (vcc) dependent, with the required s_nop
    TIME(R32(asm volatile("v_cmp_lt_f32 vcc, %0, %1\n s_nop 1\n v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a) : "v"(b) : "vcc");))
    // 7: independent v_sqrt_f32 x4
    TIME(R8(asm volatile("v_sqrt_f32 %0, %4\n v_sqrt_f32 %1, %4\n v_sqrt_f32 %2, %4\n v_sqrt_f32 %3, %4" : "=v"(a), "=v"(c), "=v"(e), "=v"(g) : "v"(b));))
    // 8: dependent v_sqrt_f32
    TIME(R32(asm volatile("v_sqrt_f32 %0, %0" : "+v"(a));))
    // 9: s_nop 0
    TIME(R32(asm volatile("s_nop 0");))
    // 10: v_med3_f32 dependent
    TIME(R32(asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));))
    // 11: dependent v_fma_f32
    TIME(R32(asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));))
    // 12: LPF-like: pk_mul (indep) then 4 dependent adds
    TIME(R8(asm volatile("v_pk_mul_f32 %1, %3, %2\n v_add_f32 %0, %0, %4\n v_add_f32 %0, %0, %4\n v_sub_f32 %0, %0, %4\n v_sub_f32 %0, %0, %4" : "+v"(a), "=v"(pc) : "v"(pb), "v"(pa), "v"(b));))
    // 13: ds_read_b128 + wait (latency)
    {
        __shared__ float4 lds[256];
        lds[threadIdx.x] = make_float4(a, b, c, d);
        __syncthreads();
        float4 v;
        TIME(R8(asm volatile("ds_read_b128 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(v) : "v"((unsigned)(threadIdx.x * 16)) : "memory"); a += v.x;))
    }
    if (threadIdx.x == 0) out[blockIdx.x * 32 + 31] = __float_as_uint(a + b + c + d + e + f + g + h + pa.x + pa.y + pb.x + pc.y + pd.x);
}

int main() {
    unsigned long long *d, h[32 * 2];
    if (hipMalloc(&d, sizeof h) != hipSuccess) return 2;
    bench<<<1, 64>>>(d, 1.0f);  // warm
    bench<<<1, 64>>>(d, 1.0f);
    if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(h, d, sizeof(unsigned long long) * 32, hipMemcpyDeviceToHost) != hipSuccess) return 2;
    const char *names[] = {"dep v_add_f32", "4x indep v_add_f32", "dep v_pk_add_f32", "4x indep v_pk_add_f32",
                           "dep v_pk_mul_f32", "dep v_mul_f32", "cmp+nop1+cndmask (per pair)", "4x indep v_sqrt_f32",
                           "dep v_sqrt_f32", "s_nop 0", "dep v_med3_f32", "dep v_fma_f32",
                           "LPF-like pk_mul+4 dep add (per 5)", "ds_read_b128+wait (per read)"};
    const double per[] = {32, 32, 32, 32, 32, 32, 32, 32, 32, 32, 32, 32, 8 * 5, 8};
    for (int i = 0; i < 14; i++) printf("%-36s %7.2f cyc/instr\n", names[i], (double)h[i] / (256.0 * per[i]));
    return 0;
}

// Lab: cycles per sample of the SSB low-pass step (y = (((v + a1 z1) + a2 z2) - b1 z1) - b2 z2, the products as
// two v_pk_mul_f32 broadcasting z1 and z2), written with fixed registers so nothing but the step is measured,
// against variants of its instruction form.  One wave alone; s_memtime cycles per sample.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/lab/lpf_step tools/lab/lpf_step.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
constexpr int REP = 1024;

// two samples per asm block: z1/z2 alternate between v[40:41] and v[42:43], so no register moves
#define LPF_PK2                                                                                \
    "v_pk_mul_f32 v[44:45], v[50:51], v[40:41] op_sel_hi:[1,0]\n"                              \
    "v_pk_mul_f32 v[46:47], v[52:53], v[42:43] op_sel_hi:[1,0]\n"                              \
    "v_add_f32 v48, v44, v54\n"                                                                \
    "v_add_f32 v48, v46, v48\n"                                                                \
    "v_add_f32 v48, v45, v48\n"                                                                \
    "v_add_f32 v42, v47, v48\n"                                                                \
    "v_pk_mul_f32 v[44:45], v[50:51], v[42:43] op_sel_hi:[1,0]\n"                              \
    "v_pk_mul_f32 v[46:47], v[52:53], v[40:41] op_sel_hi:[1,0]\n"                              \
    "v_add_f32 v48, v44, v54\n"                                                                \
    "v_add_f32 v48, v46, v48\n"                                                                \
    "v_add_f32 v48, v45, v48\n"                                                                \
    "v_add_f32 v40, v47, v48\n"

// the same with the z2 product issued first (it does not depend on the previous output)
#define LPF_PK2_Z2FIRST                                                                        \
    "v_pk_mul_f32 v[46:47], v[52:53], v[42:43] op_sel_hi:[1,0]\n"                              \
    "v_pk_mul_f32 v[44:45], v[50:51], v[40:41] op_sel_hi:[1,0]\n"                              \
    "v_add_f32 v48, v44, v54\n"                                                                \
    "v_add_f32 v48, v46, v48\n"                                                                \
    "v_add_f32 v48, v45, v48\n"                                                                \
    "v_add_f32 v42, v47, v48\n"                                                                \
    "v_pk_mul_f32 v[46:47], v[52:53], v[40:41] op_sel_hi:[1,0]\n"                              \
    "v_pk_mul_f32 v[44:45], v[50:51], v[42:43] op_sel_hi:[1,0]\n"                              \
    "v_add_f32 v48, v44, v54\n"                                                                \
    "v_add_f32 v48, v46, v48\n"                                                                \
    "v_add_f32 v48, v45, v48\n"                                                                \
    "v_add_f32 v40, v47, v48\n"

// scalar products: a1 z1 on the chain, the other three off it
#define LPF_SCALAR2                                                                            \
    "v_mul_f32 v44, v50, v40\n"                                                                \
    "v_mul_f32 v46, v52, v42\n"                                                                \
    "v_mul_f32 v45, v51, v40\n"                                                                \
    "v_mul_f32 v47, v53, v42\n"                                                                \
    "v_add_f32 v48, v44, v54\n"                                                                \
    "v_add_f32 v48, v46, v48\n"                                                                \
    "v_add_f32 v48, v45, v48\n"                                                                \
    "v_add_f32 v42, v47, v48\n"                                                                \
    "v_mul_f32 v44, v50, v42\n"                                                                \
    "v_mul_f32 v46, v52, v40\n"                                                                \
    "v_mul_f32 v45, v51, v42\n"                                                                \
    "v_mul_f32 v47, v53, v40\n"                                                                \
    "v_add_f32 v48, v44, v54\n"                                                                \
    "v_add_f32 v48, v46, v48\n"                                                                \
    "v_add_f32 v48, v45, v48\n"                                                                \
    "v_add_f32 v40, v47, v48\n"

// the dependent chain alone: 4 adds per sample, products not recomputed (a lower bound)
#define CHAIN_ONLY2                                                                            \
    "v_add_f32 v48, v44, v40\n"                                                                \
    "v_add_f32 v48, v46, v48\n"                                                                \
    "v_add_f32 v48, v45, v48\n"                                                                \
    "v_add_f32 v40, v47, v48\n"                                                                \
    "v_add_f32 v48, v44, v40\n"                                                                \
    "v_add_f32 v48, v46, v48\n"                                                                \
    "v_add_f32 v48, v45, v48\n"                                                                \
    "v_add_f32 v40, v47, v48\n"


// the compiled form: coefficient pairs in SGPRs (uniform values), as hipcc emits for the pipeline kernel
#define LPF_PK2_SGPR                                                                           \
    "v_pk_mul_f32 v[44:45], s[44:45], v[40:41] op_sel_hi:[1,0]\n"                              \
    "v_pk_mul_f32 v[46:47], s[46:47], v[42:43] op_sel_hi:[1,0]\n"                              \
    "v_add_f32 v48, v44, v54\n"                                                                \
    "v_add_f32 v48, v46, v48\n"                                                                \
    "v_add_f32 v48, v45, v48\n"                                                                \
    "v_add_f32 v42, v47, v48\n"                                                                \
    "v_pk_mul_f32 v[44:45], s[44:45], v[42:43] op_sel_hi:[1,0]\n"                              \
    "v_pk_mul_f32 v[46:47], s[46:47], v[40:41] op_sel_hi:[1,0]\n"                              \
    "v_add_f32 v48, v44, v54\n"                                                                \
    "v_add_f32 v48, v46, v48\n"                                                                \
    "v_add_f32 v48, v45, v48\n"                                                                \
    "v_add_f32 v40, v47, v48\n"

#define KERNEL(NAME, BODY)                                                                      \
    __global__ void NAME(float *out, unsigned long long *cyc, float s) {                        \
        float r = 0.f;                                                                          \
        unsigned long long t0 = 0, t1 = 0;                                                      \
        asm volatile(                                                                           \
            "v_mov_b32 v40, %3\n v_mov_b32 v41, 0\n v_mov_b32 v42, %3\n v_mov_b32 v43, 0\n"     \
            "v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v46, 0\n v_mov_b32 v47, 0\n"       \
            "v_mov_b32 v50, 0x3f7fbe77\n v_mov_b32 v51, 0xbf7fbe77\n"                           \
            "v_mov_b32 v52, 0x3a83126f\n v_mov_b32 v53, 0x3a03126f\n v_mov_b32 v54, %3\n"       \
            "s_mov_b32 s44, 0x3f7fbe77\n s_mov_b32 s45, 0xbf7fbe77\n"                           \
            "s_mov_b32 s46, 0x3a83126f\n s_mov_b32 s47, 0x3a03126f\n"                           \
            "s_waitcnt lgkmcnt(0)\n"                                                            \
            "s_memtime %0\n s_waitcnt lgkmcnt(0)\n"                                             \
            "s_mov_b32 s40, %4\n"                                                               \
            "1:\n" BODY BODY BODY BODY BODY BODY BODY BODY                                       \
            "s_sub_u32 s40, s40, 1\n s_cmp_lg_u32 s40, 0\n s_cbranch_scc1 1b\n"                  \
            "s_memtime %1\n s_waitcnt lgkmcnt(0)\n"                                             \
            "v_mov_b32 %2, v40\n"                                                               \
            : "=&s"(t0), "=&s"(t1), "=v"(r)                                                     \
            : "v"(s), "i"(REP)                                                                  \
            : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v50", "v51", "v52",   \
              "v53", "v54", "s40", "s44", "s45", "s46", "s47", "scc", "memory");                                            \
        out[threadIdx.x] = r;                                                                   \
        if (threadIdx.x == 0) cyc[0] = t1 - t0;                                                 \
    }

KERNEL(k_pk2, LPF_PK2)
KERNEL(k_pk2_z2first, LPF_PK2_Z2FIRST)
KERNEL(k_scalar2, LPF_SCALAR2)
KERNEL(k_chain2, CHAIN_ONLY2)
KERNEL(k_pk2_sgpr, LPF_PK2_SGPR)

template <class K>
void run(const char *name, K k, int threads, int blocks = 1) {
    float *o; unsigned long long *c, h = 0;
    hipMalloc(&o, 4096 * 4); hipMalloc(&c, 8);
    for (int w = 0; w < 2; w++) {
        hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, o, c, 1e-3f);
        hipDeviceSynchronize();
    }
    hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
    const double samples = (double)REP * 8 * 2;  // 8 bodies of 2 samples per iteration
    printf("%-14s %3d x %4d thr: %6.2f cycles per sample\n", name, blocks, threads, h / samples);
    hipFree(o); hipFree(c);
}
int main() {
    const int cfg[][2] = {{1, 64}, {1, 768}};
    for (auto &c : cfg) {
        run("pk vgpr coef", k_pk2, c[1], c[0]);
        run("pk sgpr coef", k_pk2_sgpr, c[1], c[0]);
        run("scalar muls", k_scalar2, c[1], c[0]);
        run("4-add chain", k_chain2, c[1], c[0]);
    }
    return 0;
}

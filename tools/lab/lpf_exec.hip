// Lab: the low-pass step (2 v_pk_mul_f32 + 4 dependent v_add_f32 per sample) on registers only, one wave alone:
// operand order of the dependent adds (running value as src0 or src1) x EXEC pattern, s_memtime cycles
// per sample.  Build: hipcc --offload-arch=gfx950 -O3 -o tools/lab/lpf_exec tools/lab/lpf_exec.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
constexpr int REP = 512;
// z1 in v0 (pair v[0:1] lo), z2 in v2 (pair v[2:3] lo), x in v10; outputs alternate v0 / v2
#define S_SRC0(Z1, Z2, Y)                                                                         \
    "v_pk_mul_f32 v[4:5], v[20:21], v[" #Z1 ":" #Z1 "+1] op_sel_hi:[1,0]\n"                       \
    "v_pk_mul_f32 v[6:7], v[22:23], v[" #Z2 ":" #Z2 "+1] op_sel_hi:[1,0]\n"                       \
    "v_add_f32 v8, v10, v4\n"                                                                     \
    "v_add_f32 v8, v8, v6\n"                                                                      \
    "v_add_f32 v8, v8, v5\n"                                                                      \
    "v_add_f32 v" #Y ", v8, v7\n"
#define S_SRC1(Z1, Z2, Y)                                                                         \
    "v_pk_mul_f32 v[4:5], v[20:21], v[" #Z1 ":" #Z1 "+1] op_sel_hi:[1,0]\n"                       \
    "v_pk_mul_f32 v[6:7], v[22:23], v[" #Z2 ":" #Z2 "+1] op_sel_hi:[1,0]\n"                       \
    "v_add_f32 v8, v4, v10\n"                                                                     \
    "v_add_f32 v8, v6, v8\n"                                                                      \
    "v_add_f32 v8, v5, v8\n"                                                                      \
    "v_add_f32 v" #Y ", v7, v8\n"
#define BODY(S) S(0, 2, 2) S(2, 0, 0) S(0, 2, 2) S(2, 0, 0) S(0, 2, 2) S(2, 0, 0) S(0, 2, 2) S(2, 0, 0)

template <int V, unsigned long long MASK>
__global__ void k(unsigned long long *out) {
    const int lane = threadIdx.x & 63;
    unsigned long long t0 = 0, t1 = 0;
    if ((MASK >> lane) & 1) {
        asm volatile("v_mov_b32 v0, 0.5\n v_mov_b32 v2, 0.25\n v_mov_b32 v10, 0.125\n v_mov_b32 v20, 0.5\n v_mov_b32 v21, -0.25\n"
                     "v_mov_b32 v22, 0.125\n v_mov_b32 v23, -0.0625\n" ::: "v0", "v2", "v10", "v20", "v21", "v22", "v23");
        t0 = __builtin_amdgcn_s_memtime();
        for (int r = 0; r < REP; r++) {
            if constexpr (V == 0) asm volatile(BODY(S_SRC0) ::: "v0", "v2", "v4", "v5", "v6", "v7", "v8");
            else asm volatile(BODY(S_SRC1) ::: "v0", "v2", "v4", "v5", "v6", "v7", "v8");
        }
        t1 = __builtin_amdgcn_s_memtime();
    }
    if (lane == __builtin_ctzll(MASK)) out[0] = t1 - t0;
}
template <int V, unsigned long long MASK>
void run(const char *name, unsigned long long *d) {
    unsigned long long h = 0;
    for (int r = 0; r < 3; r++) k<V, MASK><<<1, 64>>>(d);
    if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost) != hipSuccess) return;
    printf("%-28s exec %016llx: %6.2f cyc/sample\n", name, MASK, h / (double)(REP * 8));
}
int main() {
    unsigned long long *d;
    if (hipMalloc(&d, 64) != hipSuccess) return 2;
    run<0, ~0ull>("running value as src0", d);
    run<1, ~0ull>("running value as src1", d);
    run<0, 0xffffull>("running value as src0", d);
    run<1, 0xffffull>("running value as src1", d);
    run<0, 1ull>("running value as src0", d);
    // 16 lanes spread over the four 16-lane quarters (4 each / 1 in 4), 32 lanes (two quarters / spread)
    run<0, 0x000f000f000f000full>("running value as src0", d);
    run<0, 0x1111111111111111ull>("running value as src0", d);
    run<0, 0x0001000100010001ull>("running value as src0", d);
    run<0, 0xffffffffull>("running value as src0", d);
    run<0, 0x00ff00ff00ff00ffull>("running value as src0", d);
    run<0, 0x5555555555555555ull>("running value as src0", d);
    return 0;
}

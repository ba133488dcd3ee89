// valu6.hip — the SSB low-pass recurrence (6 VALU per sample, 5-op dependent chain) under the pipeline's per-chunk
// structure: MODE 0 registers only; 1 = read the 64-sample chunk row from LDS, chain, write it back; 2 = as 1 plus
// a workgroup barrier per chunk with W idle waves; 3 = as 2 with lanes >= 16 masked off (16 streams per wave).
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "../../sdr-for-android-lib_amd/csrc/ssb_lpf_asm.h"
#include "../lab/lab_lpf_asm.h"  // the split / no-LDS lab forms

typedef float f2v __attribute__((ext_vector_type(2)));
#pragma clang fp contract(off)

constexpr int CH = 64, ROW = CH + 4, NCH = 256;

template <int MODE>
__global__ void k(unsigned long long *out, const float *xs) {
    __shared__ float lds[2][16 * ROW];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < 2 * 16 * ROW; i += blockDim.x) (&lds[0][0])[i] = xs[i % 97];
    __syncthreads();
    float z1 = 0.1f, z2 = 0.2f;
    const f2v c1 = {1.99f, -0.9901f}, c2 = {-0.99f, 0.0001f};
    unsigned long long dt = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int c = 0; c < NCH; c++) {
        if (MODE >= 4 && w == 0 && ((MODE != 6 && MODE != 8 && MODE != 9) || lane < 16)) {
            // the product's hand-scheduled chunk (csrc/ssb_lpf_asm.h): 4 = 64 lanes alone, 5 = 64 lanes + barrier,
            // 6 = 16 lanes + barrier
            f2v z = {z1, z2};
            const uint32_t src = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) float *)&lds[c & 1][(lane & 15) * ROW];
            const uint32_t dst = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) float *)&lds[(c + 1) & 1][(lane & 15) * ROW];
            if constexpr (MODE == 9) {  // VALU on all 64 lanes, LDS on the caller's 16 (SPLIT), + barrier
                unsigned long long sv;
                asm volatile(SDRG_LPF_CHUNK_SPLIT_ASM : [z] "+v"(z), [sv] "=&s"(sv) : [src] "v"(src), [dst] "v"(dst), [c1] "s"(c1), [c2] "s"(c2)
                             : SDRG_CHUNK_CLOBBERS, "memory");
            } else if constexpr (MODE >= 7)  // register data only: 7 = 64 lanes, 8 = 16 lanes (+ barrier, 12 waves)
                asm volatile(SDRG_LPF_CHUNK_NOLDS_ASM : [z] "+v"(z) : [src] "v"(src), [dst] "v"(dst), [c1] "s"(c1), [c2] "s"(c2)
                             : SDRG_CHUNK_CLOBBERS, "memory");
            else
                asm volatile(SDRG_LPF_CHUNK_ASM : [z] "+v"(z) : [src] "v"(src), [dst] "v"(dst), [c1] "s"(c1), [c2] "s"(c2)
                             : SDRG_CHUNK_CLOBBERS, "memory");
            z1 = z.x;
            z2 = z.y;
        } else if (MODE < 4 && w == 0 && (MODE < 3 || lane < 16)) {
            float v[CH];
            const float *src = &lds[c & 1][(lane & 15) * ROW];
            if constexpr (MODE == 0) {
#pragma unroll
                for (int q = 0; q < CH; q++) v[q] = xs[q] + (float)c;  // loop-variant, no memory in the loop
            } else {
#pragma unroll
                for (int q = 0; q < CH; q += 4) {
                    const float4 r = *reinterpret_cast<const float4 *>(src + q);
                    v[q] = r.x; v[q + 1] = r.y; v[q + 2] = r.z; v[q + 3] = r.w;
                }
            }
#pragma unroll
            for (int q = 0; q < CH; q++) {
                const f2v p1 = c1 * z1, p2 = c2 * z2;
                const float y = (((v[q] + p1.x) + p2.x) + p1.y) + p2.y;
                z2 = z1;
                z1 = y;
                v[q] = y;
            }
            if constexpr (MODE == 0) {
                if (z1 == 1234.5f) out[5] = v[7];
            } else if (lane < 16) {
                float *dst = &lds[(c + 1) & 1][lane * ROW];
#pragma unroll
                for (int q = 0; q < CH; q += 4) *reinterpret_cast<float4 *>(dst + q) = make_float4(v[q], v[q + 1], v[q + 2], v[q + 3]);
            }
        }
        if constexpr (MODE >= 2 && MODE != 4) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
    dt = __builtin_amdgcn_s_memtime() - t0;
    if (threadIdx.x == 0) out[0] = dt;
    if (z1 == 12345.f) out[9] = 1;
}

template <int MODE>
void run(const char *name, unsigned long long *d, const float *xs, int waves) {
    unsigned long long h[10];
    for (int r = 0; r < 3; r++) k<MODE><<<1, 64 * waves>>>(d, xs);
    if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return;
    printf("%-44s waves %2d: %6.2f cyc/sample\n", name, waves, h[0] / (double)(NCH * CH));
}

int main() {
    unsigned long long *d;
    float *xs;
    if (hipMalloc(&d, 10 * sizeof(unsigned long long)) != hipSuccess || hipMalloc(&xs, 256 * 4) != hipSuccess) return 2;
    float h[256];
    for (int i = 0; i < 256; i++) h[i] = 0.01f * (i % 17) - 0.05f;
    if (hipMemcpy(xs, h, sizeof h, hipMemcpyHostToDevice) != hipSuccess) return 2;
    run<0>("registers only", d, xs, 1);
    run<1>("LDS row in/out", d, xs, 1);
    run<2>("LDS row in/out + barrier", d, xs, 1);
    run<2>("LDS row in/out + barrier", d, xs, 12);
    run<3>("LDS + barrier, 16 lanes", d, xs, 12);
    run<4>("asm chunk, 64 lanes", d, xs, 1);
    run<5>("asm chunk + barrier, 64 lanes", d, xs, 12);
    run<6>("asm chunk + barrier, 16 lanes", d, xs, 12);
    run<7>("asm chunk no LDS + barrier, 64 lanes", d, xs, 12);
    run<8>("asm chunk no LDS + barrier, 16 lanes", d, xs, 12);
    run<9>("asm split (VALU 64, LDS 16) + barrier", d, xs, 12);
    run<9>("asm split (VALU 64, LDS 16) + barrier", d, xs, 1);
    run<6>("asm chunk + barrier, 16 lanes", d, xs, 1);
    run<8>("asm chunk no LDS + barrier, 16 lanes", d, xs, 1);
    return 0;
}

// Lab probe (not product): how far from correctly rounded are gfx950's v_sqrt_f32 / v_rcp_f32 over the AGC's operand
// range, and which shorter sequences stay exact?  For every float m in [1e-8, FLT_MAX] (the AGC's sqrt operand
// fabsf(x) + 1e-8f, adaptiveAGC ssb_demod_opt.cpp:104-107):
//   sqrt: hardware estimate above / below IEEE sqrtf(m) (counts), and the one-sided corrections that fix it;
//   div : target / (sqrtf(m) + 1e-6f) for the four targets by shorter sequences than ssb_math.h's div_rn2.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -Isdr-for-android-lib_amd/csrc tools/lab/agc_probe.hip -o tools/lab/agc_probe
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <string.h>

#pragma clang fp contract(off)

enum { HW_HI, HW_LO, S_DN_ONLY, S_UP_ONLY, D_NO_NEWTON_1, D_NEWTON_1, D_NO_NEWTON_2, S_F64, S_RSQ, NCOUNT };

__device__ __forceinline__ float dn1(float s) { return __int_as_float(__float_as_int(s) - 1); }
__device__ __forceinline__ float up1(float s) { return __int_as_float(__float_as_int(s) + 1); }

__global__ void sweep(unsigned lo, unsigned hi, const float *targets, int nt, unsigned long long *cnt) {
    unsigned long long c[NCOUNT] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    const unsigned stride = gridDim.x * blockDim.x;
    for (unsigned long long b = lo + (blockIdx.x * blockDim.x + threadIdx.x); b <= hi; b += stride) {
        const float m = __uint_as_float((unsigned)b);
        const float ok = sqrtf(m);
        const float s = __builtin_amdgcn_sqrtf(m);
        c[HW_HI] += s > ok;
        c[HW_LO] += s < ok;
        // only the downward check (s - 1 ulp when m - dn*s <= 0), only the upward one (s + 1 ulp when m - up*s > 0)
        const float d = dn1(s), u = up1(s);
        const float sd = (fmaf(-d, s, m) <= 0.0f) ? d : s;
        const float su = (fmaf(-u, s, m) > 0.0f) ? u : s;
        c[S_DN_ONLY] += sd != ok;
        c[S_UP_ONLY] += su != ok;
        // the hardware double sqrt of the float, rounded once to float
        c[S_F64] += (float)__builtin_amdgcn_sqrt((double)m) != ok;
        // m * rsq(m) with one residual step: s1 = s0 + r/2 * e, e = m - s0*s0
        const float r0 = __builtin_amdgcn_rsqf(m), s0 = m * r0;
        c[S_RSQ] += fmaf(fmaf(-s0, s0, m), 0.5f * r0, s0) != ok;
        const float den = ok + 1e-6f;
        for (int t = 0; t < nt; t++) {
            const float n = targets[t], q_ok = n / den;
            const float r0 = __builtin_amdgcn_rcpf(den);
            const float r1 = fmaf(fmaf(-den, r0, 1.0f), r0, r0);
            float q = n * r0;
            q = fmaf(fmaf(-den, q, n), r0, q);
            c[D_NO_NEWTON_1] += q != q_ok;
            float q1 = n * r1;
            q1 = fmaf(fmaf(-den, q1, n), r1, q1);
            c[D_NEWTON_1] += q1 != q_ok;
            float q2 = n * r0;
            q2 = fmaf(fmaf(-den, q2, n), r0, q2);
            q2 = fmaf(fmaf(-den, q2, n), r0, q2);
            c[D_NO_NEWTON_2] += q2 != q_ok;
        }
    }
    for (int k = 0; k < NCOUNT; k++)
        if (c[k]) atomicAdd(&cnt[k], c[k]);
}

int main() {
    const float h_targets[4] = {0.35f, 0.45f, 0.40f, 0.30f};
    float *targets;
    unsigned long long *cnt;
    if (hipMalloc(&targets, sizeof h_targets) != hipSuccess || hipMalloc(&cnt, NCOUNT * 8) != hipSuccess) return 2;
    if (hipMemcpy(targets, h_targets, sizeof h_targets, hipMemcpyHostToDevice) != hipSuccess) return 2;
    if (hipMemset(cnt, 0, NCOUNT * 8) != hipSuccess) return 2;
    const float lo_f = 1e-8f;
    unsigned lo;
    memcpy(&lo, &lo_f, 4);
    sweep<<<65536, 256>>>(lo, 0x7f7fffffu, targets, 4, cnt);
    unsigned long long h[NCOUNT];
    if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(h, cnt, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 2;
    printf("operands %u: hw sqrt above %llu below %llu | down-only fix wrong %llu, up-only fix wrong %llu | "
           "div (4 targets): rcp+1 corr wrong %llu, newton+1 corr wrong %llu, rcp+2 corr wrong %llu | "
           "sqrt via f64 wrong %llu, via rsq + 1 step wrong %llu\n",
           0x7f7fffffu - lo + 1, h[HW_HI], h[HW_LO], h[S_DN_ONLY], h[S_UP_ONLY], h[D_NO_NEWTON_1], h[D_NEWTON_1],
           h[D_NO_NEWTON_2], h[S_F64], h[S_RSQ]);
    return 0;
}

// ssb_math.h — correctly rounded float sqrt and division for the AGC "desired" level, two lanes per op.
//
// adaptiveAGC (src/ssb/ssb_demod_opt.cpp:104-107) computes, per sample,
//     desired = target / (sqrtf(fabsf(x) + 1e-8f) + 1e-6f)
// with IEEE sqrt and division.  The compiler's IEEE expansions guard against denormal and huge operands
// (pre-scaling, v_div_scale / v_div_fixup, class checks).  Here the operands are bounded away from both:
//   sqrt operand m >= 1e-8 (far above the 2^-96 pre-scale threshold), finite;
//   divisor d = sqrt(m) + 1e-6 in [1e-4, 2^64), numerator = the mode's AGC target (0.35 .. 0.45),
// so the guards never fire and the remaining arithmetic is the same sequence of correctly rounded steps:
//   sqrt: hardware estimate s, then pick s-1ulp / s / s+1ulp by the sign of the exact residuals
//         m - s'*s (fma), as the compiler's expansion does;
//   div : reciprocal estimate, quotient n * r refined by ONE fma residual step.  Shorter than the general correctly
//         rounded sequence (Newton step on r, two residual steps), and exact on this operand set: every divisor
//         sqrtf(m) + 1e-6f for every float m in [1e-8, FLT_MAX] with the targets 0.30, 0.35, 0.40, 0.45 gives the IEEE
//         quotient (tools/lab/agc_probe.hip on gfx950: 0 of 5.2e9 differ; so do the longer sequences).  The hardware
//         sqrt estimate, by contrast, is above the IEEE root for 7.6e4 of the 1.3e9 operands and below it for 1.96e8,
//         so both of its corrections stay.
// The residual fmas and the Newton steps run as packed (two-lane) f32 ops.  tests/cpp/agc_exact.hip
// checks this bit for bit against sqrtf / operator/ over every float the sqrt operand can take.
#pragma once

#include <hip/hip_runtime.h>

namespace sdrg {

typedef float f2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f2v fma2(f2v a, f2v b, f2v c) { return __builtin_elementwise_fma(a, b, c); }

__device__ __forceinline__ float next_down(float s) { return __int_as_float(__float_as_int(s) - 1); }
__device__ __forceinline__ float next_up(float s) { return __int_as_float(__float_as_int(s) + 1); }

// Correctly rounded sqrt of two finite floats >= 2^-96.
__device__ __forceinline__ f2v sqrt_rn2(f2v m) {
    const f2v s = {__builtin_amdgcn_sqrtf(m.x), __builtin_amdgcn_sqrtf(m.y)};
    const f2v dn = {next_down(s.x), next_down(s.y)};
    const f2v up = {next_up(s.x), next_up(s.y)};
    const f2v r_dn = fma2(-dn, s, m);  // m - dn*s, exact sign
    const f2v r_up = fma2(-up, s, m);  // m - up*s
    f2v r;
    r.x = (r_dn.x <= 0.0f) ? dn.x : s.x;
    r.y = (r_dn.y <= 0.0f) ? dn.y : s.y;
    r.x = (r_up.x > 0.0f) ? up.x : r.x;
    r.y = (r_up.y > 0.0f) ? up.y : r.y;
    return r;
}

// n / d, correctly rounded for the AGC's operands (target in {0.30, 0.35, 0.40, 0.45}, d = sqrtf(m) + 1e-6f for
// m >= 1e-8f: checked exhaustively, tests/cpp/agc_exact.hip); one residual step on the hardware reciprocal.
__device__ __forceinline__ f2v div_rn2(f2v n, f2v d) {
    const f2v r = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
    const f2v q = n * r;
    const f2v rem = fma2(-d, q, n);
    return fma2(rem, r, q);
}

// adaptiveAGC's desired level for two samples, from |a| (a = the demodulated value, any finite float).
__device__ __forceinline__ f2v agc_desired_abs2(f2v abs_a, float target) {
    const f2v m = abs_a + f2v{1e-8f, 1e-8f};
    const f2v den = sqrt_rn2(m) + f2v{1e-6f, 1e-6f};
    return div_rn2(f2v{target, target}, den);
}

__device__ __forceinline__ f2v agc_desired2(f2v a, float target) {
    return agc_desired_abs2(f2v{fabsf(a.x), fabsf(a.y)}, target);
}

}  // namespace sdrg

// ssb_math.h — correctly rounded float sqrt and division for the AGC "desired" level, two lanes per op.
//
// adaptiveAGC (src/ssb/ssb_demod_opt.cpp:104-107) computes, per sample,
//     desired = target / (sqrtf(fabsf(x) + 1e-8f) + 1e-6f)
// with IEEE sqrt and division.  The compiler's IEEE expansions guard against denormal and huge operands
// (pre-scaling, v_div_scale / v_div_fixup, class checks) and pick the result by residual tests.  Here the operands
// are bounded away from both:
//   sqrt operand m >= 1e-8 (far above the 2^-96 pre-scale threshold), finite;
//   divisor d = sqrt(m) + 1e-6 in [1e-4, 2^64), numerator = the mode's AGC target (0.35 or 0.45),
// and on this finite operand set shorter sequences already give the IEEE results (verified on every operand):
//   sqrt: s0 = m * rsq(m) and one residual step (exact on this operand set, below);
//   div : reciprocal estimate, quotient n * r refined by ONE fma residual step.  Shorter than the general correctly
//         rounded sequence (Newton step on r, two residual steps), and exact on this operand set: every divisor
//         sqrtf(m) + 1e-6f for every float m in [1e-8, FLT_MAX] with the targets 0.30, 0.35, 0.40, 0.45 gives the IEEE
//         quotient (tools/lab/agc_probe.hip on gfx950: 0 of 5.2e9 differ; so do the longer sequences).  (The bare
//         hardware sqrt estimate is above the IEEE root for 7.6e4 of the 1.3e9 operands and below it for 1.96e8; the
//         rsq-based form with its residual step is exact on all of them.)
// The products and residual fmas run as packed (two-lane) f32 ops.  tests/cpp/agc_exact.hip checks the sequences bit
// for bit against sqrtf / operator/ over every float the sqrt operand can take (a GPU test of the suite).
#pragma once

#include <hip/hip_runtime.h>

namespace sdrg {

typedef float f2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f2v fma2(f2v a, f2v b, f2v c) { return __builtin_elementwise_fma(a, b, c); }

// sqrt, correctly rounded for the AGC's operands (every float m in [1e-8, FLT_MAX]: checked exhaustively,
// tests/cpp/agc_exact.hip): s0 = m * rsq(m), then one residual step s0 + (m - s0^2) * rsq(m) / 2 (tools/lab/agc_probe.hip:
// 0 of 1.3e9 differ from IEEE sqrtf).  Six operations per pair of samples instead of the estimate-and-select
// expansion's sixteen (hardware sqrt, both neighbours, two residuals, two selects per sample).
__device__ __forceinline__ f2v sqrt_rn2(f2v m) {
    const f2v r = {__builtin_amdgcn_rsqf(m.x), __builtin_amdgcn_rsqf(m.y)};
    const f2v s0 = m * r;
    const f2v e = fma2(-s0, s0, m);
    return fma2(e, r * f2v{0.5f, 0.5f}, s0);
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

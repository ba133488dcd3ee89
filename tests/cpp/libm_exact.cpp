// libm_exact.cpp — exhaustive host check of csrc/glibc_logf.h against the running glibc.
//
// For every float bit pattern in [+0, +inf] (2^31 - 2^23 + 1 values):
//   sdrg::glibc::logf(x)   == ::logf(x)     (bitwise)
//   sdrg::glibc::log10f(x) == ::log10f(x)   (bitwise), and so do log10f_fast and log10f_fast_fold (the statistics' paths)
// and both are monotone non-decreasing over that range (log10f(next float) >= log10f(float)), which the
// statistics kernels use to evaluate the focus window's dB only near its largest power (csrc/stats.hip).
// Prints "mismatches logf N log10f M monotone K" (first failing bit patterns too) and exits non-zero on any
// difference.  Build: g++ -O2 -std=c++17 -fopenmp -ffp-contract=off -fno-builtin (tests/cpp/Makefile).
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "glibc_logf.h"

static float bits(uint32_t u) {
    float f;
    memcpy(&f, &u, 4);
    return f;
}
static uint32_t ubits(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    return u;
}

int main() {
    unsigned long long bad_ln = 0, bad_lg = 0, non_mono = 0;
    uint32_t first_ln = 0xffffffffu, first_lg = 0xffffffffu;
    const long long hi = 0x7f800000ll;
    sdrg::glibc::LogfFold fold[sdrg::glibc::LOGF_FOLD_N];
    for (int i = 0; i < sdrg::glibc::LOGF_FOLD_N; i++) fold[i] = sdrg::glibc::logf_fold_entry(i, sdrg::glibc::logf_table());
#pragma omp parallel for schedule(static, 1 << 20) reduction(+ : bad_ln, bad_lg, non_mono) reduction(min : first_ln, first_lg)
    for (long long b = 0; b <= hi; b++) {
        const float x = bits((uint32_t)b);
        volatile float xv = x;  // keep the library calls real calls on a runtime operand
        const float want_ln = ::logf(xv), want_lg = ::log10f(xv);
        if (ubits(sdrg::glibc::logf(x)) != ubits(want_ln)) {
            bad_ln++;
            if ((uint32_t)b < first_ln) first_ln = (uint32_t)b;
        }
        if (b > 0) {  // -inf at +0, then non-decreasing up to +inf
            const float xp = bits((uint32_t)(b - 1));
            non_mono += (sdrg::glibc::log10f(x) < sdrg::glibc::log10f(xp)) + (sdrg::glibc::logf(x) < sdrg::glibc::logf(xp));
        }
        // the branch-free path the statistics use (log10f_fast), over every float it is called with here
        if (ubits(sdrg::glibc::log10f_fast(x, sdrg::glibc::logf_table())) != ubits(want_lg)) {
            bad_lg++;
            if ((uint32_t)b < first_lg) first_lg = (uint32_t)b;
        }
        if (ubits(sdrg::glibc::log10f_fast_fold(x, fold)) != ubits(want_lg)) {  // the wide statistics' path
            bad_lg++;
            if ((uint32_t)b < first_lg) first_lg = (uint32_t)b;
        }
        if (ubits(sdrg::glibc::log10f(x)) != ubits(want_lg)) {
            bad_lg++;
            if ((uint32_t)b < first_lg) first_lg = (uint32_t)b;
        }
    }
    // the sign bit set (-0, negatives, -inf, -NaN) and the positive NaNs: -inf for -0, otherwise NaN like glibc
    unsigned long long bad_neg = 0;
#pragma omp parallel for schedule(static, 1 << 20) reduction(+ : bad_neg)
    for (long long b = 0x7f800001ll; b <= 0xffffffffll; b++) {
        const float x = bits((uint32_t)b);
        volatile float xv = x;
        const float a = sdrg::glibc::logf(x), c = sdrg::glibc::log10f(x), wa = ::logf(xv), wc = ::log10f(xv);
        const float cf = sdrg::glibc::log10f_fast(x, sdrg::glibc::logf_table());
        const float cg = sdrg::glibc::log10f_fast_fold(x, fold);
        bad_neg += !((isnan(a) && isnan(wa)) || ubits(a) == ubits(wa)) + !((isnan(c) && isnan(wc)) || ubits(c) == ubits(wc)) +
                   !((isnan(cf) && isnan(wc)) || ubits(cf) == ubits(wc)) + !((isnan(cg) && isnan(wc)) || ubits(cg) == ubits(wc));
    }
    printf("mismatches logf %llu log10f %llu monotone %llu negative/nan %llu first 0x%08x 0x%08x\n", bad_ln, bad_lg,
           non_mono, bad_neg, first_ln, first_lg);
    return (bad_ln || bad_lg || non_mono || bad_neg) ? 1 : 0;
}

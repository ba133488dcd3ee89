// libm_exact.cpp — exhaustive host check of csrc/glibc_logf.h against the running glibc.
//
// For every float bit pattern in [+0, +inf] (2^31 - 2^23 + 1 values):
//   sdrg::glibc::logf(x)   == ::logf(x)     (bitwise)
//   sdrg::glibc::log10f(x) == ::log10f(x)   (bitwise)
// Prints "mismatches logf N log10f M" (first failing bit patterns too) and exits non-zero on any
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
    unsigned long long bad_ln = 0, bad_lg = 0;
    uint32_t first_ln = 0xffffffffu, first_lg = 0xffffffffu;
    const long long hi = 0x7f800000ll;
#pragma omp parallel for schedule(static, 1 << 20) reduction(+ : bad_ln, bad_lg) reduction(min : first_ln, first_lg)
    for (long long b = 0; b <= hi; b++) {
        const float x = bits((uint32_t)b);
        volatile float xv = x;  // keep the library calls real calls on a runtime operand
        const float want_ln = ::logf(xv), want_lg = ::log10f(xv);
        if (ubits(sdrg::glibc::logf(x)) != ubits(want_ln)) {
            bad_ln++;
            if ((uint32_t)b < first_ln) first_ln = (uint32_t)b;
        }
        if (ubits(sdrg::glibc::log10f(x)) != ubits(want_lg)) {
            bad_lg++;
            if ((uint32_t)b < first_lg) first_lg = (uint32_t)b;
        }
    }
    printf("mismatches logf %llu log10f %llu first 0x%08x 0x%08x\n", bad_ln, bad_lg, first_ln, first_lg);
    return (bad_ln || bad_lg) ? 1 : 0;
}

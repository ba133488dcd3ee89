// glibc_logf.h — the reference's libm, restated: glibc 2.35 logf and log10f on x86-64, bit for bit.
//
// The statistics (src/dsp/fft_process.cpp:146-155, :196-210, :256, :282, :304) turn powers into dB with
// log10f and take std::log(float(focusLen)).  The reference's golden build is the x86-64 one,
// so every dB value — and with it the focus peak index (first strict maximum of dB, :146-154), the window
// sort by meanDb (:218-247) and the pooled gaps — is decided by glibc's rounding, which ocml's log10f does
// not reproduce (it differs in the last ulp on a few percent of inputs).  These functions compute the same
// floats as the container's glibc 2.35 (Ubuntu 22.04) on a CPU with FMA:
//
//   logf   — sysdeps/ieee754/flt-32/e_logf.c (the table-driven double-precision algorithm from ARM's
//            optimized-routines, LOGF_TABLE_BITS = 4, a degree-3 polynomial in r = z/c − 1), as the x86-64
//            ifunc selects it on FMA hardware (sysdeps/x86_64/fpu/multiarch/e_logf-fma.c: the same C source
//            built with -mfma, so GCC contracts every a·b + c of the evaluation into one fma);
//   log10f — sysdeps/ieee754/flt-32/e_log10f.c (the fdlibm reduction x = 2^k·m, m in [1, 2) or [0.5, 1)
//            for k < 0; log10(x) = k·log10_2lo + ivln10·logf(m) + k·log10_2hi in float, generic build,
//            no contraction) calling the logf above through __ieee754_logf.
//
// The constants are glibc's published data (e_logf_data.c, e_log10f.c).  tests/cpp/libm_exact.cpp checks the
// host instantiation and tests/cpp/libm_exact.hip the device one against the running glibc on every
// non-negative float, infinities included; negative and NaN inputs give a NaN as glibc's do (not necessarily the
// same NaN bits), -0 gives -inf.
#pragma once

#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define SDRG_HD __host__ __device__ __forceinline__
#else
#define SDRG_HD static inline
#endif

namespace sdrg {
namespace glibc {

struct LogfEntry {
    double invc, logc;
};

// e_logf_data.c: 1/c and log(c) for the 16 subintervals of [OFF, 2·OFF), OFF = 0x3f330000
#define SDRG_LOGF_TAB                                                                                          \
    {{0x1.661ec79f8f3bep+0, -0x1.57bf7808caadep-2}, {0x1.571ed4aaf883dp+0, -0x1.2bef0a7c06ddbp-2},             \
     {0x1.49539f0f010bp+0, -0x1.01eae7f513a67p-2},  {0x1.3c995b0b80385p+0, -0x1.b31d8a68224e9p-3},             \
     {0x1.30d190c8864a5p+0, -0x1.6574f0ac07758p-3}, {0x1.25e227b0b8eap+0, -0x1.1aa2bc79c81p-3},                \
     {0x1.1bb4a4a1a343fp+0, -0x1.a4e76ce8c0e5ep-4}, {0x1.12358f08ae5bap+0, -0x1.1973c5a611cccp-4},             \
     {0x1.0953f419900a7p+0, -0x1.252f438e10c1ep-5}, {0x1p+0, 0x0p+0},                                          \
     {0x1.e608cfd9a47acp-1, 0x1.aa5aa5df25984p-5},  {0x1.ca4b31f026aap-1, 0x1.c5e53aa362eb4p-4},               \
     {0x1.b2036576afce6p-1, 0x1.526e57720db08p-3},  {0x1.9c2d163a1aa2dp-1, 0x1.bc2860d22477p-3},               \
     {0x1.886e6037841edp-1, 0x1.1058bc8a07ee1p-2},  {0x1.767dcf5534862p-1, 0x1.4043057b6ee09p-2}}

#if defined(__HIPCC__)
__device__ __constant__ static const LogfEntry kLogfTabDev[16] = SDRG_LOGF_TAB;
#endif
static const LogfEntry kLogfTabHost[16] = SDRG_LOGF_TAB;

SDRG_HD const LogfEntry *logf_table() {
#if defined(__HIP_DEVICE_COMPILE__)
    return kLogfTabDev;
#else
    return kLogfTabHost;
#endif
}

SDRG_HD uint32_t f2u(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    return u;
}
SDRG_HD float u2f(uint32_t u) {
    float f;
    memcpy(&f, &u, 4);
    return f;
}

SDRG_HD double fma_d(double a, double b, double c) { return __builtin_fma(a, b, c); }

// e_logf.c (__logf): +-0 gives -inf, +inf gives +inf, negative or NaN gives NaN.  `tab` is the 16-entry table (a copy in LDS
// on the device: the index is data-dependent, and an LDS read is far shorter than a global one).
SDRG_HD float logf_with(float x, const LogfEntry *tab) {
    const double Ln2 = 0x1.62e42fefa39efp-1;
    const double A0 = -0x1.00ea348b88334p-2, A1 = 0x1.5575b0be00b6ap-2, A2 = -0x1.ffffef20a4123p-2;
    uint32_t ix = f2u(x);
    if (ix == 0x3f800000u) return 0.0f;
    if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u) {
        if (ix * 2 == 0) return -__builtin_inff();
        if (ix == 0x7f800000u) return x;
        if ((ix & 0x80000000u) || ix * 2 >= 0xff000000u) return __builtin_nanf("");  // negative or NaN: NaN
        ix = f2u(x * 0x1p23f);  // subnormal: normalise
        ix -= 23u << 23;
    }
    const uint32_t tmp = ix - 0x3f330000u;
    const int i = (int)((tmp >> (23 - 4)) % 16);
    const int k = (int32_t)tmp >> 23;
    const uint32_t iz = ix - (tmp & 0xff800000u);
    const double invc = tab[i].invc, logc = tab[i].logc;
    const double z = (double)u2f(iz);
    // the FMA build's contraction of: r = z*invc - 1; y0 = logc + k*Ln2; y = A1*r + A2; y = A0*r2 + y;
    // y = y*r2 + (y0 + r)
    const double r = fma_d(z, invc, -1.0);
    const double y0 = fma_d((double)k, Ln2, logc);
    const double r2 = r * r;
    double y = fma_d(A1, r, A2);
    y = fma_d(A0, r2, y);
    y = fma_d(y, r2, y0 + r);
    return (float)y;
}

// e_log10f.c (__ieee754_log10f) for x >= 0, in float without contraction.
SDRG_HD float log10f_with(float x, const LogfEntry *tab) {
    const float two25 = 3.3554432000e+07f, ivln10 = 4.3429449201e-01f, log10_2hi = 3.0102920532e-01f,
                log10_2lo = 7.9034151668e-07f;
    int32_t hx = (int32_t)f2u(x);
    int32_t k = 0;
    if (hx < 0x00800000) {
        if ((hx & 0x7fffffff) == 0) return -__builtin_inff();
        if (hx < 0) return __builtin_nanf("");  // log(-x) = NaN
        k -= 25;
        x *= two25;
        hx = (int32_t)f2u(x);
    }
    if (hx >= 0x7f800000) return x + x;
    k += (hx >> 23) - 127;
    const int32_t i = (int32_t)(((uint32_t)k & 0x80000000u) >> 31);
    hx = (hx & 0x007fffff) | ((0x7f - i) << 23);
    const float y = (float)(k + i);
    x = u2f((uint32_t)hx);
    const float a = y * log10_2lo;
    const float b = ivln10 * logf_with(x, tab);
    const float z = a + b;
    const float c = y * log10_2hi;
    return z + c;
}

// log10f_with for a positive, normal, finite x (FLT_MIN <= x <= FLT_MAX): the same operations without the special
// cases -- no branch on the path the statistics take (their operands are power + 1e-20).  For x == 1 the logf
// step gives +0 without glibc's explicit check (r = 0, y0 = 0, table entry 9 = {1, 0}).
SDRG_HD float log10f_posnormal(float x, const LogfEntry *tab) {
    const float ivln10 = 4.3429449201e-01f, log10_2hi = 3.0102920532e-01f, log10_2lo = 7.9034151668e-07f;
    const double Ln2 = 0x1.62e42fefa39efp-1;
    const double A0 = -0x1.00ea348b88334p-2, A1 = 0x1.5575b0be00b6ap-2, A2 = -0x1.ffffef20a4123p-2;
    const int32_t hx = (int32_t)f2u(x);
    const int32_t k = (hx >> 23) - 127;
    const int32_t i = (int32_t)((uint32_t)k >> 31);                           // m in [0.5, 1) when k < 0
    const uint32_t ix = (uint32_t)((hx & 0x007fffff) | ((0x7f - i) << 23));  // the bits of m
    const float y = (float)(k + i);
    // logf(m), m in [0.5, 2): normal, so e_logf.c's special cases never apply
    const uint32_t tmp = ix - 0x3f330000u;
    const int ti = (int)((tmp >> (23 - 4)) & 15u);
    const int kk = (int32_t)tmp >> 23;
    const uint32_t iz = ix - (tmp & 0xff800000u);
    const double invc = tab[ti].invc, logc = tab[ti].logc;
    const double z = (double)u2f(iz);
    const double r = fma_d(z, invc, -1.0);
    const double y0 = fma_d((double)kk, Ln2, logc);
    const double r2 = r * r;
    double yy = fma_d(A1, r, A2);
    yy = fma_d(A0, r2, yy);
    yy = fma_d(yy, r2, y0 + r);
    const float lnm = (float)yy;
    const float a = y * log10_2lo;
    const float b = ivln10 * lnm;
    const float zz = a + b;
    const float c = y * log10_2hi;
    return zz + c;
}

// The table folded with e_logf.c's k: for m in [0.5, 2), (int32)(bits(m) - OFF) >> 19 = kk * 16 + i with kk in
// {-1, 0, 1}, so one 48-entry table indexed by that value + 16 holds 1/c and y0 = fma(kk, Ln2, log c) -- the same
// double that log10f_posnormal computes per call, so the same bits, one conversion and one f64 fma fewer per log
// (the wide statistics kernels, whose producers evaluate a log per reference-window bin).
struct LogfFold {
    double invc, y0;
};
constexpr int LOGF_FOLD_N = 48;
SDRG_HD LogfFold logf_fold_entry(int idx, const LogfEntry *tab) {
    const double Ln2 = 0x1.62e42fefa39efp-1;
    const int j = idx - 16;
    const LogfEntry e = tab[j & 15];
    return LogfFold{e.invc, fma_d((double)(j >> 4), Ln2, e.logc)};
}

SDRG_HD float log10f_posnormal_fold(float x, const LogfFold *fold) {
    const float ivln10 = 4.3429449201e-01f, log10_2hi = 3.0102920532e-01f, log10_2lo = 7.9034151668e-07f;
    const double A0 = -0x1.00ea348b88334p-2, A1 = 0x1.5575b0be00b6ap-2, A2 = -0x1.ffffef20a4123p-2;
    const int32_t hx = (int32_t)f2u(x);
    const int32_t k = (hx >> 23) - 127;
    const int32_t i = (int32_t)((uint32_t)k >> 31);
    const uint32_t ix = (uint32_t)((hx & 0x007fffff) | ((0x7f - i) << 23));
    const float y = (float)(k + i);
    const uint32_t tmp = ix - 0x3f330000u;
    const LogfFold f = fold[((int32_t)tmp >> 19) + 16];
    const uint32_t iz = ix - (tmp & 0xff800000u);
    const double z = (double)u2f(iz);
    const double r = fma_d(z, f.invc, -1.0);
    const double r2 = r * r;
    double yy = fma_d(A1, r, A2);
    yy = fma_d(A0, r2, yy);
    yy = fma_d(yy, r2, f.y0 + r);
    const float lnm = (float)yy;
    const float a = y * log10_2lo;
    const float b = ivln10 * lnm;
    const float zz = a + b;
    const float c = y * log10_2hi;
    return zz + c;
}

SDRG_HD float log10f_fast_fold(float x, const LogfFold *fold) {
    const uint32_t u = f2u(x);
    if (__builtin_expect(u - 0x00800000u < 0x7f000000u, 1)) return log10f_posnormal_fold(x, fold);
    return log10f_with(x, logf_table());
}

// log10f_with, branch-free for positive normal finite x (the common case), the general path otherwise
SDRG_HD float log10f_fast(float x, const LogfEntry *tab) {
    const uint32_t u = f2u(x);
    if (__builtin_expect(u - 0x00800000u < 0x7f000000u, 1)) return log10f_posnormal(x, tab);  // [FLT_MIN, FLT_MAX]
    return log10f_with(x, tab);
}

SDRG_HD float logf(float x) { return logf_with(x, logf_table()); }
SDRG_HD float log10f(float x) { return log10f_with(x, logf_table()); }

}  // namespace glibc
}  // namespace sdrg

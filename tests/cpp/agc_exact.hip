// agc_exact.hip — exhaustive check of csrc/ssb_math.h against IEEE sqrtf and division.
//
// For every float m in [1e-8, FLT_MAX] (every value the AGC's sqrt operand fabsf(x) + 1e-8f can take):
//   sqrt_rn2(m)                              == sqrtf(m)
//   div_rn2(target, sqrt_rn2(m) + 1e-6f)     == target / (sqrtf(m) + 1e-6f)   for each mode's target
// and agc_desired2(a) == the reference expression on a spread of demodulated values (zeros, denormals,
// huge).  Prints "mismatches N" and exits non-zero on any difference.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <string.h>

#include "ssb_math.h"

#pragma clang fp contract(off)

using namespace sdrg;

__device__ float ref_desired(float a, float target) { return target / (sqrtf(fabsf(a) + 1e-8f) + 1e-6f); }

__global__ void sweep(unsigned lo, unsigned hi, const float *targets, int n_targets, unsigned long long *bad,
                      unsigned *first) {
    const unsigned stride = gridDim.x * blockDim.x * 2u;
    for (unsigned long long b = lo + 2ull * (blockIdx.x * blockDim.x + threadIdx.x); b <= hi; b += stride) {
        const unsigned b0 = (unsigned)b, b1 = (b + 1 <= hi) ? (unsigned)(b + 1) : (unsigned)b;
        const f2v m = {__uint_as_float(b0), __uint_as_float(b1)};
        const f2v s = sqrt_rn2(m);
        int n = (__float_as_uint(s.x) != __float_as_uint(sqrtf(m.x))) + (__float_as_uint(s.y) != __float_as_uint(sqrtf(m.y)));
        const f2v den = s + f2v{1e-6f, 1e-6f};
        for (int t = 0; t < n_targets; t++) {
            const float tg = targets[t];
            const f2v q = div_rn2(f2v{tg, tg}, den);
            n += __float_as_uint(q.x) != __float_as_uint(tg / (sqrtf(m.x) + 1e-6f));
            n += __float_as_uint(q.y) != __float_as_uint(tg / (sqrtf(m.y) + 1e-6f));
        }
        if (n) {
            atomicAdd(bad, (unsigned long long)n);
            atomicMin(first, b0);
        }
    }
}

__global__ void spread(const float *targets, int n_targets, unsigned long long *bad, unsigned *first) {
    // demodulated values: both signs, zero, denormals, every exponent
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;  // 2^24 values
    const unsigned bits = (i << 8) | (i >> 16);
    const f2v a = {__uint_as_float(bits & 0x7fffffffu) * ((i & 1) ? -1.0f : 1.0f), __uint_as_float(i & 0x807fffffu)};
    if (!(fabsf(a.x) <= 3.0e38f) || !(fabsf(a.y) <= 3.0e38f)) return;
    for (int t = 0; t < n_targets; t++) {
        const f2v d = agc_desired2(a, targets[t]);
        const int n = (__float_as_uint(d.x) != __float_as_uint(ref_desired(a.x, targets[t]))) +
                      (__float_as_uint(d.y) != __float_as_uint(ref_desired(a.y, targets[t])));
        if (n) {
            atomicAdd(bad, (unsigned long long)n);
            atomicMin(first, bits);
        }
    }
}

#define CK(x)                                                              \
    do {                                                                   \
        if ((x) != hipSuccess) {                                           \
            printf("hip error at %s:%d\n", __FILE__, __LINE__);           \
            return 2;                                                      \
        }                                                                  \
    } while (0)

int main() {
    const float h_targets[4] = {0.35f, 0.45f, 0.40f, 0.30f};
    float *targets;
    unsigned long long *bad;
    unsigned *first;
    CK(hipMalloc(&targets, sizeof h_targets));
    CK(hipMalloc(&bad, sizeof *bad));
    CK(hipMalloc(&first, sizeof *first));
    CK(hipMemcpy(targets, h_targets, sizeof h_targets, hipMemcpyHostToDevice));
    CK(hipMemset(bad, 0, sizeof *bad));
    CK(hipMemset(first, 0xff, sizeof *first));
    const float lo_f = 1e-8f;
    unsigned lo;
    memcpy(&lo, &lo_f, 4);
    sweep<<<65536, 256>>>(lo, 0x7f7fffffu, targets, 4, bad, first);
    spread<<<(1u << 24) / 256, 256>>>(targets, 4, bad, first);
    unsigned long long h_bad = 0;
    unsigned h_first = 0;
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(&h_bad, bad, sizeof h_bad, hipMemcpyDeviceToHost));
    CK(hipMemcpy(&h_first, first, sizeof h_first, hipMemcpyDeviceToHost));
    printf("mismatches %llu first 0x%08x\n", h_bad, h_first);
    return h_bad ? 1 : 0;
}

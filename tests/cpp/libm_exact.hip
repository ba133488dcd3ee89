// libm_exact.hip — exhaustive device check of csrc/glibc_logf.h against the running glibc.
//
// For every float bit pattern in [+0, +inf] the GPU evaluates sdrg::glibc::logf and ::log10f — once with
// the table read from constant memory, once from an LDS copy as the statistics kernels use it — and the
// host compares each result bitwise with the C library's logf / log10f (the glibc the reference's x86-64
// build links).  The range goes in chunks of 2^26 values; the host compares a chunk on every worker thread
// while the device computes the next.  Prints "mismatches logf N log10f M ..." and exits non-zero on any
// difference.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <thread>
#include <vector>

#include "glibc_logf.h"

using sdrg::glibc::LogfEntry;

__global__ void eval(uint32_t base, uint32_t count, float *out_ln, float *out_lg, unsigned long long *lds_bad) {
    __shared__ LogfEntry tab[16];
    __shared__ sdrg::glibc::LogfFold fold[sdrg::glibc::LOGF_FOLD_N];
    if (threadIdx.x < 16) tab[threadIdx.x] = sdrg::glibc::logf_table()[threadIdx.x];
    if (threadIdx.x < sdrg::glibc::LOGF_FOLD_N)
        fold[threadIdx.x] = sdrg::glibc::logf_fold_entry(threadIdx.x, sdrg::glibc::logf_table());
    __syncthreads();
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const float x = __uint_as_float(base + i);
    const float ln = sdrg::glibc::logf(x), lg = sdrg::glibc::log10f(x);
    out_ln[i] = ln;
    out_lg[i] = lg;
    // the LDS-table instantiation must agree with the constant-table one bit for bit
    const int bad = (__float_as_uint(sdrg::glibc::logf_with(x, tab)) != __float_as_uint(ln)) +
                    (__float_as_uint(sdrg::glibc::log10f_with(x, tab)) != __float_as_uint(lg)) +
                    (__float_as_uint(sdrg::glibc::log10f_fast(x, tab)) != __float_as_uint(lg)) +  // the stats' path
                    (__float_as_uint(sdrg::glibc::log10f_fast_fold(x, fold)) != __float_as_uint(lg));  // wide stats
    if (bad) atomicAdd(lds_bad, (unsigned long long)bad);
}

#define CK(x)                                                              \
    do {                                                                   \
        if ((x) != hipSuccess) {                                           \
            printf("hip error at %s:%d\n", __FILE__, __LINE__);           \
            return 2;                                                      \
        }                                                                  \
    } while (0)

static uint32_t ubits(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    return u;
}

int main() {
    const uint64_t total = 0x7f800001ull;  // +0 .. +inf
    const uint32_t chunk = 1u << 26;
    float *d_ln[2], *d_lg[2];
    unsigned long long *d_lds_bad;
    std::vector<float> h_ln(chunk), h_lg(chunk);
    for (int b = 0; b < 2; b++) {
        CK(hipMalloc(&d_ln[b], chunk * sizeof(float)));
        CK(hipMalloc(&d_lg[b], chunk * sizeof(float)));
    }
    CK(hipMalloc(&d_lds_bad, sizeof(unsigned long long)));
    CK(hipMemset(d_lds_bad, 0, sizeof(unsigned long long)));
    const unsigned nthreads = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::atomic<unsigned long long> bad_ln{0}, bad_lg{0};
    std::atomic<uint32_t> first{0xffffffffu};
    for (uint64_t base = 0; base < total; base += chunk) {
        const uint32_t count = (uint32_t)std::min<uint64_t>(chunk, total - base);
        eval<<<(count + 255) / 256, 256>>>((uint32_t)base, count, d_ln[0], d_lg[0], d_lds_bad);
        CK(hipGetLastError());
        CK(hipMemcpy(h_ln.data(), d_ln[0], count * sizeof(float), hipMemcpyDeviceToHost));
        CK(hipMemcpy(h_lg.data(), d_lg[0], count * sizeof(float), hipMemcpyDeviceToHost));
        std::vector<std::thread> pool;
        for (unsigned t = 0; t < nthreads; t++) {
            pool.emplace_back([&, t] {
                unsigned long long bl = 0, bg = 0;
                for (uint32_t i = t; i < count; i += nthreads) {
                    float x;
                    const uint32_t b = (uint32_t)base + i;
                    memcpy(&x, &b, 4);
                    const int el = ubits(::logf(x)) != ubits(h_ln[i]), eg = ubits(::log10f(x)) != ubits(h_lg[i]);
                    if (el | eg) {
                        uint32_t f = first.load();
                        while (b < f && !first.compare_exchange_weak(f, b)) {
                        }
                    }
                    bl += el;
                    bg += eg;
                }
                bad_ln += bl;
                bad_lg += bg;
            });
        }
        for (auto &th : pool) th.join();
        if ((base / chunk) % 8 == 7) {
            printf("checked through 0x%08x\n", (uint32_t)(base + count - 1));
            fflush(stdout);
        }
    }
    unsigned long long lds_bad = 0;
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(&lds_bad, d_lds_bad, sizeof lds_bad, hipMemcpyDeviceToHost));
    printf("mismatches logf %llu log10f %llu lds_vs_const %llu first 0x%08x\n", bad_ln.load(), bad_lg.load(), lds_bad,
           first.load());
    return (bad_ln || bad_lg || lds_bad) ? 1 : 0;
}

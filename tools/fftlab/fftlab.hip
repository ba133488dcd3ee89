// fftlab.hip — development harness for the spectrum kernels (not part of the product library).
// Includes csrc/spectrum.hip directly, times the kernels on B frames of N = 16384 CS8 IQ with HIP events
// (median of reps), checks each against a float64 CPU DFT on sampled frames with the parity tolerance
// |dP| <= 1e-4 P + 1e-6 max(P), and prints algorithmic GB/s (2 B in + 4 B out per sample).  Also times the
// kernel's HBM access patterns alone (store/load pattern kernels) as the memory floor.
//   build: tools/fftlab/build.sh     run: tools/fftlab/fftlab [B] [variant]
#include "../../sdr-for-android-lib_amd/csrc/spectrum.hip"

#include <algorithm>
#include <complex>
#include <cstdio>
#include <cstring>
#include <vector>

using namespace sdrg;

#define CK(x)                                                                                 \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                          \
        }                                                                                     \
    } while (0)

static void cpu_power(const int8_t *iq, int n, std::vector<double> &p) {
    // float64 radix-2 FFT of the scaled samples, |X|^2, fftshift
    std::vector<std::complex<double>> a(n);
    for (int i = 0; i < n; i++) a[i] = {iq[2 * i] / 128.0, iq[2 * i + 1] / 128.0};
    for (int i = 1, j = 0; i < n; i++) {
        int bit = n >> 1;
        for (; j & bit; bit >>= 1) j ^= bit;
        j ^= bit;
        if (i < j) std::swap(a[i], a[j]);
    }
    for (int len = 2; len <= n; len <<= 1) {
        const double ang = -2 * M_PI / len;
        for (int i = 0; i < n; i += len)
            for (int k = 0; k < len / 2; k++) {
                const std::complex<double> w = std::polar(1.0, ang * k);
                const auto u = a[i + k], v = a[i + k + len / 2] * w;
                a[i + k] = u + v;
                a[i + k + len / 2] = u - v;
            }
    }
    p.resize(n);
    for (int i = 0; i < n; i++) p[(i + n / 2) % n] = std::norm(a[i]);
}

struct Variant {
    const char *name;
    void (*launch)(const void *, int, const float *, float *, hipStream_t);
    double bytes_per_sample;
    bool check;
};

static void launch_generic(const void *iq, int nf, const float *tw, float *out, hipStream_t s) {
    // the generic LDS kernel instantiated at 16384 for comparison (its per-pass tables are built here)
    static float *d_tab = nullptr;
    if (!d_tab) {
        std::vector<float> tab(2 * 16384 + 4 * Plan<14>::TW_F4);
        fill_pass_tables<14>(tab, 2 * 16384);
        CK(hipMalloc(&d_tab, tab.size() * 4));
        CK(hipMemcpy(d_tab, tab.data(), tab.size() * 4, hipMemcpyHostToDevice));
    }
    CK((launch_t<14, SDRG_IQ_CS8>(iq, nf, d_tab, out, s)));
}
static void launch_k16(const void *iq, int nf, const float *tw, float *out, hipStream_t s) {
    CK((k16::launch<SDRG_IQ_CS8>(iq, nf, tw + spectrum_k16_tables_offset(), out, s)));
}

// the k16 kernel's HBM patterns alone: 16 x 8-B stores per thread at the fftshifted offsets / 32 strided
// 2-B loads per thread, persistent grid of 512 workgroups
__global__ __launch_bounds__(512) void store_bench(float *out, int n_frames) {
    const int t = threadIdx.x;
    for (int f = blockIdx.x; f < n_frames; f += gridDim.x) {
        float *o = out + (size_t)f * 16384;
#pragma unroll
        for (int r = 0; r < 16; ++r)
            *reinterpret_cast<float2 *>(o + 2 * t + ((r * 1024 + 8192) & 16383)) = make_float2((float)r, (float)f);
    }
}
__global__ __launch_bounds__(512) void load_bench(const char *iq, float *out, int n_frames) {
    const int t = threadIdx.x;
    float acc = 0.f;
    for (int f = blockIdx.x; f < n_frames; f += gridDim.x) {
        const __amdgpu_buffer_rsrc_t rs = frame_rsrc(iq + (size_t)f * 32768, 32768);
#pragma unroll
        for (int r = 0; r < 32; ++r) acc += (float)__builtin_amdgcn_raw_buffer_load_b16(rs, 2 * t, r * 1024, 0);
    }
    if (acc == 1.2345f) out[t] = acc;
}
static void launch_store(const void *, int nf, const float *, float *out, hipStream_t s) {
    hipLaunchKernelGGL(store_bench, dim3(512), dim3(512), 0, s, out, nf);
}
static void launch_load(const void *iq, int nf, const float *, float *out, hipStream_t s) {
    hipLaunchKernelGGL(load_bench, dim3(512), dim3(512), 0, s, (const char *)iq, out, nf);
}

int main(int argc, char **argv) {
    constexpr int N = 16384;
    const int B = argc > 1 ? atoi(argv[1]) : 4096;
    const char *only = argc > 2 ? argv[2] : nullptr;  // run only the variant with this exact name
    const int reps = 20;
    std::vector<int8_t> h_iq((size_t)B * N * 2);
    uint64_t x = 0x5D12;
    for (size_t i = 0; i < h_iq.size(); i++) {
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        const size_t f = i / (2 * N), n = (i / 2) % N;
        const double ph = 2 * M_PI * (500.0 + 37.0 * (f % 64)) * n / 2e6;
        const double tone = (i & 1) ? 60 * sin(ph) : 60 * cos(ph);
        h_iq[i] = (int8_t)std::max(-128.0, std::min(127.0, std::round(tone + (double)((int)(x % 17) - 8))));
    }
    void *d_iq;
    float *d_out, *d_tw;
    CK(hipMalloc(&d_iq, h_iq.size()));
    CK(hipMalloc(&d_out, (size_t)B * N * 4));
    std::vector<float> tw(spectrum_twiddle_floats(N));
    spectrum_fill_twiddles(N, tw.data());
    CK(hipMalloc(&d_tw, tw.size() * 4));
    CK(hipMemcpy(d_tw, tw.data(), tw.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_iq, h_iq.data(), h_iq.size(), hipMemcpyHostToDevice));

    const int check_frames[] = {0, 1, 63, B / 2, B - 1};
    std::vector<std::vector<double>> ref;
    for (int f : check_frames) {
        ref.emplace_back();
        cpu_power(h_iq.data() + (size_t)f * 2 * N, N, ref.back());
    }

    Variant vs[] = {{"generic", launch_generic, 6.0, true}, {"k16", launch_k16, 6.0, true},
                    {"store-pattern", launch_store, 4.0, false}, {"load-pattern", launch_load, 2.0, false}};
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<float> h_out((size_t)N);
    for (auto &v : vs) {
        if (only && strcmp(only, v.name) != 0) continue;
        CK(hipMemset(d_out, 0xff, (size_t)B * N * 4));
        v.launch(d_iq, B, d_tw, d_out, s);
        CK(hipStreamSynchronize(s));
        int bad = 0;
        double worst = 0;
        for (int c = 0; c < 5 && v.check; c++) {
            CK(hipMemcpy(h_out.data(), d_out + (size_t)check_frames[c] * N, N * 4, hipMemcpyDeviceToHost));
            const double mx = *std::max_element(ref[c].begin(), ref[c].end());
            for (int i = 0; i < N; i++) {
                const double d = fabs(h_out[i] - ref[c][i]), tol = 1e-4 * ref[c][i] + 1e-6 * mx;
                worst = std::max(worst, d / tol);
                bad += !(d <= tol);
            }
        }
        std::vector<float> ms;
        for (int r = 0; r < reps; r++) {
            CK(hipEventRecord(e0, s));
            v.launch(d_iq, B, d_tw, d_out, s);
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float t;
            CK(hipEventElapsedTime(&t, e0, e1));
            ms.push_back(t);
        }
        std::sort(ms.begin(), ms.end());
        const double med = ms[reps / 2];
        const double gbs = v.bytes_per_sample * N * (double)B / (med * 1e-3) / 1e9;
        printf("%-14s %8.1f us  %7.1f GB/s  (%.1f%% of 8 TB/s)  min %.1f us", v.name, med * 1e3, gbs, gbs / 80.0, ms[0] * 1e3);
        if (v.check) {
            // FNV-1a over every output bit pattern: equal hashes = the same spectra bit for bit
            std::vector<uint32_t> all((size_t)B * N);
            CK(hipMemcpy(all.data(), d_out, all.size() * 4, hipMemcpyDeviceToHost));
            uint64_t h = 1469598103934665603ull;
            for (uint32_t w : all) h = (h ^ w) * 1099511628211ull;
            printf("  check: %d bad, worst err/tol %.3f, bits %016llx", bad, worst, (unsigned long long)h);
        }
        printf("\n");
    }
    return 0;
}

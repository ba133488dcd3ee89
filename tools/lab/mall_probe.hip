// Lab: does the 256 MiB Infinity Cache serve a re-used working set faster than HBM?  (Would a four-step FFT whose
// intermediate stays in a small ring gain?)  For footprints from 8 MiB to 2 GiB, timed over repeated launches on the
// same buffers after one untimed launch:
//   copy    dst[i] = src[i]   (footprint 2 x R; read + write bytes / time), default policy and nontemporal
//   read    a reduction over R bytes (read bytes / time)
//   write   dst[i] = constant over R bytes (write bytes / time)
//   w->r    the four-step's shape: kernel 1 writes Y (R bytes) from a 16x smaller input, kernel 2 reads Y and writes a
//           16x smaller output (bytes of Y written + read / time)
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/lab/mall_probe tools/lab/mall_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float v4 __attribute__((ext_vector_type(4)));

template <bool NT>
__global__ __launch_bounds__(256) void copy_k(const v4 *__restrict__ a, v4 *__restrict__ b, size_t n) {
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        if constexpr (NT) __builtin_nontemporal_store(__builtin_nontemporal_load(a + i), b + i);
        else b[i] = a[i];
    }
}

__global__ __launch_bounds__(256) void read_k(const v4 *__restrict__ a, size_t n, float *out) {
    v4 acc = {0, 0, 0, 0};
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) acc += a[i];
    const float s = acc.x + acc.y + acc.z + acc.w;
    if (s == 1.2345f) out[0] = s;
}

__global__ __launch_bounds__(256) void write_k(v4 *__restrict__ b, size_t n) {
    const v4 c = {1, 2, 3, 4};
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) b[i] = c;
}

// Y[i] = in[i / 16] (each input v4 feeds 16 Y v4s), then out[j] = sum of Y[16 j .. 16 j + 15]
__global__ __launch_bounds__(256) void expand_k(const v4 *__restrict__ in, v4 *__restrict__ y, size_t n) {
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) y[i] = in[i >> 4];
}
__global__ __launch_bounds__(256) void reduce_k(const v4 *__restrict__ y, v4 *__restrict__ out, size_t n) {
    for (size_t j = blockIdx.x * 256 + threadIdx.x; j < n / 16; j += (size_t)gridDim.x * 256) {
        v4 acc = {0, 0, 0, 0};
#pragma unroll
        for (int k = 0; k < 16; ++k) acc += y[16 * j + k];  // lane-strided, but every line is used whole by the wave
        out[j] = acc;
    }
}

int main() {
    const size_t MAXB = (size_t)2 << 30;
    v4 *a, *b, *c;
    float *o;
    if (hipMalloc(&a, MAXB) != hipSuccess || hipMalloc(&b, MAXB) != hipSuccess || hipMalloc(&c, MAXB / 8) != hipSuccess ||
        hipMalloc(&o, 64) != hipSuccess)
        return 2;
    if (hipMemset(a, 0, MAXB) != hipSuccess || hipMemset(c, 0, MAXB / 8) != hipSuccess) return 3;
    hipEvent_t t0, t1;
    (void)hipEventCreate(&t0);
    (void)hipEventCreate(&t1);
    const int grid = 256 * 16;
    auto timed = [&](auto &&launch, int reps) {
        launch();
        (void)hipEventRecord(t0, 0);
        for (int r = 0; r < reps; ++r) launch();
        (void)hipEventRecord(t1, 0);
        (void)hipEventSynchronize(t1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, t0, t1);
        return ms / reps;
    };
    printf("%10s %12s %12s %12s %12s %14s\n", "R MiB", "copy GB/s", "copy nt", "read GB/s", "write GB/s", "w->r Y GB/s");
    for (size_t mib : {8, 16, 32, 48, 64, 96, 128, 192, 256, 384, 512, 1024, 2048}) {
        const size_t bytes = mib << 20, n = bytes / 16;
        const int reps = mib <= 64 ? 200 : mib <= 256 ? 50 : 10;
        const float mc = timed([&] { hipLaunchKernelGGL(copy_k<false>, dim3(grid), dim3(256), 0, 0, a, b, n / 2); }, reps);
        const float mn = timed([&] { hipLaunchKernelGGL(copy_k<true>, dim3(grid), dim3(256), 0, 0, a, b, n / 2); }, reps);
        const float mr = timed([&] { hipLaunchKernelGGL(read_k, dim3(grid), dim3(256), 0, 0, a, n, o); }, reps);
        const float mw = timed([&] { hipLaunchKernelGGL(write_k, dim3(grid), dim3(256), 0, 0, b, n); }, reps);
        const float mx = timed([&] {
            hipLaunchKernelGGL(expand_k, dim3(grid), dim3(256), 0, 0, c, b, n);
            hipLaunchKernelGGL(reduce_k, dim3(grid), dim3(256), 0, 0, b, c, n);
        }, reps);
        if (hipGetLastError() != hipSuccess) return 4;
        // copy: footprint R (R/2 read + R/2 written)
        printf("%10zu %12.0f %12.0f %12.0f %12.0f %14.0f\n", mib, bytes / (mc * 1e6), bytes / (mn * 1e6), bytes / (mr * 1e6),
               bytes / (mw * 1e6), 2.0 * bytes / (mx * 1e6));
        fflush(stdout);
    }
    return 0;
}

// Lab probe (not product): where do the waves of a 256-thread workgroup land?  Launches 1024 workgroups of 4 waves
// with 36 KiB of dynamic LDS (the wide statistics kernel's shape: four workgroups per CU) and records each wave's
// HW_ID / XCC_ID, then reports whether a workgroup's waves sit on four distinct SIMDs and whether the thread-group
// slots (TG_ID) of the workgroups sharing a CU are distinct mod 4.
//   hipcc --offload-arch=gfx950 -O2 tools/lab/hwid_probe.hip -o tools/lab/hwid_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <map>
#include <set>
#include <tuple>
#include <vector>

__global__ void probe(unsigned *out, int spin) {
    extern __shared__ float lds[];
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    lds[threadIdx.x] = (float)threadIdx.x;
    __syncthreads();
    // hold the CU long enough that every workgroup is resident at once
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    while (__builtin_amdgcn_s_memtime() - t0 < (unsigned long long)spin) __builtin_amdgcn_s_sleep(8);
    if ((threadIdx.x & 63) == 0) {
        out[(blockIdx.x * 4 + threadIdx.x / 64) * 2] = hw;
        out[(blockIdx.x * 4 + threadIdx.x / 64) * 2 + 1] = xcc + (lds[(threadIdx.x + 64) & 255] > 1e9f ? 1 : 0);
    }
}

int main() {
    const int B = 1024;
    unsigned *d;
    if (hipMalloc(&d, B * 4 * 2 * 4) != hipSuccess) return 1;
    hipLaunchKernelGGL(probe, dim3(B), dim3(256), 36 * 1024, 0, d, 200000);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    std::vector<unsigned> h(B * 8);
    hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
    int distinct = 0, tg_ok = 0, cus = 0;
    std::map<std::tuple<unsigned, unsigned, unsigned, unsigned>, std::vector<int>> by_cu;  // (xcc, se, sh, cu) -> blocks
    for (int b = 0; b < B; b++) {
        unsigned m = 0;
        for (int w = 0; w < 4; w++) m |= 1u << ((h[(b * 4 + w) * 2] >> 4) & 3);
        distinct += m == 15;
        const unsigned hw = h[b * 8], xcc = h[b * 8 + 1];
        by_cu[{xcc, (hw >> 13) & 7, (hw >> 12) & 1, (hw >> 8) & 15}].push_back(b);
    }
    for (auto &kv : by_cu) {
        cus++;
        std::set<unsigned> tgs;
        for (int b : kv.second) tgs.insert((h[b * 8] >> 16) & 3);
        tg_ok += tgs.size() == kv.second.size();
    }
    printf("blocks %d, waves on 4 distinct SIMDs: %d; CUs seen %d, CUs whose blocks have distinct TG_ID mod 4: %d\n", B,
           distinct, cus, tg_ok);
    for (int b = 0; b < 12; b++) {
        printf("block %4d xcc %u:", b, h[b * 8 + 1]);
        for (int w = 0; w < 4; w++) {
            const unsigned hw = h[(b * 4 + w) * 2];
            printf("  w%d simd %u slot %u cu %u sh %u se %u tg %u", w, (hw >> 4) & 3, hw & 15, (hw >> 8) & 15, (hw >> 12) & 1,
                   (hw >> 13) & 7, (hw >> 16) & 15);
        }
        printf("\n");
    }
    int shown = 0;
    for (auto &kv : by_cu) {
        if (shown++ >= 4) break;
        printf("cu (xcc %u se %u sh %u cu %u): blocks", std::get<0>(kv.first), std::get<1>(kv.first), std::get<2>(kv.first),
               std::get<3>(kv.first));
        for (int b : kv.second) printf(" %d(tg %u)", b, (h[b * 8] >> 16) & 15);
        printf("\n");
    }
    return 0;
}

"""Lab: how the low-pass wave's chunk I/O costs it (VERDICT r5 item 1 follow-up).  Generates tools/lab/lpf_io.hip: the
product's interleaved low-pass chain (tools/gen/gen_lpf_asm.py lpf_sample: 2 v_pk_mul_f32 + 4 dependent v_add_f32 per
sample, 16-sample sub-blocks in three rotating register buffers) on one wave alone, with the per-quad I/O done in
different ways, s_memtime cycles per sample:
  none      the chain on registers only
  lds_rw    the product: after each 4-sample quad one ds_write_b128 (the quad) and one ds_read_b128 (sub-block + 2)
  lds_r     the reads only;  lds_w  the writes only
  lds_rw2   the write after the quad's 2nd add of its last sample, the read after the 4th (two bubbles instead of one)
  vm_rw     global_store_dwordx4 + global_load_dwordx4 (sc0 sc1: past L1) instead, waits on vmcnt
  vm_r / vm_w
  bar       lds_rw + the product's per-chunk `s_waitcnt lgkmcnt(1); s_barrier` with 11 more waves in the workgroup that
            only meet the barrier
  cnt       lds_rw + a chunk-counter check instead (SDRG_PIPE_FLAGS form): two counter reads at sub-block 2's start,
            at the chunk's end v_min3 x 2 + 2 v_cmp + s_and + branch, then one lane's ds_add_u32 (exec switched by SALU)
  cnt_il    as cnt with the check's VALU in the chain's dependency bubbles (after add 2 of samples 1, 5, 9, 13 of the
            chunk's last sub-block)
EXEC: 16 lanes (the product's 16 streams) and 64.
Run: python tools/lab/gen_lpf_io.py > tools/lab/lpf_io.hip && hipcc --offload-arch=gfx950 -O3 -o tools/lab/lpf_io tools/lab/lpf_io.hip
"""
import sys

sys.path.insert(0, __file__.rsplit("/", 2)[0] + "/gen")
from gen_lpf_asm import BUFS, lpf_sample, pair  # noqa: E402

ROWB = 68 * 4  # the product's padded stream row (bytes)


def io_ops(kind, b, t, rb, sb2, first_half):
    """I/O after quad t of the sub-block in buffer b; rb: buffer of sub-block + 2 (reads target)"""
    w_lds = f"ds_write_b128 %[dst], v[{b + 4 * t}:{b + 4 * t + 3}] offset:{(sb2 * 16 + 4 * t) * 4}"
    r_lds = f"ds_read_b128 v[{rb + 4 * t}:{rb + 4 * t + 3}], %[src] offset:{(sb2 * 16 + 4 * t) * 4}"
    w_vm = f"global_store_dwordx4 %[gdst], v[{b + 4 * t}:{b + 4 * t + 3}], off offset:{(sb2 * 16 + 4 * t) * 4}"
    r_vm = f"global_load_dwordx4 v[{rb + 4 * t}:{rb + 4 * t + 3}], %[gsrc], off offset:{(sb2 * 16 + 4 * t) * 4} sc0 sc1"
    o8 = (sb2 * 16 + 4 * t) // 2  # 8-byte units
    w2 = f"ds_write2_b64 %[dst], v[{b + 4 * t}:{b + 4 * t + 1}], v[{b + 4 * t + 2}:{b + 4 * t + 3}] offset0:{o8} offset1:{o8 + 1}"
    wb64 = [f"ds_write_b64 %[dst], v[{b + 4 * t}:{b + 4 * t + 1}] offset:{o8 * 8}",
            f"ds_write_b64 %[dst], v[{b + 4 * t + 2}:{b + 4 * t + 3}] offset:{o8 * 8 + 8}"]
    w_vm1 = w_vm + " sc1"
    return {"none": [], "lds_rw": [w_lds, r_lds], "lds_r": [r_lds], "lds_w": [w_lds], "vm_rw": [w_vm, r_vm],
            "vm_r": [r_vm], "vm_w": [w_vm], "lds_w2": [w2], "lds_wb64": wb64, "vm_w1": [w_vm1],
            "lr_vw": [w_vm, r_lds]}[kind]


CHECK = ["v_min3_i32 v56, v56, v57, v58", "v_min3_i32 v56, v56, v59, v60", "v_cmp_le_i32 vcc, %[t2], v56",
         "v_cmp_le_i32 %[tm], %[t2], v61"]


def chunk_loop(kind):
    """64 samples (4 sub-blocks), buffers rotate (sub-block g in BUFS[g % 3]); the I/O keeps the product's counts"""
    if kind in ("bar", "cnt", "cnt_il"):
        out = []
        prev1, prev2 = pair(BUFS[2] + 15), pair(BUFS[2] + 14)
        for g in range(12):
            sb = g % 4
            b = BUFS[g % 3]
            rb = BUFS[(g + 2) % 3]
            out.append("s_waitcnt lgkmcnt(8)")
            if kind != "bar" and sb == 2:
                out += ["ds_read_b128 v[56:59], %[pb]", "ds_read_b64 v[60:61], %[pb] offset:16"]
            ci = 0
            for q in range(16):
                smp = lpf_sample(b + q, prev1, prev2)
                if kind == "cnt_il" and sb == 3 and q % 4 == 1 and ci < 4:
                    out += smp[:4] + [CHECK[ci]] + smp[4:]
                    ci += 1
                else:
                    out += smp
                if q % 4 == 3:
                    out += io_ops("lds_rw", b, q // 4, rb, sb, True)
                prev2, prev1 = prev1, pair(b + q)
            if sb == 3:
                if kind == "bar":
                    out += ["s_waitcnt lgkmcnt(1)", "s_barrier"]
                else:
                    if kind == "cnt":
                        out += CHECK
                    out += ["s_and_b64 vcc, vcc, %[tm]", "s_cbranch_vccz 1f", "1:",
                            "s_mov_b64 %[sv], exec", "s_mov_b64 exec, 1", "ds_add_u32 %[pb], v62 offset:24",
                            "s_mov_b64 exec, %[sv]"]
        return out
    out = []
    vm = kind.startswith("vm")
    wait = "s_waitcnt vmcnt({})" if vm else "s_waitcnt lgkmcnt({})"
    per_quad = 0 if kind == "none" else (2 if kind.endswith("rw") or kind in ("lds_rw2", "lds_wb64") else 1)
    if kind == "lr_vw":  # LDS reads, global stores: lgkmcnt counts only the reads
        vm, per_quad = False, 1
    prev1, prev2 = pair(BUFS[2] + 15), pair(BUFS[2] + 14)
    for g in range(12):  # three chunks so the buffer rotation returns to its start
        sb = g % 4
        b = BUFS[g % 3]
        rb = BUFS[(g + 2) % 3]
        if per_quad:
            out.append(wait.format(min(4 * per_quad, 15) if vm else 4 * per_quad))
        for q in range(16):
            smp = lpf_sample(b + q, prev1, prev2)
            if kind == "lds_rw2" and q % 4 == 3:
                t = q // 4
                ops = io_ops("lds_rw", b, t, rb, sb, True)
                out += smp[:4] + [ops[0]] + smp[4:] + [ops[1]]
            else:
                out += smp
                if q % 4 == 3 and kind not in ("none", "lds_rw2"):
                    out += io_ops(kind, b, q // 4, rb, sb, True)
            prev2, prev1 = prev1, pair(b + q)
    return out


def main():
    kinds = ["none", "lds_rw", "lds_r", "lds_w", "lds_rw2", "vm_rw", "vm_r", "vm_w", "bar", "cnt", "cnt_il", "lds_w2",
             "lds_wb64", "vm_w1", "lr_vw"]
    print("// Generated by tools/lab/gen_lpf_io.py -- lab microbenchmark, not product code")
    print("#include <hip/hip_runtime.h>\n#include <stdio.h>\n#include <stdint.h>")
    print("constexpr int REP = 64;  // x 3 chunks x 64 samples")
    print(f"constexpr int BAR_K = {kinds.index('bar')};  // the variant launched with 12 waves")
    for k in kinds:
        print(f"#define BODY_{k.upper()} \\")
        for l in chunk_loop(k):
            print(f'    "{l}\\n" \\')
        print('    ""')
    print("""
typedef float f2v __attribute__((ext_vector_type(2)));
template <int K>
__global__ __launch_bounds__(768) void k(float *gbuf, unsigned long long *out, unsigned long long mask) {
    __shared__ __attribute__((aligned(16))) float lds[16 * 68 * 4];
    __shared__ __attribute__((aligned(16))) int prog[16];
    const int lane = threadIdx.x & 63;
    if (threadIdx.x < 16) prog[threadIdx.x] = 1 << 20;
    if (threadIdx.x >= 64) {  // the other waves of the 12-wave launch (bar): meet every barrier of wave 0
        __syncthreads();
        for (int r = 0; r < REP * 3; r++) __builtin_amdgcn_s_barrier();
        return;
    }
    const uint32_t pb = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) int *)&prog[0];
    unsigned long long sv, tm;
    const int s = lane & 15;
    const uint32_t src = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) float *)&lds[s * 68];
    const uint32_t dst = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) float *)&lds[16 * 68 + s * 68];
    float *gsrc = gbuf + s * 68;
    float *gdst = gbuf + 16 * 68 * 4 + s * 68;
    for (int i = lane; i < 16 * 68 * 4; i += 64) lds[i] = 0.001f * i;
    __syncthreads();
    const int t2 = 0;
    const f2v c1 = {0.5f, -0.25f}, c2 = {0.125f, -0.0625f};
    unsigned long long t0 = 0, t1 = 0;
    if ((mask >> lane) & 1) {
        asm volatile("v_mov_b32 v46, 0.5\\n v_mov_b32 v47, 0.25\\n v_mov_b32 v62, 1\\n" ::: "v46", "v47", "v62");
        t0 = __builtin_amdgcn_s_memtime();
        for (int r = 0; r < REP; r++) {
#define RUN(B) asm volatile(B "s_waitcnt vmcnt(0) lgkmcnt(0)\\n" : [sv] "=&s"(sv), [tm] "=&s"(tm) : [src] "v"(src), [dst] "v"(dst), [gsrc] "v"(gsrc), [gdst] "v"(gdst), [c1] "s"(c1), [c2] "s"(c2), [pb] "v"(pb), [t2] "s"(t2) : \\
    "v0","v1","v2","v3","v4","v5","v6","v7","v8","v9","v10","v11","v12","v13","v14","v15","v16","v17","v18","v19","v20", \\
    "v21","v22","v23","v24","v25","v26","v27","v28","v29","v30","v31","v32","v33","v34","v35","v36","v37","v38","v39", \\
    "v40","v41","v42","v43","v44","v45","v46","v47","v48","v49","v50","v51","v56","v57","v58","v59","v60","v61","vcc","memory")""")
    for i, k in enumerate(kinds):
        print(f"            {'if' if i == 0 else 'else if'} constexpr (K == {i}) RUN(BODY_{k.upper()});")
    print("""        }
        t1 = __builtin_amdgcn_s_memtime();
    }
    if (lane == __builtin_ctzll(mask)) out[0] = t1 - t0;
}
__global__ void warm(float *x, int n) {
    float a = x[threadIdx.x];
    for (int i = 0; i < n; i++) a = a * 1.0000001f + 1e-7f;
    x[threadIdx.x] = a;
}
template <int K>
void run(const char *name, float *g, unsigned long long *d, unsigned long long mask) {
    unsigned long long h = 0, best = ~0ull;
    for (int r = 0; r < 8; r++) {  // the minimum of the last 5 of 8 launches
        k<K><<<1, K == BAR_K ? 768 : 64>>>(g, d, mask);
        if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost) != hipSuccess) return;
        if (r >= 3 && h < best) best = h;
    }
    printf("%-8s exec %016llx: %6.2f cyc/sample\\n", name, mask, best / (double)(REP * 3 * 64));
}
int main() {
    unsigned long long *d;
    float *g;
    if (hipMalloc(&d, 64) != hipSuccess || hipMalloc(&g, 1 << 20) != hipSuccess) return 2;
    if (hipMemset(g, 0, 1 << 20) != hipSuccess) return 2;
    hipLaunchKernelGGL(warm, dim3(1024), dim3(256), 0, 0, g, 1 << 18);  // a few ms of work so the clocks settle
    if (hipDeviceSynchronize() != hipSuccess) return 3;
    for (unsigned long long m : {0xffffull, ~0ull}) {""")
    for i, k in enumerate(kinds):
        print(f'        run<{i}>("{k}", g, d, m);')
    print("""    }
    return 0;
}""")


if __name__ == "__main__":
    main()

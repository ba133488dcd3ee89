// ssb64.hip — processSSB_opt (src/ssb/ssb_demod_opt.cpp:221-296) with 64 streams per serial wave.
//
// The chain's three sample-serial recurrences (removeDC :49-55, the iir2 low-pass :75-84, the AGC gain :101-115) bound a
// frame's time, and in ssb.hip's pipeline each of them runs on a wave whose 16 stream lanes leave 48 idle: a wave64
// VALU instruction occupies its SIMD for the same cycles with 16 lanes as with 64, and a dependent chain issues more
// slowly under a partial EXEC mask.  Here every role of the chain processes 64 streams, one per lane,
// so the three recurrences run on full waves and 4096 streams need 64 groups instead of 256 -- and the order-free work
// around them (unpack, the AGC's desired level, the clamp, the FIR, the equaliser) grows fourfold per group, more than
// one CU's VALU and LDS hold beside the recurrences.  A group therefore spans two workgroups:
//
//   front (4 waves): loader (raw IQ -> I floats) | removeDC + a0 x | low-pass | exporter (low-pass output y out)
//   back (12 waves): importer (y in) | desired level x 4 | AGC gain | clamp | FIR x 4 | equaliser + PCM (+ the audio
//                    pulse detector's front end)
//
// both pipelined over 64-sample chunks through LDS rings with one LDS-only barrier per chunk, as ssb.hip.  All arithmetic
// is the reference's, in its order, without contraction (bit-identical PCM); the three recurrences run the same
// hand-scheduled asm blocks as ssb.hip (csrc/ssb_lpf_asm.h, tools/gen/gen_lpf_asm.py), on all 64 lanes.
//
// Hand-off (this file's first form, SSB64_SCRATCH): the front writes each group's y rows to an HBM scratch
// [stream][samp_count] and the back kernel, launched after it, reads them -- two kernels, no cross-workgroup protocol.
#include <hip/hip_ext.h>
#include <stdio.h>

#include <vector>

#include "pulse_front.h"
#include "sdrg_internal.h"
#include "ssb_common.h"
#include "ssb_lpf_asm.h"
#include "ssb64_lpf_asm.h"
#include "ssb_math.h"

#pragma clang fp contract(off)

namespace sdrg {
namespace {

constexpr int G64 = 64;          // streams per group: one per lane of every role
constexpr int C64 = 64;          // samples per chunk
constexpr int R64 = C64 + 4;     // padded stream row (floats): conflict-free ds_read_b128 by stream lanes
constexpr int SL64 = G64 * R64;  // floats per [stream][sample] chunk slot
static_assert(SL64 * 4 == SDRG_LPF64_LOOP_SLOT_BYTES, "ring slot stride of the generated 64-lane low-pass loop");
constexpr int MAXD64 = 8;        // FIR outputs completed per stream per chunk (at most)
constexpr int NFIR = 4;          // FIR waves; each holds NSL / NFIR output slots of every stream
constexpr int MAXSL64 = 16;      // output slots per stream (NSL) at most: NSL / NFIR <= 4 per wave
constexpr int TAPS64_ROW = C64 + 256 + C64 + 4;

// ---- front workgroup ----
enum FrontRole : int { FR_LPF = 0, FR_DC = 1, FR_LOAD = 2, FR_EXP = 3 };
constexpr int FRONT_T = 4 * 64;
struct FrontLds {
    float re[2][SL64];  // loader -> DC (chunk c at iteration c)
    float a[3][SL64];   // DC (a0 x) -> low-pass: three slots, the low-pass reads the next chunk's first sub-blocks ahead
    float y[2][SL64];   // low-pass -> exporter
};

// raw-IQ chunks the front's loader keeps in flight by LDS-DMA (8 KiB per chunk at CS8, 16 KiB at CS16)
template <int FMT>
constexpr int front_raw_chunks() {
    return bytes_per_sample<FMT>() == 2 ? 4 : 2;
}
template <int FMT>
constexpr size_t front_lds_bytes() {
    return sizeof(FrontLds) + (size_t)front_raw_chunks<FMT>() * C64 * bytes_per_sample<FMT>() * G64;
}

// Lab (SDRG_SSB64_STAMPS): per wave, the cycles of its own work (body to its last LDS operation) and of its whole
// loop, at stamps[(group * 16 + slot) * 2 + {0, 1}] (front roles in slots 0-3, back roles in 4-15); null: nothing runs
#ifndef SSB64_SKIP_LOAD  // lab diagnostic (wrong results): the loader does no work, so the front's loop shows the
#define SSB64_SKIP_LOAD 0  // serial roles' own rate
#endif
#define SSB64_WORK_BEGIN() const unsigned long long st_a_ = stamps ? __builtin_amdgcn_s_memtime() : 0
#define SSB64_WORK_END()                                                                                       \
    do {                                                                                                       \
        if (stamps) {                                                                                          \
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                                 \
            st_work += __builtin_amdgcn_s_memtime() - st_a_;                                                   \
        }                                                                                                      \
    } while (0)
__device__ __forceinline__ void ssb64_stamp(unsigned long long *stamps, int slot, unsigned long long work,
                                            unsigned long long t0) {
    if (stamps && (threadIdx.x & 63) == 0) {
        stamps[(blockIdx.x * 16 + slot) * 2] = work;
        stamps[(blockIdx.x * 16 + slot) * 2 + 1] = __builtin_amdgcn_s_memtime() - t0;
    }
}

template <int FMT>
__global__ __attribute__((amdgpu_flat_work_group_size(FRONT_T, FRONT_T))) void ssb64_front_kernel(
    const char *__restrict__ iq, int n_frames, SsbParams p, SsbStreamState *__restrict__ state, float *__restrict__ ys,
    unsigned long long *__restrict__ stamps) {
    extern __shared__ __attribute__((aligned(16))) char dyn[];
    FrontLds &L = *reinterpret_cast<FrontLds *>(dyn);
    const unsigned long long st_t0 = stamps ? __builtin_amdgcn_s_memtime() : 0;
    unsigned long long st_work = 0;
    const int tid = threadIdx.x, lane = tid & 63;
    const int role = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int s = blockIdx.x * G64 + lane;
    const bool live = s < n_frames;
    const int S = p.samp_count, nch = S / C64;
    const int nit = nch + 4;  // load c = it | DC c = it - 1 | low-pass c = it - 3 (lookahead) | export c = it - 4
    if (role == FR_LPF) {
        // iir2Process (:75-84): y = ((((a0 x + a1 z1) + a2 z2) - b1 z1) - b2 z2), the products as two packed multiplies
        float z1 = 0.0f, z2 = 0.0f;  // rfFilter state, carried across frames
        if (live) {
            z1 = state[s].lpf_z1;
            z2 = state[s].lpf_z2;
        }
        const f2v c1 = {p.lpf[1], -p.lpf[3]}, c2 = {p.lpf[2], -p.lpf[4]};
        f2v z = {z1, z2};
        const uint32_t abase = lds_addr(&L.a[0][lane * R64]), ybase = lds_addr(&L.y[0][lane * R64]);
        unsigned long long sv;
        int t_it, t_cc, t_r, t_yo;
        __builtin_amdgcn_s_setprio(3);
        asm volatile(SDRG_LPF64_LOOP_IL_ASM
                     : [z] "+v"(z), [sv] "=&s"(sv), [it] "=&s"(t_it), [cc] "=&s"(t_cc), [r] "=&s"(t_r), [yo] "=&s"(t_yo)
                     : [abase] "v"(abase), [ybase] "v"(ybase), [c1] "s"(c1), [c2] "s"(c2), [nit] "s"(nit), [nch] "s"(nch)
                     : SDRG_CHUNK_CLOBBERS, "v54", "memory");
        __builtin_amdgcn_s_setprio(0);
        if (live) {
            state[s].lpf_z1 = z.x;
            state[s].lpf_z2 = z.y;
        }
        ssb64_stamp(stamps, FR_LPF, 0, st_t0);
    } else if (role == FR_DC) {
        // removeDC (:49-55), reset per call, and iir2Process's a0 x product
        float dc = 0.0f;
        const float alpha = 0.9995f, one_minus = 1.0f - 0.9995f, a0 = p.lpf[0];
        const f2v om2 = {one_minus, one_minus}, a02 = {a0, a0};
        __builtin_amdgcn_s_setprio(3);
        for (int it = 0; it < nit; ++it) {
            const int c = it - 1;
            SSB64_WORK_BEGIN();
            if (c >= 0 && c < nch) {
                const uint32_t src = lds_addr(&L.re[c & 1][lane * R64]), dst = lds_addr(&L.a[c % 3][lane * R64]);
                asm volatile(SDRG_DC_CHUNK_IL_ASM
                             : [dc] "+v"(dc)
                             : [src] "v"(src), [dst] "v"(dst), [alpha] "s"(alpha), [om2] "s"(om2), [a02] "s"(a02)
                             : SDRG_CHUNK_CLOBBERS, "memory");
            }
            SSB64_WORK_END();
            lds_barrier();
        }
        __builtin_amdgcn_s_setprio(0);
        ssb64_stamp(stamps, FR_DC, st_work, st_t0);
    } else if (role == FR_LOAD) {
        // the I channel of chunk c (lane = stream): the streams' raw bytes move by LDS-DMA into a ring of NRW chunks,
        // issued NRW - 1 chunks ahead: each DMA instruction moves whole chunk rows (U4 lanes per stream, 16 B each), so
        // the ring holds [chunk][stream][piece]; each lane then unpacks its own row into the re ring, visiting its
        // pieces in a lane-rotated order (conflict-free LDS reads) and writing each piece's samples where they belong
        constexpr int BPS = bytes_per_sample<FMT>();
        constexpr int U4 = C64 * BPS / 16;  // 16-B pieces per chunk and stream: CS8/CU8 8, CS16 16
        constexpr int PER8 = U4 / 8;        // pieces per 8 samples
        constexpr int SPI = G64 / U4;       // streams per DMA instruction
        constexpr int NRW = front_raw_chunks<FMT>();
        static_assert((NRW - 1) * U4 <= 63, "vmcnt immediates");
        uint4 *raw = reinterpret_cast<uint4 *>(dyn + sizeof(FrontLds));
        const int dma_k = lane / U4, dma_i = lane % U4;  // this lane's stream within an instruction's SPI, and piece
        auto issue = [&](int c) {
#pragma unroll
            for (int j = 0; j < U4; j++) {
                const int st = blockIdx.x * G64 + j * SPI + dma_k;
                const char *row = iq + (size_t)(st < n_frames ? st : blockIdx.x * G64) * p.n_in * BPS;
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(row + (size_t)c * C64 * BPS + 16 * dma_i),
                                                 (__attribute__((address_space(3))) void *)&raw[((c % NRW) * G64 + j * SPI) * U4], 16, 0, 0);
            }
        };
        for (int c = 0; c < NRW - 1 && c < nch && !SSB64_SKIP_LOAD; c++) issue(c);
        for (int it = 0; it < nit; ++it) {
            SSB64_WORK_BEGIN();
            if (it < nch && !SSB64_SKIP_LOAD) {
                if (it + NRW - 1 < nch) issue(it + NRW - 1);
                // chunk it has landed once at most the younger chunks' pieces are in flight
                const int younger = min(NRW - 1, nch - 1 - it);
                if (younger >= 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * U4 > 63 ? 63 : 3 * U4) : "memory");
                else if (younger == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * U4 > 63 ? 63 : 2 * U4) : "memory");
                else if (younger == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(U4) : "memory");
                else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                const uint4 *mine = &raw[((it % NRW) * G64 + lane) * U4];
                float *dst = &L.re[it & 1][lane * R64];
#pragma unroll
                for (int k = 0; k < 8; k++) {
                    const int g8 = (k + lane) & 7;  // lane-rotated: the 16 lanes of a read group hit distinct banks
                    uint4 r[PER8];
#pragma unroll
                    for (int i = 0; i < PER8; i++) r[i] = mine[g8 * PER8 + i];
                    float x[8];
                    unpack_i8<FMT>(r, x);
                    if (!live) {
#pragma unroll
                        for (int q = 0; q < 8; q++) x[q] = 0.0f;
                    }
                    *reinterpret_cast<float4 *>(dst + 8 * g8) = make_float4(x[0], x[1], x[2], x[3]);
                    *reinterpret_cast<float4 *>(dst + 8 * g8 + 4) = make_float4(x[4], x[5], x[6], x[7]);
                }
            }
            SSB64_WORK_END();
            lds_barrier();
        }
        ssb64_stamp(stamps, FR_LOAD, st_work, st_t0);
    } else {
        // exporter: chunk c's low-pass output rows to the group's y scratch
        for (int it = 0; it < nit; ++it) {
            const int c = it - 4;
            SSB64_WORK_BEGIN();
            if (c >= 0 && c < nch) {
                // [group][chunk][quad][stream] float4: each store instruction writes 1 KiB contiguous
                const float4 *src = reinterpret_cast<const float4 *>(&L.y[c & 1][lane * R64]);
                float4 *dst = reinterpret_cast<float4 *>(ys) + ((size_t)blockIdx.x * nch + c) * (C64 / 4) * G64 + lane;
#pragma unroll
                for (int j = 0; j < C64 / 4; j++) dst[j * G64] = src[j];
            }
            SSB64_WORK_END();
            lds_barrier();
        }
        ssb64_stamp(stamps, FR_EXP, st_work, st_t0);
    }
}

// ---- back workgroup ----
enum BackRole : int { BK_AGC = 0, BK_OUT = 1, BK_EQ = 2, BK_IMP = 3, BK_DES0 = 4, BK_FIR0 = 8 };
constexpr int NDES = 4;
constexpr int BACK_T = 12 * 64;
constexpr int NY = 6;  // y slots: chunk c lands at iteration c - 1 (LDS-DMA) and the FIR reads it at c + 4
struct BackLds {
    // importer -> desired (c-1) -> clamp (c-3, writes its output over y in place) -> FIR (c-4); [quad][stream] float4,
    // the layout LDS-DMA writes (one 1-KiB piece per quad) and stream lanes read without conflicts
    float4 y[NY][C64 / 4][G64];
    float dg[3][SL64];  // desired -> AGC gain (in place: d becomes g) -> clamp
    float fq[2][G64 * MAXD64];  // FIR outputs completed in a chunk -> equaliser
    // taps with C64 zeros on both sides (out-of-window FIR steps multiply by 0), in 4 copies shifted by 0..3 floats so
    // that any window of them is read with aligned ds_read_b128
    float taps_sh[4][TAPS64_ROW];
};

// The FIR slots of every stream of the group over one chunk (simpleFIRDecimate :121-143, k ascending): this wave holds
// slots {f, f + NFIR, ...} (NP of them); slot j holds the output o == j mod NSL active in the chunk.  Lane = stream,
// so the slot -> output map and the tap index are the same for every lane (broadcast tap reads).  Steps outside an
// output's window meet a zero tap, and acc + (+-0) == acc exactly (acc starts at +0).
template <int NP>
__device__ __forceinline__ void fir64_chunk(BackLds &L, const float4 *xq, int lane, int t0, int o_lo, int o_hi, int f,
                                            int nsl_mask, int D, int NT, float (&acc)[MAXSL64 / NFIR], float *fq_row) {
    const int t1 = t0 + C64;
    int k0[NP];
    bool done[NP];
    int slot_o[NP];
#pragma unroll
    for (int j = 0; j < NP; j++) {
        const int slot = f + NFIR * j;
        const int o = o_lo + ((slot - o_lo) & nsl_mask);
        const int base = D * o;
        const bool active = o <= o_hi;
        done[j] = active && base + NT <= t1;
        slot_o[j] = o;
        if (active && base >= t0) acc[j] = 0.0f;
        k0[j] = active ? (t0 - base + C64) : 0;  // taps_pad index of step 0 (inactive: the zero padding)
    }
    // whole chunk unrolled (the LDS reads issue ahead of the sums) where the registers allow
    if constexpr (NP <= 2) {
#pragma unroll
        for (int i = 0; i < C64 / 4; i++) {
            const float4 x = xq[i * G64 + lane];
            f2v lo[NP], hi[NP];
#pragma unroll
            for (int j = 0; j < NP; j++) {
                const float4 h = reinterpret_cast<const float4 *>(&L.taps_sh[k0[j] & 3][k0[j] & ~3])[i];
                lo[j] = f2v{x.x, x.y} * f2v{h.x, h.y};  // products are order-free: two per packed op
                hi[j] = f2v{x.z, x.w} * f2v{h.z, h.w};
            }
#pragma unroll
            for (int j = 0; j < NP; j++) acc[j] += lo[j].x;
#pragma unroll
            for (int j = 0; j < NP; j++) acc[j] += lo[j].y;
#pragma unroll
            for (int j = 0; j < NP; j++) acc[j] += hi[j].x;
#pragma unroll
            for (int j = 0; j < NP; j++) acc[j] += hi[j].y;
        }
    } else {
#pragma unroll 4
        for (int i = 0; i < C64 / 4; i++) {
            const float4 x = xq[i * G64 + lane];
            f2v lo[NP], hi[NP];
#pragma unroll
            for (int j = 0; j < NP; j++) {
                const float4 h = reinterpret_cast<const float4 *>(&L.taps_sh[k0[j] & 3][k0[j] & ~3])[i];
                lo[j] = f2v{x.x, x.y} * f2v{h.x, h.y};  // products are order-free: two per packed op
                hi[j] = f2v{x.z, x.w} * f2v{h.z, h.w};
            }
#pragma unroll
            for (int j = 0; j < NP; j++) acc[j] += lo[j].x;
#pragma unroll
            for (int j = 0; j < NP; j++) acc[j] += lo[j].y;
#pragma unroll
            for (int j = 0; j < NP; j++) acc[j] += hi[j].x;
#pragma unroll
            for (int j = 0; j < NP; j++) acc[j] += hi[j].y;
        }
    }
#pragma unroll
    for (int j = 0; j < NP; j++)
        if (done[j]) fq_row[slot_o[j] & (MAXD64 - 1)] = acc[j];
}

__global__ __attribute__((amdgpu_flat_work_group_size(BACK_T, BACK_T), amdgpu_waves_per_eu(3, 3))) void ssb64_back_kernel(
    const float *__restrict__ ys, int n_frames, SsbParams p, int nsl_mask, const int4 *__restrict__ chunk_out,
    const float *__restrict__ taps, SsbStreamState *__restrict__ state, int16_t *__restrict__ pcm, AudioFront af,
    unsigned long long *__restrict__ stamps) {
    extern __shared__ __attribute__((aligned(16))) char dyn[];
    BackLds &L = *reinterpret_cast<BackLds *>(dyn);
    const unsigned long long st_t0 = stamps ? __builtin_amdgcn_s_memtime() : 0;
    unsigned long long st_work = 0;
    const int tid = threadIdx.x, lane = tid & 63;
    const int role = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int s = blockIdx.x * G64 + lane;
    const bool live = s < n_frames;
    const int S = p.samp_count, nch = S / C64;
    const int D = p.decim, NT = p.n_taps, PL = p.pcm_len;
    const float demod_k = p.upper ? 2.0f : 0.0f;  // demodSSB(y, y) = y + y or y - y (:89-94) as y * k
    // import c = it | desired c = it - 1 | AGC c = it - 2 | clamp c = it - 3 | FIR c = it - 4 | equaliser c = it - 5
    const int nit = nch + 6;
    for (int i = tid; i < 4 * TAPS64_ROW; i += BACK_T) {
        const int sh = i / TAPS64_ROW, j = i % TAPS64_ROW;
        const int k = j + sh - C64;  // copy sh holds taps_pad[j + sh] at index j
        L.taps_sh[sh][j] = (k >= 0 && k < NT) ? taps[k] : 0.0f;
    }
    __syncthreads();
    if (role == BK_IMP) {
        // chunk c's y rows by LDS-DMA (no registers): the 16 pieces of chunk c + 1 are issued during iteration c, into
        // a slot the FIR has left, and waited for at the end of iteration c + 1
        const float4 *src = reinterpret_cast<const float4 *>(ys) + (size_t)blockIdx.x * nch * (C64 / 4) * G64 + lane;
        auto issue = [&](int c) {  // 1 KiB contiguous per instruction ([chunk][quad][stream] float4)
#pragma unroll
            for (int q = 0; q < C64 / 4; q++)
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(src + ((size_t)c * (C64 / 4) + q) * G64),
                                                 (__attribute__((address_space(3))) void *)&L.y[c % NY][q][0], 16, 0, 0);
        };
        if (nch > 0) issue(0);
        for (int it = 0; it < nit; ++it) {
            SSB64_WORK_BEGIN();
            if (it + 1 < nch) {
                issue(it + 1);
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(C64 / 4) : "memory");  // chunk it has landed
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            SSB64_WORK_END();
            lds_barrier();
        }
        ssb64_stamp(stamps, 4 + role, st_work, st_t0);
    } else if (role >= BK_DES0 && role < BK_DES0 + NDES) {
        // adaptiveAGC's desired level (:104-107) for samples [16 d, 16 d + 16) of the chunk, every stream
        const int d0 = (role - BK_DES0) * (C64 / NDES);
        for (int it = 0; it < nit; ++it) {
            SSB64_WORK_BEGIN();
            const int c = it - 1;
            if (c >= 0 && c < nch) {
                float4 *dr = reinterpret_cast<float4 *>(&L.dg[c % 3][lane * R64 + d0]);
                float4 yv[C64 / NDES / 4];
#pragma unroll
                for (int q = 0; q < C64 / NDES / 4; q++) yv[q] = L.y[c % NY][d0 / 4 + q][lane];
#pragma unroll
                for (int q = 0; q < C64 / NDES / 4; q++) {
                    // fabsf(demodSSB(y, y)) == |y| * k exactly (k = 2 or 0)
                    const f2v a = f2v{fabsf(yv[q].x), fabsf(yv[q].y)} * f2v{demod_k, demod_k};
                    const f2v b = f2v{fabsf(yv[q].z), fabsf(yv[q].w)} * f2v{demod_k, demod_k};
                    const f2v da = agc_desired_abs2(a, p.agc_target), db = agc_desired_abs2(b, p.agc_target);
                    dr[q] = make_float4(da.x, da.y, db.x, db.y);
                }
            }
            SSB64_WORK_END();
            lds_barrier();
        }
        ssb64_stamp(stamps, 4 + role, st_work, st_t0);
    } else if (role == BK_AGC) {
        // gain = gain*(1-rate) + desired*rate, rate = desired < gain ? fast : slow (:101-115), reset per call; in place
        float gain = 1.0f;
        const f2v rates = {p.agc_fast, 0.00035f};
        const f2v keep = {1.0f - p.agc_fast, 1.0f - 0.00035f};
        __builtin_amdgcn_s_setprio(3);
        for (int it = 0; it < nit; ++it) {
            SSB64_WORK_BEGIN();
            const int c = it - 2;
            if (c >= 0 && c < nch) {
                f2v g = {gain, gain};
                const uint32_t row = lds_addr(&L.dg[c % 3][lane * R64]);
                asm volatile(SDRG_AGC_CHUNK_IL_ASM
                             : [g] "+v"(g)
                             : [src] "v"(row), [dst] "v"(row), [keep] "s"(keep), [rates] "s"(rates)
                             : SDRG_CHUNK_CLOBBERS, "vcc", "memory");
                gain = g.x;
            }
            SSB64_WORK_END();
            lds_barrier();
        }
        ssb64_stamp(stamps, 4 + role, st_work, st_t0);
        __builtin_amdgcn_s_setprio(0);
    } else if (role == BK_OUT) {
        // clamp(demodSSB(y, y) * gain, -1, 1) (:108) over the y row in place (the FIR reads it next); y * k is y + y or
        // y - y exactly (the lower sideband's zero may carry y's sign, which the FIR's sums absorb: acc + (+-0) == acc)
        for (int it = 0; it < nit; ++it) {
            SSB64_WORK_BEGIN();
            const int c = it - 3;
            if (c >= 0 && c < nch) {
                const float4 *gr = reinterpret_cast<const float4 *>(&L.dg[c % 3][lane * R64]);
                const f2v k2 = {demod_k, demod_k};
#pragma unroll
                for (int q = 0; q < C64 / 4; q++) {
                    const float4 yv = L.y[c % NY][q][lane], gv = gr[q];
                    f2v o0 = (f2v{yv.x, yv.y} * k2) * f2v{gv.x, gv.y};
                    f2v o1 = (f2v{yv.z, yv.w} * k2) * f2v{gv.z, gv.w};
                    L.y[c % NY][q][lane] = make_float4(__builtin_amdgcn_fmed3f(o0.x, -1.0f, 1.0f), __builtin_amdgcn_fmed3f(o0.y, -1.0f, 1.0f),
                                        __builtin_amdgcn_fmed3f(o1.x, -1.0f, 1.0f), __builtin_amdgcn_fmed3f(o1.y, -1.0f, 1.0f));
                }
            }
            SSB64_WORK_END();
            lds_barrier();
        }
        ssb64_stamp(stamps, 4 + role, st_work, st_t0);
    } else if (role >= BK_FIR0 && role < BK_FIR0 + NFIR) {
        const int f = role - BK_FIR0;
        float facc[MAXSL64 / NFIR] = {};
        const int npw = (nsl_mask + 1) / NFIR;  // slots per FIR wave
        for (int it = 0; it < nit; ++it) {
            SSB64_WORK_BEGIN();
            const int c = it - 4;
            if (c >= 0 && c < nch && PL > 0) {
                const int4 r = chunk_out[c];  // outputs overlapping chunk c: [r.x, r.y] (host table)
                const float4 *xq = &L.y[c % NY][0][0];
                float *fq_row = &L.fq[c & 1][lane * MAXD64];
                if (npw == 4) fir64_chunk<4>(L, xq, lane, c * C64, r.x, r.y, f, nsl_mask, D, NT, facc, fq_row);
                else if (npw == 2) fir64_chunk<2>(L, xq, lane, c * C64, r.x, r.y, f, nsl_mask, D, NT, facc, fq_row);
                else fir64_chunk<1>(L, xq, lane, c * C64, r.x, r.y, f, nsl_mask, D, NT, facc, fq_row);
            }
            SSB64_WORK_END();
            lds_barrier();
        }
        ssb64_stamp(stamps, 4 + role, st_work, st_t0);
    } else if (role == BK_EQ) {
        // HP -> BP -> transientBoost -> floatToPCM (:177-210) on the outputs the FIR completed, lane = stream
        float h1 = 0.0f, h2 = 0.0f, q1 = 0.0f, q2 = 0.0f, prev = 0.0f;  // HP/BP state (carried), boost prev
        if (live) {
            const SsbStreamState st = state[s];
            h1 = st.hp_z1; h2 = st.hp_z2; q1 = st.bp_z1; q2 = st.bp_z2;
        }
        // audio pulse detector front end on each PCM sample (AudioPulseDetector::process(pcm), pulse_front.h)
        const bool front = af.state != nullptr;
        FrontState fst{};
        if (front && live) fst = front_load(af.state + s);
        float *my_new = front ? af.new_e + (size_t)(live ? s : 0) * (size_t)af.max_new : nullptr;
        int np = 0;
        for (int it = 0; it < nit; ++it) {
            SSB64_WORK_BEGIN();
            const int c = it - 5;
            if (c >= 0 && c < nch && live && PL > 0) {
                const int4 r = chunk_out[c];  // outputs completed in chunk c: [r.z, r.w]
                for (int o = r.z; o <= r.w; o++) {
                    const float in = L.fq[c & 1][lane * MAXD64 + (o & (MAXD64 - 1))];
                    const float yh = p.hp[0] * in + p.hp[1] * h1 + p.hp[2] * h2 - p.hp[3] * h1 - p.hp[4] * h2;
                    h2 = h1;
                    h1 = yh;
                    const float yb = p.bp[0] * yh + p.bp[1] * q1 + p.bp[2] * q2 - p.bp[3] * q1 - p.bp[4] * q2;
                    q2 = q1;
                    q1 = yb;
                    const float diff = yb - prev;
                    prev = yb;
                    const float boosted = yb + p.transient_coeff * diff;
                    const float v = clamp_ref(boosted * p.gain, -1.0f, 1.0f);
                    const int16_t q = (int16_t)(v * 32767.0f);
                    pcm[(size_t)s * PL + o] = q;
                    if (front) front_sample(af, fst, (float)q * PCM_TO_FLOAT, my_new, np);
                }
            }
            SSB64_WORK_END();
            lds_barrier();
        }
        ssb64_stamp(stamps, 4 + role, st_work, st_t0);
        if (live) {
            state[s].hp_z1 = h1;
            state[s].hp_z2 = h2;
            state[s].bp_z1 = q1;
            state[s].bp_z2 = q2;
            if (front) {
                front_store(af.state + s, fst);
                af.new_count[s] = np;
            }
        }
    } else {
        for (int it = 0; it < nit; ++it) lds_barrier();
        ssb64_stamp(stamps, 4 + role, 0, st_t0);
    }
}

}  // namespace

// Whether ssb64 runs this call (else ssb.hip's kernels): the reference chain (no NCO), whole chunks, a full frame of
// input per stream (no zero padding), 16-B aligned rows, the FIR's slots within the four waves, and the y scratch.
bool ssb64_supported(const SsbParams &p, const void *iq, int fmt, int n_frames, int nsl_mask, bool have_scratch) {
    if (n_frames % G64 != 0) return false;
    if (fmt == SDRG_IQ_CF32) return false;  // 32 KiB per raw chunk: no room for the loader's LDS-DMA ring
    const int bps = fmt == SDRG_IQ_CS16 ? 4 : 2;
    // (whole groups: the scratch holds [group][chunk][quad][stream] for n_frames streams)
    return have_scratch && !p.nco_on && p.pcm_len > 0 && p.samp_count % C64 == 0 && p.samp_count > 0 &&
           p.n_in >= p.samp_count && ((size_t)p.n_in * bps) % 16 == 0 && (reinterpret_cast<uintptr_t>(iq) & 15) == 0 &&
           nsl_mask + 1 <= MAXSL64 && (nsl_mask + 1) % NFIR == 0 && (C64 + p.decim - 1) / p.decim <= MAXD64 &&
           p.n_taps <= 256;
}

// Lab (SDRG_SSB64_STAMPS=1 in a -DSDRG_LAB=1 build): per-role work / loop cycles of every 16th call, averaged over the
// groups, printed after a synchronisation of the stream (which the stamps build's timing then includes)
static unsigned long long *ssb64_stamps(int groups, bool *report) {
    static const bool on = [] {
        const char *v = lab_getenv("SDRG_SSB64_STAMPS");
        return v && v[0] == '1';
    }();
    static unsigned long long *buf = nullptr;
    static int have = 0, calls = 0;
    *report = false;
    if (!on) return nullptr;
    if (groups > have) {
        if (buf) (void)hipFree(buf);
        if (hipMalloc(reinterpret_cast<void **>(&buf), sizeof(unsigned long long) * 32 * groups) != hipSuccess) return nullptr;
        have = groups;
    }
    *report = (calls++ % 16) == 15;
    return buf;
}

static void ssb64_report(unsigned long long *buf, int groups, hipStream_t stream) {
    std::vector<unsigned long long> h((size_t)32 * groups);
    if (hipStreamSynchronize(stream) != hipSuccess ||
        hipMemcpy(h.data(), buf, h.size() * 8, hipMemcpyDeviceToHost) != hipSuccess)
        return;
    static const char *names[16] = {"F:LPF", "F:DC", "F:LOAD", "F:EXP", "B:AGC", "B:OUT", "B:EQ", "B:IMP", "B:DES0", "B:DES1",
                                    "B:DES2", "B:DES3", "B:FIR0", "B:FIR1", "B:FIR2", "B:FIR3"};
    fprintf(stderr, "[ssb64 stamps] cycles per frame (mean over %d groups), work / loop:", groups);
    for (int r = 0; r < 16; r++) {
        double w = 0, l = 0;
        for (int g = 0; g < groups; g++) {
            w += (double)h[((size_t)g * 16 + r) * 2];
            l += (double)h[((size_t)g * 16 + r) * 2 + 1];
        }
        fprintf(stderr, " %s %.0f/%.0f", names[r], w / groups, l / groups);
    }
    fprintf(stderr, "\n");
}

hipError_t launch_ssb64(const void *iq, int fmt, int n_frames, const SsbParams &p, int nsl_mask, const int *chunk_table,
                        const float *taps, SsbStreamState *state, float *scratch, int16_t *pcm, const AudioFront *audio,
                        hipStream_t stream, hipEvent_t stop, bool *stop_recorded) {
    if (stop_recorded) *stop_recorded = false;
    const int groups = (n_frames + G64 - 1) / G64;
    bool report = false;
    unsigned long long *stamps = ssb64_stamps(groups, &report);
    const char *src = reinterpret_cast<const char *>(iq);
    hipError_t e = hipSuccess;
#define SSB64_FRONT_ATTR(F) e = ensure_dynamic_lds(reinterpret_cast<const void *>(ssb64_front_kernel<F>), (int)front_lds_bytes<F>())
    switch (fmt) {
    case SDRG_IQ_CS8: SSB64_FRONT_ATTR(SDRG_IQ_CS8); break;
    case SDRG_IQ_CU8: SSB64_FRONT_ATTR(SDRG_IQ_CU8); break;
    case SDRG_IQ_CS16: SSB64_FRONT_ATTR(SDRG_IQ_CS16); break;
    default: return hipErrorInvalidValue;
    }
#undef SSB64_FRONT_ATTR
    if (e != hipSuccess) return e;
    e = ensure_dynamic_lds(reinterpret_cast<const void *>(ssb64_back_kernel), (int)sizeof(BackLds));
    if (e != hipSuccess) return e;
#define SSB64_FRONT_LAUNCH(F)                                                                                      \
    hipLaunchKernelGGL(ssb64_front_kernel<F>, dim3(groups), dim3(FRONT_T), front_lds_bytes<F>(), stream, src, n_frames, p, \
                       state, scratch, stamps)
    switch (fmt) {
    case SDRG_IQ_CS8: SSB64_FRONT_LAUNCH(SDRG_IQ_CS8); break;
    case SDRG_IQ_CU8: SSB64_FRONT_LAUNCH(SDRG_IQ_CU8); break;
    default: SSB64_FRONT_LAUNCH(SDRG_IQ_CS16); break;
    }
#undef SSB64_FRONT_LAUNCH
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    AudioFront af{};
    if (audio) af = *audio;
    const int4 *chunk_out = reinterpret_cast<const int4 *>(chunk_table);
    if (stop) {
        hipExtLaunchKernelGGL(ssb64_back_kernel, dim3(groups), dim3(BACK_T), (uint32_t)sizeof(BackLds), stream, nullptr, stop,
                              0u, scratch, n_frames, p, nsl_mask, chunk_out, taps, state, pcm, af, stamps);
    } else {
        hipLaunchKernelGGL(ssb64_back_kernel, dim3(groups), dim3(BACK_T), sizeof(BackLds), stream, scratch, n_frames, p,
                           nsl_mask, chunk_out, taps, state, pcm, af, stamps);
    }
    e = hipGetLastError();
    if (e == hipSuccess && report) ssb64_report(stamps, groups, stream);
    if (e == hipSuccess && stop && stop_recorded) *stop_recorded = true;
    return e;
}

}  // namespace sdrg

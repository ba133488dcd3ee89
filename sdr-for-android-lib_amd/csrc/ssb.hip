// ssb.hip — the SSB audio chain for a batch of independent streams, one frame each.
//
// Replaces processSSB_opt (src/ssb/ssb_demod_opt.cpp:221-296):
//   removeDC(0.9995) -> iir2 low-pass -> demodSSB (Re+Im) -> adaptiveAGC -> 255-tap Hann-sinc FIR
//   decimate -> HP 1.2 kHz + BP 2.4 kHz biquads -> transientBoost -> floatToPCM.
//
// The chain's recurrences (DC, low-pass, AGC, biquads) are replayed sample by sample in the reference's
// float operation order with FP contraction OFF and IEEE division/sqrt, because the AGC amplifies any
// rounding difference in the low-pass output into hundreds of PCM LSBs.  The
// output is therefore bit-identical to the reference, and the parallelism comes from running many
// streams at once (one lane per stream) and from the FIR, whose outputs are independent.
//
// Kernels (the pipelined ssb_pipe_kernel below is the production path; these three are the
// straightforward lane-per-stream form, kept for configurations the pipeline does not cover):
//   ssb_chain_kernel : lane = stream; DC -> LPF -> demod -> AGC over the frame; AGC output -> scratch
//   ssb_fir_kernel   : block = 64 outputs of one stream; input window staged in LDS; each output is the
//                      reference's sequential 255-term sum
//   ssb_eq_kernel    : lane = stream; HP -> BP -> boost -> PCM over the decimated frame
#include <hip/hip_ext.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "pulse_front.h"
#include "sdrg_internal.h"
#include "ssb_common.h"
#include "ssb_lpf_asm.h"
#include "ssb_math.h"

#pragma clang fp contract(off)

namespace sdrg {
namespace {

constexpr int WAVE = 64;

struct Chain {
    // removeDC (:49-55): dc = a*dc + (1-a)*s ; s -= dc   (real part; the imaginary part never reaches PCM)
    float dc;
    // iir2Process (:75-84): y = a0 x + a1 z1 + a2 z2 - b1 z1 - b2 z2 ; z = past outputs
    float a0, a1, a2, b1, b2, z1, z2;
    // adaptiveAGC (:101-115)
    float target, fast, gain;
    int upper;

    __device__ __forceinline__ float step(float re) {
        const float alpha = 0.9995f;
        dc = alpha * dc + (1.0f - alpha) * re;
        const float x = re - dc;
        const float y = a0 * x + a1 * z1 + a2 * z2 - b1 * z1 - b2 * z2;
        z2 = z1;
        z1 = y;
        const float a = upper ? (y + y) : (y - y);  // demodSSB: Re + Im of {y, y}
        const float mag = fabsf(a) + 1e-8f;
        const float desired = target / (sqrtf(mag) + 1e-6f);
        const float rate = (desired < gain) ? fast : 0.00035f;
        gain = gain * (1.0f - rate) + desired * rate;
        return clamp_ref(a * gain, -1.0f, 1.0f);
    }
};

template <int FMT>
__global__ __launch_bounds__(WAVE) void ssb_chain_kernel(const char *__restrict__ iq, int n_frames, SsbParams p,
                                                         SsbStreamState *__restrict__ state,
                                                         float *__restrict__ scratch) {
    const int s = blockIdx.x * WAVE + threadIdx.x;
    if (s >= n_frames) return;
    const char *frame = iq + (size_t)s * p.n_in * bytes_per_sample<FMT>();
    float *out = scratch + (size_t)s * p.samp_count;
    SsbStreamState st = state[s];
    Chain c;
    c.dc = 0.0f;
    c.a0 = p.lpf[0]; c.a1 = p.lpf[1]; c.a2 = p.lpf[2]; c.b1 = p.lpf[3]; c.b2 = p.lpf[4];
    c.z1 = st.lpf_z1; c.z2 = st.lpf_z2;
    c.target = p.agc_target; c.fast = p.agc_fast; c.gain = 1.0f;
    c.upper = p.upper;

    const int S = p.samp_count;
    const int live = p.n_in < S ? p.n_in : S;  // samples present; the rest is iq.resize() zero padding
    // 16-B loads need alignment; the NCO variant (which also needs Q) runs sample by sample
    const int n8 = (!p.nco_on && (reinterpret_cast<uintptr_t>(frame) & 15) == 0) ? (live & ~7) : 0;
    int n = 0;
    for (; n < n8; n += 8) {
        float x[8];
        load_i8<FMT>(frame, n, x);
        float y[8];
#pragma unroll
        for (int q = 0; q < 8; q++) y[q] = c.step(x[q]);
        *reinterpret_cast<float4 *>(out + n) = make_float4(y[0], y[1], y[2], y[3]);
        *reinterpret_cast<float4 *>(out + n + 4) = make_float4(y[4], y[5], y[6], y[7]);
    }
    if (p.nco_on) {
        for (; n < live; n++)
            out[n] = c.step(nco_mix(p.nco_tab, p.nco_phase + p.nco_inc * (uint32_t)n, load_i1<FMT>(frame, n),
                                    load_q1<FMT>(frame, n)));
    }
    for (; n < live; n++) out[n] = c.step(load_i1<FMT>(frame, n));
    for (; n < S; n++) out[n] = c.step(0.0f);
    st.lpf_z1 = c.z1;
    st.lpf_z2 = c.z2;
    state[s] = st;
}

// simpleFIRDecimate (:121-143): out[o] = sum_{k<N} in[o*decim + k] * h[k], k ascending.
__global__ __launch_bounds__(WAVE) void ssb_fir_kernel(const float *__restrict__ audio, SsbParams p,
                                                       const float *__restrict__ taps, float *__restrict__ fir_out) {
    extern __shared__ __attribute__((aligned(16))) float win[];
    const int s = blockIdx.y;
    const int o0 = blockIdx.x * WAVE;
    const float *a = audio + (size_t)s * p.samp_count;
    const int base = o0 * p.decim;
    const int span = (WAVE - 1) * p.decim + p.n_taps;
    for (int i = threadIdx.x; i < span; i += WAVE) {
        const int g = base + i;
        win[i] = (g < p.samp_count) ? a[g] : 0.0f;
    }
    __syncthreads();
    const int o = o0 + threadIdx.x;
    if (o >= p.pcm_len) return;
    const float *w = win + threadIdx.x * p.decim;
    float acc = 0.0f;
    for (int k = 0; k < p.n_taps; k++) acc += w[k] * taps[k];
    fir_out[(size_t)s * p.pcm_len + o] = acc;
}

// HP, BP (biquadProcess :177-186), transientBoost (:191-198), floatToPCM (:203-210)
__global__ __launch_bounds__(WAVE) void ssb_eq_kernel(const float *__restrict__ fir_out, int n_frames, SsbParams p,
                                                      SsbStreamState *__restrict__ state, int16_t *__restrict__ pcm) {
    const int s = blockIdx.x * WAVE + threadIdx.x;
    if (s >= n_frames) return;
    const float *x = fir_out + (size_t)s * p.pcm_len;
    int16_t *out = pcm + (size_t)s * p.pcm_len;
    SsbStreamState st = state[s];
    float h1 = st.hp_z1, h2 = st.hp_z2, b1 = st.bp_z1, b2 = st.bp_z2, prev = 0.0f;
    const float coeff = p.transient_coeff, g = p.gain;
    for (int i = 0; i < p.pcm_len; i++) {
        const float in = x[i];
        const float yh = p.hp[0] * in + p.hp[1] * h1 + p.hp[2] * h2 - p.hp[3] * h1 - p.hp[4] * h2;
        h2 = h1;
        h1 = yh;
        const float yb = p.bp[0] * yh + p.bp[1] * b1 + p.bp[2] * b2 - p.bp[3] * b1 - p.bp[4] * b2;
        b2 = b1;
        b1 = yb;
        const float diff = yb - prev;
        prev = yb;
        const float boosted = yb + coeff * diff;
        const float v = clamp_ref(boosted * g, -1.0f, 1.0f);
        out[i] = (int16_t)(v * 32767.0f);
    }
    st.hp_z1 = h1; st.hp_z2 = h2; st.bp_z1 = b1; st.bp_z2 = b2;
    state[s] = st;
}

// ================================================================================================
// Pipelined SSB engine (the production path).
//
// The chain has three sample-serial recurrences (DC tracker, 2nd-order low-pass, AGC gain) whose
// per-sample latency, not the chip's throughput, bounds the frame time: a lone wave issues one VALU
// instruction per ~4 cycles (MI355X_MICROARCH.md, 'vector-instruction ISSUE cost'), so every
// non-recurrent operation left in a serial wave lengthens the frame.  This kernel therefore gives each
// recurrence its own wave (lane = stream), keeps ONLY the recurrence arithmetic in it, and moves every
// order-free operation (unpack, the AGC's sqrt/div "desired" level, the clamp, the FIR) to helper waves.
// The stages are pipelined over chunks of CH samples through LDS rings with one workgroup barrier per
// chunk, so while the low-pass wave works on chunk c the DC wave is on c+2 and the helpers on c-1 ... c-5:
//
//   it:  load c=it | DC c=it-1 | LPF c=it-3 | DESIRED c=it-4 | AGC c=it-5 | OUT c=it-6 | FIR c=it-7 | EQ c=it-8
//   (SDRG_LPF_LOOKAHEAD, below: the low-pass wave one chunk behind the DC wave's output; without it every role
//   from the low-pass on is one chunk closer)
//
// The FIR accumulates each output's 255 products as its samples arrive (k ascending, exactly the
// reference's order) in per-(stream, slot) accumulators, so no sample window is kept; completed outputs
// go to the EQ role (HP, BP, boost, PCM).  All arithmetic is the reference's, in its order, without
// contraction: bit-identical PCM.
//
// Workgroup = 16 streams x 12 waves, one workgroup per CU (84.8 KiB of LDS: two never fit), beside one spectrum workgroup.  A wave issues
// at most about one VALU instruction per ~10 cycles however idle its SIMD is, while a SIMD serves several
// waves at that rate (tools/microbench/valu2.hip), so the order-free work is spread over as many waves as
// keep the heaviest helper's instruction count below the low-pass wave's.  The roles are dealt to the
// SIMDs (hardware wave w runs on SIMD w % 4) by measurement (tools/gpu_map.sh): a serial wave slows the
// helpers that share its SIMD about twofold, so the FIR waves, the heaviest helpers, share the loader's:
//   SIMD0: DC,   AGC output clamp,  desired (1/4)
//   SIMD1: LPF,  EQ,                desired (1/4)
//   SIMD2: AGC,  desired (1/4),     desired (1/4)
//   SIMD3: load, FIR (slot group 0), FIR (slot group 1)
// ================================================================================================
// the low-pass wave's full chunks as one hand-scheduled asm block (1) or through row_pipeline (0)
#ifndef SDRG_LPF_ASM
#define SDRG_LPF_ASM 1
#endif
// the DC wave's chunks as one hand-scheduled asm block, its LDS reads and writes interleaved quad by quad with the
// arithmetic (2) or grouped per sub-block (1), or through row_pipeline (0)
#ifndef SDRG_DC_ASM
#define SDRG_DC_ASM 2
#endif
// the AGC gain wave's chunks, the same three forms
#ifndef SDRG_AGC_ASM
#define SDRG_AGC_ASM 2
#endif
constexpr int PG = 16;          // streams per workgroup
constexpr int CH = 64;          // samples per chunk
constexpr int ROW = CH + 4;     // padded stream row (floats): conflict-free ds_read_b128 by stream lanes
constexpr int BUFF = PG * ROW;  // floats per [stream][sample] chunk buffer
constexpr int PIPE_WAVES = 12;
constexpr int PIPE_T = PIPE_WAVES * 64;
constexpr int STAMP_SLOTS = 4;  // diagnostic stamps per wave: work, loop cycles, loop time, kernel entry (s_memrealtime)
enum PipeWave : int { W_DC = 0, W_LPF = 1, W_AGC = 2, W_LOAD = 3, W_FIR0 = 4, W_OUT = 5, W_EQ = 6, W_FIR1 = 7,
                      W_DES0 = 8, W_DES1 = 9, W_DES2 = 10, W_DES3 = 11 };
// role of hardware wave w = nibble w: w0 DC, w1 LPF, w2 AGC, w3 load, w4 OUT, w5 EQ, w6 DES2, w7 FIR0,
// w8 DES0, w9 DES1, w10 DES3, w11 FIR1
constexpr unsigned long long DEFAULT_ROLE_MAP = 0x7B984A653210ull;
// the NCO variant's loader does the mixing too: FIR1 beside the DC wave, the clamp beside it as well, DES0 beside the
// loader (w4 FIR1, w8 OUT, w11 DES0).  configs[2] 199.0-200.6 -> 202.8 G with it; the reference chain's c3 line
// loses 2.5 % under FIR1 <-> OUT alone (r5av, r5aw, tools/ab.sh, alternating, one box), so it keeps its own map.
constexpr unsigned long long NCO_ROLE_MAP = 0x8B954A673210ull;
constexpr int MAX_SLOTS = 32;   // concurrent FIR outputs per stream (up to 4 per FIR lane)
constexpr int MAX_DONE = 8;     // FIR outputs completed per stream per chunk
constexpr int PIPE_LDS_TARGET = 84 * 1024;  // > 80 KiB: at most one pipeline workgroup per CU

constexpr int TAPS_ROW = CH + 256 + CH + 4;
#ifndef SDRG_TAPS_COPIES  // lab: 2 copies (shifts 0, 1) read as 8-byte pairs free 3 KB of LDS against 4 (shifts 0-3, 16-byte reads)
#define SDRG_TAPS_COPIES 4
#endif
constexpr int TAPS_COPIES = SDRG_TAPS_COPIES;
static_assert(TAPS_COPIES == 4 || TAPS_COPIES == 2, "taps copies");
// The low-pass wave one chunk behind the DC wave's output (1): its input ring gets a third slot and the wave runs
// its whole loop as one asm block that reads the next chunk's first sub-blocks before each barrier (csrc/ssb_lpf_asm.h);
// every later role moves one iteration later.  The raw-IQ batches shrink to 256 B x 3 to keep the LDS budget.
#ifndef SDRG_LPF_LOOKAHEAD
#define SDRG_LPF_LOOKAHEAD 1
#endif
constexpr int LA = SDRG_LPF_LOOKAHEAD ? 1 : 0;
// with the lookahead: the loop's LDS reads and writes interleaved quad by quad with the chain (1) or grouped per
// sub-block (0)
#ifndef SDRG_LPF_INTERLEAVE
#define SDRG_LPF_INTERLEAVE 1
#endif
constexpr int NA = 2 + LA;  // slots of the DC -> low-pass ring
#ifndef SDRG_PIPE_RAWB  // bytes of raw IQ per stream per prefetch batch
#define SDRG_PIPE_RAWB (SDRG_LPF_LOOKAHEAD ? 256 : 512)
#endif
constexpr int RAWB = SDRG_PIPE_RAWB;
constexpr int RAW_PIECES = RAWB / 64;     // 16-B LDS-DMA pieces per loader lane (lane = 4 x stream + quarter)
constexpr int RAW_U4 = PG * RAWB / 16;    // one prefetch batch as [piece][lane 64] uint4

template <int FMT>
constexpr int batch_chunks() {  // chunks per RAWB-per-stream prefetch batch (DMA needs CH * bps <= RAWB)
    constexpr int b = RAWB / (CH * (FMT == SDRG_IQ_CF32 ? 8 : FMT == SDRG_IQ_CS16 ? 4 : 2));
    return b > 0 ? b : 1;
}
#ifndef SDRG_PIPE_NRAW  // 512 B: 2 (one batch unpacked, one in flight; 3 needs 8 KiB more LDS than co-residency allows)
#define SDRG_PIPE_NRAW (SDRG_LPF_LOOKAHEAD ? 3 : 2)
#endif
// Co-residency with the spectrum kernel (measured +4-5 % per step, tools/gpu_cores.sh): the pipeline keeps to
// 80 VGPRs (6 waves per SIMD's worth; 3 x 80 + 2 x 128 <= 512) and 84.8 KiB of LDS (+ 72.3 KiB <= 160 KiB), so
// one 512-thread spectrum workgroup fits beside it on every CU and the next call's spectrum runs while this
// call's latency-bound SSB pipeline holds the CUs.  The LDS is dynamic so that the compiler's occupancy model
// (which otherwise clamps waves-per-EU to what the static LDS allows) honours the 80-VGPR budget.
#ifndef SDRG_PIPE_DYN_LDS
#define SDRG_PIPE_DYN_LDS 1
#endif
#ifndef SDRG_PIPE_MINW  // waves per SIMD the VGPR budget must allow: 6 -> at most 80 VGPRs
#define SDRG_PIPE_MINW 6
#endif
constexpr int NRAW = SDRG_PIPE_NRAW;  // raw-IQ batches in LDS: one being unpacked, NRAW - 1 in flight
struct PipeLds {
    uint4 raw[NRAW][RAW_U4];  // raw IQ bytes of the prefetch batches (LDS-DMA), [piece][loader lane]
    float re[2][BUFF];
    float a[NA][BUFF];
    float y[4][BUFF];  // the low-pass outputs
    float d[2][BUFF];
    float g[2][BUFF];
    float out[2][BUFF];
    float fq[2][PG * MAX_DONE];
    // taps with CH zeros on both sides (out-of-window FIR steps multiply by 0), in 4 copies shifted by
    // 0..3 floats so that any 32-tap window is read with aligned ds_read_b128
    float taps_sh[TAPS_COPIES][TAPS_ROW];
};
// NCO variant only, in dynamic LDS: the current chunk's CH phasors {re, im}.  The two phasor tables (16 KiB) are read
// from global memory (L1/L2-resident) a chunk ahead by the loader: in LDS they took the pipeline workgroup to 101.7 KiB,
// and the spectrum workgroup (72.3 KiB) no longer fitted beside it on a CU (r5an: configs[2] 168 G with the tables
// in LDS)
constexpr int NCO_LDS_BYTES = 2 * CH * 4;

__device__ __forceinline__ int ceil_div_i(int a, int b) {  // b > 0, any sign of a
    return a >= 0 ? (a + b - 1) / b : -((-a) / b);
}

template <int FMT>
__device__ __forceinline__ void load_i8_masked(const char *frame, int t, int n_in, float (&x)[8]) {
    if (t + 8 <= n_in && (reinterpret_cast<uintptr_t>(frame) & 15) == 0) {
        load_i8<FMT>(frame, t, x);
    } else {
#pragma unroll
        for (int q = 0; q < 8; q++) x[q] = (t + q < n_in) ? load_i1<FMT>(frame, t + q) : 0.0f;
    }
}

// A serial role's pass over one stream's chunk row in sub-blocks of SB samples, double-buffered in registers:
// sub-block i + 1 is read from LDS while sub-block i runs through the recurrence, so the LDS latency is off
// the recurrence's critical path.  step(v) updates the role's carried state and v in place; the results go
// to dst when store (lanes that hold a stream's first copy).
#ifndef SDRG_PIPE_SB  // 16: two 16-float register sub-blocks fit the 80-VGPR budget without spills (32 spills)
#define SDRG_PIPE_SB 16
#endif
constexpr int SB = SDRG_PIPE_SB;
template <class Step>
__device__ __forceinline__ void row_pipeline(const float *src, float *dst, bool store, Step step) {
    constexpr int NSB = CH / SB;
    static_assert(NSB % 2 == 0, "pairs of sub-blocks");
    float va[SB], vb[SB];
    auto rd = [&](const float *r, float (&v)[SB]) {
#pragma unroll
        for (int i = 0; i < SB; i += 4) {
            const float4 x = *reinterpret_cast<const float4 *>(r + i);
            v[i] = x.x; v[i + 1] = x.y; v[i + 2] = x.z; v[i + 3] = x.w;
        }
    };
    auto wr = [&](float *r, const float (&v)[SB]) {
        if (store) {
#pragma unroll
            for (int i = 0; i < SB; i += 4) *reinterpret_cast<float4 *>(r + i) = make_float4(v[i], v[i + 1], v[i + 2], v[i + 3]);
        }
    };
    rd(src, va);
#pragma unroll
    for (int sb = 0; sb < NSB; sb += 2) {
        rd(src + SB * (sb + 1), vb);
        step(va);
        wr(dst + SB * sb, va);
        if (sb + 2 < NSB) rd(src + SB * (sb + 2), va);
        step(vb);
        wr(dst + SB * (sb + 1), vb);
    }
}

// The FIR slots of one stream over one chunk: lane = (stream, sub); slot 4j+sub holds the output o active
// in [t0, t1), if any.  The lane reads its stream's 32 chunk values once (8 ds_read_b128) and, per slot,
// the 32 taps that meet them (8 ds_read_b128), forms the products two per packed multiply, and
// accumulates each slot in the reference's k order; the NP slot chains interleave.  Steps outside the output's window meet a zero tap from
// the padding, and acc + (+-0) == acc exactly here: acc starts at +0 and a round-to-nearest sum never
// produces -0 from +0, so the masked steps leave the reference's sequential sum unchanged.
template <int NP, int J0 = 0>
__device__ __forceinline__ void fir_chunk(PipeLds &L, int c, int t0, int o_lo, int o_hi, int sub, int nsl_mask,
                                          int sl, int D, int NT, float (&acc)[MAX_SLOTS / 4]) {
    const int t1 = t0 + CH;
    int k0[NP];
    bool active[NP], done[NP];
    int slot_o[NP];
#pragma unroll
    for (int j = 0; j < NP; j++) {
        const int slot = 4 * (J0 + j) + sub;
        const int o = o_lo + ((slot - o_lo) & nsl_mask);  // the output this slot holds (o == slot mod NSL)
        const int base = D * o;
        active[j] = o <= o_hi;
        done[j] = active[j] && base + NT <= t1;
        slot_o[j] = o;
        if (active[j] && base >= t0) acc[J0 + j] = 0.0f;
        k0[j] = active[j] ? (t0 - base + CH) : 0;  // taps_pad index of step 0 (inactive: the zero padding)
    }
    const float4 *in = reinterpret_cast<const float4 *>(&L.out[c & 1][sl * ROW]);  // 0 beyond frame end
#pragma unroll 4
    for (int i = 0; i < CH / 4; i++) {
        const float4 x = in[i];
        f2v lo[NP], hi[NP];
#pragma unroll
        for (int j = 0; j < NP; j++) {
            float4 h;
            if constexpr (TAPS_COPIES == 4) {
                h = reinterpret_cast<const float4 *>(&L.taps_sh[k0[j] & 3][k0[j] & ~3])[i];
            } else {
                const float2 *b2 = reinterpret_cast<const float2 *>(&L.taps_sh[k0[j] & 1][k0[j] & ~1]);
                const float2 h01 = b2[2 * i], h23 = b2[2 * i + 1];
                h = make_float4(h01.x, h01.y, h23.x, h23.y);
            }
            lo[j] = f2v{x.x, x.y} * f2v{h.x, h.y};  // products are order-free: two per packed op
            hi[j] = f2v{x.z, x.w} * f2v{h.z, h.w};
        }
        // the sums keep the reference's tap order; the NP slot chains are independent and interleave
#pragma unroll
        for (int j = 0; j < NP; j++) acc[J0 + j] += lo[j].x;
#pragma unroll
        for (int j = 0; j < NP; j++) acc[J0 + j] += lo[j].y;
#pragma unroll
        for (int j = 0; j < NP; j++) acc[J0 + j] += hi[j].x;
#pragma unroll
        for (int j = 0; j < NP; j++) acc[J0 + j] += hi[j].y;
    }
#pragma unroll
    for (int j = 0; j < NP; j++)
        if (done[j]) L.fq[c & 1][sl * MAX_DONE + (slot_o[j] & (MAX_DONE - 1))] = acc[J0 + j];
}

template <int FMT, bool DMA>
__global__ __attribute__((amdgpu_flat_work_group_size(PIPE_T, PIPE_T), amdgpu_waves_per_eu(SDRG_PIPE_MINW))) void ssb_pipe_kernel(const char *__restrict__ iq, int n_frames, SsbParams p,
                                                          int nsl_mask, const int4 *__restrict__ chunk_out,
                                                          const float *__restrict__ taps,
                                                          SsbStreamState *__restrict__ state,
                                                          int16_t *__restrict__ pcm,
                                                          unsigned long long *__restrict__ stamps, int prio_mask,
                                                          int skip_mask, unsigned long long role_map, AudioFront af) {
#if SDRG_PIPE_DYN_LDS  // the whole LDS dynamic: the compiler's occupancy model then sees no LDS limit
    extern __shared__ __attribute__((aligned(16))) char pipe_dyn[];
    PipeLds &L = *reinterpret_cast<PipeLds *>(pipe_dyn);
    float *nco_lds = reinterpret_cast<float *>(pipe_dyn + sizeof(PipeLds));
#else
    __shared__ PipeLds L;
    extern __shared__ __attribute__((aligned(16))) float nco_lds[];  // NCO_LDS_BYTES when p.nco_on
#endif
    const int tid = threadIdx.x;
    const unsigned long long st_entry = stamps ? __builtin_amdgcn_s_memrealtime() : 0;  // diagnostic stamps only
    const int hw_wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // runs on SIMD hw_wave % 4
    const int wave = (int)((role_map >> (4 * hw_wave)) & 15);     // the role it plays (PipeWave)
    const int lane = tid & 63;
    const int s0 = blockIdx.x * PG;
    const int S = p.samp_count;
    const int nch = (S + CH - 1) / CH;
    const int D = p.decim, NT = p.n_taps, PL = p.pcm_len;
    auto y_row = [&](int c, int sl) { return &L.y[c & 3][sl * ROW]; };  // the low-pass outputs of chunk c, row sl

    for (int i = tid; i < TAPS_COPIES * TAPS_ROW; i += PIPE_T) {
        const int sh = i / TAPS_ROW, j = i % TAPS_ROW;
        const int k = j + sh - CH;  // copy sh holds taps_pad[j + sh] at index j
        L.taps_sh[sh][j] = (k >= 0 && k < NT) ? taps[k] : 0.0f;
    }

    const int my_s = lane & (PG - 1);  // serial roles: lane = 16 x copy + stream (all 64 lanes run; lanes < PG store)
    const float demod_k = p.upper ? 2.0f : 0.0f;  // demodSSB(y, y) = y + y or y - y (:89-94) as y * k
    const bool serial_live = (wave < 3 || wave == W_EQ) && (lane < PG) && (s0 + lane < n_frames);
    // issue priority per role: a bit mask of roles at priority 2, or (bit 31 set) two bits of priority level per role
    const int prio_lvl = prio_mask < 0 ? (prio_mask >> (2 * wave)) & 3 : ((prio_mask >> wave) & 1) * 2;
    const bool high = prio_lvl != 0;
    if (prio_lvl == 1) __builtin_amdgcn_s_setprio(1);
    else if (prio_lvl == 2) __builtin_amdgcn_s_setprio(2);
    else if (prio_lvl == 3) __builtin_amdgcn_s_setprio(3);
    const size_t bps = bytes_per_sample<FMT>();
    const int n_live = min(p.n_in, S);

    // raw-IQ prefetch of the loader wave (wave 3): batch kb = chunks [kb*BC, kb*BC+BC) = 512 B per stream,
    // moved by LDS-DMA (global_load_lds, no registers) BC iterations before its first chunk is unpacked.
    // Lane = 4 x stream + quarter of the stream's 512 B; 8 DMA pieces of 16 B per lane.
    constexpr int BC = batch_chunks<FMT>();
    constexpr int SPU = 16 / (int)bytes_per_sample<FMT>();  // samples per 16 B
    const int ld_s = lane >> 2, ld_q = lane & 3;
    const bool ld_live = (s0 + ld_s < n_frames);
    const char *ld_frame = iq + (size_t)(ld_live ? s0 + ld_s : s0) * p.n_in * bps;
    const int n_batches = (n_live + BC * CH - 1) / (BC * CH);
    auto issue_batch = [&](int kb) {
        const char *src = ld_frame + (size_t)(kb * BC * CH + ld_q * RAW_PIECES * SPU) * bps;
#pragma unroll
        for (int q = 0; q < RAW_PIECES; q++)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(src + 16 * q),
                                             (__attribute__((address_space(3))) void *)&L.raw[kb % NRAW][q * 64], 16, 0, 0);
    };
    // wait until at most `k` batches (the youngest) of this wave's LDS-DMA are still in flight
    auto wait_raw = [](int k) {
        static_assert(NRAW <= 4 && 2 * RAW_PIECES <= 63, "vmcnt immediates below");
        if (NRAW >= 4 && k >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * RAW_PIECES) : "memory");
        else if (NRAW >= 3 && k >= 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(RAW_PIECES) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    };
    if constexpr (DMA) {
        const int first = min(NRAW - 1, n_batches);  // batches 0 .. NRAW-2 in flight before the loop
        if (wave == W_LOAD)
            for (int kb = 0; kb < first; kb++) issue_batch(kb);
        wait_raw(first - 1);  // batch 0 landed
    }
    __syncthreads();

    unsigned long long st_work = 0, st_t0 = stamps ? __builtin_amdgcn_s_memtime() : 0, st_a = st_t0;
    const unsigned long long st_r0 = stamps ? __builtin_amdgcn_s_memrealtime() : 0;  // 100 MHz constant clock
    // Each role runs its own copy of the chunk loop (same trip count, one LDS barrier per iteration), so
    // the register allocator sees one role per loop and the kernel's VGPR count is the largest role's,
    // not the sum of every role's loop-invariant values.
    auto chunk_loop = [&](auto &&body) {
        for (int it = 0; it < nch + 8 + LA; ++it) {
            if (stamps) st_a = __builtin_amdgcn_s_memtime();
            body(it);
            if (stamps) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                st_work += __builtin_amdgcn_s_memtime() - st_a;
            }
            lds_barrier();
        }
    };
    // body(c) for the chunks c = 0 .. nch-1, with the barrier at iteration c + off of the common loop
    auto run = [&](int off, auto &&body) {
        chunk_loop([&](int it) {
            const int c = it - off;
            if (c >= 0 && c < nch) body(c);
        });
    };
    if ((skip_mask >> wave) & 1) {
        chunk_loop([&](int) {});
    } else if (wave == W_DC) {
        float dc = 0.0f;  // removeDC: reset per call (:50)
        // needs: the loader's chunk c; the low-pass wave done with chunk c - 3 (it reads c - 2 during c - 3)
        run(1, [&](int c) {
            // ---- removeDC (:49-55) and the a0*x term of iir2Process, chunk it-1 ----
            // the frame's last chunk runs whole too: dc restarts every frame and the samples past the frame end
            // (zeros from the loader) only feed outputs nothing reads
            const float alpha = 0.9995f, one_minus = 1.0f - 0.9995f, a0 = p.lpf[0];
            if (SDRG_DC_ASM && c >= 0 && c < nch && lane < PG) {
                // the whole chunk as one hand-scheduled block (csrc/ssb_lpf_asm.h, tools/gen/gen_lpf_asm.py)
                const f2v om2 = {one_minus, one_minus}, a02 = {a0, a0};
                const uint32_t src = lds_addr(&L.re[c & 1][my_s * ROW]), dst = lds_addr(&L.a[c % NA][my_s * ROW]);
                if (SDRG_DC_ASM == 2)
                    asm volatile(SDRG_DC_CHUNK_IL_ASM
                                 : [dc] "+v"(dc)
                                 : [src] "v"(src), [dst] "v"(dst), [alpha] "s"(alpha), [om2] "s"(om2), [a02] "s"(a02)
                                 : SDRG_CHUNK_CLOBBERS, "memory");
                else
                    asm volatile(SDRG_DC_CHUNK_ASM
                                 : [dc] "+v"(dc)
                                 : [src] "v"(src), [dst] "v"(dst), [alpha] "s"(alpha), [om2] "s"(om2), [a02] "s"(a02)
                                 : SDRG_CHUNK_CLOBBERS, "memory");
            } else if (c >= 0 && c < nch && lane < PG) {
                row_pipeline(&L.re[c & 1][my_s * ROW], &L.a[c % NA][my_s * ROW], lane < PG, [&](float (&v)[SB]) {
#pragma unroll
                    for (int q = 0; q < SB; q++) {
                        dc = alpha * dc + one_minus * v[q];
                        v[q] = a0 * (v[q] - dc);
                    }
                });
            }
        });
    } else if (wave == W_LPF) {
        float z1 = 0.0f, z2 = 0.0f;  // rfFilter state, carried across frames
        const bool lpf_asm_loop = LA && SDRG_LPF_ASM && S % CH == 0;
        if (s0 + my_s < n_frames) {
            z1 = state[s0 + my_s].lpf_z1;
            z2 = state[s0 + my_s].lpf_z2;
        }
        // y = ((((a0 x + a1 z1) + a2 z2) - b1 z1) - b2 z2): the four products as two packed multiplies (each
        // lane of v_pk_mul_f32 rounds like v_mul_f32), the adds in order; the subtractions are additions of
        // (-b) z (a - b == a + (-b) exactly, and (-b) z == -(b z))
        const f2v c1 = {p.lpf[1], -p.lpf[3]}, c2 = {p.lpf[2], -p.lpf[4]};
        static_assert(BUFF * 4 == SDRG_LPF_LOOP_SLOT_BYTES, "ring slot stride of the generated loop");
        if (lpf_asm_loop) {
            // the whole loop as one block (csrc/ssb_lpf_asm.h, tools/gen/gen_lpf_asm.py): nch + 8 + LA iterations
            // with one s_barrier each, the same count as every other role's chunk_loop
            f2v z = {z1, z2};
            const uint32_t abase = lds_addr(&L.a[0][my_s * ROW]), ybase = lds_addr(&L.y[0][my_s * ROW]);
            const int nit = nch + 8 + LA;
            unsigned long long sv;
            int t_it, t_cc, t_r, t_yo;
            if (SDRG_LPF_INTERLEAVE)
                asm volatile(SDRG_LPF_LOOP_IL_ASM
                             : [z] "+v"(z), [sv] "=&s"(sv), [it] "=&s"(t_it), [cc] "=&s"(t_cc), [r] "=&s"(t_r), [yo] "=&s"(t_yo)
                             : [abase] "v"(abase), [ybase] "v"(ybase), [c1] "s"(c1), [c2] "s"(c2), [nit] "s"(nit), [nch] "s"(nch)
                             : SDRG_CHUNK_CLOBBERS, "v54", "memory");
            else
                asm volatile(SDRG_LPF_LOOP_ASM
                             : [z] "+v"(z), [sv] "=&s"(sv), [it] "=&s"(t_it), [cc] "=&s"(t_cc), [r] "=&s"(t_r), [yo] "=&s"(t_yo)
                             : [abase] "v"(abase), [ybase] "v"(ybase), [c1] "s"(c1), [c2] "s"(c2), [nit] "s"(nit), [nch] "s"(nch)
                             : SDRG_CHUNK_CLOBBERS, "v54", "memory");
            z1 = z.x;
            z2 = z.y;
        } else run(2 + LA, [&](int c) {
            // ---- iir2Process recurrence (:75-84), chunk it-2 ----
            if (c >= 0 && c < nch && lane < PG) {
                const int lim = min(CH, S - c * CH);
                if (lim == CH && SDRG_LPF_ASM) {
                    // the whole chunk as one hand-scheduled block (csrc/ssb_lpf_asm.h, tools/gen/gen_lpf_asm.py)
                    f2v z = {z1, z2};
                    const uint32_t src = lds_addr(&L.a[c % NA][my_s * ROW]), dst = lds_addr(y_row(c, my_s));
                    asm volatile(SDRG_LPF_CHUNK_ASM
                                 : [z] "+v"(z)
                                 : [src] "v"(src), [dst] "v"(dst), [c1] "s"(c1), [c2] "s"(c2)
                                 : SDRG_LPF_CHUNK_CLOBBERS, "memory");
                    z1 = z.x;
                    z2 = z.y;
                } else if (lim == CH) {
                    row_pipeline(&L.a[c % NA][my_s * ROW], y_row(c, my_s), lane < PG, [&](float (&v)[SB]) {
#pragma unroll
                        for (int q = 0; q < SB; q++) {
                            const f2v p1 = c1 * z1, p2 = c2 * z2;
                            const float y = (((v[q] + p1.x) + p2.x) + p1.y) + p2.y;
                            z2 = z1;
                            z1 = y;
                            v[q] = y;
                        }
                    });
                } else {
                    // the frame's last, partial chunk (S not a multiple of CH): sample by sample through LDS,
                    // so the carried state is the one after exactly S samples
                    for (int q = 0; q < lim; q++) {
                        const f2v p1 = c1 * z1, p2 = c2 * z2;
                        const float y = (((L.a[c % NA][my_s * ROW + q] + p1.x) + p2.x) + p1.y) + p2.y;
                        z2 = z1;
                        z1 = y;
                        if (lane < PG) y_row(c, my_s)[q] = y;
                    }
                }
            }
        });
        if (lane < PG && s0 + my_s < n_frames) {
            state[s0 + my_s].lpf_z1 = z1;
            state[s0 + my_s].lpf_z2 = z2;
        }
    } else if (wave == W_AGC) {
        float gain = 1.0f;  // adaptiveAGC: reset per call (:102)
        // gain = gain*(1-rate) + desired*rate, rate = desired < gain ? fast : slow: both candidates (fast,
        // slow) in one packed lane pair, then the select.  The last chunk runs whole: gain restarts every
        // frame and outputs past the frame end are zeroed by the clamp role.
        const f2v rates = {p.agc_fast, 0.00035f};
        const f2v keep = {1.0f - p.agc_fast, 1.0f - 0.00035f};
        // needs: the four desired-level waves' chunk c; the clamp wave done with chunk c - 2
        run(4 + LA, [&](int c) {
            // ---- adaptiveAGC gain recurrence (:101-115), chunk it-4 ----
            if (SDRG_AGC_ASM && c >= 0 && c < nch && lane < PG) {
                // the whole chunk as one hand-scheduled block (csrc/ssb_lpf_asm.h, tools/gen/gen_lpf_asm.py)
                f2v g = {gain, gain};
                const uint32_t src = lds_addr(&L.d[c & 1][my_s * ROW]), dst = lds_addr(&L.g[c & 1][my_s * ROW]);
                if (SDRG_AGC_ASM == 2)
                    asm volatile(SDRG_AGC_CHUNK_IL_ASM
                                 : [g] "+v"(g)
                                 : [src] "v"(src), [dst] "v"(dst), [keep] "s"(keep), [rates] "s"(rates)
                                 : SDRG_CHUNK_CLOBBERS, "vcc", "memory");
                else
                    asm volatile(SDRG_AGC_CHUNK_ASM
                                 : [g] "+v"(g)
                                 : [src] "v"(src), [dst] "v"(dst), [keep] "s"(keep), [rates] "s"(rates)
                                 : SDRG_CHUNK_CLOBBERS, "vcc", "memory");
                gain = g.x;
            } else if (c >= 0 && c < nch && lane < PG) {
                row_pipeline(&L.d[c & 1][my_s * ROW], &L.g[c & 1][my_s * ROW], lane < PG, [&](float (&v)[SB]) {
#pragma unroll
                    for (int q = 0; q < SB; q++) {
                        const float desired = v[q];
                        const f2v cand = gain * keep + desired * rates;
                        gain = (desired < gain) ? cand.x : cand.y;
                        v[q] = gain;
                    }
                });
            }
        });
    } else if (wave == W_LOAD) {
        // NCO variant: the table entries of lane j's phasor for chunk c (sample c*CH + j), loaded a chunk ahead
        const float2 *nco_tab2 = reinterpret_cast<const float2 *>(p.nco_tab);
        float2 nco_h = make_float2(0.0f, 0.0f), nco_l = make_float2(0.0f, 0.0f);
        auto nco_fetch = [&](int c) {
            const uint32_t ph = p.nco_phase + p.nco_inc * (uint32_t)(c * CH + lane);
            nco_h = nco_tab2[ph >> 22];
            nco_l = nco_tab2[1024 + ((ph >> 12) & 1023)];
        };
        if (p.nco_on && nch > 0) nco_fetch(0);
        // needs: the DC wave done with chunk c - 2 (slot c mod 2)
        run(0, [&](int it) {
            const float2 nco_hc = nco_h, nco_lc = nco_l;  // chunk it's entries
            if (p.nco_on && it + 1 < nch) nco_fetch(it + 1);
            if constexpr (DMA) {
                // batch kb + 2 starts moving when batch kb's first chunk is unpacked (its buffer held batch
                // kb - 1); batch kb + 1 must have landed before the barrier that ends batch kb's last
                // iteration: wait until at most batch kb + 2's 8 DMAs are outstanding (only this wave's
                // DMAs are counted by its vmcnt)
                const int kb = it / BC;
                // batch kb + NRAW - 1 goes into the slot batch kb - 1 left; batch kb + 1 must have landed by
                // the end of batch kb
                if (it % BC == 0 && kb + NRAW - 1 < n_batches) issue_batch(kb + NRAW - 1);
                if (it % BC == BC - 1)  // batches issued beyond kb + 1 may stay in flight
                    wait_raw(min(kb + NRAW - 1, n_batches - 1) - (kb + 1));
            }
            // ---- unpack the I channel of chunk it (lane = 4 x stream + part of CH/4 samples) ----
            {
                const int c = it;
                if (c < nch) {
                    const int sl = lane >> 2, part = lane & 3;
                    float *chunk_w = nco_lds;
                    if (p.nco_on) {
                        // every stream of the engine is at the same phase, so the chunk needs CH phasors, not
                        // PG x CH: lane j forms sample c*CH + j's (the table product of nco_mix with x = 1, 0:
                        // Re(w) = 1*wr - 0*wi = wr exactly, and likewise Im), written to LDS for the whole wave,
                        // planar (CH real parts, then CH imaginary parts) so the mix below runs on sample pairs
                        static_assert(CH == 64, "one phasor per lane");
                        const float2 h = nco_hc, l = nco_lc;
                        chunk_w[lane] = h.x * l.x - h.y * l.y;
                        chunk_w[CH + lane] = h.x * l.y + h.y * l.x;
                        // this wave reads what its own lanes wrote: LDS ops of one wave complete in order
                        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    }
#pragma unroll
                    for (int g8 = 0; g8 < CH / 32; ++g8) {
                        const int within = part * (CH / 4) + g8 * 8;
                        const int t = c * CH + within;
                        float x[8], xq[8];
                        if constexpr (DMA) {
                            constexpr int U4 = 8 * (int)bytes_per_sample<FMT>() / 16;  // 16-B pieces per 8 samples
                            const int off = ((c % BC) * CH + within) * (int)bytes_per_sample<FMT>();
                            const int quarter = off / (RAWB / 4), piece = (off % (RAWB / 4)) >> 4;
                            uint4 u[U4];
#pragma unroll
                            for (int q = 0; q < U4; q++) u[q] = L.raw[(c / BC) % NRAW][(piece + q) * 64 + sl * 4 + quarter];
                            unpack_i8<FMT>(u, x);
                            if (p.nco_on) unpack_q8<FMT>(u, xq);
                        } else {
                            if (s0 + sl < n_frames) {
                                const char *frame = iq + (size_t)(s0 + sl) * p.n_in * bps;
                                load_i8_masked<FMT>(frame, t, n_live, x);
                                if (p.nco_on) {
#pragma unroll
                                    for (int q = 0; q < 8; q++) xq[q] = (t + q < n_live) ? load_q1<FMT>(frame, t + q) : 0.0f;
                                }
                            }
                        }
                        if (p.nco_on) {  // the NCO variant: Re(x w) as nco_mix, then the frame's zero padding
                            // x*wr - xq*wi on sample pairs: two packed products and a packed difference, each
                            // lane of a packed op rounding as the scalar op (no contraction)
                            const float4 *wr4 = reinterpret_cast<const float4 *>(chunk_w + within);
                            const float4 *wi4 = reinterpret_cast<const float4 *>(chunk_w + CH + within);
#pragma unroll
                            for (int h = 0; h < 2; h++) {
                                const float4 wr = wr4[h], wi = wi4[h];  // samples within + 4h .. + 4h + 3
                                const f2v a0 = f2v{x[4 * h], x[4 * h + 1]} * f2v{wr.x, wr.y};
                                const f2v b0 = f2v{xq[4 * h], xq[4 * h + 1]} * f2v{wi.x, wi.y};
                                const f2v a1 = f2v{x[4 * h + 2], x[4 * h + 3]} * f2v{wr.z, wr.w};
                                const f2v b1 = f2v{xq[4 * h + 2], xq[4 * h + 3]} * f2v{wi.z, wi.w};
                                const f2v m0 = a0 - b0, m1 = a1 - b1;
                                x[4 * h] = m0.x;
                                x[4 * h + 1] = m0.y;
                                x[4 * h + 2] = m1.x;
                                x[4 * h + 3] = m1.y;
                            }
                        }
#pragma unroll
                        for (int q = 0; q < 8; q++)
                            if (t + q >= n_live || s0 + sl >= n_frames) x[q] = 0.0f;  // iq.resize() zero padding
                        float *dst = &L.re[c & 1][sl * ROW + within];
                        *reinterpret_cast<float4 *>(dst) = make_float4(x[0], x[1], x[2], x[3]);
                        *reinterpret_cast<float4 *>(dst + 4) = make_float4(x[4], x[5], x[6], x[7]);
                    }
                }
            }
        });
        // no LDS-DMA may still be writing when the workgroup's LDS is released
        if constexpr (DMA) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else if (wave == W_FIR0 || wave == W_FIR1) {
        float facc[MAX_SLOTS / 4] = {};  // FIR accumulators (slots j*4 + lane/16)
        // needs: the clamp wave's chunk c; the equaliser done with chunk c - 2
        run(6 + LA, [&](int c) {
            // ---- FIR accumulation (:136-141) for chunk it-6: lane = (slot mod 4, stream); slot groups
            //      4j..4j+3 split between the two FIR waves ----
            if (c >= 0 && c < nch && PL > 0) {
                const int4 r = chunk_out[c];  // outputs overlapping chunk c: [r.x, r.y] (host table, no division)
                const int sl = lane % PG, sub = lane / PG;
                const int t0 = c * CH;
                if (wave == W_FIR0) {
                    if (nsl_mask == 31) fir_chunk<4, 0>(L, c, t0, r.x, r.y, sub, nsl_mask, sl, D, NT, facc);
                    else if (nsl_mask == 15) fir_chunk<2, 0>(L, c, t0, r.x, r.y, sub, nsl_mask, sl, D, NT, facc);
                    else fir_chunk<1, 0>(L, c, t0, r.x, r.y, sub, nsl_mask, sl, D, NT, facc);
                } else {
                    if (nsl_mask == 31) fir_chunk<4, 4>(L, c, t0, r.x, r.y, sub, nsl_mask, sl, D, NT, facc);
                    else if (nsl_mask == 15) fir_chunk<2, 2>(L, c, t0, r.x, r.y, sub, nsl_mask, sl, D, NT, facc);
                    else if (nsl_mask == 7) fir_chunk<1, 1>(L, c, t0, r.x, r.y, sub, nsl_mask, sl, D, NT, facc);
                }
            }
        });
    } else if (wave == W_OUT) {
        // needs: the AGC wave's chunk c (the low-pass output of chunk c is older); both FIR waves done with chunk c - 2
        run(5 + LA, [&](int c) {
            // ---- AGC output clamp(x * gain, -1, 1) (:108), chunk it-5; zero beyond the frame end ----
            // lane = 4 x stream + part of 8 samples.  x = demodSSB(y, y) = y + y (upper) or y - y (lower)
            // is y * 2 or y * 0: equal values (the lower sideband's zero may carry y's sign, which the
            // clamp keeps and the FIR's sums absorb: acc + (+-0) == acc).  clamp == med3 for non-NaN input.
            if (c >= 0 && c < nch) {
#pragma unroll
                for (int g8 = 0; g8 < CH / 32; ++g8) {
                    const int sl = lane >> 2, part = lane & 3, within = part * (CH / 4) + g8 * 8;
                    const float *gr = &L.g[c & 1][sl * ROW + within];
                    const float *yr = &L.y[c & 3][sl * ROW + within];
                    const float4 ya = *reinterpret_cast<const float4 *>(yr), yb = *reinterpret_cast<const float4 *>(yr + 4);
                    const float4 ga = *reinterpret_cast<const float4 *>(gr), gb = *reinterpret_cast<const float4 *>(gr + 4);
                    const f2v k2 = {demod_k, demod_k};
                    f2v o[4] = {(f2v{ya.x, ya.y} * k2) * f2v{ga.x, ga.y}, (f2v{ya.z, ya.w} * k2) * f2v{ga.z, ga.w},
                                (f2v{yb.x, yb.y} * k2) * f2v{gb.x, gb.y}, (f2v{yb.z, yb.w} * k2) * f2v{gb.z, gb.w}};
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        o[q].x = __builtin_amdgcn_fmed3f(o[q].x, -1.0f, 1.0f);
                        o[q].y = __builtin_amdgcn_fmed3f(o[q].y, -1.0f, 1.0f);
                    }
                    if (c * CH + CH > S) {  // the last chunk only: the FIR reads whole chunks
                        const int t = c * CH + within;
#pragma unroll
                        for (int q = 0; q < 4; q++) {
                            if (t + 2 * q >= S) o[q].x = 0.0f;
                            if (t + 2 * q + 1 >= S) o[q].y = 0.0f;
                        }
                    }
                    float *dst = &L.out[c & 1][sl * ROW + within];
                    *reinterpret_cast<float4 *>(dst) = make_float4(o[0].x, o[0].y, o[1].x, o[1].y);
                    *reinterpret_cast<float4 *>(dst + 4) = make_float4(o[2].x, o[2].y, o[3].x, o[3].y);
                }
            }
        });
    } else if (wave == W_EQ) {
        float h1 = 0.0f, h2 = 0.0f, q1 = 0.0f, q2 = 0.0f, prev = 0.0f;  // HP/BP state (carried), boost prev
        if (serial_live) {
            const SsbStreamState st = state[s0 + my_s];
            h1 = st.hp_z1; h2 = st.hp_z2; q1 = st.bp_z1; q2 = st.bp_z2;
        }
        // audio pulse detector front end on each PCM sample (AudioPulseDetector::process(pcm), pulse_front.h)
        const bool front = af.state != nullptr;
        FrontState fst{};
        if (front && serial_live) fst = front_load(af.state + s0 + my_s);
        float *my_new = front ? af.new_e + (size_t)(serial_live ? s0 + my_s : 0) * (size_t)af.max_new : nullptr;
        int np = 0;
        // needs: both FIR waves' chunk c
        run(7 + LA, [&](int ce) {
            // ---- HP -> BP -> transientBoost -> floatToPCM on the outputs the FIR completed, chunk it-7 ----
            if (ce >= 0 && ce < nch && lane < PG && s0 + my_s < n_frames && PL > 0) {
                const int c = ce;
                const int4 r = chunk_out[c];  // outputs completed in chunk c: [r.z, r.w]
                for (int o = r.z; o <= r.w; o++) {
                    const float in = L.fq[c & 1][my_s * MAX_DONE + (o & (MAX_DONE - 1))];
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
                    pcm[(size_t)(s0 + my_s) * PL + o] = q;
                    if (front) front_sample(af, fst, (float)q * PCM_TO_FLOAT, my_new, np);
                }
            }
        });
        if (serial_live) {
            state[s0 + my_s].hp_z1 = h1;
            state[s0 + my_s].hp_z2 = h2;
            state[s0 + my_s].bp_z1 = q1;
            state[s0 + my_s].bp_z2 = q2;
            if (front) {
                front_store(af.state + s0 + my_s, fst);
                af.new_count[s0 + my_s] = np;
            }
        }
    } else {
        // needs: the low-pass wave's chunk c; the AGC wave done with chunk c - 2
        run(3 + LA, [&](int c) {
            // waves 8-11: lane = CH/16 consecutive samples of one stream (256 lanes = the 16 x CH chunk)
            constexpr int SPL = CH / 16;
            const int hl = (wave == W_DES0 ? 0 : wave == W_DES1 ? 1 : wave == W_DES2 ? 2 : 3) * 64 + lane;
            const int sl = hl / (CH / SPL), i0 = (hl % (CH / SPL)) * SPL;
            // ---- AGC "desired" level (:104-107), chunk it-3 ----
            if (c >= 0 && c < nch) {
#pragma unroll
                for (int h = 0; h < SPL; h += 2) {
                    const float2 y2 = *reinterpret_cast<const float2 *>(&L.y[c & 3][sl * ROW + i0 + h]);
                    // fabsf(demodSSB(y, y)) == |y| * k exactly (k = 2 or 0)
                    const f2v a = f2v{fabsf(y2.x), fabsf(y2.y)} * f2v{demod_k, demod_k};
                    // target / (sqrtf(fabsf(a) + 1e-8f) + 1e-6f), correctly rounded, two lanes per op (ssb_math.h)
                    const f2v d = agc_desired_abs2(a, p.agc_target);
                    *reinterpret_cast<float2 *>(&L.d[c & 1][sl * ROW + i0 + h]) = make_float2(d.x, d.y);
                }
            }
        });
    }
    if (stamps && lane == 0) {  // diagnostic build only: per-wave work cycles and loop cycles
        // the low-pass wave's loop is one asm block with no work stamps: its slot holds the loop's start instead
        // (s_memrealtime, 100 MHz), for the workgroups' start skew
        stamps[(blockIdx.x * PIPE_WAVES + wave) * STAMP_SLOTS] = wave == W_LPF ? st_r0 : st_work;
        stamps[(blockIdx.x * PIPE_WAVES + wave) * STAMP_SLOTS + 1] = __builtin_amdgcn_s_memtime() - st_t0;
        stamps[(blockIdx.x * PIPE_WAVES + wave) * STAMP_SLOTS + 2] = __builtin_amdgcn_s_memrealtime() - st_r0;
        stamps[(blockIdx.x * PIPE_WAVES + wave) * STAMP_SLOTS + 3] = st_entry;
    }

    if (high) __builtin_amdgcn_s_setprio(0);
}

}  // namespace

hipError_t launch_ssb_reference(const void *iq, int fmt, int n_frames, const SsbParams &p, const float *taps,
                      SsbStreamState *state, float *scratch, int16_t *pcm, const AudioFront *audio,
                      hipStream_t stream) {
    if (n_frames <= 0) return hipSuccess;
    const dim3 grid((n_frames + WAVE - 1) / WAVE);
    const char *src = reinterpret_cast<const char *>(iq);
    switch (fmt) {
    case SDRG_IQ_CS8: hipLaunchKernelGGL(ssb_chain_kernel<SDRG_IQ_CS8>, grid, dim3(WAVE), 0, stream, src, n_frames, p, state, scratch); break;
    case SDRG_IQ_CU8: hipLaunchKernelGGL(ssb_chain_kernel<SDRG_IQ_CU8>, grid, dim3(WAVE), 0, stream, src, n_frames, p, state, scratch); break;
    case SDRG_IQ_CS16: hipLaunchKernelGGL(ssb_chain_kernel<SDRG_IQ_CS16>, grid, dim3(WAVE), 0, stream, src, n_frames, p, state, scratch); break;
    case SDRG_IQ_CF32: hipLaunchKernelGGL(ssb_chain_kernel<SDRG_IQ_CF32>, grid, dim3(WAVE), 0, stream, src, n_frames, p, state, scratch); break;
    default: return hipErrorInvalidValue;
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    float *fir_out = scratch + (size_t)n_frames * p.samp_count;
    if (p.pcm_len > 0) {
        const size_t lds = sizeof(float) * (size_t)((WAVE - 1) * p.decim + p.n_taps);
        hipLaunchKernelGGL(ssb_fir_kernel, dim3((p.pcm_len + WAVE - 1) / WAVE, n_frames), dim3(WAVE), lds, stream,
                           scratch, p, taps, fir_out);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(ssb_eq_kernel, grid, dim3(WAVE), 0, stream, fir_out, n_frames, p, state, pcm);
    e = hipGetLastError();
    if (e != hipSuccess || !audio) return e;
    return launch_audio_front(*audio, pcm, 0, p.pcm_len, p.pcm_len, n_frames, stream);
}

bool ssb_force_reference_kernels() {
    static const bool force = [] {
        const char *v = lab_getenv("SDRG_SSB_REFERENCE_KERNELS");
        return v && v[0] == '1';
    }();
    return force;
}

// Diagnostic: SDRG_PIPE_STAMPS=1 makes the pipeline record per-wave work/loop cycles (s_memtime) and
// ssb_report_stamps() print them per role.  Off by default (stamps == nullptr: no instruction executes).
// Each call writes its own slot of a 64-call ring, so the report can average steady-state calls only (a
// pipelined run's first and last calls run partly alone).
constexpr int STAMP_CALLS = 64;
static unsigned long long *g_stamps = nullptr;
static int g_stamps_groups = 0, g_stamp_call = 0;
unsigned long long *ssb_stamps_buffer(int n_frames) {
    static const bool on = [] {
        const char *v = lab_getenv("SDRG_PIPE_STAMPS");
        return v && v[0] == '1';
    }();
    if (!on) return nullptr;
    const int groups = (n_frames + PG - 1) / PG;
    const size_t per_call = (size_t)groups * PIPE_WAVES * STAMP_SLOTS;
    if (groups > g_stamps_groups) {
        if (g_stamps) (void)hipFree(g_stamps);
        if (hipMalloc(reinterpret_cast<void **>(&g_stamps), sizeof(unsigned long long) * per_call * STAMP_CALLS) !=
            hipSuccess)
            return nullptr;
        (void)hipMemset(g_stamps, 0, sizeof(unsigned long long) * per_call * STAMP_CALLS);
        (void)hipStreamSynchronize(nullptr);  // the null-stream fill before any kernel on the engine's streams
        g_stamps_groups = groups;
        g_stamp_call = 0;
    }
    return g_stamps + (size_t)(g_stamp_call++ % STAMP_CALLS) * (size_t)g_stamps_groups * PIPE_WAVES * STAMP_SLOTS;
}

// Per role: work / loop cycles, loop time and effective clock of the last call; then the same averaged over the
// recorded calls except the first and the last (the steady state of a pipelined run).
void ssb_report_stamps() {
    if (!g_stamps || g_stamp_call == 0) return;
    const size_t per_call = (size_t)g_stamps_groups * PIPE_WAVES * STAMP_SLOTS;
    const int ncalls = g_stamp_call < STAMP_CALLS ? g_stamp_call : STAMP_CALLS;
    std::vector<unsigned long long> h(per_call * STAMP_CALLS);
    if (hipMemcpy(h.data(), g_stamps, h.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) return;
    const char *names[PIPE_WAVES] = {"DC", "LPF", "AGC", "LOAD", "FIR-0", "OUT", "EQ", "FIR-1", "DES-0", "DES-1",
                                     "DES-2", "DES-3"};
    const int last = (g_stamp_call - 1) % STAMP_CALLS;
    {  // the workgroups' loop starts (the low-pass wave's slot 0) and ends (start + loop time): skew and span, in us
        double skew = 0, mean_late = 0, span = 0, prologue = 0;
        int sc = 0;
        for (int k = 0; k < ncalls; k++) {
            if (ncalls > 2 && (k == last || k == (g_stamp_call - ncalls) % STAMP_CALLS)) continue;
            const unsigned long long *c = h.data() + (size_t)k * per_call;
            unsigned long long s0 = ~0ull, s1 = 0, e1 = 0;
            double sum = 0, pro = 0;
            for (int g = 0; g < g_stamps_groups; g++) {
                const unsigned long long st = c[(g * PIPE_WAVES + W_LPF) * STAMP_SLOTS], en = st + c[(g * PIPE_WAVES + W_LPF) * STAMP_SLOTS + 2];
                pro += (double)(st - c[(g * PIPE_WAVES + W_LPF) * STAMP_SLOTS + 3]);
                s0 = std::min(s0, st);
                s1 = std::max(s1, st);
                e1 = std::max(e1, en);
                sum += (double)st;
            }
            if (s1 == 0) continue;
            skew += (s1 - s0) / 100.0;
            mean_late += (sum / g_stamps_groups - (double)s0) / 100.0;
            span += (e1 - s0) / 100.0;
            prologue += pro / g_stamps_groups / 100.0;
            sc++;
        }
        for (int j = 0; j < ncalls; j++) {  // per call, in call order: first entry, first loop start, last loop end (10 ns)
            const int k = (g_stamp_call - ncalls + j) % STAMP_CALLS;
            const unsigned long long *c = h.data() + (size_t)k * per_call;
            unsigned long long en0 = ~0ull, st0 = ~0ull, e1 = 0;
            for (int g = 0; g < g_stamps_groups; g++) {
                const unsigned long long *q = c + (size_t)(g * PIPE_WAVES + W_LPF) * STAMP_SLOTS;
                en0 = std::min(en0, q[3]);
                st0 = std::min(st0, q[0]);
                e1 = std::max(e1, q[0] + q[2]);
            }
            fprintf(stderr, "[sdrg stamps] call %d abs entry %llu loop %llu end %llu\n", j, en0, st0, e1);
        }
        if (sc)
            fprintf(stderr, "[sdrg stamps] workgroup loop starts over %d calls: last start - first %.1f us, mean start - first "
                            "%.1f us, first start to last end %.1f us, entry to loop start (mean) %.1f us\n", sc, skew / sc, mean_late / sc,
                    span / sc, prologue / sc);
    }
    for (int w = 0; w < PIPE_WAVES; w++) {
        double work = 0, loop = 0, real = 0, swork = 0, sloop = 0, sreal = 0;
        int sc = 0;
        for (int k = 0; k < ncalls; k++) {
            const unsigned long long *c = h.data() + (size_t)k * per_call;
            double a = 0, b = 0, r = 0;
            for (int g = 0; g < g_stamps_groups; g++) {
                a += c[(g * PIPE_WAVES + w) * STAMP_SLOTS];
                b += c[(g * PIPE_WAVES + w) * STAMP_SLOTS + 1];
                r += c[(g * PIPE_WAVES + w) * STAMP_SLOTS + 2];
            }
            if (k == last) {
                work = a;
                loop = b;
                real = r;
            } else if (ncalls > 2 && k != (g_stamp_call - ncalls) % STAMP_CALLS) {  // not the first recorded call
                swork += a;
                sloop += b;
                sreal += r;
                sc++;
            }
        }
        const double G = g_stamps_groups;
        // effective shader clock over the loop: s_memtime cycles / s_memrealtime (100 MHz) time
        fprintf(stderr,
                "[sdrg stamps] wave %d %-6s last: work %8.0f loop %8.0f cyc %6.1f us %.3f GHz | steady (%d calls): work "
                "%8.0f loop %8.0f cyc %6.1f us %.3f GHz\n",
                w, names[w], work / G, loop / G, real / G / 100.0, real > 0 ? loop / real * 0.1 : 0.0, sc,
                sc ? swork / G / sc : 0.0, sc ? sloop / G / sc : 0.0, sc ? sreal / G / sc / 100.0 : 0.0,
                sreal > 0 ? sloop / sreal * 0.1 : 0.0);
    }
    g_stamp_call = 0;  // the next report covers the calls after this one
    (void)hipMemset(g_stamps, 0, sizeof(unsigned long long) * per_call * STAMP_CALLS);
    (void)hipStreamSynchronize(nullptr);
}

// Outputs whose window can overlap one chunk: floor((CH + NT - 2) / D) + 1; the FIR keeps one accumulator
// per output modulo NSL (a power of two >= that count, at most MAX_SLOTS).
bool ssb_pipe_supported(const SsbParams &p, int *nsl_mask) {
    if (p.pcm_len <= 0) {
        *nsl_mask = 3;
        return true;
    }
    const int ns = (CH + p.n_taps - 2) / p.decim + 1;
    int nsl = 4;
    while (nsl < ns) nsl *= 2;
    *nsl_mask = nsl - 1;
    return nsl <= MAX_SLOTS && (CH + p.decim - 1) / p.decim <= MAX_DONE && p.n_taps <= 256;
}

int ssb_pipe_chunk(void) { return CH; }

// The pipeline kernel goes out through hipExtLaunchKernel with `stop` as its stop event (the event completes with the
// kernel's own dispatch), so the caller records no marker packet between two SSB kernels on the SSB stream, the
// pipelined step's critical path.  Measured (tools/gpu_r4r.sh, alternating, one box): the SSB stream 0.3052-0.3057 vs
// 0.3067-0.3069 ms per call, the c3 line 0.3062-0.3074 vs 0.3071-0.3076 ms.  SDRG_EXT_STOP=0: the marker packet.
#ifndef SDRG_EXT_STOP
#define SDRG_EXT_STOP 1
#endif
hipError_t launch_ssb(const void *iq, int fmt, int n_frames, const SsbParams &p, const float *taps,
                      const int *chunk_table, SsbStreamState *state, float *scratch, int16_t *pcm,
                      const AudioFront *audio, hipStream_t stream, hipEvent_t stop, bool *stop_recorded) {
    if (stop_recorded) *stop_recorded = false;
    if (n_frames <= 0) return hipSuccess;
    int nsl_mask = 3;
    const char *src = reinterpret_cast<const char *>(iq);
    const int4 *chunk_out = reinterpret_cast<const int4 *>(chunk_table);
    if (chunk_out && ssb_pipe_supported(p, &nsl_mask) && !ssb_force_reference_kernels()) {
        const dim3 grid((n_frames + PG - 1) / PG);
        size_t pad = PIPE_LDS_TARGET > (int)sizeof(PipeLds) ? PIPE_LDS_TARGET - sizeof(PipeLds) : 0;
        if (p.nco_on && pad < (size_t)NCO_LDS_BYTES) pad = NCO_LDS_BYTES;  // the dynamic part holds the chunk phasors
#if SDRG_PIPE_DYN_LDS
        pad = sizeof(PipeLds) + (p.nco_on ? NCO_LDS_BYTES : 0);
#define SDRG_PIPE_ATTR_SET(F)                                                                                          \
    {                                                                                                                  \
        hipError_t e1 = ensure_dynamic_lds(reinterpret_cast<const void *>(ssb_pipe_kernel<F, true>),                    \
                                           (int)(sizeof(PipeLds) + NCO_LDS_BYTES));                                    \
        hipError_t e2 = ensure_dynamic_lds(reinterpret_cast<const void *>(ssb_pipe_kernel<F, false>),                   \
                                           (int)(sizeof(PipeLds) + NCO_LDS_BYTES));                                    \
        if (e1 != hipSuccess) return e1;                                                                               \
        if (e2 != hipSuccess) return e2;                                                                               \
    }
        switch (fmt) {
        case SDRG_IQ_CS8: SDRG_PIPE_ATTR_SET(SDRG_IQ_CS8) break;
        case SDRG_IQ_CU8: SDRG_PIPE_ATTR_SET(SDRG_IQ_CU8) break;
        case SDRG_IQ_CS16: SDRG_PIPE_ATTR_SET(SDRG_IQ_CS16) break;
        case SDRG_IQ_CF32: SDRG_PIPE_ATTR_SET(SDRG_IQ_CF32) break;
        default: return hipErrorInvalidValue;
        }
#undef SDRG_PIPE_ATTR_SET
#endif
        const int bps = fmt == SDRG_IQ_CF32 ? 8 : fmt == SDRG_IQ_CS16 ? 4 : 2;
        const int bc = RAWB / (CH * bps) > 0 ? RAWB / (CH * bps) : 1;  // batch_chunks<FMT>()
        const int n_live = p.n_in < p.samp_count ? p.n_in : p.samp_count;
        // LDS-DMA batches need whole 16-B pieces inside every frame
        const bool dma = CH * bps <= RAWB && (n_live % (bc * CH)) == 0 && ((size_t)p.n_in * bps) % 16 == 0 &&
                         (reinterpret_cast<uintptr_t>(iq) & 15) == 0;
        unsigned long long *stamps = ssb_stamps_buffer(n_frames);
        AudioFront af{};
        if (audio) af = *audio;
        static const int prio_mask = [] {  // diagnostic override: SDRG_PIPE_PRIO = bit mask of high-priority waves
            const char *e = lab_getenv("SDRG_PIPE_PRIO");
            // default: the three recurrences at priority 3, the desired-level roles DES0-DES2 (one beside each
            // recurrence's wave on its SIMD under DEFAULT_ROLE_MAP) and the loader at 2.  c3 per step (tools/gpu_r4v.sh,
            // alternating rounds, one box): recurrences alone at 2 (0x7) 0.3086-0.3104 ms, + DES0-DES2 at 2 (0x707)
            // 0.3049-0.3079, recurrences at 3 (0x802A003F) 0.3031-0.3059, + the loader at 2 (0x802A00BF) 0.3018-0.3022
            // (at 1 or 3: 0.3019-0.3039); all four DES roles as three; the other helpers at 1 0.319-0.326
            return e ? (int)strtoul(e, nullptr, 0) : (int)0x802A00BFu;
        }();
        // role of hardware wave w = nibble w (wave w runs on SIMD w % 4); SDRG_PIPE_MAP overrides (diagnostic)
        static const unsigned long long map_override = [] {
            const char *e = lab_getenv("SDRG_PIPE_MAP");
            return e ? strtoull(e, nullptr, 16) : 0ull;
        }();
        const unsigned long long role_map = map_override ? map_override : p.nco_on ? NCO_ROLE_MAP : DEFAULT_ROLE_MAP;
        static const int skip_mask = [] {  // diagnostic only (wrong results): roles whose work is skipped
            const char *e = lab_getenv("SDRG_PIPE_SKIP");
            return e ? (int)strtol(e, nullptr, 0) : 0;
        }();
        const bool ext = SDRG_EXT_STOP && stop;
#define SDRG_PIPE_LAUNCH(F)                                                                                      \
    if (ext)                                                                                                     \
        hipExtLaunchKernelGGL(dma ? ssb_pipe_kernel<F, true> : ssb_pipe_kernel<F, false>, grid, dim3(PIPE_T),   \
                              (uint32_t)pad, stream, nullptr, stop, 0u, src, n_frames, p, nsl_mask, chunk_out, taps,   \
                              state, pcm, stamps, prio_mask, skip_mask, role_map, af);                    \
    else if (dma)                                                                                                \
        hipLaunchKernelGGL((ssb_pipe_kernel<F, true>), grid, dim3(PIPE_T), pad, stream, src, n_frames, p, nsl_mask, \
                           chunk_out, taps, state, pcm, stamps, prio_mask, skip_mask, role_map, af);                                         \
    else                                                                                                         \
        hipLaunchKernelGGL((ssb_pipe_kernel<F, false>), grid, dim3(PIPE_T), pad, stream, src, n_frames, p, nsl_mask, \
                           chunk_out, taps, state, pcm, stamps, prio_mask, skip_mask, role_map, af);
        switch (fmt) {
        case SDRG_IQ_CS8: SDRG_PIPE_LAUNCH(SDRG_IQ_CS8); break;
        case SDRG_IQ_CU8: SDRG_PIPE_LAUNCH(SDRG_IQ_CU8); break;
        case SDRG_IQ_CS16: SDRG_PIPE_LAUNCH(SDRG_IQ_CS16); break;
        case SDRG_IQ_CF32: SDRG_PIPE_LAUNCH(SDRG_IQ_CF32); break;
#undef SDRG_PIPE_LAUNCH
        default: return hipErrorInvalidValue;
        }
        const hipError_t le = hipGetLastError();
        if (le == hipSuccess && ext && stop_recorded) *stop_recorded = true;
        return le;
    }
    return launch_ssb_reference(iq, fmt, n_frames, p, taps, state, scratch, pcm, audio, stream);
}

}  // namespace sdrg

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
// Kernels:
//   ssb_chain_kernel : lane = stream; DC -> LPF -> demod -> AGC over the frame; AGC output -> scratch
//   ssb_fir_kernel   : block = 64 outputs of one stream; input window staged in LDS; each output is the
//                      reference's sequential 255-term sum
//   ssb_eq_kernel    : lane = stream; HP -> BP -> boost -> PCM over the decimated frame
#include "sdrg_internal.h"

#pragma clang fp contract(off)

namespace sdrg {
namespace {

constexpr int WAVE = 64;

__device__ __forceinline__ float clamp_ref(float v, float lo, float hi) {  // std::clamp
    return (v < lo) ? lo : (hi < v) ? hi : v;
}

// Real parts (I) of 8 consecutive samples starting at sample n of a frame (n multiple of 8, all in range).
template <int FMT>
__device__ __forceinline__ void load_i8(const char *frame, int n, float (&x)[8]) {
    if constexpr (FMT == SDRG_IQ_CS8 || FMT == SDRG_IQ_CU8) {
        const uint4 v = *reinterpret_cast<const uint4 *>(frame + 2 * (size_t)n);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int q = 0; q < 4; q++) {
            if constexpr (FMT == SDRG_IQ_CS8) {
                x[2 * q] = (float)(int8_t)(w[q] & 0xff) * (1.0f / 128.0f);
                x[2 * q + 1] = (float)(int8_t)((w[q] >> 16) & 0xff) * (1.0f / 128.0f);
            } else {
                x[2 * q] = ((float)(w[q] & 0xff) - 127.4f) * (1.0f / 128.0f);
                x[2 * q + 1] = ((float)((w[q] >> 16) & 0xff) - 127.4f) * (1.0f / 128.0f);
            }
        }
    } else if constexpr (FMT == SDRG_IQ_CS16) {
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const uint4 v = *reinterpret_cast<const uint4 *>(frame + 4 * (size_t)(n + 4 * h));
            const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int q = 0; q < 4; q++) x[4 * h + q] = (float)(int16_t)(w[q] & 0xffff) * (1.0f / 32768.0f);
        }
    } else {
#pragma unroll
        for (int h = 0; h < 4; h++) {
            const float4 v = *reinterpret_cast<const float4 *>(frame + 8 * (size_t)(n + 2 * h));
            x[2 * h] = v.x;
            x[2 * h + 1] = v.z;
        }
    }
}

template <int FMT>
__device__ __forceinline__ float load_i1(const char *frame, int n) {
    if constexpr (FMT == SDRG_IQ_CS8) return (float)(int8_t)frame[2 * (size_t)n] * (1.0f / 128.0f);
    else if constexpr (FMT == SDRG_IQ_CU8) return ((float)(uint8_t)frame[2 * (size_t)n] - 127.4f) * (1.0f / 128.0f);
    else if constexpr (FMT == SDRG_IQ_CS16)
        return (float)reinterpret_cast<const int16_t *>(frame)[2 * (size_t)n] * (1.0f / 32768.0f);
    else return reinterpret_cast<const float *>(frame)[2 * (size_t)n];
}

template <int FMT>
constexpr int bytes_per_sample() {
    return FMT == SDRG_IQ_CF32 ? 8 : FMT == SDRG_IQ_CS16 ? 4 : 2;
}

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
    const int n8 = live & ~7;
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

}  // namespace

hipError_t launch_ssb(const void *iq, int fmt, int n_frames, const SsbParams &p, const float *taps,
                      SsbStreamState *state, float *scratch, int16_t *pcm, hipStream_t stream) {
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
    return hipGetLastError();
}

}  // namespace sdrg

// fft_codelets.h — in-register FFT codelets on gfx950's packed f32 ops (v_pk_add/mul/fma_f32: one complex
// number per op, f2 = {re, im}), shared by the power-of-two kernels (spectrum.hip) and the any-N kernels
// (fftany.hip).  Included inside an anonymous namespace of each translation unit.
#pragma once

typedef float f2 __attribute__((ext_vector_type(2)));

// exp(-2 pi i k / 32), k in [0, 16)
__device__ constexpr float W32_RE[16] = {1.0f, 0.980785251f, 0.923879504f, 0.831469595f, 0.707106769f,
                                         0.555570245f, 0.382683426f, 0.195090324f, 0.0f, -0.195090324f,
                                         -0.382683426f, -0.555570245f, -0.707106769f, -0.831469595f,
                                         -0.923879504f, -0.980785251f};
__device__ constexpr float W32_IM[16] = {-0.0f, -0.195090324f, -0.382683426f, -0.555570245f, -0.707106769f,
                                         -0.831469595f, -0.923879504f, -0.980785251f, -1.0f, -0.980785251f,
                                         -0.923879504f, -0.831469595f, -0.707106769f, -0.555570245f,
                                         -0.382683426f, -0.195090324f};

template <int R>
__device__ __forceinline__ constexpr int bitrev(int i) {
    int r = 0;
    for (int b = 1; b < R; b <<= 1) {
        r = (r << 1) | (i & 1);
        i >>= 1;
    }
    return r;
}

template <int FMT>
constexpr int bytes_per_sample() {
    return FMT == SDRG_IQ_CF32 ? 8 : FMT == SDRG_IQ_CS16 ? 4 : 2;
}

// ------------------------------------------------------------------------------------------------
// Packed complex helpers (f2 = {re, im} in one 64-bit register pair)
// ------------------------------------------------------------------------------------------------
// a + (-i) b = (a.x + b.y, a.y - b.x)
__device__ __forceinline__ f2 add_mi(f2 a, f2 b) {
    f2 r;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
// a - (-i) b = (a.x - b.y, a.y + b.x)
__device__ __forceinline__ f2 sub_mi(f2 a, f2 b) {
    f2 r;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
// (b.x + b.y, b.y - b.x) = b (1 - i) = b W32^4 / c, c = 1/sqrt2
__device__ __forceinline__ f2 rot45(f2 b) {
    f2 r;
    asm("v_pk_add_f32 %0, %1, %1 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(b));
    return r;
}
// a + c (-i) s = (a.x + c s.y, a.y - c s.x)
__device__ __forceinline__ f2 fma_mi(f2 s, f2 c, f2 a) {
    f2 r;
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[0,1,1] neg_hi:[1,0,0]" : "=v"(r) : "v"(s), "v"(c), "v"(a));
    return r;
}
// a - c (-i) s = (a.x - c s.y, a.y + c s.x)
__device__ __forceinline__ f2 fma_pi(f2 s, f2 c, f2 a) {
    f2 r;
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[0,1,1] neg_lo:[1,0,0]" : "=v"(r) : "v"(s), "v"(c), "v"(a));
    return r;
}
// a * w for a twiddle w held in registers: (a.x w.x, a.x w.y), then + (-a.y w.y, a.y w.x) with the swap
// and the sign as operand modifiers (the compiler otherwise materialises (-w.y, w.x) with v_xor + v_mov)
__device__ __forceinline__ f2 cmul_v(f2 a, f2 w) {
    f2 u, r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(u) : "v"(a), "v"(w));
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]" : "=v"(r) : "v"(a), "v"(w), "v"(u));
    return r;
}

// radix-2 butterfly with twiddle W32^t on b: (a + W b, a - W b)
template <int t>
__device__ __forceinline__ void bfly(f2 &a, f2 &b) {
    constexpr float C = 0.707106769f;
    if constexpr (t == 0) {
        const f2 x = a + b, y = a - b;
        a = x; b = y;
    } else if constexpr (t == 8) {
        const f2 x = add_mi(a, b), y = sub_mi(a, b);
        a = x; b = y;
    } else if constexpr (t == 4) {
        const f2 s = rot45(b);
        const f2 x = a + s * f2{C, C}, y = a - s * f2{C, C};
        a = x; b = y;
    } else if constexpr (t == 12) {
        const f2 s = rot45(b);
        const f2 x = fma_mi(s, f2{C, C}, a), y = fma_pi(s, f2{C, C}, a);
        a = x; b = y;
    } else {
        // x = a + b W as two fmas (b.x W, then b.y iW), y = 2a - x: three packed ops instead of four
        const f2 w = {W32_RE[t], W32_IM[t]}, wi = {-W32_IM[t], W32_RE[t]};
        const f2 x = (a + b.xx * w) + b.yy * wi;
        const f2 y = a * f2{2.0f, 2.0f} - x;
        a = x; b = y;
    }
}

template <int R, int LEN, int BASE, int K>
__device__ __forceinline__ void stage_k(f2 (&v)[R]) {
    if constexpr (K < LEN / 2) {
        bfly<K * (32 / LEN)>(v[BASE + K], v[BASE + K + LEN / 2]);
        stage_k<R, LEN, BASE, K + 1>(v);
    }
}
template <int R, int LEN, int BASE>
__device__ __forceinline__ void stage(f2 (&v)[R]) {
    if constexpr (BASE < R) {
        stage_k<R, LEN, BASE, 0>(v);
        stage<R, LEN, BASE + LEN>(v);
    }
}
template <int R, int LEN>
__device__ __forceinline__ void stages(f2 (&v)[R]) {
    if constexpr (LEN <= R) {
        stage<R, LEN, 0>(v);
        stages<R, LEN * 2>(v);
    }
}

// In-register DFT of R points (R | 32), natural order in and out (radix-2 DIT, bit reversal = renaming).
template <int R>
__device__ __forceinline__ void dft(f2 (&v)[R]) {
    f2 w[R];
#pragma unroll
    for (int i = 0; i < R; ++i) w[bitrev<R>(i)] = v[i];
    stages<R, 2>(w);
#pragma unroll
    for (int i = 0; i < R; ++i) v[i] = w[i];
}


// nh_common.hpp -- shared device code for the gfx950 kernels.
//
// Integer semantics: the reference's transform accumulators are
// numpy int32 scalars, so every sum of products is taken mod 2^32.  All
// butterfly arithmetic here is done on uint32_t (well-defined wrap) and only
// converted to int32 for the arithmetic right shift of the rounding step.
// Because the butterfly is an exact regrouping of the same ring operations, the
// results equal the reference's 3-nested-loop matrix form (transform.py:178-194)
// bit for bit, wrap included.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace nh {

// ---------------------------------------------------------------------------
// Tables (transform.py:20-135, intra.py:24-34, quant.py:21-22)
// ---------------------------------------------------------------------------

// 33 distinct magnitudes of the 32-point basis; DCT32[k][n] = +-TAB[fold((2n+1)k mod 128)].
__host__ __device__ constexpr int dct_tab(int m) {
    constexpr int t[33] = {64, 90, 90, 90, 89, 88, 87, 85, 83, 82, 80, 78, 75, 73, 70, 67,
                           64, 61, 57, 54, 50, 46, 43, 38, 36, 31, 25, 22, 18, 13, 9, 4, 0};
    return t[m];
}
__host__ __device__ constexpr int dct32(int k, int n) {
    if (k == 0) return 64;
    int m = ((2 * n + 1) * k) % 128;
    return m <= 32 ? dct_tab(m) : m <= 64 ? -dct_tab(64 - m) : m <= 96 ? -dct_tab(m - 64) : dct_tab(128 - m);
}
// N-point DCT row k, column n (N | 32): even rows of DCT(2N) are DCT(N).
template <int N>
__host__ __device__ constexpr int dctc(int k, int n) { return dct32(k * (32 / N), n); }

__host__ __device__ constexpr int dst4c(int k, int n) {
    constexpr int t[4][4] = {{29, 55, 74, 84}, {74, 74, 0, -74}, {84, -29, -74, 55}, {55, -84, 74, -29}};
    return t[k][n];
}

__host__ __device__ constexpr int intra_angle(int idx) {  // INTRA_PRED_ANGLE[idx], idx in [0,33)
    constexpr int t[33] = {32, 26, 21, 17, 13, 9, 5, 2, 0, -2, -5, -9, -13, -17, -21, -26, -32,
                           -26, -21, -17, -13, -9, -5, -2, 0, 2, 5, 9, 13, 17, 21, 26, 32};
    return t[idx];
}
__host__ __device__ constexpr int inv_angle(int a) {
    return a == -2 ? -4096 : a == -5 ? -1638 : a == -9 ? -910 : a == -13 ? -630
         : a == -17 ? -482 : a == -21 ? -390 : a == -26 ? -315 : a == -32 ? -256 : 0;
}
__host__ __device__ constexpr int quant_scale(int r) {
    constexpr int t[6] = {26214, 23302, 20560, 18396, 16384, 14564};
    return t[r];
}
__host__ __device__ constexpr int dequant_scale(int r) {
    constexpr int t[6] = {40, 45, 51, 57, 64, 72};
    return t[r];
}

// ---------------------------------------------------------------------------
// Multiply policies (mad(c, x, acc) = c*x + acc mod 2^32).
//   MulWrap : full 32-bit product (v_mul_lo_u32) -- exact for any int32 data.
//   Mul24   : v_mad_i32_i24 (full rate) -- exact when the data operand fits
//             signed 24 bits (proved per call site).  Emitted as inline asm:
//             the compiler's known-bits cannot prove the 24-bit range after a
//             butterfly add, and would fall back to quarter-rate v_mul_lo_u32.
// ---------------------------------------------------------------------------
struct MulWrap {
    static __device__ __forceinline__ uint32_t mad(int c, uint32_t x, uint32_t acc) { return (uint32_t)c * x + acc; }
};
struct Mul24 {
    static __device__ __forceinline__ uint32_t mad(int c, uint32_t x, uint32_t acc) {
        uint32_t r;
        asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(r) : "v"(x), "s"(c), "v"(acc));
        return r;
    }
};

template <class M>
__device__ __forceinline__ uint32_t cmad(int c, uint32_t x, uint32_t acc) {
    if (c == 0) return acc;
    if (c == 64) return (x << 6) + acc;
    if (c == -64) return acc - (x << 6);
    return M::mad(c, x, acc);
}

// ---------------------------------------------------------------------------
// Forward N-point DCT  y[k] = bias + sum_n DCT_N[k][n] x[n]  (mod 2^32),
// recursive even/odd partial butterfly (fully unrolled).  `bias` lets the
// caller fold the rounding constant of transform.py:185 into the accumulators.
// ---------------------------------------------------------------------------
template <int N, class M>
__device__ __forceinline__ void fwd_dct(const uint32_t* x, uint32_t* y, uint32_t bias = 0) {
    if constexpr (N == 2) {
        y[0] = ((x[0] + x[1]) << 6) + bias;
        y[1] = ((x[0] - x[1]) << 6) + bias;
    } else {
        constexpr int H = N / 2;
        uint32_t E[H], O[H], ye[H];
#pragma unroll
        for (int k = 0; k < H; ++k) { E[k] = x[k] + x[N - 1 - k]; O[k] = x[k] - x[N - 1 - k]; }
        fwd_dct<H, M>(E, ye, bias);
#pragma unroll
        for (int m = 0; m < H; ++m) y[2 * m] = ye[m];
#pragma unroll
        for (int m = 0; m < H; ++m) {
            uint32_t acc = bias;
#pragma unroll
            for (int k = 0; k < H; ++k) acc = cmad<M>(dctc<N>(2 * m + 1, k), O[k], acc);
            y[2 * m + 1] = acc;
        }
    }
}

// Inverse N-point:  x[n] = bias + sum_k DCT_N[k][n] y[k]  (mod 2^32)
template <int N, class M>
__device__ __forceinline__ void inv_dct(const uint32_t* y, uint32_t* x, uint32_t bias = 0) {
    if constexpr (N == 2) {
        x[0] = ((y[0] + y[1]) << 6) + bias;
        x[1] = ((y[0] - y[1]) << 6) + bias;
    } else {
        constexpr int H = N / 2;
        uint32_t ye[H], E[H], O[H];
#pragma unroll
        for (int m = 0; m < H; ++m) ye[m] = y[2 * m];
        inv_dct<H, M>(ye, E, bias);
#pragma unroll
        for (int n = 0; n < H; ++n) {
            uint32_t acc = 0;
#pragma unroll
            for (int m = 0; m < H; ++m) acc = cmad<M>(dctc<N>(2 * m + 1, n), y[2 * m + 1], acc);
            O[n] = acc;
        }
#pragma unroll
        for (int n = 0; n < H; ++n) { x[n] = E[n] + O[n]; x[N - 1 - n] = E[n] - O[n]; }
    }
}

// 4x4 DST-VII (no butterfly symmetry): direct 4x4 products.
template <class M>
__device__ __forceinline__ void fwd_dst4(const uint32_t* x, uint32_t* y, uint32_t bias = 0) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        uint32_t acc = bias;
#pragma unroll
        for (int n = 0; n < 4; ++n) acc = cmad<M>(dst4c(k, n), x[n], acc);
        y[k] = acc;
    }
}
template <class M>
__device__ __forceinline__ void inv_dst4(const uint32_t* y, uint32_t* x, uint32_t bias = 0) {
#pragma unroll
    for (int n = 0; n < 4; ++n) {
        uint32_t acc = bias;
#pragma unroll
        for (int k = 0; k < 4; ++k) acc = cmad<M>(dst4c(k, n), y[k], acc);
        x[n] = acc;
    }
}

template <int N, bool DST, class M>
__device__ __forceinline__ void fwd1d(const uint32_t* x, uint32_t* y) {
    if constexpr (DST) fwd_dst4<M>(x, y); else fwd_dct<N, M>(x, y);
}
template <int N, bool DST, class M>
__device__ __forceinline__ void inv1d(const uint32_t* y, uint32_t* x) {
    if constexpr (DST) inv_dst4<M>(y, x); else inv_dct<N, M>(y, x);
}

// (acc + rnd) >> shift on the wrapped int32 (transform.py:185, :194)
template <int SHIFT>
__device__ __forceinline__ int32_t rshift_round(uint32_t acc) {
    return ((int32_t)(acc + (1u << (SHIFT - 1)))) >> SHIFT;
}

template <int N> struct Log2 { static constexpr int v = N == 4 ? 2 : N == 8 ? 3 : N == 16 ? 4 : 5; };

// ---------------------------------------------------------------------------
// Quantizer (quant.py:41-79) for values that fit int32 with |c| < 2^31.
// Fast form: requires a*mf + off < 2^32 (proved at call sites for N=8 int16
// input: |c| <= 2^17, mf < 2^15, off < 2^25).
// ---------------------------------------------------------------------------
struct QuantParams {
    uint32_t mf;
    uint32_t off;
    int32_t shift;
};
__device__ __forceinline__ int32_t quant_fast(int32_t c, const QuantParams& q) {
    uint32_t a = (uint32_t)(c < 0 ? -c : c);
    uint32_t l = (__umul24(a, q.mf) + q.off) >> q.shift;
    return c < 0 ? -(int32_t)l : (int32_t)l;
}
// Signed single-mad form, 4 VALU ops.  Every QUANT_SCALE entry is even, so with
// m' = mf/2, h = off>>1, s' = shift-1:
//   (a*mf + off) >> s == (a*m' + h) >> s'                      (a >= 0)
//   -((a*m' + h) >> s') == (c*m' + (2^s' - 1 - h)) >> s'         (c = -a < 0)
// so level = (c*m' + (c < 0 ? hneg : h)) >> s' with an arithmetic shift.
// Exact when |c| <= 2^17 (|c*m'| < 2^31, c fits the signed 24-bit multiply).
struct QuantS {
    int32_t mh;      // mf / 2
    uint32_t h;      // off >> 1
    uint32_t hneg;   // 2^(shift-1) - 1 - h
    int32_t sh;      // shift - 1
};
__host__ __device__ inline QuantS make_quants(const QuantParams& q) {
    QuantS r;
    r.mh = (int32_t)(q.mf / 2);
    r.h = q.off >> 1;
    r.hneg = (1u << (q.shift - 1)) - 1u - r.h;
    r.sh = q.shift - 1;
    return r;
}
__device__ __forceinline__ int32_t quant_s(int32_t c, const QuantS& q, uint32_t h_v, uint32_t hneg_v) {
    // 4 VALU ops: cmp / cndmask / mad_i32_i24 / ashr.  h_v/hneg_v live in VGPRs
    // (v_cndmask_b32_e32 already reads VCC over the constant bus, so an SGPR
    // source would exceed gfx9's one-scalar limit); mh/sh are SGPRs.
    int32_t r;
    asm("v_cmp_gt_i32_e32 vcc, 0, %1\n\t"
        "v_cndmask_b32_e32 %0, %2, %3, vcc\n\t"
        "v_mad_i32_i24 %0, %1, %4, %0\n\t"
        "v_ashrrev_i32_e32 %0, %5, %0"
        : "=&v"(r)
        : "v"(c), "v"(h_v), "v"(hneg_v), "s"(q.mh), "s"(q.sh)
        : "vcc");
    return r;
}
// quant_s with the sign-dependent rounding offset chosen by a bit-field insert
// instead of a compare + VCC select: sgn = (any value with c's sign) >> 31, the
// offset = v_bfi_b32(sgn, hneg, h).  Two full-rate-class VALU (the shifts) and two
// half-rate-class (bfi, mad) instead of one and three, and no VCC chain between
// neighbouring coefficients.  Same results as quant_s.
__device__ __forceinline__ int32_t quant_sb(int32_t c, int32_t sgn, const QuantS& q, uint32_t h_v) {
    uint32_t hs;
    int32_t r;
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(hs) : "v"(sgn), "s"(q.hneg), "v"(h_v));
    asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(r) : "v"(c), "s"(q.mh), "v"(hs));
    return r >> q.sh;
}
// General int32 form (64-bit product), abs wrapping at int32 min like np.abs.
__device__ __forceinline__ int32_t quant_i32(int32_t c, const QuantParams& q) {
    int64_t a = (c == INT32_MIN) ? (int64_t)c : (int64_t)(c < 0 ? -(int64_t)c : (int64_t)c);
    int64_t l = (int64_t)((uint64_t)a * q.mf + q.off) >> q.shift;
    int64_t s = (c > 0) - (c < 0);
    return (int32_t)(uint32_t)(uint64_t)(s * l);
}
// dequantize (quant.py:112-123) of an int32 level, int64 inside, int32 wrap out
__device__ __forceinline__ int32_t dequant_i32(int32_t l, int32_t scale, int32_t per) {
    uint64_t b = (uint64_t)(int64_t)l * (uint64_t)(int64_t)scale;
    int64_t v;
    if (per < 4) {
        int sh = 4 - per;
        v = (int64_t)(b + (1ull << (sh - 1))) >> sh;
    } else {
        v = (int64_t)(b << (per - 4));
    }
    return (int32_t)(uint32_t)(uint64_t)v;
}

// ---------------------------------------------------------------------------
// Fast unsigned division by a launch constant (n < 2^31).
// ---------------------------------------------------------------------------
struct FastDiv {
    uint32_t d, m, l;
};
static inline FastDiv make_fastdiv(uint32_t d) {
    FastDiv f;
    f.d = d;
    uint32_t l = 0;
    while ((1ull << l) < d) ++l;
    f.l = l;
    f.m = (uint32_t)((((1ull << 32) * ((1ull << l) - d)) / d) + 1);
    return f;
}
__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
    uint32_t t = __umulhi(n, f.m);
    return (t + n) >> f.l;
}

// ---------------------------------------------------------------------------
// XCD-aware workgroup order for one-shot streaming grids.  The dispatcher deals
// workgroup i to XCD i % 8; renumbering so that XCD x runs the x-th eighth of
// the logical workgroups gives each XCD one contiguous address stream (instead
// of all 8 XCDs interleaving over one window) -- +5..10 % on the 8x8 DCT+quant
// stream.  A bijection on [0, nwg): ids past the last whole
// group of 8 keep their number.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t xcd_eighths(uint32_t bid, uint32_t nwg) {
    const uint32_t q = nwg >> 3;
    if (bid >= q * 8u) return bid;
    return (bid & 7u) * q + (bid >> 3);
}

// Quantizer / dequantizer of the intra chains (configs 3-5) with uniform
// parameters, in 32 bits.  Exact whenever the residual is int16: the
// coefficients of every transform (DST4, DCT4..32) are then |c| <= 2^17
// (quant_s's range), |level| <= 52428 (N = 4, QP 0) fits the 24-bit multiply,
// and dequant = (l * dqs + dqr) >> dqsh with dqs = scale << max(0, per-4) is
// quant.py:112-123 without its int64: |l * dqs| < 2^22 at every QP and size.
struct ChainQ {
    QuantS qs;
    uint32_t h_v, hneg_v, dqr_v;   // VGPR operands
    int32_t dqs, dqsh;
};
__device__ __forceinline__ ChainQ make_chainq(const QuantParams& qp, int dq_scale, int dq_per) {
    ChainQ r;
    r.qs = make_quants(qp);
    r.h_v = r.qs.h;
    r.hneg_v = r.qs.hneg;
    r.dqs = dq_per < 4 ? dq_scale : dq_scale << (dq_per - 4);
    r.dqr_v = dq_per < 4 ? 1u << (3 - dq_per) : 0u;
    r.dqsh = dq_per < 4 ? 4 - dq_per : 0;
    asm volatile("" : "+v"(r.h_v), "+v"(r.hneg_v), "+v"(r.dqr_v));
    return r;
}
__device__ __forceinline__ int32_t dequant_s(int32_t l, const ChainQ& q) {
    int32_t r;
    asm("v_mad_i32_i24 %0, %1, %2, %3\n\t"
        "v_ashrrev_i32_e32 %0, %4, %0"
        : "=&v"(r) : "v"(l), "s"(q.dqs), "v"(q.dqr_v), "s"(q.dqsh));
    return r;
}

}  // namespace nh

// nh_packed.hpp -- packed 16-bit 1-D transforms for narrow (8-bit) TUs
// (DESIGN.md §4.4).
//
// One N-point vector per lane, held as int16 PAIRS.  The butterfly's add / sub
// stages are v_pk_add / v_pk_sub on two elements at once (the mirrored operand
// half-swapped through op_sel, no extra instruction), and every multiply stage
// is v_dot2_i32_i16 over a pair with two basis constants, the accumulator an
// int32 (the rounding constant folded in).  Against the 32-bit butterfly of
// nh_common.hpp (fwd_dct / inv_dct): about half the VALU per vector.
//
// Exactness.  Packed operands must be the true values in int16 range; the
// int32 sums are then the reference's exact integer sums (transform.py:178-194,
// :220-236) -- no wrap occurs at these magnitudes.  tools/packed_bounds.py
// enumerates the bounds for residuals in [-255, 255] (every source sample and
// neighbour 8-bit) over every TU kind and QP: largest int16 operand 8,160,
// largest int32 sum 66.6 M.  Callers take this path only for such TUs.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "nh_common.hpp"

namespace nh {

typedef short pk16 __attribute__((ext_vector_type(2)));            // (lo, hi) int16 pair
typedef unsigned short pku16 __attribute__((ext_vector_type(2)));  // the same bits, mod-2^16 arithmetic

__device__ __forceinline__ pk16 pk_swap(pk16 a) { return __builtin_shufflevector(a, a, 1, 0); }
__device__ __forceinline__ pk16 pk_pair(int32_t lo, int32_t hi) { return (pk16){(short)lo, (short)hi}; }
__device__ __forceinline__ pk16 pk_splat(int32_t v) { return (pk16){(short)v, (short)v}; }

// acc + a.lo * c0 + a.hi * c1 (v_dot2_i32_i16, no clamp); c0 / c1 fold to
// constants once the callers' loops are unrolled
__device__ __forceinline__ int32_t pdot(pk16 a, int c0, int c1, int32_t acc) {
    if (c0 == 0 && c1 == 0) return acc;
    return __builtin_amdgcn_sdot2(a, (pk16){(short)c0, (short)c1}, acc, false);
}

// The first term of a sum whose initial accumulator is the constant `init`:
// v_dot2_i32_i16 (VOP3P) with the basis pair from an SGPR (s_mov, SALU) and the
// accumulator an inline 0 or a VGPR -- one VALU instruction, where the
// builtin's VOP2 form (v_dot2c with a literal basis pair) first needs a v_mov to
// seed its accumulator.  Same arithmetic (int32, no clamp).
#ifndef NH_PDOT_FIRST
#define NH_PDOT_FIRST 1
#endif
__device__ __forceinline__ int32_t pdot_first(pk16 a, int c0, int c1, int32_t init) {
    if constexpr (!NH_PDOT_FIRST) {
        return pdot(a, c0, c1, init);
    } else {
        if (c0 == 0 && c1 == 0) return init;
        const uint32_t w = (uint32_t)(uint16_t)c0 | ((uint32_t)(uint16_t)c1 << 16);
        int32_t r;
        if (__builtin_constant_p(init) && init == 0)
            asm("v_dot2_i32_i16 %0, %1, %2, 0" : "=v"(r) : "s"(w), "v"(a));
        else
            asm("v_dot2_i32_i16 %0, %1, %2, %3" : "=v"(r) : "s"(w), "v"(a), "v"(init));
        return r;
    }
}

// Forward N-point DCT of the vector in P (P[j] = (x[2j], x[2j+1])):
// y[k] = bias + sum_n DCT_N[k][n] x[n].  E / O pairs: E[j] = (x[2j] + x[N-1-2j],
// x[2j+1] + x[N-2-2j]) = P[j] + swap(P[N/2-1-j]).
template <int N>
__device__ __forceinline__ void fwd_pk(const pk16* P, int32_t* y, int32_t bias) {
    if constexpr (N == 2) {
        y[0] = pdot_first(P[0], 64, 64, bias);
        y[1] = pdot_first(P[0], 64, -64, bias);
    } else {
        constexpr int H = N / 2, Q = N / 4;
        pk16 E[Q], O[Q];
#pragma unroll
        for (int j = 0; j < Q; ++j) {
            const pk16 m = pk_swap(P[H - 1 - j]);
            E[j] = P[j] + m;
            O[j] = P[j] - m;
        }
        int32_t ye[H];
        fwd_pk<H>(E, ye, bias);
#pragma unroll
        for (int m = 0; m < H; ++m) y[2 * m] = ye[m];
        // odd rows: y[2m+1] = bias + sum_j (O[2j], O[2j+1]) . (T[2m+1][2j], T[2m+1][2j+1])
#pragma unroll
        for (int m = 0; m < H; ++m) {
            int32_t acc = pdot_first(O[0], dctc<N>(2 * m + 1, 0), dctc<N>(2 * m + 1, 1), bias);
#pragma unroll
            for (int j = 1; j < Q; ++j) acc = pdot(O[j], dctc<N>(2 * m + 1, 2 * j), dctc<N>(2 * m + 1, 2 * j + 1), acc);
            y[2 * m + 1] = acc;
        }
    }
}

// Inverse N-point DCT, x[n] = bias + sum_k DCT_N[k][n] y[k], with the input
// pairs in the INVERSE ORDER inv_slot<N>() describes: first the N/4 odd pairs
// (y[4i+1], y[4i+3]) of this level, then the pairs of the even subsequence
// y[2m] (recursively), the last pair being (y[0], y[N/2]).  Callers gather the
// input with 16-bit LDS reads straight into that order (no permutes).
template <int N>
__device__ __forceinline__ void inv_pk(const pk16* Y, int32_t* x, int32_t bias) {
    if constexpr (N == 2) {
        x[0] = pdot_first(Y[0], 64, 64, bias);
        x[1] = pdot_first(Y[0], 64, -64, bias);
    } else {
        constexpr int H = N / 2, Q = N / 4;
        int32_t E[H];
        inv_pk<H>(Y + Q, E, bias);
#pragma unroll
        for (int n = 0; n < H; ++n) {
            int32_t o = pdot_first(Y[0], dctc<N>(1, n), dctc<N>(3, n), 0);
#pragma unroll
            for (int i = 1; i < Q; ++i) o = pdot(Y[i], dctc<N>(4 * i + 1, n), dctc<N>(4 * i + 3, n), o);
            x[n] = E[n] + o;
            x[N - 1 - n] = E[n] - o;
        }
    }
}

// Slot of coefficient k (0..N-1) in inv_pk's input order (pair = slot / 2,
// half = slot % 2).  DST4 takes natural pairs.
template <int N, bool DST>
__device__ __forceinline__ int inv_slot(int k) {
    if constexpr (DST) return k;
    if (k == 0) return N - 2;
    if (k == N / 2) return N - 1;
    const int d = __builtin_ctz((unsigned)k), ko = k >> d;   // k = 2^d * ko, ko odd, d <= log2(N) - 2
    return 2 * (N / 2 - (N >> (d + 1)) + (ko >> 2)) + ((ko >> 1) & 1);
}

// 4x4 DST-VII (transform.py:138-141) on natural pairs (x0, x1), (x2, x3)
__device__ __forceinline__ void fwd_dst4_pk(const pk16* P, int32_t* y, int32_t bias) {
#pragma unroll
    for (int k = 0; k < 4; ++k)
        y[k] = pdot(P[1], dst4c(k, 2), dst4c(k, 3), pdot_first(P[0], dst4c(k, 0), dst4c(k, 1), bias));
}
__device__ __forceinline__ void inv_dst4_pk(const pk16* Y, int32_t* x, int32_t bias) {
#pragma unroll
    for (int n = 0; n < 4; ++n)
        x[n] = pdot(Y[1], dst4c(2, n), dst4c(3, n), pdot_first(Y[0], dst4c(0, n), dst4c(1, n), bias));
}

template <int N, bool DST>
__device__ __forceinline__ void fwd1d_pk(const pk16* P, int32_t* y, int32_t bias) {
    if constexpr (DST) fwd_dst4_pk(P, y, bias); else fwd_pk<N>(P, y, bias);
}
template <int N, bool DST>
__device__ __forceinline__ void inv1d_pk(const pk16* Y, int32_t* x, int32_t bias) {
    if constexpr (DST) inv_dst4_pk(Y, x, bias); else inv_pk<N>(Y, x, bias);
}

// Sum over every aligned group of N lanes (N = 2, 4, ..., 64), each lane receiving
// its group's total.  Inside a 16-lane row the partners come by DPP -- xor 1 and
// xor 2 as quad permutations, the other quad by the half-row mirror, the other
// half-row by the row mirror -- as VALU operand modifiers, not the LDS round trip
// of __shfl_xor's ds_bpermute on the rounds' critical path; the other row of a
// 32-lane half by ds_swizzle (xor 16), the other half by two lane reads.  Integer
// addition mod 2^32 / 2^64 is associative and commutative: the same totals.
template <int CTRL>
__device__ __forceinline__ int32_t lane_perm32(int32_t v) {
    if constexpr (CTRL < 0) return __builtin_amdgcn_ds_swizzle(v, 0x401F);
    else return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}
template <int CTRL, class T>
__device__ __forceinline__ T lane_perm(T v) {
    static_assert(sizeof(T) == 4 || sizeof(T) == 8, "32/64-bit lanes");
    if constexpr (sizeof(T) == 4) {
        return (T)lane_perm32<CTRL>((int32_t)v);
    } else {
        const uint64_t u = (uint64_t)v;
        return (T)((uint64_t)(uint32_t)lane_perm32<CTRL>((int32_t)(uint32_t)u) |
                   ((uint64_t)(uint32_t)lane_perm32<CTRL>((int32_t)(uint32_t)(u >> 32)) << 32));
    }
}
// DPP with a row mask: rows outside ROWMASK keep `old` (row_bcast:15 / :31 of the gfx9 wave reduction)
template <int CTRL, int ROWMASK, class T>
__device__ __forceinline__ T lane_perm_rows(T old, T v) {
    static_assert(sizeof(T) == 4 || sizeof(T) == 8, "32/64-bit lanes");
    if constexpr (sizeof(T) == 4) {
        return (T)__builtin_amdgcn_update_dpp((int32_t)old, (int32_t)v, CTRL, ROWMASK, 0xF, false);
    } else {
        const uint64_t u = (uint64_t)v, o = (uint64_t)old;
        const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp((int32_t)(uint32_t)o, (int32_t)(uint32_t)u, CTRL,
                                                                   ROWMASK, 0xF, false);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp((int32_t)(uint32_t)(o >> 32),
                                                                   (int32_t)(uint32_t)(u >> 32), CTRL, ROWMASK, 0xF, false);
        return (T)((uint64_t)lo | ((uint64_t)hi << 32));
    }
}
template <class T>
__device__ __forceinline__ T lane_read(T v, int l) {
    if constexpr (sizeof(T) == 4) {
        return (T)__builtin_amdgcn_readlane((int32_t)v, l);
    } else {
        const uint64_t u = (uint64_t)v;
        return (T)((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int32_t)(uint32_t)u, l) |
                   ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int32_t)(uint32_t)(u >> 32), l) << 32));
    }
}
template <int N, class T>
__device__ __forceinline__ T grp_sum(T v) {
    static_assert(N >= 2 && N <= 64 && (N & (N - 1)) == 0, "group size");
    v += lane_perm<0xB1>(v);                      // quad_perm [1, 0, 3, 2]
    if constexpr (N >= 4) v += lane_perm<0x4E>(v);    // quad_perm [2, 3, 0, 1]
    if constexpr (N >= 8) v += lane_perm<0x141>(v);   // row_half_mirror
    if constexpr (N >= 16) v += lane_perm<0x140>(v);  // row_mirror
    if constexpr (N == 32) v += lane_perm<-1>(v);     // ds_swizzle: lane ^ 16 inside 32
    if constexpr (N >= 64) {   // every lane holds its row's total: row_bcast:15 then :31 leave the
        // wave's total in lane 63 -- DPP only, no ds_swizzle round trip through the LDS unit
        v += lane_perm_rows<0x142, 0xA>((T)0, v);
        v += lane_perm_rows<0x143, 0xC>((T)0, v);
        v = lane_read(v, 63);
    }
    return v;
}
// The same reduction with min (unsigned / signed per T): every lane gets its group's minimum.
template <int N, class T>
__device__ __forceinline__ T grp_min(T v) {
    static_assert(N >= 2 && N <= 64 && (N & (N - 1)) == 0, "group size");
    auto mn = [](T x, T y) { return y < x ? y : x; };
    v = mn(v, lane_perm<0xB1>(v));
    if constexpr (N >= 4) v = mn(v, lane_perm<0x4E>(v));
    if constexpr (N >= 8) v = mn(v, lane_perm<0x141>(v));
    if constexpr (N >= 16) v = mn(v, lane_perm<0x140>(v));
    if constexpr (N == 32) v = mn(v, lane_perm<-1>(v));
    if constexpr (N >= 64) {   // as grp_sum: rows outside the mask keep their own value
        v = mn(v, lane_perm_rows<0x142, 0xA>(v, v));
        v = mn(v, lane_perm_rows<0x143, 0xC>(v, v));
        v = lane_read(v, 63);
    }
    return v;
}
// __shfl_up(v, 1, 64) by DPP wave_shr:1: lane i gets lane i - 1's value, lane 0 keeps its own
// (the source lane is out of range, and without bound_ctrl the old value -- v -- stays)
__device__ __forceinline__ uint32_t lane_up1(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x138, 0xF, 0xF, false);
}

}  // namespace nh

// nh_mfma.hpp -- int8 matrix-core helpers for the 32x32 transform chain
// (v_mfma_i32_32x32x32_i8), shared by the config-5 kernel (nh_tc32.hip) and the
// config-4 CTU kernel (nh_ctu.hip).  Operand splitting, lane maps and the int8
// DCT32 basis: see nh_tc32.hip's header comment and DESIGN.md §4.5.
#pragma once
#include <hip/hip_runtime.h>
#include "nh_common.hpp"

namespace nh {

typedef int v4i_t __attribute__((ext_vector_type(4)));
typedef int v16i_t __attribute__((ext_vector_type(16)));

__device__ __forceinline__ int crow(int g, int h) { return (g & 3) + 8 * (g >> 2) + 4 * h; }

__device__ __forceinline__ v16i_t mfma(v4i_t a, v4i_t b) {
    v16i_t z = {};
    return __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, z, 0, 0, 0);
}

// Pack the low bytes of 16 int32 values into a 16-byte operand (byte j = v[j]).
__device__ __forceinline__ v4i_t pack16(const int32_t* v) {
    v4i_t r;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        uint32_t lo = __builtin_amdgcn_perm((uint32_t)v[4 * q + 1], (uint32_t)v[4 * q], 0x0c0c0400u);
        uint32_t hi = __builtin_amdgcn_perm((uint32_t)v[4 * q + 3], (uint32_t)v[4 * q + 2], 0x0c0c0400u);
        r[q] = (int)(lo | (hi << 16));
    }
    return r;
}

// Split 16 values into int8 parts (NP = 2 or 3) and pack each part.
template <int NP>
__device__ __forceinline__ void split_pack(const int32_t* v, v4i_t* parts) {
    int32_t t[16];
#pragma unroll
    for (int p = 0; p < NP; ++p) {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int32_t s = v[j] >> (7 * p);
            t[j] = (p == NP - 1) ? s : (s & 127);
        }
        parts[p] = pack16(t);
    }
}

// D = sum_p 128^p * (A_p . B)   (A from data parts)  or  (A . B_p)  (B from data parts)
template <int NP, bool DATA_IS_A>
__device__ __forceinline__ v16i_t mfma_parts(const v4i_t* parts, v4i_t c) {
    v16i_t acc = DATA_IS_A ? mfma(parts[0], c) : mfma(c, parts[0]);
#pragma unroll
    for (int p = 1; p < NP; ++p) {
        v16i_t x = DATA_IS_A ? mfma(parts[p], c) : mfma(c, parts[p]);
#pragma unroll
        for (int g = 0; g < 16; ++g) acc[g] = (int)((uint32_t)acc[g] + ((uint32_t)x[g] << (7 * p)));
    }
    return acc;
}

template <bool DATA_IS_A>
__device__ __forceinline__ v16i_t mfma_auto(const int32_t* v, v4i_t c) {
    int32_t m = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) m = max(m, abs(v[j]));
    v4i_t parts[3];
    if (__any(m >= (1 << 14))) {   // wave-uniform: 3 parts only if some |v| >= 2^14
        split_pack<3>(v, parts);
        return mfma_parts<3, DATA_IS_A>(parts, c);
    }
    split_pack<2>(v, parts);
    return mfma_parts<2, DATA_IS_A>(parts, c);
}

// int8 basis tables: T[k][n] = DCT32[k][n] and its transpose
struct Basis {
    int8_t t[32][32];
    int8_t tt[32][32];
};
inline Basis make_basis() {
    Basis b;
    for (int k = 0; k < 32; ++k)
        for (int n = 0; n < 32; ++n) {
            b.t[k][n] = (int8_t)dct32(k, n);
            b.tt[n][k] = (int8_t)dct32(k, n);
        }
    return b;
}

__device__ __forceinline__ v4i_t load_row16(const int8_t* row, int off) {
    return *(const v4i_t*)(row + off);
}
__device__ __forceinline__ v4i_t load_perm16(const int8_t* row, int h) {
    // bytes j = 0..15 of row[crow(j, h)]: four runs of 4 contiguous bytes
    v4i_t r;
#pragma unroll
    for (int q = 0; q < 4; ++q) r[q] = *(const int*)(row + 8 * q + 4 * h);
    return r;
}

__device__ __forceinline__ int32_t wrap16i(int32_t v) { return (int16_t)(uint16_t)(uint32_t)v; }

}  // namespace nh

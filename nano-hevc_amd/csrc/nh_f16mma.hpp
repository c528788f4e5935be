// nh_f16mma.hpp -- the exact f16 matrix-core pieces of the narrow 32x32 chain
// (DESIGN.md §4.4, §4.5): the DCT32 basis scaled by 2^-10 (exact in f16), its
// operand accessors, and the accumulator helpers.  Shared by the open-loop
// chain (ctu_chain32_h, nh_ctu.hip: configs 4 and 5) and the closed-loop one
// (closed_chain32_h, nh_intraloop.hip: config 4 in closed loop).
#pragma once
#include <hip/hip_runtime.h>
#include "nh_common.hpp"
#include "nh_mfma.hpp"
#include "nh_packed.hpp"

namespace nh {

// f16 DCT32 bases of the narrow 32x32 chain (ctu_chain32_h), every entry
// T[k][n] * 2^-10 (exact in f16), as the matrix and its transpose (4 KB: one
// copy per workgroup in LDS).  Each lane's MFMA operand is one 16-byte piece of
// a row (the data-side passes) or two 8-byte pieces of it in the accumulator
// row order crow (passes 2 and 4, nh_mfma.hpp).
// A per-lane 32-bit byte offset the compiler keeps as one VGPR: base (SGPRs) +
// zext(offset) selects the global_store v_off, s[base] form.
__device__ __forceinline__ uint64_t vofs(uint32_t o) {
    asm("" : "+v"(o));
    return (uint64_t)o;
}

struct BasisH {
    uint16_t t[32][32];          // [k][n] = T[k][n]   pass 1 B operand (lane k); pass 2 A operand (lane l = k)
    uint16_t tt[32][32];         // [n][k] = T[k][n]   inverse pass 1 B operand (lane n); inverse pass 2 A operand
};
inline BasisH make_basis_h() {
    auto h = [](int v) { return __builtin_bit_cast(uint16_t, (_Float16)((float)v / 1024.0f)); };
    BasisH b;
    for (int k = 0; k < 32; ++k)
        for (int n = 0; n < 32; ++n) {
            b.t[k][n] = h(dct32(k, n));
            b.tt[n][k] = h(dct32(k, n));
        }
    return b;
}

// The crow-permuted bases of the transposition-free chain (chain32_tf, round 5):
// for basis row r, MFMA slice s (k range 16s..16s+15) and lane half h, the 8
// halves [16s + 8h, +8) are the basis elements at crow(8s + e, h), e = 0..7 --
// the accumulator row order -- so every pass takes the previous pass's output as
// its A operand in registers, with one 16-B LDS read per basis operand.
struct BasisHC {
    uint16_t tc[32][32];         // [r][16s + 8h + e] = T[r][crow(8s + e, h)]   passes 1 and 2 (lane k / lane l)
    uint16_t ttc[32][32];        // [r][16s + 8h + e] = T[crow(8s + e, h)][r]   inverse passes (lane y / lane x)
    int32_t csum[32];            // S[r] = sum_k T[k][r], the column sums (even)
};
inline BasisHC make_basis_hc() {
    auto h = [](int v) { return __builtin_bit_cast(uint16_t, (_Float16)((float)v / 1024.0f)); };
    BasisHC b;
    for (int r = 0; r < 32; ++r)
        for (int s = 0; s < 2; ++s)
            for (int hh = 0; hh < 2; ++hh)
                for (int e = 0; e < 8; ++e) {
                    const int c = (e & 3) + 16 * s + 8 * (e >> 2) + 4 * hh;   // crow(8s + e, hh)
                    b.tc[r][16 * s + 8 * hh + e] = h(dct32(r, c));
                    b.ttc[r][16 * s + 8 * hh + e] = h(dct32(c, r));
                }
    for (int r = 0; r < 32; ++r) {
        b.csum[r] = 0;
        for (int k = 0; k < 32; ++k) b.csum[r] += dct32(k, r);
    }
    return b;
}

typedef _Float16 h8_t __attribute__((ext_vector_type(8)));
typedef float f16x_t __attribute__((ext_vector_type(16)));

__device__ __forceinline__ h8_t ld_h8(const uint16_t* p) { return __builtin_bit_cast(h8_t, *(const uint4*)p); }
// Elements crow(8s + j, hh), j = 0..7, of a basis row: [16s + 4hh, +4) and [16s + 8 + 4hh, +4).
__device__ __forceinline__ h8_t ld_crow_h8(const uint16_t* row, int s, int hh) {
    const uint2 p = *(const uint2*)(row + 16 * s + 4 * hh), q = *(const uint2*)(row + 16 * s + 8 + 4 * hh);
    return __builtin_bit_cast(h8_t, make_uint4(p.x, p.y, q.x, q.y));
}
// The four operand pieces of each basis a lane reads, as accessors over the LDS
// copy (BasisH) or over registers loaded once per wave (BasisRegs, k_tc32_h:
// 32 VGPRs, no LDS copy and no workgroup barrier).
__device__ __forceinline__ h8_t bq_t(const BasisH& b, int r, int hh, int s) { return ld_h8(&b.t[r][16 * s + 8 * hh]); }
__device__ __forceinline__ h8_t bq_tc(const BasisH& b, int r, int hh, int s) { return ld_crow_h8(b.t[r], s, hh); }
__device__ __forceinline__ h8_t bq_tt(const BasisH& b, int r, int hh, int s) { return ld_h8(&b.tt[r][16 * s + 8 * hh]); }
__device__ __forceinline__ h8_t bq_ttc(const BasisH& b, int r, int hh, int s) { return ld_crow_h8(b.tt[r], s, hh); }
struct BasisRegs {
    h8_t t[2], tc[2], tt[2], ttc[2];
};
__device__ __forceinline__ BasisRegs load_basis_regs(const BasisH& g, int r, int hh) {
    BasisRegs b;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        b.t[s] = bq_t(g, r, hh, s);
        b.tc[s] = bq_tc(g, r, hh, s);
        b.tt[s] = bq_tt(g, r, hh, s);
        b.ttc[s] = bq_ttc(g, r, hh, s);
    }
    return b;
}
__device__ __forceinline__ h8_t bq_t(const BasisRegs& b, int, int, int s) { return b.t[s]; }
__device__ __forceinline__ h8_t bq_tc(const BasisRegs& b, int, int, int s) { return b.tc[s]; }
__device__ __forceinline__ h8_t bq_tt(const BasisRegs& b, int, int, int s) { return b.tt[s]; }
__device__ __forceinline__ h8_t bq_ttc(const BasisRegs& b, int, int, int s) { return b.ttc[s]; }
__device__ __forceinline__ uint32_t pk_floor_h(float a, float b) {   // (floor a, floor b) as an f16 pair
    return __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(__builtin_floorf(a), __builtin_floorf(b)));
}
// Where the rounding bias enters: kBiasInit = the accumulators start at it
// (16 more live registers per pass, no adds), else it is added before floor().
#ifdef NH_ACC_INIT_BIAS
constexpr bool kBiasInit = true;
#else
constexpr bool kBiasInit = false;
#endif
__device__ __forceinline__ float addb(float x, float b) { if constexpr (kBiasInit) return x; else return x + b; }
// (int)floor(x + 0.5) of an accumulator -- the arithmetic shift of the integer
// chain -- in ONE instruction: v_cvt_rpi_i32_f32 rounds half up (floor(x + 0.5))
// as it converts, and x is a multiple of 2^-10 below 2^14, so x + 0.5 is exact
// and the result equals the add / floor / convert sequence.  With the bias in
// the accumulators (kBiasInit) it is floor alone: v_cvt_flr_i32_f32.
#ifndef NH_CVT_RPI
#define NH_CVT_RPI 1
#endif
__device__ __forceinline__ int32_t shift_rnd(float x) {
    if constexpr (!NH_CVT_RPI) {
        return (int32_t)__builtin_floorf(addb(x, 0.5f));
    } else {
        int32_t r;
        if constexpr (kBiasInit) asm("v_cvt_flr_i32_f32 %0, %1" : "=v"(r) : "v"(x));
        else asm("v_cvt_rpi_i32_f32 %0, %1" : "=v"(r) : "v"(x));
        return r;
    }
}
// shift_rnd's v_cvt_rpi is inline asm, and the compiler's hazard recognizer
// inserts no wait states for an inline-asm read of an MFMA result: a conversion
// scheduled right behind the MFMA reads the accumulator's OLD value (seen as
// wrong levels in column 0 of a closed-loop 32x32 TU at QP 0).  Every chain
// therefore passes an accumulator through this block before shift_rnd reads
// it: an s_nop run tied to the accumulator (after the MFMA that writes it,
// before every reader), 24 wait states -- more than the 32x32 MFMA's result
// latency -- for ~24 cycles per pass.
__device__ __forceinline__ void mfma_result_ready(f16x_t& acc) {
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" : "+v"(acc));
}
__device__ __forceinline__ float initb(float b) { if constexpr (kBiasInit) return b; else return 0.0f; }
__device__ __forceinline__ h8_t acc_h8(const f16x_t& acc, int s, float b) {   // registers 8s .. 8s+7 + b, floored, as f16
    uint4 u;
    u.x = pk_floor_h(addb(acc[8 * s + 0], b), addb(acc[8 * s + 1], b));
    u.y = pk_floor_h(addb(acc[8 * s + 2], b), addb(acc[8 * s + 3], b));
    u.z = pk_floor_h(addb(acc[8 * s + 4], b), addb(acc[8 * s + 5], b));
    u.w = pk_floor_h(addb(acc[8 * s + 6], b), addb(acc[8 * s + 7], b));
    return __builtin_bit_cast(h8_t, u);
}
__device__ __forceinline__ f16x_t splat16(float v) {
    f16x_t r;
#pragma unroll
    for (int g = 0; g < 16; ++g) r[g] = v;
    return r;
}

typedef float f2_t __attribute__((ext_vector_type(2)));
// (floor a, floor b) as an f16 pair, for a, b > 0 (truncation)
__device__ __forceinline__ uint32_t pk_trunc_h(float a, float b) {
    return __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(a, b));
}
// floor(acc[8s .. 8s+7] + add) as f16; every value is positive
__device__ __forceinline__ h8_t cvt_h8(const f16x_t& acc, int s, float add) {
    uint32_t u[4];
#pragma unroll
    for (int e = 0; e < 8; e += 2) {
        const f2_t x = (f2_t){acc[8 * s + e], acc[8 * s + e + 1]} + (f2_t){add, add};
        u[e / 2] = pk_trunc_h(x.x, x.y);
    }
    return __builtin_bit_cast(h8_t, make_uint4(u[0], u[1], u[2], u[3]));
}
__device__ __forceinline__ int32_t floor_i32(float x) {   // v_cvt_flr_i32_f32 (after mfma_result_ready)
    int32_t r;
    asm("v_cvt_flr_i32_f32 %0, %1" : "=v"(r) : "v"(x));
    return r;
}
// The per-lane constants of chain32_tf (lane r = lane & 31), made once per wave.
struct TfLane {
    float add1;        // pass 1 -> 2: 1536, 0 on row k = 0 (already 1536 from the residual's 768)
    float add3;        // inverse 1 -> 2: 1536 - 1.5 S[y]
    float add4;        // inverse 2 -> reconstruction: 1536 - 1.5 S[x]
    int32_t fix;       // quantizer: the +3072 of column l = 0
    uint32_t h_v, hneg_v;   // quant_s's rounding words minus fix * m'
};
__device__ __forceinline__ TfLane make_tf_lane(const ChainQ& cq, const BasisHC& bs, int r) {
    const int32_t s = bs.csum[r];   // S[r] = sum_k T[k][r] (even)
    TfLane t;
    t.add1 = r == 0 ? 0.0f : 1536.0f;
    t.add3 = 1536.0f - 1.5f * (float)s;
    t.add4 = t.add3;
    t.fix = r == 0 ? 3072 : 0;
    t.h_v = cq.h_v - (uint32_t)(t.fix * cq.qs.mh);
    t.hneg_v = cq.hneg_v - (uint32_t)(t.fix * cq.qs.mh);
    return t;
}
// quant_s against the lane's offset: c = c_off - fix; the sign test compares with
// fix and the rounding words absorb -fix * m' (|c_off * m'| < 2^31: exact)
__device__ __forceinline__ int32_t quant_tf(int32_t c_off, const QuantS& q, const TfLane& t) {
    int32_t r;
    asm("v_cmp_gt_i32_e32 vcc, %6, %1\n\t"
        "v_cndmask_b32_e32 %0, %2, %3, vcc\n\t"
        "v_mad_i32_i24 %0, %1, %4, %0\n\t"
        "v_ashrrev_i32_e32 %0, %5, %0"
        : "=&v"(r)
        : "v"(c_off), "v"(t.h_v), "v"(t.hneg_v), "s"(q.mh), "s"(q.sh), "v"(t.fix)
        : "vcc");
    return r;
}

// The four passes of the transposition-free chain, shared by the
// config-5 block kernel (chain32_tf, nh_ctu.hip) and the config-4 closed loop's
// 32x32 TUs (closed_chain32_tf, nh_intraloop.hip).  In: the residual + 768 as f16
// pairs hx (lane (r, hh) = column r, rows crow(2p, hh), +1), the chosen prediction
// as 0x6600 - pred pairs in the same layout.  put_level(g, L): the level of row
// k = crow(g, hh), column l = r.  mid(): between the quantizer and the inverse
// passes (e.g. the level rows out of a tile).  Out: the clipped reconstruction
// pairs, same layout as hx.
template <class PutLevel, class Mid>
__device__ __forceinline__ void tf_passes(const uint32_t (&hx)[8], const pku16 (&pr2)[8], const BasisHC& bs,
                                          const ChainQ& cq, const TfLane& tl, int r, int hh, PutLevel&& put_level,
                                          Mid&& mid, pku16 (&rec2)[8]) {
    const h8_t tc0 = ld_h8(&bs.tc[r][8 * hh]), tc1 = ld_h8(&bs.tc[r][16 + 8 * hh]);
    // pass 1 (transform.py:179-185): D1[x][k] = tmp[k][x] (+ 1536 on k = 0) + 0.5, lane k, registers x
    f16x_t acc = splat16(0.5f);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(h8_t, make_uint4(hx[0], hx[1], hx[2], hx[3])),
                                                 tc0, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(h8_t, make_uint4(hx[4], hx[5], hx[6], hx[7])),
                                                 tc1, acc, 0, 0, 0);
    // pass 2 (transform.py:188-194): D2[k][l] = C[k][l] (+ 3072 on l = 0) + 0.5, lane l, registers k
    f16x_t acc2 = splat16(0.5f);
    acc2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(cvt_h8(acc, 0, tl.add1), tc0, acc2, 0, 0, 0);
    acc2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(cvt_h8(acc, 1, tl.add1), tc1, acc2, 0, 0, 0);
    mfma_result_ready(acc2);   // before floor_i32's inline-asm reads
    // quantize_block, and dequantize_block on level pairs in 16 bits ((l * dqs + dqr) >> dqsh:
    // |l * dqs| < 2^15 for 8-bit blocks), entering inverse pass 1 as the f16 bits of 1536 + d
    const pk16 dqs2 = pk_splat(cq.dqs), dqr2 = pk_splat((int32_t)cq.dqr_v), dqsh2 = pk_splat(cq.dqsh);
    uint32_t dq[8];
#pragma unroll
    for (int g = 0; g < 16; g += 2) {
        const int32_t L0 = quant_tf(floor_i32(acc2[g]), cq.qs, tl), L1 = quant_tf(floor_i32(acc2[g + 1]), cq.qs, tl);
        put_level(g, L0);
        put_level(g + 1, L1);
        const pk16 l2 = __builtin_bit_cast(pk16, __builtin_amdgcn_perm((uint32_t)L1, (uint32_t)L0, 0x05040100u));
        dq[g / 2] = __builtin_bit_cast(uint32_t, ((l2 * dqs2 + dqr2) >> dqsh2) + pk_splat(0x6600));
    }
    mid();
    const h8_t tt0 = ld_h8(&bs.ttc[r][8 * hh]), tt1 = ld_h8(&bs.ttc[r][16 + 8 * hh]);
    // inverse pass 1 (transform.py:221-227): D3[l][y] = tmp'[y][l] + 1.5 S[y] + 0.5, lane y, registers l
    f16x_t acc3 = splat16(0.5f);
    acc3 = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(h8_t, make_uint4(dq[0], dq[1], dq[2], dq[3])),
                                                  tt0, acc3, 0, 0, 0);
    acc3 = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(h8_t, make_uint4(dq[4], dq[5], dq[6], dq[7])),
                                                  tt1, acc3, 0, 0, 0);
    // inverse pass 2 (transform.py:230-236): D4[y][x] = R[y][x] + 1.5 S[x] + 0.5, lane x, registers y
    f16x_t acc4 = splat16(0.5f);
    acc4 = __builtin_amdgcn_mfma_f32_32x32x16_f16(cvt_h8(acc3, 0, tl.add3), tt0, acc4, 0, 0, 0);
    acc4 = __builtin_amdgcn_mfma_f32_32x32x16_f16(cvt_h8(acc3, 1, tl.add3), tt1, acc4, 0, 0, 0);
    // reconstruct + clip (intra.py:70-78): the f16 bits of floor(1536 + R + 0.5) are 0x6600 + R for
    // |R| < 512; beyond that (|R| <= 920 for 8-bit blocks: 327 * sum |T[l][x]| / 1024, so the value
    // stays positive) they stay monotone and on the right side of 0x6600 +- 512, so
    // bits - (0x6600 - pred), saturating at 0, then min 255 is the clip of pred + R
#pragma unroll
    for (int p = 0; p < 8; ++p) {
        const f2_t x = (f2_t){acc4[2 * p], acc4[2 * p + 1]} + (f2_t){tl.add4, tl.add4};
        rec2[p] = __builtin_elementwise_min(
            __builtin_elementwise_sub_sat(__builtin_bit_cast(pku16, pk_trunc_h(x.x, x.y)), pr2[p]),
            (pku16){255, 255});
    }
}


}  // namespace nh

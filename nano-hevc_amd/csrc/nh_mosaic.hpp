// nh_mosaic.hpp -- small TUs (4x4 DST / DCT4, 8x8, 16x16) on the f16 matrix cores: MOSAICS
// (round 5).  Shared by the config-4 closed loop (nh_intraloop.hip,
// MosaicSet) and open loop (nh_ctu.hip, ctu_batch_mma): MosaicCore holds the chain from
// the prediction to the reconstruction for NM mosaics; the callers supply the samples,
// the neighbours and where levels / recon go.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "nh_common.hpp"
#include "nh_packed.hpp"
#include "nh_f16mma.hpp"

namespace nh {

// A batch of
// 64 / N TUs of size N (4x4 DST, 8x8 and 16x16 DCT) is NM = N / 4 mosaics of
// 16 x 16 samples -- 16 / N x 16 / N TUs each -- and every 1-D pass of every TU
// of a mosaic is ONE v_mfma_f32_16x16x16_f16 against a block-diagonal basis:
// lane l = (g = l / 16, c = l % 16) holds mosaic column c, rows 4g .. 4g + 3 (the
// A operand of X^T), and each pass's accumulator IS the next pass's A operand
// (it is the transposed product: D1 = temp^T, D2 = coeff, D3 = tmp^T, D4 = rres),
// so the four passes need no transpose -- where the packed chains
// (tu_closed_batch_pk2, ctu_chain_pk) move every TU through an LDS tile three times.  The
// basis enters scaled by 2^-S (exact in f16: |T| <= 90, S <= 9), so each
// accumulator is the reference's sum / 2^S exactly (integer operands below 2048,
// products exact in fp32, sums below 2^24 * 2^-S: tools/packed_bounds.py's
// bounds), and the shift's rounding is the accumulator's
// initial 0.5 then a floor:
//  * the residual enters as the f16 of 768 + n (bits 0x6200 + 2n); the pass-1
//    accumulator starts at 0.5 + 1536 - 768 rs / 2^S (rs = the lane's basis-row
//    sum), so it holds temp + 1536 + frac in [1024, 2048): the truncating
//    conversion to f16 is the floor;
//  * pass 2 starts at 0.5 - 1536 rs / 2^S and floors to the coefficient;
//  * the dequantized coefficients (<= 1024) enter as exact f16 integers, the
//    inverse pass 1 floors to tmp (<= 1936, exact in f16);
//  * the inverse pass 2 starts at 1536.5: clamped to [1280, 1792] its f16 bits
//    are 0x6600 + R' (R' = R clamped to [-256, 256]), and bits - (0x6600 - pred)
//    saturating at 0, then min 255, is the clip of pred + R.
// DCT4 (chroma 4x4): its inverse pass 1 reaches 2223, beyond f16's integers, so
// its inverse pass 2 is two MFMAs into one accumulator: tmp = 2h + b with h =
// floor(tmp / 2) (<= 1112) against the basis * 2^-(S-1), b in {0, 1} against the
// basis * 2^-S.  Same results as the packed chains on 8-bit streams.
typedef _Float16 h4_t __attribute__((ext_vector_type(4)));
typedef float f4_t __attribute__((ext_vector_type(4)));
typedef uint32_t mw4_t __attribute__((ext_vector_type(4)));   // a lane's MosaicLane words as registers
struct alignas(16) MosaicLane {   // per (kind, lane): 32 B
    uint32_t bf[2], bi[2];     // the B operands: Tb^T (passes 1, 2) and Tb (inverse passes), f16 * 2^-S
    float c1, c2;              // the initial accumulators of passes 1 and 2
    uint32_t bi2[2];           // DCT4: Tb * 2^-(S-1) (the inverse pass 2's h half)
};
// kinds: 0 DST4, 1 DCT8, 2 DCT16, 3 DCT4.  One table per translation unit, each uploading its own,
// under a name of its own (NH_MOSAIC_TABLE, defined before the include): a `static` table kept one
// device symbol name in two code objects, and the upload did not reach the kernels.
#ifndef NH_MOSAIC_TABLE
#error "define NH_MOSAIC_TABLE (this translation unit's mosaic table) before including nh_mosaic.hpp"
#endif
__constant__ MosaicLane NH_MOSAIC_TABLE[4][64];
constexpr int Log2Rt(int n) { return n == 4 ? 2 : n == 8 ? 3 : n == 16 ? 4 : 5; }
inline uint16_t f16_bits_exact(int num, int sh) {   // num * 2^-sh as f16 bits (|num| < 2048, a normal result)
    if (num == 0) return 0;
    uint16_t s = num < 0 ? 0x8000 : 0;
    unsigned m = (unsigned)(num < 0 ? -num : num);
    int e = -sh;
    while (m < 1024) { m <<= 1; --e; }   // m in [1024, 2048): value = m * 2^(e)
    return (uint16_t)(s | (uint16_t)((e + 10 + 15) << 10) | (uint16_t)(m & 1023));
}
inline void make_mosaic(MosaicLane (*out)[64]) {
    for (int kind = 0; kind < 4; ++kind) {
        const int N = kind == 1 ? 8 : kind == 2 ? 16 : 4, S = Log2Rt(N) + 5;
        auto T = [&](int k, int n) {
            return kind == 0 ? dst4c(k, n) : kind == 1 ? dctc<8>(k, n) : kind == 2 ? dctc<16>(k, n) : dctc<4>(k, n);
        };
        for (int l = 0; l < 64; ++l) {
            const int c = l & 15, g = l >> 4;
            uint16_t bf[4], bi[4], bi2[4];
            for (int r = 0; r < 4; ++r) {
                const int k = 4 * g + r, same = k / N == c / N;
                bf[r] = same ? f16_bits_exact(T(c % N, k % N), S) : 0;   // B1[k][j] = T[j][k]
                bi[r] = same ? f16_bits_exact(T(k % N, c % N), S) : 0;   // B3[k][j] = T[k][j]
                bi2[r] = same ? f16_bits_exact(T(k % N, c % N), S - 1) : 0;
            }
            int rs = 0;
            for (int n = 0; n < N; ++n) rs += T(c % N, n);
            MosaicLane& m = out[kind][l];
            m.bf[0] = bf[0] | ((uint32_t)bf[1] << 16);
            m.bf[1] = bf[2] | ((uint32_t)bf[3] << 16);
            m.bi[0] = bi[0] | ((uint32_t)bi[1] << 16);
            m.bi[1] = bi[2] | ((uint32_t)bi[3] << 16);
            m.c1 = 0.5f + 1536.0f - 768.0f * (float)rs / (float)(1 << S);
            m.c2 = 0.5f - 1536.0f * (float)rs / (float)(1 << S);
            m.bi2[0] = bi2[0] | ((uint32_t)bi2[1] << 16);
            m.bi2[1] = bi2[2] | ((uint32_t)bi2[3] << 16);
        }
    }
}
// see mfma_result_ready (nh_f16mma.hpp): 8 wait states after a 16x16x16 MFMA -- what the compiler
// itself inserts before a VALU read of such a result (tools/isa_check.py checks every such read)
__device__ __forceinline__ void mfma_result_ready4(f4_t& acc) { asm volatile("s_nop 7" : "+v"(acc)); }
// sum over the lanes of one TU of the mosaic (N = 4: 4 lanes; 8: 8 lanes + the 8 lanes 16 apart; 16: all 64)
template <int N>
__device__ __forceinline__ int32_t tu_sum(int32_t v) {
    if constexpr (N == 4) return grp_sum<4>(v);
    else if constexpr (N == 8) {
        v = grp_sum<8>(v);
        return v + lane_perm<-1>(v);
    } else return grp_sum<64>(v);
}
// DIRECT (the latency form: launches of few CTU rows): levels, recon and TU map leave straight from the
// registers, one sample per lane and store, none of the tile round trip on the chain; otherwise (many
// rows, throughput) as N / 4 whole 16-B row pieces per lane through the tile.
//
// MosaicSet<N, DST, NM>: NM mosaics of TUs of size N whose batch entries start at e0 of a round's
// (entries, cnt per plane, total) list -- one phase of the chain per method, so a batch can run one set
// (tu_closed_batch_mma) or two sets of different sizes interleaved (tu_closed_batch_mix: a round's
// 8x8 and 4x4 TUs in one call, their latencies overlapped instead of added).

// MosaicCore<N, DST, NM>: lane l = (g = l / 16, c = l % 16) of mosaic m holds column t = c % N, rows
// yr0 = 4g % N .. +3 of the batch's TU slot m * TPM + el.  predict() takes the samples sv and a
// neighbour accessor nb (nb.top(m), nb.tr(m), nb.bl(m): top[t], top[N-1], left[N-1]; nb.dcl(m):
// left[t]; nb.left2(m, y): (left[y], left[y + 1])); quant() hands each level pair to put(m, q, L0, L1)
// (rows yr0 + 2q, + 1); recon() each clipped recon pair to put(m, q, pku16).
template <int N, bool DST, int NM>
struct MosaicCore {
    static_assert(N == 4 || ((N == 8 || N == 16) && !DST), "mosaic kinds: DST4, DCT4, DCT8, DCT16");
    static constexpr int L2 = Log2<N>::v, TS = 16 / N, TPM = TS * TS;
    static constexpr int KIND = N == 4 ? (DST ? 0 : 3) : N == 8 ? 1 : 2;
    static constexpr bool SPLIT = N == 4 && !DST;   // DCT4: the inverse pass 2 in two halves
    int t, yr0, el;                                 // column in the TU, first row, TU slot in mosaic 0
    mw4_t mw0, mw1;   // vector type, not uint4: a struct copy from the constant became a memcpy that kept
                      // part of the object in memory (promoted to 20 B of LDS per lane)
    uint32_t hx[NM][2], dq[NM][2];
    pku16 pr2[NM][2];
    f4_t acc[NM];

    __device__ __forceinline__ void lane_init(int lane) {
        const int c = lane & 15, g = lane >> 4;
        t = c % N;
        yr0 = (4 * g) % N;
        el = (4 * g) / N * TS + c / N;
        mw0 = *(const mw4_t*)&NH_MOSAIC_TABLE[KIND][lane];
        mw1 = *((const mw4_t*)&NH_MOSAIC_TABLE[KIND][lane] + 1);
    }
    template <class NB>
    __device__ __forceinline__ void predict(const int32_t (&sv)[NM][4], const NB& nb) {
#pragma unroll
        for (int m = 0; m < NM; ++m) {
            const int32_t topt = nb.top(m), tr = nb.tr(m), bl = nb.bl(m);   // __main__.py:168
            // DC (intra.py:46-62): the TU's lanes of row group 0 add top[t], of row group 1 left[t] (N = 4: both)
            int32_t sdc = N == 4 ? topt + nb.dcl(m) : yr0 == 0 ? topt : yr0 == 4 ? nb.dcl(m) : 0;
            sdc = tu_sum<N>(sdc);
            const int32_t dc = (sdc + N) >> (L2 + 1);
            const pk16 dc2 = pk_splat(dc);
            pk16 o2[2];
            pku16 pl2[2];
            {   // planar (intra.py:81-113) at (y, t): (N-1-t) left[y] + (t+1) tr + (N-1-y) top[t] + (y+1) bl + N >> L2+1
                const int32_t b = (t + 1) * tr + (N - 1 - yr0) * topt + (yr0 + 1) * bl + N, st = bl - topt;
                const pku16 wl = {(unsigned short)(N - 1 - t), (unsigned short)(N - 1 - t)}, sh = {L2 + 1, L2 + 1};
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    o2[q] = pk_pair(sv[m][2 * q], sv[m][2 * q + 1]);
                    const pku16 lf = nb.left2(m, yr0 + 2 * q);
                    const pku16 bs = {(unsigned short)(b + 2 * q * st), (unsigned short)(b + (2 * q + 1) * st)};
                    pl2[q] = (lf * wl + bs) >> sh;
                }
            }
            int32_t ed = 0, ep = 0;
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const pk16 d0 = o2[q] - dc2, d1 = o2[q] - __builtin_bit_cast(pk16, pl2[q]);
                ed = __builtin_amdgcn_sdot2(d0, d0, ed, false);
                ep = __builtin_amdgcn_sdot2(d1, d1, ep, false);
            }
            // DC wins ties (__main__.py:173): ed <= ep as ONE reduction of the difference
            const bool use_dc = tu_sum<N>(ed - ep) <= 0;
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const pk16 pr = use_dc ? dc2 : __builtin_bit_cast(pk16, pl2[q]);
                const pku16 rr = __builtin_bit_cast(pku16, o2[q] - pr);   // residual, intra.py:65-67
                hx[m][q] = __builtin_bit_cast(uint32_t, rr * (pku16){2, 2} + (pku16){0x6200, 0x6200});   // f16 of 768 + n
                pr2[m][q] = (pku16){0x6600, 0x6600} - __builtin_bit_cast(pku16, pr);
            }
        }
    }
    // forward passes (transform.py:179-194)
    __device__ __forceinline__ void pass1() {
        const h4_t bf = __builtin_bit_cast(h4_t, make_uint2(mw0.x, mw0.y));
        const float c1 = __uint_as_float((uint32_t)mw1.x);
#pragma unroll
        for (int m = 0; m < NM; ++m)
            acc[m] = __builtin_amdgcn_mfma_f32_16x16x16f16(__builtin_bit_cast(h4_t, make_uint2(hx[m][0], hx[m][1])), bf,
                                                           (f4_t){c1, c1, c1, c1}, 0, 0, 0);
    }
    __device__ __forceinline__ void pass2() {
        const h4_t bf = __builtin_bit_cast(h4_t, make_uint2(mw0.x, mw0.y));
        const float c2 = __uint_as_float((uint32_t)mw1.y);   // (a bit_cast of the element itself read element 0)
#pragma unroll
        for (int m = 0; m < NM; ++m)
            acc[m] = __builtin_amdgcn_mfma_f32_16x16x16f16(
                __builtin_bit_cast(h4_t, make_uint2(pk_trunc_h(acc[m][0], acc[m][1]), pk_trunc_h(acc[m][2], acc[m][3]))),
                bf, (f4_t){c2, c2, c2, c2}, 0, 0, 0);
    }
    __device__ __forceinline__ void ready() {
#pragma unroll
        for (int m = 0; m < NM; ++m) mfma_result_ready4(acc[m]);   // before floor_i32's inline-asm reads
    }
    // quantize_block (put(m, q, L0, L1): the levels of rows yr0 + 2q, + 1) and dequantize_block in 16 bits
    template <class PUT>
    __device__ __forceinline__ void quant(const ChainQ& cq, PUT&& put) {
        const pk16 dqs2 = pk_splat(cq.dqs), dqr2 = pk_splat((int32_t)cq.dqr_v), dqsh2 = pk_splat(cq.dqsh);
#pragma unroll
        for (int m = 0; m < NM; ++m) {
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int32_t L0 = quant_s(floor_i32(acc[m][2 * q]), cq.qs, cq.h_v, cq.hneg_v);
                const int32_t L1 = quant_s(floor_i32(acc[m][2 * q + 1]), cq.qs, cq.h_v, cq.hneg_v);
                put(m, q, L0, L1);
                const pk16 l2 = __builtin_bit_cast(pk16, __builtin_amdgcn_perm((uint32_t)L1, (uint32_t)L0, 0x05040100u));
                const pk16 d2 = (l2 * dqs2 + dqr2) >> dqsh2;
                const _Float16 h0 = (_Float16)d2.x, h1 = (_Float16)d2.y;
                dq[m][q] = (uint32_t)__builtin_bit_cast(uint16_t, h0) | ((uint32_t)__builtin_bit_cast(uint16_t, h1) << 16);
            }
        }
    }
    // inverse passes (transform.py:221-236)
    __device__ __forceinline__ void inv1() {
        const h4_t bi = __builtin_bit_cast(h4_t, make_uint2(mw0.z, mw0.w));
#pragma unroll
        for (int m = 0; m < NM; ++m)
            acc[m] = __builtin_amdgcn_mfma_f32_16x16x16f16(__builtin_bit_cast(h4_t, make_uint2(dq[m][0], dq[m][1])), bi,
                                                           (f4_t){0.5f, 0.5f, 0.5f, 0.5f}, 0, 0, 0);
    }
    __device__ __forceinline__ void inv2() {
        const h4_t bi = __builtin_bit_cast(h4_t, make_uint2(mw0.z, mw0.w));
        if constexpr (SPLIT) {
            const h4_t bi2 = __builtin_bit_cast(h4_t, make_uint2(mw1.z, mw1.w));
#pragma unroll
            for (int m = 0; m < NM; ++m) {
                // floor(floor(x) / 2) = floor(x / 2); b = floor(x) - 2 h (no arrays: scalars stay in registers)
                const float h0 = __builtin_floorf(acc[m][0] * 0.5f), h1 = __builtin_floorf(acc[m][1] * 0.5f);
                const float h2 = __builtin_floorf(acc[m][2] * 0.5f), h3 = __builtin_floorf(acc[m][3] * 0.5f);
                const float b0 = __builtin_fmaf(-2.0f, h0, __builtin_floorf(acc[m][0]));
                const float b1 = __builtin_fmaf(-2.0f, h1, __builtin_floorf(acc[m][1]));
                const float b2 = __builtin_fmaf(-2.0f, h2, __builtin_floorf(acc[m][2]));
                const float b3 = __builtin_fmaf(-2.0f, h3, __builtin_floorf(acc[m][3]));
                const f4_t a4 = __builtin_amdgcn_mfma_f32_16x16x16f16(
                    __builtin_bit_cast(h4_t, make_uint2(pk_trunc_h(h0, h1), pk_trunc_h(h2, h3))), bi2,
                    (f4_t){1536.5f, 1536.5f, 1536.5f, 1536.5f}, 0, 0, 0);
                acc[m] = __builtin_amdgcn_mfma_f32_16x16x16f16(
                    __builtin_bit_cast(h4_t, make_uint2(pk_trunc_h(b0, b1), pk_trunc_h(b2, b3))), bi, a4, 0, 0, 0);
            }
        } else {
#pragma unroll
            for (int m = 0; m < NM; ++m)
                acc[m] = __builtin_amdgcn_mfma_f32_16x16x16f16(
                    __builtin_bit_cast(h4_t,
                                       make_uint2(pk_floor_h(acc[m][0], acc[m][1]), pk_floor_h(acc[m][2], acc[m][3]))),
                    bi, (f4_t){1536.5f, 1536.5f, 1536.5f, 1536.5f}, 0, 0, 0);
        }
    }
    // reconstruct + clip (intra.py:70-78): put(m, q, rv) with the pair of rows yr0 + 2q, + 1
    template <class PUT>
    __device__ __forceinline__ void recon(PUT&& put) {
#pragma unroll
        for (int m = 0; m < NM; ++m) {
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const float x0 = __builtin_amdgcn_fmed3f(acc[m][2 * q], 1280.0f, 1792.0f);
                const float x1 = __builtin_amdgcn_fmed3f(acc[m][2 * q + 1], 1280.0f, 1792.0f);
                put(m, q, __builtin_elementwise_min(
                              __builtin_elementwise_sub_sat(__builtin_bit_cast(pku16, pk_trunc_h(x0, x1)), pr2[m][q]),
                              (pku16){255, 255}));
            }
        }
    }
};

}  // namespace nh

// nh_intraloop.hip -- frame-level intra drivers on device (configs 3 and 4).
//
// Both compose the reference's per-block functions exactly as DESIGN.md §3.3 /
// §3.4 define them (the reference has no frame-level transform driver; the
// composition follows __main__.py:142-189 and the README chain README.md:55-71),
// with the neighbour rules of block.py:38-55 (source plane = open loop, D12).
// Every per-block step keeps the reference's integer semantics; the oracle
// (the test-side CPU restatement, oh_intra_rdo_plane / oh_tu_pipeline_plane) and the golden
// planes generated from the reference functions pin them.
#include <hip/hip_runtime.h>
#include <mutex>
#include <algorithm>
#include <climits>
#include <cstdlib>
#include "nh_common.hpp"
#include "nh_internal.hpp"
#include "nh_tree.hpp"
#include "nh_packed.hpp"
#include "nh_f16mma.hpp"
#include "nh_ldsdma.hpp"
#define NH_MOSAIC_TABLE c_mosaic_cl
#include "nh_mosaic.hpp"

namespace nh {

// ===========================================================================
// Config 3: 35-mode open-loop RDO per full 8x8 block.
// Workgroup = 7 blocks x 35 modes (245 of 256 lanes): lane = (block slot, mode).
// Each lane runs pred -> residual -> fwd DCT -> quant -> dequant -> inv DCT ->
// recon -> SSE for its mode; an LDS atomicMin on (sse<<6 | mode) picks the
// lowest SSE, lowest mode on ties; the winning lane writes levels/recon/mode.
// Exactness of the 24-bit mads for any int16 plane: DESIGN.md §4.3.
// ===========================================================================
constexpr int kRdoSlots = 7;
constexpr int kModes = 35;
struct RdoPlanes {   // k_intra_rdo8 over gridDim.y planes of one size: plane z = (group z / ppg, plane z % ppg)
    int64_t group_stride, plane_stride;
    int32_t ppg;
};

struct RdoSlotLds {
    int16_t orig[64];
    int16_t topA[17], leftA[17];   // [tl] + up to 16 samples (numpy slice truncation)
    int16_t topN[8], leftN[8];
    int32_t ntA, nlA;              // lengths of topA / leftA (9..17)
    int32_t valid;
    int32_t wide;                  // some orig sample outside [0, 255] (SSE needs 64-bit terms)
    unsigned long long best;
    uint32_t planar[64];           // mode 0 prediction (intra.py:81-113) as (p, 0) pairs, row-major
    uint32_t dcv[8];               // mode 1 prediction (intra.py:46-62) as (dc, 0) pairs
};
constexpr int kRefStride = 27;
__device__ __forceinline__ int16_t wrap16(int32_t v) { return (int16_t)(uint16_t)(uint32_t)v; }     // per-lane angular pair array: 25 pairs, odd stride (LDS banks)

// The per-block part of the prediction, once per block (not per mode lane):
// planar (tr = top[-1], bl = left[-1], __main__.py:168-169) and DC; also flags
// samples outside 8 bits.  k = 0..63 sample index of this thread.
__device__ __forceinline__ void rdo8_block_prep(RdoSlotLds& B, int k) {
    const int y = k >> 3, x = k & 7;
    const int32_t tr = B.topN[7], bl = B.leftN[7];
    const int32_t p = ((7 - x) * B.leftN[y] + (x + 1) * tr + (7 - y) * B.topN[x] + (y + 1) * bl + 8) >> 4;
    B.planar[k] = (uint32_t)p & 0xffffu;
    const int32_t o = B.orig[k];
    if (o < 0 || o > 255) atomicOr(&B.wide, 1);
    // neighbours outside 8 bits: the residual may leave [-255, 255], so the
    // packed 16-bit chain (rdo8_chain_n) is not exact -- wide = 2 selects the
    // 32-bit chain (its SSE in 32 bits is still exact: orig is 8-bit)
    if (k < 17) {
        const int32_t t = B.topA[k], l = B.leftA[k];
        if ((k < B.ntA && (t < 0 || t > 255)) || (k < B.nlA && (l < 0 || l > 255))) atomicOr(&B.wide, 2);
    }
    if (k < 8) {
        int32_t sum = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) sum += B.topN[i] + B.leftN[i];
        B.dcv[k] = (uint32_t)((sum + 8) >> 4) & 0xffffu;   // floor division by 16 (D7)
    }
}

typedef short v2s __attribute__((ext_vector_type(2)));
__device__ __forceinline__ v2s as_v2s(uint32_t u) { return __builtin_bit_cast(v2s, u); }
__device__ __forceinline__ uint32_t as_u32(v2s v) { return __builtin_bit_cast(uint32_t, v); }
// v_dot2_i32_i16 (VOP3P, +16): the builtin selects the accumulating dot2c form,
// which needs an extra move and hazard nops per sample
__device__ __forceinline__ int dot2_16(uint32_t a, uint32_t w) {
    int r;
    asm("v_dot2_i32_i16 %0, %1, %2, 16" : "=v"(r) : "v"(a), "v"(w));
    return r;
}
__device__ __forceinline__ uint32_t dot2_acc(uint32_t a, uint32_t acc) {   // acc + a.x^2 + a.y^2 (int16 lanes)
    uint32_t r;
    asm("v_dot2_i32_i16 %0, %1, %1, %2" : "=v"(r) : "v"(a), "v"(acc));
    return r;
}
__device__ __forceinline__ uint32_t pack16(int32_t lo, int32_t hi) {
    return __builtin_amdgcn_perm((uint32_t)hi, (uint32_t)lo, 0x05040100u);
}

// INTRA_PRED_ANGLE[mode - 2] (intra.py:24-30) and INV_ANGLE (intra.py:32-34)
// for a per-lane mode without a memory table (a constexpr array indexed by a
// lane value compiles to a global load): the 9 magnitudes {0,2,5,9,13,17,21,26,32}
// packed 6 bits each, indexed by the distance to mode 10 / 26.
__device__ __forceinline__ int intra_angle_alu(int mode) {
    constexpr uint64_t kMag = 0ull | (2ull << 6) | (5ull << 12) | (9ull << 18) | (13ull << 24) | (17ull << 30) |
                              (21ull << 36) | (26ull << 42) | (32ull << 48);
    const int d = mode < 18 ? 10 - mode : mode - 26;   // > 0: positive angle
    const int k = d < 0 ? -d : d;
    const int m = (int)((kMag >> (6 * k)) & 63);
    return d < 0 ? -m : m;
}
__device__ __forceinline__ int inv_angle_alu(int angle) {   // angle < 0: -round(8192 / |angle|)
    constexpr uint64_t kLo = 4096ull | (1638ull << 13) | (910ull << 26) | (630ull << 39);
    constexpr uint64_t kHi = 482ull | (390ull << 13) | (315ull << 26) | (256ull << 39);
    const int a = -angle;   // 2, 5, 9, 13, 17, 21, 26, 32
    const int k = a == 2 ? 0 : a == 5 ? 1 : a == 9 ? 2 : a == 13 ? 3 : a == 17 ? 4 : a == 21 ? 5 : a == 26 ? 6 : 7;
    const uint64_t t = k < 4 ? kLo : kHi;
    return -(int)((t >> (13 * (k & 3))) & 8191);
}

// Inverse pass 2 (rows) + rres.astype(int16) + reconstruct_block (int16 wrap) +
// clip_to_pixel_range(., 8) + residual_energy(residual_block(orig, recon)).
// WIDE = false: every orig sample is 8-bit, so |d| <= 255 and the 64 squares
// sum in 32 bits with v_dot2; otherwise 64-bit terms.
template <bool WIDE>
__device__ __forceinline__ unsigned long long rdo8_recon_sse(uint32_t (&X)[8][8], const uint32_t* opk,
                                                             uint32_t (&Rpk)[32]) {
    const v2s zero = {0, 0}, maxv = {255, 255};
    unsigned long long sse = 0;
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        uint32_t x[8];
        inv_dct<8, Mul24>(X[i], x, 128u);
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const v2s rr = as_v2s(pack16((int32_t)x[2 * m] >> 8, (int32_t)x[2 * m + 1] >> 8));
            v2s rc = as_v2s(Rpk[i * 4 + m]) + rr;
            rc = __builtin_elementwise_min(__builtin_elementwise_max(rc, zero), maxv);
            Rpk[i * 4 + m] = as_u32(rc);
            const v2s d = as_v2s(opk[i * 4 + m]) - rc;
            if constexpr (!WIDE) {
                acc = dot2_acc(as_u32(d), acc);
            } else {
                const int32_t d0 = d.x, d1 = d.y;
                sse += (unsigned long long)((uint32_t)(d0 * d0) + (uint32_t)(d1 * d1));
            }
        }
    }
    return WIDE ? sse : (unsigned long long)acc;
}

// One lane's mode of the cfg-3 chain on an 8x8 block whose samples and
// neighbours are in L: prediction (planar / DC / angular, intra.py:46-207) ->
// residual -> fwd DCT -> quant -> dequant -> inv DCT -> recon -> clip -> SSE.
// Returns the SSE; Rpk receives the clipped recon, Lpk the levels (int16 pairs,
// row-major; |level| <= 26214).  refp: this lane's angular pair scratch (LDS).
//
// Prediction is one code path for all 35 modes: Q[s][b] (scan s, base b) =
// ((32-f_s) * r[i] + f_s * r[i+1] + 16) >> 5 in int16 arithmetic (D8), i =
// 9 + b + (proj_s >> 5), read as one (r[i], r[i+1]) pair and one v_dot2; for
// f_s == 0 the same dot with weights (32, 0) and a 27-bit extract gives r[i]
// unwrapped (intra.py:204-206).  Planar and DC lanes read their block's
// precomputed prediction through the same path (f = 0).  P = Q for vertical
// modes and planar/DC, P = Q^T for horizontal modes (intra.py:153-156).
// Prediction of one mode into Rpk (int16 pairs along columns, row-major).
// NARROW: the block's neighbours are 8-bit (wide == 0), so every prediction sample is in
// [0, 255] before the >> 5: an arithmetic shift instead of the 11 / 27-bit extract
template <bool NARROW = false>
__device__ __forceinline__ void rdo8_predict(const RdoSlotLds& L, int mode, uint32_t* refp, uint32_t (&Rpk)[32]) {
    const uint32_t* rowp[8];
    uint32_t wf[8], wd[8];
    bool vert = true;
    if (mode >= 2) {            // _build_ref_array (intra.py:159-188) as pairs
        const int angle = intra_angle_alu(mode);
        vert = mode >= 18;
        const int16_t* pri = vert ? L.topA : L.leftA;
        const int16_t* sec = vert ? L.leftA : L.topA;
        const int np = vert ? L.ntA : L.nlA, ns = vert ? L.nlA : L.ntA;
        int32_t r[25];
#pragma unroll
        for (int i = 0; i < 8; ++i) r[i] = 0;
        r[8] = pri[0];
#pragma unroll
        for (int i = 1; i <= 16; ++i) r[8 + i] = pri[i < np ? i : np - 1];
        if (angle < 0) {
            const int inv = inv_angle_alu(angle), next = (8 * angle) >> 5;
#pragma unroll
            for (int i = -1; i >= -8; --i) {
                const int proj = ((i + 1) * inv + 128) >> 8;
                if (i >= next && proj < ns) r[8 + i] = sec[proj];
            }
        }
#pragma unroll
        for (int i = 0; i < 24; ++i) refp[i] = pack16(r[i], r[i + 1]);
        refp[24] = (uint32_t)r[24] & 0xffffu;
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            const int proj = (s + 1) * angle, f = proj & 31;
            rowp[s] = refp + 9 + (proj >> 5);
            wf[s] = (uint32_t)(32 - f) | ((uint32_t)f << 16);
            wd[s] = f ? 11u : 27u;
        }
    } else {
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            rowp[s] = mode == 0 ? L.planar + 8 * s : L.dcv;
            wf[s] = 32u;
            wd[s] = 27u;
        }
    }
    int32_t Q[8][8];
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const int t = dot2_16(rowp[s][b], wf[s]);
            Q[s][b] = NARROW ? t >> 5 : __builtin_amdgcn_sbfe(t, 5u, wd[s]);
        }
#pragma unroll
    for (int y = 0; y < 8; ++y)
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const uint32_t pv = pack16(Q[y][2 * m], Q[y][2 * m + 1]);
            const uint32_t ph = pack16(Q[2 * m][y], Q[2 * m + 1][y]);
            Rpk[y * 4 + m] = vert ? pv : ph;                       // prediction, until the recon replaces it
        }
}

__device__ __forceinline__ unsigned long long rdo8_chain_n(const RdoSlotLds& L, const ChainQ& q, uint32_t (&Rpk)[32],
                                                           uint32_t (&Lpk)[32]);

// NARROW_ONLY: the caller guarantees wide == 0 (the 32-bit path is not compiled in,
// which frees ~80 VGPRs: config 3's open loop runs 3 waves/SIMD instead of 2)
template <bool NARROW_ONLY = false>
__device__ __forceinline__ unsigned long long rdo8_chain(const RdoSlotLds& L, int mode, uint32_t* refp,
                                                         const ChainQ& q, uint32_t (&Rpk)[32], uint32_t (&Lpk)[32]) {
    rdo8_predict<NARROW_ONLY>(L, mode, refp, Rpk);
    if (NARROW_ONLY || !L.wide) return rdo8_chain_n(L, q, Rpk, Lpk);   // 8-bit block and neighbours: packed 16-bit chain
    uint32_t X[8][8];
    const uint32_t* opk = (const uint32_t*)L.orig;
#pragma unroll
    for (int y = 0; y < 8; ++y)
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const uint32_t d = as_u32(as_v2s(opk[y * 4 + m]) - as_v2s(Rpk[y * 4 + m]));   // residual_block: int16 wrap
            X[y][2 * m] = (uint32_t)(int32_t)(int16_t)(d & 0xffffu);
            X[y][2 * m + 1] = (uint32_t)((int32_t)d >> 16);
        }
#pragma unroll
    for (int j = 0; j < 8; ++j) {           // pass 1: columns
        uint32_t x[8], y[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) x[k] = X[k][j];
        fwd_dct<8, Mul24>(x, y, 128u);
#pragma unroll
        for (int i = 0; i < 8; ++i) X[i][j] = (uint32_t)((int32_t)y[i] >> 8);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {           // pass 2: rows, then quant / dequant
        uint32_t y[8];
        fwd_dct<8, Mul24>(X[i], y, 128u);
        int32_t l[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            l[j] = quant_s((int32_t)y[j] >> 8, q.qs, q.h_v, q.hneg_v);
            X[i][j] = (uint32_t)dequant_s(l[j], q);
        }
#pragma unroll
        for (int m = 0; m < 4; ++m) Lpk[i * 4 + m] = pack16(l[2 * m], l[2 * m + 1]);
    }
    // inverse pass 1: columns (transform.py:221-227)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        uint32_t yv[8], x[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) yv[k] = X[k][j];
        inv_dct<8, Mul24>(yv, x, 128u);
#pragma unroll
        for (int i = 0; i < 8; ++i) X[i][j] = (uint32_t)((int32_t)x[i] >> 8);
    }
    // inverse pass 2: rows, recon, SSE (two copies: 8-bit blocks sum d^2 in 32 bits)
    return (L.wide & 1) ? rdo8_recon_sse<true>(X, opk, Rpk) : rdo8_recon_sse<false>(X, opk, Rpk);
}

// ---------------------------------------------------------------------------
// Packed 16-bit chain for 8-bit blocks (wide == 0: orig and every neighbour in
// [0, 255], so prediction is in [0, 255] and the residual in [-255, 255]).
// Two independent 8-point vectors a, b travel as int16 pairs (a_k, b_k): the
// butterfly's add / sub stages are v_pk_add/sub_u16 on both at once, the
// multiply stages v_dot2_i32_i16 over (k, k') pairs of one vector (int32
// accumulate, the rounding constant as the accumulator), and ">> 8 then
// int16" of two int32 results is one v_perm (bytes 1..2 of each).  Exact:
// every packed operand is the true value in int16 range -- pass-1 E/O <= 510
// and EE <= 1,020; pass-1 outputs >> 8 <= 510 (row sums of |DCT8| <= 512);
// pass-2 EE <= 2,040; coefficients |C| <= 1,020; dequantized
// values <= 720 at every QP (quant.py's shift includes log2 N, its dequant
// does not: D3/D4); inverse pass-1 outputs >> 8 <= 1,347 (column sums of
// |DCT8| = 479), pass-2 >> 8 <= 2,520 -- and the int32 sums are the
// reference's, which never wrap at these sizes (bounds enumerated over QP
// 0..51 in DESIGN.md §4.3).
// The same mod-2^32 results as rdo8_chain's 32-bit path, element for element.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t pk_add16(uint32_t a, uint32_t b) {
    uint32_t r;
    asm("v_pk_add_u16 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ uint32_t pk_sub16(uint32_t a, uint32_t b) {
    uint32_t r;
    asm("v_pk_sub_u16 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
// acc + a.lo * w.lo + a.hi * w.hi (signed int16 pairs, int32 accumulate)
__device__ __forceinline__ int32_t dot2w(uint32_t a, uint32_t w, int32_t acc) {
    int32_t r;
    asm("v_dot2_i32_i16 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(w), "v"(acc));
    return r;
}
__device__ __forceinline__ uint32_t lo_pair(uint32_t x, uint32_t y) { return __builtin_amdgcn_perm(y, x, 0x05040100u); }  // (x.lo, y.lo)
__device__ __forceinline__ uint32_t hi_pair(uint32_t x, uint32_t y) { return __builtin_amdgcn_perm(y, x, 0x07060302u); }  // (x.hi, y.hi)
__device__ __forceinline__ uint32_t shr8_pair(int32_t x, int32_t y) {                                                   // (x >> 8, y >> 8) as int16
    return __builtin_amdgcn_perm((uint32_t)y, (uint32_t)x, 0x06050201u);
}
constexpr uint32_t wpair(int c0, int c1) { return (uint32_t)(uint16_t)(int16_t)c0 | ((uint32_t)(uint16_t)(int16_t)c1 << 16); }

// forward 8-point DCT of the two vectors in P (pairs (a_k, b_k)): ya / yb = bias + DCT8 . a / b
__device__ __forceinline__ void fwd8_pk2(const uint32_t (&P)[8], int32_t bias, int32_t (&ya)[8], int32_t (&yb)[8]) {
    uint32_t E[4], O[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        E[k] = pk_add16(P[k], P[7 - k]);
        O[k] = pk_sub16(P[k], P[7 - k]);
    }
    const uint32_t EE0 = pk_add16(E[0], E[3]), EE1 = pk_add16(E[1], E[2]);
    const uint32_t EO0 = pk_sub16(E[0], E[3]), EO1 = pk_sub16(E[1], E[2]);
    const uint32_t ee[2] = {lo_pair(EE0, EE1), hi_pair(EE0, EE1)};
    const uint32_t eo[2] = {lo_pair(EO0, EO1), hi_pair(EO0, EO1)};
    const uint32_t o01[2] = {lo_pair(O[0], O[1]), hi_pair(O[0], O[1])};
    const uint32_t o23[2] = {lo_pair(O[2], O[3]), hi_pair(O[2], O[3])};
#pragma unroll
    for (int v = 0; v < 2; ++v) {
        int32_t* y = v ? yb : ya;
        y[0] = dot2w(ee[v], wpair(64, 64), bias);
        y[4] = dot2w(ee[v], wpair(64, -64), bias);
        y[2] = dot2w(eo[v], wpair(dctc<4>(1, 0), dctc<4>(1, 1)), bias);
        y[6] = dot2w(eo[v], wpair(dctc<4>(3, 0), dctc<4>(3, 1)), bias);
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const int r = 2 * m + 1;
            y[r] = dot2w(o23[v], wpair(dctc<8>(r, 2), dctc<8>(r, 3)),
                         dot2w(o01[v], wpair(dctc<8>(r, 0), dctc<8>(r, 1)), bias));
        }
    }
}

// inverse 8-point DCT of the two vectors in P: xa / xb = bias + DCT8^T . a / b
__device__ __forceinline__ void inv8_pk2(const uint32_t (&P)[8], int32_t bias, int32_t (&xa)[8], int32_t (&xb)[8]) {
    const uint32_t y13[2] = {lo_pair(P[1], P[3]), hi_pair(P[1], P[3])};
    const uint32_t y57[2] = {lo_pair(P[5], P[7]), hi_pair(P[5], P[7])};
    const uint32_t y04[2] = {lo_pair(P[0], P[4]), hi_pair(P[0], P[4])};
    const uint32_t y26[2] = {lo_pair(P[2], P[6]), hi_pair(P[2], P[6])};
#pragma unroll
    for (int v = 0; v < 2; ++v) {
        int32_t* x = v ? xb : xa;
        int32_t O[4];
#pragma unroll
        for (int n = 0; n < 4; ++n)
            O[n] = dot2w(y57[v], wpair(dctc<8>(5, n), dctc<8>(7, n)), dot2w(y13[v], wpair(dctc<8>(1, n), dctc<8>(3, n)), 0));
        const int32_t EO0 = dot2w(y26[v], wpair(dctc<4>(1, 0), dctc<4>(3, 0)), 0);
        const int32_t EO1 = dot2w(y26[v], wpair(dctc<4>(1, 1), dctc<4>(3, 1)), 0);
        const int32_t EE0 = dot2w(y04[v], wpair(64, 64), bias);
        const int32_t EE1 = dot2w(y04[v], wpair(64, -64), bias);
        const int32_t E[4] = {EE0 + EO0, EE1 + EO1, EE1 - EO1, EE0 - EO0};
#pragma unroll
        for (int n = 0; n < 4; ++n) {
            x[n] = E[n] + O[n];
            x[7 - n] = E[n] - O[n];
        }
    }
}

// The chain after prediction (Rpk = prediction pairs along columns) for a
// wide == 0 block; same outputs as rdo8_chain's 32-bit path.
__device__ __forceinline__ unsigned long long rdo8_chain_n(const RdoSlotLds& L, const ChainQ& q, uint32_t (&Rpk)[32],
                                                           uint32_t (&Lpk)[32]) {
    const uint32_t* opk = (const uint32_t*)L.orig;
    uint32_t D[8][4];   // residual, (column 2m, 2m+1) pairs per row: D[row][m]
#pragma unroll
    for (int y = 0; y < 8; ++y)
#pragma unroll
        for (int m = 0; m < 4; ++m) D[y][m] = pk_sub16(opk[y * 4 + m], Rpk[y * 4 + m]);   // residual_block
    uint32_t T[4][8];   // pass-1 output >> 8, (row 2i, 2i+1) pairs per column: T[i][col]
#pragma unroll
    for (int m = 0; m < 4; ++m) {           // forward pass 1: columns 2m, 2m+1 (transform.py:179-185)
        uint32_t P[8];
        int32_t ya[8], yb[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) P[k] = D[k][m];
        fwd8_pk2(P, 128, ya, yb);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            T[i][2 * m] = shr8_pair(ya[2 * i], ya[2 * i + 1]);
            T[i][2 * m + 1] = shr8_pair(yb[2 * i], yb[2 * i + 1]);
        }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {           // forward pass 2: rows 2i, 2i+1, then quant / dequant
        int32_t za[8], zb[8];
        fwd8_pk2(T[i], 128, za, zb);
        int32_t la[8], lb[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            la[j] = quant_sb(za[j] >> 8, za[j] >> 31, q.qs, q.h_v);
            lb[j] = quant_sb(zb[j] >> 8, zb[j] >> 31, q.qs, q.h_v);
        }
        // dequantize_block on the level pairs (v_pk_mad + v_pk_ashr): l * dqs + dqr stays within
        // int16 for 8-bit 8x8 blocks at every QP (tools/packed_bounds.py rdo8_dequant_bounds)
        const pk16 dqs2 = pk_splat(q.dqs), dqr2 = pk_splat((int32_t)q.dqr_v), dqsh2 = pk_splat(q.dqsh);
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            Lpk[(2 * i) * 4 + m] = pack16(la[2 * m], la[2 * m + 1]);
            Lpk[(2 * i + 1) * 4 + m] = pack16(lb[2 * m], lb[2 * m + 1]);
            D[2 * i][m] = __builtin_bit_cast(uint32_t, (__builtin_bit_cast(pk16, Lpk[(2 * i) * 4 + m]) * dqs2 + dqr2) >> dqsh2);
            D[2 * i + 1][m] = __builtin_bit_cast(uint32_t, (__builtin_bit_cast(pk16, Lpk[(2 * i + 1) * 4 + m]) * dqs2 + dqr2) >> dqsh2);
        }
    }
#pragma unroll
    for (int m = 0; m < 4; ++m) {           // inverse pass 1: columns 2m, 2m+1 (transform.py:221-227)
        uint32_t P[8];
        int32_t xa[8], xb[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) P[k] = D[k][m];
        inv8_pk2(P, 128, xa, xb);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            T[i][2 * m] = shr8_pair(xa[2 * i], xa[2 * i + 1]);
            T[i][2 * m + 1] = shr8_pair(xb[2 * i], xb[2 * i + 1]);
        }
    }
    const v2s zero = {0, 0}, maxv = {255, 255};
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {           // inverse pass 2: rows 2i, 2i+1 + recon + clip + SSE
        int32_t ra[8], rb[8];
        inv8_pk2(T[i], 128, ra, rb);
#pragma unroll
        for (int half = 0; half < 2; ++half) {
            const int y = 2 * i + half;
            const int32_t* r = half ? rb : ra;
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const v2s rr = as_v2s(shr8_pair(r[2 * m], r[2 * m + 1]));   // rres.astype(int16)
                v2s rc = as_v2s(Rpk[y * 4 + m]) + rr;                        // reconstruct_block (int16)
                rc = __builtin_elementwise_min(__builtin_elementwise_max(rc, zero), maxv);
                Rpk[y * 4 + m] = as_u32(rc);
                const v2s d = as_v2s(opk[y * 4 + m]) - rc;
                acc = dot2_acc(as_u32(d), acc);
            }
        }
    }
    return (unsigned long long)acc;
}


// CHAIN: 0 = either chain per block; 1 = the packed chain only -- a group with
// any wide block is marked (modes = 0xFF) and left to the CHAIN 2 launch that
// follows, which skips every group not so marked (ONESHOT only).
template <int WAVES, bool ONESHOT, int CHAIN = 0>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WAVES))) k_intra_rdo8(const int16_t* __restrict__ src, int w, int h, int pitch,
                                                    QuantParams qp, int dq_scale, int dq_per, uint8_t* modes,
                                                    int32_t* lvl, int16_t* recon, unsigned long long* sse_out,
                                                    uint32_t ngroups, int vec_out, RdoPlanes pg) {
    __shared__ RdoSlotLds S[kRdoSlots];
    __shared__ uint32_t refs[kRdoSlots * kModes][kRefStride];
    __shared__ unsigned long long wg_sse;
    const int bw = w / 8, bh = h / 8;
    const int nblk = bw * bh;
    const int t = threadIdx.x;
    const int slot = t / kModes, mode = t - slot * kModes;
    const bool lane_on = slot < kRdoSlots;
    {   // plane blockIdx.y of the set (nh_intra_rdo_planes): its samples, levels and recon at the plane's
        // offset, its modes after the previous planes' and its own SSE word
        const int pz = (int)blockIdx.y, gz = pz / pg.ppg;
        const int64_t poff = (int64_t)gz * pg.group_stride + (int64_t)(pz - gz * pg.ppg) * pg.plane_stride;
        src += poff;
        lvl += poff;
        recon += poff;
        modes += (int64_t)pz * nblk;
        if (sse_out) sse_out += pz;
    }
    // A workgroup adds its SSE to *sse_out ONCE (one 64-bit word takes ~90
    // atomic adds/us: an atomic per block serialised the whole launch).
    // ONESHOT: one group of 7 blocks per workgroup; else persistent, groups
    // walked with stride gridDim.x.
    if (t == 0) wg_sse = 0;   // (first read after the barriers below)
    if constexpr (CHAIN == 2) {   // fallback launch: only the groups the packed-only launch left
        if (modes[(int64_t)blockIdx.x * kRdoSlots] != 0xFF) return;
    }
    auto body = [&](const uint32_t grp) __attribute__((always_inline)) {

    // ---- cooperative load of the 7 blocks' samples and neighbours ----
    // Every global load is issued before the first LDS write, so the workgroup
    // waits for one memory latency, not one per loop trip.
    const int b0 = (int)grp * kRdoSlots;
    int16_t vo0 = 0, vo1 = 0, vn = 128, vtl = 128;
    auto orig_at = [&](int e) -> const int16_t* {
        const int b = b0 + e / 64, k = e % 64;
        const int by = b / bw, bx = b - by * bw;
        return src + (int64_t)(by * 8 + k / 8) * pitch + bx * 8 + (k % 8);
    };
    const bool o0 = b0 + t / 64 < nblk;                          // e = t (t < 256 <= 448)
    const bool o1 = t + 256 < kRdoSlots * 64 && b0 + (t + 256) / 64 < nblk;
    if (o0) vo0 = *orig_at(t);
    if (o1) vo1 = *orig_at(t + 256);
    const int nsl = t / 32, nk = t % 32;                         // neighbour sample (t < 224)
    const bool nv = t < kRdoSlots * 32 && b0 + nsl < nblk;
    int nby = 0, nbx = 0;
    if (nv) {
        const int b = b0 + nsl;
        nby = b / bw;
        nbx = b - nby * bw;
        const int x = nbx * 8, y = nby * 8;
        // top row samples x..x+15 (block.py:38-43) / left column y..y+15 (block.py:45-50)
        const bool top = nk < 16;
        const int kk = nk - 16;
        const bool in = top ? (y > 0 && x + nk < w) : (x > 0 && y + kk < h);
        const int ry = top ? y - 1 : y + kk, rx = top ? x + nk : x - 1;
        if (in) vn = src[(int64_t)ry * pitch + rx];
    }
    const bool tv = t < kRdoSlots && b0 + t < nblk;
    int tby = 0, tbx = 0;
    if (tv) {
        tby = (b0 + t) / bw;
        tbx = b0 + t - tby * bw;
        if (tby > 0 && tbx > 0) vtl = src[(int64_t)(tby * 8 - 1) * pitch + tbx * 8 - 1];
    }
    if (o0) S[t / 64].orig[t % 64] = vo0;
    if (o1) S[(t + 256) / 64].orig[(t + 256) % 64] = vo1;
    if (nv) {
        if (nk < 16) {
            S[nsl].topA[1 + nk] = vn;
            if (nk < 8) S[nsl].topN[nk] = vn;
        } else {
            S[nsl].leftA[1 + nk - 16] = vn;
            if (nk < 24) S[nsl].leftN[nk - 16] = vn;
        }
    }
    if (t < kRdoSlots) {
        S[t].valid = tv;
        if (tv) {
            const int x = tbx * 8, y = tby * 8;
            S[t].topA[0] = vtl;
            S[t].leftA[0] = vtl;
            S[t].ntA = 1 + (y == 0 ? 16 : min(16, w - x));
            S[t].nlA = 1 + (x == 0 ? 16 : min(16, h - y));
        }
        S[t].best = ULLONG_MAX;
        S[t].wide = 0;
    }
    __syncthreads();
    for (int e = t; e < kRdoSlots * 64; e += 256)
        if (S[e / 64].valid) rdo8_block_prep(S[e / 64], e % 64);
    __syncthreads();
    if constexpr (CHAIN == 1) {   // a wide block in the group: leave the group to the fallback launch
        bool any_wide = false;
#pragma unroll
        for (int k = 0; k < kRdoSlots; ++k) any_wide |= S[k].valid && S[k].wide;
        if (any_wide) {
            if (t < kRdoSlots && S[t].valid) modes[b0 + t] = 0xFF;
            return;   // uniform over the workgroup; nothing of wg_sse to add
        }
    }
    const bool active = lane_on && S[lane_on ? slot : 0].valid;
    RdoSlotLds& L = S[lane_on ? slot : 0];
    const ChainQ rq = make_chainq(qp, dq_scale, dq_per);

    // ---- the mode's chain ----
    uint32_t P[32], Lv[32];
    unsigned long long key = ULLONG_MAX;
    if (active) {
        const unsigned long long sse = rdo8_chain<CHAIN == 1>(L, mode, refs[t], rq, P, Lv);
        key = (sse << 6) | (unsigned long long)mode;
        atomicMin(&L.best, key);
    }
    __syncthreads();
    if (active && key == L.best) {
        const int b = b0 + slot;
        const int by = b / bw, bx = b - by * bw;
        modes[b] = (uint8_t)mode;
        atomicAdd(&wg_sse, key >> 6);   // LDS: no register lives across the loop
        // (A/B: handing the block to the workgroup through LDS for wave-wide
        // stores measured 0.225 vs 0.222 ms/frame -- the winners' stores overlap
        // the other wave's chain here; kept in the closed loop, where they do not)
        if (vec_out) {   // 16-B aligned rows (the launch checks pitch and bases): 3 stores a row, not 16
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                int32_t* lrow = lvl + (int64_t)(by * 8 + i) * pitch + bx * 8;
                int16_t* rrow = recon + (int64_t)(by * 8 + i) * pitch + bx * 8;
                *(uint4*)rrow = make_uint4(P[i * 4], P[i * 4 + 1], P[i * 4 + 2], P[i * 4 + 3]);
                int32_t lv[8];
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    lv[2 * m] = __builtin_amdgcn_sbfe((int32_t)Lv[i * 4 + m], 0u, 16u);
                    lv[2 * m + 1] = (int32_t)Lv[i * 4 + m] >> 16;
                }
                *(int4*)lrow = make_int4(lv[0], lv[1], lv[2], lv[3]);
                *(int4*)(lrow + 4) = make_int4(lv[4], lv[5], lv[6], lv[7]);
            }
        } else {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                int32_t* lrow = lvl + (int64_t)(by * 8 + i) * pitch + bx * 8;
                int16_t* rrow = recon + (int64_t)(by * 8 + i) * pitch + bx * 8;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    lrow[j] = (int32_t)(int16_t)(Lv[i * 4 + j / 2] >> (16 * (j & 1)));
                    rrow[j] = (int16_t)(P[i * 4 + j / 2] >> (16 * (j & 1)));
                }
            }
        }
    }
    __syncthreads();   // S / refs are refilled by the next group
    };
    if constexpr (ONESHOT) {
        body(blockIdx.x);
    } else {
        for (uint32_t grp = blockIdx.x; grp < ngroups; grp += gridDim.x) body(grp);
    }
    if (sse_out && t == 0) atomicAdd(sse_out, wg_sse);   // after the last barrier
}

#if NH_AB   // the mosaic forms of config 3 (A/B build only: not faster, see nh_intra_rdo_plane)
// ---------------------------------------------------------------------------
// Config 3 on f16 MFMA MOSAICS (round 6): the same 35 chains per 8x8 block, but
// a chain is no longer one lane's registers.  Each 8x8 TU (block, mode) is a
// quarter of a 16x16 mosaic (MosaicCore<8, false, 2>, nh_mosaic.hpp: the
// closed loop's exact f16 chain) -- lane (g, c) holds column
// c % 8, rows 4g % 8 .. +3 of one TU -- so each 1-D pass of 4 TUs is one
// v_mfma_f32_16x16x16_f16, and a lane's VALU work is its 4 samples'
// prediction, conversions, quantizer and reconstruction instead of a TU's
// butterflies.  Phases per group of 7 blocks (8-bit only: a group with a wide
// block is left to the general fallback launch, as k_intra_rdo8<.., 1>):
//   A. lane (slot, mode) builds its mode's angular reference pairs in LDS
//      (_build_ref_array, intra.py:159-188; as rdo8_predict);
//   B. the waves walk the 245 TUs 8 at a time (two mosaics per call): each lane
//      predicts its 4 samples (intra.py:46-207 through the same pair/dot2 path
//      as rdo8_predict), the chain runs, the TU's SSE of orig - recon
//      (residual_energy(residual_block(orig, recon))) is reduced over its 16
//      lanes and (sse << 6 | mode) goes to the block's LDS minimum: lowest SSE,
//      lowest mode on ties (__main__.py:97);
//   C. wave 0 runs the 7 winning TUs again with their levels, recon and mode
//      map written out (1 extra call per 245 TUs), and the group adds the
//      winners' SSE to the plane's total once.
// Same outputs as k_intra_rdo8 (every operand exact: tools/packed_bounds.py
// mosaic_bounds, DCT8 row).
// REF16: the reference as 25 int16 samples (13 words per TU: LDS for 8 waves per SIMD), a pair read as
// two samples; else as 25 (r[i], r[i + 1]) pairs
template <bool REF16>
__device__ __forceinline__ void rdo8_build_refs(const RdoSlotLds& L, int mode, uint32_t* refp) {
    const int angle = intra_angle_alu(mode);
    const bool vert = mode >= 18;
    const int16_t* pri = vert ? L.topA : L.leftA;
    const int16_t* sec = vert ? L.leftA : L.topA;
    const int np = vert ? L.ntA : L.nlA, ns = vert ? L.nlA : L.ntA;
    int32_t r[25];
#pragma unroll
    for (int i = 0; i < 8; ++i) r[i] = 0;
    r[8] = pri[0];
#pragma unroll
    for (int i = 1; i <= 16; ++i) r[8 + i] = pri[i < np ? i : np - 1];
    if (angle < 0) {
        const int inv = inv_angle_alu(angle), next = (8 * angle) >> 5;
#pragma unroll
        for (int i = -1; i >= -8; --i) {
            const int proj = ((i + 1) * inv + 128) >> 8;
            if (i >= next && proj < ns) r[8 + i] = sec[proj];
        }
    }
    if constexpr (REF16) {
#pragma unroll
        for (int i = 0; i < 12; ++i) refp[i] = pack16(r[2 * i], r[2 * i + 1]);
        refp[12] = (uint32_t)r[24] & 0xffffu;
    } else {
#pragma unroll
        for (int i = 0; i < 24; ++i) refp[i] = pack16(r[i], r[i + 1]);
        refp[24] = (uint32_t)r[24] & 0xffffu;
    }
}
template <bool REF16>
__device__ __forceinline__ uint32_t rdo8_ref_pair(const uint32_t* refp, int i) {   // (r[i], r[i + 1])
    if constexpr (REF16) {
        const int16_t* q = (const int16_t*)refp;
        return pack16(q[i], q[i + 1]);
    } else {
        return refp[i];
    }
}
// The prediction of rows y0 .. y0 + 3 of column x for mode `mode` (rdo8_predict's Q / P)
template <bool REF16>
__device__ __forceinline__ void rdo8_pred_col4(const RdoSlotLds& L, const uint32_t* refp, int mode, int y0, int x,
                                               int32_t (&pr)[4]) {
    if (mode < 2) {
#pragma unroll
        for (int r = 0; r < 4; ++r) pr[r] = mode == 0 ? (int16_t)L.planar[8 * (y0 + r) + x] : (int16_t)L.dcv[0];
        return;
    }
    const int angle = intra_angle_alu(mode);
    if (mode >= 18) {   // vertical: P = Q, scan line = row
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int proj = (y0 + r + 1) * angle, f = proj & 31;
            const int tt = dot2_16(rdo8_ref_pair<REF16>(refp, 9 + x + (proj >> 5)), (uint32_t)(32 - f) | ((uint32_t)f << 16));
            pr[r] = __builtin_amdgcn_sbfe(tt, 5u, f ? 11u : 27u);
        }
    } else {            // horizontal: P = Q^T (intra.py:153-156), scan line = column: one weight pair
        const int proj = (x + 1) * angle, f = proj & 31;
        const uint32_t wf = (uint32_t)(32 - f) | ((uint32_t)f << 16), wd = f ? 11u : 27u;
        const int i0 = 9 + y0 + (proj >> 5);
#pragma unroll
        for (int r = 0; r < 4; ++r) pr[r] = __builtin_amdgcn_sbfe(dot2_16(rdo8_ref_pair<REF16>(refp, i0 + r), wf), 5u, wd);
    }
}
// One call: two mosaics = 8 TUs; tu_of(k) gives TU k's (slot, mode) or slot < 0 (idle).
// keep(m, q, L0, L1, rv...) hooks: OUT = true writes levels / recon / mode (the winners).
template <bool OUT, int NM, bool REF16, class TuOf>
__device__ __forceinline__ void rdo8_mma_call(const RdoSlotLds* S, const uint32_t* refs, int rstride, const ChainQ& rq,
                                              TuOf&& tu_of, uint32_t* best, int b0, int bw, int pitch, int32_t* lvl,
                                              int16_t* recon, uint8_t* modes) {
    using MC = MosaicCore<8, false, NM>;
    MC mc;
    mc.lane_init(threadIdx.x & 63);
    int slot[NM], mode[NM];
    int32_t sv[NM][4];
#pragma unroll
    for (int m = 0; m < NM; ++m) {
        tu_of(4 * m + mc.el, slot[m], mode[m]);
        const int sl = slot[m] < 0 ? 0 : slot[m], md = slot[m] < 0 ? 1 : mode[m];   // idle: block 0's DC
        const RdoSlotLds& L = S[sl];
        int32_t pr[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) sv[m][r] = L.orig[8 * (mc.yr0 + r) + mc.t];
        rdo8_pred_col4<REF16>(L, refs + (sl * kModes + md) * rstride, md, mc.yr0, mc.t, pr);
#pragma unroll
        for (int q = 0; q < 2; ++q) {   // as MosaicCore::predict: residual + 768 as f16, 0x6600 - pred
            const pk16 o2 = pk_pair(sv[m][2 * q], sv[m][2 * q + 1]), p2 = pk_pair(pr[2 * q], pr[2 * q + 1]);
            const pku16 rr = __builtin_bit_cast(pku16, o2 - p2);   // residual_block, intra.py:65-67
            mc.hx[m][q] = __builtin_bit_cast(uint32_t, rr * (pku16){2, 2} + (pku16){0x6200, 0x6200});
            mc.pr2[m][q] = (pku16){0x6600, 0x6600} - __builtin_bit_cast(pku16, p2);
        }
    }
    mc.pass1();
    mc.pass2();
    mc.ready();
    auto bpos = [&](int m, int row) -> int64_t {   // sample offset of (row, column t) of TU m's block
        const int b = b0 + slot[m], by = b / bw, bx = b - by * bw;
        return (int64_t)(by * 8 + row) * pitch + bx * 8 + mc.t;
    };
    mc.quant(rq, [&](int m, int q, int32_t L0, int32_t L1) {
        if constexpr (OUT) {
            if (slot[m] < 0) return;
            const int64_t o = bpos(m, mc.yr0 + 2 * q);
            lvl[o] = L0;
            lvl[o + pitch] = L1;
        }
    });
    mc.inv1();
    mc.inv2();
    int32_t e[NM];
#pragma unroll
    for (int m = 0; m < NM; ++m) e[m] = 0;
    mc.recon([&](int m, int q, pku16 rv) {
        const pk16 d = pk_pair(sv[m][2 * q], sv[m][2 * q + 1]) - __builtin_bit_cast(pk16, rv);   // |d| <= 255
        e[m] = __builtin_amdgcn_sdot2(d, d, e[m], false);
        if constexpr (OUT) {
            if (slot[m] < 0) return;
            const int64_t o = bpos(m, mc.yr0 + 2 * q);
            recon[o] = (int16_t)rv.x;
            recon[o + pitch] = (int16_t)rv.y;
        }
    });
#pragma unroll
    for (int m = 0; m < NM; ++m) {
        const int32_t sse = tu_sum<8>(e[m]);   // the TU's 64 squared differences (< 2^22)
        if (slot[m] >= 0 && mc.t == 0 && mc.yr0 == 0) {
            if constexpr (OUT) {
                modes[b0 + slot[m]] = (uint8_t)mode[m];
            } else {
                atomicMin(&best[slot[m]], ((uint32_t)sse << 6) | (uint32_t)mode[m]);
            }
        }
    }
}

// NMS: mosaics per call in phase B (2: 8 TUs, 4: 16 TUs); REF16: int16 reference arrays
template <int WAVES, int NMS = 2, bool REF16 = false>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WAVES)))
k_intra_rdo8_mma(const int16_t* __restrict__ src, int w, int h, int pitch, QuantParams qp, int dq_scale, int dq_per,
                 uint8_t* modes, int32_t* lvl, int16_t* recon, unsigned long long* sse_out) {
    __shared__ RdoSlotLds S[kRdoSlots];
    constexpr int RS = REF16 ? 13 : kRefStride;   // words per TU's reference (odd: conflict-free)
    __shared__ uint32_t refs[kRdoSlots * kModes * RS];
    __shared__ uint32_t best[kRdoSlots];
    const int bw = w / 8, bh = h / 8;
    const int nblk = bw * bh;
    const int t = threadIdx.x, wv = t >> 6;
    const int b0 = (int)blockIdx.x * kRdoSlots;
    // ---- the 7 blocks' samples and neighbours (as k_intra_rdo8) ----
    int16_t vo0 = 0, vo1 = 0, vn = 128, vtl = 128;
    auto orig_at = [&](int e) -> const int16_t* {
        const int b = b0 + e / 64, k = e % 64;
        const int by = b / bw, bx = b - by * bw;
        return src + (int64_t)(by * 8 + k / 8) * pitch + bx * 8 + (k % 8);
    };
    const bool o0 = b0 + t / 64 < nblk;
    const bool o1 = t + 256 < kRdoSlots * 64 && b0 + (t + 256) / 64 < nblk;
    if (o0) vo0 = *orig_at(t);
    if (o1) vo1 = *orig_at(t + 256);
    const int nsl = t / 32, nk = t % 32;
    const bool nv = t < kRdoSlots * 32 && b0 + nsl < nblk;
    if (nv) {
        const int b = b0 + nsl, nby = b / bw, nbx = b - nby * bw;
        const int x = nbx * 8, y = nby * 8;
        const bool top = nk < 16;   // top row x..x+15 (block.py:38-43) / left column y..y+15 (block.py:45-50)
        const int kk = nk - 16;
        const bool in = top ? (y > 0 && x + nk < w) : (x > 0 && y + kk < h);
        const int ry = top ? y - 1 : y + kk, rx = top ? x + nk : x - 1;
        if (in) vn = src[(int64_t)ry * pitch + rx];
    }
    const bool tv = t < kRdoSlots && b0 + t < nblk;
    int tby = 0, tbx = 0;
    if (tv) {
        tby = (b0 + t) / bw;
        tbx = b0 + t - tby * bw;
        if (tby > 0 && tbx > 0) vtl = src[(int64_t)(tby * 8 - 1) * pitch + tbx * 8 - 1];
    }
    if (o0) S[t / 64].orig[t % 64] = vo0;
    if (o1) S[(t + 256) / 64].orig[(t + 256) % 64] = vo1;
    if (nv) {
        if (nk < 16) {
            S[nsl].topA[1 + nk] = vn;
            if (nk < 8) S[nsl].topN[nk] = vn;
        } else {
            S[nsl].leftA[1 + nk - 16] = vn;
            if (nk < 24) S[nsl].leftN[nk - 16] = vn;
        }
    }
    if (t < kRdoSlots) {
        S[t].valid = tv;
        if (tv) {
            const int x = tbx * 8, y = tby * 8;
            S[t].topA[0] = vtl;
            S[t].leftA[0] = vtl;
            S[t].ntA = 1 + (y == 0 ? 16 : min(16, w - x));
            S[t].nlA = 1 + (x == 0 ? 16 : min(16, h - y));
        }
        S[t].wide = 0;
        best[t] = 0xFFFFFFFFu;
    }
    __syncthreads();
    for (int e = t; e < kRdoSlots * 64; e += 256)
        if (S[e / 64].valid) rdo8_block_prep(S[e / 64], e % 64);
    __syncthreads();
    {   // a wide block in the group: leave the group to the fallback launch (k_intra_rdo8<.., 2>)
        bool any_wide = false;
#pragma unroll
        for (int k = 0; k < kRdoSlots; ++k) any_wide |= S[k].valid && S[k].wide;
        if (any_wide) {
            if (t < kRdoSlots && S[t].valid) modes[b0 + t] = 0xFF;
            return;   // uniform over the workgroup
        }
    }
    // ---- A. the angular reference pairs of every (block, mode) ----
    {
        const int slot = t / kModes, mode = t - slot * kModes;
        if (slot < kRdoSlots && S[slot].valid && mode >= 2) rdo8_build_refs<REF16>(S[slot], mode, refs + t * RS);
    }
    __syncthreads();
    // ---- B. the 245 chains, 8 TUs a call ----
    const ChainQ rq = make_chainq(qp, dq_scale, dq_per);
    constexpr int kTus = kRdoSlots * kModes, TPC = 4 * NMS;   // TUs per call
    for (int c0 = TPC * wv; c0 < kTus; c0 += 4 * TPC) {
        rdo8_mma_call<false, NMS, REF16>(S, refs, RS, rq, [&](int k, int& sl, int& md) {
            const int e = c0 + k;
            sl = e < kTus ? e / kModes : -1;
            md = e - (sl < 0 ? 0 : sl) * kModes;
            if (sl >= 0 && !S[sl].valid) sl = -1;
        }, best, b0, bw, pitch, lvl, recon, modes);
    }
    __syncthreads();
    // ---- C. the winners again, with their outputs; the group's SSE once ----
    if (wv == 0) {
        rdo8_mma_call<true, 2, REF16>(S, refs, RS, rq, [&](int k, int& sl, int& md) {
            sl = k < kRdoSlots && S[k].valid ? k : -1;
            md = (int)(best[k < kRdoSlots ? k : 0] & 63u);
        }, best, b0, bw, pitch, lvl, recon, modes);
    } else if (wv == 1 && sse_out) {
        unsigned long long s = 0;
        if (t - 64 < kRdoSlots && S[t - 64].valid) s = best[t - 64] >> 6;
        s = grp_sum<64>(s);
        if (t == 64 && s) atomicAdd(sse_out, s);
    }
}

#endif  // NH_AB

// ===========================================================================
// Config 3, closed loop: blocks in raster order, neighbours
// from the reconstruction.  Wavefront schedule: one wave per block row; rows
// are claimed by an atomic ticket (plane-major, top to bottom), so a wave only
// ever waits for a row claimed earlier by a running wave (forward progress).
// Before block bx of row r the wave waits until row r-1 has finished blocks
// 0..bx+1 (the top and top-right references).
// Cross-wave data: the only samples another row reads are block bottom rows,
// kept in a per-plane line buffer (workspace) that is written and read with
// system-scope relaxed atomics (write-through stores / coherent loads, no L2
// writeback or invalidate -- the per-XCD L2s are not coherent, and agent-scope
// release/acquire would flush/invalidate the whole L2 every block).  The
// progress counter is stored after s_waitcnt vmcnt(0) has retired the line
// stores.  One line per plane suffices: row r+1 overwrites row r's entries
// line[x0..x0+7] (block bx) only once row r has finished block bx+1, and row
// r's later reads (block bx+2 on) start at x0+15; the top-left sample is
// carried from the previous block's top read because the row has already
// overwritten that entry itself.  A wait longer than kSpinLimit polls sets a status
// error and the launch drains instead of hanging.
// ===========================================================================
struct ClosedSet {
    int64_t base, plane_stride, group_stride;
    int32_t w, h, pitch, ppg;
    int32_t bw, bh, row0, plane0;   // first global row / plane of this set
    int64_t mode0;                  // first mode-map entry of this set
    int64_t line0;                  // first line-buffer word of this set
    int32_t lw;                     // line-buffer words per plane
    int32_t np;                     // planes in this set
};
#ifndef NH_CLOSED_PRIO
#define NH_CLOSED_PRIO 1
#endif
struct ClosedArgs {
    const int16_t* src;
    int32_t* lvl;
    int16_t* rec;
    uint8_t* modes;
    int64_t* sse;                   // per plane (accumulated)
    int32_t* work;                  // [0] ticket, [1] status, [2 + row] blocks done, then line buffers
    ClosedSet set[NH_MAX_PLANE_SETS];
    int32_t nsets, total_rows;
    int64_t lines0;                 // word offset of the line buffers in work
    int64_t lines_total;            // line-buffer words
    QuantParams qp;
    int32_t dq_scale, dq_per;
    int32_t order;                  // tagged form: 0 plane-major tickets, 1 row-major across planes
    int32_t max_bh;                 // largest block-row count of any set
    int32_t probe;                  // A/B build only (NH_CLOSED_PROBE=1): skip the chain (wrong outputs); 0 otherwise
    int32_t prio_set;               // the set with the longest wavefront (bw + 2 bh block steps): its rows issue first
};
// The tagged closed-loop kernel's forms: both chains per block (0), the packed
// chain only, for streams whose every source sample is 8-bit (1), both chains
// for the other streams (2).  Forms 1 / 2 read the stream's wide flag
// (work[2 + total_rows], set by k_closed_any_wide) and return at once unless it
// names them; the packed-only form needs fewer registers.
enum { kClosedBoth = 0, kClosedNarrow = 1, kClosedWide = 2 };
constexpr int kSpinLimit = 1 << 20;   // ~1 s of polling; a legitimate wait is a few block steps

__device__ __forceinline__ int ld_sys(const int32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(int32_t* p, int v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint64_t ld_sys64(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys64(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}


// Tagged-line form (default): the line buffer holds 64-bit words
// (tag << 32 | int16 pair), written with one single-copy-atomic coherent store
// per word, tag = producing block row + 1.  A row polls the 8 words of the top
// and top-right blocks directly until their tags name the row above, so the
// wait and the reference read are ONE coherent round trip per block (the
// progress-counter form needs two: poll the counter, then read the line), and
// no vmcnt(0) orders a progress store behind the line stores.  WAR safety is
// the progress form's argument (row r+1 overwrites block bx's words only after
// reading them for blocks bx-1 and bx; the top-left sample is carried).  Words
// past the last full block are never written: they read as 0 without a wait.
// The winner hands its recon / levels to the wave through LDS and the 64
// lanes store one sample each (2 store instructions instead of 128
// single-lane ones on the row's critical path).
// Ticket -> (set, plane, block row).  order 0: plane-major (every row of
// plane 0, then plane 1, ...).  order 1: row-major across planes (block row 0
// of every plane of every set, then block row 1, ...): a row waits for the
// row above from step 2*by of its plane on, so claiming rows in by order keeps
// the 1,024 resident waves on rows that can start (plane-major parks the
// lower rows of the first planes on their wavefront lag while later planes
// wait for a slot): 874 -> 590 block steps for 8 1080p YUV420 frames in a
// slot simulation.  Both orders claim row by-1 of a plane before row by, so a
// wave only waits on a running or finished row.
__device__ __forceinline__ void closed_ticket(const ClosedArgs& a, int t, int& si, int& pl, int& by) {
    if (a.order == 0) {
        si = 0;
        for (int k = 1; k < a.nsets; ++k)
            if (t >= a.set[k].row0) si = k;
        const ClosedSet& S = a.set[si];
        const int local = t - S.row0;
        pl = local / S.bh;
        by = local - pl * S.bh;
        return;
    }
    // prefix(b) = rows with block row < b = sum_k np_k * min(b, bh_k); largest b with prefix(b) <= t
    int lo = 0, hi = a.max_bh - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        int64_t pre = 0;
        for (int k = 0; k < a.nsets; ++k) pre += (int64_t)a.set[k].np * min(mid, a.set[k].bh);
        if (pre <= t) lo = mid; else hi = mid - 1;
    }
    by = lo;
    int64_t r = t;
    for (int k = 0; k < a.nsets; ++k) r -= (int64_t)a.set[k].np * min(by, a.set[k].bh);
    si = 0;
    for (int k = 0; k < a.nsets; ++k) {
        if (by >= a.set[k].bh || a.set[k].np == 0) continue;
        if (r < a.set[k].np) { si = k; break; }
        r -= a.set[k].np;
    }
    pl = (int)r;
}

template <int WAVES, int FORM = kClosedBoth>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WAVES))) k_intra_rdo8_closed_tag(ClosedArgs a) {
    if constexpr (FORM != kClosedBoth) {
        if ((__builtin_nontemporal_load(&a.work[2 + a.total_rows]) != 0) != (FORM == kClosedWide)) return;
    }
    __shared__ RdoSlotLds L;
    __shared__ uint32_t refs[64][kRefStride];
    __shared__ uint32_t outP[32], outL[32];   // the winner's recon / level pairs, row-major
    __shared__ int32_t topw[9];
    __shared__ int row_s, stall_s, win_s;
    const int lane = threadIdx.x;
    const ChainQ rq = make_chainq(a.qp, a.dq_scale, a.dq_per);
    uint64_t* lines = reinterpret_cast<uint64_t*>(a.work + a.lines0);
    for (;;) {
        if (lane == 0) {
            row_s = atomicAdd(&a.work[0], 1);
            stall_s = 0;
        }
        __syncthreads();
        const int row = row_s;
        if (row >= a.total_rows) break;
        int si, pl, by;
        closed_ticket(a, row, si, pl, by);
        if (NH_CLOSED_PRIO) {   // the critical (longest) wavefront's rows issue before the others' (s_setprio)
            if (si == a.prio_set) __builtin_amdgcn_s_setprio(2);
            else __builtin_amdgcn_s_setprio(0);
        }
        const ClosedSet& S = a.set[si];
        const int g = pl / S.ppg, c = pl - g * S.ppg;
        const int64_t off = S.base + (int64_t)g * S.group_stride + (int64_t)c * S.plane_stride;
        const int16_t* src = a.src + off;
        int16_t* rec = a.rec + off;
        int32_t* lvl = a.lvl + off;
        uint64_t* line = lines + S.line0 + (int64_t)pl * S.lw;
        const int y0 = by * 8, full_words = S.bw * 4;
        int16_t tl_next = 128;
        unsigned long long row_sse = 0;
        for (int bx = 0; bx < S.bw; ++bx) {
            const int x0 = bx * 8;
            const int16_t ov = src[(int64_t)(y0 + lane / 8) * S.pitch + x0 + (lane % 8)];
            if (by > 0) {
                // lanes 0..7: words x0/2 .. x0/2+7 (samples x0 .. x0+15) of the row above
                const int wi = x0 / 2 + lane;
                const bool need = lane < 8 && wi < full_words;
                uint32_t val = 0;
                int spins = 0;
                for (;;) {
                    bool ok = true;
                    if (need) {
                        const uint64_t v = ld_sys64(line + wi);
                        ok = (int)(v >> 32) == by;
                        val = (uint32_t)v;
                    }
                    if (__builtin_amdgcn_read_exec() == __ballot(ok)) break;   // every needed word is there
                    __builtin_amdgcn_s_sleep(1);
                    ++spins;
                    if (spins > kSpinLimit || ((spins & 1023) == 0 && ld_sys(&a.work[1]))) {
                        if (lane == 0) atomicMax(&a.work[1], 1);
                        stall_s = 1;
                        break;
                    }
                }
                if (lane < 8) topw[1 + lane] = (int32_t)val;
            }
            __syncthreads();
            if (stall_s) break;
            {
                const int k = lane;
                L.orig[k] = ov;
                if (k < 16) {
                    int16_t v = 128;
                    if (y0 > 0 && x0 + k < S.w) v = (int16_t)(topw[1 + (k >> 1)] >> ((k & 1) * 16));
                    L.topA[1 + k] = v;
                    if (k < 8) L.topN[k] = v;
                } else if (k < 24) {
                    const int kk = k - 16;
                    const int16_t v = x0 == 0 ? (int16_t)128 : (int16_t)(outP[kk * 4 + 3] >> 16);
                    L.leftA[1 + kk] = v;
                    L.leftN[kk] = v;
                } else if (k == 24) {
                    const int16_t tl = (y0 == 0 || x0 == 0) ? (int16_t)128 : tl_next;
                    L.topA[0] = tl;
                    L.leftA[0] = tl;
                    L.ntA = 1 + (y0 == 0 ? 16 : min(16, S.w - x0));
                    L.nlA = 1 + 8;
                    L.wide = 0;
                }
            }
            __syncthreads();
            rdo8_block_prep(L, lane);
            __syncthreads();
            tl_next = L.topA[8];
            uint32_t P[32], Lv[32];
            unsigned long long key = ULLONG_MAX;
#if NH_AB   // timing probe of the A/B build only: skip the chain (wrong outputs)
            if (a.probe) {
#pragma unroll
                for (int q = 0; q < 32; ++q) P[q] = Lv[q] = (uint32_t)L.orig[q];
                if (lane < kModes) key = lane;
            } else
#endif
            if (lane < kModes) {
                key = (rdo8_chain<FORM == kClosedNarrow>(L, lane, refs[lane], rq, P, Lv) << 6) | lane;
            }
            const unsigned long long best = grp_min<64>(key);   // DPP / swizzle / lane reads (nh_packed.hpp)
            if (key == best) {
                // publish the bottom row first (the next row polls these words)
                const uint64_t tag = (uint64_t)(uint32_t)(by + 1) << 32;
#pragma unroll
                for (int q = 0; q < 4; ++q) st_sys64(line + x0 / 2 + q, tag | P[28 + q]);
#pragma unroll
                for (int q = 0; q < 32; ++q) {
                    outP[q] = P[q];
                    outL[q] = Lv[q];
                }
                win_s = lane;
                row_sse += best >> 6;
            }
            __syncthreads();
            {   // every lane stores one sample of the winner's block
                const int i = lane >> 3, j = lane & 7;
                const int64_t e = (int64_t)(y0 + i) * S.pitch + x0 + j;
                rec[e] = (int16_t)(outP[i * 4 + j / 2] >> (16 * (j & 1)));
                lvl[e] = (int32_t)(int16_t)(outL[i * 4 + j / 2] >> (16 * (j & 1)));
                if (lane == 0) a.modes[S.mode0 + (int64_t)pl * S.bw * S.bh + (int64_t)by * S.bw + bx] = (uint8_t)win_s;
            }
        }
        row_sse = grp_sum<64>(row_sse);
        if (lane == 0 && row_sse) atomicAdd((unsigned long long*)&a.sse[S.plane0 + pl], row_sse);
        __syncthreads();
        if (stall_s) break;
    }
}


// Samples outside full 8x8 blocks read as 0 (Frame.zeros) by the closed loop.
__global__ void k_zero_partial(int16_t* rec, ClosedSet S, int nplanes) {
    const int p = blockIdx.y;
    if (p >= nplanes) return;
    const int g = p / S.ppg, c = p - g * S.ppg;
    int16_t* r = rec + S.base + (int64_t)g * S.group_stride + (int64_t)c * S.plane_stride;
    const int fw = S.bw * 8, fh = S.bh * 8;
    for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < (int64_t)S.w * S.h; i += (int64_t)gridDim.x * 256) {
        const int y = (int)(i / S.w), x = (int)(i - (int64_t)y * S.w);
        if (x >= fw || y >= fh) r[(int64_t)y * S.pitch + x] = 0;
    }
}

// ===========================================================================
// Config 4: mixed 4/8/16/32 TU pipeline.
//   tu_leaf      : the seeded quadtree's leaf containing a sample (<= 3 hashes);
//   k_tu_process : one launch per TU size over the N-aligned positions of the
//                  band, keeping the positions whose leaf is NxN; N threads per
//                  TU (thread t = column t, then row t), LDS tiles;
//                  DC-vs-planar open-loop choice (__main__.py:165-178), then the
//                  full residual -> transform -> quant -> dequant -> inverse ->
//                  recon chain with exact int32/int64 arithmetic.
// ===========================================================================
// MODE kAll (config 5): TU idx is the idx-th full NxN block of the plane in
// raster order (grid_bw blocks per row, grid_n blocks), no TU map.
// MODE kTree (config 4): the workgroup's candidates are N-aligned positions of
// CTU rows [row0, row1); a position is a TU iff its quadtree leaf is exactly
// NxN (tu_leaf) -- no global lists or atomics, deterministic; the TU writes
// its map.
// Multiplies are 24-bit (v_mad_i32_i24): exact for the whole chain because the
// residual is int16 (forward operands < 2^21), dequantized coefficients are
// ~|c|*2^20/2^(17+log2N) < 2^19, and inverse pass-2 operands are a >> S of an
// int32 sum bounded by 2^27 -> < 2^21.
// Candidates per workgroup: kTree walks every N-aligned position but only
// ~1/2 (N = 32) to ~1/6 (N = 4, 8) of them are TUs of that size, so a
// workgroup tests R * G positions, compacts the TUs into an LDS list (wave
// ballots, no global atomics) and runs the chain over the list in rounds of G.

template <int N, int MODE>
constexpr int tu_cands_per_wg() { return (256 / N) * (MODE == 1 ? (N == 32 ? 2 : 4) : 1); }

template <int N, bool DST, int MODE>
__global__ void __launch_bounds__(256) k_tu_process(const int16_t* __restrict__ src, int w, int h, int pitch,
                                                    QuantParams qp, int dq_scale, int dq_per, int32_t* lvl,
                                                    int16_t* recon, uint8_t* tu_log2, int grid_bw, int grid_n,
                                                    TreeArgs ta) {
    constexpr int G = 256 / N;            // TUs per round
    constexpr int P = N + 1;              // padded LDS row
    constexpr int S = Log2<N>::v + 5;
    constexpr int K = tu_cands_per_wg<N, MODE>();
    {   // this workgroup's plane of the batch
        const int pz = blockIdx.y, gz = pz / ta.ppg, cz = pz - gz * ta.ppg;
        const int64_t poff = (int64_t)gz * ta.group_stride + (int64_t)cz * ta.plane_stride;
        src += poff;
        lvl += poff;
        recon += poff;
        if (tu_log2) tu_log2 += (int64_t)pz * ta.tu_plane;
        ta.plane_id += cz;
    }
    __shared__ int32_t tile[G][N][P];
    __shared__ int16_t orig[G][N][N];
    __shared__ int16_t topv[G][N], leftv[G][N];
    __shared__ long long e_dc[G][N], e_pl[G][N];
    __shared__ uint32_t list[MODE == kTree ? K : 1];
    __shared__ int wave_cnt[4], list_n;
    const int g = threadIdx.x / N, t = threadIdx.x % N;
    const ChainQ cq = make_chainq(qp, dq_scale, dq_per);
    // recon rows as vectors when every row start is 16-B aligned (x0 is a multiple of N)
    const bool rec_vec = ((uintptr_t)recon & 15) == 0 && (pitch & 7) == 0;
    int ntu;
    if constexpr (MODE == kTree) {
        // phase 1: which candidate positions are TUs of size N (tu_leaf), compacted
        const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
        if (threadIdx.x == 0) list_n = 0;
        __syncthreads();
        for (int k0 = 0; k0 < K; k0 += 256) {
            const int k = k0 + threadIdx.x;
            const uint32_t c = blockIdx.x * (uint32_t)K + k;
            bool f = false;
            if (k < K && c < (uint32_t)grid_n) {
                const int cx = (c % grid_bw) * N, cy = (c / grid_bw) * N + ta.y_base;
                f = (cx + N <= w) && (cy + N <= h) && tu_leaf(w, h, ta.ctb, ta.plane_id, ta.seed, cx, cy) == N;
            }
            const uint64_t m = __ballot(f);
            if (lane == 0) wave_cnt[wv] = __popcll(m);
            __syncthreads();
            int base = list_n;
            for (int q = 0; q < wv; ++q) base += wave_cnt[q];
            if (f) list[base + __popcll(m & ((1ull << lane) - 1))] = c;
            __syncthreads();
            if (threadIdx.x == 0) list_n += wave_cnt[0] + wave_cnt[1] + wave_cnt[2] + wave_cnt[3];
            __syncthreads();
        }
        ntu = list_n;
    } else {
        ntu = grid_n - (int)(blockIdx.x * G);
        ntu = ntu < G ? ntu : G;
    }
    for (int r0 = 0; r0 < ntu; r0 += G) {   // rounds of G TUs (uniform over the workgroup)
    bool active = r0 + g < ntu;
    int x0 = 0, y0 = 0;
    if (active) {
        const uint32_t idx = MODE == kTree ? list[r0 + g] : blockIdx.x * G + g;
        x0 = (idx % grid_bw) * N;
        y0 = (idx / grid_bw) * N + (MODE == kTree ? ta.y_base : 0);
    }
    if (active) {
        // neighbours (block.py:38-50): count N, 128 outside the plane (full TUs: no truncation).
        // All N + 2 loads are issued before the first LDS write (one memory
        // latency per round, not one per sample).
        int16_t ov[N];
#pragma unroll
        for (int i = 0; i < N; ++i) ov[i] = src[(int64_t)(y0 + i) * pitch + x0 + t];
        const int16_t tv = y0 == 0 ? (int16_t)128 : src[(int64_t)(y0 - 1) * pitch + x0 + t];
        const int16_t lv = x0 == 0 ? (int16_t)128 : src[(int64_t)(y0 + t) * pitch + x0 - 1];
        topv[g][t] = tv;
        leftv[g][t] = lv;
#pragma unroll
        for (int i = 0; i < N; ++i) orig[g][i][t] = ov[i];
    }
    __syncthreads();
    // DC (intra.py:46-62) and planar (intra.py:81-113) for column t
    int32_t dc = 0, tr = 0, bl = 0;
    if (active) {
        long long s = 0;
        for (int k = 0; k < N; ++k) s += topv[g][k] + leftv[g][k];
        dc = (int32_t)((s + N) >> (Log2<N>::v + 1));   // floor((s+N)/(2N)), 2N a power of two
        tr = topv[g][N - 1];
        bl = leftv[g][N - 1];
        long long ed = 0, ep = 0;
        for (int y = 0; y < N; ++y) {
            const int32_t o = orig[g][y][t];
            const int32_t pl = ((N - 1 - t) * leftv[g][y] + (t + 1) * tr + (N - 1 - y) * topv[g][t] + (y + 1) * bl + N) >>
                               (Log2<N>::v + 1);
            const int32_t d1 = wrap16(o - dc), d2 = wrap16(o - pl);
            ed += (long long)d1 * d1;
            ep += (long long)d2 * d2;
        }
        e_dc[g][t] = ed;
        e_pl[g][t] = ep;
    }
    __syncthreads();
    bool use_dc = true;
    if (active) {
        long long ed = 0, ep = 0;
        for (int k = 0; k < N; ++k) { ed += e_dc[g][k]; ep += e_pl[g][k]; }
        use_dc = ed <= ep;                               // __main__.py:173: DC wins ties
    }
    auto pred_at = [&](int y, int x) -> int32_t {
        if (use_dc) return dc;
        return ((N - 1 - x) * leftv[g][y] + (x + 1) * tr + (N - 1 - y) * topv[g][x] + (y + 1) * bl + N) >> (Log2<N>::v + 1);
    };
    uint32_t v[N], r[N];
    // forward pass 1 on column t of the residual
    if (active) {
#pragma unroll
        for (int k = 0; k < N; ++k) v[k] = (uint32_t)(int32_t)wrap16((int32_t)orig[g][k][t] - pred_at(k, t));
        fwd1d<N, DST, Mul24>(v, r);
#pragma unroll
        for (int i = 0; i < N; ++i) tile[g][i][t] = rshift_round<S>(r[i]);
    }
    __syncthreads();
    // forward pass 2 on row t, quant, dequant
    if (active) {
#pragma unroll
        for (int k = 0; k < N; ++k) v[k] = (uint32_t)tile[g][t][k];
        fwd1d<N, DST, Mul24>(v, r);
        int32_t* lrow = lvl + (int64_t)(y0 + t) * pitch + x0;
#pragma unroll
        for (int j = 0; j < N; ++j) {
            const int32_t l = quant_s(rshift_round<S>(r[j]), cq.qs, cq.h_v, cq.hneg_v);
            lrow[j] = l;
            v[j] = (uint32_t)dequant_s(l, cq);
        }
    }
    __syncthreads();
    if (active) {
#pragma unroll
        for (int j = 0; j < N; ++j) tile[g][t][j] = (int32_t)v[j];
    }
    __syncthreads();
    // inverse pass 1 on column t
    if (active) {
#pragma unroll
        for (int k = 0; k < N; ++k) v[k] = (uint32_t)tile[g][k][t];
        inv1d<N, DST, Mul24>(v, r);
    }
    __syncthreads();
    if (active) {
#pragma unroll
        for (int i = 0; i < N; ++i) tile[g][i][t] = rshift_round<S>(r[i]);
    }
    __syncthreads();
    // inverse pass 2 on row t, reconstruct + clip
    if (active) {
#pragma unroll
        for (int k = 0; k < N; ++k) v[k] = (uint32_t)tile[g][t][k];
        inv1d<N, DST, Mul24>(v, r);
        int16_t* rrow = recon + (int64_t)(y0 + t) * pitch + x0;
        uint32_t rcp[N / 2];
#pragma unroll
        for (int j = 0; j < N; j += 2) {
            int32_t rc2[2];
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int32_t rr = wrap16(rshift_round<S>(r[j + q]));
                const int32_t rc = wrap16(pred_at(t, j + q) + rr);
                rc2[q] = rc < 0 ? 0 : (rc > 255 ? 255 : rc);
            }
            rcp[j / 2] = (uint32_t)rc2[0] | ((uint32_t)rc2[1] << 16);
        }
        if (rec_vec) {   // one row = N int16: 8..64 B vector stores
            constexpr int A = 2 * N < 16 ? 2 * N : 16;
            __builtin_memcpy(__builtin_assume_aligned(rrow, A), rcp, 2 * N);
        } else {
#pragma unroll
            for (int j = 0; j < N; ++j) rrow[j] = (int16_t)(rcp[j / 2] >> (16 * (j & 1)));
        }
        if (MODE == kTree && t < N / 4) {
            const int w4 = w / 4;
            for (int j = 0; j < N / 4; ++j) tu_log2[(int64_t)(y0 / 4 + t) * w4 + x0 / 4 + j] = (uint8_t)Log2<N>::v;
        }
    }
    __syncthreads();   // the next round reuses the LDS tiles
    }
}

static void qp_split(int qp, int* per, int* rem) {
    qp = qp < 0 ? 0 : (qp > 51 ? 51 : qp);
    *per = qp / 6;
    *rem = qp % 6;
}
static QuantParams qparams(int qp, int log2n, bool intra) {
    int per, rem;
    qp_split(qp, &per, &rem);
    QuantParams q;
    q.shift = 14 + per + log2n;
    q.mf = quant_scale(rem);
    q.off = (uint32_t)(intra ? (1ull << q.shift) / 3 : (1ull << q.shift) / 6);
    return q;
}


// ===========================================================================
// Config 4 in closed loop: CTUs in raster order, TUs in
// quadtree z-order, each TU's top / left neighbours (N samples, BlockView
// rules) from the reconstruction built so far.  A TU only reads the row above
// and the column to its left, so CTU (cx, cy) depends on (cx-1, cy) and
// (cx, cy-1) only.  One wave per CTU row (tickets row-major across planes, so
// a wave only waits on a CTU row claimed before it); the CTU being coded lives
// in LDS with its top row and left column (rc[1 + y][1 + x]), so every
// neighbour read is an LDS read.  The only cross-wave data is each CTU's
// bottom row, published as tagged 64-bit line words (tag = CTU row + 1, as the
// config-3 closed loop) that the next CTU row polls before the CTU.  TUs are
// found by walking the CTU's 4x4 units in Morton order: a unit is a TU origin
// iff tu_leaf says its leaf starts there (Morton order of leaf origins is the
// quadtree's z-order).  A TU runs on lanes 0..N-1 (column t, then row t) with
// the chain of k_tu_process: same arithmetic, same results.
// ===========================================================================
struct Closed4Args {
    const int16_t* src;
    int32_t* lvl;
    int16_t* rec;
    uint8_t* tu;
    int32_t* work;          // [0] ticket, [1] status; 64-bit line words from int32 word lines0
    int64_t lines0;
    int64_t group_stride, plane_stride, tu_plane;
    int32_t w, h, pitch, ctb, plane_id, ppg, nplanes, crows, ccols, lw, is_luma;
    uint32_t seed;
    QuantParams q[4];       // log2 N = 2..5
    int32_t dqs, dq_per;
    const uint8_t* plan;    // k_tu_closed_pair: per-(plane of the group, CTU) TU schedules (k_closed4_plan)
    int32_t probe;          // A/B timing probes (k_tu_closed_pair; wrong outputs): 1 no wait on the row
                            // above, 2 no chains, 4 no rounds, 8 no recon-image clear, 16 no quadtree
                            // hashes, 32 no source loads in the chains, 64 no level / recon / TU-map
                            // stores in the chains (0 in the product)
    int32_t mfma32;         // k_tu_closed_pair: 32x32 TUs on the f16 matrix cores (closed_chain32_tf); set
                            // for luma when the level / recon rows allow 16-B stores
    int32_t srctile;        // k_tu_closed_pair: each CTU's source samples land in an LDS tile by LDS-DMA
                            // under the wait on the row above; the chains read them there
    int32_t rec_ctu;        // k_tu_closed_pair: a whole CTU's packed-chain recon leaves from the LDS
                            // reconstruction at the CTU's end, as 64-B row pieces (the rows 8-B aligned)
    uint64_t* stamps;       // A/B build only (NH_CLOSED4_STAMPS): per (ticket, CTU) shader-clock stamps
};
__constant__ BasisHC c_basis_hc_cl;   // the f16 DCT32 bases of closed_chain32_tf (copied to LDS per workgroup)

// cnt TUs of size N at once: lane l codes column / row t = l % N of TU j = l / N
// (local origin (slx[j], sly[j]) in the CTU); reductions over a TU's N lanes are
// xor-shuffles inside the aligned N-lane group.  TUs of one batch are
// independent (none reads another's samples), and the CTU-sized LDS tile holds
// every TU at its own position.
template <int N, bool DST>
__device__ __forceinline__ void tu_closed_batch(const Closed4Args& a, const int16_t* src, int32_t* lvl, int16_t* rec,
                                                uint8_t* tu, int x0c, int y0c, int cnt, const int* slx, const int* sly,
                                                int16_t (*rc)[33], int32_t (*tile)[33], const ChainQ& cq) {
    constexpr int S = Log2<N>::v + 5;
    const int j = threadIdx.x / N, t = threadIdx.x % N;
    const bool on = j < cnt;
    const int lx = on ? slx[j] : 0, ly = on ? sly[j] : 0, x = x0c + lx, y = y0c + ly;
    int32_t o[N];
    int32_t topt = 0, leftt = 0;
    if (on) {
#pragma unroll
        for (int i = 0; i < N; ++i) o[i] = src[(int64_t)(y + i) * a.pitch + x + t];
        topt = rc[ly][lx + 1 + t];       // sample (y - 1, x + t)
        leftt = rc[ly + 1 + t][lx];      // sample (y + t, x - 1)
    }
    // DC (intra.py:46-62): sum over the TU's N lanes
    int32_t sum = topt + leftt;
    sum = grp_sum<N>(sum);
    const int32_t dc = (sum + N) >> (Log2<N>::v + 1);
    const int32_t tr = on ? rc[ly][lx + N] : 0, bl = on ? rc[ly + N][lx] : 0;   // top[-1], left[-1]
    auto planar = [&](int yy, int xx) -> int32_t {
        return ((N - 1 - xx) * (int32_t)rc[ly + 1 + yy][lx] + (xx + 1) * tr + (N - 1 - yy) * (int32_t)rc[ly][lx + 1 + xx] +
                (yy + 1) * bl + N) >> (Log2<N>::v + 1);
    };
    long long ed = 0, ep = 0;
    if (on) {
#pragma unroll
        for (int i = 0; i < N; ++i) {
            const int32_t d1 = wrap16(o[i] - dc), d2 = wrap16(o[i] - planar(i, t));
            ed += (long long)d1 * d1;
            ep += (long long)d2 * d2;
        }
    }
    ed = grp_sum<N>(ed);
    ep = grp_sum<N>(ep);
    const bool use_dc = ed <= ep;                        // __main__.py:173: DC wins ties
    auto pred_at = [&](int yy, int xx) -> int32_t { return use_dc ? dc : planar(yy, xx); };
    uint32_t v[N], r[N];
    if (on) {                                            // forward pass 1: column t
#pragma unroll
        for (int k = 0; k < N; ++k) v[k] = (uint32_t)wrap16(o[k] - pred_at(k, t));
        fwd1d<N, DST, Mul24>(v, r);
#pragma unroll
        for (int i = 0; i < N; ++i) tile[ly + i][lx + t] = rshift_round<S>(r[i]);
    }
    __syncthreads();
    if (on) {                                            // forward pass 2: row t, quant, dequant
#pragma unroll
        for (int k = 0; k < N; ++k) v[k] = (uint32_t)tile[ly + t][lx + k];
        fwd1d<N, DST, Mul24>(v, r);
        int32_t* lrow = lvl + (int64_t)(y + t) * a.pitch + x;
#pragma unroll
        for (int jj = 0; jj < N; ++jj) {
            const int32_t l = quant_s(rshift_round<S>(r[jj]), cq.qs, cq.h_v, cq.hneg_v);
            lrow[jj] = l;
            v[jj] = (uint32_t)dequant_s(l, cq);
        }
    }
    __syncthreads();
    if (on) {
#pragma unroll
        for (int jj = 0; jj < N; ++jj) tile[ly + t][lx + jj] = (int32_t)v[jj];
    }
    __syncthreads();
    if (on) {                                            // inverse pass 1: column t
#pragma unroll
        for (int k = 0; k < N; ++k) v[k] = (uint32_t)tile[ly + k][lx + t];
        inv1d<N, DST, Mul24>(v, r);
    }
    __syncthreads();
    if (on) {
#pragma unroll
        for (int i = 0; i < N; ++i) tile[ly + i][lx + t] = rshift_round<S>(r[i]);
    }
    __syncthreads();
    if (on) {                                            // inverse pass 2: row t, reconstruct, clip
#pragma unroll
        for (int k = 0; k < N; ++k) v[k] = (uint32_t)tile[ly + t][lx + k];
        inv1d<N, DST, Mul24>(v, r);
        int16_t* rrow = rec + (int64_t)(y + t) * a.pitch + x;
#pragma unroll
        for (int jj = 0; jj < N; ++jj) {
            const int32_t rr = wrap16(rshift_round<S>(r[jj]));
            int32_t q = wrap16(pred_at(t, jj) + rr);
            q = q < 0 ? 0 : (q > 255 ? 255 : q);
            rrow[jj] = (int16_t)q;
            // the TU's own samples: no TU of this batch reads them (planar reads the row
            // above and the column left of each TU, coded in earlier rounds)
            rc[ly + 1 + t][lx + 1 + jj] = (int16_t)q;
        }
        if (t < N / 4) {
            const int w4 = a.w / 4;
            for (int jj = 0; jj < N / 4; ++jj) tu[(int64_t)(y / 4 + t) * w4 + x / 4 + jj] = (uint8_t)Log2<N>::v;
        }
    }
    __syncthreads();
}

// tu_closed_batch for a stream whose every source sample is 8-bit (the
// reconstruction is clipped to [0, 255], so neighbours are too): the packed
// 16-bit chain of DESIGN.md §4.4 (nh_packed.hpp; bounds: tools/packed_bounds.py)
// with an int16 view of the tile (rows of TP = 34: pair reads conflict-free).
// Same results as tu_closed_batch on such input.
__device__ __forceinline__ int opaque_lane64() {
    int l = threadIdx.x & 63;
#ifndef NH_PLAIN_LANE64   // A/B builds: -DNH_PLAIN_LANE64 lets the compiler hoist lane-derived values
    asm volatile("" : "+v"(l));
#endif
    return l;
}
template <int N, bool DST>
__device__ __forceinline__ void tu_closed_batch_pk(const Closed4Args& a, const int16_t* src, int32_t* lvl, int16_t* rec,
                                                   uint8_t* tu, int x0c, int y0c, int cnt, const int* slx,
                                                   const int* sly, int16_t (*rc)[33], int16_t* t16, const ChainQ& cq) {
    constexpr int L2 = Log2<N>::v, S = L2 + 5, H = N / 2, TP = 34;
    constexpr int32_t BIAS = 1 << (S - 1);
    const int lane = opaque_lane64(), j = lane / N, t = lane % N;
    const bool on = j < cnt;
    const int lx = on ? slx[j] : slx[0], ly = on ? sly[j] : sly[0], x = x0c + lx, y = y0c + ly;
    int16_t* tl = t16 + ly * TP + lx;   // tl[line * TP + slot]
    const int32_t topt = rc[ly][lx + 1 + t], leftt = rc[ly + 1 + t][lx];
    const int32_t tr = rc[ly][lx + N], bl = rc[ly + N][lx];   // top[-1], left[-1] (__main__.py:168)
    int32_t sum = topt + leftt;                                // DC (intra.py:46-62)
    sum = grp_sum<N>(sum);
    const int32_t dc = (sum + N) >> (L2 + 1);
    const pk16 dc2 = pk_splat(dc);
    pk16 o2[H];
    pku16 pl2[H];
    {
        const int32_t b = (t + 1) * tr + (N - 1) * topt + bl + N, st = bl - topt;
        pku16 bs = {(unsigned short)b, (unsigned short)(b + st)};
        const pku16 st2 = {(unsigned short)(2 * st), (unsigned short)(2 * st)};
        const pku16 wl = {(unsigned short)(N - 1 - t), (unsigned short)(N - 1 - t)};
        const pku16 sh = {(unsigned short)(L2 + 1), (unsigned short)(L2 + 1)};
        const int16_t* sp = src + (int64_t)y * a.pitch + x + t;
#pragma unroll
        for (int m = 0; m < H; ++m) {
            o2[m] = pk_pair(sp[(2 * m) * a.pitch], sp[(2 * m + 1) * a.pitch]);
            const pku16 lf = {(unsigned short)rc[ly + 1 + 2 * m][lx], (unsigned short)rc[ly + 2 + 2 * m][lx]};
            pl2[m] = (lf * wl + bs) >> sh;
            bs += st2;
        }
    }
    int32_t ed = 0, ep = 0;
#pragma unroll
    for (int m = 0; m < H; ++m) {
        const pk16 d0 = o2[m] - dc2, d1 = o2[m] - __builtin_bit_cast(pk16, pl2[m]);
        ed = __builtin_amdgcn_sdot2(d0, d0, ed, false);
        ep = __builtin_amdgcn_sdot2(d1, d1, ep, false);
    }
    ed = grp_sum<N>(ed);
    ep = grp_sum<N>(ep);
    const bool use_dc = ed <= ep;   // __main__.py:173: DC wins ties
    pk16 r2[H];
#pragma unroll
    for (int m = 0; m < H; ++m) r2[m] = o2[m] - (use_dc ? dc2 : __builtin_bit_cast(pk16, pl2[m]));
    int32_t yv[N];
    fwd1d_pk<N, DST>(r2, yv, BIAS);   // forward pass 1 (transform.py:179-185): column t -> line i, slot t
    if (on) {
#pragma unroll
        for (int i = 0; i < N; ++i) tl[i * TP + t] = (int16_t)(yv[i] >> S);
    }
    __syncthreads();
    const int st = inv_slot<N, DST>(t);
    {
        pk16 P[H];   // forward pass 2 (transform.py:188-194): row t
#pragma unroll
        for (int m = 0; m < H; ++m) P[m] = pk_pair(tl[t * TP + 2 * m], tl[t * TP + 2 * m + 1]);
        fwd1d_pk<N, DST>(P, yv, BIAS);
    }
    __syncthreads();
    if (on) {   // quantize_block -> levels; dequantize_block -> line k, slot inv_slot(t)
        int32_t* lrow = lvl + (int64_t)(y + t) * a.pitch + x;
#pragma unroll
        for (int k = 0; k < N; ++k) {
            const int32_t l = quant_s(yv[k] >> S, cq.qs, cq.h_v, cq.hneg_v);
            lrow[k] = l;
            tl[k * TP + st] = (int16_t)dequant_s(l, cq);
        }
    }
    __syncthreads();
    int32_t xv[N];
    {
        pk16 Y[H];   // inverse pass 1 (transform.py:221-227): column t -> line i, slot inv_slot(t)
#pragma unroll
        for (int m = 0; m < H; ++m) Y[m] = pk_pair(tl[t * TP + 2 * m], tl[t * TP + 2 * m + 1]);
        inv1d_pk<N, DST>(Y, xv, BIAS);
    }
    __syncthreads();
    if (on) {
#pragma unroll
        for (int i = 0; i < N; ++i) tl[i * TP + st] = (int16_t)(xv[i] >> S);
    }
    __syncthreads();
    {
        pk16 Y[H];   // inverse pass 2 (transform.py:230-236): row t
#pragma unroll
        for (int m = 0; m < H; ++m) Y[m] = pk_pair(tl[t * TP + 2 * m], tl[t * TP + 2 * m + 1]);
        inv1d_pk<N, DST>(Y, xv, BIAS);
    }
    if (on) {   // reconstruct + clip (intra.py:70-78); planar in row layout
        const int32_t b = (N - 1) * leftt + tr + (t + 1) * bl + N, stv = tr - leftt;
        int16_t* rrow = rec + (int64_t)(y + t) * a.pitch + x;
#pragma unroll
        for (int k = 0; k < N; ++k) {
            const int32_t p = use_dc ? dc : ((N - 1 - t) * (int32_t)rc[ly][lx + 1 + k] + b + k * stv) >> (L2 + 1);
            int32_t q = p + (xv[k] >> S);
            q = q < 0 ? 0 : (q > 255 ? 255 : q);
            rrow[k] = (int16_t)q;
            // the TU's own samples: no TU of this batch reads them
            rc[ly + 1 + t][lx + 1 + k] = (int16_t)q;
        }
        if (t < N / 4) {
            const int w4 = a.w / 4;
            for (int jj = 0; jj < N / 4; ++jj) tu[(int64_t)(y / 4 + t) * w4 + x / 4 + jj] = (uint8_t)L2;
        }
    }
    __syncthreads();
}

// NARROW: the packed chain; the launch pairs it with the 32-bit form and the
// stream's wide flag (work[2], set by k_closed_any_wide -- or, after the pair
// kernel, by the pair kernel itself when a TU's source sample left [0, 255])
// makes exactly one of the two code the stream -- the other returns before
// taking a ticket.  The 32-bit form takes its tickets from work[3] and tags its
// line words kWideTag higher: it may run after the pair kernel has used both.
constexpr int kWideTag = 1 << 20;
template <int WAVES, bool NARROW = false>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WAVES))) k_tu_closed(Closed4Args a) {
    __shared__ int16_t rc[33][33];
    __shared__ int32_t tile[32][33];
    __shared__ int owner_of[64], done_of[64], slx[16], sly[16];
    __shared__ int row_s, stall_s;
    if ((__builtin_nontemporal_load(&a.work[2]) != 0) == NARROW) return;   // the other form codes this stream
    constexpr int TK = NARROW ? 0 : 3, TG = NARROW ? 0 : kWideTag;   // ticket word, line-word tag offset
    const int lane = threadIdx.x;
    const int ctb = a.ctb;
    ChainQ cq[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) cq[k] = make_chainq(a.q[k], a.dqs, a.dq_per);
    uint64_t* lines = reinterpret_cast<uint64_t*>(a.work + a.lines0);
    const int total = a.crows * a.nplanes;
    for (;;) {
        if (lane == 0) {
            row_s = atomicAdd(&a.work[TK], 1);
            stall_s = 0;
        }
        __syncthreads();
        const int tk = row_s;
        if (tk >= total) break;
        const int cy = tk / a.nplanes, pl = tk - cy * a.nplanes;   // row-major across planes
        const int g = pl / a.ppg, c = pl - g * a.ppg;
        const int64_t off = (int64_t)g * a.group_stride + (int64_t)c * a.plane_stride;
        const int16_t* src = a.src + off;
        int32_t* lvl = a.lvl + off;
        int16_t* rec = a.rec + off;
        uint8_t* tu = a.tu + (int64_t)pl * a.tu_plane;
        uint64_t* line = lines + (int64_t)pl * a.lw;
        const int pid = a.plane_id + c, y0c = cy * ctb;
        for (int i = lane; i < 33 * 33; i += 64) (&rc[0][0])[i] = 0;   // recon starts as zeros (Frame.zeros)
        __syncthreads();
        for (int i = lane; i < ctb; i += 64) rc[1 + i][0] = 128;        // x == 0: left = 128 (block.py:45-50)
        for (int cx = 0; cx < a.ccols; ++cx) {
            const int x0c = cx * ctb;
            // top row of this CTU: 128 at y == 0, else the CTU above's bottom row (tagged line words)
            if (cy == 0) {
                for (int i = lane; i < ctb; i += 64) rc[0][1 + i] = 128;
            } else {
                const int nw = (min(ctb, a.w - x0c) + 1) / 2;
                const bool need = lane < nw;
                uint32_t val = 0;
                int spins = 0;
                for (;;) {
                    bool ok = true;
                    if (need) {
                        const uint64_t v = ld_sys64(line + x0c / 2 + lane);
                        ok = (int)(v >> 32) == cy + TG;
                        val = (uint32_t)v;
                    }
                    if (__builtin_amdgcn_read_exec() == __ballot(ok)) break;
                    __builtin_amdgcn_s_sleep(1);
                    ++spins;
                    if (spins > kSpinLimit || ((spins & 1023) == 0 && ld_sys(&a.work[1]))) {
                        if (lane == 0) atomicMax(&a.work[1], 1);
                        stall_s = 1;
                        break;
                    }
                }
                if (need) {
                    rc[0][1 + 2 * lane] = (int16_t)(val & 0xffffu);
                    if (2 * lane + 1 < ctb) rc[0][2 + 2 * lane] = (int16_t)(val >> 16);
                }
            }
            __syncthreads();
            if (stall_s) break;
            // the CTU's TUs in dataflow rounds: lane u = 4x4 unit (ux, uy) of the CTU finds its
            // quadtree leaf (tu_leaf); a TU is ready once the TUs holding the units above and
            // left of it are done (z-order guarantees they precede it), and every round codes
            // its ready TUs batched by size -- the same TUs, in an order that respects every
            // dependency of the sequential z-order walk, so the same results
            const int U = ctb / 4, UU = U * U;
            int tn = 0, ox = 0, oy = 0;
            bool pending = false;
            if (lane < UU) {
                const int ux = lane % U, uy = lane / U, x = x0c + 4 * ux, y = y0c + 4 * uy;
                int own = lane;
                if (x < a.w && y < a.h) {
                    const int n = tu_leaf(a.w, a.h, ctb, pid, a.seed, x, y), nu = n / 4;
                    ox = ux - ux % nu;
                    oy = uy - uy % nu;
                    own = oy * U + ox;
                    pending = ox == ux && oy == uy && x + n <= a.w && y + n <= a.h;
                    tn = n;
                }
                owner_of[lane] = own;
                done_of[lane] = 0;
            }
            __syncthreads();
            for (int round = 0; round < UU && __ballot(pending); ++round) {
                bool ready = pending;
                if (pending) {
                    const int nu = tn / 4;
                    for (int k = 0; k < nu; ++k) {
                        if (oy > 0 && !done_of[owner_of[(oy - 1) * U + ox + k]]) ready = false;
                        if (ox > 0 && !done_of[owner_of[(oy + k) * U + ox - 1]]) ready = false;
                    }
                }
                const uint64_t lt = (1ull << lane) - 1ull;
#define NH_BATCH(NN, DST, Q)                                                                                 \
                {                                                                                            \
                    const uint64_t m = __ballot(ready && tn == NN);                                          \
                    const int cnt = __popcll(m);                                                             \
                    if (ready && tn == NN) {                                                                 \
                        const int k = __popcll(m & lt);                                                      \
                        slx[k] = ox * 4;                                                                     \
                        sly[k] = oy * 4;                                                                     \
                    }                                                                                        \
                    __syncthreads();                                                                         \
                    for (int c0 = 0; c0 < cnt; c0 += 64 / NN) {                                             \
                        if constexpr (NARROW)                                                                \
                            tu_closed_batch_pk<NN, DST>(a, src, lvl, rec, tu, x0c, y0c, min(cnt - c0, 64 / NN), \
                                                        slx + c0, sly + c0, rc, (int16_t*)&tile[0][0], Q);   \
                        else                                                                                 \
                            tu_closed_batch<NN, DST>(a, src, lvl, rec, tu, x0c, y0c, min(cnt - c0, 64 / NN), \
                                                     slx + c0, sly + c0, rc, tile, Q);                       \
                    }                                                                                        \
                }
                NH_BATCH(32, false, cq[3]);
                NH_BATCH(16, false, cq[2]);
                NH_BATCH(8, false, cq[1]);
                if (a.is_luma) NH_BATCH(4, true, cq[0]) else NH_BATCH(4, false, cq[0])
#undef NH_BATCH
                if (ready) {
                    done_of[lane] = 1;
                    pending = false;
                }
                __syncthreads();
            }
            // publish the bottom row (the next CTU row polls it), then slide: right column -> left column
            if (cy + 1 < a.crows) {
                const int nw = (min(ctb, a.w - x0c) + 1) / 2;
                if (lane < nw) {
                    const uint32_t lo = (uint16_t)rc[ctb][1 + 2 * lane];
                    const uint32_t hi = 2 * lane + 1 < ctb ? (uint16_t)rc[ctb][2 + 2 * lane] : 0u;
                    st_sys64(line + x0c / 2 + lane, ((uint64_t)(uint32_t)(cy + 1 + TG) << 32) | lo | (hi << 16));
                }
            }
            __syncthreads();
            int16_t keep = 0;
            if (lane < ctb) keep = rc[1 + lane][ctb];
            __syncthreads();
            for (int i = lane; i < 33 * 33; i += 64) (&rc[0][0])[i] = 0;
            __syncthreads();
            if (lane < ctb) rc[1 + lane][0] = keep;
            __syncthreads();
        }
        __syncthreads();
        if (stall_s) break;
    }
}

// ---------------------------------------------------------------------------
// Config 4 closed loop, 8-bit streams: PLANE PAIRS.  The seeded quadtree of a
// plane depends on its plane id, not on its frame, so the same CTU of two
// frames has the same TUs and the same dataflow rounds.  A wave codes one CTU
// row of two such planes (groups 2p and 2p + 1 of the set, same plane in the
// group) in lock-step: each round's batch carries the ready TUs of both planes
// (entry e < cnt: plane 0's TU e, else plane 1's TU e - cnt), so a round whose
// TUs filled a quarter of the lanes for one plane fills half of them for two.
// Every TU runs the same packed chain as tu_closed_batch_pk on its own plane's
// LDS reconstruction and tile: same results.  The planes of a pair never
// exchange data; each publishes and polls its own line words.
// Round 5: a wave may code NPL planes (2 for luma, 4 for chroma): the planes of
// a group are consecutive groups of the set, so plane s of the wave lies s group
// strides past plane 0 (and its TU map s * ppg TU planes past), no pointer table.
struct PairPlanes {
    const int16_t* src0;
    int32_t* lvl0;
    int16_t* rec0;
    uint8_t* tu0;
    int64_t gs, ts;   // elements / TU-map bytes from one plane of the wave to the next
    const __attribute__((address_space(3))) int16_t* stile;   // the CTU's source samples in LDS ([plane][row][stp]),
                                                             // or null: read src
    int32_t stp;            // the tile's row pitch (CTB)
    __device__ const int16_t* src(int p) const { return src0 + p * gs; }
    __device__ int32_t* lvl(int p) const { return lvl0 + p * gs; }
    __device__ int16_t* rec(int p) const { return rec0 + p * gs; }
    __device__ uint8_t* tu(int p) const { return tu0 + p * ts; }
};
// plane of batch entry e (< total = cnt * planes): e / cnt for up to 4 planes, without a division
__device__ __forceinline__ int entry_plane(int e, int cnt) {
    return (e >= cnt ? 1 : 0) + (e >= 2 * cnt ? 1 : 0) + (e >= 3 * cnt ? 1 : 0);
}

// k_tu_closed_pair runs ONE wave per workgroup: its LDS accesses execute in
// program order, so a wave-level code-motion barrier is all the chains and the
// round loop need between an LDS write and another lane's read (no
// s_waitcnt on the LDS queue, no barrier).  -DNH_CLOSED4_WGSYNC=1 builds the
// previous workgroup barriers (A/B).
#ifndef NH_CLOSED4_WGSYNC
#define NH_CLOSED4_WGSYNC 0
#endif
#ifndef NH_CLOSED4_PAIR_CLEAR   // 1: clear the pair kernel's LDS reconstruction before every CTU (A/B)
#define NH_CLOSED4_PAIR_CLEAR 0
#endif
#ifndef NH_CLOSED4_PRIO   // the luma wavefront's waves issue at a higher priority than chroma's (s_setprio):
#define NH_CLOSED4_PRIO 1   // 0.1196-0.1200 vs 0.1205-0.1209 ms per 4K YUV420 frame concurrent (-DNH_CLOSED4_PRIO=0)
#endif
#ifndef NH_CLOSED4_TL_INNER   // 1: closed_chain32_tf's per-lane constants made per TU, not held
#define NH_CLOSED4_TL_INNER 0
#endif
#ifndef NH_CLOSED4_MOSAIC   // 1: 16x16, 8x8 and luma 4x4 TUs on the f16 matrix cores (tu_closed_batch_mma); 2: + chroma 4x4
#define NH_CLOSED4_MOSAIC 2
#endif
#ifndef NH_CLOSED4_DIRECT   // 1: launches of few CTU rows (REC = false) store the mosaics' outputs from registers
#define NH_CLOSED4_DIRECT 1
#endif
#ifndef NH_CLOSED4_MIX   // 1: a round's 8x8 and 4x4 TUs in one call when each fits one mosaic (tu_closed_batch_mix)
#define NH_CLOSED4_MIX 1
#endif
#ifndef NH_CLOSED4_EARLYPOLL
#define NH_CLOSED4_EARLYPOLL 0   // measured 2 % slower (profiles/r03/closed4/ab_libs_closed4_r03l.jsonl)
#endif
__device__ __forceinline__ void pair_sync() {
#if NH_CLOSED4_WGSYNC
    __syncthreads();
#else
    __builtin_amdgcn_wave_barrier();
#endif
}

template <int N, bool DST, int RP = 33>
__device__ __forceinline__ void tu_closed_batch_pk2(const Closed4Args& a, const PairPlanes& pp, int x0c, int y0c,
                                                    int cnt, int total, int c0, const uint8_t* ent,
                                                    int16_t (*rc2)[RP][RP], int16_t* t16, const ChainQ& cq,
                                                    uint32_t& wb, uint64_t* ph = nullptr, bool rec_later = false) {
    constexpr int L2 = Log2<N>::v, S = L2 + 5, H = N / 2, TP = 34;
    // A/B build, NH_CLOSED4_STAMPS: shader cycles of the batch's phases, summed per TU size into ph
    // (LDS, lane 0) -- the s_memtime reads drain the LDS queue, so they sit where the chain syncs anyway
    uint64_t ph_t = 0;
    auto phase = [&](int k) {
        if (NH_AB && ph) {
            const uint64_t tnow = __builtin_amdgcn_s_memtime();
            if (k >= 0 && __lane_id() == 0) ph[8 * (5 - L2) + k] += tnow - ph_t;
            ph_t = tnow;
        }
    };
    phase(-1);
    constexpr int32_t BIAS = 1 << (S - 1);
    const int lane = opaque_lane64(), t = lane % N, e = c0 + lane / N;
    const bool on = e < total;
    const int p = on ? entry_plane(e, cnt) : 0, k = on ? e - p * cnt : 0;   // idle lanes shadow plane 0's first TU
    const int code = ent[k], lx = (code & 7) * 4, ly = ((code >> 3) & 7) * 4, x = x0c + lx, y = y0c + ly;
    int16_t (*rc)[RP] = rc2[p];
    const int16_t* src = pp.src(p);
    int16_t* tl = t16 + p * ((RP - 1) * TP) + ly * TP + lx;   // tl[line * TP + slot]
    // the TU's source column, every load issued before any use: the waits for them then
    // overlap the neighbour reads and the DC / planar sums, not one round trip per row pair
    int32_t sv[N];
    {
        const int16_t* sp = src + (int64_t)y * a.pitch + x + t;
        if (pp.stile) {
#pragma unroll
            for (int i = 0; i < N; ++i) sv[i] = pp.stile[(p * pp.stp + ly + i) * pp.stp + lx + t];
        } else {
#pragma unroll
            for (int i = 0; i < N; ++i)
                sv[i] = (NH_AB && (a.probe & 32)) ? rc[ly + 1 + i][lx + 1 + t]   // A/B probe: no source loads
                                                  : sp[(int64_t)i * a.pitch];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < N; ++i) wb |= (uint32_t)sv[i];   // the stream's wide check (k_tu_closed_pair)
    }
    const int32_t topt = rc[ly][lx + 1 + t], leftt = rc[ly + 1 + t][lx];
    const int32_t tr = rc[ly][lx + N], bl = rc[ly + N][lx];   // top[-1], left[-1] (__main__.py:168)
    int32_t sum = topt + leftt;                                // DC (intra.py:46-62)
    sum = grp_sum<N>(sum);
    const int32_t dc = (sum + N) >> (L2 + 1);
    const pk16 dc2 = pk_splat(dc);
    pk16 o2[H];
    pku16 pl2[H];
    {
        const int32_t b = (t + 1) * tr + (N - 1) * topt + bl + N, st = bl - topt;
        pku16 bs = {(unsigned short)b, (unsigned short)(b + st)};
        const pku16 st2 = {(unsigned short)(2 * st), (unsigned short)(2 * st)};
        const pku16 wl = {(unsigned short)(N - 1 - t), (unsigned short)(N - 1 - t)};
        const pku16 sh = {(unsigned short)(L2 + 1), (unsigned short)(L2 + 1)};
#pragma unroll
        for (int m = 0; m < H; ++m) {
            o2[m] = pk_pair(sv[2 * m], sv[2 * m + 1]);
            const pku16 lf = {(unsigned short)rc[ly + 1 + 2 * m][lx], (unsigned short)rc[ly + 2 + 2 * m][lx]};
            pl2[m] = (lf * wl + bs) >> sh;
            bs += st2;
        }
    }
    int32_t ed = 0, ep = 0;
#pragma unroll
    for (int m = 0; m < H; ++m) {
        const pk16 d0 = o2[m] - dc2, d1 = o2[m] - __builtin_bit_cast(pk16, pl2[m]);
        ed = __builtin_amdgcn_sdot2(d0, d0, ed, false);
        ep = __builtin_amdgcn_sdot2(d1, d1, ep, false);
    }
    ed = grp_sum<N>(ed);
    ep = grp_sum<N>(ep);
    const bool use_dc = ed <= ep;   // __main__.py:173: DC wins ties
    phase(0);
    pk16 r2[H];
#pragma unroll
    for (int m = 0; m < H; ++m) r2[m] = o2[m] - (use_dc ? dc2 : __builtin_bit_cast(pk16, pl2[m]));
    int32_t yv[N];
    fwd1d_pk<N, DST>(r2, yv, BIAS);   // forward pass 1 (transform.py:179-185): column t -> line i, slot t
    if (on) {
#pragma unroll
        for (int i = 0; i < N; ++i) tl[i * TP + t] = (int16_t)(yv[i] >> S);
    }
    pair_sync();
    phase(1);
    const int st = inv_slot<N, DST>(t);
    {
        pk16 P[H];   // forward pass 2 (transform.py:188-194): row t
#pragma unroll
        for (int m = 0; m < H; ++m) P[m] = pk_pair(tl[t * TP + 2 * m], tl[t * TP + 2 * m + 1]);
        fwd1d_pk<N, DST>(P, yv, BIAS);
    }
    pair_sync();
    phase(2);
    if (on) {   // quantize_block -> levels; dequantize_block -> line k, slot inv_slot(t)
        int32_t* lrow = pp.lvl(p) + (int64_t)(y + t) * a.pitch + x;
#pragma unroll
        for (int q4 = 0; q4 < N / 4; ++q4) {   // 4 levels per piece, stored together
            int32_t l4[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int kk = 4 * q4 + e;
                l4[e] = quant_s(yv[kk] >> S, cq.qs, cq.h_v, cq.hneg_v);
                tl[kk * TP + st] = (int16_t)dequant_s(l4[e], cq);
            }
            if (NH_AB && (a.probe & 64)) continue;
#pragma unroll
            for (int e = 0; e < 4; ++e) lrow[4 * q4 + e] = l4[e];   // (adjacent: one 16-B store)
        }
    }
    pair_sync();
    phase(3);
    int32_t xv[N];
    {
        pk16 Y[H];   // inverse pass 1 (transform.py:221-227): column t -> line i, slot inv_slot(t)
#pragma unroll
        for (int m = 0; m < H; ++m) Y[m] = pk_pair(tl[t * TP + 2 * m], tl[t * TP + 2 * m + 1]);
        inv1d_pk<N, DST>(Y, xv, BIAS);
    }
    pair_sync();
    if (on) {
#pragma unroll
        for (int i = 0; i < N; ++i) tl[i * TP + st] = (int16_t)(xv[i] >> S);
    }
    pair_sync();
    phase(4);
    {
        pk16 Y[H];   // inverse pass 2 (transform.py:230-236): row t
#pragma unroll
        for (int m = 0; m < H; ++m) Y[m] = pk_pair(tl[t * TP + 2 * m], tl[t * TP + 2 * m + 1]);
        inv1d_pk<N, DST>(Y, xv, BIAS);
    }
    if (on) {   // reconstruct + clip (intra.py:70-78); planar in row layout
        const int32_t b = (N - 1) * leftt + tr + (t + 1) * bl + N, stv = tr - leftt;
        int16_t* rrow = pp.rec(p) + (int64_t)(y + t) * a.pitch + x;
#pragma unroll
        for (int q4 = 0; q4 < N / 4; ++q4) {   // 4 samples per piece, stored together
            int32_t r4[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int kk = 4 * q4 + e;
                const int32_t pr = use_dc ? dc : ((N - 1 - t) * (int32_t)rc[ly][lx + 1 + kk] + b + kk * stv) >> (L2 + 1);
                int32_t q = pr + (xv[kk] >> S);
                r4[e] = q < 0 ? 0 : (q > 255 ? 255 : q);
                rc[ly + 1 + t][lx + 1 + kk] = (int16_t)r4[e];   // no TU of this batch reads the TU's own samples
            }
            if ((NH_AB && (a.probe & 64)) || rec_later) continue;   // (rec_later: the CTU's rows leave from rc)
#pragma unroll
            for (int e = 0; e < 4; ++e) rrow[4 * q4 + e] = (int16_t)r4[e];   // (adjacent: one 8-B store)
        }
        if (t < N / 4 && !(NH_AB && (a.probe & 64))) {
            uint8_t* tu = pp.tu(p);
            const int w4 = a.w / 4;
            for (int jj = 0; jj < N / 4; ++jj) tu[(int64_t)(y / 4 + t) * w4 + x / 4 + jj] = (uint8_t)L2;
        }
    }
    pair_sync();
    phase(5);
}

// ---------------------------------------------------------------------------
template <int N, bool DST, int NM, int RP, bool DIRECT>
struct MosaicSet : MosaicCore<N, DST, NM> {
    using C = MosaicCore<N, DST, NM>;
    using C::t; using C::yr0; using C::el; using C::L2; using C::TPM;
    int pm[NM], lxm[NM], lym[NM];
    bool onm[NM];
    int32_t sv[NM][4];

    __device__ __forceinline__ void init(int lane, const uint8_t* ent, int cnt, int total, int e0) {
        C::lane_init(lane);
#pragma unroll
        for (int m = 0; m < NM; ++m) {
            const int e = e0 + m * TPM + el;
            onm[m] = e < total;
            pm[m] = onm[m] ? entry_plane(e, cnt) : 0;
            const int code = ent[onm[m] ? e - pm[m] * cnt : 0];   // idle lanes shadow plane 0's first TU
            lxm[m] = (code & 7) * 4;
            lym[m] = ((code >> 3) & 7) * 4;
        }
    }
    // the TUs' source samples, every load issued before any use
    __device__ __forceinline__ void load(const Closed4Args& a, const PairPlanes& pp, int x0c, int y0c,
                                         int16_t (*rc2)[RP][RP]) {
        if (pp.stile) {
#pragma unroll
            for (int m = 0; m < NM; ++m) {
                const __attribute__((address_space(3))) int16_t* tp =
                    pp.stile + (pm[m] * pp.stp + lym[m] + yr0) * pp.stp + lxm[m] + t;
#pragma unroll
                for (int r = 0; r < 4; ++r) sv[m][r] = tp[r * pp.stp];
            }
        } else {
#pragma unroll
            for (int m = 0; m < NM; ++m) {
                const int16_t* sp = pp.src(pm[m]) + (int64_t)(y0c + lym[m] + yr0) * a.pitch + x0c + lxm[m] + t;
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    sv[m][r] = (NH_AB && (a.probe & 32)) ? rc2[pm[m]][lym[m] + 1 + yr0 + r][lxm[m] + 1 + t]
                                                         : sp[(int64_t)r * a.pitch];
            }
        }
    }
    // the neighbours from the pair's LDS reconstruction
    struct Nb {
        const MosaicSet& s;
        int16_t (*rc2)[RP][RP];
        __device__ int32_t top(int m) const { return rc2[s.pm[m]][s.lym[m]][s.lxm[m] + 1 + s.t]; }
        __device__ int32_t tr(int m) const { return rc2[s.pm[m]][s.lym[m]][s.lxm[m] + N]; }
        __device__ int32_t bl(int m) const { return rc2[s.pm[m]][s.lym[m] + N][s.lxm[m]]; }
        __device__ int32_t dcl(int m) const { return rc2[s.pm[m]][s.lym[m] + 1 + s.t][s.lxm[m]]; }
        __device__ pku16 left2(int m, int y) const {
            return (pku16){(unsigned short)rc2[s.pm[m]][s.lym[m] + 1 + y][s.lxm[m]],
                           (unsigned short)rc2[s.pm[m]][s.lym[m] + 2 + y][s.lxm[m]]};
        }
    };
    __device__ __forceinline__ void predict(int16_t (*rc2)[RP][RP], uint32_t& wb) {
#pragma unroll
        for (int m = 0; m < NM; ++m)
#pragma unroll
            for (int r = 0; r < 4; ++r) wb |= (uint32_t)sv[m][r];   // the stream's wide check
        C::predict(sv, Nb{*this, rc2});
    }
    // quantize_block (levels: straight out, or into the tile) and dequantize_block
    __device__ __forceinline__ void quant(const Closed4Args& a, const PairPlanes& pp, int x0c, int y0c,
                                          const ChainQ& cq, int32_t* tile) {
        C::quant(cq, [&](int m, int q, int32_t L0, int32_t L1) {
            if constexpr (DIRECT) {
                if (onm[m] && !(NH_AB && (a.probe & 64))) {
                    int32_t* lp = pp.lvl(pm[m]) + (int64_t)(y0c + lym[m] + yr0 + 2 * q) * a.pitch + x0c + lxm[m] + t;
                    lp[0] = L0;
                    lp[a.pitch] = L1;
                }
            } else {
                int32_t* tl = tile + ((m * TPM + el) * N + yr0) * N + t;
                tl[(2 * q) * N] = L0;
                tl[(2 * q + 1) * N] = L1;
            }
        });
    }
    // reconstruct + clip (intra.py:70-78) into rc (no TU of the batch reads another's samples)
    __device__ __forceinline__ void recon(const Closed4Args& a, const PairPlanes& pp, int x0c, int y0c,
                                          int16_t (*rc2)[RP][RP], bool rec_later) {
        C::recon([&](int m, int q, pku16 rv) {
            if (onm[m]) {
                int16_t (*rc)[RP] = rc2[pm[m]];
                rc[lym[m] + 1 + yr0 + 2 * q][lxm[m] + 1 + t] = (int16_t)rv.x;
                rc[lym[m] + 2 + yr0 + 2 * q][lxm[m] + 1 + t] = (int16_t)rv.y;
                if (DIRECT && !rec_later && !(NH_AB && (a.probe & 64))) {
                    int16_t* rp = pp.rec(pm[m]) + (int64_t)(y0c + lym[m] + yr0 + 2 * q) * a.pitch + x0c + lxm[m] + t;
                    rp[0] = (int16_t)rv.x;
                    rp[a.pitch] = (int16_t)rv.y;
                }
                if (DIRECT && q == 1 && (t & 3) == 0 && !(NH_AB && (a.probe & 64)))   // the TU map: a byte per 4x4 unit
                    pp.tu(pm[m])[(int64_t)((y0c + lym[m] + yr0) / 4) * (a.w / 4) + (x0c + lxm[m] + t) / 4] = (uint8_t)L2;
            }
        });
    }
    // the tile form's outputs (after the recon's sync): 16-B level rows from the tile, 8-B recon rows
    // from rc, the TU map; piece i = 4 samples of one TU row, N / 4 pieces per lane for NM = N / 4
    __device__ __forceinline__ void stores(const Closed4Args& a, const PairPlanes& pp, int x0c, int y0c,
                                           int16_t (*rc2)[RP][RP], const int32_t* tile, const uint8_t* ent, int cnt,
                                           int total, int e0, bool rec_later, int lane) {
        const bool st = !(NH_AB && (a.probe & 64));
        constexpr int PIECES = NM * TPM * N * N / 4;   // the set's level pieces
#pragma unroll
        for (int i = 0; i < (PIECES + 63) / 64; ++i) {
            const int pc = lane + 64 * i, tl = pc / (N * N / 4), row = (pc / (N / 4)) % N, c4 = pc % (N / 4);
            const int e = e0 + tl;
            if (pc < PIECES && e < total && st) {
                const int p = entry_plane(e, cnt), code = ent[e - p * cnt];
                const int lx = (code & 7) * 4, ly = ((code >> 3) & 7) * 4;
                const int64_t o = (int64_t)(y0c + ly + row) * a.pitch + x0c + lx + 4 * c4;
                const int4 lv = *(const int4*)&tile[(tl * N + row) * N + 4 * c4];
                int32_t* lp = pp.lvl(p) + o;
                lp[0] = lv.x;
                lp[1] = lv.y;
                lp[2] = lv.z;
                lp[3] = lv.w;
                if (!rec_later) {
                    const int16_t* q4 = &rc2[p][ly + 1 + row][lx + 1 + 4 * c4];
                    int16_t* rp = pp.rec(p) + o;
                    rp[0] = q4[0];
                    rp[1] = q4[1];
                    rp[2] = q4[2];
                    rp[3] = q4[3];
                }
                if (c4 == 0 && (row & 3) == 0) {
                    uint8_t* tu = pp.tu(p);
                    const int w4 = a.w / 4;
#pragma unroll
                    for (int jj = 0; jj < N / 4; ++jj)
                        tu[(int64_t)((y0c + ly + row) / 4) * w4 + (x0c + lx) / 4 + jj] = (uint8_t)L2;
                }
            }
        }
    }
};

template <int N, bool DST, int RP = 33, bool DIRECT = false, int NMS = N / 4>
__device__ __forceinline__ void tu_closed_batch_mma(const Closed4Args& a, const PairPlanes& pp, int x0c, int y0c,
                                                    int cnt, int total, int c0, const uint8_t* ent,
                                                    int16_t (*rc2)[RP][RP], int32_t* tile, const ChainQ& cq,
                                                    uint32_t& wb, uint64_t* ph = nullptr, bool rec_later = false) {
    constexpr int L2 = Log2<N>::v;
    uint64_t ph_t = 0;
    auto phase = [&](int k) {   // A/B build, NH_CLOSED4_STAMPS (as tu_closed_batch_pk2)
        if (NH_AB && ph) {
            const uint64_t tnow = __builtin_amdgcn_s_memtime();
            if (k >= 0 && __lane_id() == 0) ph[8 * (5 - L2) + k] += tnow - ph_t;
            ph_t = tnow;
        }
    };
    phase(-1);
    const int lane = opaque_lane64();
    MosaicSet<N, DST, NMS, RP, DIRECT> ms;   // (4x4 rounds of more than 16 TUs: two mosaics in one call)
    ms.init(lane, ent, cnt, total, c0);
    ms.load(a, pp, x0c, y0c, rc2);
    __builtin_amdgcn_sched_barrier(0);
    ms.predict(rc2, wb);
    phase(0);
    ms.pass1();
    ms.pass2();
    ms.ready();
    phase(1);
    ms.quant(a, pp, x0c, y0c, cq, tile);
    phase(2);
    ms.inv1();
    ms.inv2();
    phase(3);
    ms.recon(a, pp, x0c, y0c, rc2, rec_later);
    pair_sync();
    phase(4);
    if constexpr (!DIRECT) {
        ms.stores(a, pp, x0c, y0c, rc2, tile, ent, cnt, total, c0, rec_later, lane);
        pair_sync();   // the tile's and rc's reads before the next batch writes them
    }
    phase(5);
}

// A round's 8x8 TUs (tot8 <= 4: one mosaic) and 4x4 TUs (tot4 <= 16: one mosaic) in ONE call: the two
// sets' chains interleaved phase by phase, so the round pays one chain's latency, not two
template <bool DST4, int RP = 33, bool DIRECT = false>
__device__ __forceinline__ void tu_closed_batch_mix(const Closed4Args& a, const PairPlanes& pp, int x0c, int y0c,
                                                    int cnt8, const uint8_t* ent8, int cnt4, const uint8_t* ent4,
                                                    int npl, int16_t (*rc2)[RP][RP], int32_t* tile,
                                                    const ChainQ& cq8, const ChainQ& cq4, uint32_t& wb,
                                                    bool rec_later) {
    const int lane = opaque_lane64();
    MosaicSet<8, false, 1, RP, DIRECT> s8;
    MosaicSet<4, DST4, 1, RP, DIRECT> s4;
    const int tot8 = cnt8 * npl, tot4 = cnt4 * npl;
    s8.init(lane, ent8, cnt8, tot8, 0);
    s4.init(lane, ent4, cnt4, tot4, 0);
    s8.load(a, pp, x0c, y0c, rc2);
    s4.load(a, pp, x0c, y0c, rc2);
    __builtin_amdgcn_sched_barrier(0);
    s8.predict(rc2, wb);
    s4.predict(rc2, wb);
    s8.pass1();
    s4.pass1();
    s8.pass2();
    s4.pass2();
    s8.ready();
    s4.ready();
    s8.quant(a, pp, x0c, y0c, cq8, tile);
    s4.quant(a, pp, x0c, y0c, cq4, tile + 256);
    s8.inv1();
    s4.inv1();
    s8.inv2();
    s4.inv2();
    s8.recon(a, pp, x0c, y0c, rc2, rec_later);
    s4.recon(a, pp, x0c, y0c, rc2, rec_later);
    pair_sync();
    if constexpr (!DIRECT) {
        s8.stores(a, pp, x0c, y0c, rc2, tile, ent8, cnt8, tot8, 0, rec_later, lane);
        s4.stores(a, pp, x0c, y0c, rc2, tile + 256, ent4, cnt4, tot4, 0, rec_later, lane);
        pair_sync();
    }
}

// A 32x32 luma TU of the closed loop on the f16 matrix cores: the config-5
// block chain's transposition-free passes (tf_passes, nh_f16mma.hpp; DESIGN.md
// §4.5: exact integer sums in the fp32 accumulators) with the closed loop's
// inputs -- the neighbours from the plane's LDS reconstruction rc (top row
// rc[0][1 + x], left column rc[1 + y][0], tr = rc[0][32], bl = rc[32][0]) and the
// source samples from global memory.  Lane (r, hh) = column r, rows crow(2p, hh)
// and +1.  Levels and reconstruction leave through the tile ot (the packed
// chains' transpose tile; no other TU of the CTU runs) in whole rows, as in
// config 5: 4 + 2 store instructions of 16 B per lane instead of 32 + 16 of one
// sample per lane (the launch checks the rows' 16-B alignment,
// Closed4Args::mfma32).  A 32x32 TU is the whole CTU, so only its bottom row and
// right column go into rc (the CTU's publish and slide read nothing else; the
// next CTU's TUs rewrite the rest).  Same results as tu_closed_batch_pk2<32>.
constexpr int kClOutP = 36, kClRecP = 24;   // int32 per tile row: levels, recon (48 halves; 16-B rows)
__device__ __forceinline__ void closed_chain32_tf(const Closed4Args& a, const int16_t* src,
                                                  const __attribute__((address_space(3))) int16_t* stl,
                                                  int32_t* lvl, int16_t* rec,
                                                  uint8_t* tu, int x0c, int y0c, int16_t (*rc)[33], int32_t* ot,
                                                  const BasisHC& bs, const ChainQ& cq, const TfLane& tl, uint32_t& wb) {
    const int l = opaque_lane64(), r = l & 31, hh = l >> 5;
    // the TU's source column, every load issued before any use (one wait, not one per row pair)
    int32_t sv[16];
    if (stl) {   // the CTU's source tile (rows of 32)
#pragma unroll
        for (int p = 0; p < 8; ++p) {
            const int c = 2 * (p & 1) + 8 * (p >> 1);   // y_p - 4 hh
#pragma unroll
            for (int e = 0; e < 2; ++e) sv[2 * p + e] = stl[(4 * hh + c + e) * 32 + r];
        }
    } else {
        const int16_t* sp = src + (int64_t)(y0c + 4 * hh) * a.pitch + x0c + r;
#pragma unroll
        for (int p = 0; p < 8; ++p) {
            const int c = 2 * (p & 1) + 8 * (p >> 1);   // y_p - 4 hh
#pragma unroll
            for (int e = 0; e < 2; ++e)
                sv[2 * p + e] = (NH_AB && (a.probe & 32)) ? rc[1 + 4 * hh + c + e][1 + r]   // A/B probe: no source loads
                                                          : sp[(int64_t)(c + e) * a.pitch];
        }
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int k = 0; k < 16; ++k) wb |= (uint32_t)sv[k];   // the stream's wide check
    const int32_t topr = rc[0][1 + r], tr = rc[0][32], bl = rc[32][0];
    int32_t sdc = hh ? (int32_t)rc[1 + r][0] : topr;   // DC (intra.py:46-62): lane halves hold top / left
    sdc = grp_sum<64>(sdc);
    const int32_t dc = (sdc + 32) >> 6;
    const pk16 dc2 = pk_splat(dc);
    pk16 o2[8];
    pku16 pl2[8];
    {   // planar (intra.py:81-113) at (y, r): (31 - r) left[y] + b(y) >> 6, b(y) = b(4 hh) + (y - 4 hh)(bl - top[r])
        const pku16 wl = {(unsigned short)(31 - r), (unsigned short)(31 - r)}, sh = {6, 6};
        const int32_t d = bl - topr, b0 = (r + 1) * tr + (31 - 4 * hh) * topr + (4 * hh + 1) * bl + 32;
        const pku16 d2 = {(unsigned short)d, (unsigned short)d}, bb0 = {(unsigned short)b0, (unsigned short)(b0 + d)};
#pragma unroll
        for (int p = 0; p < 8; ++p) {
            const int c = 2 * (p & 1) + 8 * (p >> 1), y = 4 * hh + c;
            o2[p] = pk_pair(sv[2 * p], sv[2 * p + 1]);
            const pku16 lf = {(unsigned short)rc[1 + y][0], (unsigned short)rc[2 + y][0]};
            pl2[p] = (lf * wl + (bb0 + (pku16){(unsigned short)c, (unsigned short)c} * d2)) >> sh;
        }
    }
    int32_t ed = 0, ep = 0;
#pragma unroll
    for (int p = 0; p < 8; ++p) {
        const pk16 d0 = o2[p] - dc2, d1 = o2[p] - __builtin_bit_cast(pk16, pl2[p]);
        ed = __builtin_amdgcn_sdot2(d0, d0, ed, false);
        ep = __builtin_amdgcn_sdot2(d1, d1, ep, false);
    }
    // DC wins ties (__main__.py:173): ed <= ep as ONE wave reduction of the difference (|.| < 2^27)
    const bool use_dc = grp_sum<64>(ed - ep) <= 0;
    uint32_t hx[8];
    pku16 pr2[8];
#pragma unroll
    for (int p = 0; p < 8; ++p) {
        const pk16 pr = use_dc ? dc2 : __builtin_bit_cast(pk16, pl2[p]);
        const pku16 rr = __builtin_bit_cast(pku16, o2[p] - pr);   // residual, intra.py:65-67
        hx[p] = __builtin_bit_cast(uint32_t, rr * (pku16){2, 2} + (pku16){0x6200, 0x6200});   // f16 of n + 768
        pr2[p] = (pku16){0x6600, 0x6600} - __builtin_bit_cast(pku16, pr);
    }
    const bool st = !(NH_AB && (a.probe & 64));
    const int32_t op = a.pitch;
    char* lb = (char*)(lvl + (int64_t)y0c * a.pitch + x0c);
    pku16 rec2[8];
    tf_passes(hx, pr2, bs, cq, tl, r, hh, [&](int g, int32_t L) { ot[crow(g, hh) * kClOutP + r] = L; },
              [&] {
                  pair_sync();
#pragma unroll
                  for (int i = 0; i < 4; ++i) {   // 4 instructions of 8 whole 128-B level rows
                      const int rr = (l >> 3) + 8 * i, c = 4 * (l & 7);
                      const int4 v = *(const int4*)&ot[rr * kClOutP + c];
                      if (st) *(int4*)(lb + vofs((rr * op + c) * 4)) = v;
                  }
                  pair_sync();   // the tile's reads before the recon reuses it
              },
              rec2);
    int16_t* rt = (int16_t*)ot;
#pragma unroll
    for (int p = 0; p < 8; ++p) {
        const int y = 2 * (p & 1) + 8 * (p >> 1) + 4 * hh;
        rt[y * 2 * kClRecP + r] = (int16_t)rec2[p].x;
        rt[(y + 1) * 2 * kClRecP + r] = (int16_t)rec2[p].y;
        if (r == 31) {   // the right column (the next CTU's left neighbours)
            rc[1 + y][32] = (int16_t)rec2[p].x;
            rc[2 + y][32] = (int16_t)rec2[p].y;
        }
    }
    if (hh == 1) rc[32][1 + r] = (int16_t)rec2[7].y;   // row 31 (= y_7 + 1 of the upper half): the bottom row
    pair_sync();
    char* rb = (char*)(rec + (int64_t)y0c * a.pitch + x0c);
#pragma unroll
    for (int i = 0; i < 2; ++i) {   // 2 instructions of 16 whole 64-B recon rows
        const int rr = (l >> 2) + 16 * i, c = 4 * (l & 3);
        const uint4 v = *(const uint4*)&ot[rr * kClRecP + c];
        if (st) *(uint4*)(rb + vofs((rr * op + 2 * c) * 2)) = v;
    }
    const int w4 = a.w / 4;   // the TU map: 8 x 8 units of log2 size 5
    if (st) tu[(int64_t)(y0c / 4 + (l >> 3)) * w4 + x0c / 4 + (l & 7)] = (uint8_t)5;
    pair_sync();   // the tile's reads before the next TU's writes
}

// The TU schedule of one CTU of one plane id (k_closed4_plan, NH_CLOSED4_PLAN):
// the quadtree and so the dataflow rounds depend on (plane id, CTU) only, not
// on the frame, so they are found once per launch instead of once per CTU row of
// every plane pair.  Record (128 B): bytes 0..63 the TUs' codes
// (ox | oy << 3 | size index << 6, in 4x4 units; size index 0 = 32 .. 3 = 4) in
// execution order -- round by round, sizes 32, 16, 8, 4, lane order within --
// and bytes 64..127 the count of each (round, size) pair, 4 * round + size.
#ifndef NH_CLOSED4_PLAN
#define NH_CLOSED4_PLAN 1
#endif
constexpr int kPlanBytes = 128;
__global__ void __launch_bounds__(64) k_closed4_plan(Closed4Args a, uint8_t* plan) {
    __shared__ int owner_of[64], done_of[64];
    const int lane = threadIdx.x, ctb = a.ctb, U = ctb / 4, UU = U * U;
    const int cx = (int)blockIdx.x % a.ccols, cy = (int)blockIdx.x / a.ccols, c = (int)blockIdx.y;
    const int pid = a.plane_id + c, x0c = cx * ctb, y0c = cy * ctb;
    uint8_t* rec = plan + ((int64_t)c * a.crows * a.ccols + blockIdx.x) * kPlanBytes;
    int tn = 0, ox = 0, oy = 0;
    bool pending = false;
    if (lane < UU) {
        const int ux = lane % U, uy = lane / U, x = x0c + 4 * ux, y = y0c + 4 * uy;
        int own = lane;
        if (x < a.w && y < a.h) {
            const int n = tu_leaf(a.w, a.h, ctb, pid, a.seed, x, y), nu = n / 4;
            ox = ux - ux % nu;
            oy = uy - uy % nu;
            own = oy * U + ox;
            pending = ox == ux && oy == uy && x + n <= a.w && y + n <= a.h;
            tn = n;
        }
        owner_of[lane] = own;
        done_of[lane] = 0;
    }
    rec[64 + lane] = 0;
    __syncthreads();
    const uint64_t lt = (1ull << lane) - 1ull;
    int off = 0;
    for (int round = 0; round < 16 && __ballot(pending); ++round) {
        bool ready = pending;
        if (pending) {
            const int nu = tn / 4;
            for (int k = 0; k < nu; ++k) {
                if (oy > 0 && !done_of[owner_of[(oy - 1) * U + ox + k]]) ready = false;
                if (ox > 0 && !done_of[owner_of[(oy + k) * U + ox - 1]]) ready = false;
            }
        }
#pragma unroll
        for (int si = 0; si < 4; ++si) {
            const bool mine = ready && tn == (32 >> si);
            const uint64_t m = __ballot(mine);
            if (mine) rec[off + __popcll(m & lt)] = (uint8_t)(ox | (oy << 3) | (si << 6));
            if (lane == 0) rec[64 + 4 * round + si] = (uint8_t)__popcll(m);
            off += __popcll(m);
        }
        __syncthreads();
        if (ready) {
            done_of[lane] = 1;
            pending = false;
        }
        __syncthreads();
    }
}

// The pair form of k_tu_closed (NARROW streams only: the wide flag work[2]
// makes it return when the 32-bit form codes the stream).  Tickets run
// row-major over the pairs: ticket t = CTU row t / npairs of pair t % npairs;
// pair q = (group pair q / ppg, plane q % ppg); a wave only waits on the same
// pair's CTU row above, claimed before it.
// The compiler's allocation (135 VGPRs, 3 waves/SIMD): 0.150 ms per 4K YUV420
// frame vs 0.164 capped at 4 waves (128 VGPRs, 1 spilled), DESIGN.md §4.4a.
#ifndef NH_CLOSED4_WAVES32   // waves-per-EU target of the CTB 32 (luma) instance
#define NH_CLOSED4_WAVES32 3
#endif
constexpr int kPairWaves = NH_CLOSED4_WAVES32;
#ifndef NH_CLOSED4_NPL16   // planes per wave of the CTB <= 16 (chroma) instance: 2 or 4
#define NH_CLOSED4_NPL16 4
#endif
#ifndef NH_CLOSED4_WAVES16   // its waves-per-EU target
#define NH_CLOSED4_WAVES16 3
#endif
constexpr int kPairWaves16 = NH_CLOSED4_WAVES16;
constexpr int kStampWords = 48;   // A/B stamps per (ticket, CTU)
// REC: whole CTUs' packed-chain recon leaves from rc at the CTU's end (Closed4Args::rec_ctu); a
// separate instantiation, so the per-TU form's code is the same as without the flush
// CTBM: the largest CTB the instance codes (32: luma, 16: chroma; rc rows of CTBM + 1), NPL: planes
// per wave (2 or 4; lanes [64 / NPL q, 64 / NPL (q + 1)) serve plane q's line words and left column)
template <int WAVES, bool REC, int CTBM = 32, int NPL = 2>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WAVES))) k_tu_closed_pair(Closed4Args a) {
    constexpr int TP = 34, RP = CTBM + 1, LPP = 64 / NPL;
    static_assert((NPL == 2 || NPL == 4) && CTBM <= LPP && (CTBM == 32 || CTBM == 16), "plane group shape");
    __shared__ int16_t rc[NPL][RP][RP];
    // the packed chains' int16 tiles (NPL x CTBM rows of TP), the mosaics' level tile (1,024 ints) or
    // closed_chain32_tf's level / recon tile (CTBM 32)
    constexpr int kT32 = std::max({NPL * CTBM * TP / 2, 1024, CTBM == 32 ? 32 * kClOutP : 0});
    __shared__ __attribute__((aligned(16))) int32_t t32[kT32];
    int16_t* const t16 = (int16_t*)t32;
    // the CTU's source samples, [plane][row][CTBM] (LDS-DMA under the poll; Closed4Args::srctile)
    __shared__ __attribute__((aligned(16))) int16_t stile[NPL * CTBM * CTBM];
    // closed_chain32_tf reads its bases from the constant table (L1 / L2 hits), not an LDS copy:
    // the 4 KB went to the source tile at the same occupancy
    const BasisHC& basis_s = c_basis_hc_cl;
#if !NH_CLOSED4_PLAN
    __shared__ int owner_of[64], done_of[64];
#endif
    __shared__ __attribute__((aligned(16))) uint8_t ent_s[NH_CLOSED4_PLAN ? kPlanBytes : 16];
    __shared__ int row_s, stall_s;
    __shared__ uint64_t ph_s[NH_AB ? 32 : 1];   // A/B stamps: per-(TU size, phase) cycle sums of the CTU's batches
    uint64_t* const ph = (NH_AB && a.stamps) ? ph_s : nullptr;
    if (NH_AB && a.stamps && threadIdx.x < 32) ph_s[threadIdx.x] = 0;
    if (__builtin_nontemporal_load(&a.work[2]) != 0) return;   // wide stream: the 32-bit form codes it
    if (NH_CLOSED4_PRIO && a.is_luma) __builtin_amdgcn_s_setprio(2);   // the critical (luma) wavefront issues first
    const int lane = threadIdx.x;
    const int ctb = a.ctb;
    // the stream's wide check, fused: the OR of every source sample the chains load; one outside
    // [0, 255] sets work[2] at the row's end, and the 32-bit form launched behind this kernel then
    // recodes the whole set (the packed chains are exact only on 8-bit TUs; samples no TU reads
    // never matter) -- instead of a scan of the whole set before the launch
    uint32_t wb = 0;
    ChainQ cq[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) cq[k] = make_chainq(a.q[k], a.dqs, a.dq_per);
#if !NH_CLOSED4_TL_INNER
    TfLane tl{};
    if constexpr (CTBM == 32) tl = make_tf_lane(cq[3], basis_s, lane & 31);   // (read only when a.mfma32)
#endif
    uint64_t* lines = reinterpret_cast<uint64_t*>(a.work + a.lines0);
    const int ngroups = a.nplanes / a.ppg, npairs = ((ngroups + NPL - 1) / NPL) * a.ppg;
    const int total = a.crows * npairs;
    const int hq = lane / LPP, hl = lane % LPP;
    for (;;) {
        if (lane == 0) {
            row_s = atomicAdd(&a.work[0], 1);
            stall_s = 0;
        }
        pair_sync();
        const int tk = row_s;
        if (tk >= total) break;
        const int cy = tk / npairs, q = tk - cy * npairs;
        const int c = q % a.ppg, g0 = NPL * (q / a.ppg);
        const int npl = min(NPL, ngroups - g0);   // planes this wave codes (the set's last group may have fewer)
        PairPlanes pp;
        {
            const int64_t off = (int64_t)g0 * a.group_stride + (int64_t)c * a.plane_stride;
            const int pl = g0 * a.ppg + c;
            pp.src0 = a.src + off;
            pp.lvl0 = a.lvl + off;
            pp.rec0 = a.rec + off;
            pp.tu0 = a.tu + (int64_t)pl * a.tu_plane;
            pp.gs = a.group_stride;
            pp.ts = (int64_t)a.ppg * a.tu_plane;
            pp.stile = a.srctile ? (const __attribute__((address_space(3))) int16_t*)(lds_void_t*)stile : nullptr;
            pp.stp = CTBM;
        }
        // plane hq's line words (lanes of planes past npl never touch them)
        uint64_t* const lineq = lines + (int64_t)((g0 + hq) * a.ppg + c) * a.lw;
        const int y0c = cy * ctb;
#if !NH_CLOSED4_PLAN
        const int pid = a.plane_id + c;
#endif
        for (int i = lane; i < NPL * RP * RP; i += 64) (&rc[0][0][0])[i] = 0;   // recon starts as zeros (Frame.zeros)
        pair_sync();
        if (hl < ctb) rc[hq][1 + hl][0] = 128;                             // x == 0: left = 128 (block.py:45-50)
        // the first poll of a CTU's line words is issued at the end of the previous CTU,
        // before its publish store, so the two round trips overlap (NH_CLOSED4_EARLYPOLL)
        uint64_t early = 0;
        const uint32_t* plan_row = (const uint32_t*)(a.plan + ((int64_t)c * a.crows + cy) * a.ccols * kPlanBytes);
        for (int cx = 0; cx < a.ccols; ++cx) {
            const int x0c = cx * ctb;
            const int nw = (min(ctb, a.w - x0c) + 1) / 2;
            uint64_t st0 = 0, st1 = 0, st2 = 0;   // A/B stamps: CTU start, poll done, rounds done
            if (NH_AB && a.stamps) st0 = __builtin_amdgcn_s_memtime();
            // this CTU's TU schedule (128 B), loaded under the wait on the row above
            uint32_t planw = 0;
            if (NH_CLOSED4_PLAN && lane < kPlanBytes / 4) planw = plan_row[cx * (kPlanBytes / 4) + lane];
            if (a.srctile) {   // the CTU's source samples into the tile, 16 B a lane, under the poll below
                // (the vmcnt(0) before the rounds retires them; lgkmcnt(0): the previous CTU's tile
                // reads have returned before the DMA overwrites it)
                __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0)
                constexpr int PR = CTBM / 8, PP = CTBM * PR;   // 16-B pieces per row, per plane
#pragma unroll
                for (int i = 0; i < NPL * PP / 64; ++i) {
                    const int q = 64 * i + lane, pq = q / PP, yy = (q / PR) % CTBM, k = q % PR;
                    if (pq < npl && y0c + yy < a.h && x0c + 8 * k < a.w)
                        glds16s(pp.src(0), (uint32_t)((pq * pp.gs + (int64_t)(y0c + yy) * a.pitch + x0c + 8 * k) * 2),
                                lds_addr(stile + 64 * 8 * i));
                }
            }
            // top row of this CTU: 128 at y == 0, else the CTU above's bottom row (tagged line words)
            if (cy == 0) {
                if (hl < ctb) rc[hq][0][1 + hl] = 128;
            } else {
                const bool need = hl < nw && hq < npl;
                uint32_t val = 0;
                int spins = 0;
                for (;;) {
                    bool ok = true;
                    if (need) {
                        const uint64_t v = (NH_CLOSED4_EARLYPOLL && spins == 0 && cx > 0) ? early
                                                                                        : ld_sys64(lineq + x0c / 2 + hl);
                        ok = (int)(v >> 32) == cy || (NH_AB && (a.probe & 1));
                        val = (uint32_t)v;
                    }
                    if (__builtin_amdgcn_read_exec() == __ballot(ok)) break;
                    __builtin_amdgcn_s_sleep(1);
                    ++spins;
                    if (spins > kSpinLimit || ((spins & 1023) == 0 && ld_sys(&a.work[1]))) {
                        if (lane == 0) atomicMax(&a.work[1], 1);
                        stall_s = 1;
                        break;
                    }
                }
                if (need) {
                    rc[hq][0][1 + 2 * hl] = (int16_t)(val & 0xffffu);
                    if (2 * hl + 1 < ctb) rc[hq][0][2 + 2 * hl] = (int16_t)(val >> 16);
                }
            }
            if (NH_CLOSED4_PLAN && lane < kPlanBytes / 4) ((uint32_t*)ent_s)[lane] = planw;
            pair_sync();
            if (stall_s) break;
            // every load before the rounds (line words, schedule) has landed: said as a real
            // s_waitcnt so the compiler's wait insertion knows it -- otherwise its loop analysis
            // keeps one of them pending and puts a vmcnt(0) at the top of every batch, which then
            // also waits for the previous batch's level / recon stores
            __builtin_amdgcn_s_waitcnt(0xF70);   // vmcnt(0)
            if (NH_AB && a.stamps) st1 = __builtin_amdgcn_s_memtime();
            bool rec_flush = false;
#if NH_CLOSED4_PLAN
            {   // the CTU's TUs in dataflow rounds, from the schedule: lane rs holds the count of
                // (round rs / 4, size index rs % 4); batches run in the schedule's order
                const int cntv = ent_s[64 + lane];
                // (round, size) entries with TUs only: walk the set bits of the ballot
                uint64_t nz = __ballot(cntv != 0);
                if (NH_AB && (a.probe & 4)) nz = 0;
                // the CTU is whole and none of its TUs is a matrix-core 32x32 (which stores its own
                // rows): the packed chains leave their recon in rc only, flushed as whole rows below
                rec_flush = REC && x0c + ctb <= a.w && y0c + ctb <= a.h && !(a.mfma32 && (nz & 1));
                int off = 0;
                for (; nz; nz &= nz - 1) {
                    const int rs = __builtin_ctzll(nz);
                    const int cnt = __builtin_amdgcn_readlane(cntv, rs);
                    const int tot = cnt * npl;
                    const uint8_t* ent = ent_s + off;
                    switch (rs & 3) {
#define NH_PLAN_BATCH(NN, DST, Q)                                                                             \
                        for (int c0 = 0; c0 < tot && !(NH_AB && (a.probe & 2)); c0 += 64 / NN)                    \
                            tu_closed_batch_pk2<NN, DST>(a, pp, x0c, y0c, cnt, tot, c0, ent, rc, t16, Q, wb, ph, rec_flush);
                        case 0:   // (CTB 32: the one 32x32 TU of the CTU, in every plane)
                            if constexpr (CTBM == 32) {
                                if (a.mfma32) {   // one plane after the other, ONE copy of the chain's code:
                                    // a loop the compiler keeps (instruction-cache footprint)
#pragma clang loop unroll(disable)
                                    for (int s2 = 0; s2 < npl; ++s2) {
#if NH_CLOSED4_TL_INNER
                                        const TfLane tl = make_tf_lane(cq[3], basis_s, lane & 31);
#endif
                                        closed_chain32_tf(a, pp.src(s2), pp.stile ? pp.stile + s2 * 32 * 32 : pp.stile,
                                                          pp.lvl(s2), pp.rec(s2), pp.tu(s2), x0c, y0c,
                                                          rc[s2], t32, basis_s, cq[3], tl, wb);
                                    }
                                } else {
                                    NH_PLAN_BATCH(32, false, cq[3])
                                }
                            }
                            break;
#define NH_MOSAIC_BATCH(NN, DST, Q)                                                                           \
                        for (int c0 = 0; c0 < tot && !(NH_AB && (a.probe & 2)); c0 += 64 / NN)                    \
                            tu_closed_batch_mma<NN, DST, RP, !REC && NH_CLOSED4_DIRECT>(                               \
                                a, pp, x0c, y0c, cnt, tot, c0, ent, rc, t32, Q, wb, ph, rec_flush);
                        case 1:
                            if (NH_CLOSED4_MOSAIC) {   // (a pair's one 16x16 TU each: two mosaics, not four)
                                for (int c0 = 0; c0 < tot && !(NH_AB && (a.probe & 2)); c0 += 4) {
                                    if (tot - c0 <= 2)
                                        tu_closed_batch_mma<16, false, RP, !REC && NH_CLOSED4_DIRECT, 2>(
                                            a, pp, x0c, y0c, cnt, tot, c0, ent, rc, t32, cq[2], wb, ph, rec_flush);
                                    else
                                        tu_closed_batch_mma<16, false, RP, !REC && NH_CLOSED4_DIRECT, 4>(
                                            a, pp, x0c, y0c, cnt, tot, c0, ent, rc, t32, cq[2], wb, ph, rec_flush);
                                }
                            } else {
                                NH_PLAN_BATCH(16, false, cq[2])
                            }
                            break;
                        case 2:
                            if (NH_CLOSED4_MIX && NH_CLOSED4_MOSAIC >= 2 && (nz & (2ull << rs)) != 0) {
                                // the round's 4x4 TUs follow: both sizes in one call when each fits a mosaic
                                const int cnt4 = __builtin_amdgcn_readlane(cntv, rs + 1);
                                if (tot <= 4 && cnt4 * npl <= 16 && !(NH_AB && (a.probe & 2))) {
                                    if (a.is_luma)
                                        tu_closed_batch_mix<true, RP, !REC && NH_CLOSED4_DIRECT>(
                                            a, pp, x0c, y0c, cnt, ent, cnt4, ent + cnt, npl, rc, t32, cq[1], cq[0], wb,
                                            rec_flush);
                                    else
                                        tu_closed_batch_mix<false, RP, !REC && NH_CLOSED4_DIRECT>(
                                            a, pp, x0c, y0c, cnt, ent, cnt4, ent + cnt, npl, rc, t32, cq[1], cq[0], wb,
                                            rec_flush);
                                    nz &= ~(2ull << rs);   // the 4x4 entry is done
                                    off += cnt4;
                                    break;
                                }
                            }
                            if (NH_CLOSED4_MOSAIC) { NH_MOSAIC_BATCH(8, false, cq[1]) }
                            else { NH_PLAN_BATCH(8, false, cq[1]) }
                            break;
#define NH_MOSAIC4(DST)                                                                                       \
                        for (int c0 = 0; c0 < tot && !(NH_AB && (a.probe & 2));) {                                \
                            if (tot - c0 > 16) {                                                                  \
                                tu_closed_batch_mma<4, DST, RP, !REC && NH_CLOSED4_DIRECT, 2>(                    \
                                    a, pp, x0c, y0c, cnt, tot, c0, ent, rc, t32, cq[0], wb, ph, rec_flush);       \
                                c0 += 32;                                                                         \
                            } else {                                                                              \
                                tu_closed_batch_mma<4, DST, RP, !REC && NH_CLOSED4_DIRECT, 1>(                    \
                                    a, pp, x0c, y0c, cnt, tot, c0, ent, rc, t32, cq[0], wb, ph, rec_flush);       \
                                c0 += 16;                                                                         \
                            }                                                                                     \
                        }
                        default:
                            if (a.is_luma) {
                                if (NH_CLOSED4_MOSAIC) { NH_MOSAIC4(true) }
                                else { NH_PLAN_BATCH(4, true, cq[0]) }
                            } else {
                                if (NH_CLOSED4_MOSAIC >= 2) { NH_MOSAIC4(false) }
                                else { NH_PLAN_BATCH(4, false, cq[0]) }
                            }
#undef NH_MOSAIC4
#undef NH_PLAN_BATCH
#undef NH_MOSAIC_BATCH
                    }
                    off += cnt;
                }
            }
#else
            // the CTU's TUs in dataflow rounds (as k_tu_closed), found once for both planes
            const int U = ctb / 4, UU = U * U;
            int tn = 0, ox = 0, oy = 0;
            bool pending = false;
            if (lane < UU) {
                const int ux = lane % U, uy = lane / U, x = x0c + 4 * ux, y = y0c + 4 * uy;
                int own = lane;
                if (x < a.w && y < a.h) {
                    const int n = (NH_AB && (a.probe & 16)) ? 4 : tu_leaf(a.w, a.h, ctb, pid, a.seed, x, y), nu = n / 4;
                    ox = ux - ux % nu;
                    oy = uy - uy % nu;
                    own = oy * U + ox;
                    pending = ox == ux && oy == uy && x + n <= a.w && y + n <= a.h;
                    tn = n;
                }
                owner_of[lane] = own;
                done_of[lane] = 0;
            }
            pair_sync();
            for (int round = 0; round < UU && __ballot(pending) && !(NH_AB && (a.probe & 4)); ++round) {
                bool ready = pending;
                if (pending) {
                    const int nu = tn / 4;
                    for (int k = 0; k < nu; ++k) {
                        if (oy > 0 && !done_of[owner_of[(oy - 1) * U + ox + k]]) ready = false;
                        if (ox > 0 && !done_of[owner_of[(oy + k) * U + ox - 1]]) ready = false;
                    }
                }
                const uint64_t lt = (1ull << lane) - 1ull;
#define NH_BATCH2(NN, DST, Q)                                                                                \
                {                                                                                            \
                    const uint64_t m = __ballot(ready && tn == NN);                                          \
                    const int cnt = __popcll(m);                                                             \
                    if (ready && tn == NN) ent_s[__popcll(m & lt)] = (uint8_t)(ox | (oy << 3));            \
                    pair_sync();                                                                             \
                    const int tot = cnt * npl;                                                               \
                    for (int c0 = 0; c0 < tot && !(NH_AB && (a.probe & 2)); c0 += 64 / NN)                   \
                        tu_closed_batch_pk2<NN, DST>(a, pp, x0c, y0c, cnt, tot, c0, ent_s, rc, t16, Q, wb);  \
                }
                NH_BATCH2(32, false, cq[3]);
                NH_BATCH2(16, false, cq[2]);
                NH_BATCH2(8, false, cq[1]);
                if (a.is_luma) NH_BATCH2(4, true, cq[0]) else NH_BATCH2(4, false, cq[0])
#undef NH_BATCH2
                if (ready) {
                    done_of[lane] = 1;
                    pending = false;
                }
                pair_sync();
            }
#endif
            if (NH_AB && a.stamps) st2 = __builtin_amdgcn_s_memtime();
            if (NH_CLOSED4_EARLYPOLL && cy > 0 && cx + 1 < a.ccols) {
                const int nwn = (min(ctb, a.w - x0c - ctb) + 1) / 2;
                if (hl < nwn && hq < npl) early = ld_sys64(lineq + (x0c + ctb) / 2 + hl);
            }
            // publish both bottom rows (the next CTU row polls them), then slide: right column -> left column
            if (cy + 1 < a.crows && hl < nw && hq < npl) {
                const uint32_t lo = (uint16_t)rc[hq][ctb][1 + 2 * hl];
                const uint32_t hi = 2 * hl + 1 < ctb ? (uint16_t)rc[hq][ctb][2 + 2 * hl] : 0u;
                st_sys64(lineq + x0c / 2 + hl, ((uint64_t)(uint32_t)(cy + 1) << 32) | lo | (hi << 16));
            }
            if (rec_flush) {   // the CTU's recon rows, 8-B pieces: ctb / 4 lanes per row, 64 / (ctb / 4) rows a pass
                const int pr = ctb / 4, rpp = 64 / pr, pc = lane % pr, r0 = lane / pr;
                for (int s2 = 0; s2 < npl; ++s2) {
                    int16_t* rb = pp.rec(s2) + (int64_t)y0c * a.pitch + x0c + 4 * pc;
                    for (int r = r0; r < ctb; r += rpp) {
                        const int16_t* q4 = &rc[s2][1 + r][1 + 4 * pc];
                        const uint32_t lo = (uint16_t)q4[0] | ((uint32_t)(uint16_t)q4[1] << 16);
                        const uint32_t hi = (uint16_t)q4[2] | ((uint32_t)(uint16_t)q4[3] << 16);
                        *(uint2*)(rb + (int64_t)r * a.pitch) = make_uint2(lo, hi);
                    }
                }
            }
            pair_sync();
            int16_t keep = 0;
            if (hl < ctb) keep = rc[hq][1 + hl][ctb];
            pair_sync();
            // (the LDS reconstruction is cleared once per CTU row, above: a TU reads only
            // samples coded before it or the top row / left column rewritten per CTU;
            // samples past a ragged edge belong to no TU and are never read)
            if (NH_CLOSED4_PAIR_CLEAR && !(NH_AB && (a.probe & 8)))
                for (int i = lane; i < NPL * RP * RP; i += 64) (&rc[0][0][0])[i] = 0;
            pair_sync();
            if (hl < ctb) rc[hq][1 + hl][0] = keep;
            pair_sync();
            if (NH_AB && a.stamps && lane < 8) {   // (ticket, CTU): cy, pair, 4 stamps, the 64 schedule counts
                uint64_t* o = a.stamps + ((int64_t)tk * a.ccols + cx) * kStampWords;
                if (lane == 0) {
                    o[0] = ((uint64_t)cy << 32) | (uint32_t)q;
                    o[1] = st0;
                    o[2] = st1;
                    o[3] = st2;
                    o[4] = __builtin_amdgcn_s_memtime();
                    o[5] = __builtin_amdgcn_s_memrealtime();
                }
                o[8 + lane] = ((const uint64_t*)(ent_s + 64))[lane];
            }
            if (NH_AB && a.stamps && lane < 32) {
                a.stamps[((int64_t)tk * a.ccols + cx) * kStampWords + 16 + lane] = ph_s[lane];
                ph_s[lane] = 0;
            }
        }
        if (__ballot((wb & ~0xffu) != 0) && lane == 0) atomicOr(&a.work[2], 1);
        pair_sync();
        if (stall_s) break;
    }
}


int tc32_butterfly(const int16_t* d_src, int w, int h, int pitch, int qp, int32_t* d_lvl, int16_t* d_recon,
                   hipStream_t s) {
    const int bw = w / 32, n = bw * (h / 32);
    if (!n) return NH_OK;
    int per, rem;
    qp_split(qp, &per, &rem);
    k_tu_process<32, false, kAll><<<(n + 7) / 8, 256, 0, s>>>(d_src, w, h, pitch, qparams(qp, 5, true),
                                                             dequant_scale(rem), per, d_lvl, d_recon, nullptr, bw, n,
                                                             TreeArgs{});
    NH_HIP(hipGetLastError());
    return NH_OK;
}

}  // namespace nh

using namespace nh;

namespace nh {
// The mosaics' per-lane bases and initial accumulators (c_mosaic_cl), once per device
// (host-synchronous upload: every later kernel on any stream reads them)
int ensure_mosaic_cl() {
    static PerDeviceOnce once_m;
    return once_m.run([] {
        static MosaicLane mt[4][64];
        make_mosaic(mt);
        NH_HIP(hipMemcpyToSymbol(HIP_SYMBOL(c_mosaic_cl), mt, sizeof(mt)));
        return (int)NH_OK;
    });
}
// Config 3's product kernel: 0 = k_intra_rdo8<1, true, 1> (lane per mode); the mosaic forms
// (k_intra_rdo8_mma, A/B build only) measured 201.5-208 vs 200.4-201.8 us per 1080p frame with
// 1.17x the VALU wave-instructions (profiles/r06/cfg3/): not kept
#ifndef NH_RDO_MMA_DEFAULT
#define NH_RDO_MMA_DEFAULT 0
#endif
constexpr int kRdoMmaDefault = NH_RDO_MMA_DEFAULT;
#ifndef NH_RDO_VEC_OUT   // the winners' rows as 16-B stores (when aligned)
#define NH_RDO_VEC_OUT 1
#endif
}  // namespace nh

extern "C" int nh_intra_rdo_plane(const int16_t* d_src, int w, int h, int pitch, int qp, uint8_t* d_modes,
                                  int32_t* d_lvl, int16_t* d_recon, int64_t* d_sse, void* stream) {
    if (!d_src || !d_modes || !d_lvl || !d_recon || w < 0 || h < 0 || pitch < w) return NH_EARG;
    const int nblk = (w / 8) * (h / 8);
    if (!nblk) return NH_OK;
    int per, rem;
    qp_split(qp, &per, &rem);
    const uint32_t ngroups = (uint32_t)((nblk + kRdoSlots - 1) / kRdoSlots);
    const hipStream_t s = as_stream(stream);
    const QuantParams q = qparams(qp, 3, true);
    unsigned long long* sse = (unsigned long long*)d_sse;
    {   // the packed-chain-only launch (3 waves/SIMD), then the fallback for groups with wide blocks
        // A/B build: NH_CAP_RDO = resident workgroups per CU (LDS reservation, lds_cap)
        static const int cap_rdo = NH_KNOB("NH_CAP_RDO", 0);
        // A/B build: NH_RDO_MMA = 0 the lane-per-mode packed chains, 3 / 4 the f16 MFMA mosaics at that many
        // waves per SIMD (k_intra_rdo8_mma)
        static const int rdo_mma = NH_KNOB("NH_RDO_MMA", kRdoMmaDefault);
        // the winners' rows as 16-B stores when every row start is 16-B aligned
        const int vec_out = NH_RDO_VEC_OUT && !(pitch & 7) && !((uintptr_t)d_lvl & 15) && !((uintptr_t)d_recon & 15);
#if NH_AB
        if (rdo_mma) {
            const int rcm = ensure_mosaic_cl();
            if (rcm) return rcm;
        }
        if (rdo_mma == 4)
            k_intra_rdo8_mma<3, 4><<<ngroups, 256, lds_cap(k_intra_rdo8_mma<3, 4>, cap_rdo), s>>>(
                d_src, w, h, pitch, q, dequant_scale(rem), per, d_modes, d_lvl, d_recon, sse);
        else if (rdo_mma == 5)
            k_intra_rdo8_mma<3, 2, true><<<ngroups, 256, lds_cap(k_intra_rdo8_mma<3, 2, true>, cap_rdo), s>>>(
                d_src, w, h, pitch, q, dequant_scale(rem), per, d_modes, d_lvl, d_recon, sse);
        else if (rdo_mma == 6)
            k_intra_rdo8_mma<6, 2, true><<<ngroups, 256, lds_cap(k_intra_rdo8_mma<6, 2, true>, cap_rdo), s>>>(
                d_src, w, h, pitch, q, dequant_scale(rem), per, d_modes, d_lvl, d_recon, sse);
        else if (rdo_mma)
            k_intra_rdo8_mma<3><<<ngroups, 256, lds_cap(k_intra_rdo8_mma<3>, cap_rdo), s>>>(
                d_src, w, h, pitch, q, dequant_scale(rem), per, d_modes, d_lvl, d_recon, sse);
        else
#else
        (void)rdo_mma;
#endif
        k_intra_rdo8<1, true, 1><<<ngroups, 256, lds_cap(k_intra_rdo8<1, true, 1>, cap_rdo), s>>>(
            d_src, w, h, pitch, q, dequant_scale(rem), per, d_modes, d_lvl, d_recon, sse, ngroups, vec_out,
            RdoPlanes{0, 0, 1});
        k_intra_rdo8<1, true, 2><<<ngroups, 256, 0, s>>>(d_src, w, h, pitch, q, dequant_scale(rem), per, d_modes, d_lvl,
                                                        d_recon, sse, ngroups, vec_out, RdoPlanes{0, 0, 1});
    }
    NH_HIP(hipGetLastError());
    return NH_OK;
}

// Config 3 over every plane of plane sets (include/nanohevc.h): one launch pair per set, plane z of the
// set in grid row z -- no launch per plane, and the sets' planes share the chip instead of each
// plane's last workgroups running alone.  Modes and SSE per plane in set order; levels / recon in
// the source layout.
extern "C" int nh_intra_rdo_planes(const int16_t* d_src, const nh_plane_set* sets, int nsets, int qp,
                                   uint8_t* d_modes, int32_t* d_lvl, int16_t* d_recon, int64_t* d_sse, void* stream) {
    if (!d_src || !sets || nsets < 0 || !d_modes || !d_lvl || !d_recon) return NH_EARG;
    for (int k = 0; k < nsets; ++k) {
        const nh_plane_set& S = sets[k];
        const int64_t planes = (int64_t)S.planes_per_group * S.num_groups;
        if (S.width < 0 || S.height < 0 || S.pitch < S.width || S.planes_per_group < 1 || S.num_groups < 0 ||
            planes > 65535 || S.base < 0 || S.plane_stride < 0 || S.group_stride < 0) {
            set_error("nh_intra_rdo_planes: bad plane set");
            return NH_EARG;
        }
    }
    int per, rem;
    qp_split(qp, &per, &rem);
    const hipStream_t s = as_stream(stream);
    const QuantParams q = qparams(qp, 3, true);
    static const int cap_rdo = NH_KNOB("NH_CAP_RDO", 0);
    int64_t moff = 0, soff = 0;
    for (int k = 0; k < nsets; ++k) {
        const nh_plane_set& S = sets[k];
        const int64_t planes = (int64_t)S.planes_per_group * S.num_groups;
        const int nblk = (S.width / 8) * (S.height / 8);
        if (nblk && planes) {
            const uint32_t ngroups = (uint32_t)((nblk + kRdoSlots - 1) / kRdoSlots);
            const int vec_out = NH_RDO_VEC_OUT && !(S.pitch & 7) && !((S.base | S.plane_stride | S.group_stride) & 7) &&
                                !((uintptr_t)d_lvl & 15) && !((uintptr_t)d_recon & 15);
            const RdoPlanes pg{S.group_stride, S.plane_stride, S.planes_per_group};
            unsigned long long* sse = d_sse ? (unsigned long long*)(d_sse + soff) : nullptr;
            const dim3 grid(ngroups, (unsigned)planes);
            k_intra_rdo8<1, true, 1><<<grid, 256, lds_cap(k_intra_rdo8<1, true, 1>, cap_rdo), s>>>(
                d_src + S.base, S.width, S.height, S.pitch, q, dequant_scale(rem), per, d_modes + moff, d_lvl + S.base,
                d_recon + S.base, sse, ngroups, vec_out, pg);
            k_intra_rdo8<1, true, 2><<<grid, 256, 0, s>>>(d_src + S.base, S.width, S.height, S.pitch, q,
                                                         dequant_scale(rem), per, d_modes + moff, d_lvl + S.base,
                                                         d_recon + S.base, sse, ngroups, vec_out, pg);
            NH_HIP(hipGetLastError());
        }
        moff += planes * nblk;
        soff += planes;
    }
    return NH_OK;
}

extern "C" int64_t nh_tu_workspace_bytes(int w, int h, int ctb) {
    (void)w; (void)h; (void)ctb;
    return 0;   // no scratch: TUs are found by per-size grid walks (k_tu_process kTree)
}

namespace nh {
// nh_ctu.hip: config 4 as one CTU-granular launch (NH_EVALUE: layout needs the per-size path)
int ctu_open_launch(const int16_t* src, void* lvl, int16_t* rec, uint8_t* tu, const nh_plane_set* set, int ctb,
                    int plane_id, uint32_t seed, int is_luma, int row0, int row1, const QuantParams* q, int dqs,
                    int dq_per, hipStream_t s, int lvl_bytes = 4, int32_t* spill = nullptr);
// nh_tc32.hip: config 4's 32x32 TUs on the int8 matrix cores
int tc32_mfma_tree(const int16_t* src, int w, int h, int pitch, const QuantParams& qp, int dq_scale, int dq_per,
                   int32_t* lvl, int16_t* rec, uint8_t* tu, int bw, int n, const TreeArgs& ta, unsigned planes,
                   hipStream_t s);
}  // namespace nh

extern "C" int nh_tu_pipeline_planes(const int16_t* d_src, const nh_plane_set* set, int ctb, int plane_id,
                                     uint32_t seed, int qp, int is_luma, int row0, int row1, int32_t* d_lvl,
                                     int16_t* d_recon, uint8_t* d_tu, void* stream) {
    if (!d_src || !set || !d_lvl || !d_recon || !d_tu) return NH_EARG;
    const int w = set->width, h = set->height, pitch = set->pitch;
    const int64_t planes = (int64_t)set->planes_per_group * set->num_groups;
    if (pitch < w || w <= 0 || h <= 0 || set->planes_per_group < 1 || planes < 0 || planes > 65535) return NH_EARG;
    if (ctb != 4 && ctb != 8 && ctb != 16 && ctb != 32) return NH_EVALUE;
    if ((w & 3) || (h & 3) || w > 65535 || h > 65535) return NH_EARG;
    if (!planes) return NH_OK;
    hipStream_t s = as_stream(stream);
    const int rows = (h + ctb - 1) / ctb;
    if (row0 < 0) row0 = 0;
    if (row1 > rows) row1 = rows;
    if (row1 <= row0) return NH_OK;
    int per, rem;
    qp_split(qp, &per, &rem);
    const int dqs = dequant_scale(rem);
    // One CTU-granular launch (k_ctu_open) unless the layout
    // rules out its vector accesses; A/B build: NH_CFG4_FORM=1 forces the
    // per-size launches below.
    static const int form = NH_KNOB("NH_CFG4_FORM", 0);
    if (form == 0) {
        QuantParams q4[4];
        for (int k = 0; k < 4; ++k) q4[k] = qparams(qp, k + 2, true);
        const int rc = ctu_open_launch(d_src, d_lvl, d_recon, d_tu, set, ctb, plane_id, seed, is_luma, row0, row1, q4,
                                       dqs, per, s);
        if (rc != NH_EVALUE) return rc;
    }
    const int yb = row0 * ctb, ye = row1 * ctb < h ? row1 * ctb : h;
    TreeArgs ta{ctb, plane_id, yb, seed};
    ta.ppg = set->planes_per_group;
    ta.group_stride = set->group_stride;
    ta.plane_stride = set->plane_stride;
    ta.tu_plane = (int64_t)(h / 4) * (w / 4);
    const int16_t* src = d_src + set->base;
    int32_t* lvl = d_lvl + set->base;
    int16_t* rec = d_recon + set->base;
#define NH_TU(NN, DST)                                                                                       \
    do {                                                                                                     \
        const int bw = w / NN, bh = (ye - yb + NN - 1) / NN, n = bw * bh;                                   \
        if (NN <= ctb && n > 0)                                                                              \
            k_tu_process<NN, DST, kTree><<<dim3((n + tu_cands_per_wg<NN, kTree>() - 1) / tu_cands_per_wg<NN, kTree>(), \
                                                (unsigned)planes), 256, 0, s>>>(                                 \
                src, w, h, pitch, qparams(qp, Log2<NN>::v, true), dqs, per, lvl, rec, d_tu, bw, n, ta);          \
    } while (0)
    if (is_luma) NH_TU(4, true); else NH_TU(4, false);
    NH_TU(8, false);
    NH_TU(16, false);
    // 32x32 TUs: int8 MFMA (the config-5 A/B winner) where the layout allows its
    // 16-B row accesses; NH_TU32_BUTTERFLY=1 forces the butterfly (A/B only)
    static const bool tu32_bf = NH_KNOB("NH_TU32_BUTTERFLY", 0) == 1;
    const bool mfma_ok = !tu32_bf && !(pitch & 7) && !((ta.group_stride | ta.plane_stride) & 7) &&
                         !(((uintptr_t)src | (uintptr_t)lvl | (uintptr_t)rec) & 15);
    if (ctb == 32 && mfma_ok) {
        const int bw = w / 32, bh = (ye - yb + 31) / 32, n = bw * bh;
        if (n > 0) {
            const int rc = tc32_mfma_tree(src, w, h, pitch, qparams(qp, 5, true), dqs, per, lvl, rec, d_tu, bw, n, ta,
                                          (unsigned)planes, s);
            if (rc) return rc;
        }
    } else {
        NH_TU(32, false);
    }
#undef NH_TU
    // (A/B: forking the four size launches onto side streams with events was
    // slower -- 0.066 -> 0.068-0.071 ms per frame batched, 0.157 -> 0.275 one
    // plane at a time: profiles/r01/cfg4/cfg4_streams_*.jsonl)
    NH_HIP(hipGetLastError());
    return NH_OK;
}

// Config 4 with COMPACT levels (include/nanohevc.h): the CTU-granular launch only.
extern "C" int nh_tu_pipeline_planes_compact(const int16_t* d_src, const nh_plane_set* set, int ctb, int plane_id,
                                             uint32_t seed, int qp, int is_luma, int row0, int row1, int16_t* d_lvl,
                                             int32_t* d_spill, int16_t* d_recon, uint8_t* d_tu, void* stream) {
    if (!d_src || !set || !d_lvl || !d_spill || !d_recon || !d_tu) return NH_EARG;
    const int w = set->width, h = set->height, pitch = set->pitch;
    const int64_t planes = (int64_t)set->planes_per_group * set->num_groups;
    if (pitch < w || w <= 0 || h <= 0 || set->planes_per_group < 1 || planes < 0 || planes > 65535) return NH_EARG;
    if ((w & 3) || (h & 3) || w > 65535 || h > 65535) return NH_EARG;
    if (ctb != 16 && ctb != 32) {
        set_error("tu_pipeline_planes_compact: CTB 16 or 32");
        return NH_EARG;
    }
    if ((pitch & 7) || ((set->base | set->plane_stride | set->group_stride) & 7) ||
        (((uintptr_t)d_lvl | (uintptr_t)d_spill) & 15) || (((uintptr_t)d_src | (uintptr_t)d_recon) & 7)) {
        set_error("tu_pipeline_planes_compact: 8-sample aligned pitch / base / strides, 16-B aligned level buffers");
        return NH_EARG;
    }
    if (!planes) return NH_OK;
    hipStream_t s = as_stream(stream);
    const int rows = (h + ctb - 1) / ctb;
    if (row0 < 0) row0 = 0;
    if (row1 > rows) row1 = rows;
    if (row1 <= row0) return NH_OK;
    int per, rem;
    qp_split(qp, &per, &rem);
    QuantParams q4[4];
    for (int k = 0; k < 4; ++k) q4[k] = qparams(qp, k + 2, true);
    const int rc = ctu_open_launch(d_src, d_lvl, d_recon, d_tu, set, ctb, plane_id, seed, is_luma, row0, row1, q4,
                                   dequant_scale(rem), per, s, 2, d_spill);
    if (rc == NH_EVALUE) {
        set_error("tu_pipeline_planes_compact: layout outside the CTU-granular launch's");
        return NH_EARG;
    }
    return rc;
}

// Config 4 compact levels -> the reference's int32 levels, rows [row0 * ctb, row1 * ctb): from the
// spill plane where the sample's strip (CTB rows x 1024 / CTB columns) holds the marker at its
// origin, else the int16 level widened.  4 samples per thread (w % 4 == 0).
__global__ void __launch_bounds__(256) k_tu_widen(const int16_t* __restrict__ lc, const int32_t* __restrict__ spill,
                                                  int32_t* __restrict__ out, int64_t base, int64_t group_stride,
                                                  int64_t plane_stride, int ppg, int w4, int y0, int ny, int pitch,
                                                  int ctb, int sw) {
    const int pz = blockIdx.y, gz = pz / ppg, cz = pz - gz * ppg;
    const int64_t poff = base + (int64_t)gz * group_stride + (int64_t)cz * plane_stride;
    const int64_t n = (int64_t)w4 * ny;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int yy = (int)(i / w4), x = 4 * (int)(i - (int64_t)yy * w4), y = y0 + yy;
        const int64_t o = poff + (int64_t)y * pitch + x;
        const bool sp = lc[poff + (int64_t)(y - y % ctb) * pitch + (x - x % sw)] == (int16_t)0x8000;
        int4 v;
        if (sp) {
            v = *(const int4*)(spill + o);
        } else {
            const uint2 q = *(const uint2*)(lc + o);
            v = make_int4((int16_t)(q.x & 0xffffu), (int16_t)(q.x >> 16), (int16_t)(q.y & 0xffffu), (int16_t)(q.y >> 16));
        }
        *(int4*)(out + o) = v;
    }
}

extern "C" int nh_tu_levels_widen(const int16_t* d_lvl, const int32_t* d_spill, const nh_plane_set* set, int ctb,
                                  int row0, int row1, int32_t* d_out, void* stream) {
    if (!d_lvl || !d_spill || !d_out || !set) return NH_EARG;
    const int w = set->width, h = set->height, pitch = set->pitch;
    const int64_t planes = (int64_t)set->planes_per_group * set->num_groups;
    if (pitch < w || w <= 0 || h <= 0 || set->planes_per_group < 1 || planes < 0 || planes > 65535 || (w & 3) ||
        (pitch & 3) || ((set->base | set->plane_stride | set->group_stride) & 3) || (ctb != 16 && ctb != 32) ||
        (((uintptr_t)d_spill | (uintptr_t)d_out) & 15) || ((uintptr_t)d_lvl & 7))
        return NH_EARG;
    const int rows = (h + ctb - 1) / ctb;
    if (row0 < 0) row0 = 0;
    if (row1 > rows) row1 = rows;
    if (row1 <= row0 || !planes) return NH_OK;
    const int y0 = row0 * ctb, ny = std::min(h, row1 * ctb) - y0;
    const int64_t items = (int64_t)(w / 4) * ny;
    const dim3 grid((unsigned)std::min<int64_t>((items + 255) / 256, 4096), (unsigned)planes);
    k_tu_widen<<<grid, 256, 0, as_stream(stream)>>>(d_lvl, d_spill, d_out, set->base, set->group_stride,
                                                   set->plane_stride, set->planes_per_group, w / 4, y0, ny, pitch, ctb,
                                                   1024 / ctb);
    NH_HIP(hipGetLastError());
    return NH_OK;
}

// Sets work[2] when any source sample of the plane set is outside [0, 255]
// (the closed-loop stream then takes the 32-bit chain; the single-group path --
// the pair kernel checks its own loads).  Rows grid-strided over blockIdx.x, a
// row's samples over the threads: no per-sample division.
__global__ void __launch_bounds__(256) k_closed_any_wide(const int16_t* __restrict__ src, int64_t group_stride,
                                                         int64_t plane_stride, int ppg, int w, int h, int pitch,
                                                         int32_t* flag) {
    const int pz = blockIdx.y, gz = pz / ppg, cz = pz - gz * ppg;
    const int16_t* p = src + (int64_t)gz * group_stride + (int64_t)cz * plane_stride;
    uint32_t bits = 0;
    for (int y = blockIdx.x; y < h; y += gridDim.x) {
        const int16_t* row = p + (int64_t)y * pitch;
        for (int x = threadIdx.x; x < w; x += 256) bits |= (uint16_t)row[x];
    }
    if (__ballot((bits & 0xff00u) != 0) && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
}

static int closed4_layout(const nh_plane_set* set, int ctb, int64_t& lines0, int64_t& lw, int64_t& nplanes) {
    if (!set || (ctb != 4 && ctb != 8 && ctb != 16 && ctb != 32)) return NH_EARG;
    if (set->width < 4 || set->height < 0 || set->pitch < set->width || set->planes_per_group < 1 ||
        set->num_groups < 0 || set->width > 65535 || set->height > 65535 || (set->width & 3) || (set->height & 3))
        return NH_EARG;
    nplanes = (int64_t)set->planes_per_group * set->num_groups;
    if (nplanes > 65535) return NH_EARG;
    lines0 = 4;   // ticket, status, wide flag, pad; then 64-bit words (8-B aligned)
    lw = (set->width + 1) / 2;
    return NH_OK;
}

// Workspace: [ticket, status, wide flag, pad | 64-bit line words of every plane |
// the TU schedules of k_closed4_plan: planes per group x CTUs x kPlanBytes].
static int64_t closed4_plan_offset(int64_t lines0, int64_t lw, int64_t np) { return 4 * lines0 + 8 * lw * np; }
static int64_t closed4_plan_bytes(const nh_plane_set* set, int ctb) {
    return (int64_t)set->planes_per_group * ((set->height + ctb - 1) / ctb) * ((set->width + ctb - 1) / ctb) *
           kPlanBytes;
}

#if NH_AB
static uint64_t* g_stamps = nullptr;
static int64_t g_stamps_n = 0, g_stamps_used = 0;
// A/B build only: the pair kernel's per-(ticket, CTU) stamps of the last closed-loop launch
// (NH_CLOSED4_STAMPS=1), 8 words each; returns the number of words copied.
extern "C" int64_t nh_ab_closed4_stamps(uint64_t* host, int64_t max_words) {
    if (!g_stamps || !host) return 0;
    const int64_t n = std::min(max_words, g_stamps_used);
    if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(host, g_stamps, n * 8, hipMemcpyDeviceToHost) != hipSuccess)
        return -1;
    return n;
}
#endif

extern "C" int64_t nh_tu_pipeline_closed_workspace_bytes(const nh_plane_set* set, int ctb) {
    int64_t lines0, lw, np;
    if (closed4_layout(set, ctb, lines0, lw, np)) return -1;
    return closed4_plan_offset(lines0, lw, np) + closed4_plan_bytes(set, ctb);
}

extern "C" int nh_tu_pipeline_planes_closed(const int16_t* d_src, const nh_plane_set* set, int ctb, int plane_id,
                                            uint32_t seed, int qp, int is_luma, int32_t* d_lvl, int16_t* d_recon,
                                            uint8_t* d_tu, void* d_work, void* stream) {
    if (!d_src || !d_lvl || !d_recon || !d_tu || !d_work) return NH_EARG;
    int64_t lines0, lw, np;
    if (closed4_layout(set, ctb, lines0, lw, np)) {
        set_error("nh_tu_pipeline_planes_closed: bad plane set (w, h multiples of 4) or CTB size");
        return NH_EARG;
    }
    if ((uintptr_t)d_work & 7) {
        set_error("nh_tu_pipeline_planes_closed: workspace must be 8-byte aligned");
        return NH_EARG;
    }
    hipStream_t s = as_stream(stream);
    NH_HIP(hipMemsetAsync(d_work, 0, closed4_plan_offset(lines0, lw, np), s));   // not the schedules
    if (!np || !set->height) return NH_OK;
    Closed4Args a{};
    a.src = d_src + set->base;
    a.lvl = d_lvl + set->base;
    a.rec = d_recon + set->base;
    a.tu = d_tu;
    a.work = (int32_t*)d_work;
    a.lines0 = lines0;
    a.group_stride = set->group_stride;
    a.plane_stride = set->plane_stride;
    a.tu_plane = (int64_t)(set->height / 4) * (set->width / 4);
    a.w = set->width;
    a.h = set->height;
    a.pitch = set->pitch;
    a.ctb = ctb;
    a.plane_id = plane_id;
    a.ppg = set->planes_per_group;
    a.nplanes = (int32_t)np;
    a.crows = (set->height + ctb - 1) / ctb;
    a.ccols = (set->width + ctb - 1) / ctb;
    a.lw = (int32_t)lw;
    a.is_luma = is_luma ? 1 : 0;
    a.seed = seed;
    for (int k = 0; k < 4; ++k) a.q[k] = qparams(qp, k + 2, true);
    int per, rem;
    qp_split(qp, &per, &rem);
    a.dqs = dequant_scale(rem);
    a.dq_per = per;
    a.probe = NH_KNOB("NH_CLOSED4_PROBE", 0);
#if NH_AB   // A/B timing stamps of the pair kernel: nh_ab_closed4_stamps() copies the last launch's out
    if (NH_KNOB("NH_CLOSED4_STAMPS", 0)) {
        const int64_t need = (int64_t)a.crows * ((set->num_groups + 1) / 2) * set->planes_per_group * a.ccols * kStampWords;
        if (need > g_stamps_n) {
            if (g_stamps) (void)hipFree(g_stamps);
            NH_HIP(hipMalloc(&g_stamps, need * 8));
            g_stamps_n = need;
        }
        NH_HIP(hipMemsetAsync(g_stamps, 0, need * 8, s));
        a.stamps = g_stamps;
        g_stamps_used = need;
    }
#endif
    // 32x32 luma TUs on the f16 matrix cores (closed_chain32_tf): 16-B level and recon row pieces;
    // A/B build: NH_CLOSED4_MFMA32 = 0 keeps them on the packed butterfly chain
    static const int mfma32 = NH_KNOB("NH_CLOSED4_MFMA32", 1);
    a.mfma32 = mfma32 && ctb == 32 && !(set->pitch & 7) && !((set->base | set->plane_stride | set->group_stride) & 7) &&
               !((uintptr_t)d_lvl & 15) && !((uintptr_t)d_recon & 15);
    // packed-chain recon of whole CTUs as 64-B rows from the LDS reconstruction (8-B aligned row pieces);
    // A/B knob NH_CLOSED4_REC_CTU = 0: every TU stores its own 8-B row pieces
    static const int rec_ctu = NH_KNOB("NH_CLOSED4_REC_CTU", 1);
    a.rec_ctu = rec_ctu && !(set->pitch & 3) && !((set->base | set->plane_stride | set->group_stride) & 3) &&
                !((uintptr_t)d_recon & 7);
    // the pair kernel's LDS-DMA source tile: 16-B pieces of whole rows (width, pitch, offsets multiples of
    // 8 samples, so no piece straddles a row's end) and 32-bit byte offsets within a group of planes;
    // A/B knob NH_CLOSED4_SRCTILE = 0: the chains load their samples from global memory
    static const int srctile = NH_KNOB("NH_CLOSED4_SRCTILE", 1);
    a.srctile = srctile && !(set->width & 7) && !(set->pitch & 7) &&
                !((set->base | set->plane_stride | set->group_stride) & 7) && !((uintptr_t)d_src & 15) &&
                (3 * set->group_stride + (int64_t)set->height * set->pitch) * 2 < (1ll << 31);
    {   // tu_closed_batch_mma's per-lane bases and initial accumulators
        const int rcm = ensure_mosaic_cl();
        if (rcm) return rcm;
    }
    if (a.mfma32) {
        static PerDeviceOnce once;
        const int rcb = once.run([] {
            const BasisHC bh = make_basis_hc();
            NH_HIP(hipMemcpyToSymbol(HIP_SYMBOL(c_basis_hc_cl), &bh, sizeof(bh)));
            return (int)NH_OK;
        });
        if (rcb) return rcb;
    }
    const int64_t rows = (int64_t)a.crows * np;
    // the CTU-end flush pays when many waves share each SIMD (64 frames concurrent: 0.0964 vs 0.1027
    // ms per 4K frame); with fewer its stores' latency shows (16 frames: luma 0.240 vs 0.233 ms)
    if (rows < 4096) a.rec_ctu = 0;
    // persistent waves: every row covered, capped at what can be resident (1,024 SIMDs x 2 waves/SIMD)
    const int64_t cap = 2048;
    const unsigned waves = (unsigned)(rows < cap ? rows : cap);
    // the stream's wide flag, then the packed-chain form (codes the stream iff no
    // sample is outside [0, 255]) and the 32-bit form (iff one is); A/B knob
    // NH_TU_CLOSED_NARROW = 0: the 32-bit form for every stream
    static const int narrow_ok = NH_KNOB("NH_TU_CLOSED_NARROW", 1);
    static const int pair_ok = NH_KNOB("NH_TU_CLOSED_PAIR", 1);
    const bool pair = narrow_ok != 0 && pair_ok != 0 && set->num_groups > 1;
    if (pair) {
        // the pair kernel checks the samples it loads itself (k_tu_closed_pair: work[2] starts at 0)
    } else if (narrow_ok) {
        const unsigned gx = (unsigned)std::max(1, std::min(256, set->height));
        k_closed_any_wide<<<dim3(gx, (unsigned)np), 256, 0, s>>>(d_src + set->base, set->group_stride, set->plane_stride,
                                                              set->planes_per_group, set->width, set->height,
                                                              set->pitch, (int32_t*)d_work + 2);
    } else {
        NH_HIP(hipMemsetAsync((int32_t*)d_work + 2, 0xff, 4, s));
    }
    int cus = 0;
    NH_TRY(device_cus(&cus));
    // 8-bit streams: plane pairs (k_tu_closed_pair) when the set
    // holds more than one group; A/B build: NH_TU_CLOSED_PAIR = 0 codes one plane per wave
    if (pair) {
        int per_cu = 0;
        // CTB 32 (luma): plane pairs; CTB <= 16 (chroma): NH_CLOSED4_NPL16 planes per wave (4: the
        // chroma wavefront needs half the waves, so with luma's it fits the resident slots)
        void (*kern)(Closed4Args) =
            ctb == 32 ? (a.rec_ctu ? k_tu_closed_pair<kPairWaves, true, 32, 2> : k_tu_closed_pair<kPairWaves, false, 32, 2>)
                      : (a.rec_ctu ? k_tu_closed_pair<kPairWaves16, true, 16, NH_CLOSED4_NPL16>
                                   : k_tu_closed_pair<kPairWaves16, false, 16, NH_CLOSED4_NPL16>);
        const int npl = ctb == 32 ? 2 : NH_CLOSED4_NPL16;
        NH_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 64, 0));
        const int64_t prow = (int64_t)a.crows * ((set->num_groups + npl - 1) / npl) * set->planes_per_group;
        if (NH_CLOSED4_PLAN) {   // the TU schedule of every (plane of the group, CTU), once per launch
            uint8_t* plan = (uint8_t*)d_work + closed4_plan_offset(lines0, lw, np);
            a.plan = plan;
            k_closed4_plan<<<dim3((unsigned)(a.crows * a.ccols), (unsigned)a.ppg), 64, 0, s>>>(a, plan);
            NH_HIP(hipGetLastError());
        }
        // A/B build: resident waves per CU, for both sets or per luma / chroma set
        static const int wpc = NH_KNOB("NH_CLOSED4_WPC", 0), wpc_l = NH_KNOB("NH_CLOSED4_WPC_L", 0),
                         wpc_c = NH_KNOB("NH_CLOSED4_WPC_C", 0);
        const int wsel = is_luma ? (wpc_l > 0 ? wpc_l : wpc) : (wpc_c > 0 ? wpc_c : wpc);
#ifdef NH_CLOSED4_PERCU_CAP   // variant builds: resident waves per CU capped at compile time
        per_cu = std::min(per_cu, NH_CLOSED4_PERCU_CAP);
#endif
        const int64_t cap_n = (int64_t)(wsel > 0 ? wsel : std::max(1, per_cu)) * cus;
        kern<<<(unsigned)(prow < cap_n ? prow : cap_n), 64, 0, s>>>(a);
    } else if (narrow_ok) {
        int per_cu = 0;
        NH_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_tu_closed<1, true>, 64, 0));
        const int64_t cap_n = (int64_t)std::max(1, per_cu) * cus;
        k_tu_closed<1, true><<<(unsigned)(rows < cap_n ? rows : cap_n), 64, 0, s>>>(a);
    }
    k_tu_closed<1><<<waves, 64, 0, s>>>(a);
    NH_HIP(hipGetLastError());
    return NH_OK;
}

extern "C" int nh_tu_pipeline_plane(const int16_t* d_src, int w, int h, int pitch, int ctb, int plane_id,
                                    uint32_t seed, int qp, int is_luma, int row0, int row1, int32_t* d_lvl,
                                    int16_t* d_recon, uint8_t* d_tu, void* d_work, void* stream) {
    (void)d_work;
    nh_plane_set one{0, 0, 0, w, h, pitch, 1, 1, 0};
    return nh_tu_pipeline_planes(d_src, &one, ctb, plane_id, seed, qp, is_luma, row0, row1, d_lvl, d_recon, d_tu,
                                 stream);
}

static int closed_layout(const nh_plane_set* sets, int nsets, ClosedArgs& a, int64_t& modes_total) {
    if (!sets || nsets < 1 || nsets > NH_MAX_PLANE_SETS) return NH_EARG;
    int64_t rows = 0, planes = 0, modes = 0, lines = 0;
    a.max_bh = 0;
    for (int k = 0; k < nsets; ++k) {
        const nh_plane_set& p = sets[k];
        if (p.width < 8 || p.height < 0 || p.pitch < p.width || p.planes_per_group < 1 || p.num_groups < 0 ||
            p.width > 65535 || p.height > 65535)
            return NH_EARG;
        ClosedSet& S = a.set[k];
        S.base = p.base;
        S.plane_stride = p.plane_stride;
        S.group_stride = p.group_stride;
        S.w = p.width;
        S.h = p.height;
        S.pitch = p.pitch;
        S.ppg = p.planes_per_group;
        S.bw = p.width / 8;
        S.bh = p.height / 8;
        S.row0 = (int32_t)rows;
        S.plane0 = (int32_t)planes;
        S.mode0 = modes;
        S.lw = (p.width + 1) / 2 + 16;   // int16 pairs + slack for the top-right read past the edge
        S.line0 = lines;
        const int64_t np = (int64_t)p.planes_per_group * p.num_groups;
        S.np = (int32_t)np;
        if (S.bh > a.max_bh) a.max_bh = S.bh;
        rows += np * S.bh;
        planes += np;
        modes += np * S.bw * S.bh;
        lines += np * S.lw;
        if (rows >= (1ll << 30)) return NH_EARG;
    }
    a.nsets = nsets;
    a.total_rows = (int32_t)rows;
    a.lines0 = (2 + rows + 2) & ~1ll;   // 8-B aligned: the tagged form's 64-bit line words; word 2 + rows:
                                        // the stream's wide flag (k_closed_any_wide)
    a.lines_total = lines;
    modes_total = modes;
    return NH_OK;
}

extern "C" int64_t nh_intra_rdo_closed_workspace_bytes(const nh_plane_set* sets, int nsets) {
    ClosedArgs a;
    int64_t m = 0;
    if (closed_layout(sets, nsets, a, m)) return -1;
    return 4ll * a.lines0 + 8ll * a.lines_total;   // 64-bit line words (the int32 form uses half)
}

extern "C" int nh_intra_rdo_planes_closed(const int16_t* d_src, const nh_plane_set* sets, int nsets, int qp,
                                          uint8_t* d_modes, int32_t* d_lvl, int16_t* d_recon, int64_t* d_sse,
                                          void* d_work, void* stream) {
    if (!d_src || !d_modes || !d_lvl || !d_recon || !d_sse || !d_work) {
        set_error("nh_intra_rdo_planes_closed: null argument");
        return NH_EARG;
    }
    ClosedArgs a;
    int64_t modes_total = 0;
    if (closed_layout(sets, nsets, a, modes_total)) {
        set_error("nh_intra_rdo_planes_closed: bad plane sets (width >= 8, pitch >= width)");
        return NH_EARG;
    }
    int per, rem;
    qp_split(qp, &per, &rem);
    a.src = d_src;
    a.lvl = d_lvl;
    a.rec = d_recon;
    a.modes = d_modes;
    a.sse = d_sse;
    a.work = (int32_t*)d_work;
    a.qp = qparams(qp, 3, true);
    a.prio_set = 0;
    for (int k = 1; k < a.nsets; ++k)
        if (a.set[k].bw + 2 * a.set[k].bh > a.set[a.prio_set].bw + 2 * a.set[a.prio_set].bh) a.prio_set = k;
    a.dq_scale = dequant_scale(rem);
    a.dq_per = per;
    hipStream_t s = as_stream(stream);
    if ((uintptr_t)d_work & 7) {
        set_error("nh_intra_rdo_planes_closed: workspace must be 8-byte aligned");
        return NH_EARG;
    }
    NH_HIP(hipMemsetAsync(d_work, 0, 4ull * a.lines0 + 8ull * a.lines_total, s));
    for (int k = 0; k < nsets; ++k) {
        const int np = sets[k].planes_per_group * sets[k].num_groups;
        if (np > 0 && np <= 65535) k_zero_partial<<<dim3(64, np), 256, 0, s>>>(d_recon, a.set[k], np);
        else if (np > 65535) return NH_EARG;
    }
    if (a.total_rows > 0) {
        // persistent waves: enough to cover every row, capped at what can be resident (2 waves/SIMD)
        const int waves = a.total_rows < 2048 ? a.total_rows : 2048;
        {   // A/B knobs: NH_CLOSED_ORDER=0 plane-major tickets; NH_CLOSED_PROBE timing probes
            static const int co = NH_KNOB("NH_CLOSED_ORDER", 1);
            a.order = co ? 1 : 0;
            a.probe = NH_KNOB("NH_CLOSED_PROBE", 0);
            {
                // the stream's wide flag, then the packed-only form (codes the stream iff every source
                // sample is 8-bit: every neighbour is then too, the reconstruction being clipped) and the
                // both-chains form (codes it otherwise)
                int32_t* flag = (int32_t*)d_work + 2 + a.total_rows;
                for (int k = 0; k < nsets; ++k) {
                    const nh_plane_set& p = sets[k];
                    const int64_t np = (int64_t)p.planes_per_group * p.num_groups, n = (int64_t)p.width * p.height;
                    if (np <= 0 || n <= 0) continue;
                    const unsigned gx = (unsigned)std::min<int64_t>(256, (n + 255 * 8) / (256 * 8));
                    k_closed_any_wide<<<dim3(gx, (unsigned)np), 256, 0, s>>>(d_src + p.base, p.group_stride,
                                                                          p.plane_stride, p.planes_per_group, p.width,
                                                                          p.height, p.pitch, flag);
                }
                int cus = 0, per_cu = 0;
                NH_TRY(device_cus(&cus));
                NH_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_intra_rdo8_closed_tag<1, kClosedNarrow>,
                                                                    64, 0));
                const int64_t cap_n = (int64_t)std::max(1, per_cu) * cus;
                k_intra_rdo8_closed_tag<1, kClosedNarrow>
                    <<<(unsigned)(a.total_rows < cap_n ? a.total_rows : cap_n), 64, 0, s>>>(a);
                k_intra_rdo8_closed_tag<1, kClosedWide><<<waves, 64, 0, s>>>(a);
            }
        }
    }
    NH_HIP(hipGetLastError());
    return NH_OK;
}

// The status word lands in a pinned host slot: a direct DMA, not the staged copy of a pageable
// destination (the call sits inside every timed closed-loop launch set).  One process-wide pinned
// page of kStatusSlots slots, allocated once and kept for the process (a per-thread
// allocation was never freed); a call holds one slot for its copy + synchronize; when every slot is
// held by a concurrent call it copies into pageable memory instead (same result, slower).
namespace {
constexpr int kStatusSlots = 64;
std::mutex g_status_mu;
int32_t* g_status_page = nullptr;
uint64_t g_status_used = 0;
int status_slot_acquire() {
    std::lock_guard<std::mutex> lk(g_status_mu);
    if (!g_status_page && hipHostMalloc((void**)&g_status_page, kStatusSlots * 64, hipHostMallocDefault) != hipSuccess) {
        g_status_page = nullptr;
        return -1;
    }
    if (g_status_used == ~0ull) return -1;
    const int k = __builtin_ctzll(~g_status_used);
    g_status_used |= 1ull << k;
    return k;
}
void status_slot_release(int k) {
    std::lock_guard<std::mutex> lk(g_status_mu);
    g_status_used &= ~(1ull << k);
}
}  // namespace

extern "C" int nh_intra_rdo_closed_status(const void* d_work, int* status, void* stream) {
    if (!d_work || !status) return NH_EARG;
    hipStream_t s = as_stream(stream);
    const int k = status_slot_acquire();
    if (k < 0) {   // no free pinned slot: a pageable copy (hipMemcpyAsync then synchronizes the stream)
        int32_t v = 0;
        NH_HIP(hipMemcpyAsync(&v, (const int32_t*)d_work + 1, 4, hipMemcpyDeviceToHost, s));
        NH_HIP(hipStreamSynchronize(s));
        *status = v;
        return NH_OK;
    }
    int32_t* pinned = g_status_page + 16 * k;   // 64-B slots
    hipError_t e = hipMemcpyAsync(pinned, (const int32_t*)d_work + 1, 4, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e == hipSuccess) *status = *(volatile int32_t*)pinned;
    status_slot_release(k);
    NH_HIP(e);
    return NH_OK;
}

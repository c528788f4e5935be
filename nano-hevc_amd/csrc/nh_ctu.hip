// nh_ctu.hip -- config 4 open loop as ONE CTU-granular
// launch per plane set: every TU size of every CTU in a single kernel.
//
// Reference composition (the same chain as k_tu_process, nh_intraloop.hip):
//   open-loop DC-vs-planar choice by residual energy (__main__.py:165-178,
//   DC on ties), neighbours from the SOURCE plane (block.py:38-50, 128 outside),
//   residual (intra.py:65-67) -> forward_transform (transform.py:154-196; DST
//   for 4x4 luma, :138-141) -> quantize_block -> dequantize_block (quant.py:
//   126-150) -> inverse_transform (transform.py:199-238) -> reconstruct + clip
//   (intra.py:70-78).  TU quadtree: the seeded split hash (nh_tree.hpp).
//
// Layout of the work.  One wave owns a STRIP of 1024 samples: CTB rows x
// 1024/CTB columns (one 32x32 luma CTU, four 16x16 chroma CTUs side by side,
// ...), i.e. 64 4x4 units, one per lane; a workgroup codes a GROUP of 4 strips.
// Each wave
//   1. issues the loads of its strip, the row above it and the column left of
//      it, classifies its units while they are in flight (lane u descends the
//      quadtree to its unit's leaf, <= 3 hashes, and writes the TU map), then
//      stores the strip image in LDS (every TU neighbour is an LDS read);
//   2. the TU origins of the 4 strips are pooled into per-size LDS lists;
//   3. the waves claim batches of 64/N TUs of one size (lane l: column / row
//      l mod N of TU l / N), 32x32 TUs first.
// Two kernels per plane set: k_ctu_open codes the groups whose samples are all
// 8-bit with the packed 16-bit chain (nh_packed.hpp) and their
// 32x32 TUs on exact f16 matrix cores (§4.4d); the groups it marks in the TU
// map k_ctu_wide codes with the 32-bit chain (any int16 input).  No global
// atomics, no per-size relaunch, the source read once.  Levels and recon rows
// are stored straight from the registers.
// Exactness of the 24-bit multiplies and the 32-bit quantizer: DESIGN.md §4.3,
// §4.4 (the residual is int16).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <mutex>
#include <type_traits>
#include "nh_common.hpp"
#include "nh_internal.hpp"
#include "nh_mfma.hpp"
#include "nh_f16mma.hpp"
#include "nh_ldsdma.hpp"
#define NH_MOSAIC_TABLE c_mosaic_ctu
#include "nh_mosaic.hpp"
// The open-loop CTU kernels keep the builtin's v_dot2c seeding (pdot_first,
// nh_packed.hpp): the VOP3P form measured 1.3 % slower here (0.0390 vs 0.0385
// ms per 4K frame, profiles/r03/cfg4/ab_libs_4b_pd.jsonl) and 2-4 % faster in
// the closed loop (nh_intraloop.hip).
#ifndef NH_PDOT_FIRST
#define NH_PDOT_FIRST 0
#endif
#include "nh_packed.hpp"
#include "nh_tree.hpp"

namespace nh {

__constant__ Basis c_basis_ctu;

__constant__ BasisH c_basis_h;
__constant__ BasisHC c_basis_hc;   // chain32_tf's crow-permuted bases (config 5)

struct CtuArgs {
    const int16_t* src;
    int32_t* lvl;
    int16_t* rec;
    uint8_t* tu;
    int64_t group_stride, plane_stride, tu_plane;
    int32_t w, h, pitch, ppg, plane_id;
    int32_t row0, nrows, strips_x;   // CTU rows [row0, row0 + nrows) of the band; strips per CTU row
    uint32_t seed;
    QuantParams q[4];                // log2 N = 2..5
    int32_t dqs, dq_per;
    int32_t wide_only;               // A/B build only (NH_CTU_NARROW=0): every workgroup on the 32-bit chain
    int32_t probe;                   // A/B build only (NH_CTU_PROBE, bits): 1 = no batches, 2 = no global loads,
                                     // 4 = return at once, 8 = no TU-map stores (wrong outputs)
    uint32_t* wide_flag;             // config 5: set to `epoch` when a block is left to the int8 fix-up
    uint32_t epoch;
    int32_t* spill;                  // config 4 compact levels: k_ctu_wide's int32 levels (null: int32 levels)
    int16_t* lvl_c;                  // config 4 compact levels: the int16 level plane (k_ctu_wide's strip markers)
    const uint8_t* plan;             // config 4: the groups' TU plans (k_ctu_plan; null: classified in the kernel)
    uint8_t* plan_w;                 // k_ctu_plan's output (the same buffer)
    int32_t ngroups;                 // groups of the band (records per plane id)
};

__device__ __forceinline__ void wave_sync() { __builtin_amdgcn_wave_barrier(); }

// Level and recon rows out of the chains: plain stores.  Nontemporal ones (the
// rows are never re-read here) took 127 vs 39 us per 4K YUV420 frame: 8-16 B
// pieces of scattered rows (profiles/r02/session5/nt_ab.jsonl).
__device__ __forceinline__ void st_lvl4(int32_t* p, int4 v) { *(int4*)p = v; }
// 4 consecutive levels in the level type LT: one 16-B (int32) or 8-B (int16, compact) store
__device__ __forceinline__ void st_lvl4t(int32_t* p, const int32_t (&L)[4]) { st_lvl4(p, make_int4(L[0], L[1], L[2], L[3])); }
__device__ __forceinline__ void st_lvl4t(int16_t* p, const int32_t (&L)[4]) {
    *(uint2*)p = make_uint2(((uint32_t)L[0] & 0xffffu) | ((uint32_t)L[1] << 16), ((uint32_t)L[2] & 0xffffu) | ((uint32_t)L[3] << 16));
}
// Config 4 compact levels: the marker k_ctu_wide leaves at the origin of every strip it codes (its
// int32 levels are in the spill plane); an 8-bit TU's level never takes it (|level| <= 408,
// tools/packed_bounds.py level_bounds)
constexpr int16_t kCtuSpillMark = (int16_t)0x8000;
__device__ __forceinline__ void st_rec4(int16_t* p, uint2 v) { *(uint2*)p = v; }

// The lane id.  With NH_OPAQUE_LANE (A/B builds) it is opaque to the compiler
// (an empty asm), so lane-derived addresses and constants of a chain are
// recomputed inside each batch instead of hoisted out of the batch loop: 76
// instead of 129 VGPRs for the luma kernel.  Since the kernels are capped at 3-4
// resident waves per SIMD (lds_cap) the registers are free, and hoisting saves
// VALU: 37.2 vs 38.1 us per 4K YUV420 frame, config 5 0.129 vs 0.138 ms per 8K
// frame.
__device__ __forceinline__ int opaque_lane() {
    int l = threadIdx.x & 63;
#ifdef NH_OPAQUE_LANE
    asm volatile("" : "+v"(l));
#endif
    return l;
}

__device__ __forceinline__ int32_t sext16(int32_t v) { return (int16_t)(uint16_t)(uint32_t)v; }

// 64-bit energy of an int16-wrapped difference pair: each square <= 2^30, so
// the pair sums exactly in 32 bits before the 64-bit add.
__device__ __forceinline__ uint64_t sq2(int32_t a, int32_t b) {
    return (uint64_t)((uint32_t)__mul24(a, a) + (uint32_t)__mul24(b, b));
}

// Strip geometry: STRIP_W = 1024 / CTB columns x CTB rows; LDS image rows of
// IP int16 (sample (y, x) at [1 + y][4 + x]: 8-B aligned rows; row 0 = the row
// above the strip, column 3 = the column left of it), coefficient tile rows of
// CP int32 (odd pitch: the row pass reads conflict-free).
template <int CTB> struct Strip {
    static constexpr int SW = 1024 / CTB, UW = SW / 4, IP = SW + 8, CP = SW + 1;
    static constexpr int IMG = (CTB + 1) * IP, CF = CTB * CP;
    // narrow workgroups: an int16 tile aliasing the int32 one, rows of TP int16
    // (an odd number of dwords: the pair reads of a row pass are conflict-free)
    static constexpr int TP = SW + 2;
    // (CTB 32: room for chain32_tf's level tile, 32 rows of 36 int32 -- round 5 -- which also
    // holds ctu_chain32_h's f16 transpose tile, 32 rows of QH = 40 halves)
    static constexpr int QH = 40, T16 = CTB == 32 ? 32 * 72 : CTB * TP;
    static_assert((TP / 2) % 2 == 1 && (CTB == 32 || T16 * 2 <= CF * 4) && 32 * QH <= 32 * 72, "int16 tile layout");
};

// One batch of 64/N TUs of size N from the workgroup's size-N list: lane l
// codes column / row t = l % N of TU j = l / N.  A list entry is
// strip << 6 | unit; each lane works in its TU's strip image / tile.
template <int N, bool DST, int CTB>
__device__ __forceinline__ void ctu_chain(const CtuArgs& a, int16_t* s_img, int32_t* s_cf, const uint16_t* list,
                                          int cnt, int b0, const int* s_org, int32_t* __restrict__ lvl,
                                          int16_t* __restrict__ rec) {
    using G = Strip<CTB>;
    constexpr int L2 = Log2<N>::v, S = L2 + 5, IP = G::IP, CP = G::CP;
    const ChainQ cq = make_chainq(a.q[L2 - 2], a.dqs, a.dq_per);
    const int lane = opaque_lane(), j = lane / N, t = lane % N;
    const bool on = b0 + j < cnt;
    const int e = list[on ? b0 + j : b0], sw = e >> 6, u = e & 63;   // idle lanes shadow the batch's first TU
    const int lx = 4 * (u % G::UW), ly = 4 * (u / G::UW);
    const int16_t* img = s_img + sw * G::IMG + ly * IP + 4 + lx;   // img[r * IP + c]: sample (ly + r - 1, lx + c)
    int32_t* cf = s_cf + sw * G::CF + ly * CP + lx;                // cf[r * CP + c]:  (ly + r, lx + c)
    const int gx0 = s_org[2 * sw] + lx, gy0 = s_org[2 * sw + 1] + ly;
    int32_t o[N];
#pragma unroll
    for (int i = 0; i < N; ++i) o[i] = img[(1 + i) * IP + t];
    const int32_t topt = img[t];                  // top[t]   (block.py:38-43)
    const int32_t leftt = img[(1 + t) * IP - 1];  // left[t]  (block.py:45-50)
    const int32_t tr = img[N - 1];                // top[-1]  (__main__.py:168)
    const int32_t bl = img[N * IP - 1];           // left[-1]
    // DC (intra.py:46-62): sum over the TU's N lanes
    int32_t sum = topt + leftt;
    sum = grp_sum<N>(sum);
    const int32_t dc = (sum + N) >> (L2 + 1);
    // planar (intra.py:81-113) for column t: num(i) = (N-1-t) left[i] + (t+1) tr + (N-1-i) top[t] + (i+1) bl + N
    int32_t pl[N];
    {
        int32_t base = (t + 1) * tr + (N - 1) * topt + bl + N;
        const int32_t step = bl - topt;
#pragma unroll
        for (int i = 0; i < N; ++i) {
            pl[i] = ((N - 1 - t) * (int32_t)img[(1 + i) * IP - 1] + base) >> (L2 + 1);
            base += step;
        }
    }
    uint64_t ed = 0, ep = 0;
#pragma unroll
    for (int i = 0; i < N; i += 2) {
        ed += sq2(sext16(o[i] - dc), sext16(o[i + 1] - dc));
        ep += sq2(sext16(o[i] - pl[i]), sext16(o[i + 1] - pl[i + 1]));
    }
    ed = grp_sum<N>(ed);
    ep = grp_sum<N>(ep);
    const bool use_dc = ed <= ep;   // __main__.py:173: DC wins ties
    uint32_t v[N], r[N];
    // forward pass 1 (transform.py:179-185) on column t of the residual
#pragma unroll
    for (int k = 0; k < N; ++k) v[k] = (uint32_t)sext16(o[k] - (use_dc ? dc : pl[k]));
    fwd1d<N, DST, Mul24>(v, r);
    if (on) {
#pragma unroll
        for (int i = 0; i < N; ++i) cf[i * CP + t] = rshift_round<S>(r[i]);
    }
    wave_sync();
    // forward pass 2 (transform.py:188-194) on row t, quantize_block, levels out, dequantize_block
#pragma unroll
    for (int k = 0; k < N; ++k) v[k] = (uint32_t)cf[t * CP + k];
    fwd1d<N, DST, Mul24>(v, r);
    if (on) {
        int32_t* lrow = lvl + (int64_t)(gy0 + t) * a.pitch + gx0;
#pragma unroll
        for (int k0 = 0; k0 < N; k0 += 4) {
            int32_t L4[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                L4[q] = quant_s(rshift_round<S>(r[k0 + q]), cq.qs, cq.h_v, cq.hneg_v);
                cf[t * CP + k0 + q] = dequant_s(L4[q], cq);
            }
            st_lvl4(lrow + k0, make_int4(L4[0], L4[1], L4[2], L4[3]));
        }
    }
    wave_sync();
    // inverse pass 1 (transform.py:221-227) on column t
#pragma unroll
    for (int k = 0; k < N; ++k) v[k] = (uint32_t)cf[k * CP + t];
    inv1d<N, DST, Mul24>(v, r);
    if (on) {
#pragma unroll
        for (int i = 0; i < N; ++i) cf[i * CP + t] = rshift_round<S>(r[i]);
    }
    wave_sync();
    // inverse pass 2 (transform.py:230-236) on row t, reconstruct + clip (intra.py:70-78), recon out
#pragma unroll
    for (int k = 0; k < N; ++k) v[k] = (uint32_t)cf[t * CP + k];
    inv1d<N, DST, Mul24>(v, r);
    if (on) {
        // planar in row layout: num(k) = (N-1-k) left[t] + (k+1) tr + (N-1-t) top[k] + (t+1) bl + N
        int32_t base = (N - 1) * leftt + tr + (t + 1) * bl + N;
        const int32_t step = tr - leftt;
        uint32_t pk[N / 2];
#pragma unroll
        for (int k = 0; k < N; k += 2) {
            int32_t q2[2];
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int32_t p = use_dc ? dc : ((N - 1 - t) * (int32_t)img[k + q] + base) >> (L2 + 1);
                base += step;
                const int32_t x = sext16(p + sext16(rshift_round<S>(r[k + q])));
                q2[q] = x < 0 ? 0 : (x > 255 ? 255 : x);
            }
            pk[k / 2] = (uint32_t)q2[0] | ((uint32_t)q2[1] << 16);
        }
        int16_t* rrow = rec + (int64_t)(gy0 + t) * a.pitch + gx0;
#pragma unroll
        for (int k = 0; k < N / 2; k += 2) st_rec4(rrow + 2 * k, make_uint2(pk[k], pk[k + 1]));
    }
}

// The same chain for a NARROW workgroup (every sample of its strips and their
// neighbours in [0, 255]): int16 pairs end to end.  Source
// column, planar prediction (v_pk_mad_u16: numerators < 2^15) and residual as
// row pairs, residual energies with v_dot2 in 32 bits (<= N^2 * 255^2), the
// transforms of nh_packed.hpp, and an int16 coefficient tile: each pass stores
// its outputs with 16-bit writes at the slots the next pass reads as pairs --
// natural order into the forward row pass, inv_slot order (line = column) into
// both inverse passes, so no pass permutes.  Same results as ctu_chain for
// such TUs (bounds: tools/packed_bounds.py).
// OST: levels and recon go to the group's LDS output images (olvl / orec: strip
// sw's rows of SW at sw * CTB * SW), written out in whole rows after the
// group's batches (strip_writeout).
template <int N, bool DST, int CTB, bool OST = false, class LT = int32_t>
__device__ __forceinline__ void ctu_chain_pk(const CtuArgs& a, const int16_t* s_img, int16_t* s_t16, const uint16_t* list,
                                             int cnt, int b0, const int* s_org, LT* __restrict__ lvl,
                                             int16_t* __restrict__ rec, LT* olvl = nullptr,
                                             int16_t* orec = nullptr) {
    using G = Strip<CTB>;
    constexpr int L2 = Log2<N>::v, S = L2 + 5, IP = G::IP, TP = G::TP, H = N / 2;
    constexpr int32_t BIAS = 1 << (S - 1);
    const ChainQ cq = make_chainq(a.q[L2 - 2], a.dqs, a.dq_per);
    const int lane = opaque_lane(), j = lane / N, t = lane % N;
    const bool on = b0 + j < cnt;
    const int e = list[on ? b0 + j : b0], sw = e >> 6, u = e & 63;   // idle lanes shadow the batch's first TU
    const int lx = 4 * (u % G::UW), ly = 4 * (u / G::UW);
    const int16_t* img = s_img + sw * G::IMG + ly * IP + 4 + lx;   // img[r * IP + c]: sample (ly + r - 1, lx + c)
    int16_t* tl = s_t16 + sw * G::T16 + ly * TP + lx;              // tl[line * TP + slot]
    const int gx0 = s_org[2 * sw] + lx, gy0 = s_org[2 * sw + 1] + ly;
    const int32_t topt = img[t];                  // top[t]   (block.py:38-43)
    const int32_t leftt = img[(1 + t) * IP - 1];  // left[t]  (block.py:45-50)
    const int32_t tr = img[N - 1];                // top[-1]  (__main__.py:168)
    const int32_t bl = img[N * IP - 1];           // left[-1]
    int32_t sum = topt + leftt;                   // DC (intra.py:46-62)
    sum = grp_sum<N>(sum);
    const int32_t dc = (sum + N) >> (L2 + 1);
    const pk16 dc2 = pk_splat(dc);
    // column t: source rows (2m, 2m+1) and planar (intra.py:81-113)
    // num(i) = (N-1-t) left[i] + [(t+1) tr + (N-1-i) top[t] + (i+1) bl + N]
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
            o2[m] = pk_pair(img[(1 + 2 * m) * IP + t], img[(2 + 2 * m) * IP + t]);
            const pku16 lf = {(unsigned short)img[(1 + 2 * m) * IP - 1], (unsigned short)img[(2 + 2 * m) * IP - 1]};
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
    // forward pass 1 (transform.py:179-185), column t -> line i, slot t
    int32_t y[N];
    fwd1d_pk<N, DST>(r2, y, BIAS);
    if (on) {
#pragma unroll
        for (int i = 0; i < N; ++i) tl[i * TP + t] = (int16_t)(y[i] >> S);
    }
    wave_sync();
    // forward pass 2 (transform.py:188-194), row t; quantize_block, levels out, dequantize_block
    // -> line k (column), slot inv_slot(t)
    const int st = inv_slot<N, DST>(t);
    {
        pk16 P[H];
#pragma unroll
        for (int m = 0; m < H; ++m) P[m] = *(const pk16*)&tl[t * TP + 2 * m];
        fwd1d_pk<N, DST>(P, y, BIAS);
    }
    if (on) {
        LT* lrow = OST ? olvl + sw * (CTB * G::SW) + (ly + t) * G::SW + lx : lvl + (int64_t)(gy0 + t) * a.pitch + gx0;
#pragma unroll
        for (int k0 = 0; k0 < N; k0 += 4) {
            int32_t L4[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                L4[q] = quant_s(y[k0 + q] >> S, cq.qs, cq.h_v, cq.hneg_v);
                tl[(k0 + q) * TP + st] = (int16_t)dequant_s(L4[q], cq);
            }
            st_lvl4t(lrow + k0, L4);
        }
    }
    wave_sync();
    // inverse pass 1 (transform.py:221-227), column t -> line i (row), slot inv_slot(t)
    int32_t x[N];
    {
        pk16 Y[H];
#pragma unroll
        for (int m = 0; m < H; ++m) Y[m] = *(const pk16*)&tl[t * TP + 2 * m];
        inv1d_pk<N, DST>(Y, x, BIAS);
    }
    if (on) {
#pragma unroll
        for (int i = 0; i < N; ++i) tl[i * TP + st] = (int16_t)(x[i] >> S);
    }
    wave_sync();
    // inverse pass 2 (transform.py:230-236), row t; reconstruct + clip (intra.py:70-78), recon out
    {
        pk16 Y[H];
#pragma unroll
        for (int m = 0; m < H; ++m) Y[m] = *(const pk16*)&tl[t * TP + 2 * m];
        inv1d_pk<N, DST>(Y, x, BIAS);
    }
    if (on) {
        // planar in row layout: num(k) = (N-1-t) top[k] + [(N-1-k) left[t] + (k+1) tr + (t+1) bl + N]
        const int32_t b = (N - 1) * leftt + tr + (t + 1) * bl + N, st2v = tr - leftt;
        pku16 bs = {(unsigned short)b, (unsigned short)(b + st2v)};
        const pku16 stp = {(unsigned short)(2 * st2v), (unsigned short)(2 * st2v)};
        const pku16 wt = {(unsigned short)(N - 1 - t), (unsigned short)(N - 1 - t)};
        const pku16 sh = {(unsigned short)(L2 + 1), (unsigned short)(L2 + 1)};
        const pk16 zero = {0, 0}, maxv = {255, 255};
        uint32_t pk[H];
#pragma unroll
        for (int m = 0; m < H; ++m) {
            const pku16 tp = __builtin_bit_cast(pku16, *(const pk16*)&img[2 * m]);
            const pk16 pred = use_dc ? dc2 : __builtin_bit_cast(pk16, (pku16)((tp * wt + bs) >> sh));
            bs += stp;
            const pk16 rc = pred + pk_pair(x[2 * m] >> S, x[2 * m + 1] >> S);
            pk[m] = __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_elementwise_max(rc, zero), maxv));
        }
        int16_t* rrow = OST ? orec + sw * (CTB * G::SW) + (ly + t) * G::SW + lx : rec + (int64_t)(gy0 + t) * a.pitch + gx0;
#pragma unroll
        for (int m = 0; m < H; m += 2) st_rec4(rrow + 2 * m, make_uint2(pk[m], pk[m + 1]));
    }
}

// The same batch on MFMA mosaics (round 5, nh_mosaic.hpp): the
// closed loop's chain with the strip image as its source and neighbours (open
// loop: every neighbour is a source sample).  OST: levels / recon into the LDS
// output images (whole-row stores after the group); otherwise one sample per lane
// and store straight to memory.  NM = N / 4 mosaics hold the batch's 64 / N TUs.
template <int N, bool DST, int CTB, bool OST, class LT = int32_t>
__device__ __forceinline__ void ctu_batch_mma(const CtuArgs& a, const int16_t* s_img, const uint16_t* list, int cnt,
                                              int b0, const int* s_org, LT* __restrict__ lvl,
                                              int16_t* __restrict__ rec, LT* olvl, int16_t* orec) {
    using G = Strip<CTB>;
    constexpr int IP = G::IP, NM = N / 4;
    using MC = MosaicCore<N, DST, NM>;
    const ChainQ cq = make_chainq(a.q[MC::L2 - 2], a.dqs, a.dq_per);
    MC mc;
    mc.lane_init(opaque_lane());
    const int16_t* pm[NM];   // pm[m][(1 + y) * IP + x]: sample (y, x) of the lane's TU; x = -1: left, y = -1: top
    int swm[NM], lxm[NM], lym[NM];
    bool onm[NM];
    int32_t sv[NM][4];
#pragma unroll
    for (int m = 0; m < NM; ++m) {
        const int e = b0 + m * MC::TPM + mc.el;
        onm[m] = e < cnt;
        const int en = list[onm[m] ? e : b0], sw = en >> 6, u = en & 63;   // idle lanes shadow the batch's first TU
        swm[m] = sw;
        lxm[m] = 4 * (u % G::UW);
        lym[m] = 4 * (u / G::UW);
        pm[m] = s_img + sw * G::IMG + lym[m] * IP + 4 + lxm[m];
#pragma unroll
        for (int r = 0; r < 4; ++r) sv[m][r] = pm[m][(1 + mc.yr0 + r) * IP + mc.t];
    }
    struct Nb {
        const int16_t* p[NM];   // (copies: a reference to the array kept it in memory)
        int t;
        __device__ int32_t top(int m) const { return p[m][t]; }
        __device__ int32_t tr(int m) const { return p[m][N - 1]; }
        __device__ int32_t bl(int m) const { return p[m][N * IP - 1]; }
        __device__ int32_t dcl(int m) const { return p[m][(1 + t) * IP - 1]; }
        __device__ pku16 left2(int m, int y) const {
            return (pku16){(unsigned short)p[m][(1 + y) * IP - 1], (unsigned short)p[m][(2 + y) * IP - 1]};
        }
    };
    Nb nb;
#pragma unroll
    for (int m = 0; m < NM; ++m) nb.p[m] = pm[m];
    nb.t = mc.t;
    mc.predict(sv, nb);
    mc.pass1();
    mc.pass2();
    mc.ready();
    auto out_row = [&](int m, int q) { return lym[m] + mc.yr0 + 2 * q; };   // strip-local row of the pair
    mc.quant(cq, [&](int m, int q, int32_t L0, int32_t L1) {
        if (!onm[m]) return;
        if constexpr (OST) {
            LT* o = olvl + swm[m] * (CTB * G::SW) + out_row(m, q) * G::SW + lxm[m] + mc.t;
            o[0] = (LT)L0;
            o[G::SW] = (LT)L1;
        } else {
            LT* o = lvl + (int64_t)(s_org[2 * swm[m] + 1] + out_row(m, q)) * a.pitch + s_org[2 * swm[m]] + lxm[m] + mc.t;
            o[0] = (LT)L0;
            o[a.pitch] = (LT)L1;
        }
    });
    mc.inv1();
    mc.inv2();
    mc.recon([&](int m, int q, pku16 rv) {
        if (!onm[m]) return;
        if constexpr (OST) {
            int16_t* o = orec + swm[m] * (CTB * G::SW) + out_row(m, q) * G::SW + lxm[m] + mc.t;
            o[0] = (int16_t)rv.x;
            o[G::SW] = (int16_t)rv.y;
        } else {
            int16_t* o = rec + (int64_t)(s_org[2 * swm[m] + 1] + out_row(m, q)) * a.pitch + s_org[2 * swm[m]] + lxm[m] + mc.t;
            o[0] = (int16_t)rv.x;
            o[a.pitch] = (int16_t)rv.y;
        }
    });
}

// A 32x32 TU (a whole CTU of a CTB-32 strip) on the int8 matrix cores: the
// chain of k_tc32_mfma (nh_tc32.hip) with the block, its
// neighbours and the dequantized tile in the strip's LDS image / tile.
__device__ __forceinline__ void ctu_chain32(const CtuArgs& a, const int16_t* img, int32_t* cf, int gx0, int gy0,
                                            int32_t* __restrict__ lvl, int16_t* __restrict__ rec) {
    constexpr int IP = Strip<32>::IP, CP = Strip<32>::CP;   // img[r * IP + c]: sample (r - 1, c), c = -1: left; cf[r * CP + c]
    const ChainQ cq = make_chainq(a.q[3], a.dqs, a.dq_per);
    const int l = opaque_lane(), r = l & 31, hh = l >> 5;
    const int32_t my_nb = hh == 0 ? img[r] : img[(1 + r) * IP - 1];
    int32_t s = my_nb;
    s = grp_sum<64>(s);
    const int32_t dc = (s + 32) >> 6;
    const int32_t tr = img[31], bl = img[32 * IP - 1];
    auto planar = [&](int y, int x) -> int32_t {
        return ((31 - x) * (int32_t)img[(1 + y) * IP - 1] + (x + 1) * tr + (31 - y) * (int32_t)img[x] + (y + 1) * bl +
                32) >> 6;
    };
    uint64_t e_dc = 0, e_pl = 0;
#pragma unroll
    for (int jj = 0; jj < 16; jj += 2) {
        const int k = 16 * hh + jj;
        const int32_t o0 = img[(1 + k) * IP + r], o1 = img[(2 + k) * IP + r];
        e_dc += sq2(sext16(o0 - dc), sext16(o1 - dc));
        e_pl += sq2(sext16(o0 - planar(k, r)), sext16(o1 - planar(k + 1, r)));
    }
    e_dc = grp_sum<64>(e_dc);
    e_pl = grp_sum<64>(e_pl);
    const bool use_dc = e_dc <= e_pl;   // DC wins ties (__main__.py:173)
    int32_t X[16];
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) {
        const int k = 16 * hh + jj;
        X[jj] = sext16((int32_t)img[(1 + k) * IP + r] - (use_dc ? dc : planar(k, r)));
    }
    const v4i_t F1 = load_row16(&c_basis_ctu.t[r][0], 16 * hh);
    v16i_t acc = mfma_auto<true>(X, F1);
    int32_t V[16];
#pragma unroll
    for (int g = 0; g < 16; ++g) V[g] = rshift_round<10>((uint32_t)acc[g]);   // transform.py:185
    const v4i_t F2 = load_perm16(&c_basis_ctu.t[r][0], hh);
    acc = mfma_auto<false>(V, F2);
    int32_t* lrow = lvl + (int64_t)(gy0 + r) * a.pitch + gx0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        int32_t L4[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int g = 4 * q + e;
            L4[e] = quant_s(rshift_round<10>((uint32_t)acc[g]), cq.qs, cq.h_v, cq.hneg_v);
            cf[r * CP + crow(g, hh)] = dequant_s(L4[e], cq);
        }
        st_lvl4(lrow + 8 * q + 4 * hh, make_int4(L4[0], L4[1], L4[2], L4[3]));
    }
    wave_sync();
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) X[jj] = cf[(16 * hh + jj) * CP + r];
    const v4i_t F3 = load_row16(&c_basis_ctu.tt[r][0], 16 * hh);
    acc = mfma_auto<true>(X, F3);
#pragma unroll
    for (int g = 0; g < 16; ++g) V[g] = rshift_round<10>((uint32_t)acc[g]);   // transform.py:227
    const v4i_t F4 = load_perm16(&c_basis_ctu.tt[r][0], hh);
    acc = mfma_auto<false>(V, F4);
    int16_t* rrow = rec + (int64_t)(gy0 + r) * a.pitch + gx0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        int32_t R4[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int g = 4 * q + e, jx = crow(g, hh);
            const int32_t rr = sext16(rshift_round<10>((uint32_t)acc[g]));
            const int32_t rc = sext16((use_dc ? dc : planar(r, jx)) + rr);
            R4[e] = rc < 0 ? 0 : (rc > 255 ? 255 : rc);
        }
        st_rec4(rrow + 8 * q + 4 * hh,
                make_uint2((uint32_t)R4[0] | ((uint32_t)R4[1] << 16), (uint32_t)R4[2] | ((uint32_t)R4[3] << 16)));
    }
}

// A 32x32 TU of a NARROW group on the f16 matrix cores: one
// TU per wave, the four transform passes as v_mfma_f32_32x32x16_f16 pairs.
// Exact: every operand is an integer of at most 11 bits (residual + 1536 for
// pass 1, pass outputs <= 510, dequantized <= 180, inverse pass-1 outputs
// <= 327) against the basis scaled by 2^-10, every product is exact in fp32
// and every partial sum is a multiple of 2^-10 below 2^14 (tools/
// packed_bounds.py: at most 6,813,696 * 2^-10), so the fp32 accumulators hold
// the reference's integer sums exactly; the accumulators start at 0 (an
// inline constant: no registers hold an initial value) and the rounding
// constant 0.5 (transform.py:185) -- for pass 1 also minus the 1536 offset of
// row 0 -- is added before floor(), the arithmetic shift (still exact: the
// sums stay below 2^23 * 2^-10).  Lane (r, hh): pass 1 and inverse pass 1 take the data as the A
// operand (lane = the free index), passes 2 and 4 take the previous
// accumulator as the B operand in accumulator row order (the bases
// pre-permuted to match), and one LDS transpose sits after dequantization.
// Same results as ctu_chain / ctu_chain_pk on these TUs.
// The bases live in LDS (one copy per workgroup, copy_basis_h): as global loads
// every operand load after a store would wait for the wave's outstanding stores
// (vmcnt counts both on gfx9), draining each chain's level stores.
__device__ __forceinline__ void copy_basis_h(BasisH& dst) {
    const uint4* s4 = (const uint4*)&c_basis_h;
    uint4* d4 = (uint4*)&dst;
    constexpr int n = (int)(sizeof(BasisH) / 16);
    for (int i = threadIdx.x; i < n; i += blockDim.x) d4[i] = s4[i];
}
__device__ __forceinline__ void copy_basis_hc(BasisHC& dst) {
    const uint4* s4 = (const uint4*)&c_basis_hc;
    uint4* d4 = (uint4*)&dst;
    constexpr int n = (int)(sizeof(BasisHC) / 16);
    for (int i = threadIdx.x; i < n; i += blockDim.x) d4[i] = s4[i];
}
// TSTORE: the level and recon rows leave through an LDS tile `ot` (per wave,
// kOutP int32 per row) so that every global store instruction writes whole
// rows -- 8 rows of 128 B (levels), 16 rows of 64 B (recon) -- instead of 32-B
// / 16-B pieces of 32 rows.
constexpr int kOutP = 36, kRecP = 24;   // int32 per row: level tile, recon tile (48 halves; 16-B rows)
// The block image a chain reads: sample (y, x) for y, x in [0, 32), the row
// above (top, y = -1) and the column to the left (left, x = -1).  ImgStrip: a
// CTB-32 strip image (img[r * IP + c] = sample (r - 1, c), c = -1 the left
// column); ImgDma: the LDS-DMA image of k_tc32_hd (the block body in 64-B rows,
// the top row and left column side by side in a 64-sample edge array).
// Config 4 open loop: narrow 32x32 luma TUs on the transposition-free chain (chain32_tf, round 5);
// 0: round 4's ctu_chain32_h (LDS transpose after dequantization, bases in LDS)
#ifndef NH_CTU_TF32
#define NH_CTU_TF32 1
#endif
// Config 4 open loop, narrow 4..16 TUs on MFMA mosaics (ctu_batch_mma): 1 = the groups with LDS output
// images (chroma), 2 = every group (luma's outputs then leave one sample per lane and store)
#ifndef NH_CTU_MOSAIC
#define NH_CTU_MOSAIC 1
#endif
struct ImgStrip {
    const int16_t* p;
    static constexpr int IP = Strip<32>::IP;
    __device__ __forceinline__ int32_t at(int y, int x) const { return p[(1 + y) * IP + x]; }
    __device__ __forceinline__ int32_t top(int x) const { return p[x]; }
    __device__ __forceinline__ int32_t left(int y) const { return p[(1 + y) * IP - 1]; }
    // chain32_tf's reads (see ImgDma): rows of IP samples, 8-B aligned (sample (y, 0) at [1 + y][4])
    static constexpr int RS = IP;
    __device__ __forceinline__ const int16_t* trp(int L) const {
        return p + (1 + 4 * (L >> 5) + ((L >> 2) & 3)) * IP + 16 * ((L >> 4) & 1) + 4 * (L & 3);
    }
    __device__ __forceinline__ pku16 left2(int y) const {   // (left[y], left[y + 1])
        return (pku16){(unsigned short)left(y), (unsigned short)left(y + 1)};
    }
};
struct ImgDma {
    const int16_t* body;   // [y][x], 32 x 32
    const int16_t* edge;   // [0, 32): top[x]; [32, 96): left[y] at 32 + 2y (the 16-bit LDS-DMA writes a dword per lane)
    __device__ __forceinline__ int32_t at(int y, int x) const { return body[y * 32 + x]; }
    __device__ __forceinline__ int32_t top(int x) const { return edge[x]; }
    __device__ __forceinline__ int32_t left(int y) const { return edge[32 + 2 * y]; }
    // column x from row y0 on (element stride RS) and the left column from row y0 on (stride LS):
    // constant row offsets then sit in the LDS instructions' immediate offsets
    static constexpr int RS = 32, LS = 2;
    __device__ __forceinline__ const int16_t* colp(int x, int y0) const { return body + y0 * 32 + x; }
    __device__ __forceinline__ const int16_t* leftp(int y0) const { return edge + 32 + 2 * y0; }
    // ds_read_b64_tr_b16 (T10): lane L receives rows 8t + 4hh .. +3 of column L & 31 (hh = L >> 5)
    // as two (row, row + 1) pairs; lane 4q + p of each 16-lane group addresses row q, columns 4p..4p+3
    // of its group's 16 columns.  EXEC must be all ones.
    __device__ __forceinline__ const int16_t* trp(int L) const {
        return body + (4 * (L >> 5) + ((L >> 2) & 3)) * 32 + 16 * ((L >> 4) & 1) + 4 * (L & 3);
    }
    // (left[y], left[y + 1]) for even y: one dword each, read as one pair
    __device__ __forceinline__ pku16 left2(int y) const {
        const uint2 lw = *(const uint2*)(edge + 32 + 2 * y);
        return __builtin_bit_cast(pku16, __builtin_amdgcn_perm(lw.y, lw.x, 0x05040100u));
    }
};
template <bool TSTORE = false, class B = BasisH, class IMG = ImgStrip>
__device__ __forceinline__ void ctu_chain32_h(const CtuArgs& a, const IMG& img, uint16_t* qt, const B& bs,
                                              int gx0, int gy0,
                                              int32_t* __restrict__ lvl, int16_t* __restrict__ rec,
                                              int32_t* ot = nullptr, int64_t opitch = -1) {
    const int64_t op = opitch >= 0 ? opitch : (int64_t)a.pitch;   // row pitch of lvl / rec (an LDS image's: OST)
    constexpr int QH = Strip<32>::QH;
    const ChainQ cq = make_chainq(a.q[3], a.dqs, a.dq_per);
    const int l = opaque_lane(), r = l & 31, hh = l >> 5;
    const int32_t topr = img.top(r), leftr = img.left(r), tr = img.top(31), bl = img.left(31);
    int32_t sdc = hh ? leftr : topr;   // DC (intra.py:46-62): lane halves hold top / left
    sdc = grp_sum<64>(sdc);
    const int32_t dc = (sdc + 32) >> 6;
    const pk16 dc2 = pk_splat(dc);
    // column x = r, rows y = 8hh + 16c + j (the pass-1 A operand), as row pairs p = 4c + q
    pk16 o2[8];
    pku16 pl2[8];
    {
        const pku16 wl = {(unsigned short)(31 - r), (unsigned short)(31 - r)}, sh = {6, 6};
#pragma unroll
        for (int p = 0; p < 8; ++p) {
            const int y = 8 * hh + 16 * (p >> 2) + 2 * (p & 3);
            o2[p] = pk_pair(img.at(y, r), img.at(y + 1, r));
            const int32_t b = (r + 1) * tr + (31 - y) * topr + (y + 1) * bl + 32;   // planar, intra.py:81-113
            const pku16 bs = {(unsigned short)b, (unsigned short)(b + bl - topr)};
            const pku16 lf = {(unsigned short)img.left(y), (unsigned short)img.left(y + 1)};
            pl2[p] = (lf * wl + bs) >> sh;
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
    // residual (intra.py:65-67) + 1536 as f16 bits: 0x6600 + n for |n| < 512
    uint32_t hx[8];
#pragma unroll
    for (int p = 0; p < 8; ++p) {
        const pk16 rr = o2[p] - (use_dc ? dc2 : __builtin_bit_cast(pk16, pl2[p]));
        hx[p] = __builtin_bit_cast(uint32_t, __builtin_bit_cast(pku16, rr) + (pku16){0x6600, 0x6600});
    }
    // pass 1 (transform.py:179-185): D1[x][k] = tmp[k][x]; the 1536 offset removed with the rounding bias
    // b1 (row 0 only: every other DCT32 row sums to 0)
    const float b1 = r == 0 ? 0.5f - 3072.0f : 0.5f;
    f16x_t acc = splat16(initb(b1));
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(h8_t, make_uint4(hx[0], hx[1], hx[2], hx[3])),
                                                 bq_t(bs, r, hh, 0), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(h8_t, make_uint4(hx[4], hx[5], hx[6], hx[7])),
                                                 bq_t(bs, r, hh, 1), acc, 0, 0, 0);
    // pass 2 (transform.py:188-194): D2[l][k] = C[k][l], lane k, registers l = crow(g, hh)
    f16x_t acc2 = splat16(initb(0.5f));
    acc2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(bq_tc(bs, r, hh, 0), acc_h8(acc, 0, b1), acc2, 0, 0, 0);
    acc2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(bq_tc(bs, r, hh, 1), acc_h8(acc, 1, b1), acc2, 0, 0, 0);
    mfma_result_ready(acc2);   // before shift_rnd's inline-asm reads
    // quantize_block -> levels (row k = r), dequantize_block -> f16 into the transpose tile qt[l][k]
    int32_t* lrow = lvl + (int64_t)(gy0 + r) * op + gx0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        int32_t L4[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int g = 4 * q + e;
            L4[e] = quant_s(shift_rnd(acc2[g]), cq.qs, cq.h_v, cq.hneg_v);
            qt[crow(g, hh) * QH + r] = __builtin_bit_cast(uint16_t, (_Float16)(int16_t)dequant_s(L4[e], cq));
        }
        if constexpr (TSTORE) *(int4*)&ot[r * kOutP + 8 * q + 4 * hh] = make_int4(L4[0], L4[1], L4[2], L4[3]);
        else st_lvl4(lrow + 8 * q + 4 * hh, make_int4(L4[0], L4[1], L4[2], L4[3]));
    }
    wave_sync();
    if constexpr (TSTORE) {   // 4 instructions of 8 whole 128-B level rows
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int rr = (l >> 3) + 8 * i, c = 4 * (l & 7);
            st_lvl4(lvl + (int64_t)(gy0 + rr) * op + gx0 + c, *(const int4*)&ot[rr * kOutP + c]);
        }
        wave_sync();   // the tile's reads before the recon tile reuses it
    }
    // inverse pass 1 (transform.py:221-227): D3[l][y] = tmp[y][l], data lane l
    f16x_t acc3 = splat16(initb(0.5f));
    acc3 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ld_h8(qt + r * QH + 8 * hh), bq_tt(bs, r, hh, 0), acc3,
                                                  0, 0, 0);
    acc3 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ld_h8(qt + r * QH + 16 + 8 * hh),
                                                  bq_tt(bs, r, hh, 1), acc3, 0, 0, 0);
    // inverse pass 2 (transform.py:230-236): D4[x][y] = R[y][x], lane y, registers x = crow(g, hh)
    f16x_t acc4 = splat16(initb(0.5f));
    acc4 = __builtin_amdgcn_mfma_f32_32x32x16_f16(bq_ttc(bs, r, hh, 0), acc_h8(acc3, 0, 0.5f), acc4, 0, 0, 0);
    acc4 = __builtin_amdgcn_mfma_f32_32x32x16_f16(bq_ttc(bs, r, hh, 1), acc_h8(acc3, 1, 0.5f), acc4, 0, 0, 0);
    mfma_result_ready(acc4);
    // reconstruct + clip (intra.py:70-78), row y = r
    int16_t* rrow = rec + (int64_t)(gy0 + r) * op + gx0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        int32_t R4[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int x = 8 * q + 4 * hh + e;
            const int32_t p = use_dc ? dc
                                     : ((31 - x) * leftr + (x + 1) * tr + (31 - r) * img.top(x) + (r + 1) * bl + 32) >> 6;
            const int32_t v = p + shift_rnd(acc4[4 * q + e]);
            R4[e] = v < 0 ? 0 : (v > 255 ? 255 : v);
        }
        const uint2 pk = make_uint2((uint32_t)R4[0] | ((uint32_t)R4[1] << 16), (uint32_t)R4[2] | ((uint32_t)R4[3] << 16));
        if constexpr (TSTORE) *(uint2*)&ot[r * kRecP + 4 * q + 2 * hh] = pk;
        else st_rec4(rrow + 8 * q + 4 * hh, pk);
    }
    if constexpr (TSTORE) {   // 2 instructions of 16 whole 64-B recon rows
        wave_sync();
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int rr = (l >> 2) + 16 * i, c = 4 * (l & 3);
            *(uint4*)(rec + (int64_t)(gy0 + rr) * op + gx0 + 2 * c) = *(const uint4*)&ot[rr * kRecP + c];
        }
    }
}

// A 32x32 block of an 8-bit stream on the f16 matrix cores WITHOUT a transpose
// (round 5, config 5): every one of the four passes takes the previous pass's
// output as its A operand straight from the accumulator registers -- each MFMA
// output has its column index in the lanes and its row index in the registers,
// the row index is the next pass's contraction index, and the bases are stored
// crow-permuted (BasisHC) to match.  The data then walks
//   X[n][x] (lane x) -> tmp[k][x] (lane k) -> C[k][l] (lane l) -> tmp'[y][l]
//   (lane y) -> R[y][x] (lane x),
// ending in the input's own layout, so the reconstruction adds the prediction
// pairs kept from the residual stage.
//
// Between passes floor(acc + 0.5) (the arithmetic shift of transform.py:185)
// becomes an f16 operand in ONE v_cvt_pkrtz_f16_f32 per pair: the accumulators
// start at 0.5 (an inline constant), the value is moved into the binade [1024,
// 2048) -- where f16 holds every integer and nothing between -- by adding 1536,
// and there, all values being positive, rounding toward zero IS the floor.
// Every operand is then 1536 + v, and the offsets are exact integers the next
// pass turns into known constants:
//  * the residual enters as the f16 of n + 768 (bits 0x6200 + 2n, |n| <= 255);
//    DCT row 0 sums it to tmp[0][x] + 1536 (every other row sums to 0), so row
//    k = 0's lanes add 0 instead of 1536 (kTfAdd1);
//  * pass 2 of 1536 + tmp1 leaves +3072 on column l = 0 (row sums again): the
//    quantizer of lanes l = 0 compares and rounds against it (QuantTf);
//  * the dequantized coefficients enter as 1536 + d (the fma's bias), and the
//    inverse passes leave 1.5 * S on their outputs, S[y] = sum_k T[k][y] (a
//    column sum, even): lane y adds 1536 - 1.5 S[y] before converting, lane x
//    subtracts 1.5 S[x] from its prediction pairs at the reconstruction.
// Every pass's operands are integers <= 2046 against the basis * 2^-10, so each
// product is exact in fp32 and every partial sum a multiple of 2^-10 below 2^13:
// the accumulators hold the reference's integer sums exactly.
constexpr int kRecH = 2 * kRecP;   // recon tile row pitch in int16
// LT: the level element type in HBM.  int32_t is the reference's dtype; int16_t /
// int8_t are exact for 8-bit blocks (|level| <= 51 at every QP for N = 32:
// tools/packed_bounds.py level_bounds, tests/test_range_proofs.py) and cut the
// level rows to 4 / 2 store instructions of 16 / 32 whole rows (config 5's compact
// levels; the wide blocks' int32 levels go to a spill plane).
template <class LT> struct LvlTile {
    static_assert(sizeof(LT) == 1 || sizeof(LT) == 2 || sizeof(LT) == 4, "level type");
    // tile row pitch in LT elements (16-B aligned rows): int32 kOutP, int16 the recon tile's, int8 48 B
    static constexpr int P = sizeof(LT) == 4 ? kOutP : sizeof(LT) == 2 ? kRecH : 48;
    static constexpr int STORES = (int)sizeof(LT);   // level-row store instructions: 4 / 2 / 1
};
// NT: nontemporal level / recon stores (A/B form)
template <class IMG, class LT = int32_t, bool NT = false>
__device__ __forceinline__ void chain32_tf(const CtuArgs& a, const IMG& img, const BasisHC& bs, int gx0, int gy0,
                                           LT* __restrict__ lvl, int16_t* __restrict__ rec, int32_t* ot,
                                           const ChainQ& cq, const TfLane& tl) {
    const int64_t op = a.pitch;
    const int l = opaque_lane(), r = l & 31, hh = l >> 5;
    const int32_t topr = img.top(r), tr = img.top(31), bl = img.left(31);
    int32_t sdc = hh ? img.left(r) : topr;   // DC (intra.py:46-62): lane halves hold top / left
    sdc = grp_sum<64>(sdc);
    const int32_t dc = (sdc + 32) >> 6;
    const pk16 dc2 = pk_splat(dc);
    // column x = r, row pairs (y_p, y_p + 1), y_p = crow(2p, hh) = c_p + 4 hh: the pass-1 A operand in
    // register order.  Planar (intra.py:81-113) at (y, r): (31 - r) left[y] + b(y) >> 6 with
    // b(y) = (r + 1) tr + (31 - y) top[r] + (y + 1) bl + 32 = b(4 hh) + (y - 4 hh) (bl - top[r]).
    pk16 o2[8];
    pku16 pl2[8];
    {
        typedef short v4s __attribute__((ext_vector_type(4)));
        typedef __attribute__((address_space(3))) v4s lds_v4s;
        lds_v4s* tp = (lds_v4s*)(lds_void_t*)img.trp(l);
#pragma unroll
        for (int t = 0; t < 4; ++t) {   // rows 8t + 4hh .. +3 of column r: o2[2t], o2[2t + 1]
            const v4s v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(tp + 2 * IMG::RS * t);
            o2[2 * t] = (pk16){v[0], v[1]};
            o2[2 * t + 1] = (pk16){v[2], v[3]};
        }
        const pku16 wl = {(unsigned short)(31 - r), (unsigned short)(31 - r)}, sh = {6, 6};
        const int32_t d = bl - topr, b0 = (r + 1) * tr + (31 - 4 * hh) * topr + (4 * hh + 1) * bl + 32;
        const pku16 d2 = {(unsigned short)d, (unsigned short)d}, bb0 = {(unsigned short)b0, (unsigned short)(b0 + d)};
#pragma unroll
        for (int p = 0; p < 8; ++p) {
            const int c = 2 * (p & 1) + 8 * (p >> 1);   // y_p - 4 hh
            const pku16 lf = img.left2(4 * hh + c);   // (left[y_p], left[y_p + 1])
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
    pku16 pr2[8];                   // 0x6600 (the f16 bits of 1536) - the chosen prediction
    uint32_t hx[8];
#pragma unroll
    for (int p = 0; p < 8; ++p) {
        const pk16 pr = use_dc ? dc2 : __builtin_bit_cast(pk16, pl2[p]);
        const pku16 rr = __builtin_bit_cast(pku16, o2[p] - pr);   // residual, intra.py:65-67
        hx[p] = __builtin_bit_cast(uint32_t, rr * (pku16){2, 2} + (pku16){0x6200, 0x6200});   // f16 of n + 768
        pr2[p] = (pku16){0x6600, 0x6600} - __builtin_bit_cast(pku16, pr);
    }
    // the passes; levels into the tile (row k, column l), out as whole rows between the passes
    char* lb = (char*)(lvl + (int64_t)gy0 * op + gx0);
    pku16 rec2[8];
    constexpr int LP = LvlTile<LT>::P;
    LT* lt = (LT*)ot;
    tf_passes(hx, pr2, bs, cq, tl, r, hh, [&](int g, int32_t L) { lt[crow(g, hh) * LP + r] = (LT)L; },
              [&] {
                  wave_sync();
                  // whole 16-B row pieces: 4 instructions of 8 128-B rows (int32), 2 of 16 64-B rows (int16),
                  // 1 of 32 32-B rows (int8)
                  constexpr int PER = 16 / (int)sizeof(LT), RPI = 64 / (32 / PER);   // elements per lane, rows per instr
#pragma unroll
                  for (int i = 0; i < 32 / RPI; ++i) {
                      const int rr = l / (32 / PER) + RPI * i, c = PER * (l % (32 / PER));
                      int4* dst = (int4*)(lb + vofs((rr * (int32_t)op + c) * (int32_t)sizeof(LT)));
                      if constexpr (NT) __builtin_nontemporal_store(*(const v4i_t*)&lt[rr * LP + c], (v4i_t*)dst);
                      else *dst = *(const int4*)&lt[rr * LP + c];
                  }
                  wave_sync();   // the tile's reads before the recon tile reuses it
              },
              rec2);
    // the reconstruction (rows (y_p, y_p + 1) of column x = r) out through the tile in whole rows
    int16_t* rt = (int16_t*)ot;
#pragma unroll
    for (int p = 0; p < 8; ++p) {
        const int y = 2 * (p & 1) + 8 * (p >> 1) + 4 * hh;
        rt[y * kRecH + r] = (int16_t)rec2[p].x;
        rt[(y + 1) * kRecH + r] = (int16_t)rec2[p].y;
    }
    wave_sync();
    char* rb = (char*)(rec + (int64_t)gy0 * op + gx0);
#pragma unroll
    for (int i = 0; i < 2; ++i) {   // 2 instructions of 16 whole 64-B recon rows
        const int rr = (l >> 2) + 16 * i, c = 4 * (l & 3);
        uint4* dst = (uint4*)(rb + vofs((rr * (int32_t)op + 2 * c) * 2));
        if constexpr (NT) __builtin_nontemporal_store(*(const v4i_t*)&ot[rr * kRecP + c], (v4i_t*)dst);
        else *dst = *(const uint4*)&ot[rr * kRecP + c];
    }
}

// Shared memory of one workgroup = GS strips (a group).  Narrow kernels keep
// the coefficient tile in int16 (half the LDS: more workgroups per CU).
template <int CTB, bool NARROW, bool BASIS = false, int GS = 4, bool OST = false, class LT = int32_t> struct CtuSmem {
    using G = Strip<CTB>;
    struct Empty {};
    static constexpr int TILE32 = NARROW ? (GS * G::T16 + 1) / 2 : GS * G::CF;
    __attribute__((aligned(16))) int16_t img[GS * G::IMG];
    __attribute__((aligned(16))) int32_t tile[TILE32];
    uint16_t list[4][64 * GS];   // per TU size: entry = strip << 6 | unit
    int cnt[GS][4], org[2 * GS], next, wide[GS];
    std::conditional_t<BASIS, BasisH, Empty> basis;   // ctu_chain32_h's f16 bases
    // OST: the group's level / recon images, strip-major rows of SW (whole-row stores at the end)
    __attribute__((aligned(16))) LT olvl[OST ? GS * CTB * G::SW : 8];
    __attribute__((aligned(16))) int16_t orec[OST ? GS * CTB * G::SW : 8];
};

// One group of 4 strips (one per wave for loading and classification); the
// TUs of all 4 strips are pooled per size, so a batch of 64/N TUs fills its
// lanes (a strip alone holds ~half a batch per size), and the batches are
// claimed by the 4 waves in descending cost (32x32 chains first).
// NARROW: the packed 16-bit chain.  A group with any sample (strip, row above,
// column left) outside [0, 255] is not coded here: its strips are marked in
// the TU map (bit 7 of each strip's origin byte) for k_ctu_wide.
// !NARROW: the 32-bit chain, any int16 input.
// The seeded quadtree of a strip's CTUs, node-parallel: lane i evaluates node i
// (CTU i / NPC, node i % NPC: level d, Morton index within the level) -- ONE
// split hash per lane instead of up to log2(CTB / 4) per unit along its path --
// and the split bits come back as a wave mask.  A node reaching past the plane
// splits without a hash, as in tu_leaf (nh_tree.hpp).
template <int CTB> struct QuadNodes {
    static constexpr int L = CTB == 32 ? 3 : CTB == 16 ? 2 : CTB == 8 ? 1 : 0;   // split levels
    static constexpr int NPC = ((1 << (2 * L)) - 1) / 3;                         // nodes per CTU
    static constexpr int CPS = 1024 / (CTB * CTB);                                // CTUs per strip
    static_assert(NPC * CPS <= 64, "one node per lane");
};
__device__ __forceinline__ int level_base(int d) { return ((1 << (2 * d)) - 1) / 3; }

template <int CTB>
__device__ __forceinline__ uint64_t strip_splits(uint32_t seed, int pid, int sx0, int sy0, int w, int h) {
    using Q = QuadNodes<CTB>;
    if constexpr (Q::L == 0) {
        return 0;
    } else {
        const int i = opaque_lane();
        bool sp = false;
        if (i < Q::NPC * Q::CPS) {
            const int c = i / Q::NPC, k = i - c * Q::NPC;
            const int d = k >= level_base(2) ? 2 : k >= level_base(1) ? 1 : 0;
            const int m = k - level_base(d);
            int nx = sx0 + c * CTB, ny = sy0;
#pragma unroll
            for (int j = 0; j < 2; ++j) {   // Morton digits, most significant first
                if (j < d) {
                    const int dig = (m >> (2 * (d - 1 - j))) & 3;
                    nx += (dig & 1) * (CTB >> (j + 1));
                    ny += (dig >> 1) * (CTB >> (j + 1));
                }
            }
            const int ns = CTB >> d;
            sp = nx + ns > w || ny + ns > h || tu_split(seed, pid, nx, ny, ns);
        }
        return __ballot(sp);
    }
}

// Leaf of unit (ux, uy) of the strip from the split mask: returns log2 of its
// size and its origin (cx, cy).  Same leaf as tu_leaf.
template <int CTB>
__device__ __forceinline__ int unit_leaf(uint64_t split, int ux, int uy, int sx0, int sy0, int& cx, int& cy) {
    using Q = QuadNodes<CTB>;
    constexpr int UPC = CTB / 4;   // units per CTU side
    const int c = ux / UPC, lx = ux - c * UPC, ly = uy;
    cx = sx0 + c * CTB;
    cy = sy0;
    int m = 0, s = CTB;
#pragma unroll
    for (int d = 0; d < Q::L; ++d) {
        if (!((split >> (c * Q::NPC + level_base(d) + m)) & 1)) break;
        s >>= 1;
        const int qx = (lx * 4) & s ? 1 : 0, qy = (ly * 4) & s ? 1 : 0;   // quadrant at this level
        cx += qx * s;
        cy += qy * s;
        m = 4 * m + 2 * qy + qx;
    }
    return s == 4 ? 2 : s == 8 ? 3 : s == 16 ? 4 : 5;
}

// A strip's source samples in flight: issued by strip_issue, written to the
// LDS image by strip_store (the split lets the persistent kernel keep the next
// group's loads in flight under the current group's chains).
template <int CTB> struct StripLoad {
    static constexpr int NV = (CTB * Strip<CTB>::UW + 63) / 64;
    uint2 v[NV];
    uint2 top;
    int32_t left;
};

template <int CTB, int GS = 4>
__device__ __forceinline__ int strip_of(const CtuArgs& a, int grp, int wv, int& sx0, int& sy0) {
    const int strip = grp * GS + wv;
    sx0 = (strip % a.strips_x) * Strip<CTB>::SW;
    sy0 = (a.row0 + strip / a.strips_x) * CTB;
    return strip < a.strips_x * a.nrows;
}
__device__ __forceinline__ int64_t plane_off(const CtuArgs& a, int pz) {
    const int gz = pz / a.ppg, cz = pz - gz * a.ppg;
    return (int64_t)gz * a.group_stride + (int64_t)cz * a.plane_stride;
}

template <int CTB, int GS = 4>
__device__ __forceinline__ void strip_issue(const CtuArgs& a, int grp, int pz, StripLoad<CTB>& ld, int wv = -1) {
    using G = Strip<CTB>;
    constexpr int UW = G::UW;
    const int lane = opaque_lane();
    if (wv < 0) wv = threadIdx.x >> 6;
    int sx0, sy0;
    const bool valid = strip_of<CTB, GS>(a, grp, wv, sx0, sy0);
    const int16_t* __restrict__ src = a.src + plane_off(a, pz);
    const int w = a.w, h = a.h, pitch = a.pitch;
#pragma unroll
    for (int i = 0; i < ld.NV; ++i) {
        const int g = 64 * i + lane, ry = g / UW, gx = g % UW, x = sx0 + 4 * gx, y = sy0 + ry;
        ld.v[i] = make_uint2(0u, 0u);   // outside the plane: no TU reads it
        if (valid && g < CTB * UW && x < w && y < h && (!NH_AB || (a.probe & 2) == 0))
            ld.v[i] = *(const uint2*)(src + (int64_t)y * pitch + x);
    }
    ld.top = make_uint2(0x00800080u, 0x00800080u);   // 128 above the frame (block.py:41)
    {
        const int x = sx0 + 4 * lane;
        if (valid && lane < UW && sy0 > 0 && x < w) ld.top = *(const uint2*)(src + (int64_t)(sy0 - 1) * pitch + x);
    }
    ld.left = 128;   // left of the frame (block.py:48)
    {
        const int y = sy0 + lane;
        if (valid && lane < CTB && sx0 > 0) ld.left = y < h ? src[(int64_t)y * pitch + sx0 - 1] : 0;
    }
}

// Writes the strip image; returns whether any of its samples is outside [0, 255].
template <int CTB>
__device__ __forceinline__ bool strip_store(const StripLoad<CTB>& ld, int16_t* img, bool valid) {
    using G = Strip<CTB>;
    constexpr int UW = G::UW, IP = G::IP;
    const int lane = opaque_lane();
    uint32_t hi_bits = 0;
#pragma unroll
    for (int i = 0; i < ld.NV; ++i) {
        const int g = 64 * i + lane, ry = g / UW, gx = g % UW;
        if (g < CTB * UW) {
            hi_bits |= ld.v[i].x | ld.v[i].y;
            *(uint2*)&img[(1 + ry) * IP + 4 + 4 * gx] = ld.v[i];
        }
    }
    if (lane < UW) {
        hi_bits |= ld.top.x | ld.top.y;
        *(uint2*)&img[4 + 4 * lane] = ld.top;
    }
    if (lane < CTB) {
        hi_bits |= (uint16_t)ld.left;
        img[(1 + lane) * IP + 3] = (int16_t)ld.left;
    }
    return valid && (hi_bits & 0xff00ff00u) != 0;
}

// OST: a strip's level / recon rows from the group's LDS images to the plane in
// whole rows -- a wave instruction writes 1 KiB of contiguous row segments
// (16 B per lane) instead of 16-128 B pieces of N rows.
template <int CTB, class LT = int32_t>
__device__ __forceinline__ void strip_writeout(const CtuArgs& a, int sx0, int sy0, const LT* ol, const int16_t* orr,
                                               LT* lvl, int16_t* rec) {
    constexpr int SW = Strip<CTB>::SW;
    const int lane = threadIdx.x & 63, w = a.w, h = a.h;
    const int64_t pitch = a.pitch;
    if constexpr (sizeof(LT) == 4) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {   // CTB * SW int32 = 256 pieces of 16 B
            const int c = 64 * i + lane, r = c / (SW / 4), x = 4 * (c % (SW / 4));
            if (sy0 + r < h && sx0 + x < w) st_lvl4(lvl + (int64_t)(sy0 + r) * pitch + sx0 + x, *(const int4*)&ol[r * SW + x]);
        }
    } else {
#pragma unroll
        for (int i = 0; i < 2; ++i) {   // CTB * SW int16 (compact levels) = 128 pieces of 16 B
            const int c = 64 * i + lane, r = c / (SW / 8), x = 8 * (c % (SW / 8));
            if (sy0 + r < h && sx0 + x < w) {
                const uint4 v = *(const uint4*)&ol[r * SW + x];
                LT* p = lvl + (int64_t)(sy0 + r) * pitch + sx0 + x;
                if (sx0 + x + 8 <= w) *(uint4*)p = v;
                else *(uint2*)p = make_uint2(v.x, v.y);   // w % 4 == 0: the last 4 levels of a row
            }
        }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {   // CTB * SW int16 = 128 pieces of 16 B
        const int c = 64 * i + lane, r = c / (SW / 8), x = 8 * (c % (SW / 8));
        if (sy0 + r < h && sx0 + x < w) {
            const uint4 v = *(const uint4*)&orr[r * SW + x];
            int16_t* p = rec + (int64_t)(sy0 + r) * pitch + sx0 + x;
            if (sx0 + x + 8 <= w) *(uint4*)p = v;
            else st_rec4(p, make_uint2(v.x, v.y));   // w % 4 == 0: the last 4 samples of a row
        }
    }
}

// A group's TU plan (k_ctu_plan, one record per (plane id, group) of a launch's band): the TU
// byte of every (strip, unit) (0xFF: outside the plane), the pooled TU counts per size and the
// entries (strip << 6 | unit) of every size, back to back in size order.  The seeded quadtree
// depends on (plane id, position) only, so every frame of a plane set shares its records:
// k_ctu_open reads them instead of hashing and pooling per group (one barrier less).
constexpr int kCtuPlanCnt = 256, kCtuPlanEnt = 272, kCtuPlanBytes = 1024;
template <int CTB, int GS>
__global__ void __launch_bounds__(64 * GS) k_ctu_plan(CtuArgs a) {
    static_assert(GS * 64 <= kCtuPlanCnt && kCtuPlanEnt + 2 * 64 * GS <= kCtuPlanBytes, "plan record layout");
    using G = Strip<CTB>;
    constexpr int UW = G::UW;
    __shared__ int cnt_s[GS][4];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63, grp = blockIdx.x, c = blockIdx.y;
    int sx0, sy0;
    const bool valid = strip_of<CTB, GS>(a, grp, wv, sx0, sy0);
    uint8_t* pr = a.plan_w + ((int64_t)c * a.ngroups + grp) * kCtuPlanBytes;
    bool org = false, in = false;
    int ls = 0;
    if (valid) {   // as ctu_group's classification
        const uint64_t split = strip_splits<CTB>(a.seed, a.plane_id + c, sx0, sy0, a.w, a.h);
        const int ux = lane % UW, uy = lane / UW, x = sx0 + 4 * ux, y = sy0 + 4 * uy;
        in = x < a.w && y < a.h;
        int cx, cy;
        ls = unit_leaf<CTB>(split, ux, uy, sx0, sy0, cx, cy);
        org = in && cx == x && cy == y;
    }
    pr[wv * 64 + lane] = in ? (uint8_t)ls : (uint8_t)0xFF;
    uint64_t m[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        m[k] = __ballot(org && ls == k + 2);
        if (lane == 0) cnt_s[wv][k] = __popcll(m[k]);
    }
    __syncthreads();
    int base = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        int off = 0, tot = 0;
#pragma unroll
        for (int q = 0; q < GS; ++q) {
            off += q < wv ? cnt_s[q][k] : 0;
            tot += cnt_s[q][k];
        }
        if (org && ls == k + 2)
            ((uint16_t*)(pr + kCtuPlanEnt))[base + off + __popcll(m[k] & ((1ull << lane) - 1))] = (uint16_t)(wv << 6 | lane);
        if (threadIdx.x == k) ((int*)(pr + kCtuPlanCnt))[k] = tot;
        base += tot;
    }
}

// MFMA32: the 32x32 TUs on the matrix cores, one per batch (narrow: f16,
// ctu_chain32_h; wide: int8, ctu_chain32 -- A/B forms); otherwise two per
// batch on 32-point butterflies.
//
// One group of 4 strips (one per wave for loading and classification); the
// TUs of all 4 strips are pooled per size, so a batch of 64/N TUs fills its
// lanes (a strip alone holds ~half a batch per size), and the batches are
// claimed by the 4 waves in descending cost (32x32 chains first).  The
// group's loads (ld) were issued by the caller; the classification runs
// while they are in flight.
// NARROW: the packed 16-bit chain.  A group with any sample (strip, row above,
// column left) outside [0, 255] is not coded here: its strips are marked in
// the TU map (bit 7 of each strip's origin byte) for k_ctu_wide.
// !NARROW: the 32-bit chain, any int16 input.
// Returns with the workgroup's waves in the batch loop's exit (no barrier).
// LT: the level type (int16_t: config 4's compact levels, narrow groups only).
template <int CTB, bool LUMA, bool NARROW, bool MFMA32, int GS, bool OST = false, bool PLAN = false,
          class LT = int32_t, class Prefetch>
__device__ __forceinline__ void ctu_group(const CtuArgs& a, int grp, int pz,
                                          CtuSmem<CTB, NARROW, NARROW && MFMA32 && !(NH_CTU_TF32 && !OST), GS, OST, LT>& sm,
                                          StripLoad<CTB>& ld,
                                          Prefetch&& prefetch) {
    using G = Strip<CTB>;
    constexpr int UW = G::UW;
    const int wv = threadIdx.x >> 6, lane = opaque_lane();
    int sx0, sy0;
    const bool valid = strip_of<CTB, GS>(a, grp, wv, sx0, sy0);
    static_assert(NARROW || sizeof(LT) == 4, "the 32-bit chain writes int32 levels");
    const int64_t poff = plane_off(a, pz);
    LT* lvl = (LT*)a.lvl + poff;
    int16_t* rec = a.rec + poff;
    const int pid = a.plane_id + (pz % a.ppg);
    const int w = a.w, h = a.h;
    int16_t* img = sm.img + wv * G::IMG;

    // ---- 1. classify the strip's 64 units (loads in flight): leaf size / origin, TU map ----
    bool org = false;
    int ls = 0;
    const int64_t tu_org = (int64_t)pz * a.tu_plane + (int64_t)(sy0 >> 2) * (w >> 2) + (sx0 >> 2);
    uint64_t m[4];
    int pcnt[4];   // PLAN: the group's TU counts per size
    if constexpr (PLAN) {
        // the group's TUs from its plan (k_ctu_plan: same for every plane of this plane id): this
        // unit's TU byte, and the group's pooled entries straight into the per-size lists
        const uint8_t* pr = a.plan + ((int64_t)(pz % a.ppg) * a.ngroups + grp) * kCtuPlanBytes;
        const int4 cn = *(const int4*)(pr + kCtuPlanCnt);
        pcnt[0] = cn.x; pcnt[1] = cn.y; pcnt[2] = cn.z; pcnt[3] = cn.w;
        const int tub = pr[wv * 64 + lane];
        const int pe = wv * 64 + lane, b1 = cn.x, b2 = b1 + cn.y, b3 = b2 + cn.z, te = b3 + cn.w;
        const int ent = pe < te ? ((const uint16_t*)(pr + kCtuPlanEnt))[pe] : 0;
        ls = tub;
        if (valid && tub != 0xFF && (!NH_AB || (a.probe & 8) == 0)) {
            const int x = sx0 + 4 * (lane % UW), y = sy0 + 4 * (lane / UW);
            a.tu[(int64_t)pz * a.tu_plane + (int64_t)(y >> 2) * (w >> 2) + (x >> 2)] = (uint8_t)tub;
        }
        if (pe < te) {
            const int k = (pe >= b1) + (pe >= b2) + (pe >= b3);
            const int base = k == 0 ? 0 : k == 1 ? b1 : k == 2 ? b2 : b3;
            sm.list[k][pe - base] = (uint16_t)ent;
        }
    } else {
        if (valid) {
            const uint64_t split = strip_splits<CTB>(a.seed, pid, sx0, sy0, w, h);
            const int ux = lane % UW, uy = lane / UW, x = sx0 + 4 * ux, y = sy0 + 4 * uy;
            const bool in = x < w && y < h;
            int cx, cy;
            ls = unit_leaf<CTB>(split, ux, uy, sx0, sy0, cx, cy);
            if (in && (!NH_AB || (a.probe & 8) == 0))
                a.tu[(int64_t)pz * a.tu_plane + (int64_t)(y >> 2) * (w >> 2) + (x >> 2)] = (uint8_t)ls;
            org = in && cx == x && cy == y;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            m[k] = __ballot(org && ls == k + 2);
            if (lane == 0) sm.cnt[wv][k] = __popcll(m[k]);
        }
    }
    // ---- 2. the strip image: its samples, the row above and the column left, into LDS ----
    {
        const bool wide = strip_store<CTB>(ld, img, valid);
        if constexpr (NARROW) {
            const uint64_t wb = __ballot(wide);
            if (lane == 0) sm.wide[wv] = wb != 0;
        }
        if (lane == 0) {
            sm.org[2 * wv] = sx0;
            sm.org[2 * wv + 1] = sy0;
        }
    }
    prefetch();   // the next group's loads into ld (persistent kernel)
    if (threadIdx.x == 0) sm.next = 0;
    __syncthreads();
    if constexpr (NARROW) {
        int any_wide = a.wide_only;
#pragma unroll
        for (int q = 0; q < GS; ++q) any_wide |= sm.wide[q];
        if (__builtin_amdgcn_readfirstlane(any_wide)) {
            if (valid && lane == 0) a.tu[tu_org] = (uint8_t)(ls | 0x80);   // unit 0 = the strip's origin
            return;
        }
    }
    // pool the strips' TUs per size: entry = strip << 6 | unit (PLAN: pooled by k_ctu_plan, stored above)
    int cnt[4];
    if constexpr (PLAN) {
#pragma unroll
        for (int k = 0; k < 4; ++k) cnt[k] = pcnt[k];
    } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            int off = 0;
            cnt[k] = 0;
#pragma unroll
            for (int q = 0; q < GS; ++q) {
                off += q < wv ? sm.cnt[q][k] : 0;
                cnt[k] += sm.cnt[q][k];
            }
            if (org && ls == k + 2) sm.list[k][off + __popcll(m[k] & ((1ull << lane) - 1))] = (uint16_t)(wv << 6 | lane);
        }
        __syncthreads();
    }

    // ---- 3. batches, claimed in descending cost: 32x32 chains, then 16, 8, 4 ----
    if (NH_AB && (a.probe & 1)) return;
    const int n32 = CTB == 32 ? (MFMA32 ? cnt[3] : (cnt[3] + 1) / 2) : 0;
    const int n16 = CTB >= 16 ? (cnt[2] + 3) / 4 : 0, n8 = CTB >= 8 ? (cnt[1] + 7) / 8 : 0, n4 = (cnt[0] + 15) / 16;
    const int total = n32 + n16 + n8 + n4;
#define NH_CHAIN(N, DST, L, B)                                                                              \
    if constexpr (NARROW && N <= 16 && (OST ? NH_CTU_MOSAIC >= 1 : NH_CTU_MOSAIC >= 2))                    \
        ctu_batch_mma<N, DST, CTB, OST, LT>(a, sm.img, sm.list[L], cnt[L], B, sm.org, lvl, rec, sm.olvl, sm.orec); \
    else if constexpr (NARROW)                                                                              \
        ctu_chain_pk<N, DST, CTB, OST, LT>(a, sm.img, (int16_t*)sm.tile, sm.list[L], cnt[L], B, sm.org, lvl, rec, \
                                       sm.olvl, sm.orec);                                                   \
    else                                                                                                    \
        ctu_chain<N, DST, CTB>(a, sm.img, sm.tile, sm.list[L], cnt[L], B, sm.org, lvl, rec);
    for (;;) {
        int item = 0;
        if (lane == 0) item = atomicAdd(&sm.next, 1);
        item = __builtin_amdgcn_readfirstlane(__shfl(item, 0, 64));
        if (item >= total) break;
        if constexpr (CTB == 32) {
            if (item < n32) {
                if constexpr (NARROW && MFMA32 && NH_CTU_TF32 && !OST) {   // the transposition-free chain (§4.5)
                    const int e = sm.list[3][item], sw = e >> 6;
                    const ChainQ cq = make_chainq(a.q[3], a.dqs, a.dq_per);
                    const TfLane tl = make_tf_lane(cq, c_basis_hc, lane & 31);
                    chain32_tf(a, ImgStrip{sm.img + sw * G::IMG + 4}, c_basis_hc, sm.org[2 * sw], sm.org[2 * sw + 1], lvl,
                               rec, (int32_t*)((int16_t*)sm.tile + sw * G::T16), cq, tl);
                } else if constexpr (NARROW && MFMA32) {   // one TU per wave on the f16 matrix cores
                    const int e = sm.list[3][item], sw = e >> 6;
                    if constexpr (OST)
                        ctu_chain32_h(a, ImgStrip{sm.img + sw * G::IMG + 4}, (uint16_t*)sm.tile + sw * G::T16, sm.basis, 0, 0,
                                      sm.olvl + sw * (CTB * G::SW), sm.orec + sw * (CTB * G::SW), nullptr, G::SW);
                    else
                        ctu_chain32_h(a, ImgStrip{sm.img + sw * G::IMG + 4}, (uint16_t*)sm.tile + sw * G::T16, sm.basis,
                                      sm.org[2 * sw], sm.org[2 * sw + 1], lvl, rec);
                } else if constexpr (MFMA32) {   // one TU per wave on the int8 matrix cores (A/B form)
                    const int e = sm.list[3][item], sw = e >> 6;
                    ctu_chain32(a, sm.img + sw * G::IMG + 4, sm.tile + sw * G::CF, sm.org[2 * sw], sm.org[2 * sw + 1],
                                lvl, rec);
                } else {                          // two TUs per wave, 32-point butterflies
                    NH_CHAIN(32, false, 3, 2 * item)
                }
                continue;
            }
        }
        item -= n32;
        if constexpr (CTB >= 16) {
            if (item < n16) {
                NH_CHAIN(16, false, 2, 4 * item)
                continue;
            }
        }
        item -= n16;
        if constexpr (CTB >= 8) {
            if (item < n8) {
                NH_CHAIN(8, false, 1, 8 * item)
                continue;
            }
        }
        item -= n8;
        NH_CHAIN(4, LUMA, 0, 16 * item)
    }
#undef NH_CHAIN
    if constexpr (OST) {   // every TU of the group is coded: each wave writes its strip out in whole rows
        __syncthreads();
        if (valid) strip_writeout<CTB, LT>(a, sx0, sy0, sm.olvl + wv * (CTB * G::SW), sm.orec + wv * (CTB * G::SW), lvl, rec);
    }
}

// The config-4 kernel proper, packed chain, 32x32 TUs on packed butterflies
// (MFMA32: on the f16 matrix cores, A/B form).  PERSIST: a grid of
// resident workgroups walking the (group, plane) items with stride gridDim.x,
// each group's loads issued during the previous group's chains.
// WAVES: the occupancy floor (waves/SIMD) the registers are allocated for.
// PLAN: the groups' TUs from k_ctu_plan's records (a.plan) instead of classified per group.
template <int CTB, bool LUMA, bool MFMA32 = false, int PERSIST = 0, int WAVES = 5, int GS = 4, bool OST = false,
          bool PLAN = false, class LT = int32_t>
__global__ void __launch_bounds__(64 * GS) __attribute__((amdgpu_waves_per_eu(WAVES))) k_ctu_open(CtuArgs a, int items) {
    static_assert(!PLAN || (GS == 4 && PERSIST == 0), "plan records: groups of 4 strips, one group per workgroup");
    // (the transposition-free 32x32 chain reads its bases from the constant table: no LDS copy)
    constexpr bool BAS = MFMA32 && !(NH_CTU_TF32 && !OST);
    __shared__ CtuSmem<CTB, true, BAS, GS, OST, LT> sm;
    if (NH_AB && (a.probe & 4)) return;   // A/B probe: the launch of the grid alone
    if constexpr (PERSIST == 0) {
        // the bases' loads issued with the strip's and written to LDS after the
        // strip image (one wait for both; ctu_group's barrier orders them before use)
        static_assert(sizeof(BasisH) == 256 * 16 && GS >= 4, "one 16-byte piece per thread of the first 256");
        uint4 bq{};
        const bool bthr = threadIdx.x < 256;
        if constexpr (BAS) {
            if (bthr) bq = ((const uint4*)&c_basis_h)[threadIdx.x];
        }
        StripLoad<CTB> ld;
        strip_issue<CTB, GS>(a, blockIdx.x, blockIdx.y, ld);
        ctu_group<CTB, LUMA, true, MFMA32, GS, OST, PLAN, LT>(a, blockIdx.x, blockIdx.y, sm, ld, [&] {
            if constexpr (BAS) {
                if (bthr) ((uint4*)&sm.basis)[threadIdx.x] = bq;
            }
        });
    } else {
        if constexpr (BAS) copy_basis_h(sm.basis);   // ordered before use by ctu_group's barrier
        // PERSIST = 1: the next group's loads in flight under this group's chains;
        // PERSIST = 2: no prefetch (only the per-workgroup start-up amortised)
        StripLoad<CTB> ld;
        int it = blockIdx.x;
        const int gcount = (a.strips_x * a.nrows + GS - 1) / GS;
        if (PERSIST == 1 && it < items) strip_issue<CTB, GS>(a, it % gcount, it / gcount, ld);
        for (; it < items; it += gridDim.x) {
            const int nx = it + gridDim.x;
            if constexpr (PERSIST == 2) strip_issue<CTB, GS>(a, it % gcount, it / gcount, ld);
            ctu_group<CTB, LUMA, true, MFMA32, GS, OST, false, LT>(a, it % gcount, it / gcount, sm, ld, [&] {
                if (PERSIST == 1 && nx < items) strip_issue<CTB, GS>(a, nx % gcount, nx / gcount, ld);
            });
            __syncthreads();   // every wave done with this group's LDS
        }
    }
}

// The wide fix-up: workgroup b scans the origin bytes of groups [16 b, 16 b + 16)
// and codes the marked ones with the 32-bit chain (restoring their TU bytes).
// For 8-bit content nothing is marked and every workgroup exits at once.
constexpr int kWideGroups = 16;
template <int CTB, bool LUMA, bool MFMA32>
__global__ void __launch_bounds__(256) k_ctu_wide(CtuArgs a) {
    __shared__ CtuSmem<CTB, false> sm;
    __shared__ unsigned long long s_mask;
    using G = Strip<CTB>;
    const int g0 = blockIdx.x * kWideGroups, pz = blockIdx.y;
    if (threadIdx.x < kWideGroups) {
        const int nstrips = a.strips_x * a.nrows;
        bool marked = false;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int strip = 4 * (g0 + (int)threadIdx.x) + k;
            if (strip < nstrips) {
                const int sx0 = (strip % a.strips_x) * G::SW, sy0 = (a.row0 + strip / a.strips_x) * CTB;
                marked |= (a.tu[(int64_t)pz * a.tu_plane + (int64_t)(sy0 >> 2) * (a.w >> 2) + (sx0 >> 2)] & 0x80) != 0;
            }
        }
        const uint64_t mk = __ballot(marked);
        if (threadIdx.x == 0) s_mask = mk;
    }
    __syncthreads();
    uint64_t mask = s_mask;
    while (mask) {
        const int b = __builtin_ctzll(mask);
        mask &= mask - 1;
        StripLoad<CTB> ld;
        strip_issue<CTB>(a, g0 + b, pz, ld);
        if (a.spill) {   // compact levels: int32 levels into the spill plane, a marker at every strip origin
            CtuArgs aw = a;
            aw.lvl = a.spill;
            ctu_group<CTB, LUMA, false, MFMA32, 4>(aw, g0 + b, pz, sm, ld, [] {});
            int sx0, sy0;
            if (strip_of<CTB>(a, g0 + b, threadIdx.x >> 6, sx0, sy0) && (threadIdx.x & 63) == 0)
                a.lvl_c[plane_off(a, pz) + (int64_t)sy0 * a.pitch + sx0] = kCtuSpillMark;
        } else {
            ctu_group<CTB, LUMA, false, MFMA32, 4>(a, g0 + b, pz, sm, ld, [] {});
        }
        __syncthreads();
    }
}

// Config 5 for narrow blocks: one wave per full 32x32
// block of the plane (the strip machinery with strips_x = w / 32 blocks per
// row), the block image as a CTB-32 strip in LDS, ctu_chain32_h.  A wave whose
// block or neighbours leave [0, 255] codes nothing and writes the marker
// -32768 at its block's recon origin (recon is always in [0, 255]); the int8
// chain (k_tc32_mfma, nh_tc32.hip) then codes exactly the marked blocks.
constexpr int16_t kWideMark = (int16_t)0x8000;
#if NH_AB   // the round-2/3 one-block-per-wave forms (A/B build only; the product runs k_tc32_hd)
// K blocks per wave (consecutive in raster order), block k+1's loads issued
// before block k's chain.  K = 1 in the product: K = 4 measured slower (0.177
// vs 0.159 ms per 8K frame; 114 registers, 4 waves/SIMD), DESIGN.md §4.5.
// XCD: the workgroup grid renumbered so that XCD x runs the x-th eighth of the
// (plane, block) order (xcd_eighths, as the hot kernel; A/B).  TSTORE: the
// chain's outputs leave in whole rows through an LDS tile (ctu_chain32_h).
// The strip loads are issued before the bases are copied to LDS, so the copy
// and its barrier run under the loads.
// BREG: every lane keeps its basis operands in registers (BasisRegs, loaded
// from the constant copy under the strip loads): no LDS copy, no barrier.
template <int K, bool XCD = false, bool TSTORE = false, bool BREG = false>
__global__ void __launch_bounds__(256) k_tc32_h(CtuArgs a, int nblk) {
    using G = Strip<32>;
    __shared__ __attribute__((aligned(16))) int16_t s_img[4][G::IMG];
    __shared__ __attribute__((aligned(16))) uint16_t s_q[4][32 * G::QH];
    __shared__ std::conditional_t<BREG, int, BasisH> s_basis;
    __shared__ __attribute__((aligned(16))) int32_t s_out[TSTORE ? 4 : 1][TSTORE ? 32 * kOutP : 4];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint32_t bx = blockIdx.x, by = blockIdx.y;
    if constexpr (XCD) {
        const uint32_t id = xcd_eighths(by * gridDim.x + bx, gridDim.x * gridDim.y);
        by = id / gridDim.x;
        bx = id - by * gridDim.x;
    }
    const int b0 = ((int)bx * 4 + wv) * K;
    const int pz = (int)by;
    StripLoad<32> ld;
    // strip_issue addresses strip 4 * grp + wave: block b is grp = b / 4 with this wave's slot b % 4
    auto issue = [&](int b) { strip_issue<32>(a, b >> 2, pz, ld, b & 3); };
    if (b0 < nblk) issue(b0);   // in flight under the bases' copy and the barrier
    std::conditional_t<BREG, BasisRegs, int> breg;
    if constexpr (BREG) {
        if (b0 >= nblk) return;   // whole wave
        breg = load_basis_regs(c_basis_h, lane & 31, lane >> 5);
    } else {
        copy_basis_h(s_basis);
        __syncthreads();
        if (b0 >= nblk) return;   // whole wave
    }
    const int64_t poff = plane_off(a, pz);
    for (int k = 0; k < K; ++k) {
        const int b = b0 + k;
        if (b >= nblk) break;
        const int sx0 = (b % a.strips_x) * 32, sy0 = (b / a.strips_x) * 32;
        const bool wide = __any(strip_store<32>(ld, s_img[wv], true));
        if (k + 1 < K && b + 1 < nblk) issue(b + 1);
        wave_sync();
        if (wide) {
            if (lane == 0) {
                a.rec[poff + (int64_t)sy0 * a.pitch + sx0] = kWideMark;
                if (a.wide_flag) *a.wide_flag = a.epoch;   // the fix-up launch has work
            }
        } else {
            if constexpr (BREG)
                ctu_chain32_h<TSTORE>(a, ImgStrip{s_img[wv] + 4}, s_q[wv], breg, sx0, sy0, a.lvl + poff, a.rec + poff,
                                      TSTORE ? s_out[TSTORE ? wv : 0] : nullptr);
            else
                ctu_chain32_h<TSTORE>(a, ImgStrip{s_img[wv] + 4}, s_q[wv], s_basis, sx0, sy0, a.lvl + poff, a.rec + poff,
                                      TSTORE ? s_out[TSTORE ? wv : 0] : nullptr);
        }
        wave_sync();   // this wave's LDS reads of block k before block k+1's image writes
    }
}
#endif

// Config 5, 8-bit blocks, with the next block's image loaded under this one's
// chain: a wave codes KB consecutive blocks; block k+1's
// body (two 1-KiB LDS-DMA pieces: 16 B per lane, rows of 64 B), its top row and
// its left column land in the wave's other LDS slot by LDS-DMA while block k
// runs -- no registers hold them.  Before block k+1 reads its slot the wave
// waits with vmcnt(4 + the stores block k issued): the loads complete in issue
// order, so that retires exactly block k+1's DMA and leaves the next block's in
// flight; `lgkmcnt(0)` before a DMA is issued retires the wave's reads of the
// slot it overwrites.  At the frame's top / left edge the DMA reads the block's
// own row / column and the 128s of block.py:41-48 overwrite it after the wait.
// Same chain (ctu_chain32_h over an ImgDma image), same marks for wide blocks.
// The two counts below are what the compiler emits; tools/isa_check.py runs the
// built kernel's control flow as a model of the in-order vmcnt queue and fails
// (tests/test_isa_checks.py) unless every wait retires exactly block k's DMA.
#ifndef NH_TC32HD_STORES_NARROW   // (overridable only so that tests/test_isa_checks.py can miscount on purpose)
#define NH_TC32HD_STORES_NARROW 6
#endif
#ifndef NH_TC32HD_STORES_WIDE
#define NH_TC32HD_STORES_WIDE 2
#endif
constexpr int kTc32hdStoresNarrow = NH_TC32HD_STORES_NARROW;   // chain32_tf, int32 levels: 4 level-row + 2 recon-row stores
constexpr int kTc32hdStoresWide = NH_TC32HD_STORES_WIDE;       // the wide mark and the wide flag (never null here)
// LT: the level element type (LvlTile): int16 / int8 levels take 2 / 1 level-row stores instead of 4
template <class LT> constexpr int tc32hd_stores_narrow() { return kTc32hdStoresNarrow - 4 + LvlTile<LT>::STORES; }
// ILV: wave w of workgroup g codes blocks 4 KB g + w + 4 k (k < KB), so the 4 waves work on 4
// horizontally adjacent blocks at a time (their row pieces form 4x longer contiguous runs in HBM);
// otherwise blocks KB (4 g + w) + k.
// W: waves per workgroup (A/B: 8); NT: nontemporal output stores (A/B)
template <int KB, class LT = int32_t, bool ILV = false, int W = 4, bool NT = false>
__global__ void __launch_bounds__(64 * W) __attribute__((amdgpu_waves_per_eu(3))) k_tc32_hd(CtuArgs a, int nblk) {
    constexpr int kNarrow = tc32hd_stores_narrow<LT>();
    static_assert(kNarrow > 0, "store count");   // (equal to the wide count: one wait serves both kinds)
    __shared__ __attribute__((aligned(16))) int16_t s_body[W][2][32 * 32];
    __shared__ __attribute__((aligned(16))) int16_t s_edge[W][2][96];
    __shared__ BasisHC s_basis;
    // the level / recon tile: int32 level rows (kOutP), else the recon tile's kRecP (compact levels fit in it)
    __shared__ __attribute__((aligned(16))) int32_t s_out[W][32 * (sizeof(LT) == 4 ? kOutP : kRecP)];
    // the wave index in an SGPR: block index, `next` and the loop are scalar
    // branches, so one wave never runs both sides of a block's wait selection
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    constexpr int BS = ILV ? W : 1;   // block stride of a wave
    const int b0 = ILV ? (int)blockIdx.x * W * KB + wv : ((int)blockIdx.x * W + wv) * KB, pz = (int)blockIdx.y;
    const int64_t poff = plane_off(a, pz);
    const int16_t* src = a.src + poff;
    const ChainQ cq = make_chainq(a.q[3], a.dqs, a.dq_per);
    copy_basis_hc(s_basis);
    __syncthreads();   // (before any DMA is in flight)
    const TfLane tl = make_tf_lane(cq, s_basis, lane & 31);   // chain32_tf's per-lane offsets
    if (b0 >= nblk) return;   // whole wave
    // per-lane byte offsets of the DMA pieces from the block's (uniform) origin
    const uint32_t o_body = (uint32_t)(((lane >> 2) * a.pitch + 8 * (lane & 3)) * 2), o_body2 = 16u * a.pitch * 2;
    const uint32_t o_top = 16u * lane, o_left = (uint32_t)(lane * a.pitch * 2);
    auto issue = [&](int b, int slot) {   // 4 DMA instructions per block
        const int sx0 = (b % a.strips_x) * 32, sy0 = (b / a.strips_x) * 32;
        const int16_t* blk = src + (int64_t)sy0 * a.pitch + sx0;
        glds16s(blk, o_body, lds_addr(&s_body[wv][slot][0]));
        glds16s(blk, o_body + o_body2, lds_addr(&s_body[wv][slot][512]));
        if (lane < 4) glds16s(blk - (sy0 > 0 ? (int64_t)a.pitch : 0), o_top, lds_addr(&s_edge[wv][slot][0]));
        if (lane < 32) glds2s(blk - (sx0 > 0 ? 1 : 0), o_left, lds_addr(&s_edge[wv][slot][32]));
    };
    issue(b0, 0);
    int prev = 0;   // store instructions the previous block issued (0: none, kTc32hdStoresWide, kNarrow)
    for (int k = 0; k < KB; ++k) {
        const int b = b0 + BS * k;
        if (b >= nblk) break;
        const int slot = k & 1;
        const bool next = k + 1 < KB && b + BS < nblk;
        if (next) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // WAR on the slot block k+1 overwrites
            issue(b + BS, slot ^ 1);
        }
        // retire block b's DMA: it was issued before the previous block's stores and block b+1's DMA
        if (next) {
            if (prev == kNarrow) wait_vm<4 + kNarrow>();
            else if (prev == kTc32hdStoresWide) wait_vm<4 + kTc32hdStoresWide>();
            else wait_vm<4>();
        } else {
            if (prev == kNarrow) wait_vm<kNarrow>();
            else if (prev == kTc32hdStoresWide) wait_vm<kTc32hdStoresWide>();
            else wait_vm<0>();
        }
        const int sx0 = (b % a.strips_x) * 32, sy0 = (b / a.strips_x) * 32;
        const int16_t* body = s_body[wv][slot];
        int16_t* edge = s_edge[wv][slot];
        if (sy0 == 0 && lane < 32) edge[lane] = 128;        // above the frame (block.py:41)
        if (sx0 == 0 && lane < 32) edge[32 + 2 * lane] = 128;   // left of the frame (block.py:48)
        wave_sync();
        uint32_t hi;   // any sample of the block, its top row or its left column outside [0, 255]?
        {
            const uint4 v0 = ((const uint4*)body)[lane], v1 = ((const uint4*)body)[64 + lane];
            hi = v0.x | v0.y | v0.z | v0.w | v1.x | v1.y | v1.z | v1.w;
            if (lane < 48) hi |= ((const uint32_t*)edge)[lane];
        }
        const bool wide = __any((hi & 0xff00ff00u) != 0);
        if (wide) {
            if (lane == 0) {
                a.rec[poff + (int64_t)sy0 * a.pitch + sx0] = kWideMark;
                *a.wide_flag = a.epoch;   // the fix-up launch has work
            }
            prev = kTc32hdStoresWide;
        } else {
            chain32_tf<ImgDma, LT, NT>(a, ImgDma{body, edge}, s_basis, sx0, sy0, (LT*)a.lvl + poff, a.rec + poff, s_out[wv], cq, tl);
            prev = kNarrow;
        }
        wave_sync();
    }
}



// The bases in constant memory, once per device.  hipMemcpyToSymbol is
// host-synchronous, so every kernel queued afterwards -- on any stream -- reads
// the uploaded values.
static int ensure_basis_ctu() {
    static PerDeviceOnce once;
    return once.run([] {
        const Basis b = make_basis();
        NH_HIP(hipMemcpyToSymbol(HIP_SYMBOL(c_basis_ctu), &b, sizeof(b)));
        const BasisH bh = make_basis_h();
        NH_HIP(hipMemcpyToSymbol(HIP_SYMBOL(c_basis_h), &bh, sizeof(bh)));
        const BasisHC bhc = make_basis_hc();
        NH_HIP(hipMemcpyToSymbol(HIP_SYMBOL(c_basis_hc), &bhc, sizeof(bhc)));
        static MosaicLane mt[4][64];   // ctu_batch_mma's per-lane bases (this translation unit's copy)
        make_mosaic(mt);
        NH_HIP(hipMemcpyToSymbol(HIP_SYMBOL(c_mosaic_ctu), mt, sizeof(mt)));
        return (int)NH_OK;
    });
}

// Launches k_ctu_open over CTU rows [row0, row1) of every plane of the set.
// Returns NH_EVALUE when the layout does not allow the kernel's vector accesses
// (8-B rows / 16-B level rows): the caller then takes the per-size path.
// lvl_bytes = 2: config 4's compact levels (int16 level plane `lvl`, int32 `spill` for the wide groups
// k_ctu_wide codes, a marker at each of their strip origins; CTB 16 / 32 only, 16-B aligned rows).
int ctu_open_launch(const int16_t* src, void* lvl, int16_t* rec, uint8_t* tu, const nh_plane_set* set, int ctb,
                    int plane_id, uint32_t seed, int is_luma, int row0, int row1, const QuantParams* q, int dqs,
                    int dq_per, hipStream_t s, int lvl_bytes, int32_t* spill) {
    const int64_t planes = (int64_t)set->planes_per_group * set->num_groups;
    if ((set->pitch & 3) || ((set->base | set->plane_stride | set->group_stride) & 3) ||
        (((uintptr_t)src | (uintptr_t)rec) & 7) || ((uintptr_t)lvl & 15))
        return NH_EVALUE;
    const bool compact = lvl_bytes == 2;
    if (compact && ((ctb != 16 && ctb != 32) || (set->pitch & 7) || ((set->base | set->plane_stride | set->group_stride) & 7) ||
                    !spill || ((uintptr_t)spill & 15)))
        return NH_EVALUE;
    const int rc = ensure_basis_ctu();
    if (rc) return rc;
    CtuArgs a{};
    a.src = src + set->base;
    if (compact) {
        a.lvl = (int32_t*)((int16_t*)lvl + set->base);   // k_ctu_open<.., int16_t> reads it as int16_t*
        a.lvl_c = (int16_t*)lvl + set->base;
        a.spill = spill + set->base;
    } else {
        a.lvl = (int32_t*)lvl + set->base;
    }
    a.rec = rec + set->base;
    a.tu = tu;
    a.group_stride = set->group_stride;
    a.plane_stride = set->plane_stride;
    a.tu_plane = (int64_t)(set->height / 4) * (set->width / 4);
    a.w = set->width;
    a.h = set->height;
    a.pitch = set->pitch;
    a.ppg = set->planes_per_group;
    a.plane_id = plane_id;
    a.row0 = row0;
    a.nrows = row1 - row0;
    a.strips_x = (set->width + 1024 / ctb - 1) / (1024 / ctb);
    a.seed = seed;
    for (int k = 0; k < 4; ++k) a.q[k] = q[k];
    a.dqs = dqs;
    a.dq_per = dq_per;
    const int64_t strips = (int64_t)a.strips_x * a.nrows;
    if (strips <= 0 || planes <= 0) return NH_OK;
    const int64_t groups = (strips + 3) / 4;   // k_ctu_wide's groups of 4 strips
    if (groups * planes > INT32_MAX) return NH_EARG;
    const dim3 grid_wide((unsigned)((groups + kWideGroups - 1) / kWideGroups), (unsigned)planes);
    // Narrow groups (8-bit content) are coded by k_ctu_open with the packed
    // chain, their 32x32 TUs on the f16 matrix cores (rocprof: 428.5 vs 459.9
    // us per 16 luma planes for the packed butterflies); the
    // groups it marks (any sample outside [0, 255]) by k_ctu_wide with the
    // 32-bit chain.  A/B build: NH_CTU_T32 = 0 (narrow 32x32 TUs on packed
    // butterflies) / 1 (wide 32x32 TUs on int8 MFMA), NH_CTU_PERSIST = 1 / 2
    // (resident grid, loads one group ahead / without prefetch), NH_CTU_NARROW = 0 (every group on
    // the 32-bit path), NH_CTU_PROBE = bits 1 / 2 / 4 / 8 (no batches / no global loads /
    // return at once / no TU-map stores).
    static const int t32 = NH_KNOB("NH_CTU_T32", 2);
    static const int persist = NH_KNOB("NH_CTU_PERSIST", 0);
    // The luma f16-MFMA form runs at 6 waves/SIMD: 76 VGPRs with zero-initialised
    // accumulators (90 with the rounding constant as their initial value) and
    // 27 KB of LDS per workgroup with the 4 KB bases.
    a.wide_only = NH_KNOB("NH_CTU_NARROW", 1) == 0;
    a.probe = NH_KNOB("NH_CTU_PROBE", 0);
    // Group size GS (strips pooled per workgroup of 64 GS threads) and the
    // occupancy cap (resident workgroups per CU, lds_cap).
    // A/B build: NH_CTU_GS = 4 / 6 / 8, NH_CTU_CAP = workgroups per CU,
    // NH_OCC_CAP = 0 uncapped.
    static const int gs_knob = NH_KNOB("NH_CTU_GS", 4), cap_knob = NH_KNOB("NH_CTU_CAP", 0);
    // A/B build: NH_CTU_OST = bit 1 luma / bit 2 chroma with whole-row output stores (LDS output images)
    static const int ost_knob = NH_KNOB("NH_CTU_OST", 0);
    (void)ost_knob;
    // A/B build only, NH_CTU_PLAN = 1: the groups' TU plans (k_ctu_plan, one 1-KB record per (plane
    // id, group)) in stream-ordered memory, built by a prologue launch and read by k_ctu_open instead
    // of classifying every group: 0.0342-0.0344 vs 0.0341-0.0346 ms per 4K frame, not kept
    // (profiles/r06/cfg4/ab_NH_CTU_PLAN_4b_r06f.jsonl; the classification runs under the strip loads)
    static const int plan_knob = NH_KNOB("NH_CTU_PLAN", 0);
    static const int w4_knob = NH_KNOB("NH_CTU_W4", 0);   // A/B: int32 levels with registers for 4 waves/SIMD
    (void)w4_knob;
    const bool plan_on = NH_AB && plan_knob != 0 && gs_knob == 4 && persist == 0;
    a.ngroups = (int)groups;
    void* plan_buf = nullptr;
    if (plan_on) {
        NH_HIP(hipMallocAsync(&plan_buf, (size_t)groups * a.ppg * kCtuPlanBytes, s));
        a.plan = (const uint8_t*)plan_buf;
        a.plan_w = (uint8_t*)plan_buf;
    }
    auto launch_plan = [&](auto ctb_c) {
#if NH_AB
        constexpr int C = decltype(ctb_c)::value;
        if (plan_buf) k_ctu_plan<C, 4><<<dim3((unsigned)groups, (unsigned)a.ppg), 256, 0, s>>>(a);
#else
        (void)ctb_c;
#endif
    };
    auto launch_open = [&](auto kern, auto gs_c, int cap_default = 0) -> int {
        constexpr int GSZ = decltype(gs_c)::value;
        const int64_t ngrp = (strips + GSZ - 1) / GSZ;
        if (ngrp * planes > INT32_MAX) return NH_EARG;
        const int items = (int)(ngrp * planes);
        const dim3 grid((unsigned)ngrp, (unsigned)planes);
        const int cap_wgs = cap_knob > 0 ? cap_knob : cap_default > 0 ? cap_default : GSZ == 4 ? 3 : 2;   // (CTB <= 16: the LDS allows 3 anyway)
        if (NH_AB != 0 && persist) {
            int cus = 0, per_cu = 0;
            NH_TRY(device_cus(&cus));
            const unsigned pad = lds_cap(kern, cap_wgs);
            NH_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 64 * GSZ, pad));
            const int res = std::max(1, cus * per_cu);
            kern<<<dim3((unsigned)std::min(items, res), 1), 64 * GSZ, pad, s>>>(a, items);
        } else {
            kern<<<grid, 64 * GSZ, lds_cap(kern, cap_wgs), s>>>(a, items);
        }
        return NH_OK;
    };
    // CTB 32 luma: 32x32 TUs on the matrix cores unless the A/B build says otherwise
    auto launch_ctb = [&](auto ctb_c, auto luma_c) -> int {
        constexpr int C = decltype(ctb_c)::value;
        constexpr bool L = decltype(luma_c)::value;
        constexpr bool M32 = C == 32 && L;
        int rc3;
        launch_plan(ctb_c);
        using G4 = std::integral_constant<int, 4>;
        if (compact) {   // (CTB 16 / 32: the configurations' CTB sizes)
            // registers for 4 waves per SIMD, residency left to registers and LDS (chroma's output images
            // are half the size: 36.8 KB, 4 workgroups per CU): 29.1-29.5 vs 32.5-32.6 us per 4K frame
            // capped at 3 workgroups (profiles/r06/cfg4/ab_env_4bc_r06k.jsonl)
            if constexpr (C == 32) rc3 = launch_open(k_ctu_open<C, L, M32, 0, 4, 4, false, false, int16_t>, G4{}, 5);
            else if constexpr (C == 16) rc3 = launch_open(k_ctu_open<C, L, M32, 0, 4, 4, true, false, int16_t>, G4{}, 5);
            else rc3 = NH_EVALUE;
            k_ctu_wide<C, L, false><<<grid_wide, 256, 0, s>>>(a);
        } else if constexpr (NH_AB != 0) {
            const bool m = M32 && t32 != 0;
            const bool ost_on = (ost_knob & (L ? 1 : 2)) != 0;
            if (m) rc3 = persist == 1   ? launch_open(k_ctu_open<C, L, M32, 1>, G4{})
                         : persist == 2 ? launch_open(k_ctu_open<C, L, M32, 2>, G4{})
                         : gs_knob == 6 ? launch_open(k_ctu_open<C, L, M32, 0, 5, 6>, std::integral_constant<int, 6>{})
                         : gs_knob == 8 ? launch_open(k_ctu_open<C, L, M32, 0, 5, 8>, std::integral_constant<int, 8>{})
                         : ost_on       ? (plan_on ? launch_open(k_ctu_open<C, L, M32, 0, 3, 4, true, true>, G4{})
                                                   : launch_open(k_ctu_open<C, L, M32, 0, 3, 4, true>, G4{}))
                         : plan_on      ? launch_open(k_ctu_open<C, L, M32, 0, 3, 4, false, true>, G4{})
                         : w4_knob      ? launch_open(k_ctu_open<C, L, M32, 0, 4, 4>, G4{})
                                        : launch_open(k_ctu_open<C, L, M32, 0, 3, 4>, G4{});
            else rc3 = persist == 1   ? launch_open(k_ctu_open<C, L, false, 1>, G4{})
                       : persist == 2 ? launch_open(k_ctu_open<C, L, false, 2>, G4{})
                       : gs_knob == 6 ? launch_open(k_ctu_open<C, L, false, 0, 5, 6>, std::integral_constant<int, 6>{})
                       : gs_knob == 8 ? launch_open(k_ctu_open<C, L, false, 0, 5, 8>, std::integral_constant<int, 8>{})
                       : w4_knob && ost_on ? launch_open(k_ctu_open<C, L, false, 0, 4, 4, true>, G4{})
                       : plan_on && ost_on ? launch_open(k_ctu_open<C, L, false, 0, 3, 4, true, true>, G4{})
                       : ost_on       ? launch_open(k_ctu_open<C, L, false, 0, 3, 4, true>, G4{})
                       : plan_on      ? launch_open(k_ctu_open<C, L, false, 0, 3, 4, false, true>, G4{})
                                      : launch_open(k_ctu_open<C, L, false, 0, 3, 4>, G4{});
            if (C == 32 && t32 == 1) k_ctu_wide<C, L, C == 32><<<grid_wide, 256, 0, s>>>(a);
            else k_ctu_wide<C, L, false><<<grid_wide, 256, 0, s>>>(a);
        } else {
            // register budget = the occupancy the LDS allows: 3 waves per SIMD (luma: the
            // cap; chroma (CTB 16): its ~45 KB of LDS -- the strip images plus the output
            // images through which it writes whole rows: 36.8-37.5 vs 37.7-38.3 us per 4K
            // YUV420 frame, luma does not gain (40.0-40.5, profiles/r03/cfg4/ab_ctu_ost.jsonl)
            // -- fit 3 workgroups per CU)
            if constexpr (C == 32) rc3 = launch_open(k_ctu_open<C, L, M32, 0, 3, 4>, G4{});
            else rc3 = launch_open(k_ctu_open<C, L, M32, 0, 3, 4, true>, G4{});
            k_ctu_wide<C, L, false><<<grid_wide, 256, 0, s>>>(a);
        }
        return rc3;
    };
    using std::integral_constant;
    int rc2 = NH_OK;
    switch (ctb) {
        case 4: rc2 = is_luma ? launch_ctb(integral_constant<int, 4>{}, std::true_type{})
                              : launch_ctb(integral_constant<int, 4>{}, std::false_type{}); break;
        case 8: rc2 = is_luma ? launch_ctb(integral_constant<int, 8>{}, std::true_type{})
                              : launch_ctb(integral_constant<int, 8>{}, std::false_type{}); break;
        case 16: rc2 = is_luma ? launch_ctb(integral_constant<int, 16>{}, std::true_type{})
                               : launch_ctb(integral_constant<int, 16>{}, std::false_type{}); break;
        case 32: rc2 = is_luma ? launch_ctb(integral_constant<int, 32>{}, std::true_type{})
                               : launch_ctb(integral_constant<int, 32>{}, std::false_type{}); break;
        default: rc2 = NH_EVALUE;
    }
    if (plan_buf) NH_HIP(hipFreeAsync(plan_buf, s));   // (stream-ordered: after the kernels that read it)
    if (rc2) return rc2;
    NH_HIP(hipGetLastError());
    return NH_OK;
}

// Config 5's narrow launch over one plane set (full 32x32 blocks only); levels
// of lvl_bytes = 4 / 2 / 1 bytes (int32, or the compact int16 / int8 levels).
int tc32_narrow_launch(const int16_t* src, void* lvl, int lvl_bytes, int16_t* rec, const nh_plane_set& S,
                       const QuantParams& q, int dqs, int dq_per, uint32_t* wide_flag, uint32_t epoch, hipStream_t s) {
    const int rc = ensure_basis_ctu();
    if (rc) return rc;
    if (lvl_bytes != 4 && lvl_bytes != 2 && lvl_bytes != 1) return NH_EARG;
    CtuArgs a{};
    a.src = src + S.base;
    a.lvl = (int32_t*)((char*)lvl + S.base * lvl_bytes);   // k_tc32_hd<KB, LT> reads it as LT*
    a.rec = rec + S.base;
    a.group_stride = S.group_stride;
    a.plane_stride = S.plane_stride;
    a.w = S.width;
    a.h = S.height;
    a.pitch = S.pitch;
    a.ppg = S.planes_per_group;
    a.strips_x = S.width / 32;
    a.nrows = S.height / 32;
    a.q[3] = q;
    a.dqs = dqs;
    a.dq_per = dq_per;
    a.wide_flag = wide_flag;
    a.epoch = epoch;
    const int nblk = a.strips_x * a.nrows, planes = S.planes_per_group * S.num_groups;
    if (!nblk || !planes) return NH_OK;
    if (!wide_flag) {   // k_tc32_hd's wait counts assume the wide path's two stores
        set_error("tc32: the narrow launch needs a wide flag word");
        return NH_EARG;
    }
    // capped at 3 resident workgroups per CU (k_tc32_h: 0.137 vs 0.153 ms per 8K YUV420 frame
    // uncapped; k_tc32_hd's 50 KB of LDS allow 3 anyway).  A/B build:
    // NH_TC32H_CAP = workgroups per CU, NH_TC32H_K = k_tc32_h blocks per wave (2 / 4),
    // NH_TC32H_FORM = 1 XCD-ordered grid, 3 the same with whole-row stores,
    // 4 row-piece stores from registers (the round-2 form), NH_TC32H_BREG = bases in registers.
    static const int cap = NH_KNOB("NH_TC32H_CAP", 3), cap_c = NH_KNOB("NH_TC32H_CAP_C", 3);
    static const int ilv = NH_KNOB("NH_TC32H_ILV", 0);   // A/B: 2 = the round-5 block order (k_tc32_hd !ILV)
    (void)ilv;
    auto launch = [&](auto kern, int K, int wgs, int W = 4) {
        kern<<<dim3((unsigned)((nblk + W * K - 1) / (W * K)), (unsigned)planes), 64 * W, lds_cap(kern, wgs), s>>>(a,
                                                                                                            nblk);
    };
    // two blocks per wave, the second's image by LDS-DMA under the first's chain (k_tc32_hd<2>):
    // 0.0966-0.0976 vs 0.0982-0.0983 ms per 8K YUV420 frame for one block per wave loading its
    // own strip (k_tc32_h, A/B build), 4 / 8 blocks per wave 0.102 / 0.107
    // (profiles/r04/cfg5/ab_tc32hd_r04h.jsonl; A/B knob NH_TC32H_DMA = blocks per wave, 0 = k_tc32_h).
    // Its 16-B DMA pieces need 16-B aligned rows, which nh_tc32_planes guarantees.
    static const int dma = NH_KNOB("NH_TC32H_DMA", 2);
    if (((S.pitch | S.base | S.plane_stride | S.group_stride) & 7) || ((uintptr_t)src & 15)) {
        set_error("tc32: rows must be 16-byte aligned");
        return NH_EARG;
    }
    if (!NH_AB || dma == 2 || lvl_bytes != 4) {
        // compact levels: a 3-KB tile per wave (34 KB per workgroup), so the A/B knob NH_TC32H_CAP_C
        // may also allow 4 resident workgroups per CU
        bool done = false;
#if NH_AB
        {
          // A/B: the round-5 order (NH_TC32H_ILV=2), 4 blocks per wave (NH_TC32H_DMA=4), 8-wave
          // workgroups (NH_TC32H_W=8), nontemporal output stores (NH_TC32H_NT=1)
          static const int wk = NH_KNOB("NH_TC32H_W", 4), nt = NH_KNOB("NH_TC32H_NT", 0);
          if (ilv == 2 || dma == 4 || wk == 8 || nt) {
            done = true;
            auto by_lt = [&](auto kb_c, auto ilv_c, auto w_c, auto nt_c) {
                constexpr int K = decltype(kb_c)::value, WW = decltype(w_c)::value;
                constexpr bool I = decltype(ilv_c)::value, N = decltype(nt_c)::value;
                if (lvl_bytes == 4) launch(k_tc32_hd<K, int32_t, I, WW, N>, K, cap, WW);
                else if (lvl_bytes == 2) launch(k_tc32_hd<K, int16_t, I, WW, N>, K, cap_c, WW);
                else launch(k_tc32_hd<K, int8_t, I, WW, N>, K, cap_c, WW);
            };
            using K2 = std::integral_constant<int, 2>;
            using K4 = std::integral_constant<int, 4>;
            using W4 = std::integral_constant<int, 4>;
            using W8 = std::integral_constant<int, 8>;
            using T = std::true_type;
            using F = std::false_type;
            if (dma == 4) ilv == 2 ? by_lt(K4{}, F{}, W4{}, F{}) : by_lt(K4{}, T{}, W4{}, F{});
            else if (ilv == 2) by_lt(K2{}, F{}, W4{}, F{});   // the round-5 order (blocks 2w, 2w + 1)
            else if (wk == 8) nt ? by_lt(K2{}, T{}, W8{}, T{}) : by_lt(K2{}, T{}, W8{}, F{});
            else by_lt(K2{}, T{}, W4{}, T{});
          }
        }
#endif
        // the 4 waves of a workgroup on 4 horizontally adjacent blocks at a time (ILV): 0.078 vs
        // 0.088-0.090 ms per 8K YUV420 frame (int32 levels), 0.067 vs 0.074 (int16), 0.063 vs 0.065
        // (int8) -- profiles/r06/cfg5/ab_tc32_r06e.jsonl
        if (done) {
        } else if (lvl_bytes == 4) launch(k_tc32_hd<2, int32_t, true>, 2, cap);
        else if (lvl_bytes == 2) launch(k_tc32_hd<2, int16_t, true>, 2, cap_c);
        else launch(k_tc32_hd<2, int8_t, true>, 2, cap_c);
        NH_HIP(hipGetLastError());
        return NH_OK;
    }
#if NH_AB
    static const int kk = NH_KNOB("NH_TC32H_K", 1), form = NH_KNOB("NH_TC32H_FORM", 0);
    if (dma == 4) launch(k_tc32_hd<4>, 4, cap);
    else if (dma == 8) launch(k_tc32_hd<8>, 8, cap);
    else if (kk == 2) launch(k_tc32_h<2, false, true>, 2, cap);
    else if (kk == 4) launch(k_tc32_h<4, false, true>, 4, cap);
    else if (form == 1) launch(k_tc32_h<1, true, false>, 1, cap);
    else if (form == 4) launch(k_tc32_h<1, false, false>, 1, cap);
    else if (form == 3) launch(k_tc32_h<1, true, true>, 1, cap);
    // whole-row output stores: 0.106 vs 0.125 ms per 8K YUV420 frame (forms 2 vs 0 of
    // profiles/r03/cfg5/ab_tc32h_forms.jsonl; the XCD-ordered grid is slower, 0.132)
    else if (NH_KNOB("NH_TC32H_BREG", 0)) launch(k_tc32_h<1, false, true, true>, 1, cap);
    else launch(k_tc32_h<1, false, true>, 1, cap);
#endif
    NH_HIP(hipGetLastError());
    return NH_OK;
}

}  // namespace nh

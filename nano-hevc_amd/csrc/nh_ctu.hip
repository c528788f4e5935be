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
// ...), i.e. 64 4x4 units, one per lane.  The wave
//   1. loads the strip, the row above it and the column left of it into an
//      LDS image with 8-byte coalesced loads (every TU neighbour is then an
//      LDS read);
//   2. classifies its units: lane u descends the quadtree to its unit's leaf
//      (<= 3 hashes), writes the TU map entry, and the TU origins are compacted
//      into per-size LDS lists with wave ballots;
//   3. codes the TUs of the workgroup's 4 strips pooled by size, 64/N at a
//      time: lane l takes column / row l mod N of TU l / N (32-point to 4-point
//      butterflies; the 32x32 TUs alternatively on the int8 matrix cores, one
//      per wave -- A/B only, not faster here), transposes through an LDS tile
//      of the strip (every TU at its own place, so TUs never collide).
// No workgroup barriers (a wave only touches its own LDS slices, and LDS
// executes one wave's instructions in order), no global atomics, no per-size
// relaunch, the source read once.  Levels and recon rows are stored straight
// from the registers (N contiguous int32 / int16 per lane).
// Exactness of the 24-bit multiplies and the 32-bit quantizer: DESIGN.md §4.3,
// §4.4 (the residual is int16).
#include <hip/hip_runtime.h>
#include "nh_common.hpp"
#include "nh_internal.hpp"
#include "nh_mfma.hpp"
#include "nh_packed.hpp"
#include "nh_tree.hpp"

namespace nh {

__constant__ Basis c_basis_ctu;

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
};

__device__ __forceinline__ void wave_sync() { __builtin_amdgcn_wave_barrier(); }

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
    static constexpr int TP = SW + 2, T16 = CTB * TP;
    static_assert((TP / 2) % 2 == 1 && T16 * 2 <= CF * 4, "int16 tile layout");
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
    const int lane = threadIdx.x & 63, j = lane / N, t = lane % N;
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
#pragma unroll
    for (int m = 1; m < N; m <<= 1) sum += __shfl_xor(sum, m, 64);
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
#pragma unroll
    for (int m = 1; m < N; m <<= 1) {
        ed += __shfl_xor(ed, m, 64);
        ep += __shfl_xor(ep, m, 64);
    }
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
            *(int4*)(lrow + k0) = make_int4(L4[0], L4[1], L4[2], L4[3]);
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
        for (int k = 0; k < N / 2; k += 2) *(uint2*)(rrow + 2 * k) = make_uint2(pk[k], pk[k + 1]);
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
template <int N, bool DST, int CTB>
__device__ __forceinline__ void ctu_chain_pk(const CtuArgs& a, const int16_t* s_img, int16_t* s_t16, const uint16_t* list,
                                             int cnt, int b0, const int* s_org, int32_t* __restrict__ lvl,
                                             int16_t* __restrict__ rec) {
    using G = Strip<CTB>;
    constexpr int L2 = Log2<N>::v, S = L2 + 5, IP = G::IP, TP = G::TP, H = N / 2;
    constexpr int32_t BIAS = 1 << (S - 1);
    const ChainQ cq = make_chainq(a.q[L2 - 2], a.dqs, a.dq_per);
    const int lane = threadIdx.x & 63, j = lane / N, t = lane % N;
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
#pragma unroll
    for (int m = 1; m < N; m <<= 1) sum += __shfl_xor(sum, m, 64);
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
#pragma unroll
    for (int m = 1; m < N; m <<= 1) {
        ed += __shfl_xor(ed, m, 64);
        ep += __shfl_xor(ep, m, 64);
    }
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
        int32_t* lrow = lvl + (int64_t)(gy0 + t) * a.pitch + gx0;
#pragma unroll
        for (int k0 = 0; k0 < N; k0 += 4) {
            int32_t L4[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                L4[q] = quant_s(y[k0 + q] >> S, cq.qs, cq.h_v, cq.hneg_v);
                tl[(k0 + q) * TP + st] = (int16_t)dequant_s(L4[q], cq);
            }
            *(int4*)(lrow + k0) = make_int4(L4[0], L4[1], L4[2], L4[3]);
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
        int16_t* rrow = rec + (int64_t)(gy0 + t) * a.pitch + gx0;
#pragma unroll
        for (int m = 0; m < H; m += 2) *(uint2*)(rrow + 2 * m) = make_uint2(pk[m], pk[m + 1]);
    }
}

// A 32x32 TU (a whole CTU of a CTB-32 strip) on the int8 matrix cores: the
// chain of k_tc32_mfma (nh_tc32.hip) with the block, its
// neighbours and the dequantized tile in the strip's LDS image / tile.
__device__ __forceinline__ void ctu_chain32(const CtuArgs& a, const int16_t* img, int32_t* cf, int gx0, int gy0,
                                            int32_t* __restrict__ lvl, int16_t* __restrict__ rec) {
    constexpr int IP = Strip<32>::IP, CP = Strip<32>::CP;   // img[r * IP + c]: sample (r - 1, c), c = -1: left; cf[r * CP + c]
    const ChainQ cq = make_chainq(a.q[3], a.dqs, a.dq_per);
    const int l = threadIdx.x & 63, r = l & 31, hh = l >> 5;
    const int32_t my_nb = hh == 0 ? img[r] : img[(1 + r) * IP - 1];
    int32_t s = my_nb;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
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
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        e_dc += __shfl_xor(e_dc, o, 64);
        e_pl += __shfl_xor(e_pl, o, 64);
    }
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
        *(int4*)(lrow + 8 * q + 4 * hh) = make_int4(L4[0], L4[1], L4[2], L4[3]);
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
        *(uint2*)(rrow + 8 * q + 4 * hh) =
            make_uint2((uint32_t)R4[0] | ((uint32_t)R4[1] << 16), (uint32_t)R4[2] | ((uint32_t)R4[3] << 16));
    }
}

// A workgroup = 4 strips (one per wave for loading and classification); the
// TUs of all 4 strips are pooled per size, so a batch of 64/N TUs fills its
// lanes (a strip alone holds ~half a batch per size), and the batches are
// claimed by the 4 waves in descending cost (32x32 chains first).
template <int CTB, bool LUMA, int WAVES, bool MFMA32>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WAVES))) k_ctu_open(CtuArgs a) {
    using G = Strip<CTB>;
    constexpr int SW = G::SW, UW = G::UW, IP = G::IP;
    __shared__ __attribute__((aligned(16))) int16_t s_img[4 * G::IMG];
    __shared__ int32_t s_cf[4 * G::CF];
    __shared__ uint16_t s_list[4][256];
    __shared__ int s_cnt[4][4], s_org[8], s_next, s_wide[4];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int strip = blockIdx.x * 4 + wv;
    const bool valid = strip < a.strips_x * a.nrows;
    const int pz = blockIdx.y, gz = pz / a.ppg, cz = pz - gz * a.ppg;
    const int64_t poff = (int64_t)gz * a.group_stride + (int64_t)cz * a.plane_stride;
    const int16_t* __restrict__ src = a.src + poff;
    int32_t* lvl = a.lvl + poff;
    int16_t* rec = a.rec + poff;
    const int pid = a.plane_id + cz;
    const int w = a.w, h = a.h, pitch = a.pitch;
    const int sx0 = (strip % a.strips_x) * SW, sy0 = (a.row0 + strip / a.strips_x) * CTB;
    int16_t* img = s_img + wv * G::IMG;

    // ---- 1. each wave: its strip, the row above and the column left, into LDS (8-B loads) ----
    uint32_t hi_bits = 0;   // any sample outside [0, 255]: the workgroup takes the 32-bit chain
    if (valid) {
#pragma unroll
        for (int g0 = 0; g0 < CTB * UW; g0 += 64) {
            const int g = g0 + lane, ry = g / UW, gx = g % UW, x = sx0 + 4 * gx, y = sy0 + ry;
            uint2 v = make_uint2(0u, 0u);   // outside the plane: no TU reads it
            if (x < w && y < h) v = *(const uint2*)(src + (int64_t)y * pitch + x);
            hi_bits |= v.x | v.y;
            *(uint2*)&img[(1 + ry) * IP + 4 + 4 * gx] = v;
        }
        if (lane < UW) {
            const int x = sx0 + 4 * lane;
            uint2 v = make_uint2(0x00800080u, 0x00800080u);   // 128 above the frame (block.py:41)
            if (sy0 > 0 && x < w) v = *(const uint2*)(src + (int64_t)(sy0 - 1) * pitch + x);
            hi_bits |= v.x | v.y;
            *(uint2*)&img[4 + 4 * lane] = v;
        }
        if (lane < CTB) {
            const int y = sy0 + lane;
            const int16_t v = sx0 == 0 ? (int16_t)128 : (y < h ? src[(int64_t)y * pitch + sx0 - 1] : (int16_t)0);
            hi_bits |= (uint16_t)v;
            img[(1 + lane) * IP + 3] = v;
        }
        if (lane == 0) {
            s_org[2 * wv] = sx0;
            s_org[2 * wv + 1] = sy0;
        }
    }
    {
        const uint64_t wide = __ballot((hi_bits & 0xff00ff00u) != 0);
        if (lane == 0) s_wide[wv] = wide != 0;
    }

    // ---- 2. classify the strip's 64 units: leaf size / origin (<= 3 hashes), TU map ----
    bool org = false;
    int ls = 0;
    if (valid) {
        const int ux = lane % UW, uy = lane / UW, x = sx0 + 4 * ux, y = sy0 + 4 * uy;
        const bool in = x < w && y < h;
        int s = CTB, cx = sx0 + (4 * ux / CTB) * CTB, cy = sy0;
        while (s > 4 && (cx + s > w || cy + s > h || tu_split(a.seed, pid, cx, cy, s))) {
            s >>= 1;
            cx += x >= cx + s ? s : 0;
            cy += y >= cy + s ? s : 0;
        }
        ls = s == 4 ? 2 : s == 8 ? 3 : s == 16 ? 4 : 5;
        if (in) a.tu[(int64_t)pz * a.tu_plane + (int64_t)(y >> 2) * (w >> 2) + (x >> 2)] = (uint8_t)ls;
        org = in && cx == x && cy == y;
    }
    uint64_t m[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        m[k] = __ballot(org && ls == k + 2);
        if (lane == 0) s_cnt[wv][k] = __popcll(m[k]);
    }
    if (threadIdx.x == 0) s_next = 0;
    __syncthreads();
    // pool the strips' TUs per size: entry = strip << 6 | unit
    int cnt[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        int off = 0;
        cnt[k] = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            off += q < wv ? s_cnt[q][k] : 0;
            cnt[k] += s_cnt[q][k];
        }
        if (org && ls == k + 2) s_list[k][off + __popcll(m[k] & ((1ull << lane) - 1))] = (uint16_t)(wv << 6 | lane);
    }
    __syncthreads();

    // ---- 3. batches, claimed in descending cost: 32x32 chains, then 16, 8, 4 ----
    // NARROW (every sample of the 4 strips and their neighbours 8-bit): the
    // packed 16-bit chain; otherwise the 32-bit chain (any int16 input).
    const bool narrow =
        __builtin_amdgcn_readfirstlane((s_wide[0] | s_wide[1] | s_wide[2] | s_wide[3] | a.wide_only) == 0);
    int16_t* s_t16 = (int16_t*)s_cf;
    const int n32 = CTB == 32 ? (MFMA32 ? cnt[3] : (cnt[3] + 1) / 2) : 0;
    const int n16 = CTB >= 16 ? (cnt[2] + 3) / 4 : 0, n8 = CTB >= 8 ? (cnt[1] + 7) / 8 : 0, n4 = (cnt[0] + 15) / 16;
    const int total = n32 + n16 + n8 + n4;
#define NH_CHAIN(N, DST, L, B)                                                          \
    if (narrow) ctu_chain_pk<N, DST, CTB>(a, s_img, s_t16, s_list[L], cnt[L], B, s_org, lvl, rec); \
    else ctu_chain<N, DST, CTB>(a, s_img, s_cf, s_list[L], cnt[L], B, s_org, lvl, rec);
    for (;;) {
        int item = 0;
        if (lane == 0) item = atomicAdd(&s_next, 1);
        item = __builtin_amdgcn_readfirstlane(__shfl(item, 0, 64));
        if (item >= total) break;
        if constexpr (CTB == 32) {
            if (item < n32) {
                if constexpr (MFMA32) {   // one TU per wave on the int8 matrix cores (A/B form)
                    const int e = s_list[3][item], sw = e >> 6;
                    ctu_chain32(a, s_img + sw * G::IMG + 4, s_cf + sw * G::CF, s_org[2 * sw], s_org[2 * sw + 1], lvl,
                                rec);
                } else {                  // two TUs per wave, 32-point butterflies
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
}

static int ensure_basis_ctu() {
    static unsigned long long ready = 0;   // one bit per device
    int dev = 0;
    NH_HIP(hipGetDevice(&dev));
    if (dev < 0 || dev >= 64) return NH_EARG;
    if (!(ready >> dev & 1ull)) {
        const Basis b = make_basis();
        NH_HIP(hipMemcpyToSymbol(HIP_SYMBOL(c_basis_ctu), &b, sizeof(b)));
        ready |= 1ull << dev;
    }
    return NH_OK;
}

// Launches k_ctu_open over CTU rows [row0, row1) of every plane of the set.
// Returns NH_EVALUE when the layout does not allow the kernel's vector accesses
// (8-B rows / 16-B level rows): the caller then takes the per-size path.
int ctu_open_launch(const int16_t* src, int32_t* lvl, int16_t* rec, uint8_t* tu, const nh_plane_set* set, int ctb,
                    int plane_id, uint32_t seed, int is_luma, int row0, int row1, const QuantParams* q, int dqs,
                    int dq_per, hipStream_t s) {
    const int64_t planes = (int64_t)set->planes_per_group * set->num_groups;
    if ((set->pitch & 3) || ((set->base | set->plane_stride | set->group_stride) & 3) ||
        (((uintptr_t)src | (uintptr_t)rec) & 7) || ((uintptr_t)lvl & 15))
        return NH_EVALUE;
    const int rc = ensure_basis_ctu();
    if (rc) return rc;
    CtuArgs a{};
    a.src = src + set->base;
    a.lvl = lvl + set->base;
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
    if ((strips + 3) / 4 > INT32_MAX) return NH_EARG;
    const dim3 grid((unsigned)((strips + 3) / 4), (unsigned)planes);
    // 32x32 TUs: 32-point butterflies, two TUs per wave (128 VGPRs, 4 waves/SIMD)
    // by default; the int8-MFMA chain (one TU per wave, capped at 3 waves/SIMD =
    // 168 VGPRs without spills; uncapped 228 registers) measured equal in
    // rocprof (584.7 vs 586.6 us per 16 luma planes), so the
    // north star's rule keeps the butterfly.  A/B build: NH_CTU_T32 = 1 (MFMA) /
    // 0, NH_CTU_WAVES = 1 (compiler) / 3 / 4 / 5, NH_CTU_NARROW = 0 (no packed chain).
    static const int cw = NH_KNOB("NH_CTU_WAVES", 0);
    static const int t32 = NH_KNOB("NH_CTU_T32", 0);
    a.wide_only = NH_KNOB("NH_CTU_NARROW", 1) == 0;
#define NH_CTU(C, W, M)                                                             \
    if (is_luma) k_ctu_open<C, true, W, M><<<grid, 256, 0, s>>>(a);                 \
    else k_ctu_open<C, false, W, M><<<grid, 256, 0, s>>>(a);
    switch (ctb) {
        case 4: NH_CTU(4, 1, false) break;
        case 8: NH_CTU(8, 1, false) break;
        case 16: NH_CTU(16, 1, false) break;
        case 32:
#if NH_AB
            if (t32 == 1) {
                if (cw == 1) { NH_CTU(32, 1, true) break; }
                if (cw == 4) { NH_CTU(32, 4, true) break; }
                NH_CTU(32, 3, true) break;
            }
            if (cw == 3) { NH_CTU(32, 3, false) break; }
            if (cw == 4) { NH_CTU(32, 4, false) break; }
            if (cw == 5) { NH_CTU(32, 5, false) break; }
#endif
            (void)cw;
            (void)t32;
            NH_CTU(32, 1, false) break;
        default: return NH_EVALUE;
    }
#undef NH_CTU
    NH_HIP(hipGetLastError());
    return NH_OK;
}

}  // namespace nh

// nh_fused8x8.hpp -- device code of the hot path shared by the product
// launchers (nh_fused8x8.hip) and the A/B launch forms (ab/nh_fused8x8_ab.hip,
// compiled only into libnanohevc_ab.so).
#pragma once
// Roofline: 128 B in + 128 B out per block (HBM-bound; ~1.2k VALU ops/block).
#include <hip/hip_runtime.h>
#include <mutex>
#include "nh_common.hpp"
#include "nh_internal.hpp"

namespace nh {

struct SetDev {
    int64_t base, plane_stride, group_stride;
    int32_t pitch;
    uint32_t nblocks;
    uint32_t wg_start;  // first workgroup of this set
    FastDiv bpp, bpr, ppg;
    uint32_t blk0;      // index of this set's first block in the launch (epilogue outputs)
};

struct Fused8Args {
    const int16_t* in;
    int16_t* out;
    SetDev set[NH_MAX_PLANE_SETS];
    int32_t nsets;
    QuantS q;
    uint32_t xcd_chunk;   // k_fwd8x8_quant<..., XCD=true> (the default launch): workgroups per XCD run
    uint32_t xcd_rot;     // A/B: XCD x starts its run x * xcd_rot workgroups in (mod the run)
};

typedef int v4i __attribute__((ext_vector_type(4)));

// Cache policy of the streaming accesses: 0 default, 1 nontemporal loads and
// stores, 2 nontemporal loads only, 3 nontemporal stores only; A/B only:
// 4 nontemporal loads + write-through `sc0 sc1` stores (the line leaves L2),
// 5 nontemporal loads + `sc1` stores.
template <int POLICY>
__device__ __forceinline__ v4i ld16(const int16_t* p) {
    if constexpr (POLICY == 1 || POLICY == 2 || POLICY >= 4) return __builtin_nontemporal_load((const v4i*)p);
    else return *(const v4i*)p;
}
template <int POLICY>
__device__ __forceinline__ void st16(int16_t* p, v4i v) {
    if constexpr (POLICY == 1 || POLICY == 3) __builtin_nontemporal_store(v, (v4i*)p);
    else if constexpr (POLICY == 4) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" :: "v"(p), "v"(v) : "memory");
    else if constexpr (POLICY == 5) asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" :: "v"(p), "v"(v) : "memory");
    else *(v4i*)p = v;
}

// Locate block b of set S: element offset of its top-left sample.
__device__ __forceinline__ int64_t block_offset(const SetDev& S, uint32_t b) {
    const uint32_t p = fdiv(b, S.bpp), r = b - p * S.bpp.d;
    const uint32_t by = fdiv(r, S.bpr), bx = r - by * S.bpr.d;
    const uint32_t g = fdiv(p, S.ppg), c = p - g * S.ppg.d;
    return S.base + (int64_t)g * S.group_stride + (int64_t)c * S.plane_stride + (int64_t)by * 8 * S.pitch +
           (int64_t)bx * 8;
}

template <int POLICY>
__device__ __forceinline__ void load_block(const int16_t* src, int32_t pitch, v4i (&raw)[8]) {
#pragma unroll
    for (int i = 0; i < 8; ++i) raw[i] = ld16<POLICY>(src + (int64_t)i * pitch);
}

// One 8x8 block: raw int16 rows -> int16 level rows (the whole fused computation).
// row_fn(i, L) sees each row's 8 levels as they are produced (epilogues).
struct NoRowFn {
    __device__ __forceinline__ void operator()(int, const int32_t (&)[8]) const {}
};
template <class RowFn = NoRowFn>
__device__ __forceinline__ void dct8_quant_block(const v4i (&raw)[8], v4i (&outv)[8], const QuantS& q,
                                                 uint32_t h_v, uint32_t hneg_v, RowFn&& row_fn = RowFn()) {
    uint32_t X[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int w[4] = {raw[i].x, raw[i].y, raw[i].z, raw[i].w};
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            X[i][2 * m] = (uint32_t)(int32_t)(int16_t)(w[m] & 0xffff);
            X[i][2 * m + 1] = (uint32_t)(w[m] >> 16);
        }
    }
    // ---- pass 1: columns, temp = T.X, (acc+128)>>8  (transform.py:179-185) ----
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        uint32_t x[8], y[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) x[k] = X[k][j];
        fwd_dct<8, Mul24>(x, y, 128u);   // rounding constant folded into the accumulators
#pragma unroll
        for (int i = 0; i < 8; ++i) X[i][j] = (uint32_t)((int32_t)y[i] >> 8);
    }
    // ---- pass 2: rows, coeff = temp.T^T  (transform.py:188-194) + quant + pack ----
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        uint32_t y[8];
        fwd_dct<8, Mul24>(X[i], y, 128u);
        int32_t L[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) L[j] = quant_s((int32_t)y[j] >> 8, q, h_v, hneg_v);
        row_fn(i, L);
        int w[4];
#pragma unroll
        for (int m = 0; m < 4; ++m) w[m] = (int)__builtin_amdgcn_perm((uint32_t)L[2 * m + 1], (uint32_t)L[2 * m], 0x05040100u);
        outv[i] = v4i{w[0], w[1], w[2], w[3]};
    }
}

__device__ __forceinline__ int select_set(const Fused8Args& a, SetDev& S, uint32_t wid) {
    int s = 0;
#pragma unroll
    for (int k = 1; k < NH_MAX_PLANE_SETS; ++k)
        if (k < a.nsets && wid >= a.set[k].wg_start) s = k;
    S = a.set[0];
#pragma unroll
    for (int k = 1; k < NH_MAX_PLANE_SETS; ++k)
        if (s == k) S = a.set[k];
    return s;
}
__device__ __forceinline__ int select_set(const Fused8Args& a, SetDev& S) { return select_set(a, S, blockIdx.x); }

// XCD-aware workgroup order: with chunk C the 8C consecutive hardware ids of a
// super-group are renumbered so that XCD x gets C consecutive logical
// workgroups; C = nwg / 8 is xcd_eighths (nh_common.hpp).  The last partial
// super-group keeps the identity order, so the map is a bijection.
__device__ __forceinline__ uint32_t xcd_logical_wg(uint32_t bid, uint32_t chunk) {
    const uint32_t span = 8u * chunk, sup = bid / span;
    if ((sup + 1) * span > gridDim.x) return bid;
    const uint32_t w = bid - sup * span;
    return sup * span + (w & 7u) * chunk + (w >> 3);
}
__device__ __forceinline__ uint32_t xcd_logical_wg_rot(uint32_t bid, uint32_t chunk, uint32_t rot) {
    const uint32_t span = 8u * chunk;
    if (span > gridDim.x || bid >= span) return bid;
    const uint32_t x = bid & 7u, k = (bid >> 3) + x * rot;
    return x * chunk + (k >= chunk ? k - chunk : k);   // x * rot < chunk
}

// One thread = one block.  POLICY: cache policy (ld16/st16); WAVES: minimum
// waves per SIMD requested from the register allocator (1 = compiler choice).
template <int POLICY, int WAVES, int TPB = 256, bool XCD = false>
__global__ void __launch_bounds__(TPB) __attribute__((amdgpu_waves_per_eu(WAVES))) k_fwd8x8_quant(Fused8Args a) {
    const uint32_t wid = !XCD ? blockIdx.x
                       : a.xcd_rot ? xcd_logical_wg_rot(blockIdx.x, a.xcd_chunk, a.xcd_rot)
                                   : xcd_logical_wg(blockIdx.x, a.xcd_chunk);
    SetDev S;
    select_set(a, S, wid);
    uint32_t h_v = a.q.h, hneg_v = a.q.hneg;
    asm volatile("" : "+v"(h_v), "+v"(hneg_v));  // pin the two offsets in VGPRs
    const uint32_t b = (wid - S.wg_start) * (uint32_t)TPB + threadIdx.x;
    if (b >= S.nblocks) return;
    const int64_t off = block_offset(S, b);
    v4i raw[8], outv[8];
    load_block<POLICY>(a.in + off, S.pitch, raw);
    dct8_quant_block(raw, outv, a.q, h_v, hneg_v);
#pragma unroll
    for (int i = 0; i < 8; ++i) st16<POLICY>(a.out + off + (int64_t)i * S.pitch, outv[i]);
}


static inline int build_args(const int16_t* d_res, int16_t* d_lvl, const nh_plane_set* sets, int nsets, int qp,
                      int is_intra, Fused8Args& a, uint32_t& total_wg, int pairs = 0, int tpb = 256) {
    if (!d_res || !d_lvl || !sets || nsets < 1 || nsets > NH_MAX_PLANE_SETS) return NH_EARG;
    if (((uintptr_t)d_res & 15) || ((uintptr_t)d_lvl & 15)) {
        set_error("fwd8x8: buffers must be 16-byte aligned");
        return NH_EARG;
    }
    a = Fused8Args{};
    a.in = d_res;
    a.out = d_lvl;
    a.nsets = nsets;
    int q = qp < 0 ? 0 : (qp > 51 ? 51 : qp);  // quant.py:35
    const int per = q / 6, rem = q % 6;
    const int shift = 14 + per + 3;             // quant.py:77, log2(8) = 3
    QuantParams qp0;
    qp0.mf = quant_scale(rem);
    qp0.off = is_intra ? (1u << shift) / 3 : (1u << shift) / 6;
    qp0.shift = shift;
    a.q = make_quants(qp0);
    uint64_t wg = 0, blk = 0;
    for (int k = 0; k < nsets; ++k) {
        const nh_plane_set& p = sets[k];
        if (p.width < 0 || p.height < 0 || p.pitch < p.width || p.planes_per_group < 1 || p.num_groups < 0 ||
            (p.base | p.plane_stride | p.group_stride | p.pitch) & 7) {
            set_error("fwd8x8: plane set must have pitch>=width and 8-element aligned base/pitch/strides");
            return NH_EARG;
        }
        const uint64_t bpr = p.width / 8, rows = p.height / 8;
        const uint64_t bpp = bpr * rows, planes = (uint64_t)p.planes_per_group * p.num_groups;
        const uint64_t nb = bpp * planes;
        if (nb >= (1ull << 31)) { set_error("fwd8x8: > 2^31 blocks per set"); return NH_EARG; }
        SetDev& d = a.set[k];
        d.base = p.base;
        d.plane_stride = p.plane_stride;
        d.group_stride = p.group_stride;
        d.pitch = p.pitch;
        d.nblocks = (uint32_t)nb;
        d.wg_start = (uint32_t)wg;
        d.bpp = make_fastdiv(bpp ? (uint32_t)bpp : 1);
        d.bpr = make_fastdiv(bpr ? (uint32_t)bpr : 1);
        d.ppg = make_fastdiv((uint32_t)p.planes_per_group);
        d.blk0 = (uint32_t)blk;
        blk += nb;
        const uint64_t nthr = pairs == 2 ? (nb + 1) / 2 : pairs ? (rows * planes + 1) / 2 * bpr : nb;
        wg += (nthr + tpb - 1) / tpb;
    }
    for (int k = nsets; k < NH_MAX_PLANE_SETS; ++k) a.set[k].wg_start = 0xffffffffu;
    if (wg >= (1ull << 31) || blk >= (1ull << 32)) return NH_EARG;
    total_wg = (uint32_t)wg;
    return NH_OK;
}

}  // namespace nh

// nh_fused8x8.hip -- THE HOT PATH (config 2 / north-star metric):
// forward 8x8 integer DCT (transform.py:154-196) fused with quantize_block
// (quant.py:126-137, :41-79) over every full 8x8 block (block.py:68-74) of
// int16 residual planes, int16 levels written back at the block's raster
// position.
//
// Design:
//   * one thread = one 8x8 block, entirely in VGPRs -- no LDS round trip.
//     Lane l of a wave owns block bx0+l of a block row, so each of the 8 row
//     loads is one 16-B dwordx4 per lane = one contiguous 1 KiB segment per
//     wave instruction (and the same for the 8 row stores);
//   * both 1-D passes are the recursive even/odd butterfly of nh_common.hpp
//     (E/O adds + 24-bit mads, v_mad_i32_i24, full rate).  Exactness: int16
//     input => pass-1 operands |O| <= 2^16, pass-2 operands <= 2^18, all
//     within the signed 24-bit multiply; sums stay < 2^31 so the int32 ring of
//     the reference (D1/D2) is reproduced exactly;
//   * quantizer in 4 ops (quant_s in nh_common.hpp: signed v_mad_i32_i24 with a
//     sign-selected offset, exact for |c| <= 2^17 which int16 input guarantees);
//     |level| <= 26214 always fits int16;
//   * workgroups never straddle two plane sets, so the set lookup is scalar.
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
};

typedef int v4i __attribute__((ext_vector_type(4)));

// Cache policy of the streaming accesses: 0 default, 1 nontemporal loads and
// stores, 2 nontemporal loads only, 3 nontemporal stores only.
template <int POLICY>
__device__ __forceinline__ v4i ld16(const int16_t* p) {
    if constexpr (POLICY == 1 || POLICY == 2) return __builtin_nontemporal_load((const v4i*)p);
    else return *(const v4i*)p;
}
template <int POLICY>
__device__ __forceinline__ void st16(int16_t* p, v4i v) {
    if constexpr (POLICY == 1 || POLICY == 3) __builtin_nontemporal_store(v, (v4i*)p);
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

__device__ __forceinline__ int select_set(const Fused8Args& a, SetDev& S) {
    int s = 0;
#pragma unroll
    for (int k = 1; k < NH_MAX_PLANE_SETS; ++k)
        if (k < a.nsets && blockIdx.x >= a.set[k].wg_start) s = k;
    S = a.set[0];
#pragma unroll
    for (int k = 1; k < NH_MAX_PLANE_SETS; ++k)
        if (s == k) S = a.set[k];
    return s;
}

// One thread = one block.  POLICY: cache policy (ld16/st16); WAVES: minimum
// waves per SIMD requested from the register allocator (1 = compiler choice).
template <int POLICY, int WAVES>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WAVES))) k_fwd8x8_quant(Fused8Args a) {
    SetDev S;
    select_set(a, S);
    uint32_t h_v = a.q.h, hneg_v = a.q.hneg;
    asm volatile("" : "+v"(h_v), "+v"(hneg_v));  // pin the two offsets in VGPRs
    const uint32_t b = (blockIdx.x - S.wg_start) * 256u + threadIdx.x;
    if (b >= S.nblocks) return;
    const int64_t off = block_offset(S, b);
    v4i raw[8], outv[8];
    load_block<POLICY>(a.in + off, S.pitch, raw);
    dct8_quant_block(raw, outv, a.q, h_v, hneg_v);
#pragma unroll
    for (int i = 0; i < 8; ++i) st16<POLICY>(a.out + off + (int64_t)i * S.pitch, outv[i]);
}

// ---------------------------------------------------------------------------
// Level-side epilogue (quant.py:153-178): per block
//   nnz  = count_nonzero(levels)            (uint8; is_all_zero == !nnz)
//   bits = int(estimate_bits(levels))       (int32)
// estimate_bits = np.sum(log2(|l|+1) + (|l|>0)*2) in float64: the 64 terms of
// an 8x8 block are summed in numpy's pairwise order for n = 64 (8 running
// accumulators over the flattened block, then ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7))).
// Terms come from a table built on the device with the same log2 expression
// as nh_estimate_bits (|level| <= 26214 for N = 8).
// ---------------------------------------------------------------------------
constexpr int kEbTab = 26215;
__device__ double g_eb_tab[kEbTab];

__global__ void k_init_eb_tab() {
    const int a = blockIdx.x * 256 + threadIdx.x;
    if (a < kEbTab) g_eb_tab[a] = a ? log2((double)(a + 1)) + 2.0 : 0.0;
}

struct EpiArgs {
    uint8_t* nnz;
    int32_t* bits;
};

constexpr int kEbLds = 1024;   // terms for |level| < 1024 staged in LDS (8 KB per workgroup)

template <int POLICY, bool BITS, int WAVES>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WAVES))) k_fwd8x8_quant_epi(Fused8Args a, EpiArgs e) {
    __shared__ double tab[BITS ? kEbLds : 1];
    if constexpr (BITS) {
#pragma unroll
        for (int k = 0; k < kEbLds / 256; ++k) tab[k * 256 + threadIdx.x] = g_eb_tab[k * 256 + threadIdx.x];
        __syncthreads();
    }
    SetDev S;
    select_set(a, S);
    uint32_t h_v = a.q.h, hneg_v = a.q.hneg;
    asm volatile("" : "+v"(h_v), "+v"(hneg_v));
    const uint32_t b = (blockIdx.x - S.wg_start) * 256u + threadIdx.x;
    if (b >= S.nblocks) return;
    const int64_t off = block_offset(S, b);
    v4i raw[8], outv[8];
    load_block<POLICY>(a.in + off, S.pitch, raw);
    dct8_quant_block(raw, outv, a.q, h_v, hneg_v);
#pragma unroll
    for (int i = 0; i < 8; ++i) st16<POLICY>(a.out + off + (int64_t)i * S.pitch, outv[i]);
    int nz = 0;
    bool big = false;
    double r[8];
    // row by row (r[c] = numpy's running sum c over the flattened block); the
    // fast path reads only the LDS table, blocks with a |level| >= kEbLds
    // (rare: low QP) are summed again from the full table below
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int w[4] = {outv[i].x, outv[i].y, outv[i].z, outv[i].w};
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const int l = (int16_t)(c & 1 ? (w[c >> 1] >> 16) : (w[c >> 1] & 0xffff));
            const int av = l < 0 ? -l : l;
            nz += av != 0;
            if constexpr (BITS) {
                big |= av >= kEbLds;
                const double t = tab[av < kEbLds ? av : 0];   // tab[0] == 0
                r[c] = i ? r[c] + t : t;
            }
        }
        if constexpr (BITS) __builtin_amdgcn_sched_barrier(0);   // <= 8 term loads in flight
    }
    if constexpr (BITS) {
        if (big) {
#pragma unroll 1
            for (int i = 0; i < 8; ++i) {
                const int w[4] = {outv[i].x, outv[i].y, outv[i].z, outv[i].w};
#pragma unroll
                for (int c = 0; c < 8; ++c) {
                    const int l = (int16_t)(c & 1 ? (w[c >> 1] >> 16) : (w[c >> 1] & 0xffff));
                    const double t = g_eb_tab[l < 0 ? -l : l];
                    r[c] = i ? r[c] + t : t;
                }
            }
        }
    }
    const uint32_t gb = S.blk0 + b;
    if (e.nnz) e.nnz[gb] = (uint8_t)nz;
    if constexpr (BITS)
        e.bits[gb] = (int32_t)(((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7])));
}

// Vertical-pair form: one thread = blocks b and b + blocks_per_row (block rows
// 2r and 2r+1 of the set's linear row numbering; a pair may straddle two
// planes, block_offset handles that).  16 row loads in flight per lane; the
// pattern probe of this shape streams ~4 % faster than the one-block form
// (profiles/r01/ab_shapes.json).
template <int POLICY, int WAVES>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WAVES))) k_fwd8x8_quant_v2(Fused8Args a) {
    SetDev S;
    select_set(a, S);
    uint32_t h_v = a.q.h, hneg_v = a.q.hneg;
    asm volatile("" : "+v"(h_v), "+v"(hneg_v));
    const uint32_t t = (blockIdx.x - S.wg_start) * 256u + threadIdx.x;
    const uint32_t r = fdiv(t, S.bpr), c = t - r * S.bpr.d;
    const uint32_t b0 = 2 * r * S.bpr.d + c, b1 = b0 + S.bpr.d;
    if (b0 >= S.nblocks) return;
    const bool two = b1 < S.nblocks;
    const int64_t o0 = block_offset(S, b0), o1 = two ? block_offset(S, b1) : o0;
    v4i raw0[8], raw1[8], outv[8];
    load_block<POLICY>(a.in + o0, S.pitch, raw0);
    if (two) load_block<POLICY>(a.in + o1, S.pitch, raw1);
    dct8_quant_block(raw0, outv, a.q, h_v, hneg_v);
#pragma unroll
    for (int i = 0; i < 8; ++i) st16<POLICY>(a.out + o0 + (int64_t)i * S.pitch, outv[i]);
    if (two) {
        dct8_quant_block(raw1, outv, a.q, h_v, hneg_v);
#pragma unroll
        for (int i = 0; i < 8; ++i) st16<POLICY>(a.out + o1 + (int64_t)i * S.pitch, outv[i]);
    }
}

// Persistent, software-pipelined form: a fixed grid of workgroups walks the
// 256-block tiles with stride gridDim.x; each thread prefetches its block of
// the NEXT tile (8 x 16 B) before computing the current one, so every wave
// keeps a tile of loads in flight under its own compute.
// Set descriptor of a tile, read from the kernarg segment with a wave-uniform
// index (scalar loads; indexing the by-value argument struct dynamically would
// make the compiler copy it to scratch).
__device__ __forceinline__ bool tile_set(const Fused8Args& a, uint32_t tile, SetDev& S) {
    int s = 0;
#pragma unroll
    for (int k = 1; k < NH_MAX_PLANE_SETS; ++k)
        if (k < a.nsets && tile >= a.set[k].wg_start) s = k;
    s = __builtin_amdgcn_readfirstlane(s);
    const Fused8Args* ka = (const Fused8Args*)__builtin_amdgcn_kernarg_segment_ptr();
    S = ka->set[s];
    return true;
}

template <int POLICY, int WAVES>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WAVES)))
k_fwd8x8_quant_pipe(Fused8Args a, uint32_t ntiles) {
    uint32_t h_v = a.q.h, hneg_v = a.q.hneg;
    asm volatile("" : "+v"(h_v), "+v"(hneg_v));
    uint32_t tile = blockIdx.x;
    if (tile >= ntiles) return;
    SetDev S;
    tile_set(a, tile, S);
    uint32_t b = (tile - S.wg_start) * 256u + threadIdx.x;
    int64_t off = b < S.nblocks ? block_offset(S, b) : -1;
    v4i raw[8];
    if (off >= 0) load_block<POLICY>(a.in + off, S.pitch, raw);
    for (;;) {
        const uint32_t nt = tile + gridDim.x;
        SetDev Sn = S;
        int64_t noff = -1;
        v4i nraw[8];
        if (nt < ntiles) {
            tile_set(a, nt, Sn);
            const uint32_t nb = (nt - Sn.wg_start) * 256u + threadIdx.x;
            if (nb < Sn.nblocks) {
                noff = block_offset(Sn, nb);
                load_block<POLICY>(a.in + noff, Sn.pitch, nraw);
            }
        }
        if (off >= 0) {
            v4i outv[8];
            dct8_quant_block(raw, outv, a.q, h_v, hneg_v);
#pragma unroll
            for (int i = 0; i < 8; ++i) st16<POLICY>(a.out + off + (int64_t)i * S.pitch, outv[i]);
        }
        if (nt >= ntiles) break;
        tile = nt;
        S = Sn;
        off = noff;
#pragma unroll
        for (int i = 0; i < 8; ++i) raw[i] = nraw[i];
    }
}

// Memory-only probe with the kernel's exact access pattern (8 rows x 16 B per
// thread, same block walk): copies input to output.  Measurement helper for the
// achievable-bandwidth ceiling of this pattern; not a product path.
template <int POLICY>
__global__ void __launch_bounds__(256) k_probe_copy8x8(Fused8Args a) {
    SetDev S;
    select_set(a, S);
    const uint32_t b = (blockIdx.x - S.wg_start) * 256u + threadIdx.x;
    if (b >= S.nblocks) return;
    const int64_t off = block_offset(S, b);
    v4i raw[8];
    load_block<POLICY>(a.in + off, S.pitch, raw);
#pragma unroll
    for (int i = 0; i < 8; ++i) st16<POLICY>(a.out + off + (int64_t)i * S.pitch, raw[i]);
}

// Shape probes (same copy, 2 blocks per thread): SHAPE 1 = the horizontally
// adjacent pair (b, b+1: 32 B per row per lane), 2 = lane-interleaved pair
// (b, b+64 within a wave's 128 blocks: two contiguous 1 KiB runs per row),
// 3 = vertical pair (b, b + blocks_per_row: 16 rows).  Blocks are taken in
// pairs of the set's block walk; the launch has twice the workgroups needed.
template <int POLICY, int SHAPE>
__global__ void __launch_bounds__(256) k_probe_copy8x8_pair(Fused8Args a) {
    SetDev S;
    select_set(a, S);
    const uint32_t t = (blockIdx.x - S.wg_start) * 256u + threadIdx.x;
    uint32_t b0, b1;
    if (SHAPE == 1) { b0 = 2 * t; b1 = b0 + 1; }
    else if (SHAPE == 2) { b0 = (t / 64) * 128 + (t % 64); b1 = b0 + 64; }
    else { const uint32_t r = t / S.bpr.d, c = t - r * S.bpr.d; b0 = 2 * r * S.bpr.d + c; b1 = b0 + S.bpr.d; }
    if (b1 >= S.nblocks) return;   // (probe: a ragged tail is skipped)
    const int64_t o0 = block_offset(S, b0), o1 = block_offset(S, b1);
    v4i r0[8], r1[8];
    load_block<POLICY>(a.in + o0, S.pitch, r0);
    load_block<POLICY>(a.in + o1, S.pitch, r1);
#pragma unroll
    for (int i = 0; i < 8; ++i) st16<POLICY>(a.out + o0 + (int64_t)i * S.pitch, r0[i]);
#pragma unroll
    for (int i = 0; i < 8; ++i) st16<POLICY>(a.out + o1 + (int64_t)i * S.pitch, r1[i]);
}

// Memory-only probe: plain linear streaming copy of n 16-B chunks (grid-stride),
// the HBM ceiling this device reaches with the simplest possible pattern.
template <int POLICY>
__global__ void __launch_bounds__(256) k_probe_linear(const int16_t* __restrict__ in, int16_t* __restrict__ out,
                                                     int64_t nchunks) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nchunks; i += stride)
        st16<POLICY>(out + i * 8, ld16<POLICY>(in + i * 8));
}

// pairs: 1 = one thread per vertical block pair (rows 2r, 2r+1 of the set's
// linear block-row numbering): per set ceil(rows/2) * blocks_per_row threads.
static int build_args(const int16_t* d_res, int16_t* d_lvl, const nh_plane_set* sets, int nsets, int qp,
                      int is_intra, Fused8Args& a, uint32_t& total_wg, int pairs = 0) {
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
        const uint64_t nthr = pairs ? (rows * planes + 1) / 2 * bpr : nb;
        wg += (nthr + 255) / 256;
    }
    for (int k = nsets; k < NH_MAX_PLANE_SETS; ++k) a.set[k].wg_start = 0xffffffffu;
    if (wg >= (1ull << 31) || blk >= (1ull << 32)) return NH_EARG;
    total_wg = (uint32_t)wg;
    return NH_OK;
}

}  // namespace nh

using namespace nh;

static constexpr int kDefaultVariant = 5;

extern "C" int nh_fwd8x8_quant_planes_variant(const int16_t* d_res, int16_t* d_lvl, const nh_plane_set* sets,
                                              int nsets, int qp, int is_intra, int variant, void* stream) {
    // variant = cache policy (0..3, see ld16/st16) + 4 * occupancy class (0 compiler, 1 >= 5 waves/SIMD)
    //           + 8 * persistent software-pipelined form (grid = min(tiles, 256 CUs x 8))
    //           + 16 * vertical block pair per thread (with occ: >= 4 waves/SIMD)
    const int policy = variant & 3, occ = (variant >> 2) & 1, pipe = (variant >> 3) & 1, pair = (variant >> 4) & 1;
    if (variant < 0 || variant > 31 || (pipe && pair)) return NH_EARG;
    Fused8Args a;
    uint32_t wg = 0;
    int rc = build_args(d_res, d_lvl, sets, nsets, qp, is_intra, a, wg, pair);
    if (rc) return rc;
    if (!wg) return NH_OK;
    hipStream_t s = as_stream(stream);
    if (pair) {
#define NH_V(P) do { if (occ) k_fwd8x8_quant_v2<P, 4><<<wg, 256, 0, s>>>(a); else k_fwd8x8_quant_v2<P, 1><<<wg, 256, 0, s>>>(a); } while (0)
        switch (policy) {
            case 0: NH_V(0); break;
            case 1: NH_V(1); break;
            case 2: NH_V(2); break;
            default: NH_V(3); break;
        }
#undef NH_V
        NH_HIP(hipGetLastError());
        return NH_OK;
    }
    if (pipe) {
        const uint32_t g = wg < 2048u ? wg : 2048u;
#define NH_P(P) do { if (occ) k_fwd8x8_quant_pipe<P, 4><<<g, 256, 0, s>>>(a, wg); else k_fwd8x8_quant_pipe<P, 1><<<g, 256, 0, s>>>(a, wg); } while (0)
        switch (policy) {
            case 0: NH_P(0); break;
            case 1: NH_P(1); break;
            case 2: NH_P(2); break;
            default: NH_P(3); break;
        }
#undef NH_P
        NH_HIP(hipGetLastError());
        return NH_OK;
    }
#define NH_L(P) do { if (occ) k_fwd8x8_quant<P, 5><<<wg, 256, 0, s>>>(a); else k_fwd8x8_quant<P, 1><<<wg, 256, 0, s>>>(a); } while (0)
    switch (policy) {
        case 0: NH_L(0); break;
        case 1: NH_L(1); break;
        case 2: NH_L(2); break;
        default: NH_L(3); break;
    }
#undef NH_L
    NH_HIP(hipGetLastError());
    return NH_OK;
}

extern "C" int nh_fwd8x8_quant_planes(const int16_t* d_res, int16_t* d_lvl, const nh_plane_set* sets, int nsets,
                                      int qp, int is_intra, void* stream) {
    // default launch = variant 5: nontemporal loads+stores (streamed once, keep
    // them out of L2/MALL) and >= 5 waves/SIMD (74 VGPRs -> 6 waves); fastest
    // in the interleaved A/B (profiles/r01/ab_variants.json).
    return nh_fwd8x8_quant_planes_variant(d_res, d_lvl, sets, nsets, qp, is_intra, kDefaultVariant, stream);
}

extern "C" int nh_probe_copy8x8_planes(const int16_t* d_in, int16_t* d_out, const nh_plane_set* sets, int nsets,
                                       int policy, void* stream) {
    // policy = cache policy (0..3) + 4 * shape (0 = the kernel's pattern, 1..3 = pair probes)
    const int shape = policy >> 2;
    policy &= 3;
    if (shape < 0 || shape > 3) return NH_EARG;
    Fused8Args a;
    uint32_t wg = 0;
    int rc = build_args(d_in, d_out, sets, nsets, 32, 1, a, wg);
    if (rc) return rc;
    if (!wg) return NH_OK;
    hipStream_t s = as_stream(stream);
    if (shape) {
#define NH_PP(P) do { if (shape == 1) k_probe_copy8x8_pair<P, 1><<<wg, 256, 0, s>>>(a); \
                      else if (shape == 2) k_probe_copy8x8_pair<P, 2><<<wg, 256, 0, s>>>(a); \
                      else k_probe_copy8x8_pair<P, 3><<<wg, 256, 0, s>>>(a); } while (0)
        if (policy == 1) NH_PP(1); else NH_PP(0);
#undef NH_PP
        NH_HIP(hipGetLastError());
        return NH_OK;
    }
    switch (policy) {
        case 0: k_probe_copy8x8<0><<<wg, 256, 0, s>>>(a); break;
        case 1: k_probe_copy8x8<1><<<wg, 256, 0, s>>>(a); break;
        case 2: k_probe_copy8x8<2><<<wg, 256, 0, s>>>(a); break;
        default: k_probe_copy8x8<3><<<wg, 256, 0, s>>>(a); break;
    }
    NH_HIP(hipGetLastError());
    return NH_OK;
}

extern "C" int nh_probe_copy_linear(const int16_t* d_in, int16_t* d_out, int64_t nelems, int policy, int grid,
                                    void* stream) {
    if (!d_in || !d_out || nelems < 0 || (nelems & 7) || policy < 0 || policy > 3) return NH_EARG;
    hipStream_t s = as_stream(stream);
    const int64_t chunks = nelems / 8;
    int64_t g = grid > 0 ? grid : (chunks + 255) / 256;
    if (g > (1 << 30)) g = 1 << 30;
    if (!chunks) return NH_OK;
    switch (policy) {
        case 0: k_probe_linear<0><<<(unsigned)g, 256, 0, s>>>(d_in, d_out, chunks); break;
        case 1: k_probe_linear<1><<<(unsigned)g, 256, 0, s>>>(d_in, d_out, chunks); break;
        case 2: k_probe_linear<2><<<(unsigned)g, 256, 0, s>>>(d_in, d_out, chunks); break;
        default: k_probe_linear<3><<<(unsigned)g, 256, 0, s>>>(d_in, d_out, chunks); break;
    }
    NH_HIP(hipGetLastError());
    return NH_OK;
}

extern "C" int nh_fwd8x8_quant_planes_ex(const int16_t* d_res, int16_t* d_lvl, const nh_plane_set* sets, int nsets,
                                         int qp, int is_intra, uint8_t* d_nnz, int32_t* d_bits, void* stream) {
    Fused8Args a;
    uint32_t wg = 0;
    int rc = build_args(d_res, d_lvl, sets, nsets, qp, is_intra, a, wg);
    if (rc) return rc;
    if (!wg) return NH_OK;
    hipStream_t s = as_stream(stream);
    if (d_bits) {   // the term table, once per device (stream-ordered before first use)
        static std::mutex mu;
        static bool ready[64] = {};
        int dev = 0;
        NH_HIP(hipGetDevice(&dev));
        std::lock_guard<std::mutex> lk(mu);
        if (dev < 0 || dev >= 64) return NH_EARG;
        if (!ready[dev]) {
            k_init_eb_tab<<<(kEbTab + 255) / 256, 256, 0, s>>>();
            NH_HIP(hipGetLastError());
            NH_HIP(hipStreamSynchronize(s));
            ready[dev] = true;
        }
    }
    EpiArgs e{d_nnz, d_bits};
    // occupancy targets: the largest without spills (bits: 104 VGPRs, nnz only: 75)
    if (d_bits) k_fwd8x8_quant_epi<1, true, 4><<<wg, 256, 0, s>>>(a, e);
    else k_fwd8x8_quant_epi<1, false, 5><<<wg, 256, 0, s>>>(a, e);
    NH_HIP(hipGetLastError());
    return NH_OK;
}

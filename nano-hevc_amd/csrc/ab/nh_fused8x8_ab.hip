// ab/nh_fused8x8_ab.hip -- the A/B launch forms of the hot path and the memory
// probes: compiled only into libnanohevc_ab.so (make ab),
// never into the product library.  Same device code as the product
// (../nh_fused8x8.hpp); nh_fused8x8.hip dispatches every non-default launch
// variant here through nh_fwd8x8_ab_variant (a weak stub in the product).
#include <hip/hip_runtime.h>
#include <string>
#include "../nh_fused8x8.hpp"

namespace nh {

// Horizontal-pair form (A/B): one thread = blocks 2p and 2p+1 (left / right
// neighbours in a block row when blocks per row is even), so a wave covers
// 2 KiB of each of the 8 rows and a 256-thread workgroup 8 KiB -- about one
// whole 4K luma stripe row -- with 16 row loads in flight per lane; workgroups
// in the XCD-aware order.
template <int POLICY>
__global__ void __launch_bounds__(256) k_fwd8x8_quant_h2(Fused8Args a) {
    const uint32_t wid = xcd_eighths(blockIdx.x, gridDim.x);
    SetDev S;
    select_set(a, S, wid);
    uint32_t h_v = a.q.h, hneg_v = a.q.hneg;
    asm volatile("" : "+v"(h_v), "+v"(hneg_v));
    const uint32_t b0 = 2u * ((wid - S.wg_start) * 256u + threadIdx.x);
    if (b0 >= S.nblocks) return;
    const bool two = b0 + 1 < S.nblocks;
    const int64_t o0 = block_offset(S, b0), o1 = two ? block_offset(S, b0 + 1) : o0;
    v4i raw0[8], raw1[8], outv[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        raw0[i] = ld16<POLICY>(a.in + o0 + (int64_t)i * S.pitch);
        if (two) raw1[i] = ld16<POLICY>(a.in + o1 + (int64_t)i * S.pitch);
    }
    dct8_quant_block(raw0, outv, a.q, h_v, hneg_v);
#pragma unroll
    for (int i = 0; i < 8; ++i) st16<POLICY>(a.out + o0 + (int64_t)i * S.pitch, outv[i]);
    if (two) {
        dct8_quant_block(raw1, outv, a.q, h_v, hneg_v);
#pragma unroll
        for (int i = 0; i < 8; ++i) st16<POLICY>(a.out + o1 + (int64_t)i * S.pitch, outv[i]);
    }
}


// Vertical-pair form: one thread = blocks b and b + blocks_per_row (block rows
// 2r and 2r+1 of the set's linear row numbering; a pair may straddle two
// planes, block_offset handles that).  16 row loads in flight per lane; the
// pattern probe of this shape streams ~4 % faster than the one-block form
// (round-1 probe; its record was not kept).
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

// ---------------------------------------------------------------------------
// Stripe form: HBM access in linear order.  A workgroup (512 threads) owns a
// tile of k whole 8-row stripes of one plane (k*8 rows x all full blocks of a
// row; k chosen on the host so a tile is ~60 KiB: 1 stripe of a 4K luma plane,
// 2 of a 4K chroma plane).  When the plane's pitch equals its processed width
// the tile is ONE contiguous byte range (the stripe form requires it), so
//   load phase : chunk q (16 B) of the tile -> LDS byte 16q, q = it*512 + t
//                (every wave instruction = 1 KiB, consecutive instructions of a
//                workgroup = consecutive 8 KiB: a linear stream);
//   compute    : thread = block, its 8 rows read from / written back to LDS
//                (ds_read/write_b128, consecutive lanes = consecutive 16 B:
//                conflict-free);
//   store phase: the same linear walk from LDS to HBM.
// STAGE 0 = LDS-DMA (global_load_lds_dwordx4, no VGPR staging), 1 = register
// staging (global_load_dwordx4 + ds_write_b128).  COPY = memory-only probe
// (the compute phase is skipped: the access pattern's ceiling).
// ---------------------------------------------------------------------------
struct StripeSetDev {
    int64_t base, plane_stride, group_stride;
    int32_t pitch;
    uint32_t bpr;        // full blocks per row (= 16-B chunks per row of the tile)
    uint32_t rows;       // block rows (stripes) per plane
    uint32_t k;          // stripes per tile
    uint32_t wg_start;   // first workgroup of this set
    FastDiv tpp, ppg, cw; // tiles per plane, planes per group, blocks per row (= bpr)
};

struct StripeArgs {
    const int16_t* in;
    int16_t* out;
    StripeSetDev set[NH_MAX_PLANE_SETS];
    int32_t nsets;
    QuantS q;
    int32_t xcd;   // XCD-aware workgroup order (xcd_eighths), A/B
};

constexpr int kStripeThreads = 512;

template <int POLICY, int STAGE, bool COPY>
__global__ void __launch_bounds__(kStripeThreads) k_fwd8x8_quant_stripe(StripeArgs a) {
    extern __shared__ __attribute__((aligned(16))) int16_t tile[];
    const uint32_t wid = a.xcd ? xcd_eighths(blockIdx.x, gridDim.x) : blockIdx.x;
    int s = 0;
#pragma unroll
    for (int k = 1; k < NH_MAX_PLANE_SETS; ++k)
        if (k < a.nsets && wid >= a.set[k].wg_start) s = k;
    StripeSetDev S = a.set[0];
#pragma unroll
    for (int k = 1; k < NH_MAX_PLANE_SETS; ++k)
        if (s == k) S = a.set[k];
    const uint32_t t = threadIdx.x;
    const uint32_t wt = wid - S.wg_start;
    const uint32_t p = fdiv(wt, S.tpp), ti = wt - p * S.tpp.d;
    const uint32_t g = fdiv(p, S.ppg), c = p - g * S.ppg.d;
    const uint32_t st0 = ti * S.k;
    const uint32_t nst = S.rows - st0 < S.k ? S.rows - st0 : S.k;
    const int64_t tb = S.base + (int64_t)g * S.group_stride + (int64_t)c * S.plane_stride + (int64_t)st0 * 8 * S.pitch;
    const uint32_t nchunks = nst * 8 * S.bpr;
    const int16_t* src = a.in + tb;   // the tile is contiguous (host: pitch == 8 * bpr)
    int16_t* dst = a.out + tb;
    // ---- load phase ----
    if constexpr (STAGE == 0) {
        for (uint32_t q = t; q < nchunks; q += kStripeThreads) {
            // LDS destination = wave-uniform base + lane * 16: q's of a wave are consecutive
            const uint32_t wq = __builtin_amdgcn_readfirstlane(q & ~63u);
            __builtin_amdgcn_global_load_lds((const void*)(src + (int64_t)q * 8),
                                             (__attribute__((address_space(3))) void*)(tile + wq * 8), 16, 0,
                                             (POLICY == 1 || POLICY == 2) ? 2 : 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
        constexpr int kMaxIt = 8;   // host guarantees nchunks <= 8 * 512
        v4i r[kMaxIt];
#pragma unroll
        for (int it = 0; it < kMaxIt; ++it) {
            const uint32_t q = it * kStripeThreads + t;
            if (q < nchunks) r[it] = ld16<POLICY>(src + (int64_t)q * 8);
        }
#pragma unroll
        for (int it = 0; it < kMaxIt; ++it) {
            const uint32_t q = it * kStripeThreads + t;
            if (q < nchunks) *(v4i*)(tile + q * 8) = r[it];
        }
    }
    __syncthreads();
    // ---- compute: thread = block, in place in LDS ----
    if constexpr (!COPY) {
        uint32_t h_v = a.q.h, hneg_v = a.q.hneg;
        asm volatile("" : "+v"(h_v), "+v"(hneg_v));
        const uint32_t nblk = nst * S.bpr;
        const uint32_t W = S.bpr * 8;
        for (uint32_t b = t; b < nblk; b += kStripeThreads) {
            const uint32_t sr = fdiv(b, S.cw), bx = b - sr * S.bpr;
            int16_t* base = tile + sr * 8 * W + bx * 8;
            v4i raw[8], outv[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) raw[i] = *(const v4i*)(base + i * W);
            dct8_quant_block(raw, outv, a.q, h_v, hneg_v);
#pragma unroll
            for (int i = 0; i < 8; ++i) *(v4i*)(base + i * W) = outv[i];
        }
        __syncthreads();
    }
    // ---- store phase ----
    // (4 LDS reads in flight before their stores, not one read-wait-store per chunk)
    for (uint32_t q0 = t; q0 < nchunks; q0 += 4 * kStripeThreads) {
        v4i v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t q = q0 + j * kStripeThreads;
            v[j] = *(const v4i*)(tile + (q < nchunks ? q : q0) * 8);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t q = q0 + j * kStripeThreads;
            if (q < nchunks) st16<POLICY>(dst + (int64_t)q * 8, v[j]);
        }
    }
}

// Persistent, double-buffered stripe form: one 512-thread workgroup per CU walks
// the tiles with stride gridDim.x; the LDS-DMA of tile n+1 (into the other LDS
// buffer) is issued before tile n is computed and stored, so every CU keeps a
// whole tile of loads in flight under its compute and stores.  Waits are
// counted: vmcnt counts loads, stores and LDS-DMA together in issue order
// (MI355X_MICROARCH.md), and after the DMA of tile n+1 a wave issues at least
// floor(chunks / 512) stores of tile n, so vmcnt(that) retires the DMA without
// waiting for those stores.  Raw s_barrier (a __syncthreads() would add vmcnt(0)).
struct TileLoc {
    int64_t tb;          // element offset of the tile
    uint32_t nchunks;    // 16-B chunks (= 8 * blocks)
    uint32_t bpr;
};

__device__ __forceinline__ TileLoc locate_tile(const StripeArgs& a, uint32_t tile) {
    int s = 0;
#pragma unroll
    for (int k = 1; k < NH_MAX_PLANE_SETS; ++k)
        if (k < a.nsets && tile >= a.set[k].wg_start) s = k;
    s = __builtin_amdgcn_readfirstlane(s);
    const StripeArgs* ka = (const StripeArgs*)__builtin_amdgcn_kernarg_segment_ptr();
    const StripeSetDev& S = ka->set[s];
    const uint32_t wt = tile - S.wg_start;
    const uint32_t p = fdiv(wt, S.tpp), ti = wt - p * S.tpp.d;
    const uint32_t g = fdiv(p, S.ppg), c = p - g * S.ppg.d;
    const uint32_t st0 = ti * S.k;
    const uint32_t nst = S.rows - st0 < S.k ? S.rows - st0 : S.k;
    TileLoc L;
    L.tb = S.base + (int64_t)g * S.group_stride + (int64_t)c * S.plane_stride + (int64_t)st0 * 8 * S.pitch;
    L.nchunks = nst * 8 * S.bpr;
    L.bpr = S.bpr;
    return L;
}

__device__ __forceinline__ void wait_vm_at_most(uint32_t n) {   // s_waitcnt vmcnt(n), n wave-uniform
    switch (n) {
        case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
        case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
        case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
        case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
        case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
        case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
        case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
        case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
        case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
        case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
    }
}

template <int POLICY>
__device__ __forceinline__ void glds_tile(const int16_t* src, int16_t* buf, uint32_t nchunks, uint32_t t) {
    for (uint32_t q = t; q < nchunks; q += kStripeThreads) {
        const uint32_t wq = __builtin_amdgcn_readfirstlane(q & ~63u);
        __builtin_amdgcn_global_load_lds((const void*)(src + (int64_t)q * 8),
                                         (__attribute__((address_space(3))) void*)(buf + wq * 8), 16, 0,
                                         (POLICY == 1 || POLICY == 2) ? 2 : 0);
    }
}

template <int POLICY>
__global__ void __launch_bounds__(kStripeThreads) k_fwd8x8_quant_stripe_pipe(StripeArgs a, uint32_t ntiles,
                                                                              uint32_t buf_elems) {
    extern __shared__ __attribute__((aligned(16))) int16_t lds[];
    const uint32_t t = threadIdx.x;
    uint32_t tile = blockIdx.x;
    if (tile >= ntiles) return;
    uint32_t h_v = a.q.h, hneg_v = a.q.hneg;
    asm volatile("" : "+v"(h_v), "+v"(hneg_v));
    TileLoc cur = locate_tile(a, tile);
    glds_tile<POLICY>(a.in + cur.tb, lds, cur.nchunks, t);
    uint32_t pend = 0;   // stores of the previous tile issued after this tile's DMA (lower bound)
    for (uint32_t n = 0;; ++n) {
        int16_t* buf = lds + (n & 1) * buf_elems;
        wait_vm_at_most(pend);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        const uint32_t nxt = tile + gridDim.x;
        TileLoc nl = cur;
        if (nxt < ntiles) {
            nl = locate_tile(a, nxt);
            glds_tile<POLICY>(a.in + nl.tb, lds + ((n + 1) & 1) * buf_elems, nl.nchunks, t);
        }
        // compute: thread = block, in place
        const uint32_t W = cur.bpr * 8, nblk = cur.nchunks / 8;
        for (uint32_t b = t; b < nblk; b += kStripeThreads) {
            const uint32_t sr = b / cur.bpr, bx = b - sr * cur.bpr;
            int16_t* base = buf + sr * 8 * W + bx * 8;
            v4i raw[8], outv[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) raw[i] = *(const v4i*)(base + i * W);
            dct8_quant_block(raw, outv, a.q, h_v, hneg_v);
#pragma unroll
            for (int i = 0; i < 8; ++i) *(v4i*)(base + i * W) = outv[i];
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        // store
        int16_t* dst = a.out + cur.tb;
        for (uint32_t q0 = t; q0 < cur.nchunks; q0 += 4 * kStripeThreads) {
            v4i v[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t q = q0 + j * kStripeThreads;
                v[j] = *(const v4i*)(buf + (q < cur.nchunks ? q : q0) * 8);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t q = q0 + j * kStripeThreads;
                if (q < cur.nchunks) st16<POLICY>(dst + (int64_t)q * 8, v[j]);
            }
        }
        if (nxt >= ntiles) break;
        pend = cur.nchunks / kStripeThreads;
        tile = nxt;
        cur = nl;
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
                                                     int64_t nchunks, int xcd) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    const uint32_t wid = xcd ? xcd_eighths(blockIdx.x, gridDim.x) : blockIdx.x;
    for (int64_t i = (int64_t)wid * 256 + threadIdx.x; i < nchunks; i += stride)
        st16<POLICY>(out + i * 8, ld16<POLICY>(in + i * 8));
}

// Linear probe with M chunks per thread: a workgroup copies 256*M consecutive
// chunks, thread t chunks t + 256 i (every wave instruction 1 KiB; all M loads
// issued before the M stores, as the 8x8 kernel does with its 8 rows).
template <int POLICY, int M>
__global__ void __launch_bounds__(256) k_probe_linear_m(const int16_t* __restrict__ in, int16_t* __restrict__ out,
                                                       int64_t nchunks) {
    const int64_t c0 = (int64_t)blockIdx.x * 256 * M + threadIdx.x;
    v4i v[M];
#pragma unroll
    for (int i = 0; i < M; ++i)
        if (c0 + 256 * i < nchunks) v[i] = ld16<POLICY>(in + (c0 + 256 * i) * 8);
#pragma unroll
    for (int i = 0; i < M; ++i)
        if (c0 + 256 * i < nchunks) st16<POLICY>(out + (c0 + 256 * i) * 8, v[i]);
}

// Row-per-wave probe: a workgroup of 64*R threads owns 64 consecutive blocks of
// the set's block walk; wave w copies rows w*8/R .. of those blocks, one 16-B
// chunk per lane and row (each wave instruction = one 1 KiB row segment; every
// thread moves 8/R chunks instead of 8).
template <int POLICY, int R>
__global__ void __launch_bounds__(64 * R) k_probe_rowwave(Fused8Args a) {
    SetDev S;
    select_set(a, S);
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t b = (blockIdx.x - S.wg_start) * 64u + lane;
    if (b >= S.nblocks) return;
    const int64_t off = block_offset(S, b);
    constexpr int RPW = 8 / R;
    v4i v[RPW];
#pragma unroll
    for (int i = 0; i < RPW; ++i) v[i] = ld16<POLICY>(a.in + off + (int64_t)(w * RPW + i) * S.pitch);
#pragma unroll
    for (int i = 0; i < RPW; ++i) st16<POLICY>(a.out + off + (int64_t)(w * RPW + i) * S.pitch, v[i]);
}

// Row-per-wave probe through LDS with the two workgroup barriers a row-per-lane
// kernel needs (rows in, exchange, levels out): wave w loads row w of 64 blocks,
// ds_write, barrier, every lane reads another lane's chunk back (the transpose
// traffic), barrier, wave w stores row w.
template <int POLICY>
__global__ void __launch_bounds__(512) k_probe_rowwave_lds(Fused8Args a) {
    __shared__ v4i t0[512];
    SetDev S;
    select_set(a, S);
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t b = (blockIdx.x - S.wg_start) * 64u + lane;
    const bool ok = b < S.nblocks;
    const int64_t off = ok ? block_offset(S, b) + (int64_t)w * S.pitch : 0;
    if (ok) t0[threadIdx.x] = ld16<POLICY>(a.in + off);
    __syncthreads();
    v4i v = t0[(threadIdx.x * 8 + (threadIdx.x >> 6)) & 511];   // a transposed read
    __syncthreads();
    t0[(threadIdx.x * 8 + (threadIdx.x >> 6)) & 511] = v;
    __syncthreads();
    if (ok) st16<POLICY>(a.out + off, t0[threadIdx.x]);
}

// pairs: 1 = one thread per vertical block pair (rows 2r, 2r+1 of the set's
// linear block-row numbering): per set ceil(rows/2) * blocks_per_row threads.

// Stripe-form launch description (see k_fwd8x8_quant_stripe).  Returns
// NH_EARG when a set's stripe does not fit the LDS (full blocks per row > 1280).
constexpr uint32_t kStripeTileBytes = 61440;   // ~60 KiB per workgroup: 2 workgroups per CU
constexpr uint32_t kStripeMaxLds = 160 * 1024;

static int build_stripe_args(const int16_t* d_res, int16_t* d_lvl, const nh_plane_set* sets, int nsets, int qp,
                             int is_intra, bool reg_stage, StripeArgs& a, uint32_t& total_wg, uint32_t& lds_bytes) {
    Fused8Args f;
    uint32_t wg0 = 0;
    int rc = build_args(d_res, d_lvl, sets, nsets, qp, is_intra, f, wg0);   // shared validation + quantizer
    if (rc) return rc;
    a = StripeArgs{};
    a.in = d_res;
    a.out = d_lvl;
    a.nsets = nsets;
    a.q = f.q;
    uint64_t wg = 0;
    lds_bytes = 16;
    for (int k = 0; k < nsets; ++k) {
        const nh_plane_set& p = sets[k];
        const uint32_t bpr = (uint32_t)p.width / 8, rows = (uint32_t)p.height / 8;
        const uint64_t planes = (uint64_t)p.planes_per_group * p.num_groups;
        StripeSetDev& d = a.set[k];
        d.base = p.base;
        d.plane_stride = p.plane_stride;
        d.group_stride = p.group_stride;
        d.pitch = p.pitch;
        d.bpr = bpr;
        d.rows = rows;
        d.wg_start = (uint32_t)wg;
        if (!bpr || !rows || !planes) {   // nothing to do in this set
            d.k = 1;
            d.tpp = make_fastdiv(1);
            d.ppg = make_fastdiv((uint32_t)p.planes_per_group);
            d.cw = make_fastdiv(1);
            continue;
        }
        if ((uint32_t)p.pitch != bpr * 8) { set_error("fwd8x8 stripe form: needs pitch == 8 * (width / 8)"); return NH_EARG; }
        const uint32_t stripe_bytes = bpr * 128u;
        if (stripe_bytes > kStripeMaxLds) { set_error("fwd8x8 stripe form: row too wide for LDS"); return NH_EARG; }
        uint32_t kk = kStripeTileBytes / stripe_bytes;
        if (kk < 1) kk = 1;
        if (kk > rows) kk = rows;
        if (reg_stage && kk * 8 * bpr > 8u * kStripeThreads) {
            set_error("fwd8x8 stripe form (register staging): tile > 4096 chunks");
            return NH_EARG;
        }
        d.k = kk;
        const uint32_t tpp = (rows + kk - 1) / kk;
        d.tpp = make_fastdiv(tpp);
        d.ppg = make_fastdiv((uint32_t)p.planes_per_group);
        d.cw = make_fastdiv(bpr);
        if (kk * stripe_bytes > lds_bytes) lds_bytes = kk * stripe_bytes;
        wg += (uint64_t)tpp * planes;
    }
    for (int k = nsets; k < NH_MAX_PLANE_SETS; ++k) a.set[k].wg_start = 0xffffffffu;
    if (wg >= (1ull << 31)) return NH_EARG;
    total_wg = (uint32_t)wg;
    return NH_OK;
}

template <int POLICY, int STAGE, bool COPY>
static int launch_stripe(const StripeArgs& a, uint32_t wg, uint32_t lds, hipStream_t s) {
    static std::once_flag once;
    static hipError_t attr_rc = hipSuccess;
    std::call_once(once, [] {
        attr_rc = hipFuncSetAttribute((const void*)k_fwd8x8_quant_stripe<POLICY, STAGE, COPY>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)kStripeMaxLds);
    });
    NH_HIP(attr_rc);
    k_fwd8x8_quant_stripe<POLICY, STAGE, COPY><<<wg, kStripeThreads, lds, s>>>(a);
    NH_HIP(hipGetLastError());
    return NH_OK;
}

template <int POLICY>
static int launch_stripe_pipe(const StripeArgs& a, uint32_t ntiles, uint32_t lds, hipStream_t s) {
    static std::once_flag once;
    static hipError_t attr_rc = hipSuccess;
    std::call_once(once, [] {
        attr_rc = hipFuncSetAttribute((const void*)k_fwd8x8_quant_stripe_pipe<POLICY>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)kStripeMaxLds);
    });
    NH_HIP(attr_rc);
    int dev = 0, cus = 0;
    NH_HIP(hipGetDevice(&dev));
    NH_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const uint32_t grid = ntiles < (uint32_t)cus ? ntiles : (uint32_t)cus;   // one workgroup per CU (LDS)
    const uint32_t buf_elems = (lds + 15) / 16 * 8;
    k_fwd8x8_quant_stripe_pipe<POLICY><<<grid, kStripeThreads, 2 * buf_elems * 2, s>>>(a, ntiles, buf_elems);
    NH_HIP(hipGetLastError());
    return NH_OK;
}

static int run_stripe_pipe(const int16_t* d_in, int16_t* d_out, const nh_plane_set* sets, int nsets, int qp,
                           int is_intra, int policy, hipStream_t s) {
    StripeArgs a;
    uint32_t wg = 0, lds = 0;
    int rc = build_stripe_args(d_in, d_out, sets, nsets, qp, is_intra, false, a, wg, lds);
    if (rc) return rc;
    if (!wg) return NH_OK;
    if (2 * lds > kStripeMaxLds) { set_error("fwd8x8 pipelined stripe form: two tiles exceed the LDS"); return NH_EARG; }
    switch (policy) {
        case 0: return launch_stripe_pipe<0>(a, wg, lds, s);
        case 1: return launch_stripe_pipe<1>(a, wg, lds, s);
        case 2: return launch_stripe_pipe<2>(a, wg, lds, s);
        default: return launch_stripe_pipe<3>(a, wg, lds, s);
    }
}

static int run_stripe(const int16_t* d_in, int16_t* d_out, const nh_plane_set* sets, int nsets, int qp, int is_intra,
                      int policy, bool reg_stage, bool copy, hipStream_t s, bool xcd = false) {
    StripeArgs a;
    uint32_t wg = 0, lds = 0;
    int rc = build_stripe_args(d_in, d_out, sets, nsets, qp, is_intra, reg_stage, a, wg, lds);
    if (rc) return rc;
    if (!wg) return NH_OK;
    a.xcd = xcd ? 1 : 0;
#define NH_S(P) (reg_stage ? (copy ? launch_stripe<P, 1, true>(a, wg, lds, s) : launch_stripe<P, 1, false>(a, wg, lds, s)) \
                           : (copy ? launch_stripe<P, 0, true>(a, wg, lds, s) : launch_stripe<P, 0, false>(a, wg, lds, s)))
    switch (policy) {
        case 0: return NH_S(0);
        case 1: return NH_S(1);
        case 2: return NH_S(2);
        default: return NH_S(3);
    }
#undef NH_S
}


}  // namespace nh

using namespace nh;
extern "C" int nh_fwd8x8_ab_variant(const int16_t* d_res, int16_t* d_lvl, const nh_plane_set* sets, int nsets,
                                    int qp, int is_intra, int variant, void* stream) {
    if (variant > 32768 && variant <= 32768 + 8) {   // A/B: eighths with XCD x's run rotated by x * r/8 of a run
        Fused8Args a;
        uint32_t wg = 0;
        int rc = build_args(d_res, d_lvl, sets, nsets, qp, is_intra, a, wg);
        if (rc) return rc;
        if (!wg) return NH_OK;
        a.xcd_chunk = wg / 8 ? wg / 8 : 1;
        a.xcd_rot = (a.xcd_chunk * (uint32_t)(variant - 32768)) / 64u;   // x * rot < chunk for x <= 7
        if (!a.xcd_rot) a.xcd_rot = 1;
        k_fwd8x8_quant<1, 5, 256, true><<<wg, 256, 0, as_stream(stream)>>>(a);
        NH_HIP(hipGetLastError());
        return NH_OK;
    }
    if (variant >= 16384 && variant < 16388) {   // horizontal-pair form, XCD order, cache policy variant & 3 (A/B)
        Fused8Args a;
        uint32_t wg = 0;
        int rc = build_args(d_res, d_lvl, sets, nsets, qp, is_intra, a, wg, 2);
        if (rc) return rc;
        if (!wg) return NH_OK;
        hipStream_t s = as_stream(stream);
        switch (variant & 3) {
            case 0: k_fwd8x8_quant_h2<0><<<wg, 256, 0, s>>>(a); break;
            case 1: k_fwd8x8_quant_h2<1><<<wg, 256, 0, s>>>(a); break;
            case 2: k_fwd8x8_quant_h2<2><<<wg, 256, 0, s>>>(a); break;
            default: k_fwd8x8_quant_h2<3><<<wg, 256, 0, s>>>(a); break;
        }
        NH_HIP(hipGetLastError());
        return NH_OK;
    }
    if (variant >= 8192 + 32 && variant < 8192 + 128 && !((variant - 8192) & 28))   // stripe forms + XCD order (A/B)
        return run_stripe(d_res, d_lvl, sets, nsets, qp, is_intra, variant & 3, ((variant - 8192) >> 6) & 1, false,
                          as_stream(stream), true);
    if (variant >= 4096 && variant < 4096 + 16 * 16) {
        const int c = (variant - 4096) >> 4, pol = variant & 3, occ8 = (variant & 12) == 8;
        if ((variant & 12) != 4 && !occ8) return NH_EARG;
        Fused8Args a;
        uint32_t wg = 0;
        int rc = build_args(d_res, d_lvl, sets, nsets, qp, is_intra, a, wg);
        if (rc) return rc;
        if (!wg) return NH_OK;
        a.xcd_chunk = c == 15 ? (wg / 8 ? wg / 8 : 1) : (1u << c);
        hipStream_t s = as_stream(stream);
        if (occ8) {   // A/B: >= 8 waves/SIMD (64 VGPRs)
            if (pol == 1) k_fwd8x8_quant<1, 8, 256, true><<<wg, 256, 0, s>>>(a);
            else k_fwd8x8_quant<3, 8, 256, true><<<wg, 256, 0, s>>>(a);
            NH_HIP(hipGetLastError());
            return NH_OK;
        }
        switch (pol) {
            case 0: k_fwd8x8_quant<0, 5, 256, true><<<wg, 256, 0, s>>>(a); break;
            case 1: k_fwd8x8_quant<1, 5, 256, true><<<wg, 256, 0, s>>>(a); break;
            case 2: k_fwd8x8_quant<2, 5, 256, true><<<wg, 256, 0, s>>>(a); break;
            default: k_fwd8x8_quant<3, 5, 256, true><<<wg, 256, 0, s>>>(a); break;
        }
        NH_HIP(hipGetLastError());
        return NH_OK;
    }
    if (variant == 2052 || variant == 2053) {
        Fused8Args a;
        uint32_t wg = 0;
        int rc = build_args(d_res, d_lvl, sets, nsets, qp, is_intra, a, wg);
        if (rc) return rc;
        if (!wg) return NH_OK;
        hipStream_t s = as_stream(stream);
        if (variant == 2052) k_fwd8x8_quant<4, 5><<<wg, 256, 0, s>>>(a);
        else k_fwd8x8_quant<5, 5><<<wg, 256, 0, s>>>(a);
        NH_HIP(hipGetLastError());
        return NH_OK;
    }
    if (variant >= 256) {
        const int k = variant >> 8, pol = variant & 3, oc = (variant >> 2) & 1;
        if (k > 3 || (variant & 248)) return NH_EARG;
        const int tpb = k == 1 ? 512 : k == 2 ? 1024 : 128;
        Fused8Args a;
        uint32_t wg = 0;
        int rc = build_args(d_res, d_lvl, sets, nsets, qp, is_intra, a, wg, 0, tpb);
        if (rc) return rc;
        if (!wg) return NH_OK;
        hipStream_t s = as_stream(stream);
#define NH_T(P, T) do { if (oc) k_fwd8x8_quant<P, 5, T><<<wg, T, 0, s>>>(a); else k_fwd8x8_quant<P, 1, T><<<wg, T, 0, s>>>(a); } while (0)
#define NH_TT(P) do { if (tpb == 512) NH_T(P, 512); else if (tpb == 1024) NH_T(P, 1024); else NH_T(P, 128); } while (0)
        if (pol == 1) NH_TT(1); else NH_TT(0);
#undef NH_TT
#undef NH_T
        NH_HIP(hipGetLastError());
        return NH_OK;
    }
    const int policy = variant & 3, occ = (variant >> 2) & 1, pipe = (variant >> 3) & 1, pair = (variant >> 4) & 1;
    if (variant >= 128 && variant < 132)
        return run_stripe_pipe(d_res, d_lvl, sets, nsets, qp, is_intra, policy, as_stream(stream));
    if (variant >= 32 && variant < 128 && !(variant & 28))
        return run_stripe(d_res, d_lvl, sets, nsets, qp, is_intra, policy, (variant >> 6) & 1, false, as_stream(stream));
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

extern "C" int nh_probe_copy8x8_planes(const int16_t* d_in, int16_t* d_out, const nh_plane_set* sets, int nsets,
                                       int policy, void* stream) {
    // policy = cache policy (0..3) + 4 * shape (0 = the kernel's pattern, 1..3 = pair probes,
    //          4 = stripe form through LDS by LDS-DMA, 5 = stripe form, register staging)
    const bool xcd = (policy >> 6) & 1;   // + 64: XCD-aware order (stripe shapes only)
    const int shape = (policy >> 2) & 15;
    policy &= 3;
    if (shape == 4 || shape == 5)
        return run_stripe(d_in, d_out, sets, nsets, 32, 1, policy, shape == 5, true, as_stream(stream), xcd);
    if (shape >= 6 && shape <= 8) {   // row-per-wave probes: 8 waves x 1 row, 4 waves x 2 rows per 64 blocks, 8 x 1 via LDS
        Fused8Args a;
        uint32_t wg = 0;
        int rc = build_args(d_in, d_out, sets, nsets, 32, 1, a, wg);
        if (rc) return rc;
        uint64_t wg64 = 0;
        for (int k = 0; k < nsets; ++k) {
            a.set[k].wg_start = (uint32_t)wg64;
            wg64 += (a.set[k].nblocks + 63) / 64;
        }
        if (!wg64) return NH_OK;
        hipStream_t s = as_stream(stream);
#define NH_RW(P) do { if (shape == 8) k_probe_rowwave_lds<P><<<(unsigned)wg64, 512, 0, s>>>(a); \
                      else if (shape == 6) k_probe_rowwave<P, 8><<<(unsigned)wg64, 512, 0, s>>>(a); \
                      else k_probe_rowwave<P, 4><<<(unsigned)wg64, 256, 0, s>>>(a); } while (0)
        if (policy == 1) NH_RW(1); else NH_RW(0);
#undef NH_RW
        NH_HIP(hipGetLastError());
        return NH_OK;
    }
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
    // policy = cache policy (0..3) + 4 * log2(M): M > 1 = k_probe_linear_m (grid ignored)
    //          + 16: XCD-aware workgroup order (xcd_eighths; M = 1 only)
    const int xcd = (policy >> 4) & 1;
    const int lm = (policy >> 2) & 3;
    if (policy >> 5 || (xcd && lm)) return NH_EARG;
    policy &= 3;
    if (!d_in || !d_out || nelems < 0 || (nelems & 7) || lm < 0 || lm > 3) return NH_EARG;
    hipStream_t s = as_stream(stream);
    const int64_t chunks = nelems / 8;
    if (lm) {
        if (!chunks) return NH_OK;
        const int64_t per = 256ll << lm;
        const unsigned gm = (unsigned)((chunks + per - 1) / per);
#define NH_LM(P) do { if (lm == 1) k_probe_linear_m<P, 2><<<gm, 256, 0, s>>>(d_in, d_out, chunks); \
                      else if (lm == 2) k_probe_linear_m<P, 4><<<gm, 256, 0, s>>>(d_in, d_out, chunks); \
                      else k_probe_linear_m<P, 8><<<gm, 256, 0, s>>>(d_in, d_out, chunks); } while (0)
        if (policy == 1) NH_LM(1); else NH_LM(0);
#undef NH_LM
        NH_HIP(hipGetLastError());
        return NH_OK;
    }
    int64_t g = grid > 0 ? grid : (chunks + 255) / 256;
    if (g > (1 << 30)) g = 1 << 30;
    if (!chunks) return NH_OK;
    switch (policy) {
        case 0: k_probe_linear<0><<<(unsigned)g, 256, 0, s>>>(d_in, d_out, chunks, xcd); break;
        case 1: k_probe_linear<1><<<(unsigned)g, 256, 0, s>>>(d_in, d_out, chunks, xcd); break;
        case 2: k_probe_linear<2><<<(unsigned)g, 256, 0, s>>>(d_in, d_out, chunks, xcd); break;
        default: k_probe_linear<3><<<(unsigned)g, 256, 0, s>>>(d_in, d_out, chunks, xcd); break;
    }
    NH_HIP(hipGetLastError());
    return NH_OK;
}

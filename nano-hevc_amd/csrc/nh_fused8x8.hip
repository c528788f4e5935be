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
#include <hip/hip_runtime.h>
#include <mutex>
#include <string>
#include "nh_common.hpp"
#include "nh_internal.hpp"
#include "nh_fused8x8.hpp"

namespace nh {

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
    const uint32_t wid = xcd_eighths(blockIdx.x, gridDim.x);   // XCD-aware order, as the default launch
    SetDev S;
    select_set(a, S, wid);
    uint32_t h_v = a.q.h, hneg_v = a.q.hneg;
    asm volatile("" : "+v"(h_v), "+v"(hneg_v));
    const uint32_t b = (wid - S.wg_start) * 256u + threadIdx.x;
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


}  // namespace nh

using namespace nh;

// Every launch variant other than the default and its plain-order form is an A/B
// form (ab/nh_fused8x8_ab.hip): this weak stub is what the product library links;
// libnanohevc_ab.so links the strong definition.
extern "C" __attribute__((weak)) int nh_fwd8x8_ab_variant(const int16_t*, int16_t*, const nh_plane_set*, int, int, int,
                                                         int variant, void*) {
    set_error("fwd8x8: launch variant " + std::to_string(variant) + " is an A/B form (libnanohevc_ab.so, make ab)");
    return NH_EVALUE;
}

static constexpr int kDefaultVariant = 4096 + 16 * 15 + 5;   // 4341

extern "C" int nh_fwd8x8_quant_planes_variant(const int16_t* d_res, int16_t* d_lvl, const nh_plane_set* sets,
                                              int nsets, int qp, int is_intra, int variant, void* stream) {
    // variant = cache policy (0..3, see ld16/st16) + 4 * occupancy class (0 compiler, 1 >= 5 waves/SIMD)
    //           + 8 * persistent software-pipelined form (grid = min(tiles, 256 CUs x 8))
    //           + 16 * vertical block pair per thread (with occ: >= 4 waves/SIMD)
    //           + 32 * stripe form (linear HBM walk through LDS; +64: register staging instead of LDS-DMA)
    //           + 128 * persistent double-buffered stripe form (LDS-DMA of the next tile under this one)
    //           + 256 * k: the plain form with 512 (k=1), 1024 (k=2) or 128 (k=3) threads per workgroup
    //           2048 + p: the plain form (>= 5 waves/SIMD) with store policy p = 4 / 5 (see st16)
    //           8192 + 32..127: the stripe forms above with the XCD-aware workgroup order (A/B)
    //           16384 + p: horizontal block pair per thread, XCD-aware order, cache policy p (A/B)
    //           4096 + 16 * c + 4 + p: the plain form (>= 5 waves/SIMD, cache policy p; + 8 instead of + 4:
    //           >= 8 waves/SIMD, p = 1 or 3) with XCD-aware workgroup
    //           order, chunk 2^c workgroups (c = 15: 1/8 of the grid); 4341 = policy 1, eighths: the default
    // The product library carries the default (4341) and its plain-order form (5); every other
    // variant is an A/B form compiled only into libnanohevc_ab.so (make ab).
    if (variant == kDefaultVariant || variant == 5) {
        Fused8Args a;
        uint32_t wg = 0;
        int rc = build_args(d_res, d_lvl, sets, nsets, qp, is_intra, a, wg);
        if (rc) return rc;
        if (!wg) return NH_OK;
        hipStream_t s = as_stream(stream);
        if (variant == 5) {
            k_fwd8x8_quant<1, 5><<<wg, 256, 0, s>>>(a);
        } else {
            a.xcd_chunk = wg / 8 ? wg / 8 : 1;
            // capped at 4 resident workgroups per CU (LDS reservation, lds_cap): +0.3-0.9 % in every
            // placement regime; A/B build: NH_CAP_FWD8 = 0 uncapped
            k_fwd8x8_quant<1, 5, 256, true>
                <<<wg, 256, lds_cap(k_fwd8x8_quant<1, 5, 256, true>, NH_KNOB("NH_CAP_FWD8", 4)), s>>>(a);
        }
        NH_HIP(hipGetLastError());
        return NH_OK;
    }
    return nh_fwd8x8_ab_variant(d_res, d_lvl, sets, nsets, qp, is_intra, variant, stream);
}

extern "C" int nh_fwd8x8_quant_planes(const int16_t* d_res, int16_t* d_lvl, const nh_plane_set* sets, int nsets,
                                      int qp, int is_intra, void* stream) {
    // default launch = variant 4341: variant 5 (nontemporal loads+stores --
    // streamed once, kept out of L2/MALL -- and >= 5 waves/SIMD: 74 VGPRs -> 6
    // waves) with the XCD-aware workgroup order (XCD x streams the x-th
    // eighth of the launch): +5..10 % over variant 5 in the interleaved A/B
    // (profiles/r01/xcd/ab_xcd_*.json).
    return nh_fwd8x8_quant_planes_variant(d_res, d_lvl, sets, nsets, qp, is_intra, kDefaultVariant, stream);
}

extern "C" __attribute__((weak)) int nh_probe_copy8x8_planes(const int16_t* d_in, int16_t* d_out, const nh_plane_set* sets, int nsets,
                                       int policy, void* stream) {
    // policy = cache policy (0..3) + 4 * shape (0 = the kernel's pattern, 1..3 = pair probes,
    //          4 = stripe form through LDS by LDS-DMA, 5 = stripe form, register staging)
    (void)d_in; (void)d_out; (void)sets; (void)nsets; (void)policy; (void)stream;
    set_error("nh_probe_copy8x8_planes: memory probes are in the A/B library only (make ab)");
    return NH_EVALUE;
}

// The achievable streaming rate the hot kernel is read against (bench.py's
// roofline context): a linear copy, 16 B per lane, so every
// wave instruction moves one contiguous KiB, one chunk per thread.
template <int POLICY>
__global__ void __launch_bounds__(256) k_copy_stream(const int16_t* __restrict__ in, int16_t* __restrict__ out,
                                                     int64_t nchunks, int xcd) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    const uint32_t wid = xcd ? xcd_eighths(blockIdx.x, gridDim.x) : blockIdx.x;
    for (int64_t i = (int64_t)wid * 256 + threadIdx.x; i < nchunks; i += stride)
        st16<POLICY>(out + i * 8, ld16<POLICY>(in + i * 8));
}

// Product form: M = 1 with every cache policy and the XCD order; the A/B
// library's strong definition adds the M > 1 probe shapes.
extern "C" __attribute__((weak)) int nh_probe_copy_linear(const int16_t* d_in, int16_t* d_out, int64_t nelems, int policy, int grid,
                                    void* stream) {
    // policy = cache policy (0..3, 1 = nontemporal loads + stores) + 4 * log2(M) (M > 1: A/B library only)
    //          + 16: XCD-aware workgroup order (xcd_eighths)
    const int xcd = (policy >> 4) & 1, lm = (policy >> 2) & 3;
    if (policy >> 5 || !d_in || !d_out || nelems < 0 || (nelems & 7)) return NH_EARG;
    if (lm) {
        set_error("nh_probe_copy_linear: M > 1 probe shapes are in the A/B library only (make ab)");
        return NH_EVALUE;
    }
    const int64_t chunks = nelems / 8;
    if (!chunks) return NH_OK;
    int64_t g = grid > 0 ? grid : (chunks + 255) / 256;
    if (g > (1 << 30)) g = 1 << 30;
    hipStream_t s = as_stream(stream);
    switch (policy & 3) {
        case 0: k_copy_stream<0><<<(unsigned)g, 256, 0, s>>>(d_in, d_out, chunks, xcd); break;
        case 1: k_copy_stream<1><<<(unsigned)g, 256, 0, s>>>(d_in, d_out, chunks, xcd); break;
        case 2: k_copy_stream<2><<<(unsigned)g, 256, 0, s>>>(d_in, d_out, chunks, xcd); break;
        default: k_copy_stream<3><<<(unsigned)g, 256, 0, s>>>(d_in, d_out, chunks, xcd); break;
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
    if (d_bits) {   // the term table, once per device (synchronised: visible to every stream)
        static PerDeviceOnce once;
        rc = once.run([&] {
            k_init_eb_tab<<<(kEbTab + 255) / 256, 256, 0, s>>>();
            NH_HIP(hipGetLastError());
            NH_HIP(hipStreamSynchronize(s));
            return (int)NH_OK;
        });
        if (rc) return rc;
    }
    EpiArgs e{d_nnz, d_bits};
    // occupancy targets: the largest without spills (bits: 104 VGPRs, nnz only: 75)
    if (d_bits) k_fwd8x8_quant_epi<1, true, 4><<<wg, 256, 0, s>>>(a, e);
    else k_fwd8x8_quant_epi<1, false, 5><<<wg, 256, 0, s>>>(a, e);
    NH_HIP(hipGetLastError());
    return NH_OK;
}

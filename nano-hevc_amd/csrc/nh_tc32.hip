// nh_tc32.hip -- config 5: the 32x32 transform-coding chain, MFMA variant.
//
// Semantics: every full 32x32 block of a plane goes through
// the config-4 TU chain at N=32 (DC-vs-planar by residual energy,
// __main__.py:165-178; residual -> forward_transform (transform.py:154-196) ->
// quantize_block -> dequantize_block (quant.py:126-150) -> inverse_transform
// (transform.py:199-238) -> reconstruct + clip (intra.py:70-78)).  The
// butterfly variant is k_tu_process<32> (nh_intraloop.hip, grid mode); this
// file holds the matrix-core variant and the dispatcher.
//
// MFMA formulation (one wave = one block, v_mfma_i32_32x32x32_i8):
//   int8 operands, int32 accumulation: every data operand v is split into
//   int8 parts v = sum_p 128^p * part_p (2 parts when |v| < 2^14, else 3;
//   wave-uniform choice), each part multiplied by the int8 basis (|T| <= 90),
//   partial products recombined with shifts.  All of it is ring arithmetic
//   mod 2^32, so results equal the reference's int32 matrix products exactly.
//   Data never needs an explicit transpose between the two passes of a
//   transform: the accumulator (column on the lane, rows in registers) feeds
//   the next MFMA as its B operand with the basis' k index permuted to the
//   accumulator's row order; one LDS transpose sits between quantization and
//   the inverse transform.
// Lane maps (gfx950, i8 32x32x32, checked by nh_probe_mfma_i8 in the tests):
//   A: lane l holds A[l&31][16(l>>5) + j], j = 0..15 (bytes of a 16-B operand)
//   B: lane l holds B[16(l>>5) + j][l&31]
//   C/D: register g of lane l is D[(g&3) + 8(g>>2) + 4(l>>5)][l&31]
#include <hip/hip_runtime.h>
#include <algorithm>
#include <atomic>
#include "nh_common.hpp"
#include "nh_internal.hpp"
#include "nh_tree.hpp"
#include "nh_mfma.hpp"
#include "nh_packed.hpp"

namespace nh {

__constant__ Basis c_basis;

constexpr int kOP = 40;  // LDS row pitch (elements) of the per-wave tiles: 16-B aligned rows
// Compact levels: the marker at a wide block's origin (its levels are in the spill plane)
constexpr int16_t kTc32SpillMark16 = (int16_t)0x8000;
constexpr int8_t kTc32SpillMark8 = (int8_t)0x80;
// k_tc32_hd addresses a block's rows as a wave-uniform 64-bit base (SGPRs) plus a
// 32-bit per-lane byte offset (the saddr forms: glds16s / glds2s, vofs stores),
// at most (31 * pitch + 28) * 4 bytes from the block's origin (int32 level rows),
// computed in int32: pitches up to 2^24 samples keep it below 2^31.
constexpr int kTc32MaxPitch = 1 << 24;

// TREE (config 4's 32x32 TUs): block b walks the 32-aligned positions of the
// band (rows from ta.y_base) of plane blockIdx.y of the batch, and a wave only
// proceeds where the seeded quadtree's leaf is exactly 32x32 (tu_leaf); it
// then also writes its 8x8 entries of the TU map.  Same per-TU chain as
// k_tu_process<32>.
// FIXUP (config 5): code only the blocks k_tc32_h marked wide (recon origin ==
// -32768, nh_ctu.hip).  A small grid walks the blocks with stride gridDim.x * 4
// waves, and returns at once unless k_tc32_h set *wide_flag to this launch's
// epoch -- 8-bit content (no marked block) costs one small launch, not a wave
// per block.

// One 32x32 block b of the plane blockIdx.y: the chain of k_tc32_mfma, in this
// wave's LDS tiles.
template <bool TREE, bool FIXUP>
__device__ __forceinline__ void tc32_block(const int16_t* __restrict__ src, int w, int h, int pitch, int nbx, int b,
                                           QuantParams qp, int dq_scale, int dq_per, int32_t* lvl, int16_t* recon,
                                           TreeArgs ta, uint8_t* tu_log2, int16_t (*s_orig_w)[kOP],
                                           int32_t (*s_dq_w)[kOP], int16_t* s_top_w, int16_t* s_left_w,
                                           char* mark = nullptr, int mark_bytes = 0) {
    const int l = threadIdx.x & 63, r = l & 31, hh = l >> 5;
    const ChainQ cq = make_chainq(qp, dq_scale, dq_per);   // 32-bit quant/dequant (int16 residual)
    {   // this workgroup's plane of the batch (blockIdx.y; ta.ppg >= 1)
        const int pz = blockIdx.y, gz = pz / ta.ppg, cz = pz - gz * ta.ppg;
        const int64_t poff = (int64_t)gz * ta.group_stride + (int64_t)cz * ta.plane_stride;
        src += poff;
        lvl += poff;
        recon += poff;
        if (mark) mark += poff * mark_bytes;
        if constexpr (TREE) {
            tu_log2 += (int64_t)pz * ta.tu_plane;
            ta.plane_id += cz;
        }
    }
    const int x0 = (b % nbx) * 32, y0 = (b / nbx) * 32 + (TREE ? ta.y_base : 0);
    if constexpr (FIXUP) {
        if (recon[(int64_t)y0 * pitch + x0] != (int16_t)0x8000) return;
        // compact levels (k_tc32_hd<KB, int16 / int8>): this block's int32 levels go to the spill
        // plane (lvl) and its compact origin holds the marker, a value no 8-bit block's level takes
        // (|level| <= 51, tools/packed_bounds.py level_bounds)
        if (mark && l == 0) {
            char* m = mark + ((int64_t)y0 * pitch + x0) * mark_bytes;
            if (mark_bytes == 2) *(int16_t*)m = kTc32SpillMark16;
            else *(int8_t*)m = kTc32SpillMark8;
        }
    }
    if constexpr (TREE) {
        if (x0 + 32 > w || y0 + 32 > h || tu_leaf(w, h, ta.ctb, ta.plane_id, ta.seed, x0, y0) != 32) return;
        tu_log2[(int64_t)(y0 / 4 + (l >> 3)) * (w / 4) + x0 / 4 + (l & 7)] = 5;
    }

    // ---- load the block (2 x 16 B per lane) and its neighbours (block.py:38-50) ----
    {
        const int row = l >> 1, half = l & 1;
        const int16_t* g = src + (int64_t)(y0 + row) * pitch + x0 + half * 16;
        v4i_t a0 = *(const v4i_t*)g, a1 = *(const v4i_t*)(g + 8);
        *(v4i_t*)&s_orig_w[row][half * 16] = a0;
        *(v4i_t*)&s_orig_w[row][half * 16 + 8] = a1;
        if (hh == 0) s_top_w[r] = y0 == 0 ? (int16_t)128 : src[(int64_t)(y0 - 1) * pitch + x0 + r];
        else s_left_w[r] = x0 == 0 ? (int16_t)128 : src[(int64_t)(y0 + r) * pitch + x0 - 1];
    }
    // Each wave touches only its own LDS slices, and LDS executes one wave's
    // instructions in order: a wave barrier (no s_barrier) orders write -> read.
    __builtin_amdgcn_wave_barrier();

    // ---- DC (intra.py:46-62) and planar (intra.py:81-113) ----
    const int32_t my_nb = hh == 0 ? s_top_w[r] : s_left_w[r];
    int32_t s = my_nb;
    s = grp_sum<64>(s);
    const int32_t dc = (s + 32) >> 6;
    const int32_t tr = s_top_w[31], bl = s_left_w[31];
    auto planar = [&](int y, int x) -> int32_t {
        return ((31 - x) * s_left_w[y] + (x + 1) * tr + (31 - y) * s_top_w[x] + (y + 1) * bl + 32) >> 6;
    };
    // this lane's operand slice of the block: column j = r, rows k = 16hh .. 16hh+15
    long long e_dc = 0, e_pl = 0;
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) {
        const int k = 16 * hh + jj;
        const int32_t o = s_orig_w[k][r];
        const int32_t d1 = wrap16i(o - dc), d2 = wrap16i(o - planar(k, r));
        e_dc += (long long)d1 * d1;
        e_pl += (long long)d2 * d2;
    }
    e_dc = grp_sum<64>(e_dc);
    e_pl = grp_sum<64>(e_pl);
    const bool use_dc = e_dc <= e_pl;                      // DC wins ties (__main__.py:173)
    int32_t X[16];
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) {
        const int k = 16 * hh + jj;
        X[jj] = wrap16i((int32_t)s_orig_w[k][r] - (use_dc ? dc : planar(k, r)));
    }

    // ---- forward pass 1: tempPre^T = X^T . T^T   (lane = i, registers = j) ----
    const v4i_t F1 = load_row16(&c_basis.t[r][0], 16 * hh);     // B[k][i] = T[i][k]
    v16i_t acc = mfma_auto<true>(X, F1);
    int32_t V[16];
#pragma unroll
    for (int g = 0; g < 16; ++g) V[g] = rshift_round<10>((uint32_t)acc[g]);   // transform.py:185
    // ---- forward pass 2: coeff^T = T . temp^T  (B from the accumulator, k permuted) ----
    const v4i_t F2 = load_perm16(&c_basis.t[r][0], hh);         // A[j][k] = T[j][k]
    acc = mfma_auto<false>(V, F2);
    // the inverse bases before the level stores: a load issued after a store
    // waits for it (vmcnt counts both on gfx9)
    const v4i_t F3 = load_row16(&c_basis.tt[r][0], 16 * hh);    // B[k][i] = T[k][i]
    const v4i_t F4 = load_perm16(&c_basis.tt[r][0], hh);        // A[j][k] = T[k][j]
    asm volatile("" ::: "memory");
    // ---- quant / dequant, levels out (lane = row i, registers = columns crow(g)) ----
    int32_t* lrow = lvl + (int64_t)(y0 + r) * pitch + x0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        int32_t L4[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int g = 4 * q + e;
            L4[e] = quant_s(rshift_round<10>((uint32_t)acc[g]), cq.qs, cq.h_v, cq.hneg_v);
            s_dq_w[r][crow(g, hh)] = dequant_s(L4[e], cq);
        }
        *(v4i_t*)(lrow + 8 * q + 4 * hh) = v4i_t{L4[0], L4[1], L4[2], L4[3]};
    }
    __builtin_amdgcn_wave_barrier();
    // ---- inverse pass 1: temp2^T = dq^T . T   (A = dq^T via the LDS transpose) ----
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) X[jj] = s_dq_w[16 * hh + jj][r];
    acc = mfma_auto<true>(X, F3);
#pragma unroll
    for (int g = 0; g < 16; ++g) V[g] = rshift_round<10>((uint32_t)acc[g]);   // transform.py:227
    // ---- inverse pass 2: res^T = T^T . temp2^T ----
    acc = mfma_auto<false>(V, F4);
    // ---- reconstruct + clip (intra.py:70-78), recon out ----
    int16_t* rrow = recon + (int64_t)(y0 + r) * pitch + x0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        int16_t R4[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int g = 4 * q + e, j = crow(g, hh);
            const int32_t rr = wrap16i(rshift_round<10>((uint32_t)acc[g]));
            int32_t rc = wrap16i((use_dc ? dc : planar(r, j)) + rr);
            R4[e] = (int16_t)(rc < 0 ? 0 : (rc > 255 ? 255 : rc));
        }
        *(uint2*)(rrow + 8 * q + 4 * hh) =
            make_uint2((uint16_t)R4[0] | ((uint32_t)(uint16_t)R4[1] << 16), (uint16_t)R4[2] | ((uint32_t)(uint16_t)R4[3] << 16));
    }
}

template <bool TREE, bool FIXUP = false>
__global__ void __launch_bounds__(256) k_tc32_mfma(const int16_t* __restrict__ src, int w, int h, int pitch,
                                                   int nbx, int nblk, QuantParams qp, int dq_scale, int dq_per,
                                                   int32_t* lvl, int16_t* recon, TreeArgs ta, uint8_t* tu_log2,
                                                   const uint32_t* wide_flag = nullptr, uint32_t epoch = 0,
                                                   char* mark = nullptr, int mark_bytes = 0) {
    __shared__ int16_t s_orig[4][32][kOP];
    __shared__ int32_t s_dq[4][32][kOP];
    __shared__ int16_t s_top[4][32], s_left[4][32];
    const int wv = threadIdx.x >> 6;
    if constexpr (FIXUP) {
        if (*wide_flag != epoch) return;   // k_tc32_h left no block of this launch's planes to the fix-up
        for (int b = blockIdx.x * 4 + wv; b < nblk; b += gridDim.x * 4)   // wave-uniform walk
            tc32_block<TREE, true>(src, w, h, pitch, nbx, b, qp, dq_scale, dq_per, lvl, recon, ta, tu_log2, s_orig[wv],
                                   s_dq[wv], s_top[wv], s_left[wv], mark, mark_bytes);
    } else {
        const int b = blockIdx.x * 4 + wv;
        if (b >= nblk) return;                       // whole wave exits together
        tc32_block<TREE, false>(src, w, h, pitch, nbx, b, qp, dq_scale, dq_per, lvl, recon, ta, tu_log2, s_orig[wv],
                                s_dq[wv], s_top[wv], s_left[wv]);
    }
}

// Probe: D = A . B for row-major int8 32x32 A, B using the assumed lane maps.
__global__ void k_probe_mfma_i8(const int8_t* A, const int8_t* B, int32_t* D) {
    const int l = threadIdx.x, r = l & 31, hh = l >> 5;
    int32_t a[16], bb[16];
    for (int j = 0; j < 16; ++j) {
        a[j] = A[r * 32 + 16 * hh + j];
        bb[j] = B[(16 * hh + j) * 32 + r];
    }
    v16i_t d = mfma(pack16(a), pack16(bb));
    for (int g = 0; g < 16; ++g) D[crow(g, hh) * 32 + r] = d[g];
}

// The int8 basis in constant memory, once per device (host-synchronous upload).
static int ensure_basis(hipStream_t s) {
    (void)s;
    static PerDeviceOnce once;
    return once.run([] {
        Basis b = make_basis();
        NH_HIP(hipMemcpyToSymbol(HIP_SYMBOL(c_basis), &b, sizeof(b)));
        return (int)NH_OK;
    });
}

}  // namespace nh

using namespace nh;

// butterfly variant lives in nh_intraloop.hip; the narrow f16 launch in nh_ctu.hip
namespace nh {
int tc32_narrow_launch(const int16_t* src, void* lvl, int lvl_bytes, int16_t* rec, const nh_plane_set& S,
                       const QuantParams& q, int dqs, int dq_per, uint32_t* wide_flag, uint32_t epoch, hipStream_t s);

// Config 5's wide flags: a ring of words per device, one per f16 launch (slot =
// epoch mod kFlagRing), so concurrent launches on other streams use other
// slots.  k_tc32_h stores the launch's epoch into its slot when it leaves a
// block to the int8 fix-up, which returns at once otherwise.
constexpr uint32_t kFlagRing = 1024;
static int wide_flag_slot(uint32_t** flag, uint32_t* epoch) {
    static PerDeviceOnce once;
    static uint32_t* ring[64] = {};
    static std::atomic<uint32_t> next{1};
    int dev = 0;
    NH_HIP(hipGetDevice(&dev));
    const int rc = once.run([&] {
        NH_HIP(hipMalloc(&ring[dev], kFlagRing * sizeof(uint32_t)));
        NH_HIP(hipMemset(ring[dev], 0, kFlagRing * sizeof(uint32_t)));   // epochs start at 1
        return (int)NH_OK;
    });
    if (rc) return rc;
    uint32_t e = next.fetch_add(1);
    if (e == 0) e = next.fetch_add(1);   // 0 never names a launch (the ring's initial value)
    *epoch = e;
    *flag = ring[dev] + (e % kFlagRing);
    return NH_OK;
}
int tc32_butterfly(const int16_t* d_src, int w, int h, int pitch, int qp, int32_t* d_lvl, int16_t* d_recon,
                   hipStream_t s);
}

extern "C" int nh_tc32_plane(const int16_t* d_src, int w, int h, int pitch, int qp, int32_t* d_lvl,
                             int16_t* d_recon, int variant, void* stream) {
    if (!d_src || !d_lvl || !d_recon || w < 0 || h < 0 || pitch < w) return NH_EARG;
    if ((pitch & 7) || ((uintptr_t)d_src & 15) || ((uintptr_t)d_lvl & 15) || ((uintptr_t)d_recon & 15)) {
        set_error("tc32: pitch must be a multiple of 8 and buffers 16-byte aligned");
        return NH_EARG;
    }
    hipStream_t s = as_stream(stream);
    const int nbx = w / 32, nblk = nbx * (h / 32);
    if (!nblk) return NH_OK;
    if (variant == 0) return tc32_butterfly(d_src, w, h, pitch, qp, d_lvl, d_recon, s);
    if (variant != 1 && variant != 2) return NH_EARG;
    nh_plane_set one{0, 0, 0, w, h, pitch, 1, 1, 0};
    return nh_tc32_planes(d_src, &one, 1, qp, d_lvl, d_recon, variant, stream);
}
// Config 5 over every plane of the sets.  lvl holds levels of lvl_bytes = 4
// (int32, every variant) or 2 / 1 (the compact int16 / int8 levels, variant 1
// only: 8-bit blocks store them directly; a wide block's int32 levels go to
// `spill` -- same layout as src -- and its compact origin gets the marker, so
// nh_tc32_levels_widen restores the reference's int32 levels exactly).
static int tc32_planes_impl(const int16_t* d_src, const nh_plane_set* sets, int nsets, int qp, void* d_lvl,
                            int lvl_bytes, int32_t* d_spill, int16_t* d_recon, int variant, void* stream) {
    if (!d_src || !d_lvl || !d_recon || !sets || nsets < 0 || nsets > NH_MAX_PLANE_SETS) return NH_EARG;
    if (((uintptr_t)d_src & 15) || ((uintptr_t)d_lvl & 15) || ((uintptr_t)d_recon & 15) || ((uintptr_t)d_spill & 15)) {
        set_error("tc32_planes: buffers must be 16-byte aligned");
        return NH_EARG;
    }
    if (lvl_bytes != 4 && !(variant == 1 && (lvl_bytes == 2 || lvl_bytes == 1) && d_spill)) {
        set_error("tc32_planes: compact (int16 / int8) levels need variant 1 and a spill plane");
        return NH_EARG;
    }
    // 16-B level row pieces: rows, planes and groups at 16-B aligned level offsets
    const int lal = lvl_bytes == 1 ? 15 : 7;
    for (int k = 0; k < nsets; ++k) {
        const nh_plane_set& S = sets[k];
        const int64_t planes = (int64_t)S.planes_per_group * S.num_groups;
        if (S.width < 0 || S.height < 0 || S.pitch < S.width || S.planes_per_group < 1 || S.num_groups < 0 ||
            planes > 65535 || ((S.base | S.plane_stride | S.group_stride | S.pitch) & lal)) {
            set_error(lvl_bytes == 1 ? "tc32_planes: int8 levels need pitch >= width and 16-element aligned "
                                       "base/pitch/strides"
                                     : "tc32_planes: plane set must have pitch >= width, 8-element aligned "
                                       "base/pitch/strides");
            return NH_EARG;
        }
    }
    if (variant < 0 || variant > 2) return NH_EARG;
    for (int k = 0; k < nsets; ++k)
        if (sets[k].pitch > kTc32MaxPitch) {
            set_error("tc32_planes: pitch beyond 2^24 samples (32-bit per-lane offsets, DESIGN.md §4.5)");
            return NH_EARG;
        }
    hipStream_t s = as_stream(stream);
    int q = qp < 0 ? 0 : (qp > 51 ? 51 : qp);
    const int per = q / 6, rem = q % 6;
    QuantParams p;
    p.shift = 14 + per + 5;
    p.mf = quant_scale(rem);
    p.off = (uint32_t)((1ull << p.shift) / 3);
    if (variant != 0) {
        int rc = ensure_basis(s);
        if (rc) return rc;
    }
    int32_t* lvl32 = lvl_bytes == 4 ? (int32_t*)d_lvl : d_spill;   // where the int32 chains write
    for (int k = 0; k < nsets; ++k) {
        const nh_plane_set& S = sets[k];
        const int planes = S.planes_per_group * S.num_groups;
        const int nbx = S.width / 32, nblk = nbx * (S.height / 32);
        if (!nblk || !planes) continue;
        if (variant == 0) {   // butterfly A/B leg: one launch per plane
            for (int pz = 0; pz < planes; ++pz) {
                const int gz = pz / S.planes_per_group, cz = pz - gz * S.planes_per_group;
                const int64_t off = S.base + (int64_t)gz * S.group_stride + (int64_t)cz * S.plane_stride;
                int rc = tc32_butterfly(d_src + off, S.width, S.height, S.pitch, qp, lvl32 + off, d_recon + off, s);
                if (rc) return rc;
            }
            continue;
        }
        TreeArgs ta{};
        ta.ppg = S.planes_per_group;
        ta.group_stride = S.group_stride;
        ta.plane_stride = S.plane_stride;
        const dim3 grid((nblk + 3) / 4, planes);
        if (variant == 1) {   // narrow blocks on the f16 matrix cores, then the marked wide ones on int8
            uint32_t* flag = nullptr;
            uint32_t epoch = 0;
            int rc = wide_flag_slot(&flag, &epoch);
            if (rc) return rc;
            rc = tc32_narrow_launch(d_src, d_lvl, lvl_bytes, d_recon, S, p, dequant_scale(rem), per, flag, epoch, s);
            if (rc) return rc;
            int cus = 0;
            NH_TRY(device_cus(&cus));
            const dim3 gfix((unsigned)std::min<int64_t>((nblk + 3) / 4, 2 * cus), (unsigned)planes);
            char* mark = lvl_bytes == 4 ? nullptr : (char*)d_lvl + S.base * lvl_bytes;
            k_tc32_mfma<false, true><<<gfix, 256, 0, s>>>(d_src + S.base, S.width, S.height, S.pitch, nbx, nblk, p,
                                                          dequant_scale(rem), per, lvl32 + S.base, d_recon + S.base,
                                                          ta, nullptr, flag, epoch, mark, mark ? lvl_bytes : 0);
        } else {              // int8 matrix cores only (A/B)
            k_tc32_mfma<false><<<grid, 256, lds_cap(k_tc32_mfma<false>, NH_KNOB("NH_CAP_TC32", 0)), s>>>(d_src + S.base, S.width, S.height, S.pitch, nbx, nblk, p,
                                                    dequant_scale(rem), per, lvl32 + S.base, d_recon + S.base, ta,
                                                    nullptr);
        }
        NH_HIP(hipGetLastError());
    }
    return NH_OK;
}
extern "C" int nh_tc32_planes(const int16_t* d_src, const nh_plane_set* sets, int nsets, int qp, int32_t* d_lvl,
                              int16_t* d_recon, int variant, void* stream) {
    return tc32_planes_impl(d_src, sets, nsets, qp, d_lvl, 4, nullptr, d_recon, variant, stream);
}
extern "C" int nh_tc32_planes_compact(const int16_t* d_src, const nh_plane_set* sets, int nsets, int qp, void* d_lvl,
                                      int lvl_bytes, int32_t* d_spill, int16_t* d_recon, void* stream) {
    if (lvl_bytes != 2 && lvl_bytes != 1) return NH_EARG;
    return tc32_planes_impl(d_src, sets, nsets, qp, d_lvl, lvl_bytes, d_spill, d_recon, 1, stream);
}

namespace nh {
// Compact levels -> the reference's int32 levels: every sample of every full
// 32x32 block (8 per thread), from the spill plane where the block's compact
// origin holds the marker, else the compact value widened.  Samples outside
// full blocks are not written (the int32 path leaves them untouched too).
template <class LT>
__global__ void __launch_bounds__(256) k_tc32_widen(const LT* __restrict__ lc, const int32_t* __restrict__ spill,
                                                    int32_t* __restrict__ out, int64_t base, int64_t group_stride,
                                                    int64_t plane_stride, int ppg, int fw8, int fh, int pitch) {
    const LT mk = sizeof(LT) == 2 ? (LT)kTc32SpillMark16 : (LT)kTc32SpillMark8;
    const int pz = blockIdx.y, gz = pz / ppg, cz = pz - gz * ppg;
    const int64_t poff = base + (int64_t)gz * group_stride + (int64_t)cz * plane_stride;
    const int64_t n = (int64_t)fw8 * fh;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int y = (int)(i / fw8), x = 8 * (int)(i - (int64_t)y * fw8);
        const int64_t o = poff + (int64_t)y * pitch + x;
        const bool sp = lc[poff + (int64_t)(y & ~31) * pitch + (x & ~31)] == mk;
        int32_t v[8];
        if (sp) {
            const int4 a = *(const int4*)(spill + o), b = *(const int4*)(spill + o + 4);
            v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
        } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = lc[o + e];
        }
        *(int4*)(out + o) = make_int4(v[0], v[1], v[2], v[3]);
        *(int4*)(out + o + 4) = make_int4(v[4], v[5], v[6], v[7]);
    }
}
}  // namespace nh

extern "C" int nh_tc32_levels_widen(const void* d_lvl, int lvl_bytes, const int32_t* d_spill,
                                    const nh_plane_set* sets, int nsets, int32_t* d_out, void* stream) {
    if (!d_lvl || !d_spill || !d_out || !sets || nsets < 0 || nsets > NH_MAX_PLANE_SETS) return NH_EARG;
    if ((lvl_bytes != 2 && lvl_bytes != 1) || (((uintptr_t)d_spill | (uintptr_t)d_out) & 15)) return NH_EARG;
    hipStream_t s = as_stream(stream);
    for (int k = 0; k < nsets; ++k) {
        const nh_plane_set& S = sets[k];
        const int64_t planes = (int64_t)S.planes_per_group * S.num_groups;
        if (S.width < 0 || S.height < 0 || S.pitch < S.width || S.planes_per_group < 1 || S.num_groups < 0 ||
            planes > 65535 || ((S.base | S.plane_stride | S.group_stride | S.pitch) & 3)) {
            set_error("tc32_levels_widen: plane set must have pitch >= width, 4-element aligned base/pitch/strides");
            return NH_EARG;
        }
        const int fw8 = (S.width / 32) * 4, fh = (S.height / 32) * 32;
        if (!fw8 || !fh || !planes) continue;
        const int64_t items = (int64_t)fw8 * fh;
        const dim3 grid((unsigned)std::min<int64_t>((items + 255) / 256, 4096), (unsigned)planes);
        if (lvl_bytes == 2)
            k_tc32_widen<int16_t><<<grid, 256, 0, s>>>((const int16_t*)d_lvl, d_spill, d_out, S.base, S.group_stride,
                                                       S.plane_stride, S.planes_per_group, fw8, fh, S.pitch);
        else
            k_tc32_widen<int8_t><<<grid, 256, 0, s>>>((const int8_t*)d_lvl, d_spill, d_out, S.base, S.group_stride,
                                                      S.plane_stride, S.planes_per_group, fw8, fh, S.pitch);
        NH_HIP(hipGetLastError());
    }
    return NH_OK;
}

namespace nh {
// Config 4's 32x32 TUs on the int8 matrix cores (called by nh_tu_pipeline_planes).
int tc32_mfma_tree(const int16_t* src, int w, int h, int pitch, const QuantParams& qp, int dq_scale, int dq_per,
                   int32_t* lvl, int16_t* rec, uint8_t* tu, int bw, int n, const TreeArgs& ta, unsigned planes,
                   hipStream_t s) {
    if ((pitch & 7) || (((uintptr_t)src | (uintptr_t)lvl | (uintptr_t)rec) & 15) ||
        ((ta.group_stride | ta.plane_stride) & 7))
        return NH_EARG;   // the MFMA kernel's vector row accesses need 16-B aligned rows
    int rc = ensure_basis(s);
    if (rc) return rc;
    k_tc32_mfma<true><<<dim3((n + 3) / 4, planes), 256, 0, s>>>(src, w, h, pitch, bw, n, qp, dq_scale, dq_per, lvl, rec,
                                                                ta, tu);
    NH_HIP(hipGetLastError());
    return NH_OK;
}
}  // namespace nh

extern "C" int nh_probe_mfma_i8(const int8_t* d_a, const int8_t* d_b, int32_t* d_d, void* stream) {
    if (!d_a || !d_b || !d_d) return NH_EARG;
    k_probe_mfma_i8<<<1, 64, 0, as_stream(stream)>>>(d_a, d_b, d_d);
    NH_HIP(hipGetLastError());
    return NH_OK;
}

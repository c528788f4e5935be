// nh_frame.hip -- frame I/O casts and the frame-level intra driver
// (DESIGN.md §3.6, §4.7).
//
//   k_widen / k_narrow      frame.py:44-54, :87-115, :176-183 (astype casts)
//   k_encode_dcpl<T, N>     __main__.py:142-189 encode_frame_intra (and the
//                           demo's per-block decision, __main__.py:75-100)
//   k_encode_any<T>         the same for block sizes other than 4/8/16/32/64
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <type_traits>
#include "nh_common.hpp"
#include "nh_internal.hpp"
#include "nh_packed.hpp"

namespace nh {

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------
// uint8 <-> int16 casts: nontemporal streaming (the best policy of the
// linear-copy probe), a scalar tail, a scalar kernel for
// unaligned views.
// ---------------------------------------------------------------------------
typedef unsigned int v2u __attribute__((ext_vector_type(2)));

// 8 samples per thread: an 8-B load and ONE 16-B store, so every store
// instruction of a wave covers 1 KB contiguously.
__global__ void __launch_bounds__(256) k_widen(const uint8_t* __restrict__ in, int16_t* __restrict__ out,
                                               int64_t nchunks, int64_t n, int xcd) {
    const int64_t i = (xcd ? xcd_eighths(blockIdx.x, gridDim.x) : blockIdx.x) * 256ll + threadIdx.x;
    if (i < nchunks) {
        const v2u b = __builtin_nontemporal_load((const v2u*)in + i);
        v4u o;   // 8 bytes -> 8 int16, zero-extended (uint8 values are non-negative)
        o[0] = __builtin_amdgcn_perm(0u, b[0], 0x0c010c00u);
        o[1] = __builtin_amdgcn_perm(0u, b[0], 0x0c030c02u);
        o[2] = __builtin_amdgcn_perm(0u, b[1], 0x0c010c00u);
        o[3] = __builtin_amdgcn_perm(0u, b[1], 0x0c030c02u);
        __builtin_nontemporal_store(o, (v4u*)out + i);
    } else {
        const int64_t j = nchunks * 8 + (i - nchunks);
        if (j < n) out[j] = in[j];
    }
}

// 8 samples per thread: ONE 16-B load and an 8-B store.
__global__ void __launch_bounds__(256) k_narrow(const int16_t* __restrict__ in, uint8_t* __restrict__ out,
                                                int64_t nchunks, int64_t n, int xcd) {
    const int64_t i = (xcd ? xcd_eighths(blockIdx.x, gridDim.x) : blockIdx.x) * 256ll + threadIdx.x;
    if (i < nchunks) {
        const v4u a = __builtin_nontemporal_load((const v4u*)in + i);
        v2u o;   // low byte of each int16 (numpy's wrapping astype(np.uint8))
        o[0] = __builtin_amdgcn_perm(a[1], a[0], 0x06040200u);
        o[1] = __builtin_amdgcn_perm(a[3], a[2], 0x06040200u);
        __builtin_nontemporal_store(o, (v2u*)out + i);
    } else {
        const int64_t j = nchunks * 8 + (i - nchunks);
        if (j < n) out[j] = (uint8_t)in[j];
    }
}

// Unaligned views: one sample per thread.
__global__ void k_widen_scalar(const uint8_t* in, int16_t* out, int64_t n) {
    for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) out[i] = in[i];
}
__global__ void k_narrow_scalar(const int16_t* in, uint8_t* out, int64_t n) {
    for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) out[i] = (uint8_t)in[i];
}

// ---------------------------------------------------------------------------
// encode_frame_intra.  N lanes per block, lane r owns block row r: it loads its
// source row and the block's top row (one vector load each when the layout is
// 16-element aligned: AL), left[r] and bl = left[N-1]; the segment (N lanes,
// 64 % N == 0) sums left[] for DC; both residual energies are segment-reduced
// and the winner's clipped prediction row is stored.  A workgroup walks one
// plane with a stride of gridDim.x (<= 512 workgroups per plane), so each
// stats word takes <= 512 atomics.
// ---------------------------------------------------------------------------
struct EncArgs {
    const void* src;
    int16_t* rec;
    uint8_t* rec8;
    int64_t* stats;          // stats of this set's plane 0
    int64_t base, plane_stride, group_stride;
    int32_t w, h, pitch, ppg;
    FastDiv nbx;             // blocks per row (partial included)
    uint32_t nblk;
    uint32_t xcd;            // k_encode_u8: XCD-aware workgroup order (NH_ENC_TUNE 5th field, A/B)
    uint32_t nostats;        // A/B probe only (NH_ENC_TUNE 6th field): skip the stats atomics
};

template <int N, class V>
__device__ __forceinline__ V seg_sum(V v) { return grp_sum<N>(v); }   // DPP group sum (nh_packed.hpp)

// N samples of T at p into v[] (AL: p is aligned to min(16, N*sizeof(T)) bytes).
template <class T, int N, bool AL>
__device__ __forceinline__ void load_row(const T* p, int (&v)[N]) {
    if constexpr (AL) {
        constexpr int B = N * (int)sizeof(T), A = B < 16 ? B : 16;
        T t[N];
        __builtin_memcpy(t, __builtin_assume_aligned(p, A), B);
#pragma unroll
        for (int x = 0; x < N; ++x) v[x] = t[x];
    } else {
#pragma unroll
        for (int x = 0; x < N; ++x) v[x] = p[x];
    }
}
template <class T, int N, bool AL>
__device__ __forceinline__ void store_row(T* p, const int (&v)[N]) {
    T t[N];
#pragma unroll
    for (int x = 0; x < N; ++x) t[x] = (T)v[x];
    if constexpr (AL) {
        constexpr int B = N * (int)sizeof(T), A = B < 16 ? B : 16;
        __builtin_memcpy(__builtin_assume_aligned(p, A), t, B);
    } else {
#pragma unroll
        for (int x = 0; x < N; ++x) p[x] = t[x];
    }
}

template <class T, int N, bool AL>
__global__ void __launch_bounds__(256) k_encode_dcpl(EncArgs a) {
    constexpr int L2 = N == 4 ? 2 : N == 8 ? 3 : N == 16 ? 4 : N == 32 ? 5 : 6;
    // uint8 sources: every energy of a block (<= 64*64*255^2) fits int32
    using Acc = typename std::conditional<std::is_same<T, uint8_t>::value, int32_t, int64_t>::type;
    const int p = blockIdx.y;
    const int g = p / a.ppg, c = p - g * a.ppg;
    const int64_t off = a.base + (int64_t)g * a.group_stride + (int64_t)c * a.plane_stride;
    const T* src = static_cast<const T*>(a.src) + off;
    const int lane = threadIdx.x & 63, r = lane & (N - 1);
    constexpr uint32_t kPerWG = 256 / N;
    int64_t st_blocks = 0, st_dc = 0, st_edc = 0, st_epl = 0, st_sse = 0;

    for (uint32_t b0 = blockIdx.x * kPerWG; b0 < a.nblk; b0 += gridDim.x * kPerWG) {
        const uint32_t b = b0 + threadIdx.x / N;
        const bool act = b < a.nblk;
        const uint32_t by = act ? fdiv(b, a.nbx) : 0, bx = act ? b - by * a.nbx.d : 0;
        const int x0 = bx * N, y0 = by * N, y = y0 + r;
        const bool full = act && x0 + N <= a.w && y0 + N <= a.h;   // uniform per segment
        int o[N], top[N], lt = 128, bl = 128;
#pragma unroll
        for (int x = 0; x < N; ++x) o[x] = top[x] = 128;
        if (full) {
            load_row<T, N, AL>(src + (int64_t)y * a.pitch + x0, o);
            if (y0 > 0) load_row<T, N, AL>(src + (int64_t)(y0 - 1) * a.pitch + x0, top);
            if (x0 > 0) {
                lt = src[(int64_t)y * a.pitch + x0 - 1];
                bl = src[(int64_t)(y0 + N - 1) * a.pitch + x0 - 1];
            }
        }
        int tsum = 0;
#pragma unroll
        for (int x = 0; x < N; ++x) tsum += top[x];
        const int dc = (int16_t)((tsum + seg_sum<N>(lt) + N) >> (L2 + 1));   // floor division by 2N
        const int tr = top[N - 1];
        int pl[N];
        Acc edc = 0, epl = 0;
#pragma unroll
        for (int x = 0; x < N; ++x) {
            pl[x] = (int16_t)(((N - 1 - x) * lt + (x + 1) * tr + (N - 1 - r) * top[x] + (r + 1) * bl + N) >> (L2 + 1));
            const Acc rd = (int16_t)(o[x] - dc), rp = (int16_t)(o[x] - pl[x]);
            edc += rd * rd;
            epl += rp * rp;
        }
        const Acc sdc = seg_sum<N>(edc), spl = seg_sum<N>(epl);
        if (full) {
            const bool use_dc = sdc <= spl;
            Acc sse = 0;
#pragma unroll
            for (int x = 0; x < N; ++x) {
                const int v = use_dc ? dc : pl[x];
                pl[x] = v < 0 ? 0 : v > 255 ? 255 : v;
                const int d = (int)(uint8_t)o[x] - pl[x];
                sse += d * d;
            }
            const int64_t i = off + (int64_t)y * a.pitch + x0;
            if (a.rec) store_row<int16_t, N, AL>(a.rec + i, pl);
            if (a.rec8) store_row<uint8_t, N, AL>(a.rec8 + i, pl);
            st_sse += sse;
            if (r == 0) {
                st_blocks += 1;
                st_dc += use_dc;
                st_edc += sdc;
                st_epl += spl;
            }
        } else if (act && y < a.h) {   // samples outside full blocks: recon stays 0
            for (int x = 0; x < N && x0 + x < a.w; ++x) {
                const int64_t i = (int64_t)y * a.pitch + x0 + x;
                if (a.rec) a.rec[off + i] = 0;
                if (a.rec8) a.rec8[off + i] = 0;
                const int d = (uint8_t)src[i];
                st_sse += d * d;
            }
        }
    }
    // workgroup reduction, then one atomic per stats word
    __shared__ int64_t part[4][5];
    int64_t v[5] = {st_blocks, st_dc, st_edc, st_epl, st_sse};
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        v[k] = grp_sum<64>(v[k]);
        if (lane == 0) part[threadIdx.x >> 6][k] = v[k];
    }
    __syncthreads();
    if (threadIdx.x == 0 && !a.nostats) {
        int64_t t[5];
        for (int k = 0; k < 5; ++k) t[k] = part[0][k] + part[1][k] + part[2][k] + part[3][k];
        int64_t* s = a.stats + (int64_t)p * NH_ENC_STATS;
        const int64_t add[NH_ENC_STATS] = {t[0], t[1], t[0] - t[1], t[2], t[3], t[4]};
        for (int k = 0; k < NH_ENC_STATS; ++k)
            if (add[k]) atomicAdd((unsigned long long*)(s + k), (unsigned long long)add[k]);
    }
}

// Lane-per-block form for N in {4, 8} (the CLI default: 8x8 luma, 4x4
// chroma).  Each lane takes U blocks (b, b + 256, ...), issues all their row
// loads first (U * (N + 1) rows in flight per lane), then decides each block.
// A wave covers 64 consecutive blocks, so every row access of a wave is one
// contiguous 64 * N-sample run; the left column is the previous lane's last
// column (lane shuffle), loaded only by lane 0 of a wave.
template <class T, int N>
struct RowT;   // one block row of N samples of T, packed in dwords
template <> struct RowT<uint8_t, 4> { typedef unsigned int type; };
template <> struct RowT<uint8_t, 8> { typedef v2u type; };
template <> struct RowT<int16_t, 4> { typedef v2u type; };
template <> struct RowT<int16_t, 8> { typedef v4u type; };

template <class T, class R>
__device__ __forceinline__ unsigned word(const R& r, int k) {
    if constexpr (sizeof(R) == 4) return r;
    else return r[k];
}
template <class T, class R>
__device__ __forceinline__ int elem(const R& r, int x) {
    if constexpr (sizeof(T) == 1) return (word<T>(r, x >> 2) >> (8 * (x & 3))) & 0xff;
    else return (int16_t)(word<T>(r, x >> 1) >> (16 * (x & 1)));
}
template <class T, int N, bool AL>
__device__ __forceinline__ typename RowT<T, N>::type load_rowv(const T* p) {
    typedef typename RowT<T, N>::type R;
    if constexpr (AL) {
        return *(const R*)p;
    } else {
        T t[N];
#pragma unroll
        for (int x = 0; x < N; ++x) t[x] = p[x];
        R r;
        __builtin_memcpy(&r, t, sizeof(R));
        return r;
    }
}

template <class T, int N, int U, bool AL>
__global__ void __launch_bounds__(256) k_encode_small(EncArgs a) {
    constexpr int L2 = N == 4 ? 2 : 3;
    typedef typename RowT<T, N>::type R;
    using Acc = typename std::conditional<std::is_same<T, uint8_t>::value, int32_t, int64_t>::type;
    const int p = blockIdx.y;
    const int g = p / a.ppg, c = p - g * a.ppg;
    const int64_t off = a.base + (int64_t)g * a.group_stride + (int64_t)c * a.plane_stride;
    const T* src = static_cast<const T*>(a.src) + off;
    const int lane = threadIdx.x & 63;
    int64_t st_blocks = 0, st_dc = 0, st_edc = 0, st_epl = 0, st_sse = 0;

    for (uint32_t b0 = blockIdx.x * 256u * U; b0 < a.nblk; b0 += gridDim.x * 256u * U) {
        R o[U][N], top[U];
        int x0[U], y0[U];
        bool act[U], full[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {   // load phase
            const uint32_t b = b0 + u * 256u + threadIdx.x;
            act[u] = b < a.nblk;
            const uint32_t by = act[u] ? fdiv(b, a.nbx) : 0, bx = act[u] ? b - by * a.nbx.d : 0;
            x0[u] = bx * N;
            y0[u] = by * N;
            full[u] = act[u] && x0[u] + N <= a.w && y0[u] + N <= a.h;
            const T* blk = src + (int64_t)y0[u] * a.pitch + x0[u];
#pragma unroll
            for (int i = 0; i < N; ++i) o[u][i] = full[u] ? load_rowv<T, N, AL>(blk + (int64_t)i * a.pitch) : R{};
            top[u] = full[u] && y0[u] > 0 ? load_rowv<T, N, AL>(blk - a.pitch) : R{};
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {   // decide + store phase
            int left[N];
#pragma unroll
            for (int i = 0; i < N; ++i) {
                // previous lane = block b-1 = (bx-1, by) whenever bx > 0
                const unsigned last = word<T>(o[u][i], (int)(sizeof(R) / 4) - 1);
                const unsigned prev = lane_up1(last);
                left[i] = sizeof(T) == 1 ? (int)(prev >> 24) : (int)(int16_t)(prev >> 16);
            }
            if (x0[u] == 0) {
#pragma unroll
                for (int i = 0; i < N; ++i) left[i] = 128;
            } else if (lane == 0 && full[u]) {
#pragma unroll
                for (int i = 0; i < N; ++i) left[i] = src[(int64_t)(y0[u] + i) * a.pitch + x0[u] - 1];
            }
            int tp[N], tsum = 0, lsum = 0;
#pragma unroll
            for (int x = 0; x < N; ++x) {
                tp[x] = y0[u] > 0 ? elem<T>(top[u], x) : 128;
                tsum += tp[x];
                lsum += left[x];
            }
            const int dc = (int16_t)((tsum + lsum + N) >> (L2 + 1));   // floor division by 2N
            const int tr = tp[N - 1], bl = left[N - 1];
            Acc edc = 0, epl = 0;
#pragma unroll
            for (int y = 0; y < N; ++y)
#pragma unroll
                for (int x = 0; x < N; ++x) {
                    const int ov = elem<T>(o[u][y], x);
                    const int pl = (int16_t)(((N - 1 - x) * left[y] + (x + 1) * tr + (N - 1 - y) * tp[x] +
                                              (y + 1) * bl + N) >> (L2 + 1));
                    const Acc rd = (int16_t)(ov - dc), rp = (int16_t)(ov - pl);
                    edc += rd * rd;
                    epl += rp * rp;
                }
            if (full[u]) {
                const bool use_dc = edc <= epl;
                Acc sse = 0;
#pragma unroll
                for (int y = 0; y < N; ++y) {
                    int rv[N];
#pragma unroll
                    for (int x = 0; x < N; ++x) {
                        const int v = use_dc ? dc : (int16_t)(((N - 1 - x) * left[y] + (x + 1) * tr +
                                                               (N - 1 - y) * tp[x] + (y + 1) * bl + N) >> (L2 + 1));
                        rv[x] = v < 0 ? 0 : v > 255 ? 255 : v;
                        const int d = (elem<T>(o[u][y], x) & 0xff) - rv[x];
                        sse += d * d;
                    }
                    const int64_t i = off + (int64_t)(y0[u] + y) * a.pitch + x0[u];
                    if (a.rec) store_row<int16_t, N, AL>(a.rec + i, rv);
                    if (a.rec8) store_row<uint8_t, N, AL>(a.rec8 + i, rv);
                }
                st_sse += sse;
                st_blocks += 1;
                st_dc += use_dc;
                st_edc += edc;
                st_epl += epl;
            } else if (act[u]) {   // samples outside full blocks: recon stays 0
                for (int y = y0[u]; y < y0[u] + N && y < a.h; ++y)
                    for (int x = x0[u]; x < x0[u] + N && x < a.w; ++x) {
                        const int64_t i = (int64_t)y * a.pitch + x;
                        if (a.rec) a.rec[off + i] = 0;
                        if (a.rec8) a.rec8[off + i] = 0;
                        const int d = (uint8_t)src[i];
                        st_sse += d * d;
                    }
            }
        }
    }
    __shared__ int64_t part[4][5];
    int64_t v[5] = {st_blocks, st_dc, st_edc, st_epl, st_sse};
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        v[k] = grp_sum<64>(v[k]);
        if (lane == 0) part[threadIdx.x >> 6][k] = v[k];
    }
    __syncthreads();
    if (threadIdx.x == 0 && !a.nostats) {
        int64_t t[5];
        for (int k = 0; k < 5; ++k) t[k] = part[0][k] + part[1][k] + part[2][k] + part[3][k];
        int64_t* s = a.stats + (int64_t)p * NH_ENC_STATS;
        const int64_t add[NH_ENC_STATS] = {t[0], t[1], t[0] - t[1], t[2], t[3], t[4]};
        for (int k = 0; k < NH_ENC_STATS; ++k)
            if (add[k]) atomicAdd((unsigned long long*)(s + k), (unsigned long long)add[k]);
    }
}

// 8-bit sources (YUV420p bytes -- the reference CLI's input), N in {4, 8}:
// the same lane-per-block walk in packed 16-bit arithmetic.  Samples are
// unpacked two per dword (v_perm); planar numerators
//   ((N-1-x)L + (x+1)tr + N + (y+1)bl) + (N-1-y)T[x]  <= 2N*255 + N < 2^16
// come from two v_pk_mad_u16 (exact mod 2^16, hence exact) and a packed
// shift; residual energies accumulate with v_dot2_i32_i16.  A weighted
// average of 8-bit neighbours lies in [0, 255], so clip_to_pixel_range is the
// identity and the int16 recon pairs are stored as computed.
typedef unsigned short v2us __attribute__((ext_vector_type(2)));
typedef short v2s __attribute__((ext_vector_type(2)));

__device__ __forceinline__ v2us as_us(unsigned v) { return __builtin_bit_cast(v2us, v); }
__device__ __forceinline__ v2s as_s(v2us v) { return __builtin_bit_cast(v2s, v); }
__device__ __forceinline__ unsigned as_u(v2us v) { return __builtin_bit_cast(unsigned, v); }
__device__ __forceinline__ v2us pair_u8(unsigned w, int k) {   // bytes 2k, 2k+1 of w, zero-extended
    return as_us(__builtin_amdgcn_perm(0u, w, k ? 0x0c030c02u : 0x0c010c00u));
}

template <int N>
struct BlkU8 {   // one block's raw rows (4 samples per dword) and top row
    unsigned o[N][N / 4], top[N / 4];
    int x0, y0;
    bool act, full;
};

template <int N>
__device__ __forceinline__ void load_blk_u8(const EncArgs& a, const uint8_t* src, uint32_t b, BlkU8<N>& k) {
    constexpr int W = N / 4;
    k.act = b < a.nblk;
    const uint32_t by = k.act ? fdiv(b, a.nbx) : 0, bx = k.act ? b - by * a.nbx.d : 0;
    k.x0 = bx * N;
    k.y0 = by * N;
    k.full = k.act && k.x0 + N <= a.w && k.y0 + N <= a.h;
    const uint8_t* blk = src + (int64_t)k.y0 * a.pitch + k.x0;
#pragma unroll
    for (int i = 0; i < N; ++i) {
        if constexpr (W == 1) {
            k.o[i][0] = k.full ? *(const unsigned*)(blk + (int64_t)i * a.pitch) : 0u;
        } else {
            const v2u r = k.full ? *(const v2u*)(blk + (int64_t)i * a.pitch) : v2u{0u, 0u};
            k.o[i][0] = r[0];
            k.o[i][1] = r[1];
        }
    }
    if constexpr (W == 1) {
        k.top[0] = k.full && k.y0 > 0 ? *(const unsigned*)(blk - a.pitch) : 0x80808080u;
    } else {
        const v2u r = k.full && k.y0 > 0 ? *(const v2u*)(blk - a.pitch) : v2u{0x80808080u, 0x80808080u};
        k.top[0] = r[0];
        k.top[1] = r[1];
    }
}

struct EncStats {
    int64_t blocks = 0, dc = 0, edc = 0, epl = 0, sse = 0;
};

// Decide one block per lane and store its recon row by row.  Every lane of the
// wave must call this (the left column comes from the previous lane).
template <int N>
__device__ __forceinline__ void decide_blk_u8(const EncArgs& a, const uint8_t* src, int64_t off, int lane,
                                              const BlkU8<N>& k, EncStats& st) {
    constexpr int L2 = N == 4 ? 2 : 3, W = N / 4;
    int left[N];
#pragma unroll
    for (int i = 0; i < N; ++i) left[i] = (int)(lane_up1(k.o[i][W - 1]) >> 24);
    if (k.x0 == 0) {
#pragma unroll
        for (int i = 0; i < N; ++i) left[i] = 128;
    } else if (lane == 0 && k.full) {
#pragma unroll
        for (int i = 0; i < N; ++i) left[i] = src[(int64_t)(k.y0 + i) * a.pitch + k.x0 - 1];
    }
    unsigned tsum = 0;
#pragma unroll
    for (int q = 0; q < W; ++q) tsum = __builtin_amdgcn_udot4(k.top[q], 0x01010101u, tsum, false);
    int lsum = 0;
#pragma unroll
    for (int i = 0; i < N; ++i) lsum += left[i];
    const unsigned dc = (tsum + lsum + N) >> (L2 + 1);
    const unsigned tr = k.top[W - 1] >> 24, bl = left[N - 1];
    const v2us dc2 = {(unsigned short)dc, (unsigned short)dc};
    v2us T2[N / 2], X2[N / 2];
#pragma unroll
    for (int q = 0; q < N / 2; ++q) {
        T2[q] = pair_u8(k.top[q >> 1], q & 1);
        X2[q] = v2us{(unsigned short)(2 * q), (unsigned short)(2 * q + 1)};
    }
    // row y: num(x) = [(N-1)L + tr + N + (y+1)bl] + x(tr - L) + (N-1-y) T[x]
    auto planar_row = [&](int y, int q) -> v2us {
        const unsigned short cy = (unsigned short)((N - 1) * left[y] + tr + N + (y + 1) * bl);
        const unsigned short dy = (unsigned short)(tr - left[y]);
        const unsigned short sy = (unsigned short)(N - 1 - y);
        const v2us c2 = {cy, cy}, d2 = {dy, dy}, s2 = {sy, sy};
        return (T2[q] * s2 + (X2[q] * d2 + c2)) >> (unsigned short)(L2 + 1);
    };
    int edc = 0, epl = 0;
#pragma unroll
    for (int y = 0; y < N; ++y)
#pragma unroll
        for (int q = 0; q < N / 2; ++q) {
            const v2us o2 = pair_u8(k.o[y][q >> 1], q & 1);
            const v2s rd = as_s(o2 - dc2), rp = as_s(o2 - planar_row(y, q));
            edc = __builtin_amdgcn_sdot2(rd, rd, edc, false);
            epl = __builtin_amdgcn_sdot2(rp, rp, epl, false);
        }
    if (k.full) {
        const bool use_dc = edc <= epl;
        // the recon is the chosen prediction (clip is the identity here), so its
        // SSE against the source is that prediction's energy
        const int sse = use_dc ? edc : epl;
#pragma unroll
        for (int y = 0; y < N; ++y) {
            unsigned rv[N / 2];
#pragma unroll
            for (int q = 0; q < N / 2; ++q) rv[q] = as_u(use_dc ? dc2 : planar_row(y, q));
            const int64_t i = off + (int64_t)(k.y0 + y) * a.pitch + k.x0;
            if (a.rec) {
                if constexpr (N == 4) __builtin_nontemporal_store(v2u{rv[0], rv[1]}, (v2u*)(a.rec + i));
                else __builtin_nontemporal_store(v4u{rv[0], rv[1], rv[2], rv[3]}, (v4u*)(a.rec + i));
            }
            if (a.rec8) {
                if constexpr (N == 4) *(unsigned*)(a.rec8 + i) = __builtin_amdgcn_perm(rv[1], rv[0], 0x06040200u);
                else *(v2u*)(a.rec8 + i) = v2u{__builtin_amdgcn_perm(rv[1], rv[0], 0x06040200u),
                                               __builtin_amdgcn_perm(rv[3], rv[2], 0x06040200u)};
            }
        }
        st.sse += sse;
        st.blocks += 1;
        st.dc += use_dc;
        st.edc += edc;
        st.epl += epl;
    } else if (k.act) {   // samples outside full blocks: recon stays 0
        for (int y = k.y0; y < k.y0 + N && y < a.h; ++y)
            for (int x = k.x0; x < k.x0 + N && x < a.w; ++x) {
                const int64_t i = (int64_t)y * a.pitch + x;
                if (a.rec) a.rec[off + i] = 0;
                if (a.rec8) a.rec8[off + i] = 0;
                const int d = src[i];
                st.sse += d * d;
            }
    }
}

__device__ __forceinline__ void flush_enc_stats(const EncArgs& a, int p, EncStats st) {
    __shared__ int64_t part[4][5];
    const int lane = threadIdx.x & 63;
    int64_t v[5] = {st.blocks, st.dc, st.edc, st.epl, st.sse};
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        v[k] = grp_sum<64>(v[k]);
        if (lane == 0) part[threadIdx.x >> 6][k] = v[k];
    }
    __syncthreads();
    if (threadIdx.x == 0 && !a.nostats) {
        int64_t t[5];
        for (int k = 0; k < 5; ++k) t[k] = part[0][k] + part[1][k] + part[2][k] + part[3][k];
        int64_t* s = a.stats + (int64_t)p * NH_ENC_STATS;
        const int64_t add[NH_ENC_STATS] = {t[0], t[1], t[0] - t[1], t[2], t[3], t[4]};
        for (int k = 0; k < NH_ENC_STATS; ++k)
            if (add[k]) atomicAdd((unsigned long long*)(s + k), (unsigned long long)add[k]);
    }
}

// U blocks per lane per pass, loads first; PIPE: the next pass's blocks are
// loaded before this pass's blocks are decided (the grid is capped so that a
// workgroup makes several passes).
template <int N, int U, bool PIPE, int WAVES = 1>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WAVES))) k_encode_u8(EncArgs a) {
    // XCD-aware order over the (slot, plane) grid: XCD x runs the x-th eighth
    // of the planes' workgroup slots (xcd_eighths), else the hardware order
    uint32_t wx = blockIdx.x, wy = blockIdx.y;
    if (a.xcd) {
        const uint32_t l = xcd_eighths(blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gridDim.y);
        wy = l / gridDim.x;
        wx = l - wy * gridDim.x;
    }
    const int p = wy;
    const int g = p / a.ppg, c = p - g * a.ppg;
    const int64_t off = a.base + (int64_t)g * a.group_stride + (int64_t)c * a.plane_stride;
    const uint8_t* src = static_cast<const uint8_t*>(a.src) + off;
    const int lane = threadIdx.x & 63;
    const uint32_t stride = gridDim.x * 256u * U;
    EncStats st;
    uint32_t b0 = wx * 256u * U;
    BlkU8<N> cur[U];
    if (PIPE && b0 < a.nblk) {
#pragma unroll
        for (int u = 0; u < U; ++u) load_blk_u8<N>(a, src, b0 + u * 256u + threadIdx.x, cur[u]);
    }
    for (; b0 < a.nblk; b0 += stride) {
        BlkU8<N> nxt[U];
        if constexpr (PIPE) {
            if (b0 + stride < a.nblk) {
#pragma unroll
                for (int u = 0; u < U; ++u) load_blk_u8<N>(a, src, b0 + stride + u * 256u + threadIdx.x, nxt[u]);
            }
        } else {
#pragma unroll
            for (int u = 0; u < U; ++u) load_blk_u8<N>(a, src, b0 + u * 256u + threadIdx.x, cur[u]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) decide_blk_u8<N>(a, src, off, lane, cur[u], st);
        if constexpr (PIPE) {
#pragma unroll
            for (int u = 0; u < U; ++u) cur[u] = nxt[u];
        }
    }
    flush_enc_stats(a, p, st);
}

// Any block size N >= 1 (encode_frame_intra takes any block_size,
// __main__.py:156-158; the demo passes it unclamped, __main__.py:75-91): one
// wave per block, lanes stride over its N*N samples.  DC is the floor division
// of intra.py:61 (2N need not be a power of two), planar's shift is
// int(log2 N) + 1 (intra.py:105), so for N not a power of two its weights do not
// normalise and a wide-range int16 plane can leave int16 -- the reference's
// store raises OverflowError there (intra.py:111), reported through *err.  Two
// passes over the block (energies, then the winner's clipped samples); the
// neighbour and source re-reads of the second pass hit the caches.
template <class T>
__global__ void __launch_bounds__(256) k_encode_any(EncArgs a, int n, int log2n, int* err) {
    const int p = blockIdx.y;
    const int g = p / a.ppg, c = p - g * a.ppg;
    const int64_t off = a.base + (int64_t)g * a.group_stride + (int64_t)c * a.plane_stride;
    const T* src = static_cast<const T*>(a.src) + off;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t nn = (int64_t)n * n;
    int64_t st_blocks = 0, st_dc = 0, st_edc = 0, st_epl = 0, st_sse = 0;
    for (uint32_t b = blockIdx.x * 4 + wv; b < a.nblk; b += gridDim.x * 4) {
        const uint32_t by = b / a.nbx.d, bx = b - by * a.nbx.d;   // wave-uniform
        const int64_t x0 = (int64_t)bx * n, y0 = (int64_t)by * n;
        if (x0 + n > a.w || y0 + n > a.h) {        // partial block: recon stays 0 (Frame.zeros)
            const int64_t pw = std::min<int64_t>(n, a.w - x0), ph = std::min<int64_t>(n, a.h - y0);
            for (int64_t i = lane; i < pw * ph; i += 64) {
                const int64_t y = y0 + i / pw, x = x0 + i % pw, k = y * a.pitch + x;
                if (a.rec) a.rec[off + k] = 0;
                if (a.rec8) a.rec8[off + k] = 0;
                const int d = (uint8_t)src[k];
                st_sse += d * d;
            }
            continue;
        }
        const T* row_above = src + (y0 - 1) * a.pitch + x0;
        const T* col_left = src + y0 * a.pitch + x0 - 1;
        auto top = [&](int64_t i) -> int64_t { return y0 > 0 ? (int64_t)row_above[i] : 128; };
        auto left = [&](int64_t i) -> int64_t { return x0 > 0 ? (int64_t)col_left[i * a.pitch] : 128; };
        int64_t s = 0;
        for (int64_t i = lane; i < n; i += 64) s += top(i) + left(i);
        s = grp_sum<64>(s) + n;
        const int64_t d2 = 2 * (int64_t)n, q = s / d2;
        const int64_t dc = q - ((s % d2) != 0 && s < 0);                     // Python floor division
        const int64_t tr = top(n - 1), bl = left(n - 1);
        auto planar = [&](int64_t y, int64_t x) -> int64_t {
            return ((n - 1 - x) * left(y) + (x + 1) * tr + (n - 1 - y) * top(x) + (y + 1) * bl + n) >> (log2n + 1);
        };
        int64_t edc = 0, epl = 0;
        bool ovf = false;
        for (int64_t i = lane; i < nn; i += 64) {
            const int64_t y = i / n, x = i - y * n;
            const int o = src[(y0 + y) * a.pitch + x0 + x];
            const int64_t pl = planar(y, x);
            ovf |= pl < -32768 || pl > 32767;
            const int64_t rd = (int16_t)(o - (int)dc), rp = (int16_t)(o - (int)(int16_t)pl);
            edc += rd * rd;
            epl += rp * rp;
        }
        if (ovf && err) atomicOr(err, 1);
        edc = grp_sum<64>(edc);
        epl = grp_sum<64>(epl);
        const bool use_dc = edc <= epl;
        for (int64_t i = lane; i < nn; i += 64) {
            const int64_t y = i / n, x = i - y * n, k = (y0 + y) * a.pitch + x0 + x;
            const int64_t v = use_dc ? dc : (int16_t)planar(y, x);
            const int r = v < 0 ? 0 : v > 255 ? 255 : (int)v;
            if (a.rec) a.rec[off + k] = (int16_t)r;
            if (a.rec8) a.rec8[off + k] = (uint8_t)r;
            const int d = (int)(uint8_t)src[k] - r;
            st_sse += d * d;
        }
        if (lane == 0) {
            st_blocks += 1;
            st_dc += use_dc;
            st_edc += edc;
            st_epl += epl;
        }
    }
    __shared__ int64_t part[4][5];
    int64_t v[5] = {st_blocks, st_dc, st_edc, st_epl, st_sse};
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        v[k] = grp_sum<64>(v[k]);
        if (lane == 0) part[wv][k] = v[k];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int64_t t[5];
        for (int k = 0; k < 5; ++k) t[k] = part[0][k] + part[1][k] + part[2][k] + part[3][k];
        int64_t* st = a.stats + (int64_t)p * NH_ENC_STATS;
        const int64_t add[NH_ENC_STATS] = {t[0], t[1], t[0] - t[1], t[2], t[3], t[4]};
        for (int k = 0; k < NH_ENC_STATS; ++k)
            if (add[k]) atomicAdd((unsigned long long*)(st + k), (unsigned long long)add[k]);
    }
}

// Launch shape of the N = 4 / 8 kernels: blocks per lane per pass (u4, u8),
// prefetching form (pipe) and its total workgroup cap.  Tuning knob for
// measurement: NH_ENC_TUNE="u4,u8,pipe,cap[,xcd]", read once.
struct EncTune {
    int u4 = 1, u8 = 1, pipe = 1, cap = 4096;   // measured best (profiles/r01/frame)
    int xcd = 0;       // XCD-aware workgroup order: 0.480 vs 0.487 ms per 64 4K frames without it (profiles/r01/xcd)
    int nostats = 0;   // A/B probe only: skip the stats atomics (stats are then wrong)
    int waves = 0;     // A/B: N = 8 pipelined form with >= 4 waves/SIMD (register cap 128)
};
static const EncTune& enc_tune() {
    static EncTune t;
#if NH_AB   // A/B build only: launch shapes from NH_ENC_TUNE (tools/enc_tune_ab.sh)
    static bool init = false;
    if (!init) {
        init = true;
        if (const char* e = getenv("NH_ENC_TUNE")) {
            EncTune r;
            if (sscanf(e, "%d,%d,%d,%d,%d,%d,%d", &r.u4, &r.u8, &r.pipe, &r.cap, &r.xcd, &r.nostats, &r.waves) >= 2 &&
                (r.u4 == 1 || r.u4 == 2 || r.u4 == 4) && (r.u8 == 1 || r.u8 == 2 || r.u8 == 4) && r.cap > 0)
                t = r;
        }
    }
#endif
    return t;
}
static void small_unroll(int& u4, int& u8) {
    u4 = enc_tune().u4;
    u8 = enc_tune().u8;
}

template <class T, int N, bool AL>
static void launch_small(int u, const EncArgs& a, dim3 grid, hipStream_t s) {
    if constexpr (std::is_same<T, uint8_t>::value && AL) {   // packed 16-bit path
        if (enc_tune().pipe) {
            if (N == 8 && u == 1 && enc_tune().waves == 4) k_encode_u8<N, 1, true, 4><<<grid, 256, 0, s>>>(a);
            else if (u == 1) k_encode_u8<N, 1, true><<<grid, 256, lds_cap(k_encode_u8<N, 1, true>, NH_KNOB("NH_CAP_ENC", 0)), s>>>(a);
            else if (u == 2) k_encode_u8<N, 2, true><<<grid, 256, 0, s>>>(a);
            else k_encode_u8<N, 4, true><<<grid, 256, 0, s>>>(a);
        } else {
            if (u == 1) k_encode_u8<N, 1, false><<<grid, 256, 0, s>>>(a);
            else if (u == 2) k_encode_u8<N, 2, false><<<grid, 256, 0, s>>>(a);
            else k_encode_u8<N, 4, false><<<grid, 256, 0, s>>>(a);
        }
        return;
    }
    if (u == 1) k_encode_small<T, N, 1, AL><<<grid, 256, 0, s>>>(a);
    else if (u == 2) k_encode_small<T, N, 2, AL><<<grid, 256, 0, s>>>(a);
    else k_encode_small<T, N, 4, AL><<<grid, 256, 0, s>>>(a);
}

template <class T, bool AL>
static int launch_encode_al(int n, const EncArgs& a, dim3 grid, hipStream_t s) {
    int u4, u8;
    small_unroll(u4, u8);
    switch (n) {
        case 4: launch_small<T, 4, AL>(u4, a, grid, s); break;
        case 8: launch_small<T, 8, AL>(u8, a, grid, s); break;
        case 16: k_encode_dcpl<T, 16, AL><<<grid, 256, 0, s>>>(a); break;
        case 32: k_encode_dcpl<T, 32, AL><<<grid, 256, 0, s>>>(a); break;
        case 64: k_encode_dcpl<T, 64, AL><<<grid, 256, 0, s>>>(a); break;
        default: return NH_EARG;
    }
    return NH_OK;
}
template <class T>
static int launch_encode(int n, bool al, const EncArgs& a, dim3 grid, hipStream_t s) {
    return al ? launch_encode_al<T, true>(n, a, grid, s) : launch_encode_al<T, false>(n, a, grid, s);
}

}  // namespace nh

using namespace nh;

extern "C" {

int nh_widen_u8_i16(const uint8_t* d_in, int16_t* d_out, int64_t n, void* stream) {
    if (n < 0 || (n > 0 && (!d_in || !d_out))) { set_error("nh_widen_u8_i16: bad arguments"); return NH_EARG; }
    if (n == 0) return NH_OK;
    const hipStream_t s = as_stream(stream);
    if (((uintptr_t)d_in & 7) == 0 && ((uintptr_t)d_out & 15) == 0) {
        const int64_t chunks = n / 8, threads = chunks + (n - chunks * 8);
        k_widen<<<(unsigned)((threads + 255) / 256), 256, lds_cap(k_widen, NH_KNOB("NH_CAP_IO", 0)), s>>>(
            d_in, d_out, chunks, n, xcd_order());
    } else {
        k_widen_scalar<<<(unsigned)std::min<int64_t>((n + 255) / 256, 65536), 256, 0, s>>>(d_in, d_out, n);
    }
    NH_HIP(hipGetLastError());
    return NH_OK;
}

int nh_narrow_i16_u8(const int16_t* d_in, uint8_t* d_out, int64_t n, void* stream) {
    if (n < 0 || (n > 0 && (!d_in || !d_out))) { set_error("nh_narrow_i16_u8: bad arguments"); return NH_EARG; }
    if (n == 0) return NH_OK;
    const hipStream_t s = as_stream(stream);
    if (((uintptr_t)d_in & 15) == 0 && ((uintptr_t)d_out & 7) == 0) {
        const int64_t chunks = n / 8, threads = chunks + (n - chunks * 8);
        k_narrow<<<(unsigned)((threads + 255) / 256), 256, lds_cap(k_narrow, NH_KNOB("NH_CAP_IO", 0)), s>>>(
            d_in, d_out, chunks, n, xcd_order());
    } else {
        k_narrow_scalar<<<(unsigned)std::min<int64_t>((n + 255) / 256, 65536), 256, 0, s>>>(d_in, d_out, n);
    }
    NH_HIP(hipGetLastError());
    return NH_OK;
}

int nh_encode_intra_planes(const void* d_src, int src_is_u8, const nh_plane_set* sets, int nsets,
                           const int32_t* block_sizes, int16_t* d_recon, uint8_t* d_recon_u8,
                           int64_t* d_stats, int32_t* d_status, void* stream) {
    if (!d_src || !sets || !block_sizes || !d_stats || nsets < 0 || nsets > NH_MAX_PLANE_SETS) {
        set_error("nh_encode_intra_planes: bad arguments");
        return NH_EARG;
    }
    const hipStream_t s = as_stream(stream);
    int64_t plane0 = 0;
    for (int k = 0; k < nsets; ++k) {
        const nh_plane_set& S = sets[k];
        const int n = block_sizes[k];
        const int64_t planes = (int64_t)S.planes_per_group * S.num_groups;
        if (S.width < 0 || S.height < 0 || S.pitch < S.width || S.planes_per_group < 1 || S.num_groups < 0 ||
            planes > 65535 || n < 1 || n > 65536) {
            set_error("nh_encode_intra_planes: bad plane set or block size (1..65536)");
            return NH_EARG;
        }
        const bool fast = n == 4 || n == 8 || n == 16 || n == 32 || n == 64;
        if (!fast && !src_is_u8 && !d_status) {   // only the generic form on int16 samples can overflow
            set_error("nh_encode_intra_planes: block size not a power of two in 4..64 on int16 samples needs d_status");
            return NH_EARG;
        }
        if (planes == 0 || S.width == 0 || S.height == 0) continue;
        EncArgs a;
        a.src = d_src;
        a.rec = d_recon;
        a.rec8 = d_recon_u8;
        a.stats = d_stats + plane0 * NH_ENC_STATS;
        a.base = S.base;
        a.plane_stride = S.plane_stride;
        a.group_stride = S.group_stride;
        a.w = S.width;
        a.h = S.height;
        a.pitch = S.pitch;
        a.ppg = S.planes_per_group;
        const int64_t nbx = (S.width + n - 1) / n, nblk = nbx * ((S.height + n - 1) / n);
        if (nblk * n >= (1ll << 31)) {
            set_error("nh_encode_intra_planes: plane too large");
            return NH_EARG;
        }
        a.nbx = make_fastdiv((uint32_t)nbx);
        a.nblk = (uint32_t)nblk;
        a.xcd = enc_tune().xcd;
        a.nostats = enc_tune().nostats;
        // vector row access when every row start is 16-element aligned
        const auto al16 = [](const void* q) { return ((uintptr_t)q & 15) == 0; };
        const bool al = al16(d_src) && (!d_recon || al16(d_recon)) && (!d_recon_u8 || al16(d_recon_u8)) &&
                        S.base % 16 == 0 && S.plane_stride % 16 == 0 && S.group_stride % 16 == 0 && S.pitch % 16 == 0;
        if (!fast) {   // k_encode_any: one wave per block, <= 512 workgroups (atomics) per plane
            int log2n = 0;
            while ((2 << log2n) <= n) ++log2n;                                      // int(np.log2(n))
            const dim3 grid((unsigned)std::min<int64_t>((nblk + 3) / 4, 512), (unsigned)planes);
            int* err = (int*)d_status;   // NULL for uint8 samples: planar stays below 511 there
            if (src_is_u8) k_encode_any<uint8_t><<<grid, 256, 0, s>>>(a, n, log2n, err);
            else k_encode_any<int16_t><<<grid, 256, 0, s>>>(a, n, log2n, err);
            NH_HIP(hipGetLastError());
            plane0 += planes;
            continue;
        }
        int u4, u8;
        small_unroll(u4, u8);
        const int64_t per_wg = n == 4 ? 256 * u4 : n == 8 ? 256 * u8 : 256 / n;   // blocks per workgroup pass
        const int64_t wgs = (nblk + per_wg - 1) / per_wg;
        int64_t cap = 512;   // <= 512 workgroups (atomics) per plane
        if (src_is_u8 && al && (n == 4 || n == 8) && enc_tune().pipe)
            cap = std::max<int64_t>(1, std::min<int64_t>(512, enc_tune().cap / planes));
        const dim3 grid((unsigned)std::min<int64_t>(wgs, cap), (unsigned)planes);
        const int rc = src_is_u8 ? launch_encode<uint8_t>(n, al, a, grid, s) : launch_encode<int16_t>(n, al, a, grid, s);
        if (rc) return rc;
        NH_HIP(hipGetLastError());
        plane0 += planes;
    }
    return NH_OK;
}

}  // extern "C"

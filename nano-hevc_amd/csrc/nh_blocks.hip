// nh_blocks.hip -- generic gfx950 kernels for every reference hot-path function
// plus the C-ABI entry points that expose them one block at a time (the
// drop-in path behind the nano_hevc ctypes shim) or batched on device memory.
//
// Reference map:
//   k_intra_dc        intra.py:37-62           (A2, A3)
//   k_intra_planar    intra.py:81-113          (A4)
//   k_intra_angular   intra.py:116-207         (A5)
//   k_residual / k_reconstruct / k_clip        intra.py:65-78 (A6-A8)
//   k_transform<N,DST,FWD>  transform.py:154-238 (A9-A11)
//   k_quant_i64 / k_dequant_i64 / k_quant_i32 / k_dequant_i32  quant.py:41-150 (A12-A13)
//   k_count_nonzero / k_estimate_bits          quant.py:153-173
#include <hip/hip_runtime.h>
#include <atomic>
#include <chrono>
#include <climits>
#include <cstddef>
#include <type_traits>
#include <cstdio>
#include <cstring>
#include <string>
#include "nh_common.hpp"
#include "nh_internal.hpp"
#include "nh_packed.hpp"

namespace nh {

// ---------------------------------------------------------------------------
// error reporting
// ---------------------------------------------------------------------------
static thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }

// Kernel status word: first error in raster order wins.  key = idx<<8 | -code.
__device__ __forceinline__ void report(unsigned long long* st, long long idx, int code) {
    atomicMin(st, ((unsigned long long)idx << 8) | (unsigned long long)(-code));
}

// ---------------------------------------------------------------------------
// intra prediction kernels (per-block form)
// ---------------------------------------------------------------------------

// intra.py:37-62.  One workgroup: int64 sum over the whole arrays (D7), then fill.
__device__ __forceinline__ void dev_intra_dc(const int64_t* top, int64_t nt, const int64_t* left,
                                                  int64_t nl, int64_t size, int variant, int16_t* out,
                                                  unsigned long long* st) {
    __shared__ long long part[256];
    __shared__ long long dcs;
    long long s = 0;
    for (int64_t i = threadIdx.x; i < nt; i += 256) s += top[i];
    for (int64_t i = threadIdx.x; i < nl; i += 256) s += left[i];
    part[threadIdx.x] = s;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) part[threadIdx.x] += part[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        long long tot = part[0], dc;
        if (variant) dc = (tot + 4) >> 3;                      // intra.py:42
        else {                                                  // intra.py:61 floor division
            long long d = 2 * size, q = (tot + size) / d, r = (tot + size) % d;
            if (r != 0 && ((r < 0) != (d < 0))) --q;
            dc = q;
        }
        if (dc < -32768 || dc > 32767) report(st, 0, NH_EOVERFLOW);  // np.full int16 (D9)
        dcs = dc;
    }
    __syncthreads();
    const int64_t n = variant ? 16 : size * size;
    const int16_t v = (int16_t)dcs;
    for (int64_t i = threadIdx.x; i < n; i += 256) out[i] = v;
}

// Scalar kinds of planar's corner arithmetic (intra.py:109-111 under numpy 2 /
// NEP 50): NH_NP_PYINT (0) = a Python int (exact), NH_NP_FLOAT (1) = a float
// (h and v become floats, the >> raises TypeError), +8/16/32/64 = numpy uintN,
// -8/-16/-32/-64 = numpy intN (np.bool_ corners arrive as int64: Python int
// times np.bool_ is int64).  Values are carried exactly in 128 bits; a numpy
// kind's value always lies in its range.
typedef __int128 i128;
constexpr int kNpFloat = 1;   // int64 + uint64 (or intN + uint64) promotes to float64
__device__ __forceinline__ bool np_fits(int k, i128 v) {
    if (k == 0) return true;
    const int w = k < 0 ? -k : k;
    if (k < 0) return v >= -((i128)1 << (w - 1)) && v < ((i128)1 << (w - 1));
    return v >= 0 && v < ((i128)1 << w);
}
__device__ __forceinline__ i128 np_wrap(int k, i128 v) {   // numpy's modular scalar result
    if (k == 0) return v;
    const int w = k < 0 ? -k : k;
    const unsigned __int128 m = ((unsigned __int128)1 << w) - 1, u = (unsigned __int128)v & m;
    if (k < 0 && (u >> (w - 1))) return (i128)u - ((i128)1 << w);
    return (i128)u;
}
__device__ __forceinline__ int np_promote(int a, int b) {   // numpy's result kind of a (+) b
    if ((a < 0) == (b < 0)) return a < 0 ? (a < b ? a : b) : (a > b ? a : b);
    const int s = a < 0 ? -a : -b, u = a < 0 ? b : a;   // signed width, unsigned width
    if (u < s) return -s;
    return u < 64 ? -2 * u : kNpFloat;
}
__device__ __forceinline__ i128 np_value(int k, int64_t bits) {   // the corner argument's value
    return k == 64 ? (i128)(uint64_t)bits : (i128)bits;
}

// intra.py:81-113 in the reference's own loop order, per sample (y, x):
//   h = (size-1-x)*int(left[y]) + (x+1)*top_right
//   v = (size-1-y)*int(top[x])  + (y+1)*bottom_left
//   pred[y, x] = (h + v + size) >> (log2_size + 1)        (int16 store, D9)
// With Python-int corners this is exact integer math.  A numpy-integer corner
// makes (x+1)*corner and the sums numpy scalars: the Python-int operand is
// converted to the corner's dtype (OverflowError when out of range), the result
// wraps in that dtype, two numpy operands promote, int64 with uint64 becomes
// float64 and the >> raises TypeError.  Every step that can raise has its own
// stage, so the status word keeps the first error in the reference's order.
__device__ __forceinline__ void dev_intra_planar(const int64_t* top, int64_t nt, const int64_t* left, int64_t nl,
                               int64_t trb, int ktr, int64_t blb, int kbl, int64_t size, int64_t log2size,
                               int16_t* out, unsigned long long* st) {
    const int64_t n = size * size;
    const i128 tr = np_value(ktr, trb), bl = np_value(kbl, blb);
    const int sh = (int)(log2size + 1 < 127 ? log2size + 1 : 127);
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t y = i / size, x = i - y * size;
        const int64_t at = i * 16;   // status key: position, then stage
        // h (stages 0-2) and v (stages 3-5): Python part first, then the corner term, then their sum
        auto term = [&](int64_t ri, int64_t nr, const int64_t* ref, int64_t w, int64_t c, i128 corner, int k,
                        int s0, i128& out_v) -> bool {
            if (ri >= nr) { report(st, at + s0, NH_EINDEX); return false; }
            const i128 py = (i128)w * ref[ri];
            if (k == 0) { out_v = py + (i128)c * corner; return true; }
            if (k == kNpFloat) { out_v = 0; return true; }   // a float corner: h / v are floats
            if (!np_fits(k, c)) { report(st, at + s0 + 1, NH_EOVERFLOW); return false; }
            const i128 m = np_wrap(k, (i128)c * corner);
            if (!np_fits(k, py)) { report(st, at + s0 + 2, NH_EOVERFLOW); return false; }
            out_v = np_wrap(k, py + m);
            return true;
        };
        i128 h, v;
        if (!term(y, nl, left, size - 1 - x, x + 1, tr, ktr, 0, h)) continue;
        if (!term(x, nt, top, size - 1 - y, y + 1, bl, kbl, 3, v)) continue;
        int k;   // kind of h + v (stage 6)
        i128 s;
        if (ktr == kNpFloat || kbl == kNpFloat) {
            k = kNpFloat;
            s = 0;
        } else if (ktr == 0 || kbl == 0) {
            k = ktr | kbl;
            if (!np_fits(k, ktr == 0 ? h : v)) { report(st, at + 6, NH_EOVERFLOW); continue; }
            s = np_wrap(k, h + v);
        } else {
            k = np_promote(ktr, kbl);
            s = k == kNpFloat ? 0 : np_wrap(k, h + v);
        }
        if (k == kNpFloat) { report(st, at + 8, NH_ETYPE); continue; }   // float64 >> int (stage 8)
        if (!np_fits(k, size)) { report(st, at + 7, NH_EOVERFLOW); continue; }
        s = np_wrap(k, s + size) >> sh;                                   // floor shift (numpy's too)
        if (s < -32768 || s > 32767) { report(st, at + 9, NH_EOVERFLOW); continue; }
        out[i] = (int16_t)s;
    }
}

// intra.py:116-207.  Thread 0 builds the int16 reference array in LDS in the
// reference's order (so the first error raised is the reference's), then the
// workgroup projects every sample with int16 arithmetic (D8).
constexpr int kMaxAngSize = 2048;  // 3N+1 int16 in LDS (12 KB)
__device__ __forceinline__ void dev_intra_angular(const int64_t* top, int64_t nt, const int64_t* left,
                                                       int64_t nl, int64_t corner, int angle, int vert,
                                                       int64_t size, int16_t* out, unsigned long long* st) {
    __shared__ int16_t ref[3 * kMaxAngSize + 1];
    __shared__ int ok;
    const int64_t N = size;
    if (threadIdx.x == 0) {
        const int64_t* pri = vert ? top : left;
        const int64_t* sec = vert ? left : top;
        const int64_t np = vert ? nt : nl, ns = vert ? nl : nt;
        int good = 1;
        for (int64_t i = 0; i < 3 * N + 1; ++i) ref[i] = 0;
        if (corner < -32768 || corner > 32767) { report(st, 0, NH_EOVERFLOW); good = 0; }
        for (int64_t i = 1; good && i <= 2 * N; ++i) {          // intra.py:174-178
            int64_t v;
            if (i < np) v = pri[i];
            else if (np == 0) { report(st, 0, NH_EINDEX); good = 0; break; }
            else v = pri[np - 1];
            if (v < -32768 || v > 32767) { report(st, 0, NH_EOVERFLOW); good = 0; break; }
            ref[N + i] = (int16_t)v;
        }
        if (good) ref[N] = (int16_t)corner;
        if (good && angle < 0) {                                 // intra.py:180-186 (D5)
            const int64_t inv = inv_angle(angle), next = (N * angle) >> 5;
            for (int64_t i = -1; i > next - 1; --i) {
                int64_t proj = ((i + 1) * inv + 128) >> 8;
                if (proj < ns) {
                    int64_t v = sec[proj];
                    if (v < -32768 || v > 32767) { report(st, 0, NH_EOVERFLOW); good = 0; break; }
                    ref[N + i] = (int16_t)v;
                }
            }
        }
        ok = good;
    }
    __syncthreads();
    if (!ok) return;
    for (int64_t i = threadIdx.x; i < N * N; i += 256) {        // intra.py:191-207
        int64_t y = i / N, x = i - y * N;
        int64_t base = vert ? x : y, scan = vert ? y : x;
        int64_t proj = (scan + 1) * angle;
        int64_t idx = N + base + 1 + (proj >> 5);
        int f = (int)(proj & 31);
        int16_t p;
        if (f == 0) p = ref[idx];
        else {
            int32_t s = (32 - f) * ref[idx] + f * ref[idx + 1] + 16;
            p = (int16_t)((int16_t)(uint16_t)(uint32_t)s >> 5);
        }
        out[i] = p;
    }
}

// intra.py:65-78
__device__ __forceinline__ void dev_residual(const int16_t* a, const int16_t* b, int64_t n, int16_t* out, int add) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint32_t x = (uint16_t)a[i], y = (uint16_t)b[i];
        out[i] = (int16_t)(uint16_t)(add ? x + y : x - y);
    }
}
__device__ __forceinline__ void dev_clip(const int64_t* x, int64_t n, int64_t maxval, int16_t* out) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        int64_t v = x[i];
        v = v < 0 ? 0 : (v > maxval ? maxval : v);
        out[i] = (int16_t)(uint16_t)(uint64_t)v;
    }
}

// ---------------------------------------------------------------------------
// Generic batched transforms: N threads per block, LDS-staged so global
// accesses are coalesced and both passes read conflict-free (row pitch N+1).
// Full 32-bit wrap arithmetic (MulWrap): exact for any int32 input.
// ---------------------------------------------------------------------------
// tile: LDS for min(nblocks, 256 / N) blocks of N x (N + 1) int32.
template <int N, bool DST, bool FWD>
__device__ __forceinline__ void dev_transform_on(const int32_t* __restrict__ in, int32_t* __restrict__ out,
                                                 int64_t nblocks, int32_t (*tile)[N][N + 1]) {
    constexpr int BPW = 256 / N;  // blocks per workgroup
    constexpr int S = Log2<N>::v + 5;  // transform.py:173 (D1: same shift both passes)
    const int64_t b0 = (int64_t)blockIdx.x * BPW;
    const int nb = (int)((nblocks - b0) < BPW ? (nblocks - b0) : BPW);
    // coalesced load of nb blocks
    const int32_t* src = in + b0 * N * N;
    for (int e = threadIdx.x; e < nb * N * N; e += 256) {
        int b = e / (N * N), r = (e / N) % N, c = e % N;
        tile[b][r][c] = src[e];
    }
    __syncthreads();
    const int b = threadIdx.x / N, t = threadIdx.x % N;
    uint32_t x[N], y[N];
    if (b < nb) {
        // pass 1: along columns (column t), transform.py:179-185 / :221-227
#pragma unroll
        for (int k = 0; k < N; ++k) x[k] = (uint32_t)tile[b][k][t];
        if (FWD) fwd1d<N, DST, MulWrap>(x, y); else inv1d<N, DST, MulWrap>(x, y);
#pragma unroll
        for (int i = 0; i < N; ++i) x[i] = (uint32_t)rshift_round<S>(y[i]);
    }
    __syncthreads();
    if (b < nb) {
#pragma unroll
        for (int i = 0; i < N; ++i) tile[b][i][t] = (int32_t)x[i];
    }
    __syncthreads();
    if (b < nb) {
        // pass 2: along rows (row t), transform.py:188-194 / :230-236
#pragma unroll
        for (int k = 0; k < N; ++k) x[k] = (uint32_t)tile[b][t][k];
        if (FWD) fwd1d<N, DST, MulWrap>(x, y); else inv1d<N, DST, MulWrap>(x, y);
    }
    __syncthreads();
    if (b < nb) {
#pragma unroll
        for (int j = 0; j < N; ++j) tile[b][t][j] = rshift_round<S>(y[j]);
    }
    __syncthreads();
    int32_t* dst = out + b0 * N * N;
    for (int e = threadIdx.x; e < nb * N * N; e += 256) {
        int bb = e / (N * N), r = (e / N) % N, c = e % N;
        dst[e] = tile[bb][r][c];
    }
}

template <int N, bool DST, bool FWD>
__device__ __forceinline__ void dev_transform(const int32_t* __restrict__ in, int32_t* __restrict__ out,
                                              int64_t nblocks) {
    __shared__ int32_t tile[256 / N][N][N + 1];
    dev_transform_on<N, DST, FWD>(in, out, nblocks, tile);
}

template <int N, bool DST, bool FWD>
__global__ void __launch_bounds__(256) k_transform(const int32_t* __restrict__ in, int32_t* __restrict__ out,
                                                   int64_t nblocks) {
    dev_transform<N, DST, FWD>(in, out, nblocks);
}

template <bool FWD>
static int launch_transform(const int32_t* din, int32_t* dout, int64_t nblocks, int size, int use_dst,
                            hipStream_t s) {
    if (nblocks <= 0) return NH_OK;
    const bool dst = use_dst && size == 4;
    const int bpw = 256 / size;
    const int64_t grid = (nblocks + bpw - 1) / bpw;
    if (grid > INT32_MAX) return NH_EARG;
    switch (size) {
        case 4:
            if (dst) k_transform<4, true, FWD><<<(unsigned)grid, 256, 0, s>>>(din, dout, nblocks);
            else k_transform<4, false, FWD><<<(unsigned)grid, 256, 0, s>>>(din, dout, nblocks);
            break;
        case 8: k_transform<8, false, FWD><<<(unsigned)grid, 256, 0, s>>>(din, dout, nblocks); break;
        case 16: k_transform<16, false, FWD><<<(unsigned)grid, 256, 0, s>>>(din, dout, nblocks); break;
        case 32: k_transform<32, false, FWD><<<(unsigned)grid, 256, 0, s>>>(din, dout, nblocks); break;
        default: return NH_EVALUE;
    }
    NH_HIP(hipGetLastError());
    return NH_OK;
}

// ---------------------------------------------------------------------------
// quant / dequant (quant.py:41-123)
// ---------------------------------------------------------------------------
__device__ __forceinline__ void dev_quant_i64(const int64_t* c, int64_t n, uint64_t mf, uint64_t off, int shift, int abs_bits,
                            int32_t* out) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        int64_t x = c[i], a;
        if (abs_bits < 64 && x == -(int64_t)(1ull << (abs_bits - 1))) a = x;  // np.abs wraps at dtype min
        else a = (int64_t)(x < 0 ? 0ull - (uint64_t)x : (uint64_t)x);
        int64_t l = (int64_t)((uint64_t)a * mf + off) >> shift;
        int64_t sg = (x > 0) - (x < 0);
        out[i] = (int32_t)(uint32_t)(uint64_t)(sg * l);
    }
}
// quant.py:77-78 on abs_coeff = np.abs(coeff).astype(np.int64) computed by the
// shim for float coefficients: (abs_coeff * mf + offset) >> shift in int64
// (numpy's wrapping int64 multiply); the shim applies sign * level and the
// int32 cast with the reference's own float expression (quant.py:79).
__device__ __forceinline__ void dev_quant_abs64(const int64_t* a, int64_t n, uint64_t mf, uint64_t off, int shift,
                                                int64_t* out) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = (int64_t)((uint64_t)a[i] * mf + off) >> shift;
}
__device__ __forceinline__ void dev_dequant_i64(const int64_t* l, int64_t n, int64_t scale, int per, int32_t* out) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t b = (uint64_t)l[i] * (uint64_t)scale;
        int64_t v;
        if (per < 4) { int sh = 4 - per; v = (int64_t)(b + (1ull << (sh - 1))) >> sh; }
        else v = (int64_t)(b << (per - 4));
        out[i] = (int32_t)(uint32_t)(uint64_t)v;
    }
}
__global__ void k_quant_i32(const int32_t* c, int64_t n, QuantParams q, int32_t* out) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = quant_i32(c[i], q);
}
__global__ void k_dequant_i32(const int32_t* l, int64_t n, int32_t scale, int per, int32_t* out) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = dequant_i32(l[i], scale, per);
}

// quant.py:171-173
__device__ __forceinline__ void dev_count_nonzero(const int64_t* l, int64_t n, unsigned long long* cnt) {
    unsigned long long c = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        c += l[i] != 0;
    c = grp_sum<64>(c);   // DPP / swizzle / lane reads (nh_packed.hpp): every lane holds the total
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(cnt, c);
}

// quant.py:153-168: sum(log2(|l|+1) + (|l|>0)*2) in float64, then int().
// np.sum of the (contiguous) term array is numpy's pairwise_sum over it in
// memory order (the shim hands the levels over in that order, np.ravel 'K'),
// replicated serially here so the float64 rounding sequence is numpy's.
// The term follows numpy's dtype rules for one level of dtype `code`
// (NH_EB_* in nanohevc.h; the 8-byte word holds an int64 value, a uint64 bit
// pattern or, for float kinds, a float64 bit pattern):
//   * np.abs and the +1 in the level's dtype (integers wrap; floats round);
//   * np.log2 in the float type numpy picks for that dtype: float16 for 8-bit
//     integers and float16, float32 for 16-bit integers and float32, float64
//     otherwise (bool: bool + 1 is int64) -- then widened to float64 by the
//     + int64 (abs > 0) * 2;
//   * log2 of 0 / a negative wrap is -inf / NaN exactly as numpy's, so the
//     shim's int() raises like the reference.
// log2 at float32 / float16 is the correctly rounded value (log2 in float64,
// then rounded); numpy's own float32 log2 on AVX-512 hosts (SVML) differs from
// it in the last bit for 437 of the 65,536 int16 magnitudes -- which moves the
// truncated int() only when a sum falls within ~1e-6 of an integer
// (DESIGN.md §2).
__device__ __forceinline__ double eb_log2_prec(double x, int prec) {
    if (prec == 64) return log2(x);
    const float l = (float)log2((double)(float)x);   // x is exact in the precision
    if (prec == 32) return (double)l;
    return (double)(float)(_Float16)l;               // numpy's half loop: half(log2f(float(x)))
}
__device__ double eb_term(int64_t v, int code) {
    if (code >= NH_EB_F16) {
        const double x = __longlong_as_double((long long)v);
        if (code == NH_EB_F64) {
            const double a = fabs(x);
            return log2(a + 1.0) + (double)((a > 0) * 2);
        }
        const float af = fabsf((float)x);
        if (code == NH_EB_F32) return eb_log2_prec((double)(af + 1.0f), 32) + (double)((af > 0) * 2);
        const _Float16 a1 = (_Float16)(af + 1.0f);   // numpy's half add: float add, rounded to half
        return eb_log2_prec((double)(float)a1, 16) + (double)((af > 0) * 2);
    }
    if (code == NH_EB_BOOL) {
        const int b = v != 0;
        return log2((double)(b + 1)) + (double)(b * 2);
    }
    if (code > 100) {   // unsigned: np.abs is the identity, the +1 wraps in the width
        const int w = code - 100;
        const uint64_t mask = w == 64 ? ~0ull : (1ull << w) - 1;
        const uint64_t u = (uint64_t)v & mask, u1 = (u + 1) & mask;
        return eb_log2_prec((double)u1, w == 8 ? 16 : w == 16 ? 32 : 64) + (double)((u > 0) * 2);
    }
    const int w = code;   // signed: np.abs and the +1 wrap in the width
    const uint64_t a = v < 0 ? 0ull - (uint64_t)v : (uint64_t)v, a1 = a + 1;
    int64_t as, as1;
    if (w == 8) { as = (int8_t)(uint8_t)a; as1 = (int8_t)(uint8_t)a1; }
    else if (w == 16) { as = (int16_t)(uint16_t)a; as1 = (int16_t)(uint16_t)a1; }
    else if (w == 32) { as = (int32_t)(uint32_t)a; as1 = (int32_t)(uint32_t)a1; }
    else { as = (int64_t)a; as1 = (int64_t)a1; }
    return eb_log2_prec((double)as1, w == 8 ? 16 : w == 16 ? 32 : 64) + (double)((as > 0) * 2);
}
// numpy's pairwise_sum (loops_utils.h.src) over term(i), i in [0, n), iteratively:
// below 8 terms a plain running sum from 0; up to 128 eight accumulators over
// the multiple-of-8 prefix, combined ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)), then
// the rest added in order; above 128 the halves n2 = n/2 - (n/2)%8 and n - n2.
template <class Term>
__device__ double pw_sum(int64_t n, Term term) {
#pragma clang fp contract(off)   // numpy rounds every add on its own: no fused multiply-adds with the terms
    struct Fr { int64_t off, n; int stage; double left; };
    Fr stk[48];
    int sp = 0;
    double ret = 0;
    stk[sp++] = {0, n, 0, 0};
    while (sp) {
        Fr& f = stk[sp - 1];
        if (f.n <= 128) {
            double res;
            if (f.n < 8) {
                res = 0.;
                for (int64_t i = 0; i < f.n; ++i) res += term(f.off + i);
            } else {
                double r[8];
                for (int j = 0; j < 8; ++j) r[j] = term(f.off + j);
                int64_t i;
                for (i = 8; i < f.n - (f.n % 8); i += 8)
                    for (int j = 0; j < 8; ++j) r[j] += term(f.off + i + j);
                res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
                for (; i < f.n; ++i) res += term(f.off + i);
            }
            --sp;
            ret = res;
            // propagate to parent
            while (sp) {
                Fr& p = stk[sp - 1];
                if (p.stage == 1) { p.left = ret; p.stage = 2;
                    int64_t n2 = p.n / 2; n2 -= n2 % 8;
                    stk[sp++] = {p.off + n2, p.n - n2, 0, 0};
                    break;
                } else { ret = p.left + ret; --sp; }
            }
        } else {
            int64_t n2 = f.n / 2; n2 -= n2 % 8;
            f.stage = 1;
            stk[sp++] = {f.off, n2, 0, 0};
        }
    }
    return ret;
}
__device__ __forceinline__ void dev_estimate_bits(const int64_t* l, int64_t n, int bits, double* out) {
    if (threadIdx.x || blockIdx.x) return;
    *out = n > 0 ? pw_sum(n, [=](int64_t i) { return eb_term(l[i], bits); }) : 0.0;   // the shim applies int() (quant.py:168)
}

// ---------------------------------------------------------------------------
// quality metrics (metrics.py:7-48) as device reductions
// ---------------------------------------------------------------------------
// Workgroup reduction (256 threads) then ONE atomic per workgroup: an atomic
// per wave on one word serialises (~90 adds/us per address).
template <class T, class F>
__device__ __forceinline__ void block_reduce_add(T v, unsigned long long* out, F) {
    __shared__ unsigned long long part[4];
    v = grp_sum<64>(v);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = (unsigned long long)v;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long s = 0;
        for (int k = 0; k < (int)(blockDim.x >> 6); ++k) s += part[k];
        if (s) atomicAdd(out, s);
    }
}
struct NoOp {};
// sum((a-b)^2) exactly in int64 (inputs are <= 16-bit samples widened by the shim)
__device__ __forceinline__ void dev_sum_sq_diff(const int64_t* a, const int64_t* b, int64_t n, unsigned long long* out) {
    unsigned long long s = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        int64_t d = a[i] - b[i];
        s += (unsigned long long)(d * d);
    }
    block_reduce_add(s, out, NoOp{});
}
// metrics.py:9-10 for any sample dtype: the shim casts both arrays to float64
// (the reference's .astype(np.float64)); np.mean(diff ** 2) is numpy's add
// reduction -- pairwise_sum above -- of the squares divided by n on the host.
// One thread walks the pairwise tree (the per-call arrays are block-sized).
__device__ __forceinline__ void dev_sum_sq_diff_f64(const double* a, const double* b, int64_t n, double* out) {
    if (threadIdx.x || blockIdx.x) return;
    // diff ** 2 is rounded before the sum adds it (contract(off) here and in pw_sum)
    *out = n > 0 ? 0.0 + pw_sum(n, [=](int64_t i) {
#pragma clang fp contract(off)
        const double d = a[i] - b[i];
        return d * d;
    }) : 0.0;
}
// metrics.py:24-26: int32 difference (wraps), np.abs (wraps at INT32_MIN), int64 sum
__device__ __forceinline__ void dev_sad_i32(const int32_t* a, const int32_t* b, int64_t n, unsigned long long* out) {
    unsigned long long s = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        int32_t d = (int32_t)((uint32_t)a[i] - (uint32_t)b[i]);
        int32_t ad = d == INT32_MIN ? d : (d < 0 ? -d : d);
        s += (unsigned long long)(long long)ad;
    }
    block_reduce_add(s, out, NoOp{});
}
// metrics.py:29-43: H . diff . H^T in int32 (wrap), sum |.| in int64
__device__ __forceinline__ void dev_satd_4x4(const int32_t* a, const int32_t* b, long long* out) {
    if (threadIdx.x || blockIdx.x) return;
    constexpr int H[4][4] = {{1, 1, 1, 1}, {1, 1, -1, -1}, {1, -1, -1, 1}, {1, -1, 1, -1}};
    uint32_t d[4][4], t[4][4];
    for (int i = 0; i < 16; ++i) d[i / 4][i % 4] = (uint32_t)a[i] - (uint32_t)b[i];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            uint32_t acc = 0;
            for (int k = 0; k < 4; ++k) acc += (uint32_t)H[i][k] * d[k][j];
            t[i][j] = acc;
        }
    long long s = 0;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            uint32_t acc = 0;
            for (int k = 0; k < 4; ++k) acc += t[i][k] * (uint32_t)H[j][k];
            int32_t v = (int32_t)acc;
            s += (v == INT32_MIN) ? (long long)v : (v < 0 ? -(long long)v : (long long)v);
        }
    *out = s;
}
// metrics.py:46-48: sum(r.astype(int64)**2), int64 wrap
__device__ __forceinline__ void dev_residual_energy(const int64_t* r, int64_t n, unsigned long long* out) {
    unsigned long long s = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        s += (unsigned long long)r[i] * (unsigned long long)r[i];
    block_reduce_add(s, out, NoOp{});
}
// batched: SSE between two int16 device buffers (frame PSNR without a host round trip)
__global__ void k_sse_i16(const int16_t* a, const int16_t* b, int64_t n, unsigned long long* out) {
    unsigned long long s = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        int32_t d = (int32_t)a[i] - (int32_t)b[i];
        s += (unsigned long long)(uint32_t)(d * d);
    }
    block_reduce_add(s, out, NoOp{});
}

static unsigned grid_for(int64_t n, int64_t cap = 8192);
static unsigned grid_red(int64_t n) { return grid_for(n, 1024); }
static unsigned grid_for(int64_t n, int64_t cap) {
    int64_t g = (n + 255) / 256;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (unsigned)g;
}


#define NH_TRY_(x)             \
    do {                       \
        int rc__ = (x);        \
        if (rc__) return rc__; \
    } while (0)

// ---------------------------------------------------------------------------
// The per-block call protocol (the drop-in path: host arrays in, host arrays out)
// ---------------------------------------------------------------------------
// Small calls (inputs <= kSmallIn bytes, outputs <= kSmallOut bytes: every
// block size the reference's callers use) are ONE launch of a single-workgroup
// kernel: the inputs travel in the kernel-argument segment, the outputs and the
// status word are stored straight into mapped pinned host memory, and the host
// waits on the stream once -- no DMA copy at all.  Larger calls are staged: one
// H2D copy of [inputs | status, accumulator], the grid-wide kernel, one D2H
// copy of [status, accumulator | outputs], one wait.  Both forms run the same
// device body, a __device__ lambda over (inputs, status/accumulator words,
// outputs).  Status word: ULLONG_MAX = ok, else the first error (report()).
// One context per device (stream, buffers), created on first use on that
// device and kept for the process; nh_release_staging() frees them all.
constexpr size_t kSmallIn = 3072, kSmallOut = 64 << 10;
// The kernel-argument block is sized to the call's inputs (256 B / 1 KB / 3 KB):
// the argument segment is written per launch, so a 4x4 call does not ship 3 KB.
template <size_t SZ>
struct SmallIn {
    alignas(16) uint8_t b[SZ];
};

// Host-side phases of the last per-block call on this thread (ns): marshal
// (inputs into the argument block), launch (the launch API), wait (launch
// returned -> completion word seen), finish (outputs copied back).
// nh_last_call_times() reads them (tools/percall.py --phases).
static thread_local int64_t g_call_ns[4] = {0, 0, 0, 0};
static inline int64_t now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

// The small form's status / accumulator words live in LDS (one workgroup): no
// device-memory reset and no agent-scope fence before the body.  After the body
// every wave waits for its own output stores (s_waitcnt 0) before the barrier,
// then one lane publishes status, accumulator and -- with a system-scope
// release -- the completion word.  (NH_SMALL_OLD builds the previous form:
// device-memory words reset under __threadfence(), a system fence per wave.)
// A body that needs an LDS scratch tile (the per-block transforms: their
// tiles are too large to live in the server's kernel as static LDS, DESIGN.md
// §4.6): every form hands it kScratch bytes of LDS as a fourth argument.
constexpr size_t kScratch = 32 * 33 * 4;   // one 32x32 transform tile (pitch 33)
template <class F>
struct ScratchBody {
    F f;
};
template <class F>
struct is_scratch_body : std::false_type {};
template <class F>
struct is_scratch_body<ScratchBody<F>> : std::true_type {};
template <class F>
__device__ __forceinline__ void run_body(const F& f, const uint8_t* in, unsigned long long* st, uint8_t* o,
                                         uint8_t* scratch) {
    if constexpr (is_scratch_body<F>::value) f.f(in, st, o, scratch);
    else f(in, st, o);
}

template <class F, size_t SZ>
__global__ void __launch_bounds__(256) k_small(SmallIn<SZ> in, F f, unsigned long long* dw, unsigned long long* hres,
                                               unsigned long long seq) {
#ifndef NH_SMALL_OLD
    (void)dw;
    __shared__ unsigned long long s_w[2];
    if (threadIdx.x == 0) {
        s_w[0] = ULLONG_MAX;   // status: no error yet
        s_w[1] = 0ull;         // accumulator of the reductions
    }
    __syncthreads();
    if constexpr (is_scratch_body<F>::value) {
        __shared__ __attribute__((aligned(16))) uint8_t s_scr[kScratch];
        run_body(f, in.b, s_w, (uint8_t*)(hres + 4), s_scr);
    } else {
        f(in.b, s_w, (uint8_t*)(hres + 4));
    }
    __builtin_amdgcn_s_waitcnt(0);        // this wave's result stores acknowledged
    __syncthreads();
    if (threadIdx.x == 0) {
        hres[0] = s_w[0];
        hres[1] = s_w[1];
        __hip_atomic_store(&hres[2], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);   // completion word, last
    }
#else
    if (threadIdx.x == 0) {
        atomicExch(&dw[0], ULLONG_MAX);   // status: no error yet
        atomicExch(&dw[1], 0ull);         // accumulator of the reductions
    }
    __threadfence();
    __syncthreads();
    if constexpr (is_scratch_body<F>::value) {
        __shared__ __attribute__((aligned(16))) uint8_t s_scr[kScratch];
        run_body(f, in.b, dw, (uint8_t*)(hres + 4), s_scr);
    } else {
        f(in.b, dw, (uint8_t*)(hres + 4));
    }
    __threadfence_system();               // this thread's result stores have reached host memory
    __syncthreads();
    if (threadIdx.x == 0) {
        hres[0] = atomicAdd(&dw[0], 0ull);
        hres[1] = atomicAdd(&dw[1], 0ull);
        __threadfence_system();
        __hip_atomic_store(&hres[2], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);   // completion word, last
    }
#endif
}

template <class F>
__global__ void __launch_bounds__(256) k_staged(const uint8_t* in, F f, unsigned long long* dw, uint8_t* out) {
    if constexpr (is_scratch_body<F>::value) {
        __shared__ __attribute__((aligned(16))) uint8_t s_scr[kScratch];
        run_body(f, in, dw, out, s_scr);
    } else {
        f(in, dw, out);
    }
}

// ---------------------------------------------------------------------------
// The block-call server: the small form without a launch per call.
// ---------------------------------------------------------------------------
// A per-block call spends most of its time in the launch API (~3.5 us) and in
// the dispatch of a fresh kernel.  While calls keep coming, one workgroup of
// k_srv stays resident instead and polls a request word in mapped pinned host
// memory.  The host writes the inputs, the call's captures and the device
// address of the body's thunk, then the request word (release):
// seq << 12 | flags << 8 | input bytes / 16.  The server then takes thunk
// address, captures and inputs into LDS in ONE round trip of parallel loads
// (the word already told it how many), calls the body through the thunk (an
// indirect call), waits for its wave's result stores, and after the barrier one
// lane publishes the completion word seq << 8 | error code with a system-scope
// release -- preceded, for reductions (flag 1), by the accumulator into the
// first output word.  PCIe round trips per call: poll, intake, result
// acknowledgement (+1 for reductions).  The server leaves -- writing its epoch
// into `exited`, its last act -- when no request came for `idle` ticks of the
// 100 MHz constant clock, after `life` ticks in total, after kSrvMaxPolls
// polls, or on a stop request (thunk address 0).  Every exit path is reached by
// every wave, so the grid always drains.  The host relaunches it when it finds
// `exited` equal to the epoch it launched with and the call's completion word
// unwritten.  A kernel with an indirect call allocates the static LDS of every
// address-taken callee and cannot size its stack, so the transforms take their
// tile from the server's LDS scratch (ScratchBody) and the bodies with 1.5 KB of
// stack (the float64 pairwise sums) stay on k_small.  Requests carry up to
// kSrvIn bytes of inputs (k_small's argument block: 3 KB).
constexpr size_t kSrvCap = 128;                       // bytes of a body's captures
constexpr size_t kSrvIn = 8192;                       // input bytes a served call may carry
constexpr unsigned kSrvMaxPolls = 50u * 1000u * 1000u;
constexpr unsigned long long kSrvFlagAcc = 1;         // flags: write the accumulator to output word 0
typedef void (*SrvFn)(const uint8_t*, unsigned long long*, uint8_t*, const uint8_t*, uint8_t*);

struct SrvReq {                        // mapped pinned host memory, 64-byte lines
    unsigned long long word;           // host: seq << 16 | flags << 12 | input bytes / 16, written last
    unsigned long long pad0[7];
    unsigned long long exited;         // server: the epoch it left with (its last store)
    unsigned long long pad1[7];
    unsigned long long done;           // server: seq << 8 | error code (0 = ok), the call's last store
    unsigned long long pad2[7];
    unsigned long long fn;             // host: device address of srv_thunk<F>; 0 = stop
    unsigned long long pad3[7];
    alignas(16) uint8_t cap[kSrvCap];  // host: the body's captures
    alignas(16) uint8_t in[kSrvIn];    // host: the inputs
};
constexpr unsigned kSrvFnWord = offsetof(SrvReq, fn) / 8, kSrvCapWord = offsetof(SrvReq, cap) / 8;
static_assert(offsetof(SrvReq, in) == offsetof(SrvReq, cap) + kSrvCap, "captures and inputs are contiguous");

template <class F>
__device__ __attribute__((noinline)) void srv_thunk(const uint8_t* in, unsigned long long* st, uint8_t* o,
                                                    const uint8_t* cap, uint8_t* scratch) {
    run_body(*reinterpret_cast<const F*>(cap), in, st, o, scratch);
}
template <class F>
__global__ void k_srv_addr(unsigned long long* out) {
    out[0] = (unsigned long long)(SrvFn)&srv_thunk<F>;
}

__device__ __forceinline__ unsigned long long ld_sys(const unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void __launch_bounds__(256) k_srv(SrvReq* q, unsigned long long* hout, unsigned long long last,
                                              unsigned long long epoch, unsigned long long idle,
                                              unsigned long long life) {
    __shared__ alignas(16) unsigned long long s_ci[(kSrvCap + kSrvIn) / 8];   // captures | inputs
    __shared__ alignas(16) uint8_t s_scr[kScratch];                          // ScratchBody bodies' tile
    __shared__ unsigned long long s_fn;
    __shared__ unsigned long long s_w[2];
    __shared__ unsigned long long s_word;     // the request word taken (== last: leave)
    const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
    const unsigned long long* qw = (const unsigned long long*)q;
    unsigned polls = 0;
    for (;;) {
        if (threadIdx.x == 0) {
            const unsigned long long t_idle = __builtin_amdgcn_s_memrealtime();
            unsigned long long v = last;
            for (;;) {
                v = __hip_atomic_load(&q->word, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
                if (v != last) break;
                const unsigned long long now = __builtin_amdgcn_s_memrealtime();
                if (now - t_idle > idle || now - t_start > life || ++polls > kSrvMaxPolls) break;
                __builtin_amdgcn_s_sleep(1);
            }
            s_word = v;
            s_w[0] = ULLONG_MAX;   // status: no error yet
            s_w[1] = 0ull;         // accumulator of the reductions
        }
        __syncthreads();
        const unsigned long long word = s_word;
        if (word == last) {   // idle, lifetime or poll cap
            if (threadIdx.x == 0) __hip_atomic_store(&q->exited, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            return;
        }
        // intake: thunk address, captures and inputs, one round of parallel loads
        const unsigned nwords = (unsigned)(kSrvCap / 8 + 2 * (word & 0xfff) < (kSrvCap + kSrvIn) / 8
                                               ? kSrvCap / 8 + 2 * (word & 0xfff) : (kSrvCap + kSrvIn) / 8);
        constexpr unsigned kIw = (unsigned)((kSrvCap + kSrvIn) / 8 + 255) / 256;   // words per thread
        {   // every load issued before the first use
            unsigned long long v[kIw], c = 0;
#pragma unroll
            for (unsigned k = 0; k < kIw; ++k) {
                const unsigned i = threadIdx.x + 256 * k;
                v[k] = i < nwords ? ld_sys(qw + kSrvCapWord + i) : 0ull;
            }
            if (threadIdx.x == 0) c = ld_sys(qw + kSrvFnWord);
#pragma unroll
            for (unsigned k = 0; k < kIw; ++k) {
                const unsigned i = threadIdx.x + 256 * k;
                if (i < nwords) s_ci[i] = v[k];
            }
            if (threadIdx.x == 0) s_fn = c;
        }
        __syncthreads();
        const unsigned long long fn = s_fn;
        if (fn == 0) {   // stop request
            if (threadIdx.x == 0) __hip_atomic_store(&q->exited, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            return;
        }
        const SrvFn f = (SrvFn)(((unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((unsigned)(fn >> 32)) << 32) |
                                (unsigned)__builtin_amdgcn_readfirstlane((unsigned)fn));
        f((const uint8_t*)(s_ci + kSrvCap / 8), s_w, (uint8_t*)hout, (const uint8_t*)s_ci, s_scr);
        __builtin_amdgcn_s_waitcnt(0);        // this wave's result stores acknowledged
        __syncthreads();
        if (threadIdx.x == 0) {
            const unsigned long long st = s_w[0];
            if ((word >> 12) & kSrvFlagAcc) hout[0] = s_w[1];
            __hip_atomic_store(&q->done, ((word >> 16) << 8) | (st == ULLONG_MAX ? 0ull : (st & 0xff)),
                               __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);   // completion word, last
        }
        last = word;
    }
}

struct Staging {
    std::mutex mu;
    bool ready = false;
    hipStream_t stream = nullptr;
    uint8_t* dbuf = nullptr;              // staged form: device side
    uint8_t* hbuf = nullptr;              //              pinned host side
    size_t cap = 0;
    unsigned long long* dwork = nullptr;  // small form: status, accumulator (device)
    uint8_t* hres = nullptr;              //             mapped pinned results (host view):
                                          //             status, accumulator, completion word, pad, outputs
    unsigned long long seq = 0;           //             completion sequence number of the last call
    uint8_t* hres_dev = nullptr;          //             the same memory, device view
    SrvReq* req = nullptr;                // block-call server: request block (host view)
    SrvReq* req_dev = nullptr;            //                    the same memory, device view
    unsigned long long epoch = 0;         //                    epoch of the last server launched
    bool srv_alive = false;               //                    launched and not known to have left
    unsigned long long clock_khz = 100000;  //                    the constant clock k_srv times itself with
    bool stack_ok = false;                //                    the per-thread stack limit covers the callees' stack
    int64_t n_served = 0, n_launches = 0, n_kernel = 0;   // nh_block_server_stats
};
constexpr int kMaxDevices = 64;
static Staging g_staging[kMaxDevices];

static int staging_current(Staging** out) {
    // the device count of the process is fixed: asked once (a successful answer is kept)
    static std::atomic<int> ndev{-1};
    int n = ndev.load(std::memory_order_relaxed), dev = 0;
    if (n <= 0) {
        if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
        if (n > 0) ndev.store(n, std::memory_order_relaxed);
    }
    if (n == 0) {
        set_error("no HIP device visible (nano-hevc_amd needs an MI355X; there is no CPU fallback)");
        return NH_ENODEV;
    }
    NH_HIP(hipGetDevice(&dev));
    if (dev < 0 || dev >= kMaxDevices) {
        set_error("device index out of range");
        return NH_EARG;
    }
    *out = &g_staging[dev];
    return NH_OK;
}

static void staging_free(Staging& s) {   // caller holds s.mu, current device = the context's
    if (s.dbuf) (void)hipFree(s.dbuf);
    if (s.hbuf) (void)hipHostFree(s.hbuf);
    if (s.dwork) (void)hipFree(s.dwork);
    if (s.hres) (void)hipHostFree(s.hres);
    if (s.req) (void)hipHostFree(s.req);
    if (s.stream) (void)hipStreamDestroy(s.stream);
    s.dbuf = s.hbuf = s.hres = s.hres_dev = nullptr;
    s.req = s.req_dev = nullptr;
    s.srv_alive = false;
    s.dwork = nullptr;
    s.stream = nullptr;
    s.cap = 0;
    s.ready = false;
}

// Idle time after which the block-call server leaves (us; default 200, 0 = no
// server: every small call is a k_small launch).  nh_block_server_set_idle_us().
static std::atomic<long> g_srv_idle_us{100};   // a device-wide sync after calls waits up to this long
static long server_idle_us() { return g_srv_idle_us.load(std::memory_order_relaxed); }

static int staging_init(Staging& s) {    // caller holds s.mu
    if (s.ready) return NH_OK;
    NH_HIP(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking));
    NH_HIP(hipMalloc(&s.dwork, 256));
    NH_HIP(hipHostMalloc(&s.hres, 32 + kSmallOut, hipHostMallocMapped | hipHostMallocCoherent));
    std::memset(s.hres, 0, 32);
    s.seq = 0;
    NH_HIP(hipHostGetDevicePointer((void**)&s.hres_dev, s.hres, 0));
    NH_HIP(hipHostMalloc((void**)&s.req, sizeof(SrvReq), hipHostMallocMapped | hipHostMallocCoherent));
    std::memset((void*)s.req, 0, sizeof(SrvReq));
    NH_HIP(hipHostGetDevicePointer((void**)&s.req_dev, s.req, 0));
    int dev = 0, khz = 0;
    NH_HIP(hipGetDevice(&dev));
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0) khz = 100000;
    s.clock_khz = (unsigned long long)khz;
    // k_srv's indirect calls run on the runtime's per-thread stack (hipLimitStackSize);
    // the served bodies need at most 32 B of it (inverse 32x32 transform)
    size_t stack = 0;
    s.stack_ok = hipDeviceGetLimit(&stack, hipLimitStackSize) == hipSuccess && stack >= 256;
    s.epoch = 0;
    s.srv_alive = false;
    s.ready = true;
    return NH_OK;
}

// Posts a stop request to a resident server (no wait: launches that follow on
// the context's stream queue behind its exit).  Caller holds s.mu.
static void server_post(Staging& s, unsigned long long word) {
    __atomic_store_n(&s.req->word, word, __ATOMIC_RELEASE);
}

static void server_stop(Staging& s) {
    if (!s.srv_alive) return;
    s.req->fn = 0;
    server_post(s, ++s.seq << 16);
    s.srv_alive = false;
}

// Launches a server that takes the request word now posted (last = anything else).
static int server_launch(Staging& s, unsigned long long word) {
    const unsigned long long idle = (unsigned long long)server_idle_us() * s.clock_khz / 1000ull;
    k_srv<<<1, 256, 0, s.stream>>>(s.req_dev, (unsigned long long*)(s.hres_dev + 32), ~word, ++s.epoch, idle,
                                    s.clock_khz * 1000ull /* 1 s */);
    NH_HIP(hipGetLastError());
    s.srv_alive = true;
    ++s.n_launches;
    return NH_OK;
}

// Device address of srv_thunk<F> on the current device (asked once per device).
template <class F>
static int server_fn(Staging& s, int dev, unsigned long long* fn) {
    static std::atomic<unsigned long long> addr[kMaxDevices];
    unsigned long long a = addr[dev].load(std::memory_order_acquire);
    if (!a) {
        server_stop(s);
        k_srv_addr<F><<<1, 1, 0, s.stream>>>(s.dwork);
        NH_HIP(hipGetLastError());
        NH_HIP(hipMemcpyAsync(&a, s.dwork, 8, hipMemcpyDeviceToHost, s.stream));
        NH_HIP(hipStreamSynchronize(s.stream));
        if (!a) {
            set_error("block-call server: null thunk address");
            return NH_EHIP;
        }
        addr[dev].store(a, std::memory_order_release);
    }
    *fn = a;
    return NH_OK;
}

static int staging_grow(Staging& s, size_t bytes) {   // staged form only; grow-only
    if (bytes <= s.cap) return NH_OK;
    const size_t c = align_up(bytes < (1u << 20) ? (1u << 20) : bytes * 2, 4096);
    if (s.dbuf) { (void)hipFree(s.dbuf); s.dbuf = nullptr; }
    if (s.hbuf) { (void)hipHostFree(s.hbuf); s.hbuf = nullptr; }
    s.cap = 0;
    NH_HIP(hipMalloc(&s.dbuf, c));
    NH_HIP(hipHostMalloc(&s.hbuf, c, hipHostMallocDefault));
    s.cap = c;
    return NH_OK;
}

// The small form's wait: the kernel's last store is the call's sequence number
// into mapped host memory (after every result store), so the host polls that
// word instead of a stream synchronisation (the stream keeps the calls ordered,
// so the buffer is never reused under a running kernel).  Bounded: after ~1 s
// it falls back to hipStreamSynchronize, which also reports a faulted kernel.
static int wait_completion(hipStream_t stream, const unsigned long long* word, unsigned long long seq) {
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned spins = 1;; ++spins) {
        if (__atomic_load_n(word, __ATOMIC_ACQUIRE) == seq) return NH_OK;
        if ((spins & 1023) == 0) {
            const hipError_t q = hipStreamQuery(stream);
            if (q != hipSuccess && q != hipErrorNotReady) {
                set_error(std::string("per-block kernel: ") + hipGetErrorString(q));
                return NH_EHIP;
            }
            if (q == hipSuccess || std::chrono::steady_clock::now() - t0 > std::chrono::seconds(1)) break;
        }
    }
    NH_HIP(hipStreamSynchronize(stream));
    if (__atomic_load_n(word, __ATOMIC_ACQUIRE) != seq) {
        set_error("per-block kernel finished without its completion word");
        return NH_EHIP;
    }
    return NH_OK;
}

// The served form's wait: the completion word, or -- when the server left
// without answering (its exit raced the request) -- a relaunch that takes the
// pending request.  `exited` is the server's last store, after any completion
// word, so the completion word is read again after `exited` before relaunching.
static int server_wait(Staging& s, unsigned long long word, unsigned long long* done) {
    const unsigned long long seq = word >> 16;
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned spins = 1;; ++spins) {
        unsigned long long d = __atomic_load_n(&s.req->done, __ATOMIC_ACQUIRE);
        if ((d >> 8) == seq) { *done = d; return NH_OK; }
        if (__atomic_load_n(&s.req->exited, __ATOMIC_ACQUIRE) == s.epoch) {
            d = __atomic_load_n(&s.req->done, __ATOMIC_ACQUIRE);
            if ((d >> 8) == seq) { *done = d; return NH_OK; }
            NH_TRY_(server_launch(s, word));
        }
        if ((spins & 1023) == 0) {
            const hipError_t q = hipStreamQuery(s.stream);
            if (q != hipSuccess && q != hipErrorNotReady) {
                s.srv_alive = false;
                set_error(std::string("block-call server: ") + hipGetErrorString(q));
                return NH_EHIP;
            }
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) break;
        }
    }
    s.srv_alive = false;   // the lifetime bound (1 s) has ended it by now
    NH_HIP(hipStreamSynchronize(s.stream));
    const unsigned long long d = __atomic_load_n(&s.req->done, __ATOMIC_ACQUIRE);
    if ((d >> 8) != seq) {
        set_error("block-call server: no answer within 2 s");
        return NH_EHIP;
    }
    *done = d;
    return NH_OK;
}

class BlockCall {
  public:
    // Registers an input array (copied when the call runs); returns its byte
    // offset in the call's input area (the same in both forms).
    size_t in(const void* p, size_t bytes) {
        const size_t o = end_;
        ins_[n_++] = {p, bytes, o};
        end_ = align_up(o + bytes, 16);
        return o;
    }
    // Runs body f on `grid` workgroups (staged form; the small form always runs
    // one workgroup) and returns its out_bytes of output into `out` -- or, with
    // from_acc, the 8-byte accumulator word the body's reductions added into.
    // kServe: the body may run on the block-call server (no large LDS tiles).
    template <bool kServe = true, class F>
    int run(unsigned grid, F f, void* out, size_t out_bytes, bool from_acc = false) {
        const int64_t t0 = now_ns();
        Staging* S = nullptr;
        NH_TRY_(staging_current(&S));
        std::lock_guard<std::mutex> lk(S->mu);
        NH_TRY_(staging_init(*S));
        const size_t res = from_acc ? 0 : out_bytes;
        unsigned long long st, acc;
        if constexpr (kServe) {
            static_assert(sizeof(F) <= kSrvCap && alignof(F) <= 16, "captures exceed the server's block");
            if (server_idle_us() > 0 && end_ <= kSrvIn && res <= kSmallOut &&
                (S->stack_ok || !is_scratch_body<F>::value)) {
                unsigned long long fn = 0;
                NH_TRY_(server_fn<F>(*S, (int)(S - g_staging), &fn));
                SrvReq* q = S->req;
                for (int i = 0; i < n_; ++i)
                    if (ins_[i].bytes) std::memcpy(q->in + ins_[i].off, ins_[i].p, ins_[i].bytes);
                std::memcpy(q->cap, (const void*)&f, sizeof(F));
                q->fn = fn;
                const unsigned long long word =
                    (++S->seq << 16) | ((from_acc ? kSrvFlagAcc : 0ull) << 12) | (align_up(end_, 16) / 16);
                const int64_t t1 = now_ns();
                server_post(*S, word);
                if (!S->srv_alive || __atomic_load_n(&q->exited, __ATOMIC_ACQUIRE) == S->epoch)
                    NH_TRY_(server_launch(*S, word));
                const int64_t t2 = now_ns();
                unsigned long long done = 0;
                NH_TRY_(server_wait(*S, word, &done));
                const int64_t t3 = now_ns();
                const unsigned long long* o = (const unsigned long long*)S->hres + 4;
                const int code = (int)(done & 0xff);
                if (!code && res) std::memcpy(out, o, res);
                if (!code && from_acc) std::memcpy(out, o, 8);
                ++S->n_served;
                g_call_ns[0] = t1 - t0;
                g_call_ns[1] = t2 - t1;
                g_call_ns[2] = t3 - t2;
                g_call_ns[3] = now_ns() - t3;
                return -code;
            }
        }
        server_stop(*S);   // launches below queue behind its exit on the same stream
        ++S->n_kernel;
        if (end_ <= kSmallIn && res <= kSmallOut) {
            const unsigned long long seq = ++S->seq;
            int64_t t1 = 0;
            auto launch = [&](auto sz_c) -> int {
                constexpr size_t SZ = decltype(sz_c)::value;
                SmallIn<SZ> si;
                for (int i = 0; i < n_; ++i)
                    if (ins_[i].bytes) std::memcpy(si.b + ins_[i].off, ins_[i].p, ins_[i].bytes);
                t1 = now_ns();
                k_small<<<1, 256, 0, S->stream>>>(si, f, S->dwork, (unsigned long long*)S->hres_dev, seq);
                NH_HIP(hipGetLastError());
                return NH_OK;
            };
            if (end_ <= 256) NH_TRY_(launch(std::integral_constant<size_t, 256>{}));
            else if (end_ <= 1024) NH_TRY_(launch(std::integral_constant<size_t, 1024>{}));
            else NH_TRY_(launch(std::integral_constant<size_t, kSmallIn>{}));
            const int64_t t2 = now_ns();
            unsigned long long* r = (unsigned long long*)S->hres;
            NH_TRY_(wait_completion(S->stream, &r[2], seq));
            const int64_t t3 = now_ns();
            st = r[0];
            acc = r[1];
            if (st == ULLONG_MAX && res) std::memcpy(out, r + 4, res);
            g_call_ns[0] = t1 - t0;
            g_call_ns[1] = t2 - t1;
            g_call_ns[2] = t3 - t2;
            g_call_ns[3] = now_ns() - t3;
        } else {
            const size_t wo = align_up(end_, 256), oo = wo + 256;
            NH_TRY_(staging_grow(*S, oo + res));
            for (int i = 0; i < n_; ++i)
                if (ins_[i].bytes) std::memcpy(S->hbuf + ins_[i].off, ins_[i].p, ins_[i].bytes);
            unsigned long long* hw = (unsigned long long*)(S->hbuf + wo);
            hw[0] = ULLONG_MAX;
            hw[1] = 0;
            const int64_t t1 = now_ns();
            NH_HIP(hipMemcpyAsync(S->dbuf, S->hbuf, wo + 16, hipMemcpyHostToDevice, S->stream));
            k_staged<<<grid, 256, 0, S->stream>>>(S->dbuf, f, (unsigned long long*)(S->dbuf + wo), S->dbuf + oo);
            NH_HIP(hipGetLastError());
            NH_HIP(hipMemcpyAsync(S->hbuf + wo, S->dbuf + wo, oo - wo + res, hipMemcpyDeviceToHost, S->stream));
            const int64_t t2 = now_ns();
            NH_HIP(hipStreamSynchronize(S->stream));
            const int64_t t3 = now_ns();
            st = hw[0];
            acc = hw[1];
            if (st == ULLONG_MAX && res) std::memcpy(out, S->hbuf + oo, res);
            g_call_ns[0] = t1 - t0;
            g_call_ns[1] = t2 - t1;
            g_call_ns[2] = t3 - t2;
            g_call_ns[3] = now_ns() - t3;
        }
        if (st != ULLONG_MAX) return -(int)(st & 0xff);
        if (from_acc) std::memcpy(out, &acc, 8);
        return NH_OK;
    }

  private:
    struct In {
        const void* p;
        size_t bytes, off;
    };
    In ins_[4];
    int n_ = 0;
    size_t end_ = 0;
};

}  // namespace nh

using namespace nh;

// ===========================================================================
// C ABI
// ===========================================================================
extern "C" {

const char* nh_version(void) { return "nano-hevc-amd 0.1 (gfx950)"; }
const char* nh_last_error(void) { return g_err.c_str(); }

int nh_device_count(int* count) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    *count = n;
    return NH_OK;
}

using U8 = const uint8_t*;
using ST = unsigned long long*;

int nh_staging_bytes(int device, int64_t* bytes) {
    if (device < 0 || device >= kMaxDevices || !bytes) return NH_EARG;
    Staging& s = g_staging[device];
    std::lock_guard<std::mutex> lk(s.mu);
    *bytes = s.ready ? (int64_t)(2 * s.cap + 256 + 32 + kSmallOut) : 0;
    return NH_OK;
}

int nh_release_staging(void) {
    int cur = 0;
    NH_HIP(hipGetDevice(&cur));
    int first_err = NH_OK;
    for (int d = 0; d < kMaxDevices; ++d) {
        Staging& s = g_staging[d];
        std::lock_guard<std::mutex> lk(s.mu);
        if (!s.ready) continue;
        const hipError_t e = hipSetDevice(d);
        if (e != hipSuccess) {   // skip this device, free the others, restore the caller's device, report
            if (first_err == NH_OK) {
                set_error(std::string("nh_release_staging: hipSetDevice: ") + hipGetErrorString(e));
                first_err = NH_EHIP;
            }
            continue;
        }
        server_stop(s);
        (void)hipStreamSynchronize(s.stream);
        staging_free(s);
    }
    const hipError_t e = hipSetDevice(cur);
    if (e != hipSuccess && first_err == NH_OK) {
        set_error(std::string("nh_release_staging: hipSetDevice: ") + hipGetErrorString(e));
        first_err = NH_EHIP;
    }
    return first_err;
}

int nh_block_server_stop(void) {
    bool any = false;   // no HIP call at all unless a server was started (it runs at interpreter exit)
    for (int d = 0; d < kMaxDevices && !any; ++d) {
        std::lock_guard<std::mutex> lk(g_staging[d].mu);
        any = g_staging[d].ready && g_staging[d].srv_alive;
    }
    if (!any) return NH_OK;
    int cur = 0;
    NH_HIP(hipGetDevice(&cur));
    int first_err = NH_OK;
    for (int d = 0; d < kMaxDevices; ++d) {
        Staging& s = g_staging[d];
        std::lock_guard<std::mutex> lk(s.mu);
        if (!s.ready || !s.srv_alive) continue;
        if (hipSetDevice(d) != hipSuccess) continue;
        server_stop(s);
        const hipError_t e = hipStreamSynchronize(s.stream);
        if (e != hipSuccess && first_err == NH_OK) {
            set_error(std::string("nh_block_server_stop: ") + hipGetErrorString(e));
            first_err = NH_EHIP;
        }
    }
    (void)hipSetDevice(cur);
    return first_err;
}

int nh_block_server_set_idle_us(int64_t us) {
    if (us < 0 || us > 1000000) return NH_EARG;
    g_srv_idle_us.store((long)us, std::memory_order_relaxed);
    if (us == 0) return nh_block_server_stop();
    return NH_OK;
}

int nh_block_server_stats(int device, int64_t* out) {
    if (device < 0 || device >= kMaxDevices || !out) return NH_EARG;
    Staging& s = g_staging[device];
    std::lock_guard<std::mutex> lk(s.mu);
    out[0] = s.n_served;
    out[1] = s.n_launches;
    out[2] = s.n_kernel;
    out[3] = server_idle_us();
    return NH_OK;
}

int nh_last_call_times(int64_t* ns) {
    if (!ns) return NH_EARG;
    for (int i = 0; i < 4; ++i) ns[i] = g_call_ns[i];
    return NH_OK;
}

int nh_intra_dc(const int64_t* top, int64_t ntop, const int64_t* left, int64_t nleft, int64_t size,
                int variant4x4, int16_t* out) {
    if (ntop < 0 || nleft < 0) return NH_EARG;
    if (!variant4x4 && size == 0) return NH_EZERODIV;
    if (!variant4x4 && size < 0) return NH_EARG;
    const int64_t nout = variant4x4 ? 16 : size * size;
    BlockCall c;
    const size_t ot = c.in(top, ntop * 8), ol = c.in(left, nleft * 8);
    return c.run(1, [=] __device__(U8 in, ST st, uint8_t* o) {
        dev_intra_dc((const int64_t*)(in + ot), ntop, (const int64_t*)(in + ol), nleft, size, variant4x4,
                     (int16_t*)o, st);
    }, out, nout * 2);
}

int nh_intra_planar(const int64_t* top, int64_t ntop, const int64_t* left, int64_t nleft, int64_t top_right,
                    int tr_kind, int64_t bottom_left, int bl_kind, int64_t size, int64_t log2size, int16_t* out) {
    const auto kind_ok = [](int k) { return k == 0 || k == 1 || k == 8 || k == 16 || k == 32 || k == 64 || k == -8 ||
                                            k == -16 || k == -32 || k == -64; };
    if (ntop < 0 || nleft < 0 || size < 0 || !kind_ok(tr_kind) || !kind_ok(bl_kind)) return NH_EARG;
    if (size > (1ll << 24)) { set_error("intra_planar: size > 2^24 unsupported"); return NH_EARG; }
    const int64_t nout = size * size;
    if (nout == 0) return NH_OK;
    BlockCall c;
    const size_t ot = c.in(top, ntop * 8), ol = c.in(left, nleft * 8);
    return c.run(grid_for(nout), [=] __device__(U8 in, ST st, uint8_t* o) {
        dev_intra_planar((const int64_t*)(in + ot), ntop, (const int64_t*)(in + ol), nleft, top_right, tr_kind,
                         bottom_left, bl_kind, size, log2size, (int16_t*)o, st);
    }, out, nout * 2);
}

int nh_intra_angular(const int64_t* top, int64_t ntop, const int64_t* left, int64_t nleft, int64_t corner,
                     int mode, int64_t size, int16_t* out) {
    int idx = mode - 2;  // INTRA_PRED_ANGLE[mode - 2] with Python list indexing (D10)
    if (idx < -33 || idx > 32) return NH_EINDEX;
    if (idx < 0) idx += 33;
    const int angle = intra_angle(idx);
    const int vert = mode >= 18;
    if (ntop < 0 || nleft < 0 || size < 0) return NH_EARG;
    if (size > kMaxAngSize) { set_error("intra_angular: size > 2048 unsupported"); return NH_EARG; }
    const int64_t nout = size * size;
    BlockCall c;
    const size_t ot = c.in(top, ntop * 8), ol = c.in(left, nleft * 8);
    return c.run(1, [=] __device__(U8 in, ST st, uint8_t* o) {
        dev_intra_angular((const int64_t*)(in + ot), ntop, (const int64_t*)(in + ol), nleft, corner, angle, vert, size,
                          (int16_t*)o, st);
    }, out, nout * 2);
}

static int elementwise16(const int16_t* a, const int16_t* b, int64_t n, int16_t* out, int add) {
    if (n < 0) return NH_EARG;
    if (n == 0) return NH_OK;
    BlockCall c;
    const size_t oa = c.in(a, n * 2), ob = c.in(b, n * 2);
    return c.run(grid_for(n), [=] __device__(U8 in, ST, uint8_t* o) {
        dev_residual((const int16_t*)(in + oa), (const int16_t*)(in + ob), n, (int16_t*)o, add);
    }, out, n * 2);
}
int nh_residual(const int16_t* orig, const int16_t* pred, int64_t n, int16_t* out) {
    return elementwise16(orig, pred, n, out, 0);
}
int nh_reconstruct(const int16_t* pred, const int16_t* res, int64_t n, int16_t* out) {
    return elementwise16(pred, res, n, out, 1);
}

int nh_clip(const int64_t* x, int64_t n, int64_t maxval, int16_t* out) {
    if (n < 0) return NH_EARG;
    if (n == 0) return NH_OK;
    BlockCall c;
    const size_t ox = c.in(x, n * 8);
    return c.run(grid_for(n), [=] __device__(U8 in, ST, uint8_t* o) {
        dev_clip((const int64_t*)(in + ox), n, maxval, (int16_t*)o);
    }, out, n * 2);
}

}  // extern "C"

template <int N, bool DST, bool FWD>
static int block_transform_n(const int32_t* in, int32_t* out) {
    BlockCall c;
    const size_t oi = c.in(in, N * N * 4);
    auto body = [=] __device__(U8 i, ST, uint8_t* o, uint8_t* scr) {
        dev_transform_on<N, DST, FWD>((const int32_t*)(i + oi), (int32_t*)o, 1, (int32_t (*)[N][N + 1])scr);
    };
    return c.run(1, ScratchBody<decltype(body)>{body}, out, N * N * 4);
}
template <bool FWD>
static int block_transform(const int32_t* in, int64_t size, int use_dst, int32_t* out) {
    switch (size) {   // transform.py:150-151: other sizes raise ValueError
        case 4: return use_dst ? block_transform_n<4, true, FWD>(in, out) : block_transform_n<4, false, FWD>(in, out);
        case 8: return block_transform_n<8, false, FWD>(in, out);
        case 16: return block_transform_n<16, false, FWD>(in, out);
        case 32: return block_transform_n<32, false, FWD>(in, out);
        default: return NH_EVALUE;
    }
}
extern "C" {

int nh_forward_transform(const int32_t* in, int64_t size, int use_dst, int32_t* out) {
    return block_transform<true>(in, size, use_dst, out);
}
int nh_inverse_transform(const int32_t* in, int64_t size, int use_dst, int32_t* out) {
    return block_transform<false>(in, size, use_dst, out);
}

static void qp_params(int qp, int* per, int* rem) {  // quant.py:25-38
    qp = qp < 0 ? 0 : (qp > 51 ? 51 : qp);
    *per = qp / 6;
    *rem = qp % 6;
}

int nh_quantize(const int64_t* coeff, int64_t n, int qp, int64_t log2size, int is_intra, int abs_bits,
                int32_t* out) {
    if (n < 0 || (abs_bits != 8 && abs_bits != 16 && abs_bits != 32 && abs_bits != 64)) return NH_EARG;
    int per, rem;
    qp_params(qp, &per, &rem);
    const int64_t shift = 14 + per + log2size;  // quant.py:77 (D3)
    if (shift < 0 || shift > 62) return NH_EOVERFLOW;
    const uint64_t off = is_intra ? (1ull << shift) / 3 : (1ull << shift) / 6;
    if (n == 0) return NH_OK;
    const uint64_t mf = (uint64_t)quant_scale(rem);
    BlockCall c;
    const size_t oi = c.in(coeff, n * 8);
    return c.run(grid_for(n), [=] __device__(U8 in, ST, uint8_t* o) {
        dev_quant_i64((const int64_t*)(in + oi), n, mf, off, (int)shift, abs_bits, (int32_t*)o);
    }, out, n * 4);
}

int nh_quantize_abs(const int64_t* abs_coeff, int64_t n, int qp, int64_t log2size, int is_intra, int64_t* out) {
    if (n < 0) return NH_EARG;
    int per, rem;
    qp_params(qp, &per, &rem);
    const int64_t shift = 14 + per + log2size;  // quant.py:73 (D3)
    if (shift < 0 || shift > 62) return NH_EOVERFLOW;
    const uint64_t off = is_intra ? (1ull << shift) / 3 : (1ull << shift) / 6;
    if (n == 0) return NH_OK;
    const uint64_t mf = (uint64_t)quant_scale(rem);
    BlockCall c;
    const size_t oi = c.in(abs_coeff, n * 8);
    return c.run(grid_for(n), [=] __device__(U8 in, ST, uint8_t* o) {
        dev_quant_abs64((const int64_t*)(in + oi), n, mf, off, (int)shift, (int64_t*)o);
    }, out, n * 8);
}

int nh_dequantize(const int64_t* level, int64_t n, int qp, int32_t* out) {
    if (n < 0) return NH_EARG;
    if (n == 0) return NH_OK;
    int per, rem;
    qp_params(qp, &per, &rem);
    const int64_t scale = dequant_scale(rem);
    BlockCall c;
    const size_t oi = c.in(level, n * 8);
    return c.run(grid_for(n), [=] __device__(U8 in, ST, uint8_t* o) {
        dev_dequant_i64((const int64_t*)(in + oi), n, scale, per, (int32_t*)o);
    }, out, n * 4);
}

int nh_count_nonzero(const int64_t* level, int64_t n, int64_t* count) {
    if (n < 0) return NH_EARG;
    BlockCall c;
    const size_t oi = c.in(level, n * 8);
    return c.run(grid_red(n), [=] __device__(U8 in, ST st, uint8_t*) {
        dev_count_nonzero((const int64_t*)(in + oi), n, st + 1);
    }, count, 8, true);
}

static bool eb_code_ok(int c) {
    switch (c) {
        case NH_EB_I8: case NH_EB_I16: case NH_EB_I32: case NH_EB_I64:
        case NH_EB_U8: case NH_EB_U16: case NH_EB_U32: case NH_EB_U64:
        case NH_EB_BOOL: case NH_EB_F16: case NH_EB_F32: case NH_EB_F64: return true;
        default: return false;
    }
}

int nh_estimate_bits(const int64_t* level, int64_t n, int abs_bits, double* bits) {
    if (n < 0 || !eb_code_ok(abs_bits)) return NH_EARG;
    BlockCall c;
    const size_t oi = c.in(level, n * 8);
    return c.run<false>(1, [=] __device__(U8 in, ST, uint8_t* o) {   // 1.5 KB of stack: k_small
        dev_estimate_bits((const int64_t*)(in + oi), n, abs_bits, (double*)o);
    }, bits, 8);
}

// ----- batched device entry points -----
int nh_fwd_transform_batch(const int32_t* d_in, int32_t* d_out, int64_t nblocks, int size, int use_dst,
                           void* stream) {
    if (!d_in || !d_out || nblocks < 0) return NH_EARG;
    return launch_transform<true>(d_in, d_out, nblocks, size, use_dst, as_stream(stream));
}
int nh_inv_transform_batch(const int32_t* d_in, int32_t* d_out, int64_t nblocks, int size, int use_dst,
                           void* stream) {
    if (!d_in || !d_out || nblocks < 0) return NH_EARG;
    return launch_transform<false>(d_in, d_out, nblocks, size, use_dst, as_stream(stream));
}
int nh_quant_batch(const int32_t* d_coeff, int32_t* d_level, int64_t n, int qp, int log2size, int is_intra,
                   void* stream) {
    if (!d_coeff || !d_level || n < 0) return NH_EARG;
    int per, rem;
    qp_params(qp, &per, &rem);
    const int shift = 14 + per + log2size;
    if (shift < 1 || shift > 62) return NH_EOVERFLOW;
    QuantParams q;
    q.mf = quant_scale(rem);
    q.off = (uint32_t)(is_intra ? (1ull << shift) / 3 : (1ull << shift) / 6);
    if (((1ull << shift) / 3) >> 32) return NH_EARG;
    q.shift = shift;
    if (n) k_quant_i32<<<grid_for(n), 256, 0, as_stream(stream)>>>(d_coeff, n, q, d_level);
    NH_HIP(hipGetLastError());
    return NH_OK;
}
int nh_dequant_batch(const int32_t* d_level, int32_t* d_coeff, int64_t n, int qp, void* stream) {
    if (!d_level || !d_coeff || n < 0) return NH_EARG;
    int per, rem;
    qp_params(qp, &per, &rem);
    if (n) k_dequant_i32<<<grid_for(n), 256, 0, as_stream(stream)>>>(d_level, n, dequant_scale(rem), per, d_coeff);
    NH_HIP(hipGetLastError());
    return NH_OK;
}

// ----- metrics (metrics.py:7-48) -----
int nh_sum_sq_diff(const int64_t* a, const int64_t* b, int64_t n, int64_t* out) {
    if (n < 0) return NH_EARG;
    BlockCall c;
    const size_t oa = c.in(a, n * 8), ob = c.in(b, n * 8);
    return c.run(grid_red(n), [=] __device__(U8 in, ST st, uint8_t*) {
        dev_sum_sq_diff((const int64_t*)(in + oa), (const int64_t*)(in + ob), n, st + 1);
    }, out, 8, true);
}
int nh_sum_sq_diff_f64(const double* a, const double* b, int64_t n, double* out) {
    if (n < 0) return NH_EARG;
    BlockCall c;
    const size_t oa = c.in(a, n * 8), ob = c.in(b, n * 8);
    return c.run<false>(1, [=] __device__(U8 in, ST, uint8_t* o) {   // 1.5 KB of stack: k_small
        dev_sum_sq_diff_f64((const double*)(in + oa), (const double*)(in + ob), n, (double*)o);
    }, out, 8);
}
int nh_sad(const int32_t* a, const int32_t* b, int64_t n, int64_t* out) {
    if (n < 0) return NH_EARG;
    BlockCall c;
    const size_t oa = c.in(a, n * 4), ob = c.in(b, n * 4);
    return c.run(grid_red(n), [=] __device__(U8 in, ST st, uint8_t*) {
        dev_sad_i32((const int32_t*)(in + oa), (const int32_t*)(in + ob), n, st + 1);
    }, out, 8, true);
}
int nh_satd_4x4(const int32_t* a, const int32_t* b, int64_t* out) {
    BlockCall c;
    const size_t oa = c.in(a, 64), ob = c.in(b, 64);
    return c.run(1, [=] __device__(U8 in, ST, uint8_t* o) {
        dev_satd_4x4((const int32_t*)(in + oa), (const int32_t*)(in + ob), (long long*)o);
    }, out, 8);
}
int nh_residual_energy(const int64_t* r, int64_t n, int64_t* out) {
    if (n < 0) return NH_EARG;
    BlockCall c;
    const size_t oa = c.in(r, n * 8);
    return c.run(grid_red(n), [=] __device__(U8 in, ST st, uint8_t*) {
        dev_residual_energy((const int64_t*)(in + oa), n, st + 1);
    }, out, 8, true);
}
int nh_sse_i16(const int16_t* d_a, const int16_t* d_b, int64_t n, int64_t* d_out, void* stream) {
    if (!d_a || !d_b || !d_out || n < 0) return NH_EARG;
    if (n) k_sse_i16<<<grid_red(n), 256, 0, as_stream(stream)>>>(d_a, d_b, n, (unsigned long long*)d_out);
    NH_HIP(hipGetLastError());
    return NH_OK;
}

}  // extern "C"


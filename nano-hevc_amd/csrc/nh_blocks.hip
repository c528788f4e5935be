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
#include <climits>
#include <cstdio>
#include <cstring>
#include <string>
#include "nh_common.hpp"
#include "nh_internal.hpp"

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
// staging context
// ---------------------------------------------------------------------------
Staging& staging() {
    static Staging s;
    return s;
}

int staging_reserve(Staging& s, size_t bytes) {
    int dev = 0, n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
        set_error("no HIP device visible (nano-hevc_amd needs an MI355X; there is no CPU fallback)");
        return NH_ENODEV;
    }
    NH_HIP(hipGetDevice(&dev));
    if (s.device != dev) {  // (re)initialise on the caller's current device
        s.device = dev;
        s.stream = nullptr;
        s.dbuf = s.hbuf = nullptr;
        s.cap = 0;
        s.dstatus = nullptr;
        NH_HIP(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking));
        NH_HIP(hipMalloc(&s.dstatus, 64));
    }
    if (bytes > s.cap) {
        size_t c = align_up(bytes < (1u << 20) ? (1u << 20) : bytes * 2, 4096);
        if (s.dbuf) { (void)hipFree(s.dbuf); s.dbuf = nullptr; }
        if (s.hbuf) { (void)hipHostFree(s.hbuf); s.hbuf = nullptr; }
        NH_HIP(hipMalloc(&s.dbuf, c));
        NH_HIP(hipHostMalloc(&s.hbuf, c, hipHostMallocDefault));
        s.cap = c;
    }
    unsigned long long init = ULLONG_MAX;
    NH_HIP(hipMemcpyAsync(s.dstatus, &init, sizeof(init), hipMemcpyHostToDevice, s.stream));
    return NH_OK;
}

int staging_upload(Staging& s, size_t off, const void* src, size_t bytes) {
    if (!bytes) return NH_OK;
    std::memcpy((char*)s.hbuf + off, src, bytes);
    NH_HIP(hipMemcpyAsync((char*)s.dbuf + off, (char*)s.hbuf + off, bytes, hipMemcpyHostToDevice, s.stream));
    return NH_OK;
}

int staging_download(Staging& s, void* dst, size_t off, size_t bytes) {
    (void)dst;
    if (!bytes) return NH_OK;
    NH_HIP(hipMemcpyAsync((char*)s.hbuf + off, (char*)s.dbuf + off, bytes, hipMemcpyDeviceToHost, s.stream));
    return NH_OK;
}

int staging_finish(Staging& s, int* status_out) {
    unsigned long long st = 0;
    NH_HIP(hipGetLastError());
    NH_HIP(hipMemcpyAsync(&st, s.dstatus, sizeof(st), hipMemcpyDeviceToHost, s.stream));
    NH_HIP(hipStreamSynchronize(s.stream));
    *status_out = (st == ULLONG_MAX) ? NH_OK : -(int)(st & 0xff);
    return NH_OK;
}

// Staging layout helper: sequential 256-B aligned regions.
struct Layout {
    size_t off = 0;
    size_t take(size_t bytes) { size_t o = off; off = align_up(off + bytes, 256); return o; }
};

// ---------------------------------------------------------------------------
// intra prediction kernels (per-block form)
// ---------------------------------------------------------------------------

// intra.py:37-62.  One workgroup: int64 sum over the whole arrays (D7), then fill.
__global__ void __launch_bounds__(256) k_intra_dc(const int64_t* top, int64_t nt, const int64_t* left,
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

// intra.py:81-113: Python-int arithmetic, int16 store (D9), IndexError on short refs.
__global__ void k_intra_planar(const int64_t* top, int64_t nt, const int64_t* left, int64_t nl,
                               int64_t tr, int64_t bl, int64_t size, int64_t log2size, int16_t* out,
                               unsigned long long* st) {
    const int64_t n = size * size;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        int64_t y = i / size, x = i - y * size;
        if (y >= nl || x >= nt) { report(st, i, NH_EINDEX); continue; }
        int64_t h = (size - 1 - x) * left[y] + (x + 1) * tr;
        int64_t v = (size - 1 - y) * top[x] + (y + 1) * bl;
        int64_t p = (h + v + size) >> (log2size + 1);
        if (p < -32768 || p > 32767) { report(st, i, NH_EOVERFLOW); continue; }
        out[i] = (int16_t)p;
    }
}

// intra.py:116-207.  Thread 0 builds the int16 reference array in LDS in the
// reference's order (so the first error raised is the reference's), then the
// workgroup projects every sample with int16 arithmetic (D8).
constexpr int kMaxAngSize = 2048;  // 3N+1 int16 in LDS (12 KB)
__global__ void __launch_bounds__(256) k_intra_angular(const int64_t* top, int64_t nt, const int64_t* left,
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
__global__ void k_residual(const int16_t* a, const int16_t* b, int64_t n, int16_t* out, int add) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint32_t x = (uint16_t)a[i], y = (uint16_t)b[i];
        out[i] = (int16_t)(uint16_t)(add ? x + y : x - y);
    }
}
__global__ void k_clip(const int64_t* x, int64_t n, int64_t maxval, int16_t* out) {
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
template <int N, bool DST, bool FWD>
__global__ void __launch_bounds__(256) k_transform(const int32_t* __restrict__ in, int32_t* __restrict__ out,
                                                   int64_t nblocks) {
    constexpr int BPW = 256 / N;  // blocks per workgroup
    constexpr int P = N + 1;
    constexpr int S = Log2<N>::v + 5;  // transform.py:173 (D1: same shift both passes)
    __shared__ int32_t tile[BPW][N][P];
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
__global__ void k_quant_i64(const int64_t* c, int64_t n, uint64_t mf, uint64_t off, int shift, int abs_bits,
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
__global__ void k_dequant_i64(const int64_t* l, int64_t n, int64_t scale, int per, int32_t* out) {
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
__global__ void k_count_nonzero(const int64_t* l, int64_t n, unsigned long long* cnt) {
    unsigned long long c = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        c += l[i] != 0;
    for (int o = 32; o > 0; o >>= 1) c += __shfl_down(c, o, 64);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(cnt, c);
}

// quant.py:153-168: sum(log2(|l|+1) + (|l|>0)*2) in float64, then int().
// np.sum of a contiguous float64 array is numpy's pairwise_sum over the
// flattened array (blocks of 8 accumulators, halves above 128 elements);
// replicated serially here so the float64 rounding sequence is numpy's.
// term for one level held in a `bits`-wide signed dtype (32 or 64): np.abs and
// the +1 wrap inside that dtype; log2 of a non-positive value gives -inf/NaN
// exactly as numpy does (the shim's int() then raises like the reference).
__device__ double eb_term(int64_t v, int bits) {
    uint64_t a = v < 0 ? 0ull - (uint64_t)v : (uint64_t)v;
    uint64_t a1 = a + 1;
    int64_t as, as1;
    if (bits == 32) { as = (int32_t)(uint32_t)a; as1 = (int32_t)(uint32_t)a1; }
    else { as = (int64_t)a; as1 = (int64_t)a1; }
    return log2((double)as1) + (double)((as > 0) * 2);
}
__device__ double pw_sum(const int64_t* a, int64_t n, int bits) {
    // iterative form of numpy's pairwise_sum over eb_term(a[i])
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
                for (int64_t i = 0; i < f.n; ++i) res += eb_term(a[f.off + i], bits);
            } else {
                double r[8];
                for (int j = 0; j < 8; ++j) r[j] = eb_term(a[f.off + j], bits);
                int64_t i;
                for (i = 8; i < f.n - (f.n % 8); i += 8)
                    for (int j = 0; j < 8; ++j) r[j] += eb_term(a[f.off + i + j], bits);
                res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
                for (; i < f.n; ++i) res += eb_term(a[f.off + i], bits);
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
__global__ void k_estimate_bits(const int64_t* l, int64_t n, int bits, double* out) {
    if (threadIdx.x || blockIdx.x) return;
    *out = n > 0 ? pw_sum(l, n, bits) : 0.0;   // the shim applies int() (quant.py:168)
}

// ---------------------------------------------------------------------------
// quality metrics (metrics.py:7-48) as device reductions
// ---------------------------------------------------------------------------
// Workgroup reduction (256 threads) then ONE atomic per workgroup: an atomic
// per wave on one word serialises (~90 adds/us per address).
template <class T, class F>
__device__ __forceinline__ void block_reduce_add(T v, unsigned long long* out, F) {
    __shared__ unsigned long long part[4];
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
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
__global__ void k_sum_sq_diff(const int64_t* a, const int64_t* b, int64_t n, unsigned long long* out) {
    unsigned long long s = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        int64_t d = a[i] - b[i];
        s += (unsigned long long)(d * d);
    }
    block_reduce_add(s, out, NoOp{});
}
// metrics.py:24-26: int32 difference (wraps), np.abs (wraps at INT32_MIN), int64 sum
__global__ void k_sad_i32(const int32_t* a, const int32_t* b, int64_t n, unsigned long long* out) {
    unsigned long long s = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        int32_t d = (int32_t)((uint32_t)a[i] - (uint32_t)b[i]);
        int32_t ad = d == INT32_MIN ? d : (d < 0 ? -d : d);
        s += (unsigned long long)(long long)ad;
    }
    block_reduce_add(s, out, NoOp{});
}
// metrics.py:29-43: H . diff . H^T in int32 (wrap), sum |.| in int64
__global__ void k_satd_4x4(const int32_t* a, const int32_t* b, long long* out) {
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
__global__ void k_residual_energy(const int64_t* r, int64_t n, unsigned long long* out) {
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

#define NH_STAGE_BEGIN(bytes)                         \
    Staging& S = staging();                           \
    std::lock_guard<std::mutex> lk_(S.mu);            \
    {                                                 \
        int rc_ = staging_reserve(S, (bytes));        \
        if (rc_) return rc_;                          \
    }
#define NH_TRY(x)              \
    do {                       \
        int rc__ = (x);        \
        if (rc__) return rc__; \
    } while (0)

static int finish_copy(Staging& S, void* dst, size_t off, size_t bytes) {
    NH_TRY(staging_download(S, dst, off, bytes));
    int st = 0;
    NH_TRY(staging_finish(S, &st));
    if (st) return st;
    if (bytes) std::memcpy(dst, (char*)S.hbuf + off, bytes);
    return NH_OK;
}

int nh_intra_dc(const int64_t* top, int64_t ntop, const int64_t* left, int64_t nleft, int64_t size,
                int variant4x4, int16_t* out) {
    if (ntop < 0 || nleft < 0) return NH_EARG;
    if (!variant4x4 && size == 0) return NH_EZERODIV;
    if (!variant4x4 && size < 0) return NH_EARG;
    const int64_t nout = variant4x4 ? 16 : size * size;
    Layout L;
    size_t ot = L.take(ntop * 8), ol = L.take(nleft * 8), oo = L.take(nout * 2);
    NH_STAGE_BEGIN(L.off);
    NH_TRY(staging_upload(S, ot, top, ntop * 8));
    NH_TRY(staging_upload(S, ol, left, nleft * 8));
    char* d = (char*)S.dbuf;
    k_intra_dc<<<1, 256, 0, S.stream>>>((int64_t*)(d + ot), ntop, (int64_t*)(d + ol), nleft, size, variant4x4,
                                        (int16_t*)(d + oo), (unsigned long long*)S.dstatus);
    return finish_copy(S, out, oo, nout * 2);
}

int nh_intra_planar(const int64_t* top, int64_t ntop, const int64_t* left, int64_t nleft, int64_t top_right,
                    int64_t bottom_left, int64_t size, int64_t log2size, int16_t* out) {
    if (ntop < 0 || nleft < 0 || size < 0) return NH_EARG;
    const int64_t nout = size * size;
    if (nout == 0) return NH_OK;
    Layout L;
    size_t ot = L.take(ntop * 8), ol = L.take(nleft * 8), oo = L.take(nout * 2);
    NH_STAGE_BEGIN(L.off);
    NH_TRY(staging_upload(S, ot, top, ntop * 8));
    NH_TRY(staging_upload(S, ol, left, nleft * 8));
    char* d = (char*)S.dbuf;
    k_intra_planar<<<grid_for(nout), 256, 0, S.stream>>>((int64_t*)(d + ot), ntop, (int64_t*)(d + ol), nleft,
                                                         top_right, bottom_left, size, log2size,
                                                         (int16_t*)(d + oo), (unsigned long long*)S.dstatus);
    return finish_copy(S, out, oo, nout * 2);
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
    Layout L;
    size_t ot = L.take(ntop * 8), ol = L.take(nleft * 8), oo = L.take(nout * 2 + 2);
    NH_STAGE_BEGIN(L.off);
    NH_TRY(staging_upload(S, ot, top, ntop * 8));
    NH_TRY(staging_upload(S, ol, left, nleft * 8));
    char* d = (char*)S.dbuf;
    k_intra_angular<<<1, 256, 0, S.stream>>>((int64_t*)(d + ot), ntop, (int64_t*)(d + ol), nleft, corner, angle,
                                             vert, size, (int16_t*)(d + oo), (unsigned long long*)S.dstatus);
    return finish_copy(S, out, oo, nout * 2);
}

static int elementwise16(const int16_t* a, const int16_t* b, int64_t n, int16_t* out, int add) {
    if (n < 0) return NH_EARG;
    if (n == 0) return NH_OK;
    Layout L;
    size_t oa = L.take(n * 2), ob = L.take(n * 2), oo = L.take(n * 2);
    NH_STAGE_BEGIN(L.off);
    NH_TRY(staging_upload(S, oa, a, n * 2));
    NH_TRY(staging_upload(S, ob, b, n * 2));
    char* d = (char*)S.dbuf;
    k_residual<<<grid_for(n), 256, 0, S.stream>>>((int16_t*)(d + oa), (int16_t*)(d + ob), n, (int16_t*)(d + oo), add);
    return finish_copy(S, out, oo, n * 2);
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
    Layout L;
    size_t ox = L.take(n * 8), oo = L.take(n * 2);
    NH_STAGE_BEGIN(L.off);
    NH_TRY(staging_upload(S, ox, x, n * 8));
    char* d = (char*)S.dbuf;
    k_clip<<<grid_for(n), 256, 0, S.stream>>>((int64_t*)(d + ox), n, maxval, (int16_t*)(d + oo));
    return finish_copy(S, out, oo, n * 2);
}

static int block_transform(const int32_t* in, int64_t size, int use_dst, int32_t* out, bool fwd) {
    if (size != 4 && size != 8 && size != 16 && size != 32) return NH_EVALUE;  // transform.py:150-151
    const int64_t n = size * size;
    Layout L;
    size_t oi = L.take(n * 4), oo = L.take(n * 4);
    NH_STAGE_BEGIN(L.off);
    NH_TRY(staging_upload(S, oi, in, n * 4));
    char* d = (char*)S.dbuf;
    int rc = fwd ? launch_transform<true>((int32_t*)(d + oi), (int32_t*)(d + oo), 1, (int)size, use_dst, S.stream)
                 : launch_transform<false>((int32_t*)(d + oi), (int32_t*)(d + oo), 1, (int)size, use_dst, S.stream);
    if (rc) return rc;
    return finish_copy(S, out, oo, n * 4);
}
int nh_forward_transform(const int32_t* in, int64_t size, int use_dst, int32_t* out) {
    return block_transform(in, size, use_dst, out, true);
}
int nh_inverse_transform(const int32_t* in, int64_t size, int use_dst, int32_t* out) {
    return block_transform(in, size, use_dst, out, false);
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
    Layout L;
    size_t oi = L.take(n * 8), oo = L.take(n * 4);
    NH_STAGE_BEGIN(L.off);
    NH_TRY(staging_upload(S, oi, coeff, n * 8));
    char* d = (char*)S.dbuf;
    k_quant_i64<<<grid_for(n), 256, 0, S.stream>>>((int64_t*)(d + oi), n, (uint64_t)quant_scale(rem), off,
                                                   (int)shift, abs_bits, (int32_t*)(d + oo));
    return finish_copy(S, out, oo, n * 4);
}

int nh_dequantize(const int64_t* level, int64_t n, int qp, int32_t* out) {
    if (n < 0) return NH_EARG;
    if (n == 0) return NH_OK;
    int per, rem;
    qp_params(qp, &per, &rem);
    Layout L;
    size_t oi = L.take(n * 8), oo = L.take(n * 4);
    NH_STAGE_BEGIN(L.off);
    NH_TRY(staging_upload(S, oi, level, n * 8));
    char* d = (char*)S.dbuf;
    k_dequant_i64<<<grid_for(n), 256, 0, S.stream>>>((int64_t*)(d + oi), n, dequant_scale(rem), per,
                                                     (int32_t*)(d + oo));
    return finish_copy(S, out, oo, n * 4);
}

int nh_count_nonzero(const int64_t* level, int64_t n, int64_t* count) {
    if (n < 0) return NH_EARG;
    Layout L;
    size_t oi = L.take(n * 8 + 8), oc = L.take(8);
    NH_STAGE_BEGIN(L.off);
    NH_TRY(staging_upload(S, oi, level, n * 8));
    char* d = (char*)S.dbuf;
    NH_HIP(hipMemsetAsync(d + oc, 0, 8, S.stream));
    if (n) k_count_nonzero<<<grid_red(n), 256, 0, S.stream>>>((int64_t*)(d + oi), n, (unsigned long long*)(d + oc));
    return finish_copy(S, count, oc, 8);
}

int nh_estimate_bits(const int64_t* level, int64_t n, int abs_bits, double* bits) {
    if (n < 0 || (abs_bits != 32 && abs_bits != 64)) return NH_EARG;
    Layout L;
    size_t oi = L.take(n * 8 + 8), oc = L.take(8);
    NH_STAGE_BEGIN(L.off);
    NH_TRY(staging_upload(S, oi, level, n * 8));
    char* d = (char*)S.dbuf;
    k_estimate_bits<<<1, 64, 0, S.stream>>>((int64_t*)(d + oi), n, abs_bits, (double*)(d + oc));
    return finish_copy(S, bits, oc, 8);
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
static int reduce_call(const void* a, size_t abytes, const void* b, size_t bbytes, int64_t* out, int which, int64_t n) {
    Layout L;
    size_t oa = L.take(abytes + 8), ob = L.take(bbytes + 8), oc = L.take(8);
    NH_STAGE_BEGIN(L.off);
    NH_TRY(staging_upload(S, oa, a, abytes));
    if (b) NH_TRY(staging_upload(S, ob, b, bbytes));
    char* d = (char*)S.dbuf;
    NH_HIP(hipMemsetAsync(d + oc, 0, 8, S.stream));
    unsigned long long* o = (unsigned long long*)(d + oc);
    if (which == 0 && n) k_sum_sq_diff<<<grid_red(n), 256, 0, S.stream>>>((int64_t*)(d + oa), (int64_t*)(d + ob), n, o);
    if (which == 1 && n) k_sad_i32<<<grid_red(n), 256, 0, S.stream>>>((int32_t*)(d + oa), (int32_t*)(d + ob), n, o);
    if (which == 2) k_satd_4x4<<<1, 64, 0, S.stream>>>((int32_t*)(d + oa), (int32_t*)(d + ob), (long long*)o);
    if (which == 3 && n) k_residual_energy<<<grid_red(n), 256, 0, S.stream>>>((int64_t*)(d + oa), n, o);
    return finish_copy(S, out, oc, 8);
}
int nh_sum_sq_diff(const int64_t* a, const int64_t* b, int64_t n, int64_t* out) {
    if (n < 0) return NH_EARG;
    return reduce_call(a, n * 8, b, n * 8, out, 0, n);
}
int nh_sad(const int32_t* a, const int32_t* b, int64_t n, int64_t* out) {
    if (n < 0) return NH_EARG;
    return reduce_call(a, n * 4, b, n * 4, out, 1, n);
}
int nh_satd_4x4(const int32_t* a, const int32_t* b, int64_t* out) { return reduce_call(a, 64, b, 64, out, 2, 16); }
int nh_residual_energy(const int64_t* r, int64_t n, int64_t* out) {
    if (n < 0) return NH_EARG;
    return reduce_call(r, n * 8, nullptr, 0, out, 3, n);
}
int nh_sse_i16(const int16_t* d_a, const int16_t* d_b, int64_t n, int64_t* d_out, void* stream) {
    if (!d_a || !d_b || !d_out || n < 0) return NH_EARG;
    if (n) k_sse_i16<<<grid_red(n), 256, 0, as_stream(stream)>>>(d_a, d_b, n, (unsigned long long*)d_out);
    NH_HIP(hipGetLastError());
    return NH_OK;
}

}  // extern "C"


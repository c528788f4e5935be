/*
 * nh_oracle.c -- scalar CPU restatement of the reference hot path.
 *
 * TEST INFRASTRUCTURE (see nh_oracle.h): the checker for the HIP kernels and
 * the "port" CPU baseline of bench.py.  Never linked by the product.
 *
 * Every function follows the reference file:line it cites, including the
 * reference's deviations from H.265:
 *   - transforms: int32 ring arithmetic (numpy int32 scalars wrap), the same
 *     shift log2N+5 in both passes, column pass first (transform.py:173-194);
 *   - angular: int16 interpolation arithmetic (NEP 50 weak Python ints,
 *     intra.py:207), (i+1) projection in the reference extension
 *     (intra.py:180-186), replicate-last fill (intra.py:174-178);
 *   - quant: shift 14+qp/6+log2N, abs in the input dtype (quant.py:70-79).
 * Pinned against the tests/golden npz fixtures (reference outputs) by
 * tests/test_oracle_golden.py.
 */
#include "nh_oracle.h"
#include <pthread.h>
#include <string.h>
#include <stdlib.h>

enum { NH_OK = 0, NH_EVALUE = -1, NH_EINDEX = -2, NH_EOVERFLOW = -3, NH_EZERODIV = -4 };

/* transform.py:20-135 (spec tables 8-8 / 8-9).  DCT32 even rows are DCT16 etc.;
 * only the 32-point table and DST4 are stored, the rest are sub-sampled rows. */
static const int32_t DST4[4][4] = {
    {29, 55, 74, 84}, {74, 74, 0, -74}, {84, -29, -74, 55}, {55, -84, 74, -29}};
/* DCT32 (transform.py:65-135) is generated from its 33 distinct magnitudes:
 * DCT32[k][n] = +-tab[fold((2n+1)k mod 128)], tab[m] ~ 64*sqrt(2)*cos(m*pi/64)
 * with the spec's integer adjustments.  DCT4/8/16 are its even-row
 * sub-samplings.  Pinned by tests/golden matrices.npz. */
static int32_t g_dct32[32][32];
static int g_dct_init = 0;

static void dct_init(void) {
    static const int32_t tab[33] = {64, 90, 90, 90, 89, 88, 87, 85, 83, 82, 80, 78, 75, 73, 70, 67,
                                    64, 61, 57, 54, 50, 46, 43, 38, 36, 31, 25, 22, 18, 13, 9, 4, 0};
    for (int k = 0; k < 32; ++k) {
        for (int n = 0; n < 32; ++n) {
            if (k == 0) { g_dct32[k][n] = 64; continue; }
            int m = ((2 * n + 1) * k) % 128; /* angle in units of pi/64 */
            int32_t v;
            if (m <= 32) v = tab[m];
            else if (m <= 64) v = -tab[64 - m];
            else if (m <= 96) v = -tab[m - 64];
            else v = tab[128 - m];
            g_dct32[k][n] = v;
        }
    }
    g_dct_init = 1;
}

/* transform.py:138-151 */
static int tmat(int64_t size, int use_dst, int32_t* T) {
    if (!g_dct_init) dct_init();
    if (use_dst && size == 4) { memcpy(T, DST4, sizeof(DST4)); return NH_OK; }
    int step;
    if (size == 4) step = 8; else if (size == 8) step = 4; else if (size == 16) step = 2;
    else if (size == 32) step = 1; else return NH_EVALUE;
    /* DCT_N[k][n] = DCT32[k*step][n] for n < N (even rows of DCT(2N) = DCT(N)). */
    for (int k = 0; k < size; ++k)
        for (int n = 0; n < size; ++n) T[k * size + n] = g_dct32[k * step][n];
    return NH_OK;
}

int oh_get_matrix(int64_t size, int use_dst, int32_t* T) { return tmat(size, use_dst, T); }

static int log2i(int64_t n) { int l = 0; while ((1LL << (l + 1)) <= n) ++l; return l; }

/* transform.py:154-196 */
int oh_forward_transform(const int32_t* in, int64_t size, int use_dst, int32_t* out) {
    int32_t T[32 * 32];
    int rc = tmat(size, use_dst, T);
    if (rc) return rc;
    const int N = (int)size;
    const int shift = log2i(N) + 5;
    const uint32_t rnd = 1u << (shift - 1);
    int32_t tmp[32 * 32];
    for (int i = 0; i < N; ++i)          /* transform.py:179-185: temp = T.X */
        for (int j = 0; j < N; ++j) {
            uint32_t acc = 0;
            for (int k = 0; k < N; ++k) acc += (uint32_t)T[i * N + k] * (uint32_t)in[k * N + j];
            tmp[i * N + j] = ((int32_t)(acc + rnd)) >> shift;
        }
    for (int i = 0; i < N; ++i)          /* transform.py:188-194: coeff = temp.T^T */
        for (int j = 0; j < N; ++j) {
            uint32_t acc = 0;
            for (int k = 0; k < N; ++k) acc += (uint32_t)tmp[i * N + k] * (uint32_t)T[j * N + k];
            out[i * N + j] = ((int32_t)(acc + rnd)) >> shift;
        }
    return NH_OK;
}

/* transform.py:199-238 */
int oh_inverse_transform(const int32_t* in, int64_t size, int use_dst, int32_t* out) {
    int32_t T[32 * 32];
    int rc = tmat(size, use_dst, T);
    if (rc) return rc;
    const int N = (int)size;
    const int shift = log2i(N) + 5;
    const uint32_t rnd = 1u << (shift - 1);
    int32_t tmp[32 * 32];
    for (int i = 0; i < N; ++i)          /* transform.py:221-227: temp = T^T.C */
        for (int j = 0; j < N; ++j) {
            uint32_t acc = 0;
            for (int k = 0; k < N; ++k) acc += (uint32_t)T[k * N + i] * (uint32_t)in[k * N + j];
            tmp[i * N + j] = ((int32_t)(acc + rnd)) >> shift;
        }
    for (int i = 0; i < N; ++i)          /* transform.py:230-236: res = temp.T */
        for (int j = 0; j < N; ++j) {
            uint32_t acc = 0;
            for (int k = 0; k < N; ++k) acc += (uint32_t)tmp[i * N + k] * (uint32_t)T[k * N + j];
            out[i * N + j] = ((int32_t)(acc + rnd)) >> shift;
        }
    return NH_OK;
}

/* Python floor division / arithmetic shift on int64 */
static int64_t floordiv(int64_t a, int64_t b) {
    int64_t q = a / b, r = a % b;
    if (r != 0 && ((r < 0) != (b < 0))) --q;
    return q;
}
static int fits16(int64_t v) { return v >= -32768 && v <= 32767; }

/* intra.py:37-62 */
int oh_intra_dc(const int64_t* top, int64_t ntop, const int64_t* left, int64_t nleft,
                int64_t size, int variant4x4, int16_t* out) {
    int64_t s = 0;
    for (int64_t i = 0; i < ntop; ++i) s += top[i];   /* int(top.sum()) : whole array (D7) */
    for (int64_t i = 0; i < nleft; ++i) s += left[i];
    int64_t dc;
    if (variant4x4) { dc = (s + 4) >> 3; size = 4; }   /* intra.py:42 */
    else {
        if (size == 0) return NH_EZERODIV;
        dc = floordiv(s + size, 2 * size);               /* intra.py:61 */
    }
    if (!fits16(dc)) return NH_EOVERFLOW;                /* np.full int16 (D9) */
    for (int64_t i = 0; i < size * size; ++i) out[i] = (int16_t)dc;
    return NH_OK;
}

/* intra.py:81-113 (Python-int arithmetic, int16 store) */
int oh_intra_planar(const int64_t* top, int64_t ntop, const int64_t* left, int64_t nleft,
                    int64_t tr, int64_t bl, int64_t size, int64_t log2size, int16_t* out) {
    for (int64_t y = 0; y < size; ++y)
        for (int64_t x = 0; x < size; ++x) {
            if (y >= nleft || x >= ntop) return NH_EINDEX;
            int64_t h = (size - 1 - x) * left[y] + (x + 1) * tr;
            int64_t v = (size - 1 - y) * top[x] + (y + 1) * bl;
            int64_t p = (h + v + size) >> (log2size + 1);
            if (!fits16(p)) return NH_EOVERFLOW;
            out[y * size + x] = (int16_t)p;
        }
    return NH_OK;
}

/* intra.py:24-29 */
static const int ANGLE[33] = {32, 26, 21, 17, 13, 9, 5, 2, 0, -2, -5, -9, -13, -17, -21, -26, -32,
                              -26, -21, -17, -13, -9, -5, -2, 0, 2, 5, 9, 13, 17, 21, 26, 32};
int oh_mode_to_angle(int mode, int* angle, int* is_vertical) {
    int idx = mode - 2;                  /* INTRA_PRED_ANGLE[mode - 2], Python list (D10) */
    if (idx < -33 || idx > 32) return NH_EINDEX;
    if (idx < 0) idx += 33;
    *angle = ANGLE[idx];
    *is_vertical = mode >= 18;
    return NH_OK;
}
/* intra.py:31-34 */
static int inv_angle(int a) {
    switch (a) {
        case -2: return -4096; case -5: return -1638; case -9: return -910; case -13: return -630;
        case -17: return -482; case -21: return -390; case -26: return -315; case -32: return -256;
    }
    return 0;
}

/* intra.py:116-207 */
int oh_intra_angular(const int64_t* top, int64_t ntop, const int64_t* left, int64_t nleft,
                     int64_t corner, int angle, int is_vertical, int64_t size, int16_t* out) {
    const int64_t* pri = is_vertical ? top : left;    /* intra.py:145-153 */
    const int64_t* sec = is_vertical ? left : top;
    int64_t npri = is_vertical ? ntop : nleft, nsec = is_vertical ? nleft : ntop;
    const int64_t N = size;
    int16_t* ref = (int16_t*)calloc((size_t)(3 * N + 1), sizeof(int16_t));
    if (!ref) return NH_EVALUE;
    int rc = NH_OK;
    /* _build_ref_array intra.py:159-188 */
    if (!fits16(corner)) { rc = NH_EOVERFLOW; goto done; }
    ref[N] = (int16_t)corner;
    for (int64_t i = 1; i <= 2 * N; ++i) {
        int64_t v;
        if (i < npri) v = pri[i];
        else { if (npri == 0) { rc = NH_EINDEX; goto done; } v = pri[npri - 1]; }
        if (!fits16(v)) { rc = NH_EOVERFLOW; goto done; }
        ref[N + i] = (int16_t)v;
    }
    if (angle < 0) {
        int inv = inv_angle(angle);
        int64_t next = (N * angle) >> 5;
        for (int64_t i = -1; i > next - 1; --i) {
            int64_t proj = ((i + 1) * inv + 128) >> 8;   /* (i+1): D5 */
            if (proj < nsec) {
                int64_t v = sec[proj];
                if (!fits16(v)) { rc = NH_EOVERFLOW; goto done; }
                ref[N + i] = (int16_t)v;
            }
        }
    }
    /* _project_sample_at intra.py:191-207, int16 arithmetic (D8) */
    for (int64_t y = 0; y < N; ++y)
        for (int64_t x = 0; x < N; ++x) {
            int64_t base = is_vertical ? x : y, scan = is_vertical ? y : x;
            int64_t proj = (scan + 1) * angle;
            int64_t ip = proj >> 5, f = proj & 31;
            int64_t idx = N + base + 1 + ip;
            int16_t p;
            if (f == 0) p = ref[idx];
            else {
                int32_t s = (int32_t)((32 - f) * ref[idx] + f * ref[idx + 1] + 16);
                p = (int16_t)(((int16_t)(uint16_t)(uint32_t)s) >> 5);
            }
            out[y * N + x] = p;
        }
done:
    free(ref);
    return rc;
}

/* intra.py:65-67, 70-72 (int16 wrap) and 75-78 */
void oh_residual(const int16_t* a, const int16_t* b, int64_t n, int16_t* out) {
    for (int64_t i = 0; i < n; ++i) out[i] = (int16_t)(uint16_t)((uint32_t)(uint16_t)a[i] - (uint32_t)(uint16_t)b[i]);
}
void oh_reconstruct(const int16_t* a, const int16_t* b, int64_t n, int16_t* out) {
    for (int64_t i = 0; i < n; ++i) out[i] = (int16_t)(uint16_t)((uint32_t)(uint16_t)a[i] + (uint32_t)(uint16_t)b[i]);
}
void oh_clip(const int64_t* x, int64_t n, int64_t maxval, int16_t* out) {
    for (int64_t i = 0; i < n; ++i) {
        int64_t v = x[i] < 0 ? 0 : (x[i] > maxval ? maxval : x[i]);
        out[i] = (int16_t)(uint16_t)(uint64_t)v;
    }
}

/* quant.py:21-38 */
static const int32_t QS[6] = {26214, 23302, 20560, 18396, 16384, 14564};
static const int32_t DQS[6] = {40, 45, 51, 57, 64, 72};
static void qp_params(int qp, int* per, int* rem) {
    if (qp < 0) qp = 0;
    if (qp > 51) qp = 51;
    *per = qp / 6; *rem = qp % 6;
}

/* quant.py:41-79 */
int oh_quantize(const int64_t* c, int64_t n, int qp, int64_t log2size, int is_intra,
                int abs_bits, int32_t* out) {
    int per, rem;
    qp_params(qp, &per, &rem);
    const int64_t mf = QS[rem];
    const int64_t shift = 14 + per + log2size;
    if (shift < 0 || shift > 62) return NH_EOVERFLOW;
    const int64_t off = is_intra ? (1LL << shift) / 3 : (1LL << shift) / 6;
    for (int64_t i = 0; i < n; ++i) {
        int64_t x = c[i];
        int64_t a;
        if (abs_bits < 64 && x == -(1LL << (abs_bits - 1))) a = x;   /* np.abs wraps at dtype min */
        else a = (int64_t)((x < 0) ? (uint64_t)0 - (uint64_t)x : (uint64_t)x);
        int64_t lvl = (int64_t)((uint64_t)a * (uint64_t)mf + (uint64_t)off) >> shift;
        int64_t sg = (x > 0) - (x < 0);
        out[i] = (int32_t)(uint32_t)(uint64_t)(sg * lvl);
    }
    return NH_OK;
}

/* quant.py:82-123 */
int oh_dequantize(const int64_t* l, int64_t n, int qp, int32_t* out) {
    int per, rem;
    qp_params(qp, &per, &rem);
    const int64_t sc = DQS[rem];
    for (int64_t i = 0; i < n; ++i) {
        uint64_t b = (uint64_t)l[i] * (uint64_t)sc;
        int64_t v;
        if (per < 4) {
            int sh = 4 - per;
            v = (int64_t)(b + (1ull << (sh - 1))) >> sh;
        } else v = (int64_t)(b << (per - 4));
        out[i] = (int32_t)(uint32_t)(uint64_t)v;
    }
    return NH_OK;
}

/* ------------------------------------------------------------------ */
/* frame-level drivers                                                 */
/* ------------------------------------------------------------------ */

/* cfg 2.  transform.py:154-196 + quant.py:126-137 per full 8x8 block; block
 * walk of block.py:68-74 (partial edge blocks skipped). */
void oh_fwd8x8_quant_plane(const int16_t* res, int16_t* lvl, int w, int h, int pitch,
                           int qp, int is_intra) {
    int32_t blk[64], coef[64], q[64];
    int64_t c64[64];
    for (int by = 0; by + 8 <= h; by += 8)
        for (int bx = 0; bx + 8 <= w; bx += 8) {
            for (int i = 0; i < 8; ++i)
                for (int j = 0; j < 8; ++j) blk[i * 8 + j] = res[(int64_t)(by + i) * pitch + bx + j];
            oh_forward_transform(blk, 8, 0, coef);
            for (int k = 0; k < 64; ++k) c64[k] = coef[k];
            oh_quantize(c64, 64, qp, 3, is_intra, 32, q);
            for (int i = 0; i < 8; ++i)
                for (int j = 0; j < 8; ++j) lvl[(int64_t)(by + i) * pitch + bx + j] = (int16_t)q[i * 8 + j];
        }
}

/* Same walk split over nthreads POSIX threads by block row (SURVEY.md §8(d)
 * D-4: the all-cores CPU baseline).  Block rows are independent (D12), so the
 * output equals oh_fwd8x8_quant_plane's. */
typedef struct {
    const int16_t* res; int16_t* lvl; int w, h, pitch, qp, is_intra, row0, row1;
} oh_band;

static void* oh_band_run(void* p) {
    const oh_band* b = (const oh_band*)p;
    oh_fwd8x8_quant_plane(b->res + (int64_t)b->row0 * 8 * b->pitch, b->lvl + (int64_t)b->row0 * 8 * b->pitch,
                          b->w, (b->row1 - b->row0) * 8, b->pitch, b->qp, b->is_intra);
    return NULL;
}

int oh_fwd8x8_quant_plane_mt(const int16_t* res, int16_t* lvl, int w, int h, int pitch,
                             int qp, int is_intra, int nthreads) {
    enum { kMaxThreads = 256 };
    if (nthreads < 1) nthreads = 1;
    if (nthreads > kMaxThreads) nthreads = kMaxThreads;
    int rows = h / 8;
    if (nthreads > rows) nthreads = rows > 0 ? rows : 1;
    if (!g_dct_init) dct_init();   /* lazy table init stays single-threaded */
    pthread_t tid[kMaxThreads];
    oh_band band[kMaxThreads];
    int spawned[kMaxThreads];
    for (int t = 0; t < nthreads; ++t) {
        oh_band b = {res, lvl, w, h, pitch, qp, is_intra, rows * t / nthreads, rows * (t + 1) / nthreads};
        band[t] = b;
        /* the last band runs on the caller; a failed spawn runs inline too */
        spawned[t] = t < nthreads - 1 && pthread_create(&tid[t], NULL, oh_band_run, &band[t]) == 0;
        if (!spawned[t]) oh_band_run(&band[t]);
    }
    for (int t = 0; t < nthreads; ++t)
        if (spawned[t]) pthread_join(tid[t], NULL);
    return 0;
}

/* block.py:38-55 neighbour rules, source plane (open loop, D12). */
static void get_top(const int16_t* src, int w, int pitch, int x, int y, int count,
                    int64_t* out, int64_t* n) {
    if (y == 0) { for (int i = 0; i < count; ++i) out[i] = 128; *n = count; return; }
    int m = count; if (x + m > w) m = w - x;   /* numpy slice truncation at the right edge */
    for (int i = 0; i < m; ++i) out[i] = src[(int64_t)(y - 1) * pitch + x + i];
    *n = m;
}
static void get_left(const int16_t* src, int h, int pitch, int x, int y, int count,
                     int64_t* out, int64_t* n) {
    if (x == 0) { for (int i = 0; i < count; ++i) out[i] = 128; *n = count; return; }
    int m = count; if (y + m > h) m = h - y;
    for (int i = 0; i < m; ++i) out[i] = src[(int64_t)(y + i) * pitch + x - 1];
    *n = m;
}

/* One TU of the reconstruction chain (README.md:55-71 chain, intra.py/transform.py/quant.py).
 * Returns SSE(orig, recon) (metrics.py:46-48 on residual_block(orig, recon)). */
static int64_t tu_chain(const int16_t* orig, const int16_t* pred, int N, int use_dst, int qp,
                        int32_t* lvl_out, int16_t* rec_out) {
    int32_t r[1024], c[1024], l[1024], d[1024], rr[1024];
    int64_t t[1024];
    int16_t r16[1024];
    int lg = log2i(N);
    oh_residual(orig, pred, N * N, r16);
    for (int i = 0; i < N * N; ++i) r[i] = r16[i];
    oh_forward_transform(r, N, use_dst, c);
    for (int i = 0; i < N * N; ++i) t[i] = c[i];
    oh_quantize(t, N * N, qp, lg, 1, 32, l);
    for (int i = 0; i < N * N; ++i) t[i] = l[i];
    oh_dequantize(t, N * N, qp, d);
    oh_inverse_transform(d, N, use_dst, rr);
    int64_t sse = 0;
    for (int i = 0; i < N * N; ++i) {
        int16_t rr16 = (int16_t)(uint16_t)(uint32_t)rr[i];          /* .astype(np.int16) */
        int16_t rc = (int16_t)(uint16_t)((uint32_t)(uint16_t)pred[i] + (uint32_t)(uint16_t)rr16);
        int64_t cv = rc < 0 ? 0 : (rc > 255 ? 255 : rc);             /* clip_to_pixel_range(.,8) */
        int16_t d16 = (int16_t)(uint16_t)((uint32_t)(uint16_t)orig[i] - (uint32_t)cv);
        sse += (int64_t)d16 * d16;
        if (rec_out) rec_out[i] = (int16_t)cv;
        if (lvl_out) lvl_out[i] = l[i];
    }
    return sse;
}

/* cfg 3: 35-mode RDO per full 8x8 block.  Open loop: the
 * neighbours come from the source plane (D12).  Closed loop:
 * blocks in raster order, neighbours from the reconstruction built so far
 * (zero-initialised like Frame.zeros, frame.py:81-88) with the BlockView rules
 * (block.py:38-55), the left reference limited to the N reconstructed samples
 * (get_left_neighbors(N)); intra.py's short-reference rule (D6) extends it. */
static void intra_rdo_plane(const int16_t* src, int w, int h, int pitch, int qp, int closed,
                            uint8_t* modes, int32_t* lvl, int16_t* recon, int64_t* sse_total) {
    const int N = 8;
    int16_t orig[64], pred[64], best_rec[64];
    int32_t best_lvl[64], l[64];
    int16_t rec[64];
    int64_t topN[8], leftN[8], top2[17], left2[17];
    int64_t nt, nl, nt2, nl2;
    int64_t total = 0;
    int bw = w / 8;
    const int16_t* nb = closed ? recon : src;   /* the plane neighbours are read from */
    if (closed)
        for (int y = 0; y < h; ++y)
            for (int x = 0; x < w; ++x) recon[(int64_t)y * pitch + x] = 0;
    for (int by = 0; by + N <= h; by += N)
        for (int bx = 0; bx + N <= w; bx += N) {
            for (int i = 0; i < N; ++i)
                for (int j = 0; j < N; ++j) orig[i * N + j] = src[(int64_t)(by + i) * pitch + bx + j];
            get_top(nb, w, pitch, bx, by, N, topN, &nt);
            get_left(nb, h, pitch, bx, by, N, leftN, &nl);
            int64_t tl = (by == 0 || bx == 0) ? 128 : nb[(int64_t)(by - 1) * pitch + bx - 1];
            top2[0] = tl; left2[0] = tl;
            get_top(nb, w, pitch, bx, by, 2 * N, top2 + 1, &nt2);
            get_left(nb, h, pitch, bx, by, closed ? N : 2 * N, left2 + 1, &nl2);
            int64_t best = -1; int bm = 0;
            for (int m = 0; m < 35; ++m) {
                if (m == 0) oh_intra_planar(topN, nt, leftN, nl, topN[nt - 1], leftN[nl - 1], N, 3, pred);
                else if (m == 1) oh_intra_dc(topN, nt, leftN, nl, N, 0, pred);
                else {
                    int a, v;
                    oh_mode_to_angle(m, &a, &v);
                    oh_intra_angular(top2, nt2 + 1, left2, nl2 + 1, tl, a, v, N, pred);
                }
                int64_t sse = tu_chain(orig, pred, N, 0, qp, l, rec);
                if (best < 0 || sse < best) {
                    best = sse; bm = m;
                    memcpy(best_rec, rec, sizeof(rec));
                    memcpy(best_lvl, l, sizeof(l));
                }
            }
            total += best;
            modes[(by / N) * bw + bx / N] = (uint8_t)bm;
            for (int i = 0; i < N; ++i)
                for (int j = 0; j < N; ++j) {
                    lvl[(int64_t)(by + i) * pitch + bx + j] = best_lvl[i * N + j];
                    recon[(int64_t)(by + i) * pitch + bx + j] = best_rec[i * N + j];
                }
        }
    if (sse_total) *sse_total = total;
}

void oh_intra_rdo_plane(const int16_t* src, int w, int h, int pitch, int qp,
                        uint8_t* modes, int32_t* lvl, int16_t* recon, int64_t* sse_total) {
    intra_rdo_plane(src, w, h, pitch, qp, 0, modes, lvl, recon, sse_total);
}

void oh_intra_rdo_plane_closed(const int16_t* src, int w, int h, int pitch, int qp,
                               uint8_t* modes, int32_t* lvl, int16_t* recon, int64_t* sse_total) {
    intra_rdo_plane(src, w, h, pitch, qp, 1, modes, lvl, recon, sse_total);
}

/* cfg 4 TU split decision: a seeded integer hash. */
static uint32_t mix32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}
int oh_tu_split(uint32_t seed, int plane_id, int x, int y, int size) {
    uint32_t k = mix32(seed ^ (0x9E3779B9U * (uint32_t)(plane_id + 1)));
    k = mix32(k ^ (uint32_t)x);
    k = mix32(k ^ ((uint32_t)y * 0x85ebca6bU));
    k = mix32(k ^ (uint32_t)size);
    return (k & 3u) < 2u;
}

/* nb: the plane the TU's neighbours are read from -- the source (open loop,
 * D12) or the reconstruction built so far (closed loop). */
static void tu_one(const int16_t* src, const int16_t* nb, int w, int h, int pitch, int x, int y, int N,
                   int qp, int is_luma, int32_t* lvl, int16_t* recon, uint8_t* tu_log2) {
    int16_t orig[1024], dc[1024], pl[1024], r16[1024];
    int32_t l[1024];
    int16_t rec[1024];
    int64_t top[32], left[32], nt, nl;
    for (int i = 0; i < N; ++i)
        for (int j = 0; j < N; ++j) orig[i * N + j] = src[(int64_t)(y + i) * pitch + x + j];
    get_top(nb, w, pitch, x, y, N, top, &nt);
    get_left(nb, h, pitch, x, y, N, left, &nl);
    /* __main__.py:165-178: DC vs planar by residual energy, DC wins ties */
    oh_intra_dc(top, nt, left, nl, N, 0, dc);
    oh_intra_planar(top, nt, left, nl, top[nt - 1], left[nl - 1], N, log2i(N), pl);
    int64_t edc = 0, epl = 0;
    oh_residual(orig, dc, N * N, r16);
    for (int i = 0; i < N * N; ++i) edc += (int64_t)r16[i] * r16[i];
    oh_residual(orig, pl, N * N, r16);
    for (int i = 0; i < N * N; ++i) epl += (int64_t)r16[i] * r16[i];
    const int16_t* pred = (edc <= epl) ? dc : pl;
    tu_chain(orig, pred, N, is_luma && N == 4, qp, l, rec);
    int lg = log2i(N);
    for (int i = 0; i < N; ++i)
        for (int j = 0; j < N; ++j) {
            lvl[(int64_t)(y + i) * pitch + x + j] = l[i * N + j];
            recon[(int64_t)(y + i) * pitch + x + j] = rec[i * N + j];
        }
    int w4 = w / 4;
    for (int i = 0; i < N / 4; ++i)
        for (int j = 0; j < N / 4; ++j) tu_log2[(int64_t)(y / 4 + i) * w4 + x / 4 + j] = (uint8_t)lg;
}

static void tu_tree(const int16_t* src, const int16_t* nb, int w, int h, int pitch, int x, int y, int s,
                    int plane_id, uint32_t seed, int qp, int is_luma,
                    int32_t* lvl, int16_t* recon, uint8_t* tu_log2) {
    if (x >= w || y >= h) return;
    int overhang = (x + s > w) || (y + s > h);
    if (s > 4 && (overhang || oh_tu_split(seed, plane_id, x, y, s))) {
        int hs = s / 2;   /* z-order: top-left, top-right, bottom-left, bottom-right */
        tu_tree(src, nb, w, h, pitch, x, y, hs, plane_id, seed, qp, is_luma, lvl, recon, tu_log2);
        tu_tree(src, nb, w, h, pitch, x + hs, y, hs, plane_id, seed, qp, is_luma, lvl, recon, tu_log2);
        tu_tree(src, nb, w, h, pitch, x, y + hs, hs, plane_id, seed, qp, is_luma, lvl, recon, tu_log2);
        tu_tree(src, nb, w, h, pitch, x + hs, y + hs, hs, plane_id, seed, qp, is_luma, lvl, recon, tu_log2);
        return;
    }
    if (overhang) return;
    tu_one(src, nb, w, h, pitch, x, y, s, qp, is_luma, lvl, recon, tu_log2);
}

void oh_tu_pipeline_plane(const int16_t* src, int w, int h, int pitch, int ctb,
                          int plane_id, uint32_t seed, int qp, int is_luma,
                          int row0, int row1, int32_t* lvl, int16_t* recon, uint8_t* tu_log2) {
    int rows = (h + ctb - 1) / ctb;
    if (row1 > rows) row1 = rows;
    for (int cy = row0; cy < row1; ++cy)
        for (int cx = 0; cx * ctb < w; ++cx)
            tu_tree(src, src, w, h, pitch, cx * ctb, cy * ctb, ctb, plane_id, seed, qp, is_luma,
                    lvl, recon, tu_log2);
}

/* Same walk split over nthreads POSIX threads by CTU row (SURVEY.md §8(d) D-4,
 * the all-cores leg of config 4's CPU baseline).  Open loop: a CTU row reads
 * only source samples (D12), so the rows are independent and the output equals
 * oh_tu_pipeline_plane's. */
typedef struct {
    const int16_t* src; int w, h, pitch, ctb, plane_id; uint32_t seed; int qp, is_luma, row0, row1;
    int32_t* lvl; int16_t* recon; uint8_t* tu_log2;
} oh_tu_band;

static void* oh_tu_band_run(void* p) {
    const oh_tu_band* b = (const oh_tu_band*)p;
    oh_tu_pipeline_plane(b->src, b->w, b->h, b->pitch, b->ctb, b->plane_id, b->seed, b->qp, b->is_luma, b->row0,
                         b->row1, b->lvl, b->recon, b->tu_log2);
    return NULL;
}

int oh_tu_pipeline_plane_mt(const int16_t* src, int w, int h, int pitch, int ctb, int plane_id, uint32_t seed,
                            int qp, int is_luma, int row0, int row1, int32_t* lvl, int16_t* recon,
                            uint8_t* tu_log2, int nthreads) {
    enum { kMaxThreads = 256 };
    int rows = (h + ctb - 1) / ctb;
    if (row1 > rows) row1 = rows;
    if (row0 < 0) row0 = 0;
    if (row1 <= row0) return 0;
    if (nthreads < 1) nthreads = 1;
    if (nthreads > kMaxThreads) nthreads = kMaxThreads;
    if (nthreads > row1 - row0) nthreads = row1 - row0;
    if (!g_dct_init) dct_init();   /* lazy table init stays single-threaded */
    pthread_t tid[kMaxThreads];
    oh_tu_band band[kMaxThreads];
    int spawned[kMaxThreads];
    const int n = row1 - row0;
    for (int t = 0; t < nthreads; ++t) {
        oh_tu_band b = {src, w, h, pitch, ctb, plane_id, seed, qp, is_luma, row0 + n * t / nthreads,
                        row0 + n * (t + 1) / nthreads, lvl, recon, tu_log2};
        band[t] = b;
        spawned[t] = t < nthreads - 1 && pthread_create(&tid[t], NULL, oh_tu_band_run, &band[t]) == 0;
        if (!spawned[t]) oh_tu_band_run(&band[t]);
    }
    for (int t = 0; t < nthreads; ++t)
        if (spawned[t]) pthread_join(tid[t], NULL);
    return 0;
}

/* cfg 4 in closed loop: CTUs in raster order, TUs in z-order,
 * neighbours from the reconstruction built so far (zero-initialised,
 * frame.py:41-43) with the BlockView rules (block.py:38-50). */
void oh_tu_pipeline_plane_closed(const int16_t* src, int w, int h, int pitch, int ctb,
                                 int plane_id, uint32_t seed, int qp, int is_luma,
                                 int32_t* lvl, int16_t* recon, uint8_t* tu_log2) {
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) recon[(int64_t)y * pitch + x] = 0;
    for (int cy = 0; cy * ctb < h; ++cy)
        for (int cx = 0; cx * ctb < w; ++cx)
            tu_tree(src, recon, w, h, pitch, cx * ctb, cy * ctb, ctb, plane_id, seed, qp, is_luma,
                    lvl, recon, tu_log2);
}

/* cfg 5: every full 32x32 block of a plane (block.py:68-74
 * raster walk, partial blocks skipped) through the cfg-4 TU chain at N=32. */
void oh_tc32_plane(const int16_t* src, int w, int h, int pitch, int qp, int32_t* lvl, int16_t* recon) {
    int w4 = w / 4;
    uint8_t* tmap = (uint8_t*)calloc((size_t)(h / 4 + 1) * (w4 + 1), 1);
    for (int by = 0; by + 32 <= h; by += 32)
        for (int bx = 0; bx + 32 <= w; bx += 32) tu_one(src, src, w, h, pitch, bx, by, 32, qp, 1, lvl, recon, tmap);
    free(tmap);
}

/* Frame-level intra driver, one plane (__main__.py:142-189 encode_frame_intra;
 * the demo's per-block loop __main__.py:75-100 is the same decision on luma).
 * Blocks in raster order (block.py:68-74; partial blocks skipped, their
 * samples stay 0 in the zero-initialised recon, frame.py:81-88).  Per block:
 * top/left from the SOURCE plane with 128 at the frame border (block.py:38-50),
 * DC (intra.py:46-62) and planar with tr=top[-1], bl=left[-1]
 * (__main__.py:165-168, intra.py:81-113); energies = residual_energy of
 * residual_block (metrics.py:46-48, intra.py:65-67: int16 wrap); DC wins ties
 * (__main__.py:171); recon = clip_to_pixel_range(best) (intra.py:75-78).
 * stats[6] += {blocks, dc wins, planar wins, sum dc energy, sum planar energy,
 *             SSE of (uint8)src vs (uint8)recon over the whole plane}. */
void oh_encode_intra_plane(const int16_t* src, int w, int h, int pitch, int N, int16_t* recon,
                           int64_t* stats) {
    int l2 = 0;
    while ((2 << l2) <= N) ++l2;                       /* int(np.log2(size)) */
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) recon[(int64_t)y * pitch + x] = 0;
    /* any block size N >= 1 (__main__.py:156-158 takes any block_size) */
    int64_t* top = (int64_t*)malloc(sizeof(int64_t) * (size_t)(N > 0 ? N : 1));
    int64_t* left = (int64_t*)malloc(sizeof(int64_t) * (size_t)(N > 0 ? N : 1));
    for (int by = 0; N > 0 && by + N <= h; by += N)
        for (int bx = 0; bx + N <= w; bx += N) {
            int64_t nt, nl, sum = 0;
            get_top(src, w, pitch, bx, by, N, top, &nt);
            get_left(src, h, pitch, bx, by, N, left, &nl);
            for (int i = 0; i < N; ++i) sum += top[i] + left[i];
            const int64_t dc = floordiv(sum + N, 2 * N);
            const int64_t tr = top[N - 1], bl = left[N - 1];
            int64_t edc = 0, epl = 0;
            for (int i = 0; i < N; ++i)
                for (int j = 0; j < N; ++j) {
                    const int64_t o = src[(int64_t)(by + i) * pitch + bx + j];
                    const int64_t pl = ((N - 1 - j) * left[i] + (j + 1) * tr + (N - 1 - i) * top[j] +
                                        (i + 1) * bl + N) >> (l2 + 1);
                    const int64_t rd = (int16_t)(uint16_t)(o - (int16_t)dc);
                    const int64_t rp = (int16_t)(uint16_t)(o - (int16_t)pl);
                    edc += rd * rd;
                    epl += rp * rp;
                }
            const int use_dc = edc <= epl;
            for (int i = 0; i < N; ++i)
                for (int j = 0; j < N; ++j) {
                    int64_t p = use_dc ? dc : ((N - 1 - j) * left[i] + (j + 1) * tr + (N - 1 - i) * top[j] +
                                               (i + 1) * bl + N) >> (l2 + 1);
                    p = (int16_t)p;                         /* the predictor's int16 store */
                    recon[(int64_t)(by + i) * pitch + bx + j] = (int16_t)(p < 0 ? 0 : p > 255 ? 255 : p);
                }
            stats[0] += 1;
            stats[1] += use_dc;
            stats[2] += !use_dc;
            stats[3] += edc;
            stats[4] += epl;
        }
    free(top);
    free(left);
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
            const int64_t d = (int64_t)(uint8_t)src[(int64_t)y * pitch + x] -
                              (int64_t)(uint8_t)recon[(int64_t)y * pitch + x];
            stats[5] += d * d;
        }
}

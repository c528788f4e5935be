/*
 * nanohevc.h -- C ABI of the MI355X-native HEVC intra-block hot path.
 *
 * The reference (Luodian/nano-hevc) is pure Python + numpy and has no FFI; its
 * drop-in boundary is the set of Python functions re-exported by
 * nano_hevc/__init__.py:50-91.  This header is what a binding of that boundary
 * calls (ctypes shim: nano-hevc_amd/nano_hevc/_lib.py).
 *
 * Two groups of entry points:
 *   (i)  per-block, host pointers, synchronous -- one reference call each
 *        (inputs already converted by the shim exactly as the reference
 *        converts them: .astype(np.int32) for transforms, int64 for sums);
 *   (ii) batched, device pointers, asynchronous on a caller hipStream_t
 *        (passed as void*; NULL = the null stream) -- the frame-level path.
 * No entry point allocates caller-visible memory; no C++ exception crosses the
 * ABI.  Every function returns NH_OK (0) or a negative NH_E* code; the shim
 * maps codes to the exception the reference raises in the same situation.
 */
#ifndef NANOHEVC_H
#define NANOHEVC_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NH_OK 0
#define NH_EVALUE (-1)    /* ValueError("Unsupported transform size: N") transform.py:150-151 */
#define NH_EINDEX (-2)    /* IndexError (mode >= 35, short refs) intra.py:142, :177 */
#define NH_EOVERFLOW (-3) /* OverflowError: int16 store out of range (numpy 2) intra.py:62,111,173 */
#define NH_EZERODIV (-4)  /* ZeroDivisionError: intra_dc_predict size 0, intra.py:61 */
#define NH_EARG (-5)      /* bad argument (null pointer, misaligned plane, negative count) */
#define NH_ETYPE (-6)     /* TypeError: planar's float h + v (float corner, or int64 + uint64 corners) >> int, intra.py:111 */
#define NH_ENODEV (-10)   /* no HIP device visible */
#define NH_EHIP (-11)     /* HIP runtime error (message: nh_last_error()) */

/* ---------------- library / device ---------------- */
const char* nh_version(void);
const char* nh_last_error(void);
int nh_device_count(int* count);
/* Per-device contexts of the per-block (host-pointer) entry points: bytes held
 * on `device` (0 before its first per-block call), and release of every
 * context (the next per-block call re-creates the current device's). */
int nh_staging_bytes(int device, int64_t* bytes);
int nh_release_staging(void);
/* Host-side phases of the calling thread's last per-block call, in ns:
 * [0] marshal (inputs into the kernel-argument block or the staging buffer),
 * [1] launch (the launch API calls), [2] wait (launch returned -> completion
 * seen), [3] finish (outputs copied back).  Diagnostics (tools/percall.py). */
int nh_last_call_times(int64_t* ns);
/* The block-call server: while per-block calls keep coming,
 * one resident workgroup per device takes them from mapped host memory instead
 * of a kernel launch per call; it leaves after the idle time (default 200 us)
 * without a call.  set_idle_us: that time for servers launched from now on
 * (0 = never start one: every call is its own launch; 0 also stops the resident
 * ones).  stop: ask every resident server to leave now and wait for it.
 * stats (device): [0] calls served, [1] server launches, [2] calls run as their
 * own kernel (k_small / staged), [3] the idle time in us.  Runtime control, no
 * reference counterpart. */
int nh_block_server_set_idle_us(int64_t us);
int nh_block_server_stop(void);
int nh_block_server_stats(int device, int64_t* out);

/* ---------------- (i) per-block entry points (host pointers) ---------------- */

/* intra.py:37-43 intra_dc_predict_4x4 (variant4x4=1, size ignored) and
 * intra.py:46-62 intra_dc_predict: dc over the WHOLE top/left arrays (D7). out: size*size */
int nh_intra_dc(const int64_t* top, int64_t ntop, const int64_t* left, int64_t nleft,
                int64_t size, int variant4x4, int16_t* out);
/* intra.py:81-113 intra_planar_predict; log2size = int(np.log2(size)).
 * tr_kind / bl_kind: the corner argument's scalar kind, which decides numpy 2's
 * (NEP 50) arithmetic at intra.py:109-111: NH_NP_PYINT = a Python int (exact
 * math); NH_NP_FLOAT = a float (value ignored: h and v become floats and the >>
 * raises, NH_ETYPE); 8/16/32/64 = numpy uintN (value passed as its bits), -8..-64 = numpy
 * intN (np.bool_ = -64).  Python-int operands are converted to the corner's
 * dtype (NH_EOVERFLOW out of range), results wrap in it, int64 with uint64
 * promotes to float64 (NH_ETYPE at the >>); the first error in the reference's
 * loop order is returned. */
#define NH_NP_PYINT 0
#define NH_NP_FLOAT 1
int nh_intra_planar(const int64_t* top, int64_t ntop, const int64_t* left, int64_t nleft,
                    int64_t top_right, int tr_kind, int64_t bottom_left, int bl_kind,
                    int64_t size, int64_t log2size, int16_t* out);
/* intra.py:116-207 intra_angular_predict (+ _build_ref_array, _project_sample_at);
 * mode uses Python list indexing into INTRA_PRED_ANGLE (D10) */
int nh_intra_angular(const int64_t* top, int64_t ntop, const int64_t* left, int64_t nleft,
                     int64_t corner, int mode, int64_t size, int16_t* out);
/* intra.py:65-67 residual_block / :70-72 reconstruct_block on int16 (wrap) */
int nh_residual(const int16_t* orig, const int16_t* pred, int64_t n, int16_t* out);
int nh_reconstruct(const int16_t* pred, const int16_t* res, int64_t n, int16_t* out);
/* intra.py:75-78 clip_to_pixel_range: clamp to [0, maxval] then wrap to int16 */
int nh_clip(const int64_t* x, int64_t n, int64_t maxval, int16_t* out);
/* transform.py:154-196 forward_transform / :199-238 inverse_transform on an
 * int32 size x size block (row-major) */
int nh_forward_transform(const int32_t* in, int64_t size, int use_dst, int32_t* out);
int nh_inverse_transform(const int32_t* in, int64_t size, int use_dst, int32_t* out);
/* quant.py:41-79 quantize: abs_bits = bit width in which np.abs wraps (8/16/32/64) */
int nh_quantize(const int64_t* coeff, int64_t n, int qp, int64_t log2size, int is_intra,
                int abs_bits, int32_t* out);
/* quant.py:77-78 for FLOAT coefficients: out = (abs_coeff * MF + offset) >> shift
 * in int64 (wrapping), abs_coeff = np.abs(coeff).astype(np.int64) from the
 * shim, which then applies quant.py:79's (np.sign(coeff) * level).astype(np.int32). */
int nh_quantize_abs(const int64_t* abs_coeff, int64_t n, int qp, int64_t log2size, int is_intra,
                    int64_t* out);
/* quant.py:82-123 dequantize (size unused, D4) */
int nh_dequantize(const int64_t* level, int64_t n, int qp, int32_t* out);
/* quant.py:171-173 count_nonzero */
int nh_count_nonzero(const int64_t* level, int64_t n, int64_t* count);
/* quant.py:153-168 estimate_bits: the float64 sum (numpy pairwise order, over
 * the n words in the order given) of log2(|l|+1) + 2*(|l|>0) under numpy's
 * dtype rules for levels of dtype abs_bits (an NH_EB_* code): |l| and the +1
 * in that dtype (integers wrap, floats round), log2 in float16 (8-bit
 * integers, float16), float32 (16-bit integers, float32) or float64.  Each
 * 8-byte word holds the level as an int64, a uint64 bit pattern (unsigned
 * codes) or a float64 bit pattern (float codes).  The caller applies int()
 * (which raises on NaN/inf exactly as the reference). */
#define NH_EB_BOOL 1
#define NH_EB_I8 8
#define NH_EB_I16 16
#define NH_EB_I32 32
#define NH_EB_I64 64
#define NH_EB_U8 108
#define NH_EB_U16 116
#define NH_EB_U32 132
#define NH_EB_U64 164
#define NH_EB_F16 216
#define NH_EB_F32 232
#define NH_EB_F64 264
int nh_estimate_bits(const int64_t* level, int64_t n, int abs_bits, double* bits);

/* metrics.py:7-48 as device reductions.
 * nh_sum_sq_diff: exact int64 sum((a-b)^2) (mse = sum / n; psnr from mse);
 * nh_sad: int32 difference/abs (wrapping like the int32 arrays of metrics.py:26);
 * nh_satd_4x4: H.diff.H^T in int32, sum |.| (metrics.py:29-43), 16 samples;
 * nh_residual_energy: sum(int64(r)^2) mod 2^64 (metrics.py:46-48). */
int nh_sum_sq_diff(const int64_t* a, const int64_t* b, int64_t n, int64_t* out);
/* metrics.py:9-10 for samples of any dtype (float, wide ints): the float64 sum
 * of (a-b)^2 over a, b already cast to float64 by the shim, in numpy's pairwise
 * summation order (np.mean = this / n) -- bit-identical to the reference's. */
int nh_sum_sq_diff_f64(const double* a, const double* b, int64_t n, double* out);
int nh_sad(const int32_t* a, const int32_t* b, int64_t n, int64_t* out);
int nh_satd_4x4(const int32_t* a, const int32_t* b, int64_t* out);
int nh_residual_energy(const int64_t* r, int64_t n, int64_t* out);

/* ---------------- (ii) batched device entry points ---------------- */

/* SSE between two int16 device buffers, added into *d_out (one int64): frame
 * PSNR / RDO distortion without a host round trip. */
int nh_sse_i16(const int16_t* d_a, const int16_t* d_b, int64_t n, int64_t* d_out, void* stream);

/* A set of equally shaped raster planes inside one buffer (e.g. the Y planes,
 * or the U+V planes, of a stream of YUV420 frames).  Offsets/pitches are in
 * elements.  Plane p = g*planes_per_group + c lives at
 *   base + g*group_stride + c*plane_stride.
 * Only full 8x8 blocks are processed (block.py:68-74 skips partial blocks). */
typedef struct nh_plane_set {
    int64_t base;
    int64_t plane_stride;
    int64_t group_stride;
    int32_t width, height, pitch;
    int32_t planes_per_group;
    int32_t num_groups;
    int32_t reserved;
} nh_plane_set;

#define NH_MAX_PLANE_SETS 8

/* THE HOT PATH (config 2 / north-star metric): forward 8x8 integer DCT
 * (transform.py:154-196) fused with quantize_block (quant.py:126-137) over
 * every full 8x8 block of int16 residual planes.  Levels are written as int16
 * at the block's raster position in d_lvl (same layout as d_res).  Exact for
 * every int16 input: |level| <= 26214 always fits int16 for N=8.
 * Requires base/pitch/strides to be multiples of 8 elements (16-B rows). */
int nh_fwd8x8_quant_planes(const int16_t* d_res, int16_t* d_lvl, const nh_plane_set* sets,
                           int nsets, int qp, int is_intra, void* stream);
/* Same computation, launch variants kept for A/B measurement (identical
 * output): variant = cache policy (0 default, 1 nontemporal loads+stores,
 * 2 nontemporal loads, 3 nontemporal stores) + 4 * occupancy class
 * (0 compiler choice, 1 >= 5 waves/SIMD; 4 for the pipelined form) + 8 *
 * persistent software-pipelined form (next tile's loads under this tile's
 * compute); + 16 vertical block pair; 32..131 stripe forms; 256*k workgroup
 * sizes; 2048+p store policies; 4096 + 16*c + 5: variant 5 with XCD-aware
 * workgroup order, 2^c workgroups per XCD run (c = 15: 1/8 of the grid per
 * XCD -- the default launch, 4341).  Full list in nh_fused8x8.hip. */
int nh_fwd8x8_quant_planes_variant(const int16_t* d_res, int16_t* d_lvl, const nh_plane_set* sets,
                                   int nsets, int qp, int is_intra, int variant, void* stream);
/* The hot path plus the level-side helpers of quant.py:153-178 fused as an
 * epilogue: per full 8x8 block, d_nnz[i] =
 * count_nonzero(levels) (0..64; is_all_zero == (d_nnz[i] == 0)) and d_bits[i] =
 * int(estimate_bits(levels)) (float64 sum in numpy's order, truncated).  Blocks
 * are numbered set by set in the launch's order (plane, block row, block
 * column).  Either output may be NULL; d_lvl as nh_fwd8x8_quant_planes.  The
 * first call with d_bits on a device fills a static 210 KB term table. */
int nh_fwd8x8_quant_planes_ex(const int16_t* d_res, int16_t* d_lvl, const nh_plane_set* sets, int nsets,
                              int qp, int is_intra, uint8_t* d_nnz, int32_t* d_bits, void* stream);
/* Measurement helper (not a product path): copies d_in to d_out over the same
 * blocks with the hot kernel's exact access pattern -- the achievable-bandwidth
 * ceiling for that pattern.  policy: as the variant's cache policy (0..3),
 * + 4 * shape for 2-blocks-per-thread pattern probes (1 horizontal pair, 2
 * lane-interleaved pair, 3 vertical pair; policies 0/1 only). */
int nh_probe_copy8x8_planes(const int16_t* d_in, int16_t* d_out, const nh_plane_set* sets, int nsets,
                            int policy, void* stream);
/* Measurement helper: plain linear 16-B-per-lane streaming copy of nelems
 * (multiple of 8) int16 (grid <= 0: one chunk per thread, else grid-stride). */
int nh_probe_copy_linear(const int16_t* d_in, int16_t* d_out, int64_t nelems, int policy, int grid,
                         void* stream);

/* nblocks contiguous size x size int32 blocks (row-major) */
int nh_fwd_transform_batch(const int32_t* d_in, int32_t* d_out, int64_t nblocks, int size,
                           int use_dst, void* stream);
int nh_inv_transform_batch(const int32_t* d_in, int32_t* d_out, int64_t nblocks, int size,
                           int use_dst, void* stream);
/* elementwise over n int32 values (abs wraps at 32 bits, as for int32 input) */
int nh_quant_batch(const int32_t* d_coeff, int32_t* d_level, int64_t n, int qp, int log2size,
                   int is_intra, void* stream);
int nh_dequant_batch(const int32_t* d_level, int32_t* d_coeff, int64_t n, int qp, void* stream);

/* Config 3: 35-mode open-loop RDO over every full 8x8 block of an int16
 * source plane: per block and mode, the README chain
 * pred -> residual_block -> forward_transform -> quantize_block ->
 * dequantize_block -> inverse_transform -> reconstruct_block ->
 * clip_to_pixel_range(.,8); cost = SSE(orig, recon), ties -> lowest mode.
 * d_modes: (h/8)*(w/8) u8 (mode 0 planar, 1 DC, 2..34 angular);
 * d_lvl (int32) / d_recon (int16): raster with the given pitch;
 * d_sse (optional, one int64): the chosen SSEs are added to it. */
int nh_intra_rdo_plane(const int16_t* d_src, int w, int h, int pitch, int qp,
                       uint8_t* d_modes, int32_t* d_lvl, int16_t* d_recon, int64_t* d_sse,
                       void* stream);

/* Config 3 over every plane of nsets plane sets in one launch pair per set
 * (frame streams: no launch per plane).  d_modes: the planes' mode maps back
 * to back in set order ((h/8)*(w/8) each); d_sse (optional): one int64 per
 * plane, in the same order, the chosen SSEs added to it; d_lvl / d_recon in the
 * source layout (each plane at its set's offsets, pitch).  Same results as
 * nh_intra_rdo_plane plane by plane. */
int nh_intra_rdo_planes(const int16_t* d_src, const nh_plane_set* sets, int nsets, int qp,
                        uint8_t* d_modes, int32_t* d_lvl, int16_t* d_recon, int64_t* d_sse,
                        void* stream);

/* Config 4: mixed 4/8/16/32 TU pipeline on one plane over CTU rows
 * [row0, row1): seeded quadtree per CTB (ctb 32 luma / 16
 * chroma), per TU the __main__.py:165-178 DC-vs-planar choice then the full
 * reconstruction chain (DST for 4x4 luma).  d_tu: (h/4)*(w/4) u8 log2 TU size;
 * d_work: nh_tu_workspace_bytes(w, h, ctb) bytes of device scratch (currently
 * 0: TUs are found by per-size grid walks; NULL accepted). */
int64_t nh_tu_workspace_bytes(int w, int h, int ctb);
int nh_tu_pipeline_plane(const int16_t* d_src, int w, int h, int pitch, int ctb, int plane_id,
                         uint32_t seed, int qp, int is_luma, int row0, int row1,
                         int32_t* d_lvl, int16_t* d_recon, uint8_t* d_tu, void* d_work,
                         void* stream);
/* The same over every plane of one plane set in one launch per TU size (a
 * stream of frames): plane p = g * planes_per_group + c has plane id
 * plane_id + c (e.g. the U+V set of yuv420 frames: plane_id 1 -> U 1, V 2),
 * d_lvl / d_recon use the source layout, d_tu holds (h/4)*(w/4) entries per
 * plane in plane order. */
int nh_tu_pipeline_planes(const int16_t* d_src, const nh_plane_set* set, int ctb, int plane_id,
                          uint32_t seed, int qp, int is_luma, int row0, int row1, int32_t* d_lvl,
                          int16_t* d_recon, uint8_t* d_tu, void* stream);

/* Config 4 in CLOSED loop over every plane of one plane set:
 * CTUs in raster order, TUs in quadtree z-order, every TU's top / left
 * neighbours from the reconstruction built so far (BlockView rules on a
 * zero-initialised recon).  Device wavefront over CTU rows; d_work: device
 * memory of nh_tu_pipeline_closed_workspace_bytes() bytes, 8-B aligned
 * (zeroed by the call); a wait that cannot complete sets the status word
 * (read it with nh_intra_rdo_closed_status).  Width and height multiples of 4;
 * recon / levels of samples outside every TU are left untouched (callers pass
 * zeroed outputs, as Frame.zeros). */
int64_t nh_tu_pipeline_closed_workspace_bytes(const nh_plane_set* set, int ctb);
int nh_tu_pipeline_planes_closed(const int16_t* d_src, const nh_plane_set* set, int ctb, int plane_id,
                                 uint32_t seed, int qp, int is_luma, int32_t* d_lvl, int16_t* d_recon,
                                 uint8_t* d_tu, void* d_work, void* stream);

/* Config 4 with COMPACT levels: int16 levels in the source layout (exact: an
 * 8-bit TU's level satisfies |level| <= 408 at every QP and size,
 * tools/packed_bounds.py).  Groups of strips with a sample outside [0, 255]
 * (k_ctu_wide's 32-bit chain) write their int32 levels into d_spill (int32,
 * source layout, only those strips touched) and -32768 at each of their strip
 * origins in d_lvl (strips: CTB rows x 1024/CTB columns); nh_tu_levels_widen
 * turns (d_lvl, d_spill) into the int32 levels nh_tu_pipeline_planes writes.
 * CTB 16 or 32; pitch, base and strides multiples of 8; level buffers 16-B
 * aligned. */
int nh_tu_pipeline_planes_compact(const int16_t* d_src, const nh_plane_set* set, int ctb, int plane_id,
                                  uint32_t seed, int qp, int is_luma, int row0, int row1, int16_t* d_lvl,
                                  int32_t* d_spill, int16_t* d_recon, uint8_t* d_tu, void* stream);
int nh_tu_levels_widen(const int16_t* d_lvl, const int32_t* d_spill, const nh_plane_set* set, int ctb, int row0,
                       int row1, int32_t* d_out, void* stream);

/* Config 5: every full 32x32 block of an int16 source plane through the
 * config-4 chain at N=32.  variant 0 = butterfly
 * (k_tu_process<32>), 1 = matrix cores: blocks whose samples and neighbours
 * are 8-bit on f16 MFMA (exact), the others on int8 MFMA
 * (v_mfma_i32_32x32x32_i8 with exact int8 part splitting), 2 = int8 MFMA for
 * every block (A/B).  Identical outputs.  pitch % 8 == 0. */
int nh_tc32_plane(const int16_t* d_src, int w, int h, int pitch, int qp, int32_t* d_lvl,
                  int16_t* d_recon, int variant, void* stream);
/* Config 5 over every plane of up to NH_MAX_PLANE_SETS plane sets (a stream of
 * frames): variant 1 = one f16-MFMA launch + one int8 fix-up launch per set
 * (blockIdx.y = plane), 2 = one int8-MFMA launch per set, 0 = the butterfly,
 * one launch per plane (A/B).  Levels / recon use
 * the source layout.  Same per-plane results as nh_tc32_plane. */
int nh_tc32_planes(const int16_t* d_src, const nh_plane_set* sets, int nsets, int qp, int32_t* d_lvl,
                   int16_t* d_recon, int variant, void* stream);
/* Config 5 with COMPACT levels (variant 1 only): levels of lvl_bytes = 2
 * (int16) or 1 (int8) in the source layout.  Exact: an 8-bit block's 32x32
 * levels satisfy |level| <= 51 at every QP (tools/packed_bounds.py).  A block
 * that is not 8-bit writes its int32 levels into d_spill (int32, source
 * layout, never read) and the marker -32768 / -128 at its compact origin;
 * nh_tc32_levels_widen turns (d_lvl, d_spill) into the int32 levels
 * nh_tc32_planes writes.  int8: base / pitch / strides multiples of 16. */
int nh_tc32_planes_compact(const int16_t* d_src, const nh_plane_set* sets, int nsets, int qp, void* d_lvl,
                           int lvl_bytes, int32_t* d_spill, int16_t* d_recon, void* stream);
int nh_tc32_levels_widen(const void* d_lvl, int lvl_bytes, const int32_t* d_spill, const nh_plane_set* sets,
                         int nsets, int32_t* d_out, void* stream);
/* Measurement / validation helper: D = A.B for row-major int8 32x32 A, B
 * (int32 D) with the lane maps the config-5 MFMA kernel assumes. */
int nh_probe_mfma_i8(const int8_t* d_a, const int8_t* d_b, int32_t* d_d, void* stream);

/* Config 3, CLOSED loop: the same
 * 35-mode chain per full 8x8 block, blocks in raster order, neighbours from
 * the reconstruction built so far (BlockView rules on a zero-initialised
 * recon plane; left reference = the N reconstructed samples, extended by the
 * reference's replicate-last rule).  Scheduled as a wavefront: one wave per
 * block row, rows claimed in order by ticket, each waiting on the row above.
 * Planes of every set are independent.  d_modes: (h/8)*(w/8) per plane,
 * planes numbered set by set (g * planes_per_group + c); d_lvl (int32) and
 * d_recon (int16) use the source layout (recon outside full blocks = 0);
 * d_sse: one int64 per plane, ACCUMULATED.  d_work: caller-owned device
 * memory of nh_intra_rdo_closed_workspace_bytes() bytes (zeroed by the call).
 * A wavefront wait that cannot complete sets the status word instead of
 * hanging: read it with nh_intra_rdo_closed_status (0 = ok). */
int64_t nh_intra_rdo_closed_workspace_bytes(const nh_plane_set* sets, int nsets);
int nh_intra_rdo_planes_closed(const int16_t* d_src, const nh_plane_set* sets, int nsets, int qp,
                               uint8_t* d_modes, int32_t* d_lvl, int16_t* d_recon, int64_t* d_sse,
                               void* d_work, void* stream);
int nh_intra_rdo_closed_status(const void* d_work, int* status, void* stream);

/* ---- Frame I/O and the frame-level intra driver ----
 * Frame.from_yuv420p / Plane.from_buffer + .astype(np.int16) (frame.py:44-54,
 * :87-110) and Frame.to_yuv420p / PackedFrame.to_yuv420p's .astype(np.uint8)
 * (frame.py:112-115, :176-183) as device-to-device element casts over n
 * samples (any frame count: YUV420p frames are contiguous Y, U, V planes). */
int nh_widen_u8_i16(const uint8_t* d_in, int16_t* d_out, int64_t n, void* stream);
/* int16 -> uint8 keeps the low byte (numpy's wrapping astype) */
int nh_narrow_i16_u8(const int16_t* d_in, uint8_t* d_out, int64_t n, void* stream);

/* encode_frame_intra (__main__.py:142-189) over every plane of the given plane
 * sets: per full block_sizes[s] block (raster order, partial blocks skipped:
 * block.py:68-74), DC (intra.py:46-62) vs planar with tr=top[-1], bl=left[-1]
 * (__main__.py:165-168), neighbours from the SOURCE plane with 128 at the
 * border (block.py:38-50), energies = residual_energy(residual_block(..))
 * (metrics.py:46-48, int16 residual wrap), DC wins ties (__main__.py:171),
 * recon = clip_to_pixel_range(best pred) (intra.py:75-78); samples outside
 * full blocks get recon 0 (Frame.zeros, frame.py:81-88).
 * d_src: uint8 (src_is_u8 = 1) or int16 samples.  block_sizes[s] >= 1 (any
 * size, like the reference's driver: 4/8/16/32/64 have their own kernels, other
 * sizes a generic wave-per-block kernel).  d_status (int32, zero it first) is
 * set to 1 when a planar prediction leaves int16 -- the
 * reference raises OverflowError at intra.py:111; possible only for int16
 * samples at a block size that is not a power of two, where d_status is
 * required (NULL otherwise allowed).  d_recon (int16) and d_recon_u8 (the recon's
 * .astype(np.uint8), i.e. to_yuv420p bytes) are optional and use the source
 * layout.  d_stats (NH_ENC_STATS int64 per plane, planes numbered set by set
 * in plane order g * planes_per_group + c) is ACCUMULATED into (zero it first):
 *   blocks, dc wins, planar wins, sum of DC energies, sum of planar energies,
 *   SSE of (uint8)src vs (uint8)recon over the whole plane (metrics.psnr). */
#define NH_ENC_STATS 6
int nh_encode_intra_planes(const void* d_src, int src_is_u8, const nh_plane_set* sets, int nsets,
                           const int32_t* block_sizes, int16_t* d_recon, uint8_t* d_recon_u8,
                           int64_t* d_stats, int32_t* d_status, void* stream);

#ifdef __cplusplus
}
#endif
#endif

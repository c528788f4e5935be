"""Batched, device-resident entry points (the frame-level path).

The reference functions are one block per call; these take whole device
buffers (torch tensors on an MI355X, used only as device memory + stream) and
launch the gfx950 kernels through the C ABI on the tensor's current stream.

  fwd8x8_quant        -- the hot path: fused 8x8 DCT + quant over plane sets
  yuv420_plane_sets   -- nh_plane_set descriptors for a stream of YUV420 frames
  fwd_transform_batch / inv_transform_batch / quant_batch / dequant_batch
  intra_rdo_plane     -- config 3: 35-mode RDO per 8x8 block of a plane; intra_rdo_planes: over plane sets
  intra_rdo_closed    -- config 3 in closed loop (row wavefront); _yuv420_stream: in batches, several in flight
  tu_pipeline_plane   -- config 4: mixed 4..32 TU reconstruction chain on a plane
  tu_pipeline_planes_compact / tu_levels_widen -- config 4 with exact int16 levels (+ int32 spill)
  tc32_plane          -- config 5: 32x32 chain, butterfly or matrix-core variants
  tc32_planes         -- config 5 over a frame stream (one MFMA launch per plane set)
  tc32_planes_compact / tc32_levels_widen -- config 5 with exact int16 / int8 levels (+ int32 spill)
  tu_pipeline_closed  -- config 4 in closed loop (CTU-row wavefront, TUs in z-order)
  tu_pipeline_closed_yuv420 -- the same over a YUV420 stream, luma and chroma wavefronts concurrent
  tu_pipeline_closed_yuv420_stream -- the same in batches of frames, several batches in flight
  widen_u8 / narrow_u8 -- frame I/O casts (YUV420p bytes <-> int16 planes)
  encode_intra_yuv420 -- encode_frame_intra (DC vs planar per block) over a frame stream
  block_server_stop / block_server_set_idle_us / block_server_stats -- the per-block
                        call server: after drop-in per-block calls one
                        workgroup stays resident for its idle time (100 us by default),
                        so a DEVICE-wide synchronize (torch.cuda.synchronize()) right
                        after such calls waits up to that long; block_server_stop()
                        sends it away at once, set_idle_us(0) launches per call instead
"""
from __future__ import annotations

import ctypes as C
from typing import List, Sequence

from . import _lib
from ._lib import PlaneSet, check


def _torch():
    import torch
    return torch


def _stream(stream=None, device=None) -> int:
    """Raw hipStream_t of ``stream``, default: the current stream of ``device``
    (the tensor's device), not of whichever device happens to be current."""
    torch = _torch()
    s = stream if stream is not None else torch.cuda.current_stream(device)
    if device is not None and s.device != device:
        raise ValueError(f"stream on {s.device} but the tensors are on {device}")
    return int(s.cuda_stream)


def _plane_intervals(pset: PlaneSet):
    """[start, end) element range of every plane of a set."""
    span = (pset.height - 1) * pset.pitch + pset.width if pset.height > 0 and pset.width > 0 else 0
    for g in range(pset.num_groups):
        for c in range(pset.planes_per_group):
            b = pset.base + g * pset.group_stride + c * pset.plane_stride
            yield b, b + span


def _set_key(s: PlaneSet):
    return tuple(getattr(s, f) for f, _ in PlaneSet._fields_)


_DISJOINT = {}


def sets_disjoint(a: PlaneSet, b: PlaneSet) -> bool:
    """True when no plane of ``a`` shares an element range with a plane of ``b``
    (memoised: the check walks every plane, ~0.25 ms for 64 frames, and sits before
    the launches of every timed closed-loop call)."""
    key = (_set_key(a), _set_key(b))
    r = _DISJOINT.get(key)
    if r is None:
        if len(_DISJOINT) > 256:
            _DISJOINT.clear()
        r = _DISJOINT[key] = _sets_disjoint(a, b)
    return r


def _sets_disjoint(a: PlaneSet, b: PlaneSet) -> bool:
    iv = sorted([(s, e, 0) for s, e in _plane_intervals(a) if e > s] + [(s, e, 1) for s, e in _plane_intervals(b) if e > s])
    end = {0: -1, 1: -1}
    for s, e, k in iv:
        if s < end[1 - k]:
            return False
        end[k] = max(end[k], e)
    return True


def _need(t, dtype, what):
    torch = _torch()
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise TypeError(f"{what}: expected a CUDA/HIP torch tensor")
    if t.dtype != dtype:
        raise TypeError(f"{what}: expected {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{what}: tensor must be contiguous")


def plane_set(base: int, width: int, height: int, pitch: int | None = None, planes_per_group: int = 1,
              num_groups: int = 1, plane_stride: int = 0, group_stride: int = 0) -> PlaneSet:
    return PlaneSet(base, plane_stride, group_stride, width, height, pitch or width, planes_per_group, num_groups, 0)


def yuv420_frame_elems(width: int, height: int) -> int:
    return width * height + 2 * (width // 2) * (height // 2)


def yuv420_plane_sets(num_frames: int, width: int, height: int, frame_stride: int | None = None,
                      base: int = 0) -> List[PlaneSet]:
    """Descriptors for frames laid out [Y][U][V] back to back (PackedFrame layout):
    one set for the Y planes, one for the U+V planes."""
    fs = frame_stride or yuv420_frame_elems(width, height)
    cw, ch = width // 2, height // 2
    ys = width * height
    return [plane_set(base, width, height, width, 1, num_frames, 0, fs),
            plane_set(base + ys, cw, ch, cw, 2, num_frames, cw * ch, fs)]


def blocks_in(sets: Sequence[PlaneSet]) -> int:
    return sum((s.width // 8) * (s.height // 8) * s.planes_per_group * s.num_groups for s in sets)


DEFAULT_VARIANT = 4341   # nontemporal loads+stores, >= 5 waves/SIMD, XCD-aware order (see nh_fused8x8.hip)
PRODUCT_VARIANTS = (DEFAULT_VARIANT, 5)   # 5: the same without the XCD order; the rest are A/B forms (make ab)


def sets_fit(sets: Sequence[PlaneSet], numel: int, what: str):
    """Host-side bounds check before a launch: every plane of every set must lie
    inside a buffer of ``numel`` elements (a kernel never sees the size)."""
    for s in sets:
        if s.num_groups <= 0 or s.width <= 0 or s.height <= 0:
            continue
        last = s.base + (s.num_groups - 1) * s.group_stride + (s.planes_per_group - 1) * s.plane_stride + \
            (s.height - 1) * s.pitch + s.width
        if s.base < 0 or s.plane_stride < 0 or s.group_stride < 0 or last > numel:
            raise ValueError(f"{what}: a plane set reaches outside the buffer ({last} > {numel} elements)")


def sets_fit_rows(sets: Sequence[PlaneSet], numel: int, row_lo: int, row_hi: int, what: str):
    """Like sets_fit, for a launch that touches only rows [row_lo, row_hi) of each
    plane (a band of CTU rows plus the source row above it): those rows must lie
    inside the buffer; the set's base may then point before it (a band-local
    buffer described as rows of the full plane, shard.Cfg4Layout)."""
    for s in sets:
        lo, hi = max(0, row_lo), min(s.height, row_hi)
        if s.num_groups <= 0 or s.width <= 0 or hi <= lo:
            continue
        if s.plane_stride < 0 or s.group_stride < 0:
            raise ValueError(f"{what}: negative plane strides")
        first = s.base + lo * s.pitch
        last = s.base + (s.num_groups - 1) * s.group_stride + (s.planes_per_group - 1) * s.plane_stride + \
            (hi - 1) * s.pitch + s.width
        if first < 0 or last > numel:
            raise ValueError(f"{what}: rows [{lo}, {hi}) of a plane set reach outside the buffer "
                             f"([{first}, {last}) vs {numel} elements)")


def fwd8x8_quant(res, sets: Sequence[PlaneSet], qp: int = 32, is_intra: bool = True, out=None,
                 variant: int = DEFAULT_VARIANT, stream=None):
    """Forward 8x8 DCT (transform.py:154-196) + quantize_block (quant.py:126-137) on
    every full 8x8 block of the int16 planes described by ``sets`` inside ``res``.
    Levels land at the same raster positions of ``out`` (int16)."""
    torch = _torch()
    _need(res, torch.int16, "fwd8x8_quant(res)")
    if out is None:
        out = torch.zeros_like(res)
    _need(out, torch.int16, "fwd8x8_quant(out)")
    sets_fit(sets, min(res.numel(), out.numel()), "fwd8x8_quant")
    arr = (PlaneSet * len(sets))(*sets)
    L = _lib.load() if int(variant) in PRODUCT_VARIANTS else _lib.load_ab()   # the A/B forms live in the A/B build
    check(L.nh_fwd8x8_quant_planes_variant(res.data_ptr(), out.data_ptr(), arr, len(sets), int(qp),
                                           int(bool(is_intra)), int(variant), C.c_void_p(_stream(stream, res.device))),
          "fwd8x8_quant", L)
    return out


def fwd8x8_quant_ex(res, sets: Sequence[PlaneSet], qp: int = 32, is_intra: bool = True, out=None,
                    nnz: bool = True, bits: bool = True, stream=None):
    """fwd8x8_quant plus the level-side helpers of quant.py:153-178 per block,
    fused.  Returns (levels, nnz, bits): nnz = count_nonzero
    (uint8; is_all_zero == nnz == 0) and bits = int(estimate_bits) (int32) of
    every full 8x8 block, numbered set by set in the launch's order; either may
    be skipped (None)."""
    torch = _torch()
    _need(res, torch.int16, "fwd8x8_quant_ex(res)")
    if out is None:
        out = torch.zeros_like(res)
    _need(out, torch.int16, "fwd8x8_quant_ex(out)")
    sets_fit(sets, min(res.numel(), out.numel()), "fwd8x8_quant_ex")
    nb = blocks_in(sets)
    t_nnz = torch.empty(nb, dtype=torch.uint8, device=res.device) if nnz else None
    t_bits = torch.empty(nb, dtype=torch.int32, device=res.device) if bits else None
    arr = (PlaneSet * len(sets))(*sets)
    check(_lib.load().nh_fwd8x8_quant_planes_ex(
        res.data_ptr(), out.data_ptr(), arr, len(sets), int(qp), int(bool(is_intra)),
        t_nnz.data_ptr() if nnz else None, t_bits.data_ptr() if bits else None, C.c_void_p(_stream(stream, res.device))))
    return out, t_nnz, t_bits


def fwd8x8_quant_plane(res2d, qp: int = 32, is_intra: bool = True, out=None, stream=None):
    """One raster int16 plane (H, W); W must be a multiple of 8 (row pitch = W)."""
    h, w = res2d.shape
    return fwd8x8_quant(res2d, [plane_set(0, w, h, w)], qp, is_intra, out, stream=stream)


def _blocks(x, what):
    torch = _torch()
    _need(x, torch.int32, what)
    if x.dim() != 3 or x.shape[1] != x.shape[2]:
        raise ValueError(f"{what}: expected (B, N, N) int32")
    return x.shape[0], x.shape[1]


def fwd_transform_batch(x, use_dst: bool = False, out=None, stream=None):
    """(B, N, N) int32 -> forward_transform of every block (transform.py:154-196)."""
    b, n = _blocks(x, "fwd_transform_batch")
    out = _torch().empty_like(x) if out is None else out
    check(_lib.load().nh_fwd_transform_batch(x.data_ptr(), out.data_ptr(), b, n, int(bool(use_dst)),
                                             C.c_void_p(_stream(stream, x.device))), "fwd_transform_batch")
    return out


def inv_transform_batch(x, use_dst: bool = False, out=None, stream=None):
    """(B, N, N) int32 -> inverse_transform of every block (transform.py:199-238)."""
    b, n = _blocks(x, "inv_transform_batch")
    out = _torch().empty_like(x) if out is None else out
    check(_lib.load().nh_inv_transform_batch(x.data_ptr(), out.data_ptr(), b, n, int(bool(use_dst)),
                                             C.c_void_p(_stream(stream, x.device))), "inv_transform_batch")
    return out


def quant_batch(c, qp: int, log2size: int, is_intra: bool = True, out=None, stream=None):
    """Elementwise quantize (quant.py:41-79) of an int32 tensor."""
    torch = _torch()
    _need(c, torch.int32, "quant_batch")
    out = torch.empty_like(c) if out is None else out
    check(_lib.load().nh_quant_batch(c.data_ptr(), out.data_ptr(), c.numel(), int(qp), int(log2size),
                                     int(bool(is_intra)), C.c_void_p(_stream(stream, c.device))), "quant_batch")
    return out


def dequant_batch(l, qp: int, out=None, stream=None):
    """Elementwise dequantize (quant.py:82-123) of an int32 tensor."""
    torch = _torch()
    _need(l, torch.int32, "dequant_batch")
    out = torch.empty_like(l) if out is None else out
    check(_lib.load().nh_dequant_batch(l.data_ptr(), out.data_ptr(), l.numel(), int(qp),
                                       C.c_void_p(_stream(stream, l.device))), "dequant_batch")
    return out


def intra_rdo_plane(src, qp: int = 32, pitch: int | None = None, stream=None):
    """Config 3 on one int16 plane (H, W): returns
    (modes u8 (H/8, W/8), levels int32 (H, W), recon int16 (H, W), sse int64 (1,))."""
    torch = _torch()
    _need(src, torch.int16, "intra_rdo_plane")
    h, w = src.shape
    dev = src.device
    modes = torch.zeros((h // 8, w // 8), dtype=torch.uint8, device=dev)
    lvl = torch.zeros((h, w), dtype=torch.int32, device=dev)
    rec = torch.zeros((h, w), dtype=torch.int16, device=dev)
    sse = torch.zeros(1, dtype=torch.int64, device=dev)
    check(_lib.load().nh_intra_rdo_plane(src.data_ptr(), w, h, pitch or w, int(qp), modes.data_ptr(), lvl.data_ptr(),
                                         rec.data_ptr(), sse.data_ptr(), C.c_void_p(_stream(stream, src.device))), "intra_rdo_plane")
    return modes, lvl, rec, sse


def intra_rdo_planes(src, sets: Sequence[PlaneSet], qp: int = 32, lvl=None, rec=None, stream=None):
    """Config 3 over every plane of ``sets`` -- a frame stream
    in one launch pair per set instead of a launch per plane.  Returns (modes
    uint8 [sum of per-plane (h/8)*(w/8), set order], lvl int32, recon int16
    (source layout), sse int64 per plane); the same results as ``intra_rdo_plane``
    plane by plane."""
    torch = _torch()
    _need(src, torch.int16, "intra_rdo_planes(src)")
    sets_fit(sets, src.numel(), "intra_rdo_planes")
    nmodes = sum((s.width // 8) * (s.height // 8) * s.planes_per_group * s.num_groups for s in sets)
    nplanes = sum(s.planes_per_group * s.num_groups for s in sets)
    dev = src.device
    if lvl is None:
        lvl = torch.zeros(src.shape, dtype=torch.int32, device=dev)
    if rec is None:
        rec = torch.zeros(src.shape, dtype=torch.int16, device=dev)
    _need(lvl, torch.int32, "intra_rdo_planes(lvl)")
    _need(rec, torch.int16, "intra_rdo_planes(rec)")
    if lvl.numel() < src.numel() or rec.numel() < src.numel():
        raise ValueError("intra_rdo_planes: lvl / rec smaller than src")
    modes = torch.zeros(max(1, nmodes), dtype=torch.uint8, device=dev)
    sse = torch.zeros(max(1, nplanes), dtype=torch.int64, device=dev)
    arr = (PlaneSet * len(sets))(*sets)
    check(_lib.load().nh_intra_rdo_planes(src.data_ptr(), arr, len(sets), int(qp), modes.data_ptr(), lvl.data_ptr(),
                                          rec.data_ptr(), sse.data_ptr(), C.c_void_p(_stream(stream, dev))),
          "intra_rdo_planes")
    return modes[:nmodes], lvl, rec, sse[:nplanes]


def intra_rdo_closed(src, sets: Sequence[PlaneSet], qp: int = 32, lvl=None, rec=None, stream=None):
    """Config 3 in CLOSED loop over every plane of ``sets``:
    raster block order, neighbours from the reconstruction, wavefront schedule
    on the device.  Returns (modes uint8 [sum of per-plane (h/8)*(w/8)],
    lvl int32, recon int16 (source layout), sse int64 per plane).
    Speed note: the packed 16-bit form runs only when EVERY source sample of
    the call (all sets) is in [0, 255]; one sample outside sends the whole call
    to the 32-bit form (same results, ~1.4x the time).  Split
    such streams into separate calls to keep the 8-bit ones fast."""
    torch = _torch()
    _need(src, torch.int16, "intra_rdo_closed(src)")
    sets_fit(sets, src.numel(), "intra_rdo_closed")
    L = _lib.load()
    arr = (PlaneSet * len(sets))(*sets)
    wb = int(L.nh_intra_rdo_closed_workspace_bytes(arr, len(sets)))
    if wb < 0:
        raise ValueError("intra_rdo_closed: bad plane sets")
    nmodes = sum((s.width // 8) * (s.height // 8) * s.planes_per_group * s.num_groups for s in sets)
    nplanes = sum(s.planes_per_group * s.num_groups for s in sets)
    if lvl is None:
        lvl = torch.zeros(src.shape, dtype=torch.int32, device=src.device)
    if rec is None:
        rec = torch.zeros(src.shape, dtype=torch.int16, device=src.device)
    _need(lvl, torch.int32, "intra_rdo_closed(lvl)")
    _need(rec, torch.int16, "intra_rdo_closed(rec)")
    if lvl.numel() < src.numel() or rec.numel() < src.numel():
        raise ValueError("intra_rdo_closed: lvl / rec smaller than src")
    modes = torch.zeros(max(1, nmodes), dtype=torch.uint8, device=src.device)
    sse = torch.zeros(max(1, nplanes), dtype=torch.int64, device=src.device)
    work = torch.empty((wb + 3) // 4, dtype=torch.int32, device=src.device)
    st = C.c_void_p(_stream(stream, src.device))
    check(L.nh_intra_rdo_planes_closed(src.data_ptr(), arr, len(sets), int(qp), modes.data_ptr(), lvl.data_ptr(),
                                       rec.data_ptr(), sse.data_ptr(), work.data_ptr(), st))
    status = C.c_int(0)
    check(L.nh_intra_rdo_closed_status(work.data_ptr(), C.byref(status), st))
    if status.value:
        raise RuntimeError("intra_rdo_closed: the wavefront stalled (device status word set)")
    return modes[:nmodes], lvl, rec, sse[:nplanes]


def intra_rdo_closed_yuv420_stream(src, width: int, height: int, num_frames: int, qp: int = 32,
                                   batch_frames: int = 64, depth: int = 3, lvl=None, rec=None, stream=None,
                                   frame_stride: int | None = None, base: int = 0):
    """``intra_rdo_closed`` over a stream of YUV420 frames laid out back to back
    (``yuv420_plane_sets``), in batches of ``batch_frames`` frames whose launches
    rotate over ``depth`` streams with no host round trip between them, so a
    batch's block rows fill what the previous batch's wavefront leaves idle while
    it ramps down (1080p: 0.214 vs 0.233 ms per frame for one
    64-frame call).  Same outputs, in the same layout, as one ``intra_rdo_closed``
    call over ``yuv420_plane_sets(num_frames, ...)``: modes and sse of the Y
    planes, then of the U, V planes; lvl / rec in the source layout."""
    torch = _torch()
    if batch_frames < 1 or depth < 1 or num_frames < 0:
        raise ValueError("intra_rdo_closed_yuv420_stream: batch_frames, depth >= 1 and num_frames >= 0")
    fs = frame_stride or yuv420_frame_elems(width, height)
    if fs < yuv420_frame_elems(width, height):
        raise ValueError("intra_rdo_closed_yuv420_stream: frame_stride shorter than a frame")
    all_sets = yuv420_plane_sets(num_frames, width, height, fs, base)
    sets_fit(all_sets, src.numel(), "intra_rdo_closed_yuv420_stream")
    _need(src, torch.int16, "intra_rdo_closed_yuv420_stream(src)")
    dev = src.device
    main = stream if stream is not None else torch.cuda.current_stream(dev)
    if main.device != dev:
        raise ValueError(f"intra_rdo_closed_yuv420_stream: stream on {main.device} but src on {dev}")
    ny = (width // 8) * (height // 8)          # modes per Y plane
    nc = (width // 16) * (height // 16)        # per U / V plane
    with torch.cuda.device(dev), torch.cuda.stream(main):
        if lvl is None:
            lvl = torch.zeros(src.shape, dtype=torch.int32, device=dev)
        if rec is None:
            rec = torch.zeros(src.shape, dtype=torch.int16, device=dev)
        modes = torch.zeros(max(1, num_frames * (ny + 2 * nc)), dtype=torch.uint8, device=dev)
        sse = torch.zeros(max(1, 3 * num_frames), dtype=torch.int64, device=dev)
    _need(lvl, torch.int32, "intra_rdo_closed_yuv420_stream(lvl)")
    _need(rec, torch.int16, "intra_rdo_closed_yuv420_stream(rec)")
    if lvl.numel() < src.numel() or rec.numel() < src.numel():
        raise ValueError("intra_rdo_closed_yuv420_stream: lvl / rec smaller than src")
    if num_frames == 0:
        return modes[:0], lvl, rec, sse[:0]
    L = _lib.load()
    pool = _PIPE_STREAMS3.setdefault(dev.index, [])
    while len(pool) < depth:
        pool.append(torch.cuda.Stream(device=dev))
    fork = torch.cuda.Event()
    fork.record(main)
    for s_ in pool[:depth]:
        s_.wait_event(fork)
    works, keep = [], []
    for b, f0 in enumerate(range(0, num_frames, batch_frames)):
        nb = min(batch_frames, num_frames - f0)
        sets = yuv420_plane_sets(nb, width, height, fs, base + f0 * fs)
        arr = (PlaneSet * 2)(*sets)
        wb = int(L.nh_intra_rdo_closed_workspace_bytes(arr, 2))
        if wb < 0:
            raise ValueError("intra_rdo_closed_yuv420_stream: bad frame size")
        s_ = pool[b % depth]
        with torch.cuda.stream(s_):
            md = torch.empty(nb * (ny + 2 * nc), dtype=torch.uint8, device=dev)
            ss = torch.zeros(3 * nb, dtype=torch.int64, device=dev)   # the kernels add into it
            w_ = torch.empty((wb + 3) // 4, dtype=torch.int32, device=dev)
            check(L.nh_intra_rdo_planes_closed(src.data_ptr(), arr, 2, int(qp), md.data_ptr(), lvl.data_ptr(),
                                               rec.data_ptr(), ss.data_ptr(), w_.data_ptr(), C.c_void_p(s_.cuda_stream)))
            # the batch's modes / sse into the whole stream's layout (Y planes, then U, V planes)
            modes[f0 * ny:(f0 + nb) * ny].copy_(md[:nb * ny])
            modes[num_frames * ny + 2 * f0 * nc:num_frames * ny + 2 * (f0 + nb) * nc].copy_(md[nb * ny:])
            sse[f0:f0 + nb].copy_(ss[:nb])
            sse[num_frames + 2 * f0:num_frames + 2 * (f0 + nb)].copy_(ss[nb:])
        works.append(w_)
        keep += [md, ss]
    for s_ in pool[:depth]:
        join = torch.cuda.Event()
        join.record(s_)
        main.wait_event(join)
    for t in works + keep:
        t.record_stream(main)
    with torch.cuda.device(dev), torch.cuda.stream(main):   # every status word ORed: one host round trip
        both = works[0][:2].clone()
        for w_ in works[1:]:
            both.bitwise_or_(w_[:2])
    status = C.c_int(0)
    check(L.nh_intra_rdo_closed_status(both.data_ptr(), C.byref(status), C.c_void_p(main.cuda_stream)))
    if status.value:
        raise RuntimeError("intra_rdo_closed_yuv420_stream: the wavefront stalled (device status word set)")
    return modes[:num_frames * (ny + 2 * nc)], lvl, rec, sse[:3 * num_frames]


_PIPE_STREAMS3 = {}


def tu_pipeline_plane(src, ctb: int, plane_id: int, seed: int, qp: int = 32, is_luma: bool = True,
                      row0: int = 0, row1: int = 1 << 30, lvl=None, rec=None, tu=None, work=None, stream=None):
    """Config 4 on one int16 plane (H, W), CTU rows [row0, row1).
    Returns (levels int32 (H, W), recon int16 (H, W), tu_log2 u8 (H/4, W/4))."""
    torch = _torch()
    _need(src, torch.int16, "tu_pipeline_plane")
    h, w = src.shape
    dev = src.device
    L = _lib.load()
    lvl = torch.zeros((h, w), dtype=torch.int32, device=dev) if lvl is None else lvl
    rec = torch.zeros((h, w), dtype=torch.int16, device=dev) if rec is None else rec
    tu = torch.zeros((h // 4, w // 4), dtype=torch.uint8, device=dev) if tu is None else tu
    nwork = int(L.nh_tu_workspace_bytes(w, h, ctb))
    if work is None and nwork > 0:
        work = torch.empty(nwork, dtype=torch.uint8, device=dev)
    check(L.nh_tu_pipeline_plane(src.data_ptr(), w, h, w, int(ctb), int(plane_id), int(seed) & 0xFFFFFFFF, int(qp),
                                 int(bool(is_luma)), int(row0), int(min(row1, 1 << 30)), lvl.data_ptr(), rec.data_ptr(),
                                 tu.data_ptr(), work.data_ptr() if work is not None else None,
                                 C.c_void_p(_stream(stream, src.device))), "tu_pipeline_plane")
    return lvl, rec, tu


def tu_pipeline_planes(src, pset: PlaneSet, ctb: int, plane_id: int, seed: int, qp: int = 32, is_luma: bool = True,
                       row0: int = 0, row1: int = 1 << 30, lvl=None, rec=None, tu=None, stream=None):
    """Config 4 over every plane of one plane set in one launch (plane p =
    g*ppg + c gets plane id plane_id + c), CTU rows [row0, row1).  ``lvl`` and
    ``rec`` share the source's layout; the set may describe a band-local buffer
    as rows of the full plane (shard.Cfg4Layout: only the band's rows and the
    row above are read).  Returns (lvl int32, recon int16, tu uint8 (planes,
    h/4, w/4), indexed by full-plane position))."""
    torch = _torch()
    _need(src, torch.int16, "tu_pipeline_planes(src)")
    # the launch reads rows [row0*ctb - 1, row1*ctb) (its CTU rows + the source row above) and writes its CTU rows
    sets_fit_rows([pset], src.numel(), int(row0) * ctb - 1, min(int(row1), 1 << 30) * ctb, "tu_pipeline_planes")
    planes = pset.planes_per_group * pset.num_groups
    if lvl is None:
        lvl = torch.zeros(src.shape, dtype=torch.int32, device=src.device)
    if rec is None:
        rec = torch.zeros(src.shape, dtype=torch.int16, device=src.device)
    if tu is None:
        tu = torch.zeros((planes, pset.height // 4, pset.width // 4), dtype=torch.uint8, device=src.device)
    _need(lvl, torch.int32, "tu_pipeline_planes(lvl)")
    _need(rec, torch.int16, "tu_pipeline_planes(rec)")
    _need(tu, torch.uint8, "tu_pipeline_planes(tu)")
    if lvl.numel() < src.numel() or rec.numel() < src.numel() or tu.numel() < planes * (pset.height // 4) * (pset.width // 4):
        raise ValueError("tu_pipeline_planes: output too small")
    check(_lib.load().nh_tu_pipeline_planes(src.data_ptr(), C.byref(pset), int(ctb), int(plane_id), int(seed) & 0xffffffff,
                                            int(qp), int(bool(is_luma)), int(row0), int(min(row1, 1 << 30)),
                                            lvl.data_ptr(), rec.data_ptr(), tu.data_ptr(), C.c_void_p(_stream(stream, src.device))))
    return lvl, rec, tu


def tu_pipeline_planes_compact(src, pset: PlaneSet, ctb: int, plane_id: int, seed: int, qp: int = 32,
                               is_luma: bool = True, row0: int = 0, row1: int = 1 << 30, lvl=None, rec=None, tu=None,
                               spill=None, stream=None):
    """``tu_pipeline_planes`` with COMPACT levels: int16 levels in the source
    layout (exact: |level| <= 408 for an 8-bit TU at every QP and size,
    tools/packed_bounds.py level_bounds) -- 6 instead of 8 bytes per sample.
    Strips with a sample outside [0, 255] (the 32-bit chain) write their int32
    levels into ``spill`` (int32, source layout; allocated uninitialised when
    None) and -32768 at each strip origin.  CTB 16 / 32.  Returns (lvl int16, rec,
    tu, spill); ``tu_levels_widen`` gives the int32 levels of ``tu_pipeline_planes``."""
    torch = _torch()
    _need(src, torch.int16, "tu_pipeline_planes_compact(src)")
    sets_fit_rows([pset], src.numel(), int(row0) * ctb - 1, min(int(row1), 1 << 30) * ctb, "tu_pipeline_planes_compact")
    planes = pset.planes_per_group * pset.num_groups
    if lvl is None:
        lvl = torch.zeros(src.shape, dtype=torch.int16, device=src.device)
    if rec is None:
        rec = torch.zeros(src.shape, dtype=torch.int16, device=src.device)
    if tu is None:
        tu = torch.zeros((planes, pset.height // 4, pset.width // 4), dtype=torch.uint8, device=src.device)
    if spill is None:
        spill = torch.empty(src.shape, dtype=torch.int32, device=src.device)
    _need(lvl, torch.int16, "tu_pipeline_planes_compact(lvl)")
    _need(rec, torch.int16, "tu_pipeline_planes_compact(rec)")
    _need(tu, torch.uint8, "tu_pipeline_planes_compact(tu)")
    _need(spill, torch.int32, "tu_pipeline_planes_compact(spill)")
    if min(lvl.numel(), rec.numel(), spill.numel()) < src.numel() or \
            tu.numel() < planes * (pset.height // 4) * (pset.width // 4):
        raise ValueError("tu_pipeline_planes_compact: output too small")
    check(_lib.load().nh_tu_pipeline_planes_compact(
        src.data_ptr(), C.byref(pset), int(ctb), int(plane_id), int(seed) & 0xffffffff, int(qp), int(bool(is_luma)),
        int(row0), int(min(row1, 1 << 30)), lvl.data_ptr(), spill.data_ptr(), rec.data_ptr(), tu.data_ptr(),
        C.c_void_p(_stream(stream, src.device))), "tu_pipeline_planes_compact")
    return lvl, rec, tu, spill


def tu_levels_widen(lvl, spill, pset: PlaneSet, ctb: int, row0: int = 0, row1: int = 1 << 30, out=None, stream=None):
    """(int16 levels, spill) of ``tu_pipeline_planes_compact`` -> the reference's
    int32 levels of CTU rows [row0, row1) of every plane of ``pset``."""
    torch = _torch()
    _need(lvl, torch.int16, "tu_levels_widen(lvl)")
    _need(spill, torch.int32, "tu_levels_widen(spill)")
    if out is None:
        out = torch.zeros(lvl.shape, dtype=torch.int32, device=lvl.device)
    _need(out, torch.int32, "tu_levels_widen(out)")
    sets_fit_rows([pset], min(lvl.numel(), spill.numel(), out.numel()), int(row0) * ctb,
                  min(int(row1), 1 << 30) * ctb, "tu_levels_widen")
    check(_lib.load().nh_tu_levels_widen(lvl.data_ptr(), spill.data_ptr(), C.byref(pset), int(ctb), int(row0),
                                         int(min(row1, 1 << 30)), out.data_ptr(), C.c_void_p(_stream(stream, lvl.device))),
          "tu_levels_widen")
    return out


def _tu_closed_launch(src, pset: PlaneSet, ctb: int, plane_id: int, seed: int, qp: int, is_luma: bool,
                      lvl, rec, tu, strm):
    """Stream-ordered launch of the config-4 closed loop over one plane set on the
    torch stream ``strm`` (default outputs are zero-filled on that stream too);
    returns (lvl, rec, tu, workspace) -- the workspace holds the wavefront status word."""
    torch = _torch()
    with torch.cuda.device(src.device), torch.cuda.stream(strm):
        return _tu_closed_launch_on(src, pset, ctb, plane_id, seed, qp, is_luma, lvl, rec, tu, int(strm.cuda_stream))


def _tu_closed_launch_on(src, pset, ctb, plane_id, seed, qp, is_luma, lvl, rec, tu, st: int):
    torch = _torch()
    _need(src, torch.int16, "tu_pipeline_closed(src)")
    sets_fit([pset], src.numel(), "tu_pipeline_closed")
    planes = pset.planes_per_group * pset.num_groups
    L = _lib.load()
    wb = int(L.nh_tu_pipeline_closed_workspace_bytes(C.byref(pset), int(ctb)))
    if wb < 0:
        raise ValueError("tu_pipeline_closed: bad plane set (w, h multiples of 4) or CTB size")
    if lvl is None:
        lvl = torch.zeros(src.shape, dtype=torch.int32, device=src.device)
    if rec is None:
        rec = torch.zeros(src.shape, dtype=torch.int16, device=src.device)
    if tu is None:
        tu = torch.zeros((planes, pset.height // 4, pset.width // 4), dtype=torch.uint8, device=src.device)
    _need(lvl, torch.int32, "tu_pipeline_closed(lvl)")
    _need(rec, torch.int16, "tu_pipeline_closed(rec)")
    _need(tu, torch.uint8, "tu_pipeline_closed(tu)")
    if lvl.numel() < src.numel() or rec.numel() < src.numel() or tu.numel() < planes * (pset.height // 4) * (pset.width // 4):
        raise ValueError("tu_pipeline_closed: output too small")
    work = torch.empty((wb + 7) // 8, dtype=torch.int64, device=src.device)
    check(L.nh_tu_pipeline_planes_closed(src.data_ptr(), C.byref(pset), int(ctb), int(plane_id), int(seed) & 0xffffffff,
                                         int(qp), int(bool(is_luma)), lvl.data_ptr(), rec.data_ptr(), tu.data_ptr(),
                                         work.data_ptr(), C.c_void_p(st)), "tu_pipeline_closed")
    return lvl, rec, tu, work


def _tu_closed_status(work, st: int, what: str):
    status = C.c_int(0)
    check(_lib.load().nh_intra_rdo_closed_status(work.data_ptr(), C.byref(status), C.c_void_p(st)))
    if status.value:
        raise RuntimeError("%s: the device wavefront stalled (status %d)" % (what, status.value))


def tu_pipeline_closed(src, pset: PlaneSet, ctb: int, plane_id: int, seed: int, qp: int = 32, is_luma: bool = True,
                       lvl=None, rec=None, tu=None, stream=None):
    """Config 4 in CLOSED loop over every plane of one plane
    set: TUs in z-order with neighbours from the reconstruction, a device
    wavefront over CTU rows.  Returns (lvl int32, recon int16 -- source
    layout, zeros outside every TU --, tu uint8 (planes, h/4, w/4)).
    Speed note: the packed 16-bit plane-pair form runs only when EVERY source
    sample of the set is in [0, 255]; one sample outside sends the whole set to
    the 32-bit form (same results, ~1.7x the time)."""
    torch = _torch()
    strm = stream if stream is not None else torch.cuda.current_stream(src.device)
    st = _stream(strm, src.device)
    lvl, rec, tu, work = _tu_closed_launch(src, pset, ctb, plane_id, seed, qp, is_luma, lvl, rec, tu, strm)
    _tu_closed_status(work, st, "tu_pipeline_closed")
    return lvl, rec, tu


_SIDE_STREAMS = {}


def tu_pipeline_closed_yuv420(src, luma: PlaneSet, chroma: PlaneSet, seed: int, qp: int = 32,
                              lvl=None, rec=None, tu_luma=None, tu_chroma=None, stream=None):
    """Config 4 in closed loop over a YUV420 stream: the luma set (CTB 32,
    plane id 0) and the chroma set (CTB 16, plane ids 1, 2) -- the two calls
    of ``tu_pipeline_closed`` -- run as two concurrent device wavefronts, the
    chroma one on a side stream forked from and joined back into ``stream``.
    One set's CTU rows alone leave most SIMDs with one latency-bound wave
    (DESIGN.md §4.4a).  Same results as the two calls in sequence.
    Returns (lvl, rec, tu_luma, tu_chroma)."""
    torch = _torch()
    dev = src.device
    main = stream if stream is not None else torch.cuda.current_stream(dev)
    if main.device != dev:
        raise ValueError(f"tu_pipeline_closed_yuv420: stream on {main.device} but src on {dev}")
    if not sets_disjoint(luma, chroma):
        # the two wavefronts would write shared lvl / rec elements concurrently: code them in sequence
        lvl, rec, tu_luma = tu_pipeline_closed(src, luma, 32, 0, seed, qp, True, lvl, rec, tu_luma, main)
        lvl, rec, tu_chroma = tu_pipeline_closed(src, chroma, 16, 1, seed, qp, False, lvl, rec, tu_chroma, main)
        return lvl, rec, tu_luma, tu_chroma
    side = _SIDE_STREAMS.get(dev.index)
    if side is None:
        side = _SIDE_STREAMS[dev.index] = torch.cuda.Stream(device=dev)
    with torch.cuda.device(dev), torch.cuda.stream(main):   # default outputs zero-filled in order on `main`
        if lvl is None:
            lvl = torch.zeros(src.shape, dtype=torch.int32, device=dev)
        if rec is None:
            rec = torch.zeros(src.shape, dtype=torch.int16, device=dev)
    fork = torch.cuda.Event()
    fork.record(main)
    side.wait_event(fork)
    # luma first: its wavefront is the critical path and its waves take their slots before chroma's
    # (0.1179 vs 0.1205 ms per 4K frame chroma-first)
    _, _, tu_luma, work_y = _tu_closed_launch(src, luma, 32, 0, seed, qp, True, lvl, rec, tu_luma, main)
    _, _, tu_chroma, work_c = _tu_closed_launch(src, chroma, 16, 1, seed, qp, False, lvl, rec, tu_chroma, side)
    join = torch.cuda.Event()
    join.record(side)
    main.wait_event(join)
    for t in (tu_chroma, work_c):
        t.record_stream(main)
    # one host round trip for both status words: chroma's ORed into a copy of luma's on `main`
    with torch.cuda.device(dev), torch.cuda.stream(main):
        both = work_y[:1].clone()
        both.view(torch.int32)[1:2].bitwise_or_(work_c[:1].view(torch.int32)[1:2])
    try:
        _tu_closed_status(both, int(main.cuda_stream), "tu_pipeline_closed_yuv420")
    except RuntimeError:
        _tu_closed_status(work_y, int(main.cuda_stream), "tu_pipeline_closed_yuv420 (luma)")
        _tu_closed_status(work_c, int(main.cuda_stream), "tu_pipeline_closed_yuv420 (chroma)")
        raise
    return lvl, rec, tu_luma, tu_chroma


_PIPE_STREAMS = {}


def tu_pipeline_closed_yuv420_stream(src, width: int, height: int, num_frames: int, seed: int, qp: int = 32,
                                     batch_frames: int = 128, depth: int = 3, lvl=None, rec=None, tu_luma=None,
                                     tu_chroma=None, stream=None, frame_stride: int | None = None, base: int = 0):
    """Config 4 in closed loop over a stream of YUV420 frames laid out back to
    back (PackedFrame layout, as ``yuv420_plane_sets``): batches of
    ``batch_frames`` frames, each batch's luma and chroma wavefronts
    (``tu_pipeline_closed_yuv420``) on a stream pair of their own, ``depth``
    pairs in rotation, so up to ``depth`` batches are in flight: a batch's CTU
    rows fill the SIMDs that the previous batch's wavefront leaves idle while it
    ramps down (4K: 0.048-0.049 ms per frame with the defaults,
    0.054-0.055 with 64-frame batches, vs 0.065-0.068 for one 64-frame call).
    No host round trip between batches; one status check at the end.  Same results as one ``tu_pipeline_closed_yuv420``
    call over all the frames (frames are independent).
    Returns (lvl, rec, tu_luma (num_frames, h/4, w/4), tu_chroma (2 num_frames, h/8, w/8))."""
    torch = _torch()
    if batch_frames < 1 or depth < 1 or num_frames < 0:
        raise ValueError("tu_pipeline_closed_yuv420_stream: batch_frames, depth >= 1 and num_frames >= 0")
    fs = frame_stride or yuv420_frame_elems(width, height)
    if fs < yuv420_frame_elems(width, height):
        raise ValueError("tu_pipeline_closed_yuv420_stream: frame_stride shorter than a frame")
    sets_fit(yuv420_plane_sets(num_frames, width, height, fs, base), src.numel(), "tu_pipeline_closed_yuv420_stream")
    dev = src.device
    main = stream if stream is not None else torch.cuda.current_stream(dev)
    if main.device != dev:
        raise ValueError(f"tu_pipeline_closed_yuv420_stream: stream on {main.device} but src on {dev}")
    with torch.cuda.device(dev), torch.cuda.stream(main):   # outputs zero-filled in order on `main`, before the fork
        if lvl is None:
            lvl = torch.zeros(src.shape, dtype=torch.int32, device=dev)
        if rec is None:
            rec = torch.zeros(src.shape, dtype=torch.int16, device=dev)
        if tu_luma is None:
            tu_luma = torch.zeros((num_frames, height // 4, width // 4), dtype=torch.uint8, device=dev)
        if tu_chroma is None:
            tu_chroma = torch.zeros((2 * num_frames, height // 8, width // 8), dtype=torch.uint8, device=dev)
    for t, what, n in ((tu_luma, "tu_luma", num_frames), (tu_chroma, "tu_chroma", 2 * num_frames)):
        if not t.is_contiguous() or t.dim() != 3 or t.shape[0] < n:
            raise ValueError(f"tu_pipeline_closed_yuv420_stream: {what} must be a contiguous (>= {n}, h, w) tensor")
    if num_frames == 0:
        return lvl, rec, tu_luma, tu_chroma
    pool = _PIPE_STREAMS.setdefault(dev.index, [])
    while len(pool) < depth:
        pool.append((torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)))
    fork = torch.cuda.Event()
    fork.record(main)
    for pair in pool[:depth]:
        for s_ in pair:
            s_.wait_event(fork)
    works = []
    for b, f0 in enumerate(range(0, num_frames, batch_frames)):
        nb = min(batch_frames, num_frames - f0)
        sy, suv = yuv420_plane_sets(nb, width, height, fs, base + f0 * fs)
        ls, cs = pool[b % depth]
        works.append(_tu_closed_launch(src, sy, 32, 0, seed, qp, True, lvl, rec, tu_luma[f0:f0 + nb], ls)[3])
        works.append(_tu_closed_launch(src, suv, 16, 1, seed, qp, False, lvl, rec,
                                       tu_chroma[2 * f0:2 * (f0 + nb)], cs)[3])
    for pair in pool[:depth]:
        for s_ in pair:
            join = torch.cuda.Event()
            join.record(s_)
            main.wait_event(join)
    for w_ in works:
        w_.record_stream(main)
    with torch.cuda.device(dev), torch.cuda.stream(main):   # every status word ORed: one host round trip
        both = works[0][:1].clone()
        for w_ in works[1:]:
            both.view(torch.int32)[1:2].bitwise_or_(w_[:1].view(torch.int32)[1:2])
    try:
        _tu_closed_status(both, int(main.cuda_stream), "tu_pipeline_closed_yuv420_stream")
    except RuntimeError:
        for k, w_ in enumerate(works):
            _tu_closed_status(w_, int(main.cuda_stream),
                              f"tu_pipeline_closed_yuv420_stream (batch {k // 2}, {'chroma' if k % 2 else 'luma'})")
        raise
    return lvl, rec, tu_luma, tu_chroma


def tc32_plane(src, qp: int = 32, variant: int = 1, lvl=None, rec=None, stream=None):
    """Config 5 on one int16 plane (H, W), W % 8 == 0: every full
    32x32 block through the chain.  variant 0 = butterfly, 1 = matrix cores (f16
    for 8-bit blocks, int8 otherwise), 2 = int8 MFMA only (A/B).
    Returns (levels int32 (H, W), recon int16 (H, W))."""
    torch = _torch()
    _need(src, torch.int16, "tc32_plane")
    h, w = src.shape
    lvl = torch.zeros((h, w), dtype=torch.int32, device=src.device) if lvl is None else lvl
    rec = torch.zeros((h, w), dtype=torch.int16, device=src.device) if rec is None else rec
    check(_lib.load().nh_tc32_plane(src.data_ptr(), w, h, w, int(qp), lvl.data_ptr(), rec.data_ptr(), int(variant),
                                    C.c_void_p(_stream(stream, src.device))), "tc32_plane")
    return lvl, rec


def tc32_planes(src, sets, qp: int = 32, variant: int = 1, lvl=None, rec=None, stream=None):
    """Config 5 over every plane of ``sets`` (e.g. yuv420_plane_sets of a frame
    stream): per plane set one f16-MFMA launch plus an int8 fix-up for non-8-bit
    blocks (variant 1), one int8-MFMA launch (2), or the butterfly
    per plane (variant 0).  Returns (levels int32, recon int16), source layout."""
    torch = _torch()
    _need(src, torch.int16, "tc32_planes(src)")
    sets_fit(sets, src.numel(), "tc32_planes")
    if lvl is None:
        lvl = torch.zeros(src.shape, dtype=torch.int32, device=src.device)
    if rec is None:
        rec = torch.zeros(src.shape, dtype=torch.int16, device=src.device)
    _need(lvl, torch.int32, "tc32_planes(lvl)")
    _need(rec, torch.int16, "tc32_planes(rec)")
    if lvl.numel() < src.numel() or rec.numel() < src.numel():
        raise ValueError("tc32_planes: lvl / rec smaller than src")
    arr = (PlaneSet * len(sets))(*sets)
    check(_lib.load().nh_tc32_planes(src.data_ptr(), arr, len(sets), int(qp), lvl.data_ptr(), rec.data_ptr(),
                                     int(variant), C.c_void_p(_stream(stream, src.device))), "tc32_planes")
    return lvl, rec


def tc32_planes_compact(src, sets, qp: int = 32, level_dtype=None, lvl=None, rec=None, spill=None, stream=None):
    """Config 5 (variant 1) with COMPACT levels: int16 (default) or int8 levels in
    the source layout -- exact, an 8-bit block's 32x32 levels satisfy |level| <= 51
    at every QP (tools/packed_bounds.py level_bounds) -- 6 / 5 bytes per sample of
    traffic instead of 8.  A block that is not 8-bit writes its int32 levels into
    ``spill`` (int32, source layout; allocated uninitialised when None) and the
    marker -32768 / -128 at its compact origin.  Returns (lvl, rec, spill);
    ``tc32_levels_widen(lvl, spill, sets)`` gives the int32 levels of
    ``tc32_planes``."""
    torch = _torch()
    _need(src, torch.int16, "tc32_planes_compact(src)")
    sets_fit(sets, src.numel(), "tc32_planes_compact")
    dt = level_dtype if level_dtype is not None else (lvl.dtype if lvl is not None else torch.int16)
    if dt not in (torch.int16, torch.int8):
        raise TypeError("tc32_planes_compact: level_dtype must be torch.int16 or torch.int8")
    if lvl is None:
        lvl = torch.zeros(src.shape, dtype=dt, device=src.device)
    if rec is None:
        rec = torch.zeros(src.shape, dtype=torch.int16, device=src.device)
    if spill is None:
        spill = torch.empty(src.shape, dtype=torch.int32, device=src.device)
    _need(lvl, dt, "tc32_planes_compact(lvl)")
    _need(rec, torch.int16, "tc32_planes_compact(rec)")
    _need(spill, torch.int32, "tc32_planes_compact(spill)")
    if min(lvl.numel(), rec.numel(), spill.numel()) < src.numel():
        raise ValueError("tc32_planes_compact: lvl / rec / spill smaller than src")
    arr = (PlaneSet * len(sets))(*sets)
    check(_lib.load().nh_tc32_planes_compact(src.data_ptr(), arr, len(sets), int(qp), lvl.data_ptr(),
                                             lvl.element_size(), spill.data_ptr(), rec.data_ptr(),
                                             C.c_void_p(_stream(stream, src.device))), "tc32_planes_compact")
    return lvl, rec, spill


def tc32_levels_widen(lvl, spill, sets, out=None, stream=None):
    """(compact levels, spill) of ``tc32_planes_compact`` -> the reference's int32
    levels at every sample of every full 32x32 block (other samples of ``out``
    are left as they are: zeros by default, as ``tc32_planes``)."""
    torch = _torch()
    if not isinstance(lvl, torch.Tensor) or lvl.dtype not in (torch.int16, torch.int8):
        raise TypeError("tc32_levels_widen: lvl must be an int16 / int8 device tensor")
    _need(lvl, lvl.dtype, "tc32_levels_widen(lvl)")
    _need(spill, torch.int32, "tc32_levels_widen(spill)")
    if out is None:
        out = torch.zeros(lvl.shape, dtype=torch.int32, device=lvl.device)
    _need(out, torch.int32, "tc32_levels_widen(out)")
    sets_fit(sets, min(lvl.numel(), spill.numel(), out.numel()), "tc32_levels_widen")
    arr = (PlaneSet * len(sets))(*sets)
    check(_lib.load().nh_tc32_levels_widen(lvl.data_ptr(), lvl.element_size(), spill.data_ptr(), arr, len(sets),
                                           out.data_ptr(), C.c_void_p(_stream(stream, lvl.device))),
          "tc32_levels_widen")
    return out


# ---------------------------------------------------------------------------
# Frame I/O (frame.py:44-54, :87-115, :176-183) and the frame-level intra
# driver (__main__.py:142-189) -- SURVEY.md §8(f) f-3 / f-1.
# ---------------------------------------------------------------------------
ENC_STATS = 6   # blocks, dc wins, planar wins, dc energy, planar energy, uint8 SSE


def widen_u8(src, out=None, stream=None):
    """uint8 samples (e.g. YUV420p bytes uploaded as-is) -> int16, i.e.
    Plane.from_buffer(..).data.astype(np.int16) for every plane at once."""
    torch = _torch()
    _need(src, torch.uint8, "widen_u8(src)")
    if out is None:
        out = torch.empty(src.shape, dtype=torch.int16, device=src.device)
    _need(out, torch.int16, "widen_u8(out)")
    if out.numel() != src.numel():
        raise ValueError("widen_u8: size mismatch")
    check(_lib.load().nh_widen_u8_i16(src.data_ptr(), out.data_ptr(), src.numel(), C.c_void_p(_stream(stream, src.device))))
    return out


def narrow_u8(src, out=None, stream=None):
    """int16 -> uint8 keeping the low byte: numpy's .astype(np.uint8) as used by
    Frame.to_yuv420p / PackedFrame.to_yuv420p."""
    torch = _torch()
    _need(src, torch.int16, "narrow_u8(src)")
    if out is None:
        out = torch.empty(src.shape, dtype=torch.uint8, device=src.device)
    _need(out, torch.uint8, "narrow_u8(out)")
    if out.numel() != src.numel():
        raise ValueError("narrow_u8: size mismatch")
    check(_lib.load().nh_narrow_i16_u8(src.data_ptr(), out.data_ptr(), src.numel(), C.c_void_p(_stream(stream, src.device))))
    return out


def luma_block_size(block_size: int) -> int:
    """encode_frame_intra's luma block: block_size, at least 4 (__main__.py:156-158)."""
    return max(4, block_size)


def chroma_block_size(block_size: int) -> int:
    """encode_frame_intra's chroma block: block_size // 2, at least 4 (__main__.py:156-158)."""
    return max(4, block_size // 2)


def _check_block_size(bs: int):
    if not 1 <= bs <= 65536:
        raise ValueError(f"block size {bs}: the device driver takes 1..65536")


def encode_intra_planes(src, sets: Sequence[PlaneSet], block_sizes: Sequence[int], recon=None, recon_u8=None,
                        stats=None, stream=None):
    """The per-block decision of encode_frame_intra over every plane of ``sets``
    inside ``src`` (uint8 or int16), any block size >= 1.  Returns the
    (accumulated) int64 stats tensor, one ENC_STATS row per plane, planes
    numbered set by set.  Raises OverflowError where the reference's planar
    store does (int16 samples at a block size that is not a power of two: the
    call then waits for the launch to read the status word)."""
    torch = _torch()
    if not isinstance(src, torch.Tensor) or not src.is_cuda or src.dtype not in (torch.uint8, torch.int16):
        raise TypeError("encode_intra_planes(src): expected a uint8 or int16 device tensor")
    if not src.is_contiguous():
        raise ValueError("encode_intra_planes(src): tensor must be contiguous")
    for bs in block_sizes:
        _check_block_size(int(bs))
    if len(block_sizes) != len(sets):
        raise ValueError("encode_intra_planes: one block size per plane set")
    nplanes = sum(s.planes_per_group * s.num_groups for s in sets)
    sets_fit(sets, src.numel(), "encode_intra_planes")
    if stats is None:
        stats = torch.zeros((nplanes, ENC_STATS), dtype=torch.int64, device=src.device)
    _need(stats, torch.int64, "encode_intra_planes(stats)")
    if stats.numel() < nplanes * ENC_STATS:
        raise ValueError("encode_intra_planes: stats too small")
    for t, dt, nm in ((recon, torch.int16, "recon"), (recon_u8, torch.uint8, "recon_u8")):
        if t is not None:
            _need(t, dt, f"encode_intra_planes({nm})")
            if t.numel() < src.numel():
                raise ValueError(f"encode_intra_planes: {nm} smaller than src")
    arr = (PlaneSet * len(sets))(*sets)
    bsz = (C.c_int32 * len(sets))(*[int(b) for b in block_sizes])
    wide = src.dtype == torch.int16 and any(int(b) & (int(b) - 1) or int(b) < 4 or int(b) > 64 for b in block_sizes)
    status = torch.zeros(1, dtype=torch.int32, device=src.device) if wide else None
    strm = stream if stream is not None else torch.cuda.current_stream(src.device)
    check(_lib.load().nh_encode_intra_planes(
        src.data_ptr(), int(src.dtype == torch.uint8), arr, len(sets), bsz,
        recon.data_ptr() if recon is not None else None, recon_u8.data_ptr() if recon_u8 is not None else None,
        stats.data_ptr(), status.data_ptr() if status is not None else None,
        C.c_void_p(_stream(strm, src.device))))
    if status is not None:
        strm.synchronize()   # the launch's stream only (it may not be torch's current one), not the whole device
    if status is not None and int(status.item()):
        raise OverflowError("encode_intra_planes: planar prediction out of bounds for int16 (intra.py:111)")
    return stats


def encode_intra_yuv420(frames, width: int, height: int, block_size: int, recon=None, recon_u8=None,
                        stream=None):
    """encode_frame_intra (__main__.py:142-189) on a stream of YUV420p frames laid
    out back to back in ``frames`` (uint8 bytes straight from a .yuv file, or
    int16 samples).  Returns stats as an int64 tensor (F, 3, ENC_STATS) for
    the Y, U and V planes of every frame; ``recon`` (int16) / ``recon_u8``
    (to_yuv420p bytes) receive the reconstruction when given."""
    fe = yuv420_frame_elems(width, height)
    if frames.numel() % fe:
        raise ValueError("encode_intra_yuv420: size is not a whole number of frames")
    nf = frames.numel() // fe
    sets = yuv420_plane_sets(nf, width, height)
    st = encode_intra_planes(frames, sets, [luma_block_size(block_size), chroma_block_size(block_size)], recon,
                             recon_u8, stream=stream)
    y, uv = st[:nf], st[nf:].view(nf, 2, ENC_STATS)
    return _torch().cat([y.view(nf, 1, ENC_STATS), uv], 1)


# ---------------------------------------------------------------------------
# block-call server controls (per-block drop-in calls)
# ---------------------------------------------------------------------------
def block_server_stop() -> None:
    """Ask every resident block-call server to leave now and wait until it has
    (a device-wide synchronize then no longer waits for its idle time)."""
    check(_lib.load().nh_block_server_stop(), "block_server_stop")


def block_server_set_idle_us(us: int) -> None:
    """Idle time (us) a server stays resident without a request; 0 = no server
    (every per-block call is its own kernel launch)."""
    check(_lib.load().nh_block_server_set_idle_us(int(us)), "block_server_set_idle_us")


def block_server_stats(device: int = 0) -> dict:
    out = (C.c_int64 * 4)()
    check(_lib.load().nh_block_server_stats(int(device), out), "block_server_stats")
    return {"served": out[0], "launches": out[1], "kernel_calls": out[2], "idle_us": out[3]}

"""Intra prediction -- drop-in for the reference ``nano_hevc.intra`` (intra.py:1-207).

Same names, signatures, output dtypes and exceptions; every sample is computed
by the gfx950 kernels in libnanohevc.so (k_intra_dc / k_intra_planar /
k_intra_angular / k_residual / k_clip in csrc/nh_blocks.hip).  The shim only
converts inputs the way the reference itself does (``.astype(np.int16)``,
``int(...)`` of array elements) before handing host buffers to the C ABI.
"""
from __future__ import annotations

import operator

import numpy as np

from . import _lib
from ._lib import check, ptr

# intra.py:24-29 (spec Table 8-4, 1/32-pel units), modes 2..34
INTRA_PRED_ANGLE = [
    32, 26, 21, 17, 13, 9, 5, 2, 0,
    -2, -5, -9, -13, -17, -21, -26, -32,
    -26, -21, -17, -13, -9, -5, -2, 0,
    2, 5, 9, 13, 17, 21, 26, 32,
]
# intra.py:31-34
INV_ANGLE = {-2: -4096, -5: -1638, -9: -910, -13: -630, -17: -482, -21: -390, -26: -315, -32: -256}


def _ints1d(x, what):
    """Integer 1-D view as int64 (lossless for every integer dtype but uint64 > 2^63)."""
    a = np.asarray(x)
    if a.dtype.kind not in "iub":
        raise NotImplementedError(f"{what}: nano_hevc (MI355X) takes integer sample arrays, got {a.dtype}")
    return np.ascontiguousarray(a.ravel(), dtype=np.int64)


def _corner(v, what):
    if isinstance(v, (float, np.floating)):
        raise NotImplementedError(f"{what}: integer corner sample expected")
    return operator.index(v)


def intra_dc_predict_4x4(top, left):
    """intra.py:37-43: DC = (sum(top) + sum(left) + 4) >> 3, 4x4 int16."""
    t, l = _ints1d(top, "top"), _ints1d(left, "left")
    out = np.empty((4, 4), np.int16)
    check(_lib.load().nh_intra_dc(ptr(t), t.size, ptr(l), l.size, 4, 1, ptr(out)), "intra_dc_predict_4x4")
    return out


def intra_dc_predict(top, left, size):
    """intra.py:46-62: DC = (sum(top) + sum(left) + size) // (2*size) over the WHOLE arrays."""
    size = operator.index(size)
    if size == 0:
        raise ZeroDivisionError("integer division or modulo by zero")
    if size < 0:
        raise ValueError("negative dimensions are not allowed")
    t, l = _ints1d(top, "top"), _ints1d(left, "left")
    out = np.empty((size, size), np.int16)
    check(_lib.load().nh_intra_dc(ptr(t), t.size, ptr(l), l.size, size, 0, ptr(out)), "intra_dc_predict")
    return out


def residual_block(orig, pred):
    """intra.py:65-67: orig.astype(int16) - pred.astype(int16) (int16 wrap, broadcasting)."""
    a = np.asarray(orig).astype(np.int16)
    b = np.asarray(pred).astype(np.int16)
    a, b = np.broadcast_arrays(a, b)
    a, b = np.ascontiguousarray(a), np.ascontiguousarray(b)
    out = np.empty(a.shape, np.int16)
    check(_lib.load().nh_residual(ptr(a), ptr(b), a.size, ptr(out)), "residual_block")
    return out


def reconstruct_block(pred, residual):
    """intra.py:70-72: pred.astype(int16) + residual.astype(int16) (int16 wrap)."""
    a = np.asarray(pred).astype(np.int16)
    b = np.asarray(residual).astype(np.int16)
    a, b = np.broadcast_arrays(a, b)
    a, b = np.ascontiguousarray(a), np.ascontiguousarray(b)
    out = np.empty(a.shape, np.int16)
    check(_lib.load().nh_reconstruct(ptr(a), ptr(b), a.size, ptr(out)), "reconstruct_block")
    return out


def clip_to_pixel_range(block, bit_depth: int = 8):
    """intra.py:75-78: np.clip(block, 0, 2**bd - 1).astype(int16)."""
    max_val = (1 << bit_depth) - 1
    a = np.asarray(block)
    if a.dtype.kind not in "iu":
        raise NotImplementedError(f"clip_to_pixel_range: integer blocks only, got {a.dtype}")
    np.clip(np.empty(0, a.dtype), 0, max_val)   # numpy's own bound/dtype checks (raises like the reference)
    x = np.ascontiguousarray(a, dtype=np.int64)
    out = np.empty(a.shape, np.int16)
    check(_lib.load().nh_clip(ptr(x), x.size, min(max_val, 2**63 - 1), ptr(out)), "clip_to_pixel_range")
    return out


def _narrow_corner_ok(v, n, arrays):
    """Planar with a narrow numpy-scalar corner computes in that dtype (NEP 50);
    it equals Python-int math iff nothing can overflow it.  Check the bound."""
    if not isinstance(v, np.integer) or v.dtype.itemsize >= 8:
        return
    info = np.iinfo(v.dtype)
    m = max([abs(int(v))] + [int(np.abs(a).max()) if a.size else 0 for a in arrays])
    if 2 * n * m + n > min(info.max, -info.min - 1):
        raise NotImplementedError(
            f"intra_planar_predict: {v.dtype} corner arithmetic may wrap for these samples; pass Python ints")


def intra_planar_predict(top, left, top_right, bottom_left, size):
    """intra.py:81-113: pred[y,x] = ((N-1-x)left[y] + (x+1)tr + (N-1-y)top[x] + (y+1)bl + N) >> (log2N+1)."""
    size = operator.index(size)
    if size < 0:
        raise ValueError("negative dimensions are not allowed")
    log2_size = int(np.log2(size))          # the reference's own parameter computation
    t, l = _ints1d(top, "top"), _ints1d(left, "left")
    n = min(size, t.size, l.size)
    _narrow_corner_ok(top_right, size, [t[:n], l[:n]])
    _narrow_corner_ok(bottom_left, size, [t[:n], l[:n]])
    tr, bl = _corner(top_right, "top_right"), _corner(bottom_left, "bottom_left")
    out = np.empty((size, size), np.int16)
    check(_lib.load().nh_intra_planar(ptr(t), t.size, ptr(l), l.size, tr, bl, size, log2_size, ptr(out)),
          "intra_planar_predict")
    return out


def intra_angular_predict(top, left, top_left, mode, size):
    """intra.py:116-156 (+ _build_ref_array :159-188, _project_sample_at :191-207)."""
    size = operator.index(size)
    if size < 0:
        raise ValueError("negative dimensions are not allowed")
    INTRA_PRED_ANGLE[mode - 2]              # IndexError/TypeError exactly as intra.py:142 (D10)
    t, l = _ints1d(top, "top"), _ints1d(left, "left")
    corner = _corner(top_left, "top_left")
    out = np.empty((size, size), np.int16)
    check(_lib.load().nh_intra_angular(ptr(t), t.size, ptr(l), l.size, corner, int(mode), size, ptr(out)),
          "intra_angular_predict")
    return out

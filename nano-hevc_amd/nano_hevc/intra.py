"""Intra prediction -- drop-in for the reference ``nano_hevc.intra`` (intra.py:1-207).

Same names, signatures, output dtypes and exceptions; every sample is computed
by the gfx950 kernels in libnanohevc.so (k_intra_dc / k_intra_planar /
k_intra_angular / k_residual / k_clip in csrc/nh_blocks.hip).  The shim only
converts inputs the way the reference itself does (``.astype(np.int16)``,
``int(...)`` of array elements, ``int(x.sum())``, numpy's int16 element
stores) before handing integer host buffers to the C ABI -- so float and bool
sample arrays give the reference's results and raise its exceptions.
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


_I16 = np.dtype(np.int16)
_I64_SAFE = 1 << 62   # host-converted values beyond this would leave the kernels' int64 arithmetic


def _ints1d(x, what):
    """Integer 1-D view as int64 (lossless for every integer dtype but uint64 > 2^63)."""
    a = np.asarray(x)
    if a.dtype.kind not in "iub":
        raise TypeError(f"{what}: expected an integer sample array, got {a.dtype}")
    return np.ascontiguousarray(a.ravel(), dtype=np.int64)


def _int_kind(x) -> bool:
    return np.asarray(x).dtype.kind in "iub"


def _fit_i64(v: int) -> int:
    """A Python int from the reference's int(...) of a float, handed to the int64
    kernels.  Beyond +-2^62 the reference's int16 store overflows (OverflowError)
    unless other huge values cancel it exactly; that case raises here too."""
    if not -_I64_SAFE < v < _I64_SAFE:
        raise OverflowError(f"Python integer {v} out of bounds for int16")
    return v


def _dc_sum(x, what):
    """intra.py:42 / :61: int(x.sum()).  Integer arrays go to the kernel whole (it
    sums them, D7); for float / complex / object arrays the shim evaluates the
    reference's own int(x.sum()) (numpy's sum in that dtype, then int(): the
    same truncation and the same ValueError / OverflowError / TypeError) and
    hands the kernel that one integer."""
    if type(x) is np.ndarray and x.dtype is _I16:   # the reference's callers: int16 sample rows
        return x.astype(np.int64).ravel()
    a = np.asarray(x)
    if a.dtype.kind in "iub":
        return np.ascontiguousarray(a.ravel(), dtype=np.int64)
    return np.array([_fit_i64(int(a.sum()))], np.int64)


def _corner(v, what):
    if isinstance(v, (float, np.floating)):
        raise TypeError(f"{what}: integer corner sample expected")
    return operator.index(v)


def intra_dc_predict_4x4(top, left):
    """intra.py:37-43: DC = (sum(top) + sum(left) + 4) >> 3, 4x4 int16."""
    t, l = _dc_sum(top, "top"), _dc_sum(left, "left")
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
    t, l = _dc_sum(top, "top"), _dc_sum(left, "left")
    out = np.empty((size, size), np.int16)
    rc = _lib.load().nh_intra_dc(ptr(t), t.size, ptr(l), l.size, size, 0, ptr(out))
    if rc:
        check(rc, "intra_dc_predict")
    return out


def _pair16(x, y):
    """The operands of intra.py:65-72 as two C-contiguous int16 arrays of one
    shape: x.astype(int16), y.astype(int16), broadcast.  Two C-contiguous int16
    arrays of equal shape (the reference's callers) are used as they are."""
    if (type(x) is np.ndarray and type(y) is np.ndarray and x.dtype is _I16 and y.dtype is _I16
            and x.shape == y.shape and x.flags.c_contiguous and y.flags.c_contiguous):
        return x, y
    a = np.asarray(x).astype(np.int16)
    b = np.asarray(y).astype(np.int16)
    if a.shape != b.shape:
        a, b = np.broadcast_arrays(a, b)
    return np.ascontiguousarray(a), np.ascontiguousarray(b)


def residual_block(orig, pred):
    """intra.py:65-67: orig.astype(int16) - pred.astype(int16) (int16 wrap, broadcasting)."""
    a, b = _pair16(orig, pred)
    out = np.empty(a.shape, np.int16)
    rc = _lib.load().nh_residual(ptr(a), ptr(b), a.size, ptr(out))
    if rc:
        check(rc, "residual_block")
    return out


def reconstruct_block(pred, residual):
    """intra.py:70-72: pred.astype(int16) + residual.astype(int16) (int16 wrap)."""
    a, b = _pair16(pred, residual)
    out = np.empty(a.shape, np.int16)
    rc = _lib.load().nh_reconstruct(ptr(a), ptr(b), a.size, ptr(out))
    if rc:
        check(rc, "reconstruct_block")
    return out


def clip_to_pixel_range(block, bit_depth: int = 8):
    """intra.py:75-78: np.clip(block, 0, 2**bd - 1).astype(int16).

    Integer (and bool) blocks go to the kernel as int64.  A float block is first
    put through the reference's own np.clip in its dtype, then every value v is
    handed over as the integer the reference's .astype(np.int16) starts from:
    trunc(v) when |v| < 2^31, else 0 (numpy's float -> int16 cast goes through
    int32: NaN and values outside int32 become 0); the kernel's clamp and int16
    wrap then give the reference's sample exactly."""
    max_val = (1 << bit_depth) - 1
    a = np.asarray(block)
    if a.dtype.kind in "iu":
        np.clip(np.empty(0, a.dtype), 0, max_val)   # numpy's own bound/dtype checks (raises like the reference)
        x = np.ascontiguousarray(a, dtype=np.int64)
    elif a.dtype.kind == "b":
        np.clip(a[:0], 0, max_val)
        x = np.ascontiguousarray(a, dtype=np.int64)
    else:
        c = np.asarray(np.clip(a, 0, max_val))
        if c.dtype.kind not in "f":
            raise TypeError(f"clip_to_pixel_range: cannot cast {c.dtype} samples to int16 like the reference")
        with np.errstate(invalid="ignore"):
            t = np.trunc(c.astype(np.float64))
            ok = np.abs(t) < 2.0 ** 31
        x = np.ascontiguousarray(np.where(ok, t, 0.0).astype(np.int64))
    out = np.empty(a.shape, np.int16)
    check(_lib.load().nh_clip(ptr(x), x.size, min(max_val, 2**63 - 1), ptr(out)), "clip_to_pixel_range")
    return out


def _corner_kind(v, what):
    """(value bits, NH kind) of a planar corner (nanohevc.h nh_intra_planar): a
    numpy integer scalar (or 0-d array) keeps its dtype -- intra.py:109-111 then
    computes in that dtype under NEP 50, which the kernel reproduces (wrap,
    OverflowError on converting Python ints, float64 promotion); np.bool_ acts
    as int64 there; anything else is a Python int (exact math)."""
    if isinstance(v, (float, np.floating)):
        return 0, 1                                   # NH_NP_FLOAT: TypeError at the >> (intra.py:111)
    dt = v.dtype if isinstance(v, (np.generic, np.ndarray)) and np.ndim(v) == 0 else None
    if dt is not None and dt.kind == "b":
        return int(v), -64
    if dt is not None and dt.kind in "iu":
        bits = dt.itemsize * 8
        val = int(v)
        if dt.kind == "u":
            return (val - (1 << 64) if val >= 1 << 63 else val), bits
        return val, -bits
    return _corner(v, what), 0


def _planar_float_refs(top, left, size, corners):
    """intra.py:107-111 for non-integer top/left: the loop reads int(left[y]) and
    int(top[x]), in the order left[0], top[0..size-1], left[1], left[2], ... (a
    repeated read raises nothing new); any float corner makes the first (h + v +
    size) >> k raise TypeError right after left[0] and top[0] were read (the
    kernel raises it there, after any error of the other corner's arithmetic).  The
    elements are converted here exactly as int() does (truncation; ValueError for
    NaN, OverflowError for inf) up to the first IndexError, which the kernel
    raises in the same place; the kernel then runs on those integers."""
    ta, la = np.asarray(top), np.asarray(left)
    tv = np.zeros(ta.size, np.int64)
    lv = np.zeros(la.size, np.int64)
    fl_t, fl_l = ta.ravel(), la.ravel()

    def conv(arr, flat, vals, i):
        if i >= flat.size:
            return False                                       # IndexError: the kernel's (same position)
        vals[i] = _fit_i64(int(arr[i]) if arr.ndim == 1 else int(flat[i]))
        return True

    if size <= 0:
        return tv, lv
    if not conv(la, fl_l, lv, 0):
        return tv, lv
    for x in range(size):
        if not conv(ta, fl_t, tv, x):
            return tv, lv
        if x == 0 and any(isinstance(c, (float, np.floating)) for c in corners):
            return tv, lv                                      # the kernel raises TypeError at (0, 0)
    for y in range(1, size):
        if not conv(la, fl_l, lv, y):
            break
    return tv, lv


def intra_planar_predict(top, left, top_right, bottom_left, size):
    """intra.py:81-113: pred[y,x] = ((N-1-x)left[y] + (x+1)tr + (N-1-y)top[x] + (y+1)bl + N) >> (log2N+1)."""
    size = operator.index(size)
    if size < 0:
        raise ValueError("negative dimensions are not allowed")
    log2_size = int(np.log2(size))          # the reference's own parameter computation
    if _int_kind(top) and _int_kind(left):
        t, l = _ints1d(top, "top"), _ints1d(left, "left")
    else:
        t, l = _planar_float_refs(top, left, size, (top_right, bottom_left))
    # a float corner makes the first (h + v + size) >> k raise TypeError (intra.py:111)
    # right after left[0] / top[0] were read; the kernel raises it in that place
    tr, ktr = _corner_kind(top_right, "top_right")
    bl, kbl = _corner_kind(bottom_left, "bottom_left")
    out = np.empty((size, size), np.int16)
    check(_lib.load().nh_intra_planar(ptr(t), t.size, ptr(l), l.size, tr, ktr, bl, kbl, size, log2_size, ptr(out)),
          "intra_planar_predict")
    return out


def _store16(v):
    """The int16 element store of _build_ref_array (intra.py:173, :176, :178,
    :186) for one value: numpy's own setitem (int() of a float: truncation,
    ValueError for NaN, OverflowError outside int16)."""
    z = np.zeros(1, np.int16)
    z[0] = v
    return int(z[0])


def _angular_float_refs(top, left, top_left, mode, size):
    """intra.py:159-188 for non-integer top/left or a float corner: every element
    _build_ref_array stores is converted by numpy's own int16 setitem, in the
    reference's order (corner, primary[1..2N] with replicate-last, then the
    negative-angle projections of secondary), so the first error raised is the
    reference's; the kernel then builds the reference array from those integers
    (unread elements are 0)."""
    angle = INTRA_PRED_ANGLE[mode - 2]
    vert = mode >= 18
    ta, la = np.asarray(top), np.asarray(left)
    pa, sa = (ta, la) if vert else (la, ta)
    pv, sv = np.zeros(pa.size, np.int64), np.zeros(sa.size, np.int64)
    corner = _store16(top_left)
    for i in range(1, 2 * size + 1):
        k = i if i < len(pa) else -1
        if k == -1 and len(pa) == 0:
            raise IndexError("index -1 is out of bounds for axis 0 with size 0")
        pv[k] = _store16(pa[k])
    if angle < 0:
        inv = INV_ANGLE[angle]
        for i in range(-1, ((size * angle) >> 5) - 1, -1):
            proj = ((i + 1) * inv + 128) >> 8
            if proj < len(sa):
                sv[proj] = _store16(sa[proj])
    t, l = (pv, sv) if vert else (sv, pv)
    return t, l, corner


def intra_angular_predict(top, left, top_left, mode, size):
    """intra.py:116-156 (+ _build_ref_array :159-188, _project_sample_at :191-207)."""
    size = operator.index(size)
    if size < 0:
        raise ValueError("negative dimensions are not allowed")
    INTRA_PRED_ANGLE[mode - 2]              # IndexError/TypeError exactly as intra.py:142 (D10)
    if _int_kind(top) and _int_kind(left) and not isinstance(top_left, (float, np.floating)):
        t, l = _ints1d(top, "top"), _ints1d(left, "left")
        corner = _corner(top_left, "top_left")
    else:
        t, l, corner = _angular_float_refs(top, left, top_left, mode, size)
    out = np.empty((size, size), np.int16)
    check(_lib.load().nh_intra_angular(ptr(t), t.size, ptr(l), l.size, corner, int(mode), size, ptr(out)),
          "intra_angular_predict")
    return out

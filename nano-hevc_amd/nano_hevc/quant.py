"""Quantization -- drop-in for the reference ``nano_hevc.quant`` (quant.py:1-178).

Parameters (qp clamp, qp/6, qp%6, shift, offset) are computed with the
reference's own Python expressions; the per-coefficient arithmetic runs on the
gfx950 kernels (k_quant_i64 / k_dequant_i64 / k_count_nonzero /
k_estimate_bits in csrc/nh_blocks.hip).
"""
from __future__ import annotations

import numpy as np

from . import _lib
from ._lib import check, ptr

# quant.py:21-22 (spec Table 8-10)
QUANT_SCALE = [26214, 23302, 20560, 18396, 16384, 14564]
DEQUANT_SCALE = [40, 45, 51, 57, 64, 72]


def get_qp_params(qp: int) -> tuple[int, int]:
    """quant.py:25-38."""
    qp = max(0, min(51, qp))
    return qp // 6, qp % 6


def _abs_bits(dt) -> int:
    """Width in which np.abs wraps for this integer dtype (quant.py:77); 0 for
    the dtypes quantize() hands to nh_quantize_abs instead."""
    dt = np.dtype(dt)
    if dt.kind == "i":
        return dt.itemsize * 8
    if dt.kind == "u" and dt.itemsize < 8:
        return 64
    return 0


_AB_INT32 = np.dtype(np.int32)


def _log2_size(size) -> int:
    """int(np.log2(size)) (quant.py:72); exact bit arithmetic for the power-of-two
    Python ints the reference's callers pass, numpy's own expression otherwise."""
    if type(size) is int and 0 < size < (1 << 52) and not size & (size - 1):
        return size.bit_length() - 1
    return int(np.log2(size))


def quantize(coeff, qp: int, size: int, is_intra: bool = True) -> np.ndarray:
    """quant.py:41-79: level = sign(c) * ((|c|*MF + offset) >> shift), int32."""
    qp_per, qp_rem = get_qp_params(qp)
    mf = QUANT_SCALE[qp_rem]                                  # noqa: F841 (same lookup/errors)
    log2_size = _log2_size(size)
    shift = 14 + qp_per + log2_size
    offset = (1 << shift) // 3 if is_intra else (1 << shift) // 6   # noqa: F841
    c = coeff if type(coeff) is np.ndarray else np.asarray(coeff)
    ab = 32 if c.dtype is _AB_INT32 else _abs_bits(c.dtype)
    if ab:
        x = c.astype(np.int64, order="C")
        out = np.empty(c.shape, np.int32)
        rc = _lib.load().nh_quantize(ptr(x), x.size, int(qp_per * 6 + qp_rem), log2_size, 1 if is_intra else 0, ab, ptr(out))
        if rc:
            check(rc, "quantize")
        return out
    # float (and uint64 / bool / other) coefficients: the reference's own host
    # expressions around the kernel -- np.sign (raises for bool, like quant.py:76),
    # np.abs(...).astype(np.int64), the level on the GPU, then
    # (sign * level).astype(np.int32) in float64 (quant.py:79)
    sign = np.sign(c)
    abs_coeff = np.ascontiguousarray(np.abs(c).astype(np.int64))
    level = np.empty(abs_coeff.shape, np.int64)
    check(_lib.load().nh_quantize_abs(ptr(abs_coeff), abs_coeff.size, int(qp_per * 6 + qp_rem), log2_size,
                                      int(bool(is_intra)), ptr(level)), "quantize")
    return (sign * level).astype(np.int32)


def dequantize(level, qp: int, size: int) -> np.ndarray:
    """quant.py:82-123 (size unused, D4)."""
    qp_per, qp_rem = get_qp_params(qp)
    DEQUANT_SCALE[qp_rem]
    x = np.asarray(level).astype(np.int64, order="C")   # quant.py:113 cast
    out = np.empty(x.shape, np.int32)
    rc = _lib.load().nh_dequantize(ptr(x), x.size, int(qp_per * 6 + qp_rem), ptr(out))
    if rc:
        check(rc, "dequantize")
    return out


def quantize_block(coeff, qp: int, is_intra: bool = True) -> np.ndarray:
    """quant.py:126-137."""
    size = coeff.shape[0]
    return quantize(coeff, qp, size, is_intra)


def dequantize_block(level, qp: int) -> np.ndarray:
    """quant.py:140-150."""
    size = level.shape[0]
    return dequantize(level, qp, size)


# estimate_bits dtype codes (NH_EB_* in include/nanohevc.h)
_EB_CODE = {("b", 1): 1, ("i", 1): 8, ("i", 2): 16, ("i", 4): 32, ("i", 8): 64,
            ("u", 1): 108, ("u", 2): 116, ("u", 4): 132, ("u", 8): 164,
            ("f", 2): 216, ("f", 4): 232, ("f", 8): 264}


def estimate_bits(level) -> int:
    """quant.py:153-168: int(np.sum(np.log2(|l|+1) + (|l|>0)*2)).

    numpy's dtype rules per level dtype are evaluated on the device (abs and +1
    in the dtype, log2 in float16 / float32 / float64 as numpy picks it, the
    float64 sum in numpy's pairwise order over the term array's memory order,
    which is the input's 'K' order).  Complex levels go through the reference's
    own np.abs on the host first; other dtypes raise TypeError like np.log2."""
    a = np.asarray(level)
    kind = a.dtype.kind
    if kind == "c":
        a = np.abs(a)                       # quant.py:166, complex -> float magnitude
        kind = "f"
    if kind not in "biuf":
        raise TypeError(f"ufunc 'log2' not supported for the input types (dtype {a.dtype})")
    code = _EB_CODE.get((kind, a.dtype.itemsize))
    if code is None:   # longdouble (and complex256's magnitude): numpy computes in 80-bit extended
        raise NotImplementedError(f"estimate_bits: {a.dtype} levels (extended precision) are not supported")
    flat = np.ravel(a, order="K")
    if kind == "f":
        x = np.ascontiguousarray(flat, dtype=np.float64).view(np.int64)   # exact widening, float64 bits
    elif kind == "u":
        x = np.ascontiguousarray(flat, dtype=np.uint64).view(np.int64)
    else:
        x = np.ascontiguousarray(flat, dtype=np.int64)
    bits = np.zeros(1, np.float64)
    check(_lib.load().nh_estimate_bits(ptr(x), x.size, code, ptr(bits)), "estimate_bits")
    return int(bits[0])


def _nonzero_mask(a):
    """np.count_nonzero's notion of nonzero as an integer/bool array: the value
    itself for integers and bools; != 0 for floats and complex (NaN counts);
    truthiness for objects, non-empty for strings, != 0 for the datetime kinds
    (NaT counts)."""
    k = a.dtype.kind
    if k in "iub":
        return a
    if k in "fc":
        return a != 0
    if k == "O":
        return a.astype(bool)
    if k in "US":
        return np.char.str_len(a) != 0
    if k in "mM":
        return a.view(np.int64) != 0
    raise TypeError(f"count_nonzero: unsupported dtype {a.dtype}")


def _count(mask) -> int:
    x = np.ascontiguousarray(mask, dtype=np.int64)
    cnt = np.zeros(1, np.int64)
    check(_lib.load().nh_count_nonzero(ptr(x), x.size, ptr(cnt)), "count_nonzero")
    return int(cnt[0])


def count_nonzero(level) -> int:
    """quant.py:171-173: int(np.count_nonzero(level)), the count on the GPU."""
    return _count(_nonzero_mask(np.asarray(level)))


def is_all_zero(level) -> bool:
    """quant.py:176-178: np.all(level == 0) (returns numpy.bool like np.all).
    Numeric levels: no element is nonzero (count on the GPU); other dtypes
    compare with the reference's own level == 0 first."""
    a = np.asarray(level)
    if a.dtype.kind in "iubfc":
        return np.bool_(_count(_nonzero_mask(a)) == 0)
    eq = np.asarray(a == 0)
    return np.bool_(_count(~eq.astype(bool)) == 0)

"""Quality metrics -- drop-in for the reference ``nano_hevc.metrics`` (metrics.py:7-48).

The array reductions run on the GPU (k_sum_sq_diff / k_sad_i32 / k_satd_4x4 /
k_residual_energy in csrc/nh_blocks.hip); only the final scalar formulas
(mean, log10) are evaluated on the host, with the reference's expressions.
``mse``/``psnr``: integer samples of <= 16 bits take an exact int64 SSE (the
squares are integers, so numpy's float64 sum is exact below 2**53, checked);
every other dtype (float, wider ints) is cast to float64 by the shim as the
reference does and summed on the GPU in numpy's pairwise order, bit-identical.
"""
from __future__ import annotations

import numpy as np

from . import _lib
from ._lib import check, ptr


def _small_int(a) -> bool:
    return a.dtype.kind in "iub" and a.dtype.itemsize <= 2


def _sum_sq_diff_int(a, b):
    """Exact int64 SSE of <= 16-bit samples: every partial sum is an integer below
    2^53 (checked), so numpy's float64 sum of the squares is exact in any order."""
    a = np.ascontiguousarray(a, dtype=np.int64)
    b = np.ascontiguousarray(b, dtype=np.int64)
    out = np.zeros(1, np.int64)
    check(_lib.load().nh_sum_sq_diff(ptr(a), ptr(b), a.size, ptr(out)), "mse")
    return int(out[0])


def _sum_sq_diff_f64(a, b) -> float:
    """metrics.py:9-10 for any other dtype: the reference's own host expression
    diff = a.astype(np.float64) - b.astype(np.float64) (its result is a fresh
    array laid out in the operands' 'K' order, broadcast views included), then
    the sum of diff ** 2 on the GPU in numpy's pairwise order over that array's
    memory order (np.mean reduces a contiguous array as one 1-D run)."""
    d = np.asarray(a).astype(np.float64) - np.asarray(b).astype(np.float64)
    x = np.ascontiguousarray(np.ravel(d, order="K"))
    y = np.zeros_like(x)                 # (d - 0) ** 2 == d ** 2 exactly
    out = np.zeros(1, np.float64)
    check(_lib.load().nh_sum_sq_diff_f64(ptr(x), ptr(y), x.size, ptr(out)), "mse")
    return float(out[0])


def mse(original, reconstructed) -> float:
    """metrics.py:7-10: mean((orig - recon)^2) in float64."""
    a0, b0 = np.asarray(original), np.asarray(reconstructed)
    a, b = np.broadcast_arrays(a0, b0)
    n = a.size
    if _small_int(a) and _small_int(b):
        s = _sum_sq_diff_int(a, b)
        if s < 2**53:
            return float(np.float64(s) / np.float64(n))
    return float(np.float64(_sum_sq_diff_f64(a0, b0)) / np.float64(n))


def psnr(original, reconstructed, peak: int = 255) -> float:
    """metrics.py:13-21."""
    err = mse(original, reconstructed)
    if err == 0:
        return float("inf")
    return 10 * np.log10(peak ** 2 / err)


def sad(a, b) -> int:
    """metrics.py:24-26: sum |int32(a) - int32(b)|."""
    x = np.asarray(a).astype(np.int32)
    y = np.asarray(b).astype(np.int32)
    x, y = np.broadcast_arrays(x, y)
    x, y = np.ascontiguousarray(x), np.ascontiguousarray(y)
    out = np.zeros(1, np.int64)
    check(_lib.load().nh_sad(ptr(x), ptr(y), x.size, ptr(out)), "sad")
    return int(out[0])


def satd_4x4(a, b) -> int:
    """metrics.py:29-43: sum |H . (a-b) . H^T| over a 4x4 block."""
    x, y = np.broadcast_arrays(np.asarray(a).astype(np.int32), np.asarray(b).astype(np.int32))
    if x.size != 16:       # the reference's .reshape(4, 4) error
        raise ValueError(f"cannot reshape array of size {x.size} into shape (4,4)")
    x = np.ascontiguousarray(x.reshape(4, 4))
    y = np.ascontiguousarray(y.reshape(4, 4))
    out = np.zeros(1, np.int64)
    check(_lib.load().nh_satd_4x4(ptr(x), ptr(y), ptr(out)), "satd_4x4")
    return int(out[0])


def residual_energy(residual) -> int:
    """metrics.py:46-48: sum(int64(r)^2)."""
    r = np.ascontiguousarray(np.asarray(residual).astype(np.int64))
    out = np.zeros(1, np.int64)
    check(_lib.load().nh_residual_energy(ptr(r), r.size, ptr(out)), "residual_energy")
    return int(out[0])

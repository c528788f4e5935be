"""Quality metrics -- drop-in for the reference ``nano_hevc.metrics`` (metrics.py:7-48).

The array reductions run on the GPU (k_sum_sq_diff / k_sad_i32 / k_satd_4x4 /
k_residual_energy in csrc/nh_blocks.hip); only the final scalar formulas
(mean, log10) are evaluated on the host, with the reference's expressions.
``mse``/``psnr`` are exact for integer samples of <= 16 bits: the squared
differences are integers, so numpy's float64 sum is exact whenever the total
is below 2**53 (checked; larger totals raise instead of rounding differently).
"""
from __future__ import annotations

import numpy as np

from . import _lib
from ._lib import check, ptr


def _samples(x, what):
    a = np.asarray(x)
    if a.dtype.kind not in "iub" or a.dtype.itemsize > 2:
        raise NotImplementedError(f"{what}: integer samples of <= 16 bits only (got {a.dtype})")
    return a


def _sum_sq_diff(original, reconstructed) -> int:
    a = np.ascontiguousarray(_samples(original, "mse"), dtype=np.int64)
    b = np.ascontiguousarray(_samples(reconstructed, "mse"), dtype=np.int64)
    a, b = np.broadcast_arrays(a, b)
    a, b = np.ascontiguousarray(a), np.ascontiguousarray(b)
    out = np.zeros(1, np.int64)
    check(_lib.load().nh_sum_sq_diff(ptr(a), ptr(b), a.size, ptr(out)), "mse")
    s = int(out[0])
    if s >= 2**53:
        raise NotImplementedError("mse: float64 sum would round (total >= 2**53)")
    return s, a.size


def mse(original, reconstructed) -> float:
    """metrics.py:7-10: mean((orig - recon)^2) in float64."""
    s, n = _sum_sq_diff(original, reconstructed)
    return float(np.float64(s) / np.float64(n))


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

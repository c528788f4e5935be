"""Integer DST/DCT -- drop-in for the reference ``nano_hevc.transform`` (transform.py:1-278).

forward_transform / inverse_transform keep the reference's exact integer
semantics (int32 ring, same shift log2N+5 in both passes, column pass first:
SURVEY.md §0.1 D1/D2) and run on the gfx950 partial-butterfly kernels
(k_transform in csrc/nh_blocks.hip).  The matrices are plain data here, as in
the reference (tests use them directly).
"""
from __future__ import annotations

import numpy as np

from . import _lib
from ._lib import check, ptr


def _dct32() -> np.ndarray:
    """DCT32 (transform.py:65-135), generated from the 33 distinct basis
    magnitudes: DCT32[k][n] = +-TAB[fold((2n+1)k mod 128)]."""
    tab = [64, 90, 90, 90, 89, 88, 87, 85, 83, 82, 80, 78, 75, 73, 70, 67,
           64, 61, 57, 54, 50, 46, 43, 38, 36, 31, 25, 22, 18, 13, 9, 4, 0]
    m = np.zeros((32, 32), np.int32)
    for k in range(32):
        for n in range(32):
            if k == 0:
                m[k, n] = 64
                continue
            a = (2 * n + 1) * k % 128
            m[k, n] = tab[a] if a <= 32 else -tab[64 - a] if a <= 64 else -tab[a - 64] if a <= 96 else tab[128 - a]
    return m


DCT32 = _dct32()
DCT16 = np.ascontiguousarray(DCT32[::2, :16])     # even rows of DCT(2N) = DCT(N)
DCT8 = np.ascontiguousarray(DCT32[::4, :8])
DCT4 = np.ascontiguousarray(DCT32[::8, :4])
DST4 = np.array([[29, 55, 74, 84], [74, 74, 0, -74], [84, -29, -74, 55], [55, -84, 74, -29]], dtype=np.int32)


def _get_transform_matrix(size: int, use_dst: bool = False) -> np.ndarray:
    """transform.py:138-151."""
    if use_dst and size == 4:
        return DST4
    if size == 4:
        return DCT4
    elif size == 8:
        return DCT8
    elif size == 16:
        return DCT16
    elif size == 32:
        return DCT32
    raise ValueError(f"Unsupported transform size: {size}")


def _prep(x):
    a = np.asarray(x)
    size = a.shape[0]
    _get_transform_matrix(size)                     # ValueError for unsupported sizes
    if a.ndim == 1:
        raise IndexError("too many indices for array: array is 1-dimensional, but 2 were indexed")
    if a.ndim > 2:
        # transform.py:180-185 on an N-D block: block[k, j] is an array over the
        # trailing axes, and the int32 element store temp[i, j] = ... takes it
        # only when it holds exactly one value (numpy's size-1 conversion)
        if a.shape[1] == 0:
            raise IndexError("index 0 is out of bounds for axis 1 with size 0")
        if int(np.prod(a.shape[2:])) != 1:
            raise ValueError("setting an array element with a sequence.")
        a = a.reshape(a.shape[:2])
    if a.shape[1] < size:
        raise IndexError(f"index {a.shape[1]} is out of bounds for axis 1 with size {a.shape[1]}")
    blk = np.ascontiguousarray(a.astype(np.int32)[:size, :size])   # transform.py:176 cast (wraps)
    return blk, size


def forward_transform(residual, use_dst: bool = False) -> np.ndarray:
    """transform.py:154-196: coeff = ((T.X + rnd) >> s) . T^T, rounded, int32."""
    blk, size = _prep(residual)
    out = np.empty((size, size), np.int32)
    check(_lib.load().nh_forward_transform(ptr(blk), size, int(bool(use_dst)), ptr(out)), "forward_transform")
    return out


def inverse_transform(coeff, use_dst: bool = False) -> np.ndarray:
    """transform.py:199-238: res = ((T^T.C + rnd) >> s) . T, rounded, int32."""
    blk, size = _prep(coeff)
    out = np.empty((size, size), np.int32)
    check(_lib.load().nh_inverse_transform(ptr(blk), size, int(bool(use_dst)), ptr(out)), "inverse_transform")
    return out


def forward_transform_4x4(residual, use_dst: bool = False):
    """transform.py:241-243."""
    return forward_transform(residual, use_dst)


def inverse_transform_4x4(coeff, use_dst: bool = False):
    """transform.py:246-248."""
    return inverse_transform(coeff, use_dst)


def forward_transform_8x8(residual):
    return forward_transform(residual, use_dst=False)


def inverse_transform_8x8(coeff):
    return inverse_transform(coeff, use_dst=False)


def forward_transform_16x16(residual):
    return forward_transform(residual, use_dst=False)


def inverse_transform_16x16(coeff):
    return inverse_transform(coeff, use_dst=False)


def forward_transform_32x32(residual):
    return forward_transform(residual, use_dst=False)


def inverse_transform_32x32(coeff):
    return inverse_transform(coeff, use_dst=False)

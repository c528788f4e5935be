"""Host-side frame containers (reference frame.py:16-308).

Out of the accelerated scope (frame I/O is §8f-3, "next"): these
are plain numpy-backed holders with the reference's API (Plane, Frame,
PackedFrame, FrameBufferPool) so callers importing them from ``nano_hevc`` keep
working.  They do no pixel arithmetic; the device path takes planes through
``nano_hevc.gpu`` (contiguous int16 buffers described by nh_plane_set).
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np


class Plane:
    """One colour plane; ``data`` is an (H, W) C-contiguous array (frame.py:16-54)."""
    __slots__ = ("data",)

    def __init__(self, data: np.ndarray):
        self.data = data

    height = property(lambda self: self.data.shape[0])
    width = property(lambda self: self.data.shape[1])
    shape = property(lambda self: self.data.shape[:2])

    @classmethod
    def zeros(cls, height: int, width: int, dtype=np.int16) -> "Plane":
        return cls(np.zeros((height, width), dtype=dtype, order="C"))

    @classmethod
    def from_buffer(cls, buffer: bytes, height: int, width: int, dtype=np.uint8) -> "Plane":
        return cls(np.ascontiguousarray(np.frombuffer(buffer, dtype=dtype).reshape(height, width)))

    def __repr__(self):
        return f"Plane(shape={self.shape}, dtype={self.data.dtype})"


def _yuv420_sizes(height: int, width: int):
    ys = height * width
    return ys, (height // 2) * (width // 2), height // 2, width // 2


class Frame:
    """YUV420p frame of three Planes (frame.py:57-118)."""
    __slots__ = ("y", "u", "v")

    def __init__(self, y: Plane, u: Plane, v: Plane):
        self.y, self.u, self.v = y, u, v

    height = property(lambda self: self.y.height)
    width = property(lambda self: self.y.width)

    @classmethod
    def zeros(cls, height: int, width: int, dtype=np.int16) -> "Frame":
        return cls(Plane.zeros(height, width, dtype), Plane.zeros(height // 2, width // 2, dtype),
                   Plane.zeros(height // 2, width // 2, dtype))

    @classmethod
    def from_yuv420p(cls, buffer: bytes, height: int, width: int) -> "Frame":
        ys, cs, ch, cw = _yuv420_sizes(height, width)
        return cls(Plane.from_buffer(buffer[:ys], height, width),
                   Plane.from_buffer(buffer[ys:ys + cs], ch, cw),
                   Plane.from_buffer(buffer[ys + cs:ys + 2 * cs], ch, cw))

    def to_yuv420p(self) -> bytes:
        return b"".join(p.data.astype(np.uint8).tobytes() for p in (self.y, self.u, self.v))

    def __repr__(self):
        return f"Frame(height={self.height}, width={self.width})"


class PackedFrame:
    """Y, U, V as views of one contiguous buffer [Y][U][V] (frame.py:121-189).
    This is also the device layout ``nano_hevc.gpu`` streams (one nh_plane_set
    for Y, one for U+V)."""
    __slots__ = ("_buffer", "y", "u", "v", "height", "width", "_y_size", "_uv_size")

    def __init__(self, height: int, width: int, dtype=np.int16):
        self.height, self.width = height, width
        ys, cs, ch, cw = _yuv420_sizes(height, width)
        self._y_size, self._uv_size = ys, cs
        self._buffer = np.zeros(ys + 2 * cs, dtype=dtype, order="C")
        self.y = self._buffer[:ys].reshape(height, width)
        self.u = self._buffer[ys:ys + cs].reshape(ch, cw)
        self.v = self._buffer[ys + cs:].reshape(ch, cw)

    @classmethod
    def from_yuv420p(cls, buffer: bytes, height: int, width: int) -> "PackedFrame":
        f = cls(height, width, dtype=np.uint8)
        np.copyto(f._buffer, np.frombuffer(buffer, dtype=np.uint8)[:f._buffer.size])
        return f

    @classmethod
    def from_frame(cls, frame: Frame) -> "PackedFrame":
        f = cls(frame.height, frame.width, dtype=frame.y.data.dtype)
        for dst, src in ((f.y, frame.y), (f.u, frame.u), (f.v, frame.v)):
            np.copyto(dst, src.data)
        return f

    def to_yuv420p(self) -> bytes:
        return self._buffer.astype(np.uint8).tobytes()

    def to_frame(self) -> Frame:
        return Frame(Plane(self.y.copy()), Plane(self.u.copy()), Plane(self.v.copy()))

    def clear(self) -> None:
        self._buffer.fill(0)

    def __repr__(self):
        return f"PackedFrame(height={self.height}, width={self.width}, dtype={self._buffer.dtype})"


class FrameBufferPool:
    """Fixed pool of reusable frames with acquire/release (frame.py:192-308)."""
    __slots__ = ("_pool", "_available", "_in_use", "height", "width", "dtype")

    def __init__(self, height: int, width: int, pool_size: int = 4, dtype=np.int16, use_packed: bool = True):
        self.height, self.width, self.dtype = height, width, dtype
        make = (lambda: PackedFrame(height, width, dtype=dtype)) if use_packed else \
            (lambda: Frame.zeros(height, width, dtype=dtype))
        self._pool: List = [make() for _ in range(pool_size)]
        self._available: List[int] = list(range(pool_size))
        self._in_use: set = set()

    def acquire(self, clear: bool = True) -> Tuple[int, object]:
        if not self._available:
            raise RuntimeError(f"No buffers available in pool. In use: {len(self._in_use)}, "
                               f"Total: {len(self._pool)}")
        idx = self._available.pop()
        self._in_use.add(idx)
        fr = self._pool[idx]
        if clear:
            if isinstance(fr, PackedFrame):
                fr.clear()
            else:
                for p in (fr.y, fr.u, fr.v):
                    p.data.fill(0)
        return idx, fr

    def release(self, idx: int) -> None:
        if idx not in self._in_use:
            raise ValueError(f"Buffer {idx} is not currently in use")
        self._in_use.remove(idx)
        self._available.append(idx)

    available_count = property(lambda self: len(self._available))
    in_use_count = property(lambda self: len(self._in_use))
    pool_size = property(lambda self: len(self._pool))

    def __repr__(self):
        return (f"FrameBufferPool(height={self.height}, width={self.width}, "
                f"available={self.available_count}/{self.pool_size})")

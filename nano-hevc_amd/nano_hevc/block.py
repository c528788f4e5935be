"""Block views and raster iteration (reference block.py:14-74).

These define the neighbour rules the frame-level device drivers reproduce
(SURVEY.md §8a row A14): 128 outside the plane, neighbours read from the
SOURCE plane (open loop), numpy-slice truncation at the right/bottom edge, and
partial edge blocks skipped.  Host-side views only (no arithmetic).
"""
from __future__ import annotations

from typing import Iterator, Optional, Tuple

import numpy as np

from .frame import Plane

BORDER = 128   # block.py:41-55 fill value outside the plane


class BlockView:
    """A size x size window of a Plane at (x, y), no copy (block.py:14-65)."""
    __slots__ = ("plane", "x", "y", "size")

    def __init__(self, plane: Plane, x: int, y: int, size: int):
        self.plane, self.x, self.y, self.size = plane, x, y, size

    @property
    def pixels(self) -> np.ndarray:
        return self.plane.data[self.y:self.y + self.size, self.x:self.x + self.size]

    @property
    def shape(self) -> Tuple[int, int]:
        return (self.size, self.size)

    def get_top_neighbors(self, count: Optional[int] = None) -> np.ndarray:
        n = self.size if count is None else count
        if self.y == 0:
            return np.full(n, BORDER, dtype=self.plane.data.dtype)
        return self.plane.data[self.y - 1, self.x:self.x + n].copy()

    def get_left_neighbors(self, count: Optional[int] = None) -> np.ndarray:
        n = self.size if count is None else count
        if self.x == 0:
            return np.full(n, BORDER, dtype=self.plane.data.dtype)
        return self.plane.data[self.y:self.y + n, self.x - 1].copy()

    def get_top_left_neighbor(self) -> int:
        if self.y == 0 or self.x == 0:
            return BORDER
        return int(self.plane.data[self.y - 1, self.x - 1])

    def copy_pixels(self) -> np.ndarray:
        return self.pixels.copy()

    def write_pixels(self, data: np.ndarray) -> None:
        self.plane.data[self.y:self.y + self.size, self.x:self.x + self.size] = data

    def __repr__(self):
        return f"BlockView(x={self.x}, y={self.y}, size={self.size})"


def iterate_blocks(plane: Plane, block_size: int) -> Iterator[BlockView]:
    """Raster order over full blocks only (partial right/bottom blocks skipped)."""
    for y in range(0, plane.height - block_size + 1, block_size):
        for x in range(0, plane.width - block_size + 1, block_size):
            yield BlockView(plane, x, y, block_size)

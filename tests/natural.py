"""Test helper: "natural" residual planes."""
import numpy as np


def natural_residual(src):
    """source minus the open-loop DC prediction of every
    full 8x8 block (intra.py:46-62 with block.py:38-50 neighbours: 128 at the
    border); samples outside full blocks are left as the source."""
    h, w = src.shape
    s = src.astype(np.int64)
    hb, wb = h // 8, w // 8
    pad_top = np.vstack([np.full((1, w), 128), s[:-1]])          # row above each row
    pad_left = np.hstack([np.full((h, 1), 128), s[:, :-1]])      # column left of each column
    top = pad_top[0:hb * 8:8, :wb * 8].reshape(hb, wb, 8).sum(2)
    left = pad_left[:hb * 8, 0:wb * 8:8].reshape(hb, 8, wb).sum(1)
    dc = (top + left + 8) // 16
    res = src.astype(np.int16).copy()
    res[:hb * 8, :wb * 8] -= np.repeat(np.repeat(dc, 8, 0), 8, 1).astype(np.int16)
    return res

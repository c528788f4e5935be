"""Seeded inputs of the full-size reference fixtures (tests/golden/fullsize.json):
numpy only, shared by make_fullsize.py (here) and the GPU test (on the box)."""
import numpy as np

CFG3_QP, CLOSED_QP, CFG4_QP, CFG4_SEED, CFG5_QP = 32, 27, 30, 4242, 4
CFG2_QP = 32


def natural(h, w, seed):
    """Gradient + texture + noise, 8-bit samples as int16 (the reference's Plane dtype)."""
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w]
    base = 90 + (xx // 3 + yy // 2) % 120 + ((xx // 61 + yy // 37) % 3) * 11
    return np.clip(base + rng.integers(-12, 13, (h, w)), 0, 255).astype(np.int16)


def yuv420(w, h, seed):
    return [natural(h, w, seed), natural(h // 2, w // 2, seed + 1), natural(h // 2, w // 2, seed + 2)]


def cfg3_frame():
    return yuv420(1920, 1080, 3030)


def cfg4_frame():
    return yuv420(3840, 2160, 4040)


def cfg5_plane():
    return natural(4320, 7680, 5050)


def cfg5_chroma():
    """The U and V planes of the 8K YUV420 frame whose luma is cfg5_plane()."""
    return yuv420(7680, 4320, 5050)[1:]


def cfg2_frame():
    """One 4K YUV420 frame of int16 residuals U[-255, 255] (the bench's sample
    distribution, bench.py), as [Y, U, V] planes."""
    rng = np.random.default_rng(2020)
    w, h = 3840, 2160
    return [rng.integers(-255, 256, size=(ph, pw)).astype(np.int16)
            for ph, pw in ((h, w), (h // 2, w // 2), (h // 2, w // 2))]

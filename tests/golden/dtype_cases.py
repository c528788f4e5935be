"""Non-integer inputs to the drop-in functions: float, bool,
float32/float16 sample arrays, float corners, NaN / inf / out-of-range values.

cases() rebuilds the same seeded calls every time; make_golden.py --only
dtypes.npz records the REFERENCE's result (an array / scalar, or the name of
the exception it raised) per case, and tests/test_dtypes_gpu.py runs the same
calls on the MI355X drop-in and compares bit for bit.  Each case is
(name, function name, args tuple, kwargs dict).
"""
from __future__ import annotations

import numpy as np


def cases():
    rng = np.random.default_rng(90210)
    out = []

    def add(fn, *args, **kw):
        out.append((f"{len(out):03d}_{fn}", fn, args, kw))

    nan, inf = float("nan"), float("inf")
    # ---- intra_dc_predict / _4x4 (intra.py:42, :61: int(x.sum()))
    add("intra_dc_predict", np.array([100.5, 98, 100, 101]), np.array([103, 102, 101, 99.]), 4)
    add("intra_dc_predict_4x4", np.array([100.5, 98, 100, 101]), np.array([103, 102, 101, 99.]))
    for n in (4, 8, 16, 32):
        t = rng.uniform(-20, 300, n)
        l = rng.uniform(-20, 300, n)
        add("intra_dc_predict", t, l, n)
        add("intra_dc_predict", t.astype(np.float32), l.astype(np.float32), n)
        add("intra_dc_predict", t.astype(np.float16), l.astype(np.int16), n)
        add("intra_dc_predict", rng.random(n) > 0.5, rng.random(n) > 0.3, n)
    add("intra_dc_predict", np.array([-3.9, -0.5, 2.2, 1.0]), np.array([-7.5, 0.0, 0.0, 0.0]), 4)
    add("intra_dc_predict", np.array([nan, 1.0, 2.0, 3.0]), np.array([1.0, 2.0, 3.0, 4.0]), 4)
    add("intra_dc_predict", np.array([inf, 1.0, 2.0, 3.0]), np.array([1.0, 2.0, 3.0, 4.0]), 4)
    add("intra_dc_predict", np.array([1e6, 1.0, 2.0, 3.0]), np.array([1.0, 2.0, 3.0, 4.0]), 4)
    add("intra_dc_predict_4x4", np.array([True, True, False, True]), np.array([True, False, False, True]))
    # ---- intra_planar_predict (int(left[y]) / int(top[x]); float corners -> TypeError)
    for n in (4, 8, 16, 32):
        t = rng.uniform(0, 255, n + 1)
        l = rng.uniform(0, 255, n + 1)
        add("intra_planar_predict", t, l, int(t[-1]), int(l[-1]), n)
        add("intra_planar_predict", t.astype(np.float32), l, 7, 250, n)
        add("intra_planar_predict", rng.random(n) > 0.5, rng.random(n) > 0.5, 1, 0, n)
    t = rng.uniform(0, 255, 8)
    add("intra_planar_predict", t, t, 128.0, 128, 8)
    add("intra_planar_predict", t, t, 128, np.float64(3.5), 8)
    t2 = t.copy()
    t2[5] = nan
    add("intra_planar_predict", t2, t, 10, 20, 8)
    add("intra_planar_predict", t, t2, 10, 20, 8)
    add("intra_planar_predict", np.append(t[:4], nan), t[:5], 10, 20, 4)        # NaN past size: never read
    t3 = t.copy()
    t3[3] = -inf
    add("intra_planar_predict", t3, t, 10, 20, 8)
    add("intra_planar_predict", np.array([-5.7, 3.2, 250.9, 17.0]), np.array([1.5, -2.5, 8.0, 9.9]), 100, 3, 4)
    # ---- intra_angular_predict (numpy's int16 element stores of _build_ref_array)
    for n in (4, 8):
        top = rng.uniform(0, 255, 2 * n + 1)
        left = rng.uniform(0, 255, 2 * n + 1)
        for mode in (2, 6, 10, 11, 14, 18, 21, 25, 26, 30, 34):
            add("intra_angular_predict", top, left, float(top[0]), mode, n)
        add("intra_angular_predict", top.astype(np.float32), left.astype(np.float16), 100, 18, n)
        add("intra_angular_predict", top[:n + 1], left[:n - 1], 90, 14, n)           # short refs (D6)
        add("intra_angular_predict", rng.random(2 * n + 1) > 0.5, rng.random(2 * n + 1) > 0.5, True, 22, n)
    top = rng.uniform(0, 255, 9)
    left = rng.uniform(0, 255, 9)
    add("intra_angular_predict", top, left, nan, 26, 4)
    add("intra_angular_predict", top, left, 1e6, 26, 4)
    add("intra_angular_predict", top, left, 32767.9, 26, 4)
    bad = top.copy()
    bad[3] = nan
    add("intra_angular_predict", bad, left, 10, 26, 4)
    add("intra_angular_predict", bad, left, 10, 10, 4)     # horizontal: top is the secondary array
    big = left.copy()
    big[1] = 4e4
    add("intra_angular_predict", top, big, 10, 18, 4)
    add("intra_angular_predict", top, big, 10, 34, 4)      # vertical positive angle: left never read
    # ---- residual_block / reconstruct_block (.astype(np.int16))
    a = rng.uniform(-300, 300, (8, 8))
    b = rng.uniform(-300, 300, (8, 8))
    add("residual_block", a, b)
    add("reconstruct_block", a.astype(np.float32), b)
    add("residual_block", np.array([[7e4, -7e4, 4e9, nan]]), np.array([[1.5, 2.5, 3.5, 4.5]]))
    add("reconstruct_block", rng.random((4, 4)) > 0.5, a[:4, :4])
    # ---- clip_to_pixel_range (np.clip(...).astype(np.int16))
    add("clip_to_pixel_range", np.array([[1.6, 300.]]))
    add("clip_to_pixel_range", rng.uniform(-50, 400, (8, 8)))
    add("clip_to_pixel_range", rng.uniform(-50, 400, (4, 4)).astype(np.float32))
    add("clip_to_pixel_range", rng.uniform(-50, 400, (4, 4)).astype(np.float16))
    add("clip_to_pixel_range", np.array([nan, inf, -inf, -0.5, 0.99, 254.999, 255.0, 1e300]))
    add("clip_to_pixel_range", rng.uniform(-5000, 5000, (8, 8)), 10)
    add("clip_to_pixel_range", np.array([7e4, 65535.9, 32768.5, 1e6, -1.0]), 16)
    add("clip_to_pixel_range", np.array([7e4, 65535.9, 32768.5, 1e6, 4e9, 3e9, nan]), 20)
    add("clip_to_pixel_range", np.array([7e4, 2.5e9, 4e9, 1e12, 1e19, inf]), 40)
    add("clip_to_pixel_range", rng.random((4, 4)) > 0.5)
    add("clip_to_pixel_range", rng.random((4, 4)) > 0.5, 16)
    # ---- quantize / quantize_block / dequantize (quant.py:76-79, :114)
    add("quantize", np.array([[100.7, -33.2]]), 22, 4)
    for n in (4, 8, 16, 32):
        c = rng.uniform(-2000, 2000, (n, n))
        for qp in (0, 17, 22, 32, 51):
            add("quantize", c, qp, n)
        add("quantize", c, 30, n, False)
        add("quantize_block", c.astype(np.float32), 27)
        add("dequantize", rng.uniform(-300, 300, (n, n)), 22, n)
        add("dequantize_block", rng.uniform(-300, 300, (n, n)).astype(np.float32), 40)
    add("quantize", np.array([[nan, inf, -inf, -0.0, 0.4, -0.6]]), 22, 4)
    add("quantize", np.array([[1e12, -1e12, 3e15, 2**62 * 1.0]]), 4, 8)
    add("quantize", np.array([[1e12, -1e12, 3e15]]), 51, 32)
    add("quantize", np.array([[True, False]]), 22, 4)
    add("dequantize", np.array([[nan, 1e30, -2.5, 2.5]]), 22, 4)
    add("dequantize", np.array([[True, False, True]]), 40, 4)
    # ---- count_nonzero / is_all_zero
    add("count_nonzero", np.array([0.0, nan, -0.0, 0.1, -1e-300]))
    add("is_all_zero", np.array([0.0, -0.0]))
    add("is_all_zero", np.array([0.0, nan]))
    add("count_nonzero", np.array([True, False, True]))
    # ---- metrics on floats / wide ints
    x = rng.uniform(0, 255, (16, 16))
    y = rng.uniform(0, 255, (16, 16))
    for sh in ((4, 4), (8, 8), (16, 16), (5, 7), (100,), (300,), (1000,)):
        n = int(np.prod(sh))
        u = rng.uniform(-100, 400, n).reshape(sh)
        v = rng.uniform(-100, 400, n).reshape(sh)
        add("mse", u, v)
        add("psnr", u, v)
        add("psnr", u.astype(np.float32), v.astype(np.float32), 1023)
    add("mse", x, x)
    add("psnr", x, x)
    add("mse", rng.integers(-2**40, 2**40, (8, 8)), rng.integers(-2**40, 2**40, (8, 8)))
    add("psnr", rng.integers(-2**31, 2**31, 64, dtype=np.int64).astype(np.int32),
        rng.integers(-2**31, 2**31, 64, dtype=np.int64).astype(np.int32))
    add("mse", np.asfortranarray(x), np.asfortranarray(y))
    add("mse", x, y[0])                                    # broadcasting
    add("sad", x, y)
    add("satd_4x4", x[:4, :4], y[:4, :4])
    add("residual_energy", x - y)
    add("psnr", rng.random((8, 8)) > 0.5, rng.random((8, 8)) > 0.5, 1)
    # ---- round 4 (VERDICT r3 missing #2-#3) -- appended, so the names above keep their indices
    # estimate_bits on every level dtype (quant.py:166-168: np.abs, +1 and log2 in the dtype's rules)
    lv = np.array([[3, -1], [0, 7]])
    for dt in (np.int8, np.int16, np.int32, np.int64, np.uint8, np.uint16, np.uint32, np.uint64,
               np.float16, np.float32, np.float64, bool):
        add("estimate_bits", lv.astype(dt))
        add("estimate_bits", rng.integers(-60, 60, (8, 8)).astype(dt))
        add("estimate_bits", rng.integers(0, 120, (16, 16)).astype(dt))
        add("estimate_bits", rng.integers(-100, 100, 300).astype(dt))          # > 128 terms: pairwise halves
    add("estimate_bits", np.array([[0, 1, 2, 3], [4, 5, 6, 7]], np.int16))
    add("estimate_bits", rng.integers(-32767, 32768, (8, 8)).astype(np.int16))
    add("estimate_bits", rng.integers(-32767, 32768, (32, 32)).astype(np.int16))
    add("estimate_bits", rng.integers(-127, 128, (8, 8)).astype(np.int8))
    add("estimate_bits", rng.integers(0, 255, (8, 8)).astype(np.uint8))
    add("estimate_bits", rng.integers(0, 65535, (8, 8)).astype(np.uint16))
    add("estimate_bits", np.array([5, -32768, 3], np.int16))                  # abs wraps: log2(-32767) -> NaN
    add("estimate_bits", np.array([5, -128, 3], np.int8))
    add("estimate_bits", np.array([5, 255, 3], np.uint8))                     # 255 + 1 wraps to 0: -inf
    add("estimate_bits", np.array([5, 65535], np.uint16))
    add("estimate_bits", np.array([1, 2**32 - 1], np.uint32))
    add("estimate_bits", np.array([2**63, 2**64 - 1, 7], np.uint64))
    add("estimate_bits", np.array([-2**31, 5], np.int32))
    add("estimate_bits", np.array([2**31 - 1, 5], np.int64))
    add("estimate_bits", rng.uniform(-300, 300, (8, 8)))
    add("estimate_bits", rng.uniform(-300, 300, (8, 8)).astype(np.float32))
    add("estimate_bits", rng.uniform(-300, 300, (8, 8)).astype(np.float16))
    add("estimate_bits", rng.uniform(-3e4, 3e4, 200).astype(np.float16))
    add("estimate_bits", np.array([0.25, -0.5, 1e-3, 6e4], np.float16))
    add("estimate_bits", np.array([1.5, nan, 2.0]))
    add("estimate_bits", np.array([1.5, inf], np.float32))
    add("estimate_bits", np.array([-0.0, 0.0, 1e-300]))
    add("estimate_bits", np.asfortranarray(rng.integers(-500, 500, (8, 12)).astype(np.int32)))
    add("estimate_bits", np.asfortranarray(rng.uniform(-9, 9, (12, 20))))
    add("estimate_bits", rng.integers(-500, 500, (20, 30)).astype(np.int16)[::2, 1::3])
    add("estimate_bits", rng.integers(-500, 500, 400)[::-1])
    add("estimate_bits", (rng.uniform(-9, 9, (8, 8)) + 1j * rng.uniform(-9, 9, (8, 8))).astype(np.complex64))
    add("estimate_bits", np.array([], np.int32))
    add("estimate_bits", np.array(["a", "b"]))
    # N-D blocks into the transforms (transform.py:171-194: block[k, j] over the trailing axes)
    for fn in ("forward_transform", "inverse_transform"):
        for shp in ((4, 4, 4), (8, 8, 2), (4, 4, 1), (8, 8, 1), (32, 32, 1), (4, 4, 0), (4, 5, 2), (4, 3, 2),
                    (4, 3, 1), (16, 16, 1, 1), (4, 4, 1, 2), (3, 4, 4), (4, 0, 1), (8, 8, 2, 1)):
            x = rng.integers(-255, 256, int(np.prod(shp))).reshape(shp).astype(np.int16)
            add(fn, x)
        add(fn, rng.integers(-255, 256, (4, 4, 1)).astype(np.int16), True)
        add(fn, rng.integers(-255, 256, (4, 4, 3)).astype(np.int16), True)
    # mse / psnr with mixed layouts and broadcast views (metrics.py:9-10: the diff's 'K' order)
    u = rng.uniform(0, 255, (24, 40))
    v = rng.uniform(0, 255, (40, 24))
    add("mse", np.asfortranarray(u), u)
    add("mse", u, np.asfortranarray(u + 1))
    add("mse", np.asfortranarray(u), v.T)
    add("mse", u[::2, ::3], v.T[::2, ::3])
    add("mse", u, u[:, :1])
    add("mse", u, u[:1, :].copy(order="F"))
    add("psnr", np.asfortranarray(u.astype(np.float32)), u[::-1])
    # count_nonzero / is_all_zero on object and string levels (np.count_nonzero's truthiness)
    add("count_nonzero", np.array([None, "", 0, 1, "x", 0.0, [1]], dtype=object))
    add("count_nonzero", np.array(["a", "", " "]))
    add("is_all_zero", np.array([0, 0.0, False], dtype=object))
    add("is_all_zero", np.array(["", ""]))
    # ---- round 5 (VERDICT r4 missing #2): planar with numpy-integer corners, e.g.
    # top[-1] / left[-1] of the reference rows themselves (intra.py:109-111 computes
    # (x+1)*corner and the sums in the corner's dtype under NEP 50)
    for n in (4, 8, 16, 32):
        for lo, hi in ((0, 256), (0, 1024)):                  # 8-bit and 10-bit samples
            for dt in (np.int16, np.uint8, np.int8, np.uint16, np.int32, np.int64, np.uint64):
                info = np.iinfo(dt)
                t = rng.integers(max(lo, info.min), min(hi, info.max + 1), n + 1).astype(dt)
                l = rng.integers(max(lo, info.min), min(hi, info.max + 1), n + 1).astype(dt)
                add("intra_planar_predict", t, l, t[-1], l[-1], n)
        t = np.full(n + 1, 1000, np.int16)
        add("intra_planar_predict", t, t.copy(), t[-1], t[-1], n)              # N = 32: -24 (wraps)
        add("intra_planar_predict", t, t.copy(), int(t[-1]), t[-1], n)         # one Python-int corner
        add("intra_planar_predict", t, t.copy(), t[-1], int(t[-1]), n)
    t16 = np.full(33, 1000, np.int16)
    add("intra_planar_predict", t16, t16, np.int32(30000), np.int32(30000), 32)    # int32: store OverflowError
    add("intra_planar_predict", t16, t16, np.int64(1000), np.uint64(1000), 8)      # float64 >> int: TypeError
    add("intra_planar_predict", t16, t16, np.uint64(1000), np.int8(10), 8)         # uint64 + int8: float64
    add("intra_planar_predict", t16, t16, np.uint64(2**64 - 5), np.uint64(7), 4)   # uint64 wrap
    add("intra_planar_predict", t16, t16, np.int16(1000), np.uint8(200), 16)       # int16 + uint8 -> int16
    add("intra_planar_predict", t16, t16, np.uint16(60000), np.int16(-5), 8)       # uint16 + int16 -> int32
    add("intra_planar_predict", t16, t16, np.uint32(7), np.int16(-5), 4)           # uint32 + int16 -> int64
    add("intra_planar_predict", t16, t16, np.uint8(3), np.int8(-3), 4)             # Python int > 255: Overflow
    add("intra_planar_predict", np.full(9, -3, np.int16), np.full(9, 2, np.int16), np.uint8(3), 4, 8)  # negative
    add("intra_planar_predict", np.full(5, 20, np.int8), np.full(5, 10, np.int8), np.int8(20), np.int8(10), 4)
    add("intra_planar_predict", np.full(5, 120, np.uint8), np.full(5, 2, np.uint8), np.uint8(120), np.uint8(2), 4)
    add("intra_planar_predict", t16, t16, np.True_, np.False_, 8)                  # bool_ -> int64
    add("intra_planar_predict", t16, t16, np.int8(100), 3.5, 8)                    # Overflow before TypeError
    add("intra_planar_predict", t16, t16, 3.5, np.int8(100), 8)
    add("intra_planar_predict", t16, t16, np.array(1000, np.int16), np.array(1000, np.int16), 32)   # 0-d arrays
    add("intra_planar_predict", t16[:3], t16, np.int16(1000), np.int16(1000), 8)   # IndexError vs wrap order
    add("intra_planar_predict", t16, t16[:2], np.int8(1), np.int8(1), 4)
    add("intra_planar_predict", np.full(200, 1, np.int16), np.full(200, 1, np.int16), np.int8(1), np.int8(1), 128)
    add("intra_planar_predict", np.full(300, 1, np.int16), np.full(300, 1, np.int16), np.uint8(1), np.uint8(1), 200)
    add("intra_planar_predict", rng.uniform(0, 255, 9), rng.uniform(0, 255, 9), np.int16(900), np.int16(800), 8)
    return out

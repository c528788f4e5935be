"""The value bounds behind the packed 16-bit config-3 chain (rdo8_chain_n,
nano-hevc_amd/csrc/nh_intraloop.hip), enumerated from the
reference's own constants: for 8-bit blocks with 8-bit neighbours every
operand the packed path holds in 16 bits is its true value.  Restates
transform.py:20-151 (DCT8 rows), transform.py:154-238 (shift log2N+5 per
pass) and quant.py:21-123 (quantize / dequantize) -- CPU only."""
import numpy as np

DCT8 = np.array([[64] * 8, [89, 75, 50, 18, -18, -50, -75, -89], [83, 36, -36, -83, -83, -36, 36, 83],
                 [75, -18, -89, -50, 50, 89, 18, -75], [64, -64, -64, 64, 64, -64, -64, 64],
                 [50, -89, 18, 75, -75, -18, 89, -50], [36, -83, 83, -36, -36, 83, -83, 36],
                 [18, -50, 75, -89, 89, -75, 50, -18]])
QUANT_SCALE = [26214, 23302, 20560, 18396, 16384, 14564]
DEQUANT_SCALE = [40, 45, 51, 57, 64, 72]


def _deq(level, qp):
    per, rem = qp // 6, qp % 6
    b = level * DEQUANT_SCALE[rem]
    return (b + (1 << (3 - per))) >> (4 - per) if per < 4 else b << (per - 4)


def test_packed_chain_bounds():
    row = int(np.abs(DCT8).sum(1).max())          # 512: forward passes
    col = int(np.abs(DCT8).sum(0).max())          # 479: inverse passes
    p1 = (row * 255 + 128) >> 8                   # residual in [-255, 255]
    assert p1 == 510 and 2 * p1 <= 32767 and 4 * 255 <= 32767          # pass-1 out, pass-1 E/EE
    coef = (row * p1 + 128) >> 8
    assert coef == 1020 and 4 * p1 <= 32767                             # pass-2 EE, |C|
    deq = 0
    c = np.arange(coef + 1, dtype=np.int64)
    for qp in range(52):
        shift = 14 + qp // 6 + 3
        lvl = (c * QUANT_SCALE[qp % 6] + (1 << shift) // 3) >> shift   # intra offset (the larger one)
        deq = max(deq, int(max(_deq(int(l), qp) for l in np.unique(lvl))))
    assert deq == 720
    inv1 = (col * deq + 128) >> 8
    inv2 = (col * inv1 + 128) >> 8
    assert inv1 == 1347 and inv2 == 2520 and inv2 <= 32767
    # every int32 sum stays far from 2^31 (the reference's ring never wraps here)
    assert row * 255 * 2 < 2 ** 31 and col * deq * 2 < 2 ** 31

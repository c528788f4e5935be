"""Range proof for the packed 16-bit config-4 chain.

Narrow workgroups: every source sample and neighbour in [0, 255], so the
residual is in [-255, 255].  This enumerates, for every TU kind (DST4, DCT
4/8/16/32), every QP 0..51 and intra/inter rounding, a bound on every operand
the packed chain holds in an int16 lane (butterfly E/O stages, pass outputs,
dequantized coefficients) and on every int32 dot-product sum, from the L1 norms
of the reference matrices (transform.py:20-135) and the monotone quantizer /
dequantizer (quant.py:41-123).  Prints the table and fails if any bound
reaches int16 / int32 limits.
"""
import numpy as np

TAB = [64, 90, 90, 90, 89, 88, 87, 85, 83, 82, 80, 78, 75, 73, 70, 67,
       64, 61, 57, 54, 50, 46, 43, 38, 36, 31, 25, 22, 18, 13, 9, 4, 0]


def dct32(k, n):
    if k == 0:
        return 64
    m = ((2 * n + 1) * k) % 128
    return TAB[m] if m <= 32 else -TAB[64 - m] if m <= 64 else -TAB[m - 64] if m <= 96 else TAB[128 - m]


def mat(n, dst):
    if dst:
        return np.array([[29, 55, 74, 84], [74, 74, 0, -74], [84, -29, -74, 55], [55, -84, 74, -29]], np.int64)
    return np.array([[dct32(k * (32 // n), j) for j in range(n)] for k in range(n)], np.int64)


QS = [26214, 23302, 20560, 18396, 16384, 14564]
DQ = [40, 45, 51, 57, 64, 72]


def quant(c, qp, l2, intra):
    per, rem = qp // 6, qp % 6
    sh = 14 + per + l2
    off = (1 << sh) // (3 if intra else 6)
    return (c * QS[rem] + off) >> sh


def dequant(l, qp):
    per, rem = qp // 6, qp % 6
    b = l * DQ[rem]
    return (b + (1 << (3 - per))) >> (4 - per) if per < 4 else b << (per - 4)


def shift_bound(acc, s):   # |(acc + 2^(s-1)) >> s| for |acc| <= bound
    return (acc + (1 << (s - 1))) >> s


def butterfly_operand(x, n, dst):
    """largest int16 operand of the packed forward butterfly on inputs |x| <= x:
    stage d of an n-point DCT holds sums of 2^d inputs (up to the 2-point pair)."""
    return x if dst else x * (n // 2)


def main():
    worst16, worst32 = 0, 0
    rows = []
    for n, dst in ((4, True), (4, False), (8, False), (16, False), (32, False)):
        T = mat(n, dst)
        l2 = int(np.log2(n))
        s = l2 + 5
        rowl1 = int(np.abs(T).sum(1).max())
        coll1 = int(np.abs(T).sum(0).max())
        x0 = 255
        f1_op = butterfly_operand(x0, n, dst)
        f1 = shift_bound(x0 * rowl1, s)
        f2_op = butterfly_operand(f1, n, dst)
        c = shift_bound(f1 * rowl1, s)
        dqmax = 0
        for qp in range(52):
            for intra in (True, False):
                dqmax = max(dqmax, dequant(quant(c, qp, l2, intra), qp))
        i1 = shift_bound(dqmax * coll1, s)
        i2 = shift_bound(i1 * coll1, s)
        ops16 = [f1_op, f1, f2_op, c, dqmax, i1, i2 + 255]
        sums32 = [x0 * rowl1 + (1 << s), f1 * rowl1 + (1 << s), dqmax * coll1 + (1 << s), i1 * coll1 + (1 << s),
                  n * n * 255 * 255]
        worst16 = max(worst16, max(ops16))
        worst32 = max(worst32, max(sums32))
        rows.append((("DST" if dst else "DCT") + str(n), f1_op, f1, f2_op, c, dqmax, i1, i2, max(sums32)))
    print("%-6s %8s %6s %8s %6s %6s %6s %6s %12s" % ("kind", "fwd1 op", "pass1", "fwd2 op", "coeff", "dq", "inv1",
                                                     "rres", "max int32"))
    for r in rows:
        print("%-6s %8d %6d %8d %6d %6d %6d %6d %12d" % r)
    print("largest int16 operand %d (limit 32767), largest int32 sum %d (limit 2^31-1)" % (worst16, worst32))
    assert worst16 <= 32767 and worst32 < 2 ** 31
    # f16 matrix-core 32x32 chain: operands integers of <= 11 bits,
    # every |partial sum| < 2^24 units of 2^-10 (pass 1 carries the +1536 offset)
    T = mat(32, False)
    rs, rl1, cl1 = T.sum(1), int(np.abs(T).sum(1).max()), int(np.abs(T).sum(0).max())
    x0 = 255
    p1 = max(abs(1536 * int(rs[k])) + sum(abs(int(t)) * (1536 + x0) for t in T[k]) for k in range(32))
    f1 = shift_bound(x0 * rl1, 10)
    c = shift_bound(f1 * rl1, 10)
    dq = max(dequant(quant(c, qp, 5, intra), qp) for qp in range(52) for intra in (True, False))
    i1 = shift_bound(dq * cl1, 10)
    # the accumulators start at 0; the rounding bias (0.5, pass 1 row 0: 0.5 - 3072) is added to
    # the final sum before floor(): its magnitude in 2^-10 units joins the bound
    bias = {"pass1": 3072 * 1024, "pass2": 512, "inv1": 512, "inv2": 512}
    sums = {"pass1": p1 + bias["pass1"], "pass2": f1 * rl1 + 512, "inv1": dq * cl1 + 512, "inv2": i1 * cl1 + 512}
    ops = {"residual+1536": 1536 + x0, "pass1 out": f1, "dequant": dq, "inv1 out": i1}
    print("f16 32x32 chain: operands", ops, "(exact in f16 below 2048), |sums|", sums, "(limit 2^24)")
    assert max(ops.values()) < 2048 and max(sums.values()) < 2 ** 24
    assert all(int(r) == 0 for r in rs[1:]) and int(rs[0]) == 2048
    mosaic_bounds()
    level_bounds()
    rdo8_dequant_bounds()


def mosaic_bounds():
    """The closed loop's small-TU mosaics (tu_closed_batch_mma): 16x16
    f16 MFMA passes against the basis * 2^-S.  Each accumulator in units of 2^-S must
    stay below 2^24 (exact fp32), every f16 operand an exact integer: the residual as
    768 + n (|n| <= 255, binade [512, 1024)), the pass-1 output as 1536 + t in
    [1024, 2048) (|t| <= 511: truncation = floor), the dequantized coefficients and
    the inverse-pass-1 output below 2048 -- except DCT4 (chroma 4x4), whose inverse
    pass 1 reaches 2223: its inverse pass 2 runs split (nh_mosaic.hpp MosaicCore::
    SPLIT), tmp = 2h + b with h = floor(tmp / 2) against the basis * 2^-(S-1) and
    b in {0, 1} against the basis * 2^-S, two MFMAs into one accumulator that starts
    at 1536.5.  Its bounds: |h| <= 1112 (an exact f16 integer), every partial sum of
    the two MFMAs (units 2^-S) <= (|tmp| + 1) * colL1 + 1536.5 * 2^S < 2^24, and the
    16-bit dequantization l * dqs + dqr < 2^15."""
    print("mosaic    pass1-out  pass2 op  coeff   dq  inv1-out  |sum| max (units 2^-S)  ok")
    for n, dst in ((4, True), (8, False), (16, False), (4, False)):
        T = mat(n, dst)
        l2 = int(np.log2(n))
        s = l2 + 5
        rl1, cl1 = int(np.abs(T).sum(1).max()), int(np.abs(T).sum(0).max())
        rsum = [int(v) for v in T.sum(1)]
        x0 = 255
        f1 = shift_bound(x0 * rl1, s)
        c = shift_bound(f1 * rl1, s)
        dq = max(dequant(quant(c, qp, l2, intra), qp) for qp in range(52) for intra in (True, False))
        i1 = shift_bound(dq * cl1, s)
        i2 = shift_bound(i1 * cl1, s)
        c1 = max(abs(0.5 + 1536 - 768 * r / 2 ** s) for r in rsum)
        c2 = max(abs(0.5 - 1536 * r / 2 ** s) for r in rsum)
        sums = [int(np.abs(T).sum(1).max()) * (768 + x0) + int(c1 * 2 ** s),
                rl1 * (1536 + f1) + int(c2 * 2 ** s),
                dq * cl1 + 2 ** (s - 1),
                i1 * cl1 + int(1536.5 * 2 ** s)]
        split = (n, dst) == (4, False)
        if split:   # inverse pass 2 on (h, b): tmp = 2h + b, so 2|h| <= |tmp| + 1
            h = (i1 + 1) // 2
            sums[3] = (i1 + 1) * cl1 + int(1536.5 * 2 ** s)
            inv_ok = h <= 2048 and 2 * h + 1 >= i1   # h exact in f16; tmp's range covered
        else:
            inv_ok = i1 <= 2048
        ok = f1 <= 511 and 1536 + f1 < 2048 and dq < 2048 and inv_ok and max(sums) < 2 ** 24
        print("%-8s %9d %9d %6d %4d %9d %23d  %s%s" % (("DST" if dst else "DCT") + str(n), f1, 1536 + f1, c, dq, i1,
                                                        max(sums), ok, "  (split: |h| <= %d)" % h if split else ""))
        # dequantize in 16-bit lanes: (l * dqs + dqr) >> dqsh with dqs = DQ << max(per - 4, 0)
        ldq = max(quant(c, qp, l2, intra) * (DQ[qp % 6] << max(qp // 6 - 4, 0)) + (1 << 3)
                  for qp in range(52) for intra in (True, False))
        ok = ok and ldq < 2 ** 15
        assert ok, (n, dst, ldq)
        assert i2 < 1 << 15


def level_bounds():
    """The largest |level| quantize_block gives an 8-bit block (residual in
    [-255, 255]) of every kind, over QP 0..51 and both rounding offsets.  Config
    5's compact levels (k_tc32_hd<KB, int16 / int8>) rest on the
    32x32 bound: <= 51, so int8 holds every 8-bit block's level, and the marker
    values -128 / -32768 (a wide block's levels are in the spill plane) never
    occur as a level.  Returns {kind: bound}."""
    out = {}
    for n, dst in ((4, True), (4, False), (8, False), (16, False), (32, False)):
        T = mat(n, dst)
        l2 = int(np.log2(n))
        s = l2 + 5
        rl1 = int(np.abs(T).sum(1).max())
        c = shift_bound(shift_bound(255 * rl1, s) * rl1, s)
        out[("DST" if dst else "DCT") + str(n)] = max(quant(c, qp, l2, intra) for qp in range(52)
                                                      for intra in (True, False))
    print("largest |level| of an 8-bit block:", out)
    assert out["DCT32"] <= 51 < 127
    return out


def rdo8_dequant_bounds():
    """Config 3's packed chain (rdo8_chain_n) dequantizes level PAIRS
    with v_pk_mad + v_pk_ashr: l * dqs + dqr (dqs = scale << max(per - 4, 0), dqr =
    2^(3 - per) for per < 4) must stay within int16 for every level an 8-bit 8x8 block
    can produce (intra rounding, the coefficient bound of the DCT8 row), every QP.
    Returns the largest |l * dqs + dqr| per QP."""
    T = mat(8, False)
    rl1 = int(np.abs(T).sum(1).max())
    c = shift_bound(shift_bound(255 * rl1, 8) * rl1, 8)
    worst = {}
    for qp in range(52):
        per, rem = qp // 6, qp % 6
        lmax = quant(c, qp, 3, True)
        dqs = DQ[rem] << max(per - 4, 0)
        dqr = (1 << (3 - per)) if per < 4 else 0
        v = max(lmax * dqs + dqr, lmax * dqs)
        assert v <= 32767 and -lmax * dqs + dqr >= -32768, (qp, lmax, dqs)
        assert (v >> (4 - per if per < 4 else 0)) == dequant(lmax, qp)
        worst[qp] = v
    print("config-3 packed dequant: |coeff| <= %d, max |l * dqs + dqr| %d (QP %d; limit 32767)"
          % (c, max(worst.values()), max(worst, key=worst.get)))
    return worst



if __name__ == "__main__":
    main()


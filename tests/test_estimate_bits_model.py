"""CPU check of the dtype model behind the device estimate_bits (eb_term in
csrc/nh_blocks.hip, codes NH_EB_* in include/nanohevc.h): the same steps written
with numpy scalars -- |l| and +1 in the level's dtype, log2 correctly rounded to
the float type numpy's np.log2 picks (float16 / float32 / float64), + (|l|>0)*2
in float64, numpy's pairwise sum in the levels' 'K' memory order, int() -- must
give the reference's value (or exception class) for every estimate_bits case of
tests/golden/dtypes.npz.  The GPU test (test_dtypes_gpu.py) runs the device code
on the same cases."""
import math
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
from dtype_cases import cases  # noqa: E402


def _log2_prec(x: float, prec: int) -> float:
    l = np.log2(np.float64(x)) if x > 0 else (-np.inf if x == 0 else np.nan)
    if prec == 64:
        return float(l)
    f = np.float32(l)
    return float(f) if prec == 32 else float(np.float16(f))


def _term(v, dt) -> float:
    k, w = dt.kind, dt.itemsize * 8
    if k == "b":
        b = int(bool(v))
        return math.log2(b + 1) + 2 * b
    if k == "f":
        if w == 64:
            a = abs(float(v))
            return _log2_prec(a + 1.0, 64) + 2 * (a > 0)
        af = np.float32(abs(np.float32(v)))
        a1 = np.float32(af + np.float32(1))
        if w == 32:
            return _log2_prec(float(a1), 32) + 2 * bool(af > 0)
        return _log2_prec(float(np.float16(a1)), 16) + 2 * bool(af > 0)
    prec = 16 if w == 8 else 32 if w == 16 else 64
    m = (1 << w) - 1
    if k == "u":
        u = int(v) & m
        return _log2_prec(float((u + 1) & m), prec) + 2 * (u > 0)

    def wrap(x):
        x &= m
        return x - (1 << w) if x >> (w - 1) else x
    a = wrap(abs(int(v)))
    return _log2_prec(float(wrap(a + 1)), prec) + 2 * (a > 0)


def _pairwise(t):
    n = len(t)
    if n < 8:
        r = 0.0
        for x in t:
            r += x
        return r
    if n <= 128:
        r = list(t[:8])
        i = 8
        while i < n - n % 8:
            for j in range(8):
                r[j] += t[i + j]
            i += 8
        res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]))
        for x in t[i:]:
            res += x
        return res
    n2 = n // 2
    n2 -= n2 % 8
    return _pairwise(t[:n2]) + _pairwise(t[n2:])


def _model(level):
    a = np.asarray(level)
    if a.dtype.kind == "c":
        a = np.abs(a)
    if a.dtype.kind not in "biuf":
        raise TypeError("log2")
    flat = np.ravel(a, order="K")
    return int(_pairwise([_term(v, a.dtype) for v in flat.tolist()]))


CASES = [c for c in cases() if c[1] == "estimate_bits"]


@pytest.fixture(scope="module")
def fixture():
    with np.load(os.path.join(HERE, "golden", "dtypes.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.mark.parametrize("name,fn,args,kw", CASES, ids=[c[0] for c in CASES])
def test_estimate_bits_dtype_model(fixture, name, fn, args, kw):
    import builtins
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        if "err_" + name in fixture:
            with pytest.raises(getattr(builtins, str(fixture["errbase_" + name]))):
                _model(*args)
            return
        assert _model(*args) == int(fixture["out_" + name])


def test_model_covers_every_level_dtype():
    kinds = {np.asarray(c[2][0]).dtype.str[1:] for c in CASES}
    for k in ("i1", "i2", "i4", "i8", "u1", "u2", "u4", "u8", "f2", "f4", "f8", "b1", "c8"):
        assert k in kinds, k

"""Float / bool / narrow-float inputs through the drop-in.

tests/golden/dtypes.npz holds, per call of tests/golden/dtype_cases.py, what the
REFERENCE returned (value, dtype and Python type) or which exception it raised
(recorded by make_golden.py --only dtypes.npz).  The MI355X drop-in must give
the same value bit for bit (float results included: mse / psnr are computed in
numpy's pairwise summation order on the device) or raise the same builtin
exception class."""
import builtins
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
from dtype_cases import cases  # noqa: E402

CASES = cases()


@pytest.fixture(scope="module")
def fixture():
    with np.load(os.path.join(HERE, "golden", "dtypes.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def test_fixture_covers_every_case(fixture):
    names = {n for n, *_ in CASES}
    got = {k.split("_", 1)[1] for k in fixture if k.startswith(("out_", "err_"))}
    assert names == got


@pytest.mark.parametrize("name,fn,args,kw", CASES, ids=[c[0] for c in CASES])
def test_dtype_case_matches_reference(fixture, name, fn, args, kw):
    import warnings
    from nano_hevc import intra, quant, metrics, transform
    f = next(getattr(m, fn) for m in (intra, quant, metrics, transform) if hasattr(m, fn))
    if "err_" + name in fixture:
        base = getattr(builtins, str(fixture["errbase_" + name]))
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            with pytest.raises(base):
                f(*args, **kw)
        return
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        r = f(*args, **kw)
    exp = fixture["out_" + name]
    assert type(r).__name__ == str(fixture["rtype_" + name])
    got = np.asarray(r)
    assert got.dtype == exp.dtype and got.shape == exp.shape
    assert np.array_equal(got, exp, equal_nan=got.dtype.kind == "f")

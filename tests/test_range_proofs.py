"""The range proofs behind the 8-bit chains run as CPU tests (tools/packed_bounds.py):
the packed 16-bit butterflies, the f16 32x32 matrix-core chain
(§4.5) and the closed loop's small-TU mosaics (§4.4b) -- every operand an exact
int16 / f16 integer and every accumulator below its exactness limit for residuals in
[-255, 255] at every QP."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import packed_bounds  # noqa: E402


def test_packed_and_f16_chain_bounds(capsys):
    packed_bounds.main()
    out = capsys.readouterr().out
    assert "DST4" in out and "DCT16" in out and "mosaic" in out


def test_dct4_is_excluded_from_the_mosaics():
    """DCT4's inverse pass 1 can reach 2223 (beyond f16's integers): chroma 4x4 TUs
    stay on the packed chain (tu_closed_batch_mma's static_assert)."""
    T = packed_bounds.mat(4, False)
    coll1 = int(abs(T).sum(0).max())
    assert packed_bounds.shift_bound(1152 * coll1, 7) > 2048

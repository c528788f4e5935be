"""The range proofs behind the 8-bit chains run as CPU tests (tools/packed_bounds.py):
the packed 16-bit butterflies, the f16 32x32 matrix-core chain
(§4.5), the small-TU mosaics (§4.4b, DCT4's split inverse included) and config 5's
compact level bound (§4.5) -- every operand an exact
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


def test_dct4_mosaic_split_inverse_bounds():
    """DCT4's inverse pass 1 reaches 2223 (beyond f16's integers), so the chroma 4x4
    mosaics (MosaicCore::SPLIT, the closed loop's and the open loop's default) run
    the inverse pass 2 on tmp = 2h + b: |h| <= 1112 is exact in f16, the two MFMAs'
    partial sums stay below 2^24 units of 2^-7, and the 16-bit dequantization
    below 2^15 -- asserted by mosaic_bounds for every kind, DCT4 included."""
    T = packed_bounds.mat(4, False)
    coll1 = int(abs(T).sum(0).max())
    i1 = packed_bounds.shift_bound(1152 * coll1, 7)
    assert i1 == 2223 and (i1 + 1) // 2 == 1112 < 2048
    assert (i1 + 1) * coll1 + int(1536.5 * 2 ** 7) < 2 ** 24
    packed_bounds.mosaic_bounds()   # asserts DCT4's split form with the other kinds


def test_compact_level_bound_for_config5():
    """An 8-bit 32x32 block's levels satisfy |level| <= 51 at every QP: config 5's
    int16 / int8 compact levels are exact, and the spill markers never collide."""
    b = packed_bounds.level_bounds()
    assert b["DCT32"] == 51 and max(b.values()) < 2 ** 15


def test_config3_packed_dequant_bound():
    """rdo8_chain_n dequantizes level pairs in int16 lanes: l * dqs + dqr fits int16
    at every QP for an 8-bit 8x8 block (and the shift gives dequantize_block's value)."""
    w = packed_bounds.rdo8_dequant_bounds()
    assert len(w) == 52 and max(w.values()) <= 32767

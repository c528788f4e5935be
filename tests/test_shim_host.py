"""Host-side logic of the drop-in shim (no GPU): constants, parameter
computation and the exceptions raised before any device work, all compared
with the reference's recorded values in tests/golden/."""
import numpy as np
import pytest

import nano_hevc as nh
from nano_hevc import gpu, quant, transform


def test_constants_match_reference(golden):
    g = golden("matrices.npz")
    for name in ("DST4", "DCT4", "DCT8", "DCT16", "DCT32"):
        assert np.array_equal(getattr(nh, name), g[name]) and getattr(nh, name).dtype == np.int32
    assert nh.INTRA_PRED_ANGLE[10 - 2] == 0 and nh.INTRA_PRED_ANGLE[18 - 2] == -32   # test_intra_angular.py:190-197
    assert len(nh.INTRA_PRED_ANGLE) == 33
    assert nh.QUANT_SCALE == [26214, 23302, 20560, 18396, 16384, 14564]
    assert nh.DEQUANT_SCALE == [40, 45, 51, 57, 64, 72]


def test_qp_params(golden):
    g = golden("quant.npz")
    got = np.array([quant.get_qp_params(q) for q in range(-3, 56)])
    assert np.array_equal(got, g["qp_params"])


def test_errors_raised_before_device_work():
    with pytest.raises(ValueError):
        nh.forward_transform(np.zeros((6, 6), np.int16))              # transform.py:150-151
    with pytest.raises(ValueError):
        transform._get_transform_matrix(64)
    with pytest.raises(IndexError):
        nh.intra_angular_predict(np.zeros(9, np.int16), np.zeros(9, np.int16), 0, 35, 4)   # intra.py:142
    with pytest.raises(ZeroDivisionError):
        nh.intra_dc_predict(np.zeros(4, np.int16), np.zeros(4, np.int16), 0)
    with pytest.raises(OverflowError):
        nh.quantize(np.zeros(4, np.int32), 22, 0)                   # int(np.log2(0))
    with pytest.raises(ValueError):
        nh.clip_to_pixel_range(np.zeros(3, np.int16), -1)           # 1 << -1


def test_yuv420_plane_sets():
    sets = gpu.yuv420_plane_sets(3, 3840, 2160)
    assert gpu.blocks_in(sets) == 3 * (480 * 270 + 2 * 240 * 135)   # 194,400 8x8 blocks per 4K frame
    y, uv = sets
    fs = gpu.yuv420_frame_elems(3840, 2160)
    assert (y.group_stride, uv.base, uv.plane_stride, uv.planes_per_group) == (fs, 3840 * 2160, 1920 * 1080, 2)
    # 1080p chroma (540 rows) has a partial bottom block row: skipped like block.py:72-74
    assert gpu.blocks_in(gpu.yuv420_plane_sets(1, 1920, 1080)) == 240 * 135 + 2 * 120 * 67


def test_block_iteration_rules():
    p = nh.Plane(np.arange(20 * 28, dtype=np.int16).reshape(20, 28))
    blocks = list(nh.iterate_blocks(p, 8))
    assert [(b.x, b.y) for b in blocks] == [(0, 0), (8, 0), (16, 0), (0, 8), (8, 8), (16, 8)]
    b = nh.BlockView(p, 24, 8, 8)                      # right-edge block: slice truncation
    assert b.get_top_neighbors(16).size == 4 and b.get_top_left_neighbor() == int(p.data[7, 23])
    assert np.all(nh.BlockView(p, 0, 0, 4).get_top_neighbors() == 128)


def test_frame_containers_roundtrip():
    raw = bytes(range(256)) * ((16 * 8 * 3 // 2) // 256 + 1)
    raw = raw[:16 * 8 * 3 // 2]
    f = nh.Frame.from_yuv420p(raw, 8, 16)
    assert f.to_yuv420p() == raw
    pf = nh.PackedFrame.from_frame(f)
    assert pf.to_yuv420p() == raw and pf.to_frame().u.data.shape == (4, 8)
    pool = nh.FrameBufferPool(8, 16, pool_size=2)
    i, _ = pool.acquire()
    assert pool.in_use_count == 1
    pool.release(i)
    with pytest.raises(ValueError):
        pool.release(i)


def test_create_test_frame_matches_reference(golden):
    """encoder.create_test_frame (host data generation) == the reference's demo frame."""
    from nano_hevc.encoder import create_test_frame
    g = golden("encode.npz")
    fb = create_test_frame(48, 80)
    for p, k in ((fb.y, "e_b_y"), (fb.u, "e_b_u"), (fb.v, "e_b_v")):
        assert p.data.dtype == np.int16 and np.array_equal(p.data, g[k])
    for key in ("d_64x64_bs8", "d_48x80_bs4", "d_72x40_bs16"):
        h, w = (int(v) for v in key.split("_")[1].split("x"))
        assert np.array_equal(create_test_frame(h, w).y.data, g[key + "_y"])


def test_encoder_fails_loudly_without_device():
    """No CPU fallback for the frame driver either."""
    import torch
    from nano_hevc.encoder import create_test_frame, encode_frame_intra
    if torch.cuda.is_available():
        pytest.skip("a device is present")
    with pytest.raises(Exception):
        encode_frame_intra(create_test_frame(16, 16), 8)


def test_natural_residual_helper_matches_reference_dc():
    """CPU check of tests/natural.py (used by the D-1 (b) GPU parity test)
    against intra_dc_predict's rule (intra.py:46-62) on a few blocks."""
    from natural import natural_residual
    rng = np.random.default_rng(3)
    src = rng.integers(0, 256, (24, 32)).astype(np.int64)
    res = natural_residual(src)
    for by, bx in ((0, 0), (0, 8), (8, 0), (16, 24)):
        top = np.full(8, 128) if by == 0 else src[by - 1, bx:bx + 8]
        left = np.full(8, 128) if bx == 0 else src[by:by + 8, bx - 1]
        dc = (int(top.sum()) + int(left.sum()) + 8) // 16
        assert np.array_equal(res[by:by + 8, bx:bx + 8], (src[by:by + 8, bx:bx + 8] - dc).astype(np.int16))


def test_plane_sets_disjoint():
    """tu_pipeline_closed_yuv420 runs luma and chroma concurrently only when the
    two sets write disjoint elements (else it codes them in sequence)."""
    W, H, F = 64, 32, 3
    y, uv = gpu.yuv420_plane_sets(F, W, H)
    assert gpu.sets_disjoint(y, uv) and gpu.sets_disjoint(uv, y)
    assert not gpu.sets_disjoint(y, y)
    y2, _ = gpu.yuv420_plane_sets(F, W, H, base=W * H - 1)   # overlaps the first frame's Y / U boundary
    assert not gpu.sets_disjoint(y2, uv)
    # interleaved rows: pitch 2W, set a on even rows, set b on odd rows -> interval overlap (conservative)
    a = gpu.plane_set(0, W, 4, 2 * W)
    b = gpu.plane_set(W, W, 4, 2 * W)
    assert not gpu.sets_disjoint(a, b)
    c = gpu.plane_set(8 * W, W, 4, 2 * W)
    assert gpu.sets_disjoint(a, c)


def test_estimate_bits_extended_precision_is_refused():
    """numpy computes estimate_bits of longdouble levels (and of complex256's
    magnitude) in 80-bit extended precision (quant.py:166-168); the device has no
    such type, so the drop-in refuses them instead of narrowing to float64
    (ADVICE r4).  Host-side check: no device call is made."""
    from nano_hevc.quant import estimate_bits
    if np.dtype(np.longdouble).itemsize == 8:
        pytest.skip("longdouble is float64 on this platform")
    with pytest.raises(NotImplementedError):
        estimate_bits(np.array([1.5, -3.0], np.longdouble))
    with pytest.raises(NotImplementedError):
        estimate_bits(np.array([1 + 2j], np.clongdouble))


def test_closed_stream_argument_checks():
    """tu_pipeline_closed_yuv420_stream refuses bad batch / depth / stride / size
    arguments on the host, before any device call."""
    import torch
    W, H, F = 64, 32, 3
    src = torch.zeros(F * gpu.yuv420_frame_elems(W, H), dtype=torch.int16)
    for kw in ({"batch_frames": 0}, {"depth": 0}, {"frame_stride": gpu.yuv420_frame_elems(W, H) - 1}):
        with pytest.raises(ValueError):
            gpu.tu_pipeline_closed_yuv420_stream(src, W, H, F, 1, 32, **kw)
    with pytest.raises(ValueError):   # one frame more than the buffer holds
        gpu.tu_pipeline_closed_yuv420_stream(src, W, H, F + 1, 1, 32)
    with pytest.raises(ValueError):   # the base pushes the last frame out
        gpu.tu_pipeline_closed_yuv420_stream(src, W, H, F, 1, 32, base=1)


def test_closed3_stream_argument_checks():
    """intra_rdo_closed_yuv420_stream refuses bad batch / depth / stride / size
    arguments on the host, before any device call."""
    import torch
    W, H, F = 64, 32, 3
    src = torch.zeros(F * gpu.yuv420_frame_elems(W, H), dtype=torch.int16)
    for kw in ({"batch_frames": 0}, {"depth": 0}, {"frame_stride": gpu.yuv420_frame_elems(W, H) - 1}):
        with pytest.raises(ValueError):
            gpu.intra_rdo_closed_yuv420_stream(src, W, H, F, 32, **kw)
    with pytest.raises(ValueError):
        gpu.intra_rdo_closed_yuv420_stream(src, W, H, F + 1, 32)
    with pytest.raises(TypeError):   # a host tensor: the device entry points take device memory only
        gpu.intra_rdo_closed_yuv420_stream(src, W, H, F, 32)

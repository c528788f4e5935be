"""The reference's own test scenarios, restated against the drop-in package.

Each test below re-states one scenario of the reference's suite
(tests/test_intra_dc.py, test_intra_planar.py, test_intra_angular.py,
test_quant.py, test_transform.py -- 77 cases) with the same inputs and the same
acceptance condition, calling ``nano_hevc`` exactly as a reference user would.
Every call runs on the MI355X, so this file is the "drops into the existing
tests" check (the reference itself never travels to the GPU box).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def nh():
    import nano_hevc
    from nano_hevc import _lib
    assert _lib.device_count() > 0
    return nano_hevc


ORIG = np.array([[102, 101, 100, 100], [103, 102, 101, 100], [103, 102, 100, 99], [104, 101, 99, 98]], np.int16)
TOP4 = np.array([102, 98, 100, 101], np.int16)
LEFT4 = np.array([103, 102, 101, 99], np.int16)


# ---------------------------------------------------------------- test_intra_dc.py (12 cases)

def test_dc4_spec_example(nh):                                   # :23-43
    p = nh.intra_dc_predict_4x4(TOP4, LEFT4)
    assert p.shape == (4, 4) and p.dtype == np.int16 and np.all(p == 101)


@pytest.mark.parametrize("t,l,v", [([100] * 4, [100] * 4, 100), ([1, 1, 1, 1], [1, 1, 1, 0], 1), ([0] * 4, [0] * 4, 0)])
def test_dc4_variants(nh, t, l, v):                              # :45-56
    assert np.all(nh.intra_dc_predict_4x4(np.array(t, np.int16), np.array(l, np.int16)) == v)


@pytest.mark.parametrize("n,v", [(8, 100), (16, 50)])
def test_dc_general(nh, n, v):                                    # :62-80
    p = nh.intra_dc_predict(np.full(n, v, np.int16), np.full(n, v, np.int16), size=n)
    assert p.shape == (n, n) and np.all(p == v)


def test_residual_spec_example(nh):                              # :86-127
    r = nh.residual_block(ORIG, np.full((4, 4), 101, np.int16))
    assert r.dtype == np.int16
    assert np.array_equal(r, [[1, 0, -1, -1], [2, 1, 0, -1], [2, 1, -1, -2], [3, 0, -2, -3]])


def test_residual_of_identical_blocks_is_zero(nh):               # :129-138
    b = np.full((2, 2), 100, np.int16)
    assert not nh.residual_block(b, b).any()


def test_reconstruct_inverts_residual(nh):                       # :144-157
    pred = np.full((4, 4), 101, np.int16)
    assert np.array_equal(nh.reconstruct_block(pred, nh.residual_block(ORIG, pred)), ORIG)


@pytest.mark.parametrize("bd,src,exp", [(8, [-10, 0, 128, 255, 300], [0, 0, 128, 255, 255]),
                                        (10, [-10, 0, 512, 1023, 2000], [0, 0, 512, 1023, 1023])])
def test_clip(nh, bd, src, exp):                                  # :163-177
    assert np.array_equal(nh.clip_to_pixel_range(np.array([src], np.int16), bit_depth=bd), [exp])


def test_dc_pipeline(nh):                                         # :183-211
    pred = nh.intra_dc_predict_4x4(TOP4, LEFT4)
    res = nh.residual_block(ORIG, pred)
    assert np.all(pred == 101) and np.array_equal(nh.reconstruct_block(pred, res), ORIG)


# ---------------------------------------------------------------- test_intra_planar.py (9 cases)

def test_planar_flat(nh):                                         # :21-33
    p = nh.intra_planar_predict(np.full(4, 100, np.int16), np.full(4, 100, np.int16), 100, 100, 4)
    assert p.shape == (4, 4) and p.dtype == np.int16 and np.all(p == 100)


@pytest.mark.parametrize("tr,bl,axis", [(255, 0, 1), (0, 255, 0)])
def test_planar_gradient_direction(nh, tr, bl, axis):            # :35-54
    p = nh.intra_planar_predict(np.zeros(4, np.int16), np.zeros(4, np.int16), tr, bl, 4)
    assert np.all(np.diff(p.astype(int), axis=axis) > 0)


def test_planar_corner_values(nh):                                # :56-76
    p = nh.intra_planar_predict(np.zeros(4, np.int16), np.zeros(4, np.int16), 255, 255, 4)
    assert p[0, 0] == 64 and p[3, 3] == 255


@pytest.mark.parametrize("n,v", [(4, 100), (8, 128), (16, 200), (32, 50)])
def test_planar_flat_sizes(nh, n, v):                             # :78-86
    p = nh.intra_planar_predict(np.full(n, v, np.int16), np.full(n, v, np.int16), v, v, n)
    assert p.shape == (n, n) and np.all(p == v)


def test_planar_pipeline(nh):                                     # :92-116
    pred = nh.intra_planar_predict(np.full(4, 100, np.int16), np.full(4, 100, np.int16), 100, 100, 4)
    assert np.all(pred == 100)
    assert np.array_equal(nh.reconstruct_block(pred, nh.residual_block(ORIG, pred)), ORIG)


# ---------------------------------------------------------------- test_intra_angular.py (13 cases)

T9 = np.array([99, 100, 110, 120, 130, 0, 0, 0, 0], np.int16)
L9 = np.array([99, 50, 50, 50, 50, 0, 0, 0, 0], np.int16)
RAMP = np.array([0, 10, 20, 30, 40, 50, 60, 70, 80], np.int16)


@pytest.mark.parametrize("n", [4, 8])
def test_mode26_copies_top(nh, n):                                # :25-43
    p = nh.intra_angular_predict(T9, L9, 99, mode=26, size=n)
    assert p.shape == (n, n)
    for c, v in enumerate([100, 110, 120, 130]):
        assert np.all(p[:, c] == v)


def test_mode34_diagonal(nh):                                     # :45-67
    p = nh.intra_angular_predict(RAMP, np.zeros(9, np.int16), 0, mode=34, size=4)
    assert (p[0, 0], p[0, 3], p[1, 0], p[3, 3]) == (20, 50, 30, 80)


def test_mode18_negative_extension(nh):                           # :69-85
    p = nh.intra_angular_predict(RAMP, np.array([0] + [5] * 8, np.int16), top_left=0, mode=18, size=4)
    assert np.array_equal(p, [[0, 10, 20, 30], [0, 0, 10, 20], [5, 0, 0, 10], [5, 5, 0, 0]])


def test_mode10_copies_left(nh):                                  # :91-109
    p = nh.intra_angular_predict(L9, T9, 99, mode=10, size=4)
    for r, v in enumerate([100, 110, 120, 130]):
        assert np.all(p[r, :] == v)


def test_mode2_diagonal(nh):                                      # :111-133
    p = nh.intra_angular_predict(np.zeros(9, np.int16), RAMP, 0, mode=2, size=4)
    assert (p[0, 0], p[3, 0], p[0, 1], p[3, 3]) == (20, 50, 30, 80)


def test_fractional_mode_on_flat_refs(nh):                        # :139-153
    f = np.full(9, 100, np.int16)
    assert np.all(nh.intra_angular_predict(f, f, 100, mode=27, size=4) == 100)


def test_vertical_copy_of_gradient(nh):                           # :155-169
    top = np.array([0, 0, 32, 64, 96, 128, 160, 192, 224], np.int16)
    p = nh.intra_angular_predict(top, np.zeros(9, np.int16), 0, mode=26, size=4)
    assert list(p[0, :4]) == [0, 32, 64, 96]


def test_every_mode_on_flat_refs(nh):                             # :175-188
    f = np.full(9, 128, np.int16)
    for m in range(2, 35):
        p = nh.intra_angular_predict(f, f, 128, mode=m, size=4)
        assert p.shape == (4, 4) and p.dtype == np.int16 and np.all(p == 128), m


def test_angle_table(nh):                                         # :190-197
    a = nh.INTRA_PRED_ANGLE
    assert (a[8], a[24], a[0], a[32], a[16]) == (0, 0, 32, 32, -32)


@pytest.mark.parametrize("n,mode,v", [(8, 26, 64), (16, 10, 200)])
def test_angular_larger_blocks(nh, n, mode, v):                   # :203-225
    f = np.full(2 * n + 1, v, np.int16)
    p = nh.intra_angular_predict(f, f, v, mode=mode, size=n)
    assert p.shape == (n, n) and np.all(p == v)


def test_angular_pipeline(nh):                                    # :231-255
    f = np.full(9, 100, np.int16)
    pred = nh.intra_angular_predict(f, f, 100, mode=26, size=4)
    assert np.all(pred == 100)
    assert np.array_equal(nh.reconstruct_block(pred, nh.residual_block(ORIG, pred)), ORIG)


# ---------------------------------------------------------------- test_quant.py (23 cases)

def test_qp_params(nh):                                           # :25-56 (4 cases)
    from nano_hevc.quant import get_qp_params
    assert all(get_qp_params(q) == (0, q) for q in range(6))
    assert all(get_qp_params(q) == (1, q - 6) for q in range(6, 12))
    assert get_qp_params(51) == (8, 3)
    assert get_qp_params(-5) == (0, 0) and get_qp_params(100) == (8, 3)


def test_quantize_zeros(nh):                                      # :62-69
    l = nh.quantize(np.zeros((4, 4), np.int32), qp=20, size=4)
    assert l.shape == (4, 4) and not l.any()


def test_dead_zone_at_high_qp(nh):                                # :71-78
    assert not nh.quantize(np.full((4, 4), 5, np.int32), qp=40, size=4).any()


def test_quantize_keeps_signs(nh):                                # :80-96
    c = np.array([[100, -100, 50, -50], [-200, 200, -25, 25], [75, -75, 150, -150], [-10, 10, 5, -5]], np.int32)
    l = nh.quantize(c, qp=20, size=4)
    nz = l != 0
    assert np.all(np.sign(l[nz]) == np.sign(c[nz]))


def test_higher_qp_fewer_nonzeros(nh):                            # :98-107
    from nano_hevc.quant import count_nonzero
    c = np.random.default_rng(1).integers(-100, 100, size=(4, 4)).astype(np.int32)
    c[0, 0] = 500
    assert count_nonzero(nh.quantize(c, 40, 4)) <= count_nonzero(nh.quantize(c, 10, 4))


def test_dequantize_zeros(nh):                                    # :113-120
    d = nh.dequantize(np.zeros((4, 4), np.int32), qp=20, size=4)
    assert d.shape == (4, 4) and not d.any()


def test_dequantize_nonzero(nh):                                  # :122-134
    d = nh.dequantize(np.diag([10, 5, 3, 1]).astype(np.int32), qp=20, size=4)
    assert all(d[i, i] != 0 for i in range(4))


def test_roundtrip_keeps_dc(nh):                                  # :140-156
    o = np.array([[500, 100, 50, 20], [100, 80, 30, 10], [50, 30, 20, 5], [20, 10, 5, 2]], np.int32)
    r = nh.dequantize(nh.quantize(o, qp=20, size=4), qp=20, size=4)
    assert abs(int(r[0, 0]) - 500) < 250


def test_roundtrip_low_qp(nh):                                    # :158-171
    o = np.array([[200, 100, 50, 25], [100, 80, 40, 20], [50, 40, 30, 15], [25, 20, 15, 10]], np.int32)
    r = nh.dequantize(nh.quantize(o, qp=5, size=4), qp=5, size=4)
    assert np.mean(np.abs(r - o)) < 50


def test_roundtrip_high_qp_sign(nh):                              # :173-182
    r = nh.dequantize(nh.quantize(np.full((4, 4), 100, np.int32), qp=45, size=4), qp=45, size=4)
    assert r[0, 0] == 0 or r[0, 0] > 0


@pytest.mark.parametrize("n", [8, 16, 32])
def test_quantize_block_sizes(nh, n):                             # :188-195
    c = np.random.default_rng(n).integers(-200, 200, size=(n, n)).astype(np.int32)
    l = nh.quantize(c, qp=20, size=n)
    assert l.shape == (n, n) and l.dtype == np.int32


def test_block_wrappers_infer_size(nh):                           # :201-217 (2 cases)
    rng = np.random.default_rng(2)
    c = rng.integers(-100, 100, size=(8, 8)).astype(np.int32)
    assert np.array_equal(nh.quantize(c, 20, 8), nh.quantize_block(c, 20))
    l = rng.integers(-10, 10, size=(8, 8)).astype(np.int32)
    assert np.array_equal(nh.dequantize(l, 20, 8), nh.dequantize_block(l, 20))


def test_level_helpers(nh):                                       # :223-240 (2 cases)
    from nano_hevc.quant import count_nonzero, is_all_zero
    assert count_nonzero(np.array([[10, 0, 0, 0], [0, 5, 0, 0], [0, 0, 0, 0], [0, 0, 0, 1]], np.int32)) == 3
    assert is_all_zero(np.zeros((4, 4), np.int32)) and not is_all_zero(np.array([[1, 0], [0, 0]], np.int32))


def test_six_qp_steps_halve_levels(nh):                           # :246-261
    from nano_hevc.quant import count_nonzero
    c = np.full((4, 4), 256, np.int32)
    lo, hi = nh.quantize(c, 10, 4), nh.quantize(c, 16, 4)
    assert count_nonzero(hi) <= count_nonzero(lo) and abs(int(hi[0, 0])) * 2 <= abs(int(lo[0, 0])) + 1


def test_intra_dead_zone_smaller(nh):                             # :267-277
    from nano_hevc.quant import count_nonzero
    c = np.full((4, 4), 50, np.int32)
    assert count_nonzero(nh.quantize(c, 30, 4, is_intra=True)) >= count_nonzero(nh.quantize(c, 30, 4, is_intra=False))


def test_quant_pipeline(nh):                                      # :283-322
    pred = nh.intra_dc_predict(TOP4, LEFT4, size=4)
    coeff = nh.forward_transform_4x4(nh.residual_block(ORIG, pred))
    rec_coeff = nh.dequantize(nh.quantize(coeff, qp=20, size=4), qp=20, size=4)
    rec = nh.reconstruct_block(pred, nh.inverse_transform_4x4(rec_coeff).astype(np.int16))
    assert np.max(np.abs(rec.astype(int) - ORIG)) < 20


# ---------------------------------------------------------------- test_transform.py (20 cases)

@pytest.mark.parametrize("name", ["DCT4", "DST4", "DCT8"])
def test_near_orthogonal(nh, name):                               # :27-52
    m = getattr(nh, name)
    g = m @ m.T
    d = np.diag(g)
    assert np.all(d > 0) and np.max(np.abs(g - np.diag(d))) < np.max(d) * 0.1


@pytest.mark.parametrize("n,dst", [(4, False), (8, False), (4, True)])
def test_forward_of_zeros(nh, n, dst):                            # :57-64
    c = nh.forward_transform(np.zeros((n, n), np.int16), use_dst=dst)
    assert c.shape == (n, n) and not c.any()


def test_flat_block_is_dc_only(nh):                               # :66-76
    c = nh.forward_transform_4x4(np.full((4, 4), 16, np.int16))
    ac = c.copy()
    ac[0, 0] = 0
    assert c[0, 0] != 0 and np.max(np.abs(ac)) <= abs(int(c[0, 0])) * 0.05


def test_forward_matches_explicit_products(nh):                   # :78-99
    x = np.array([[1, 2, 3, 4], [5, 6, 7, 8], [9, 0, -1, -2], [4, 3, 2, 1]], np.int16)
    T = nh.DCT4.astype(np.int64)
    ref = (((T @ x.astype(np.int64)) + 64) >> 7) @ T.T
    ref = (ref + 64) >> 7
    assert np.allclose(nh.forward_transform_4x4(x, use_dst=False), ref, atol=1)


def test_dst_differs_from_dct(nh):                                # :101-115
    x = np.add.outer(np.arange(4), np.arange(1, 5)).astype(np.int16)
    assert not np.array_equal(nh.forward_transform_4x4(x, use_dst=False), nh.forward_transform_4x4(x, use_dst=True))


@pytest.mark.parametrize("n", [4, 8])
def test_inverse_of_zeros(nh, n):                                 # :121-137
    inv = nh.inverse_transform_4x4 if n == 4 else nh.inverse_transform_8x8
    r = inv(np.zeros((n, n), np.int32))
    assert r.shape == (n, n) and not r.any()


SMALL = np.array([[5, 3, -2, 1], [2, 4, 1, -3], [-1, 2, 3, 2], [0, -1, 2, 4]], np.int16)


@pytest.mark.parametrize("dst", [False, True])
def test_roundtrip_4x4(nh, dst):                                  # :154-179
    r = nh.inverse_transform_4x4(nh.forward_transform_4x4(SMALL, use_dst=dst), use_dst=dst)
    assert np.max(np.abs(r - SMALL)) <= 2


@pytest.mark.parametrize("n,lim,mean_lim,max_lim", [(8, 50, 25, 50), (16, 50, 30, 60), (32, 30, 20, 40)])
def test_roundtrip_larger(nh, n, lim, mean_lim, max_lim):         # :181-216 (np.random.seed(42) draws)
    np.random.seed(42)
    x = np.random.randint(-lim, lim, size=(n, n), dtype=np.int16)
    err = np.abs(nh.inverse_transform(nh.forward_transform(x)) - x)
    assert np.mean(err) < mean_lim and np.max(err) <= max_lim


def test_energy_compaction_4x4(nh):                               # :222-238
    c = nh.forward_transform_4x4(np.add.outer(np.arange(10, 14), np.arange(4)).astype(np.int16))
    assert np.sum(c[:2, :2].astype(np.int64) ** 2) > np.sum(c[2:, 2:].astype(np.int64) ** 2)


def test_energy_compaction_8x8(nh):                               # :240-255
    c = nh.forward_transform_8x8(np.add.outer(np.arange(8), np.arange(8)).astype(np.int16)).astype(np.int64)
    assert np.sum(c[:4, :4] ** 2) > 0.9 * np.sum(c ** 2)


def test_dc_coefficient(nh):                                      # :261-274
    c = nh.forward_transform_4x4(np.full((4, 4), 10, np.int16))
    assert c[0, 0] != 0 and abs(int(c[0, 1])) < abs(int(c[0, 0])) * 0.1 and abs(int(c[1, 0])) < abs(int(c[0, 0])) * 0.1


def test_transform_pipeline(nh):                                  # :280-317
    pred = nh.intra_dc_predict(TOP4, LEFT4, size=4)
    rec_res = nh.inverse_transform_4x4(nh.forward_transform_4x4(nh.residual_block(ORIG, pred)))
    rec = nh.reconstruct_block(pred, rec_res.astype(np.int16))
    assert np.max(np.abs(rec.astype(int) - ORIG)) <= 2

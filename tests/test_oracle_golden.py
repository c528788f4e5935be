"""Pin the CPU restatement (oracle/) to the reference.

Two sources of truth, both data:
  * tests/golden/*.npz -- reference outputs recorded by tests/golden/make_golden.py;
  * the known answers the reference's own tests hold, restated
    here as literal vectors with the reference test file:line they come from.
CPU only (no GPU needed).
"""
import hashlib
import json
import os

import numpy as np
import pytest

from oracle import oracle as O

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def test_matrices(golden):
    g = golden("matrices.npz")
    assert np.array_equal(O.matrix(4, True), g["DST4"])
    for n in (4, 8, 16, 32):
        assert np.array_equal(O.matrix(n), g[f"DCT{n}"]), n
    with pytest.raises(ValueError):
        O.matrix(6)


@pytest.mark.parametrize("key,n,dst", [("n4_dst", 4, True), ("n4_dct", 4, False), ("n8_dct", 8, False),
                                       ("n16_dct", 16, False), ("n32_dct", 32, False)])
def test_transforms(golden, key, n, dst):
    g = golden("transform.npz")
    for x, y in zip(g[key + "_fwd_in"], g[key + "_fwd_out"]):
        assert np.array_equal(O.forward_transform(x, dst), y)
    for x, y in zip(g[key + "_inv_in"], g[key + "_inv_out"]):
        assert np.array_equal(O.inverse_transform(x, dst), y)


def test_quant(golden):
    g = golden("quant.npz")
    for a, qp in enumerate(g["q_qps"]):
        for b, size in enumerate([4, 8, 16, 32]):
            for c, intra in enumerate([True, False]):
                assert np.array_equal(O.quantize(g["q_vec32"], qp, size, intra), g["q_out32"][a, b, c]), (qp, size, intra)
                assert np.array_equal(O.quantize(g["q_vec16"], qp, size, intra), g["q_out16"][a, b, c]), (qp, size, intra)
        assert np.array_equal(O.dequantize(g["dq_in"], qp), g["dq_out"][a]), qp


@pytest.mark.parametrize("n", [4, 8, 16, 32])
def test_intra(golden, n):
    g = golden("intra.npz")
    for s in range(8):
        top = g[f"n{n}_top"][s, :g[f"n{n}_ntop"][s]]
        left = g[f"n{n}_left"][s, :g[f"n{n}_nleft"][s]]
        corner = int(g[f"n{n}_corner"][s])
        for m in range(35):
            st = g[f"n{n}_status"][s, m]
            exp = g[f"n{n}_pred"][s, m]
            if m == 0:
                t = top[:n] if top.size >= n else top
                l = left[:n] if left.size >= n else left
                fn = lambda: O.intra_planar(t, l, int(top[min(n, top.size) - 1]), int(left[min(n, left.size) - 1]), n)
            elif m == 1:
                fn = lambda: O.intra_dc(top, left, n)
            else:
                fn = lambda: O.intra_angular(top, left, corner, m, n)
            if st == 0:
                assert np.array_equal(fn(), exp), (n, s, m)
            else:
                with pytest.raises({1: OverflowError, 2: IndexError}[int(st)]):
                    fn()


def test_intra_quirks(golden):
    g = golden("intra.npz")
    t, l = g["quirk_top"], g["quirk_left"]
    assert np.array_equal(O.intra_angular(t, l, 77, 0, 4), g["quirk_ang0"])      # D10 modes 0/1
    assert np.array_equal(O.intra_angular(t, l, 77, 1, 4), g["quirk_ang1"])
    assert np.array_equal(O.intra_angular(t, l, 77, -5, 4), g["quirk_angm5"])
    assert np.array_equal(O.intra_dc(t, l, 4, variant4x4=True), g["quirk_dc4"])  # D7 whole-array sum
    assert np.array_equal(O.intra_dc(t, l, 4), g["quirk_dc4_len9"])
    with pytest.raises(IndexError):
        O.intra_angular(t, l, 77, 35, 4)
    assert np.array_equal(O.residual(g["rr_a"], g["rr_b"]), g["rr_res"])
    assert np.array_equal(O.reconstruct(g["rr_a"], g["rr_b"]), g["rr_rec"])
    for bd in [1, 8, 10, 12, 16, 40, 63]:
        assert np.array_equal(O.clip(g["clip_in"], bd), g[f"clip_bd{bd}"]), bd


def test_chain(golden):
    g = golden("chain.npz")
    pred = O.intra_dc(g["c1_top"], g["c1_left"], 4)
    assert np.array_equal(pred, g["c1_pred"])
    res = O.residual(g["c1_orig"], pred)
    assert np.array_equal(res, g["c1_res"])
    coeff = O.forward_transform(res, True)
    assert np.array_equal(coeff, g["c1_coeff"])
    for qp in (20, 22):
        lvl = O.quantize(coeff, qp, 4)
        assert np.array_equal(lvl, g[f"c1_lvl_qp{qp}"])
        deq = O.dequantize(lvl, qp)
        assert np.array_equal(deq, g[f"c1_deq_qp{qp}"])
        rres = O.inverse_transform(deq, True)
        assert np.array_equal(rres, g[f"c1_rres_qp{qp}"])
        rec = O.clip(O.reconstruct(pred, rres.astype(np.int16)), 8)
        assert np.array_equal(rec, g[f"c1_recon_qp{qp}"])


# ---- known answers from the reference's own tests (restated as data) ----

def test_reference_known_answers():
    # test_intra_dc.py:23-43 (DC = 101) and :45-56 variants
    assert np.all(O.intra_dc([102, 98, 100, 101], [103, 102, 101, 99], 4, variant4x4=True) == 101)
    assert np.all(O.intra_dc([1, 1, 1, 1], [1, 1, 1, 0], 4, variant4x4=True) == 1)
    assert np.all(O.intra_dc([100] * 8, [100] * 8, 8) == 100)                 # :62-70
    assert np.all(O.intra_dc([50] * 16, [50] * 16, 16) == 50)                 # :72-80
    # test_intra_dc.py:86-127 residual example
    orig = np.array([[102, 101, 100, 100], [103, 102, 101, 100], [103, 102, 100, 99], [104, 101, 99, 98]], np.int16)
    exp = np.array([[1, 0, -1, -1], [2, 1, 0, -1], [2, 1, -1, -2], [3, 0, -2, -3]], np.int16)
    assert np.array_equal(O.residual(orig, np.full((4, 4), 101, np.int16)), exp)
    # test_intra_dc.py:163-177 clip
    assert np.array_equal(O.clip([[-10, 0, 128, 255, 300]], 8), [[0, 0, 128, 255, 255]])
    assert np.array_equal(O.clip([[-10, 0, 512, 1023, 2000]], 10), [[0, 0, 512, 1023, 1023]])
    # test_intra_planar.py:56-76 corners
    p = O.intra_planar([0] * 4, [0] * 4, 255, 255, 4)
    assert p[0, 0] == 64 and p[3, 3] == 255
    for n, v in [(4, 100), (8, 128), (16, 200), (32, 50)]:                    # :78-86
        assert np.all(O.intra_planar([v] * n, [v] * n, v, v, n) == v)
    # test_intra_angular.py:69-85 mode 18 full matrix (pins D5)
    top = [0, 10, 20, 30, 40, 50, 60, 70, 80]
    left = [0, 5, 5, 5, 5, 5, 5, 5, 5]
    exp18 = np.array([[0, 10, 20, 30], [0, 0, 10, 20], [5, 0, 0, 10], [5, 5, 0, 0]])
    assert np.array_equal(O.intra_angular(top, left, 0, 18, 4), exp18)
    # :25-43 mode 26 with len-9 refs at sizes 4 and 8 (D6)
    t9 = [99, 100, 110, 120, 130, 0, 0, 0, 0]
    l9 = [99, 50, 50, 50, 50, 0, 0, 0, 0]
    for n in (4, 8):
        p = O.intra_angular(t9, l9, 99, 26, n)
        assert list(p[:, 0]) == [100] * n and list(p[:, 3]) == [130] * n
    # :45-67 mode 34, :111-133 mode 2
    p = O.intra_angular(top, [0] * 9, 0, 34, 4)
    assert (p[0, 0], p[0, 3], p[1, 0], p[3, 3]) == (20, 50, 30, 80)
    p = O.intra_angular([0] * 9, top, 0, 2, 4)
    assert (p[0, 0], p[3, 0], p[0, 1], p[3, 3]) == (20, 50, 30, 80)
    # :91-109 mode 10 rows
    p = O.intra_angular(l9, t9, 99, 10, 4)
    assert [int(p[i, 0]) for i in range(4)] == [100, 110, 120, 130]
    # :175-188 every mode on a flat reference
    for m in range(2, 35):
        assert np.all(O.intra_angular([128] * 9, [128] * 9, 128, m, 4) == 128)
    # test_quant.py:25-56 qp params via quantize's clamp: QP -5 == QP 0, QP 100 == QP 51
    v = np.array([1000, -1000, 77])
    assert np.array_equal(O.quantize(v, -5, 4), O.quantize(v, 0, 4))
    assert np.array_equal(O.quantize(v, 100, 4), O.quantize(v, 51, 4))
    # test_transform.py:57-64 zeros in, zeros out
    for n, d in [(4, False), (8, False), (4, True)]:
        assert not O.forward_transform(np.zeros((n, n), np.int16), d).any()


def test_planes(golden):
    g = golden("planes.npz")
    assert np.array_equal(O.fwd8x8_quant_plane(g["p2_small_in"]), g["p2_small_lvl"])
    assert np.array_equal(O.fwd8x8_quant_plane(g["p2_edge_in"], qp=0), g["p2_edge_lvl"])
    for k, qp in (("p3", 32), ("p3b", 22)):
        m, l, r, sse = O.intra_rdo_plane(g[f"{k}_src"], qp)
        assert np.array_equal(m, g[f"{k}_modes"]) and np.array_equal(l, g[f"{k}_lvl"])
        assert np.array_equal(r, g[f"{k}_rec"]) and sse == int(g[f"{k}_sse"])
    l, r, t = O.tu_pipeline_plane(g["p4y_src"], 32, 0, 1234, 32, True)
    assert np.array_equal(t, g["p4y_tu"]) and np.array_equal(l, g["p4y_lvl"]) and np.array_equal(r, g["p4y_rec"])
    l, r, t = O.tu_pipeline_plane(g["p4u_src"], 16, 1, 1234, 32, False)
    assert np.array_equal(t, g["p4u_tu"]) and np.array_equal(l, g["p4u_lvl"]) and np.array_equal(r, g["p4u_rec"])


def test_plane_hash_1080p():
    """sha256 of the reference's levels for a seeded 1080p plane."""
    man = json.load(open(os.path.join(GOLDEN, "manifest.json")))
    rng = np.random.default_rng(20260)
    plane = rng.integers(-255, 256, size=(1080, 1920)).astype(np.int16)
    lvl = O.fwd8x8_quant_plane(plane, 32)
    assert hashlib.sha256(lvl.tobytes()).hexdigest() == man["cfg2_1080p_qp32_seed20260_levels_sha256"]


def test_manifest_integrity():
    man = json.load(open(os.path.join(GOLDEN, "manifest.json")))
    assert man["numpy"].split(".")[0] == "2"      # NEP 50 semantics (D8)
    assert "metrics.npz" in man["files"]
    for name, h in man["files"].items():
        assert hashlib.sha256(open(os.path.join(GOLDEN, name), "rb").read()).hexdigest() == h, name


def test_cfg5_plane(golden):
    g = golden("cfg5.npz")
    for qp in (22, 37):
        l, r = O.tc32_plane(g["p5_src"], qp)
        assert np.array_equal(l, g[f"p5_lvl_qp{qp}"]) and np.array_equal(r, g[f"p5_rec_qp{qp}"]), qp


@pytest.mark.parametrize("threads", [2, 3, 8, 64])
def test_oracle_threaded_plane_equals_single(threads):
    """The all-cores CPU baseline (bench.py cpu_baseline) computes what the
    single-thread restatement does, ragged plane sizes included."""
    from oracle import oracle as O
    rng = np.random.default_rng(99)
    for h, w in ((72, 104), (37, 50), (8, 8), (7, 64)):
        r = rng.integers(-32768, 32768, (h, w)).astype(np.int16)
        assert np.array_equal(O.fwd8x8_quant_plane_mt(r, 27, False, threads), O.fwd8x8_quant_plane(r, 27, False))


# block sizes other than 4/8/16/32/64 recorded by make_golden.gen_encode (round 5);
# ("c", 12 / 10) are the reference's OverflowError cases (tests/test_frame_gpu.py)
ENC_ODD = {"a": (12, 24, 3, 9, 6, 20, 40, 0, -8, 128), "b": (12, 24, 5), "d": (12, 7, 24)}


def test_oracle_encode_frame_intra_golden(golden):
    """oh_encode_intra_plane against the reference's encode_frame_intra outputs
    (recon planes, stats, Y-PSNR) and the demo's printed totals."""
    g = golden("encode.npz")
    raw = g["e_a_yuv"]
    w, h = 72, 40
    ys, cs = w * h, (w // 2) * (h // 2)
    frames = {"a": (raw[:ys].reshape(h, w), raw[ys:ys + cs].reshape(h // 2, w // 2), raw[ys + cs:].reshape(h // 2, w // 2))}
    for t in "bcd":
        frames[t] = (g[f"e_{t}_y"], g[f"e_{t}_u"], g[f"e_{t}_v"])
    for tag, bss in (("a", (4, 8, 16, 32) + ENC_ODD["a"]), ("b", (4, 8, 16) + ENC_ODD["b"]), ("c", (8,)),
                     ("d", ENC_ODD["d"])):
        y, u, v = frames[tag]
        for bs in bss:
            k = f"e_{tag}_bs{bs}"
            (ry, ru, rv), st = O.encode_frame_intra(y, u, v, bs)
            for a, s in ((ry, "_ry"), (ru, "_ru"), (rv, "_rv")):
                assert np.array_equal(a, g[k + s]), (k, s)
            assert list(st[:3]) == list(g[k + "_stats"])
            _, sy = O.encode_intra_plane(y, max(4, bs))
            assert 10 * np.log10(255 ** 2 / (np.float64(sy[5]) / np.float64(y.size))) == g[k + "_psnr_y"]
    for key in ("d_64x64_bs8", "d_48x80_bs4", "d_72x40_bs16", "d_64x64_bs12", "d_48x80_bs6", "d_72x40_bs24"):
        _, st = O.encode_intra_plane(g[key + "_y"], int(key.split("bs")[1]))
        assert list(st[:5]) == list(g[key])
        assert f"{10 * np.log10(255 ** 2 / (np.float64(st[5]) / g[key + '_y'].size)):.2f}" == str(g[key + "_psnr_text"])


def test_oracle_at_full_size_equals_reference():
    """The CPU restatement at BASELINE sizes (1080p open + closed loop, 4K mixed
    TUs open + closed loop, 8K 32x32) hashes to the reference's outputs (tests/golden/fullsize.json,
    tests/golden/make_fullsize.py).  ~25 s."""
    import sys
    sys.path.insert(0, GOLDEN)
    import fullsize_inputs as FI

    def sha(a):
        return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()

    with open(os.path.join(GOLDEN, "fullsize.json")) as f:
        ref = json.load(f)
    for k, src in enumerate(FI.cfg3_frame()):
        m, l, r, s = O.intra_rdo_plane(src, FI.CFG3_QP)
        assert (sha(m), sha(l), sha(r), s) == tuple(ref[f"cfg3_p{k}"][x] for x in ("modes", "lvl", "rec", "sse")), k
        m, l, r, s = O.intra_rdo_plane(src, FI.CLOSED_QP, closed=True)
        assert (sha(m), sha(l), sha(r), s) == tuple(ref[f"closed_p{k}"][x] for x in ("modes", "lvl", "rec", "sse")), k
    for k, src in enumerate(FI.cfg4_frame()):
        l, r, t = O.tu_pipeline_plane(src, 32 if k == 0 else 16, k, FI.CFG4_SEED, FI.CFG4_QP, k == 0)
        assert (sha(l), sha(r), sha(t)) == tuple(ref[f"cfg4_p{k}"][x] for x in ("lvl", "rec", "tu")), k
    l, r = O.tc32_plane(FI.cfg5_plane(), FI.CFG5_QP)
    assert (sha(l), sha(r)) == (ref["cfg5_y"]["lvl"], ref["cfg5_y"]["rec"])
    for name, src in zip("uv", FI.cfg5_chroma()):   # 8K chroma planes
        l, r = O.tc32_plane(src, FI.CFG5_QP)
        assert (sha(l), sha(r)) == (ref[f"cfg5_{name}"]["lvl"], ref[f"cfg5_{name}"]["rec"]), name
    for k, src in enumerate(FI.cfg2_frame()):   # the headline config on one 4K YUV420 frame
        assert sha(O.fwd8x8_quant_plane(src, FI.CFG2_QP)) == ref[f"cfg2_4k_p{k}"]["lvl"], k
    for k, src in enumerate(FI.cfg4_frame()):   # config 4 in closed loop
        l, r, t = O.tu_pipeline_plane_closed(src, 32 if k == 0 else 16, k, FI.CFG4_SEED, FI.CFG4_QP, k == 0)
        assert (sha(l), sha(r), sha(t)) == tuple(ref[f"closed4_p{k}"][x] for x in ("lvl", "rec", "tu")), k


def test_oracle_tu_pipeline_closed_golden(golden):
    """Closed-loop config 4: the oracle equals planes composed
    from the reference's own BlockView / Plane / predictors / chain
    (make_golden.gen_closed4); the open-loop pipeline differs on every case."""
    g = golden("closed4.npz")
    for k in ("k4y", "k4u", "k4n", "k4r"):
        args = (g[k + "_src"], int(g[k + "_ctb"]), int(g[k + "_pid"]), 1234, int(g[k + "_qp"]), bool(g[k + "_luma"]))
        lvl, rec, tu = O.tu_pipeline_plane_closed(*args)
        assert np.array_equal(lvl, g[k + "_lvl"]) and np.array_equal(rec, g[k + "_rec"]), k
        assert np.array_equal(tu, g[k + "_tu"]), k
        assert not np.array_equal(O.tu_pipeline_plane(*args)[1], rec), k

"""Generate the golden fixtures in tests/golden/ by running the REFERENCE.

Run in the build container only (the reference never travels to the GPU box):

    python tests/golden/make_golden.py [/root/reference]

It imports the reference ``nano_hevc`` package (pure Python + numpy) and records
inputs and reference outputs as data (.npz) plus a manifest with the numpy
version (NEP 50 promotion matters: SURVEY.md §0.1 D8).  Fixture plan: SURVEY.md
§8(c) C4.  Frame-level fixtures (cfg 3 / cfg 4) compose the reference
functions exactly as DESIGN.md §3.3/§3.4 define the drivers.
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
import warnings

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def _import_reference(path):
    sys.path.insert(0, path)
    import nano_hevc  # noqa: F401  (the reference package)
    from nano_hevc import intra, transform, quant, metrics
    assert os.path.abspath(intra.__file__).startswith(os.path.abspath(path)), intra.__file__
    return intra, transform, quant, metrics


def _err(fn):
    try:
        return ("ok", fn())
    except Exception as e:  # record the reference's exception type
        return ("err", type(e).__name__)


def gen_matrices(T):
    return {"DST4": T.DST4, "DCT4": T.DCT4, "DCT8": T.DCT8, "DCT16": T.DCT16, "DCT32": T.DCT32}


def gen_transform(T, rng):
    out = {}
    for n, dst in [(4, True), (4, False), (8, False), (16, False), (32, False)]:
        key = f"n{n}_{'dst' if dst else 'dct'}"
        blocks = [rng.integers(-255, 256, size=(n, n)) for _ in range(48)]
        cb = np.indices((n, n)).sum(0) % 2
        blocks += [255 * (2 * cb - 1), -255 * (2 * cb - 1), np.zeros((n, n), int),
                   np.full((n, n), 32767), np.full((n, n), -32768),
                   32767 * (2 * cb - 1), rng.integers(-32768, 32768, size=(n, n)),
                   rng.integers(-32768, 32768, size=(n, n))]
        fin = np.stack(blocks).astype(np.int16)
        fout = np.stack([T.forward_transform(b, use_dst=dst) for b in fin])
        # inverse inputs: forward outputs + raw int32 coefficients (wrap cases)
        raw = [rng.integers(-2000, 2001, size=(n, n)) for _ in range(16)]
        raw += [rng.integers(-2**31, 2**31, size=(n, n), dtype=np.int64) for _ in range(8)]
        raw += [np.full((n, n), 2**31 - 1), np.full((n, n), -2**31)]
        iin = np.concatenate([fout, np.stack(raw).astype(np.int32)])
        iout = np.stack([T.inverse_transform(b, use_dst=dst) for b in iin])
        out[key + "_fwd_in"] = fin
        out[key + "_fwd_out"] = fout.astype(np.int32)
        out[key + "_inv_in"] = iin
        out[key + "_inv_out"] = iout.astype(np.int32)
    return out


def gen_quant(Q, rng):
    vec32 = np.concatenate([
        np.array([0, 1, -1, 2, -2, 5, -5, 1020, -1020, 32767, -32768, 2**31 - 1, -2**31,
                  131072, -131072, 1 << 20, -(1 << 20)]),
        rng.integers(-2000, 2001, size=200), rng.integers(-2**31, 2**31, size=39, dtype=np.int64),
    ]).astype(np.int32)
    vec16 = np.concatenate([np.array([0, 1, -1, 32767, -32768, -32767]),
                            rng.integers(-32768, 32768, size=58)]).astype(np.int16)
    qps = list(range(0, 52)) + [-5, 60]
    out = {"q_vec32": vec32, "q_vec16": vec16, "q_qps": np.array(qps)}
    q32 = np.zeros((len(qps), 4, 2, vec32.size), np.int32)
    q16 = np.zeros((len(qps), 4, 2, vec16.size), np.int32)
    for a, qp in enumerate(qps):
        for b, size in enumerate([4, 8, 16, 32]):
            for c, intra in enumerate([True, False]):
                q32[a, b, c] = Q.quantize(vec32, qp, size, intra)
                q16[a, b, c] = Q.quantize(vec16, qp, size, intra)
    out["q_out32"], out["q_out16"] = q32, q16
    lv = np.concatenate([np.array([0, 1, -1, 100, -100, 32767, -32768, 2**31 - 1, -2**31]),
                         rng.integers(-3000, 3001, size=100),
                         rng.integers(-2**31, 2**31, size=19, dtype=np.int64)]).astype(np.int32)
    out["dq_in"] = lv
    out["dq_out"] = np.stack([Q.dequantize(lv, qp, 4) for qp in qps]).astype(np.int32)
    out["qp_params"] = np.array([Q.get_qp_params(q) for q in range(-3, 56)])
    return out


def gen_intra(I, rng):
    """Predictions for modes 0..34 x N in {4,8,16,32} x 8 reference sets."""
    out = {}
    for n in [4, 8, 16, 32]:
        sets = []
        for s in range(8):
            if s < 4:
                top = rng.integers(0, 256, size=2 * n + 1)
                left = rng.integers(0, 256, size=2 * n + 1)
            elif s == 4:   # short refs (D6): replicate-last and secondary gating
                top = rng.integers(0, 256, size=n + 1)
                left = rng.integers(0, 256, size=max(2, n // 2))
            elif s == 5:   # 2000-valued refs: int16 wrap in interpolation (D8)
                top = rng.integers(1800, 2200, size=2 * n + 1)
                left = rng.integers(1800, 2200, size=2 * n + 1)
            elif s == 6:   # 10-bit content
                top = rng.integers(0, 1024, size=2 * n + 1)
                left = rng.integers(0, 1024, size=2 * n + 1)
            else:          # near int16 extremes
                top = rng.integers(-32768, 32768, size=2 * n + 1)
                left = rng.integers(-32768, 32768, size=2 * n + 1)
            corner = int(rng.integers(0, 256)) if s != 7 else int(rng.integers(-32768, 32768))
            sets.append((top.astype(np.int16), left.astype(np.int16), corner))
        tops = np.full((8, 2 * n + 1), -1, np.int16)
        lefts = np.full((8, 2 * n + 1), -1, np.int16)
        ntop = np.zeros(8, np.int64)
        nleft = np.zeros(8, np.int64)
        corners = np.zeros(8, np.int64)
        pred = np.zeros((8, 35, n, n), np.int16)
        status = np.zeros((8, 35), np.int8)       # 0 ok, 1 OverflowError
        for s, (top, left, corner) in enumerate(sets):
            tops[s, :top.size], lefts[s, :left.size] = top, left
            ntop[s], nleft[s], corners[s] = top.size, left.size, corner
            for m in range(35):
                if m == 0:
                    r = _err(lambda: I.intra_planar_predict(top[:n] if top.size >= n else top, left[:n] if left.size >= n else left,
                                                            int(top[min(n, top.size) - 1]), int(left[min(n, left.size) - 1]), n))
                elif m == 1:
                    r = _err(lambda: I.intra_dc_predict(top, left, n))
                else:
                    r = _err(lambda: I.intra_angular_predict(top, left, corner, m, n))
                if r[0] == "ok":
                    pred[s, m] = r[1]
                else:
                    status[s, m] = {"OverflowError": 1, "IndexError": 2}.get(r[1], 9)
        out[f"n{n}_top"], out[f"n{n}_left"] = tops, lefts
        out[f"n{n}_ntop"], out[f"n{n}_nleft"], out[f"n{n}_corner"] = ntop, nleft, corners
        out[f"n{n}_pred"], out[f"n{n}_status"] = pred, status
    # quirk modes 0/1 through the angular entry (D10) and the 4x4 DC variant
    top = rng.integers(0, 256, size=9).astype(np.int16)
    left = rng.integers(0, 256, size=9).astype(np.int16)
    out["quirk_top"], out["quirk_left"] = top, left
    out["quirk_ang0"] = I.intra_angular_predict(top, left, 77, 0, 4)
    out["quirk_ang1"] = I.intra_angular_predict(top, left, 77, 1, 4)
    out["quirk_angm5"] = I.intra_angular_predict(top, left, 77, -5, 4)
    out["quirk_dc4"] = I.intra_dc_predict_4x4(top, left)
    out["quirk_dc4_len9"] = I.intra_dc_predict(top, left, 4)
    # residual / reconstruct / clip vectors
    a = rng.integers(-32768, 32768, size=300).astype(np.int16)
    b = rng.integers(-32768, 32768, size=300).astype(np.int16)
    out["rr_a"], out["rr_b"] = a, b
    out["rr_res"], out["rr_rec"] = I.residual_block(a, b), I.reconstruct_block(a, b)
    cv = np.concatenate([np.array([-2**40, -1, 0, 1, 255, 256, 1023, 1024, 32767, 65535, 70000, 2**40]),
                         rng.integers(-5000, 70000, size=100)]).astype(np.int64)
    out["clip_in"] = cv
    for bd in [1, 8, 10, 12, 16, 40, 63]:
        out[f"clip_bd{bd}"] = I.clip_to_pixel_range(cv, bd)
    return out


def gen_chain(I, T, Q):
    """Config-1 chain (README.md:44-71, test_quant.py:283-322)."""
    top = np.array([102, 98, 100, 101], dtype=np.int16)
    left = np.array([103, 102, 101, 99], dtype=np.int16)
    orig = np.array([[102, 101, 100, 100], [103, 102, 101, 100], [103, 102, 100, 99], [104, 101, 99, 98]], dtype=np.int16)
    out = {"c1_top": top, "c1_left": left, "c1_orig": orig}
    pred = I.intra_dc_predict(top, left, 4)
    res = I.residual_block(orig, pred)
    for qp in [20, 22]:
        coeff = T.forward_transform(res, use_dst=True)
        lvl = Q.quantize_block(coeff, qp)
        deq = Q.dequantize_block(lvl, qp)
        rres = T.inverse_transform(deq, use_dst=True)
        recon = I.clip_to_pixel_range(I.reconstruct_block(pred, rres.astype(np.int16)))
        out.update({f"c1_pred": pred, f"c1_res": res, f"c1_coeff": coeff, f"c1_lvl_qp{qp}": lvl,
                    f"c1_deq_qp{qp}": deq, f"c1_rres_qp{qp}": rres, f"c1_recon_qp{qp}": recon})
    return out


def ref_plane_cfg2(T, Q, plane, qp=32):
    h, w = plane.shape
    lvl = np.zeros_like(plane)
    for by in range(0, h - 7, 8):
        for bx in range(0, w - 7, 8):
            c = T.forward_transform(plane[by:by + 8, bx:bx + 8])
            lvl[by:by + 8, bx:bx + 8] = Q.quantize_block(c, qp)
    return lvl


def _neighbors(src, x, y, count):
    """block.py:38-55 with count (numpy slices truncate at the plane edge)."""
    top = np.full(count, 128, src.dtype) if y == 0 else src[y - 1, x:x + count].copy()
    left = np.full(count, 128, src.dtype) if x == 0 else src[y:y + count, x - 1].copy()
    tl = 128 if (y == 0 or x == 0) else int(src[y - 1, x - 1])
    return top, left, tl


def _chain(I, T, Q, orig, pred, qp, use_dst):
    res = I.residual_block(orig, pred)
    lvl = Q.quantize_block(T.forward_transform(res, use_dst=use_dst), qp)
    rres = T.inverse_transform(Q.dequantize_block(lvl, qp), use_dst=use_dst)
    rec = I.clip_to_pixel_range(I.reconstruct_block(pred, rres.astype(np.int16)), 8)
    sse = int(np.sum(I.residual_block(orig, rec).astype(np.int64) ** 2))
    return lvl, rec, sse


def ref_plane_cfg3(I, T, Q, src, qp, rows=None):
    """rows = (first, last) block rows to compute (open loop: rows are
    independent); outside them the outputs stay 0."""
    h, w = src.shape
    n = 8
    modes = np.zeros((h // n, w // n), np.uint8)
    lvl = np.zeros(src.shape, np.int32)
    rec = np.zeros(src.shape, np.int16)
    total = 0
    r0, r1 = rows if rows else (0, h // n)
    for by in range(r0 * n, min(h - n + 1, r1 * n), n):
        for bx in range(0, w - n + 1, n):
            orig = src[by:by + n, bx:bx + n]
            top, left, tl = _neighbors(src, bx, by, n)
            top2, left2, _ = _neighbors(src, bx, by, 2 * n)
            topa = np.concatenate([[tl], top2]).astype(np.int16)
            lefta = np.concatenate([[tl], left2]).astype(np.int16)
            best = None
            for m in range(35):
                if m == 0:
                    pred = I.intra_planar_predict(top, left, int(top[-1]), int(left[-1]), n)
                elif m == 1:
                    pred = I.intra_dc_predict(top, left, n)
                else:
                    pred = I.intra_angular_predict(topa, lefta, tl, m, n)
                l, r, sse = _chain(I, T, Q, orig, pred, qp, False)
                if best is None or sse < best[0]:
                    best = (sse, m, l, r)
            total += best[0]
            modes[by // n, bx // n] = best[1]
            lvl[by:by + n, bx:bx + n] = best[2]
            rec[by:by + n, bx:bx + n] = best[3]
    return modes, lvl, rec, total


def _mix32(x):
    x &= 0xFFFFFFFF
    x ^= x >> 16; x = (x * 0x7feb352d) & 0xFFFFFFFF
    x ^= x >> 15; x = (x * 0x846ca68b) & 0xFFFFFFFF
    x ^= x >> 16
    return x


def tu_split(seed, plane_id, x, y, size):
    k = _mix32(seed ^ ((0x9E3779B9 * (plane_id + 1)) & 0xFFFFFFFF))
    k = _mix32(k ^ x)
    k = _mix32(k ^ ((y * 0x85ebca6b) & 0xFFFFFFFF))
    k = _mix32(k ^ size)
    return (k & 3) < 2


def ref_plane_cfg4(I, T, Q, src, ctb, plane_id, seed, qp, is_luma, ctu_rows=None):
    """ctu_rows = (first, last) CTU rows to compute (open loop: independent)."""
    h, w = src.shape
    lvl = np.zeros(src.shape, np.int32)
    rec = np.zeros(src.shape, np.int16)
    tul = np.zeros((h // 4, w // 4), np.uint8)

    def one(x, y, n):
        orig = src[y:y + n, x:x + n]
        top, left, _ = _neighbors(src, x, y, n)
        dc = I.intra_dc_predict(top, left, n)
        pl = I.intra_planar_predict(top, left, int(top[-1]), int(left[-1]), n)
        edc = int(np.sum(I.residual_block(orig, dc).astype(np.int64) ** 2))
        epl = int(np.sum(I.residual_block(orig, pl).astype(np.int64) ** 2))
        pred = dc if edc <= epl else pl
        l, r, _ = _chain(I, T, Q, orig, pred, qp, bool(is_luma and n == 4))
        lvl[y:y + n, x:x + n] = l
        rec[y:y + n, x:x + n] = r
        tul[y // 4:(y + n) // 4, x // 4:(x + n) // 4] = int(np.log2(n))

    def tree(x, y, s):
        if x >= w or y >= h:
            return
        over = (x + s > w) or (y + s > h)
        if s > 4 and (over or tu_split(seed, plane_id, x, y, s)):
            hs = s // 2
            for dy in (0, hs):
                for dx in (0, hs):
                    tree(x + dx, y + dy, hs)
            return
        if not over:
            one(x, y, s)

    c0, c1 = ctu_rows if ctu_rows else (0, (h + ctb - 1) // ctb)
    for cy in range(c0, c1):
        for cx in range((w + ctb - 1) // ctb):
            tree(cx * ctb, cy * ctb, ctb)
    return lvl, rec, tul


def gen_planes(I, T, Q, rng):
    out = {}
    # cfg 2: full 1080p residual plane -> sha256 of levels; plus a small plane in full
    small = rng.integers(-255, 256, size=(72, 136)).astype(np.int16)   # 136 % 8 == 0, 72 rows
    out["p2_small_in"] = small
    out["p2_small_lvl"] = ref_plane_cfg2(T, Q, small)
    edge = rng.integers(-32768, 32768, size=(16, 24)).astype(np.int16)
    out["p2_edge_in"], out["p2_edge_lvl"] = edge, ref_plane_cfg2(T, Q, edge, qp=0)
    # cfg 3: small YUV-like source plane with gradients + noise, and an edge-case plane
    yy, xx = np.mgrid[0:40, 0:56]
    src = np.clip(60 + 2 * xx + yy + rng.integers(-12, 13, size=xx.shape), 0, 255).astype(np.int16)
    m, l, r, tot = ref_plane_cfg3(I, T, Q, src, 32)
    out.update(p3_src=src, p3_modes=m, p3_lvl=l, p3_rec=r, p3_sse=np.int64(tot))
    src2 = rng.integers(0, 256, size=(20, 28)).astype(np.int16)        # partial edge blocks skipped
    m, l, r, tot = ref_plane_cfg3(I, T, Q, src2, 22)
    out.update(p3b_src=src2, p3b_modes=m, p3b_lvl=l, p3b_rec=r, p3b_sse=np.int64(tot))
    # cfg 4: small luma (ctb 32) and chroma (ctb 16) planes with partial CTUs
    yy, xx = np.mgrid[0:80, 0:104]
    lum = np.clip(100 + xx - yy + rng.integers(-20, 21, size=xx.shape), 0, 255).astype(np.int16)
    l, r, t = ref_plane_cfg4(I, T, Q, lum, 32, 0, 1234, 32, True)
    out.update(p4y_src=lum, p4y_lvl=l, p4y_rec=r, p4y_tu=t)
    chro = rng.integers(90, 170, size=(40, 52)).astype(np.int16)
    l, r, t = ref_plane_cfg4(I, T, Q, chro, 16, 1, 1234, 32, False)
    out.update(p4u_src=chro, p4u_lvl=l, p4u_rec=r, p4u_tu=t)
    return out


def gen_cfg5(I, T, Q, M):
    """cfg 5: every full 32x32 block through the cfg-4 chain,
    plus the reference's Y-PSNR of the reconstruction (metrics.psnr)."""
    rng = np.random.default_rng(555)
    yy, xx = np.mgrid[0:72, 0:104]
    src = np.clip(110 + 2 * xx - yy + rng.integers(-30, 31, size=xx.shape), 0, 255).astype(np.int16)
    out = {"p5_src": src}
    for qp in (22, 37):
        lvl = np.zeros(src.shape, np.int32)
        rec = np.zeros(src.shape, np.int16)
        for by in range(0, src.shape[0] - 31, 32):
            for bx in range(0, src.shape[1] - 31, 32):
                orig = src[by:by + 32, bx:bx + 32]
                top, left, _ = _neighbors(src, bx, by, 32)
                dc = I.intra_dc_predict(top, left, 32)
                pl = I.intra_planar_predict(top, left, int(top[-1]), int(left[-1]), 32)
                edc = int(np.sum(I.residual_block(orig, dc).astype(np.int64) ** 2))
                epl = int(np.sum(I.residual_block(orig, pl).astype(np.int64) ** 2))
                l, r, _ = _chain(I, T, Q, orig, dc if edc <= epl else pl, qp, False)
                lvl[by:by + 32, bx:bx + 32] = l
                rec[by:by + 32, bx:bx + 32] = r
        h32, w32 = 64, 96
        out[f"p5_lvl_qp{qp}"], out[f"p5_rec_qp{qp}"] = lvl, rec
        out[f"p5_psnr_qp{qp}"] = np.float64(M.psnr(src[:h32, :w32].astype(np.uint8), rec[:h32, :w32].astype(np.uint8)))
    return out


def gen_metrics(M):
    """metrics.py:7-48 on seeded integer samples (its own rng: other fixtures unchanged)."""
    rng = np.random.default_rng(4321)
    out = {}
    a8 = rng.integers(0, 256, size=(6, 64, 64)).astype(np.uint8)
    b8 = np.clip(a8.astype(np.int16) + rng.integers(-20, 21, size=a8.shape), 0, 255).astype(np.uint8)
    out["m_a8"], out["m_b8"] = a8, b8
    out["m_mse"] = np.array([M.mse(x, y) for x, y in zip(a8, b8)])
    out["m_psnr"] = np.array([M.psnr(x, y) for x, y in zip(a8, b8)])
    out["m_psnr1023"] = np.array([M.psnr(x, y, peak=1023) for x, y in zip(a8, b8)])
    a16 = rng.integers(-32768, 32768, size=(4, 100)).astype(np.int16)
    b16 = rng.integers(-32768, 32768, size=(4, 100)).astype(np.int16)
    out["m_a16"], out["m_b16"] = a16, b16
    out["m_mse16"] = np.array([M.mse(x, y) for x, y in zip(a16, b16)])
    out["m_sad16"] = np.array([M.sad(x, y) for x, y in zip(a16, b16)])
    out["m_energy16"] = np.array([M.residual_energy(x) for x in a16])
    a32 = rng.integers(-2**31, 2**31, size=(4, 16), dtype=np.int64).astype(np.int32)
    b32 = rng.integers(-2**31, 2**31, size=(4, 16), dtype=np.int64).astype(np.int32)
    out["m_a32"], out["m_b32"] = a32, b32
    out["m_sad32"] = np.array([M.sad(x, y) for x, y in zip(a32, b32)])            # int32 wrap
    out["m_satd32"] = np.array([M.satd_4x4(x, y) for x, y in zip(a32, b32)])
    s4a = rng.integers(0, 256, size=(8, 4, 4))
    s4b = rng.integers(0, 256, size=(8, 4, 4))
    out["m_s4a"], out["m_s4b"] = s4a, s4b
    out["m_satd"] = np.array([M.satd_4x4(x, y) for x, y in zip(s4a, s4b)])
    e64 = rng.integers(-2**40, 2**40, size=(3, 50), dtype=np.int64)
    out["m_e64"] = e64
    out["m_energy64"] = np.array([M.residual_energy(x) for x in e64])              # int64 wrap
    return out


def gen_encode(ref_path):
    """The reference's frame-level intra driver (__main__.py:142-189,
    encode_frame_intra: DC vs planar per block, open loop, recon = clip(best
    pred), partial blocks left 0) and the demo's totals (__main__.py:55-139,
    parsed from its printed report).  Own rng (other fixtures unchanged)."""
    import contextlib
    import io
    import re
    from nano_hevc import __main__ as R   # the reference's driver module
    from nano_hevc.frame import Frame, Plane
    assert os.path.abspath(R.__file__).startswith(os.path.abspath(ref_path)), R.__file__
    rng = np.random.default_rng(777)
    out = {}
    cases = []
    # (a) random 8-bit YUV420p bytes with ragged dims (partial blocks at 16/32)
    w, h = 72, 40
    raw = rng.integers(0, 256, size=w * h * 3 // 2).astype(np.uint8).tobytes()
    out["e_a_yuv"] = np.frombuffer(raw, np.uint8).copy()
    for bs in (4, 8, 16, 32):
        cases.append(("a", bs, Frame.from_yuv420p(raw, h, w)))
    # (b) the reference's demo frame (int16 planes)
    fb = R.create_test_frame(48, 80)
    out["e_b_y"], out["e_b_u"], out["e_b_v"] = fb.y.data, fb.u.data, fb.v.data
    for bs in (4, 8, 16):
        cases.append(("b", bs, fb))
    # (c) full-range int16 planes (residual_block's int16 wrap)
    fc = Frame(Plane(rng.integers(-32768, 32768, size=(32, 48)).astype(np.int16)),
               Plane(rng.integers(-32768, 32768, size=(16, 24)).astype(np.int16)),
               Plane(rng.integers(-32768, 32768, size=(16, 24)).astype(np.int16)))
    out["e_c_y"], out["e_c_u"], out["e_c_v"] = fc.y.data, fc.u.data, fc.v.data
    cases.append(("c", 8, fc))
    for tag, bs, fr in cases:
        recon, stats = R.encode_frame_intra(fr, bs)
        k = f"e_{tag}_bs{bs}"
        out[k + "_ry"], out[k + "_ru"], out[k + "_rv"] = recon.y.data, recon.u.data, recon.v.data
        out[k + "_stats"] = np.array([stats["blocks"], stats["dc"], stats["planar"]], np.int64)
        out[k + "_psnr_y"] = np.float64(R.psnr(fr.y.data.astype(np.uint8), recon.y.data.astype(np.uint8)))
    # demo_predictions report (luma only): wins and total energies, PSNR text
    for (dh, dw, bs) in ((64, 64, 8), (48, 80, 4), (72, 40, 16)):
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            R.demo_predictions(dh, dw, bs)
        txt = buf.getvalue()
        out[f"d_{dh}x{dw}_bs{bs}_y"] = R.create_test_frame(dh, dw).y.data
        num = lambda pat: int(re.search(pat, txt).group(1).replace(",", ""))
        out[f"d_{dh}x{dw}_bs{bs}"] = np.array([
            num(r"Total blocks:\s+(\d+)"), num(r"DC wins:\s+(\d+)"), num(r"Planar wins:\s+(\d+)"),
            num(r"DC total residual energy:\s+([\d,]+)"), num(r"Planar total residual energy:\s+([\d,]+)")], np.int64)
        out[f"d_{dh}x{dw}_bs{bs}_psnr_text"] = np.array(re.search(r"PSNR \(best mode\): (\S+) dB", txt).group(1))
    # round 5 (VERDICT r4 missing #3): block sizes other than 4/8/16/32/64 -- the
    # reference's driver takes any block_size (luma max(4, bs), chroma
    # max(4, bs // 2)); (d) a 10-bit-range int16 frame, where planar's
    # non-normalised weights at odd sizes can overflow int16 (OverflowError)
    fd = Frame(Plane(rng.integers(0, 1024, size=(40, 56)).astype(np.int16)),
               Plane(rng.integers(0, 1024, size=(20, 28)).astype(np.int16)),
               Plane(rng.integers(0, 1024, size=(20, 28)).astype(np.int16)))
    out["e_d_y"], out["e_d_u"], out["e_d_v"] = fd.y.data, fd.u.data, fd.v.data
    more = [("a", bs, Frame.from_yuv420p(raw, h, w)) for bs in (12, 24, 3, 9, 6, 20, 40, 0, -8, 128)]
    more += [("b", bs, fb) for bs in (12, 24, 5)]
    more += [("c", bs, fc) for bs in (12, 10)]
    more += [("d", bs, fd) for bs in (12, 7, 24)]
    for tag, bs, fr in more:
        k = f"e_{tag}_bs{bs}"
        try:
            recon, stats = R.encode_frame_intra(fr, bs)
        except Exception as e:   # the reference's exception class (planar's int16 store)
            out[k + "_err"] = np.array(type(e).__name__)
            continue
        out[k + "_ry"], out[k + "_ru"], out[k + "_rv"] = recon.y.data, recon.u.data, recon.v.data
        out[k + "_stats"] = np.array([stats["blocks"], stats["dc"], stats["planar"]], np.int64)
        out[k + "_psnr_y"] = np.float64(R.psnr(fr.y.data.astype(np.uint8), recon.y.data.astype(np.uint8)))
    for (dh, dw, bs) in ((64, 64, 12), (48, 80, 6), (72, 40, 24)):
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            R.demo_predictions(dh, dw, bs)
        txt = buf.getvalue()
        out[f"d_{dh}x{dw}_bs{bs}_y"] = R.create_test_frame(dh, dw).y.data
        num = lambda pat: int(re.search(pat, txt).group(1).replace(",", ""))
        out[f"d_{dh}x{dw}_bs{bs}"] = np.array([
            num(r"Total blocks:\s+(\d+)"), num(r"DC wins:\s+(\d+)"), num(r"Planar wins:\s+(\d+)"),
            num(r"DC total residual energy:\s+([\d,]+)"), num(r"Planar total residual energy:\s+([\d,]+)")], np.int64)
        out[f"d_{dh}x{dw}_bs{bs}_psnr_text"] = np.array(re.search(r"PSNR \(best mode\): (\S+) dB", txt).group(1))
    return out


def gen_closed(I, T, Q):
    """Closed-loop config 3, composed from the reference's own
    pieces: raster block order, neighbours fetched with BlockView
    (block.py:38-55) from the reconstruction Plane built so far
    (Plane.zeros, frame.py:41-43), left reference = get_left_neighbors(N)
    (the reconstructed samples only), top = get_top_neighbors(2N).  Own rng."""
    from nano_hevc.block import BlockView
    from nano_hevc.frame import Plane
    rng = np.random.default_rng(9090)
    out = {}
    yy, xx = np.mgrid[0:48, 0:72]
    cases = {"c3a": (np.clip(70 + 2 * xx + yy + rng.integers(-15, 16, size=xx.shape), 0, 255).astype(np.int16), 32),
             "c3b": (rng.integers(0, 256, size=(29, 37)).astype(np.int16), 22),       # partial blocks
             "c3c": (np.clip(128 + ((xx // 8 + yy // 8) % 2) * 90 - 45 + rng.integers(-3, 4, size=xx.shape),
                             0, 255).astype(np.int16), 37)}
    n = 8
    for key, (src, qp) in cases.items():
        h, w = src.shape
        recon = Plane.zeros(h, w, np.int16)
        modes = np.zeros((h // n, w // n), np.uint8)
        lvl = np.zeros(src.shape, np.int32)
        total = 0
        for by in range(0, h - n + 1, n):
            for bx in range(0, w - n + 1, n):
                blk = BlockView(recon, bx, by, n)
                orig = src[by:by + n, bx:bx + n]
                top, left, tl = blk.get_top_neighbors(), blk.get_left_neighbors(), blk.get_top_left_neighbor()
                topa = np.concatenate([[tl], blk.get_top_neighbors(2 * n)]).astype(np.int16)
                lefta = np.concatenate([[tl], blk.get_left_neighbors(n)]).astype(np.int16)
                best = None
                for m in range(35):
                    if m == 0:
                        pred = I.intra_planar_predict(top, left, int(top[-1]), int(left[-1]), n)
                    elif m == 1:
                        pred = I.intra_dc_predict(top, left, n)
                    else:
                        pred = I.intra_angular_predict(topa, lefta, tl, m, n)
                    l, r, sse = _chain(I, T, Q, orig, pred, qp, False)
                    if best is None or sse < best[0]:
                        best = (sse, m, l, r)
                total += best[0]
                modes[by // n, bx // n] = best[1]
                lvl[by:by + n, bx:bx + n] = best[2]
                blk.write_pixels(best[3])
        out.update({f"{key}_src": src, f"{key}_qp": np.int64(qp), f"{key}_modes": modes, f"{key}_lvl": lvl,
                    f"{key}_rec": recon.data, f"{key}_sse": np.int64(total)})
    return out


def ref_plane_cfg4_closed(I, T, Q, src, ctb, plane_id, seed, qp, is_luma):
    """Closed-loop config 4, composed from the reference's own
    pieces: CTUs in raster order, TUs in quadtree z-order, every TU's top / left
    neighbours (N samples each) fetched with BlockView (block.py:38-50) from the
    reconstruction Plane built so far (Plane.zeros, frame.py:41-43), then the
    open-loop TU's DC-vs-planar choice and chain, recon written back with
    BlockView.write_pixels."""
    from nano_hevc.block import BlockView
    from nano_hevc.frame import Plane
    h, w = src.shape
    recon = Plane.zeros(h, w, np.int16)
    lvl = np.zeros(src.shape, np.int32)
    tul = np.zeros((h // 4, w // 4), np.uint8)

    def one(x, y, n):
        blk = BlockView(recon, x, y, n)
        orig = src[y:y + n, x:x + n]
        top, left = blk.get_top_neighbors(), blk.get_left_neighbors()
        dc = I.intra_dc_predict(top, left, n)
        pl = I.intra_planar_predict(top, left, int(top[-1]), int(left[-1]), n)
        edc = int(np.sum(I.residual_block(orig, dc).astype(np.int64) ** 2))
        epl = int(np.sum(I.residual_block(orig, pl).astype(np.int64) ** 2))
        pred = dc if edc <= epl else pl
        l, r, _ = _chain(I, T, Q, orig, pred, qp, bool(is_luma and n == 4))
        lvl[y:y + n, x:x + n] = l
        blk.write_pixels(r)
        tul[y // 4:(y + n) // 4, x // 4:(x + n) // 4] = int(np.log2(n))

    def tree(x, y, s):
        if x >= w or y >= h:
            return
        over = (x + s > w) or (y + s > h)
        if s > 4 and (over or tu_split(seed, plane_id, x, y, s)):
            hs = s // 2
            for dy in (0, hs):
                for dx in (0, hs):
                    tree(x + dx, y + dy, hs)
            return
        if not over:
            one(x, y, s)

    for cy in range((h + ctb - 1) // ctb):
        for cx in range((w + ctb - 1) // ctb):
            tree(cx * ctb, cy * ctb, ctb)
    return lvl, recon.data, tul


def gen_closed4(I, T, Q):
    """Closed-loop config 4 planes (own rng): luma (CTB 32) with partial CTUs,
    chroma (CTB 16), 8-bit noise, a ragged plane (w, h not multiples of 4 x CTB)."""
    rng = np.random.default_rng(4040)
    out = {}
    yy, xx = np.mgrid[0:80, 0:104]
    cases = {
        "k4y": (np.clip(100 + xx - yy + rng.integers(-20, 21, size=xx.shape), 0, 255).astype(np.int16), 32, 0, True, 32),
        "k4u": (rng.integers(90, 170, size=(40, 52)).astype(np.int16), 16, 1, False, 32),
        "k4n": (rng.integers(0, 256, size=(64, 96)).astype(np.int16), 32, 0, True, 22),
        "k4r": (np.clip(80 + 2 * xx[:45, :70] + rng.integers(-9, 10, size=(45, 70)), 0, 255).astype(np.int16), 32, 0, True, 37),
    }
    for key, (src, ctb, pid, luma, qp) in cases.items():
        l, r, t = ref_plane_cfg4_closed(I, T, Q, src, ctb, pid, 1234, qp, luma)
        out.update({f"{key}_src": src, f"{key}_ctb": np.int64(ctb), f"{key}_pid": np.int64(pid),
                    f"{key}_luma": np.int64(luma), f"{key}_qp": np.int64(qp), f"{key}_lvl": l, f"{key}_rec": r,
                    f"{key}_tu": t})
    return out


def plane_hash_1080p(T, Q):
    rng = np.random.default_rng(20260)
    plane = rng.integers(-255, 256, size=(1080, 1920)).astype(np.int16)
    lvl = ref_plane_cfg2(T, Q, plane, 32)
    return hashlib.sha256(lvl.tobytes()).hexdigest()


def gen_dtypes(I, Q, M, T):
    """Non-integer inputs (tests/golden/dtype_cases.py): per case the reference's
    result (out_*, with rtype_* its Python type) or its exception (err_* the
    class name, errbase_* the builtin class it derives from)."""
    sys.path.insert(0, HERE)
    from dtype_cases import cases
    mods = (I, Q, M, T)
    out = {}
    bases = (ZeroDivisionError, OverflowError, IndexError, ValueError, TypeError, AttributeError)
    for name, fn, args, kw in cases():
        f = next(getattr(m, fn) for m in mods if hasattr(m, fn))
        try:
            r = f(*args, **kw)
        except Exception as e:
            out["err_" + name] = np.array(type(e).__name__)
            out["errbase_" + name] = np.array(next(b.__name__ for b in bases if isinstance(e, b)))
            continue
        out["out_" + name] = np.asarray(r)
        out["rtype_" + name] = np.array(type(r).__name__)
    return out


def main():
    pos = [a for i, a in enumerate(sys.argv[1:], 1) if not a.startswith("--") and sys.argv[i - 1] != "--only"]
    ref = pos[0] if pos else "/root/reference"
    warnings.simplefilter("ignore")
    I, T, Q, M = _import_reference(ref)
    rng = np.random.default_rng(1234)
    if "--only" in sys.argv:   # regenerate one file (own rng), keep the others and their manifest entries
        name = sys.argv[sys.argv.index("--only") + 1]
        gen = {"closed4.npz": lambda: gen_closed4(I, T, Q), "closed.npz": lambda: gen_closed(I, T, Q),
               "dtypes.npz": lambda: gen_dtypes(I, Q, M, T), "encode.npz": lambda: gen_encode(ref)}[name]
        p = os.path.join(HERE, name)
        np.savez_compressed(p, **gen())
        mp = os.path.join(HERE, "manifest.json")
        manifest = json.load(open(mp))
        manifest["files"][name] = hashlib.sha256(open(p, "rb").read()).hexdigest()
        with open(mp, "w") as f:
            json.dump(manifest, f, indent=1, sort_keys=True)
        print(name, manifest["files"][name])
        return
    files = {
        "matrices.npz": gen_matrices(T),
        "transform.npz": gen_transform(T, rng),
        "quant.npz": gen_quant(Q, rng),
        "intra.npz": gen_intra(I, rng),
        "chain.npz": gen_chain(I, T, Q),
        "planes.npz": gen_planes(I, T, Q, rng),
        "metrics.npz": gen_metrics(M),
        "cfg5.npz": gen_cfg5(I, T, Q, M),
        "encode.npz": gen_encode(ref),
        "closed.npz": gen_closed(I, T, Q),
        "closed4.npz": gen_closed4(I, T, Q),
        "dtypes.npz": gen_dtypes(I, Q, M, T),
    }
    manifest = {"numpy": np.__version__, "python": sys.version.split()[0],
                "generator": "tests/golden/make_golden.py", "reference": "Luodian/nano-hevc @ /root/reference",
                "files": {}}
    for name, arrays in files.items():
        p = os.path.join(HERE, name)
        np.savez_compressed(p, **arrays)
        manifest["files"][name] = hashlib.sha256(open(p, "rb").read()).hexdigest()
    if "--skip-1080p" not in sys.argv:
        manifest["cfg2_1080p_qp32_seed20260_levels_sha256"] = plane_hash_1080p(T, Q)
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)
    print(json.dumps(manifest, indent=1))


if __name__ == "__main__":
    main()

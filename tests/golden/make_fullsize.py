"""Reference outputs at BASELINE.json's full sizes, recorded as sha256 hashes.

Run in the build container only (imports the reference; the reference never
travels to the GPU box):

    python tests/golden/make_fullsize.py [/root/reference] [--procs 8]
    python tests/golden/make_fullsize.py --only-closed4     # add config 4 closed loop (3 processes, ~minutes)
    python tests/golden/make_fullsize.py --only-extra       # add the 4K YUV420 config-2 levels and the 8K config-5 chroma

Inputs are regenerated from seeds by ``fullsize_inputs`` (numpy only, imported
by tests/test_fullsize_reference_gpu.py as well), outputs are produced by the
same compositions of the reference's functions as make_golden.py (DESIGN.md
§3.3-3.5, §3.7), split over processes by independent block / CTU rows (open
loop) or by plane (closed loop), and hashed.  Written to fullsize.json.
"""
from __future__ import annotations

import hashlib
import json
import multiprocessing as mp
import os
import sys
import time
import warnings

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import fullsize_inputs as FI  # noqa: E402

_REF = None


def _init(ref):
    global _REF
    warnings.simplefilter("ignore")
    import make_golden as MG
    I, T, Q, M = MG._import_reference(ref)
    _REF = (MG, I, T, Q, M)


def _cfg3_band(args):
    src, qp, r0, r1 = args
    MG, I, T, Q, _ = _REF
    return r0, r1, MG.ref_plane_cfg3(I, T, Q, src, qp, (r0, r1))


def _cfg3_closed_plane(args):
    src, qp = args
    MG, I, T, Q, _ = _REF
    from nano_hevc.block import BlockView
    from nano_hevc.frame import Plane
    n = 8
    h, w = src.shape
    recon = Plane.zeros(h, w, np.int16)
    modes = np.zeros((h // n, w // n), np.uint8)
    lvl = np.zeros(src.shape, np.int32)
    total = 0
    for by in range(0, h - n + 1, n):       # make_golden.gen_closed, one plane
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
                l, r, sse = MG._chain(I, T, Q, orig, pred, qp, False)
                if best is None or sse < best[0]:
                    best = (sse, m, l, r)
            total += best[0]
            modes[by // n, bx // n] = best[1]
            lvl[by:by + n, bx:bx + n] = best[2]
            blk.write_pixels(best[3])
    return modes, lvl, recon.data, total


def _cfg4_band(args):
    src, ctb, pid, seed, qp, luma, c0, c1 = args
    MG, I, T, Q, _ = _REF
    return c0, c1, MG.ref_plane_cfg4(I, T, Q, src, ctb, pid, seed, qp, luma, (c0, c1))


def _cfg5_band(args):
    src, qp, r0, r1 = args
    MG, I, T, Q, _ = _REF
    lvl = np.zeros(src.shape, np.int32)
    rec = np.zeros(src.shape, np.int16)
    for by in range(r0 * 32, r1 * 32, 32):     # make_golden.gen_cfg5's per-block chain
        for bx in range(0, src.shape[1] - 31, 32):
            orig = src[by:by + 32, bx:bx + 32]
            top, left, _ = MG._neighbors(src, bx, by, 32)
            dc = I.intra_dc_predict(top, left, 32)
            pl = I.intra_planar_predict(top, left, int(top[-1]), int(left[-1]), 32)
            edc = int(np.sum(I.residual_block(orig, dc).astype(np.int64) ** 2))
            epl = int(np.sum(I.residual_block(orig, pl).astype(np.int64) ** 2))
            l, r, _ = MG._chain(I, T, Q, orig, dc if edc <= epl else pl, qp, False)
            lvl[by:by + 32, bx:bx + 32] = l
            rec[by:by + 32, bx:bx + 32] = r
    return r0, r1, lvl, rec


def _cfg2_band(args):
    src, qp, r0, r1 = args
    MG, _, T, Q, _ = _REF
    return r0, r1, MG.ref_plane_cfg2(T, Q, src[r0 * 8:r1 * 8], qp)


def _cfg4_closed_plane(args):
    src, ctb, pid, seed, qp, luma = args
    MG, I, T, Q, _ = _REF
    return MG.ref_plane_cfg4_closed(I, T, Q, src, ctb, pid, seed, qp, luma)


def _bands(nrows, k):
    step = -(-nrows // k)
    return [(a, min(nrows, a + step)) for a in range(0, nrows, step)]


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main():
    args = [a for i, a in enumerate(sys.argv[1:], 1) if not a.startswith("--") and sys.argv[i - 1] not in ("--procs", "--out")]
    ref = args[0] if args else "/root/reference"
    procs = int(sys.argv[sys.argv.index("--procs") + 1]) if "--procs" in sys.argv else 8
    out = {"generator": "tests/golden/make_fullsize.py", "inputs": "tests/golden/fullsize_inputs.py",
           "numpy": np.__version__, "reference": "Luodian/nano-hevc @ /root/reference"}
    dst = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else os.path.join(HERE, "fullsize.json")
    if "--only-extra" in sys.argv:   # add config 2 (4K YUV420) and config 5 chroma to an existing fullsize.json
        with open(dst) as f:
            out = json.load(f)
        with mp.get_context("fork").Pool(procs, initializer=_init, initargs=(ref,)) as pool:
            t0 = time.time()
            for k, src in enumerate(FI.cfg2_frame()):      # the metric's own workload: one 4K YUV420 frame
                lvl = np.zeros_like(src)
                for r0, r1, l in pool.imap_unordered(_cfg2_band, [(src, FI.CFG2_QP, a, b) for a, b in
                                                                  _bands(src.shape[0] // 8, 4 * procs)]):
                    lvl[r0 * 8:r1 * 8] = l
                out[f"cfg2_4k_p{k}"] = {"lvl": sha(lvl)}
            print("cfg2", time.time() - t0, flush=True)
            t0 = time.time()
            for k, src in enumerate(FI.cfg5_chroma(), 1):   # 8K U, V planes (3840 x 2160)
                lvl = np.zeros(src.shape, np.int32)
                rec = np.zeros(src.shape, np.int16)
                for r0, r1, l, r in pool.imap_unordered(_cfg5_band, [(src, FI.CFG5_QP, a, b) for a, b in
                                                                     _bands(src.shape[0] // 32, 4 * procs)]):
                    lvl[r0 * 32:r1 * 32] = l[r0 * 32:r1 * 32]
                    rec[r0 * 32:r1 * 32] = r[r0 * 32:r1 * 32]
                out[f"cfg5_{'uv'[k - 1]}"] = {"lvl": sha(lvl), "rec": sha(rec)}
            print("cfg5 chroma", time.time() - t0, flush=True)
        with open(dst, "w") as f:
            json.dump(out, f, indent=1, sort_keys=True)
        return
    if "--only-closed4" in sys.argv:   # add config 4 closed loop to an existing fullsize.json
        with open(dst) as f:
            out = json.load(f)
        t0 = time.time()
        with mp.get_context("fork").Pool(3, initializer=_init, initargs=(ref,)) as pool:
            jobs = [(src, 32 if k == 0 else 16, k, FI.CFG4_SEED, FI.CFG4_QP, k == 0)
                    for k, src in enumerate(FI.cfg4_frame())]
            for k, (l, r, t) in enumerate(pool.map(_cfg4_closed_plane, jobs)):
                out[f"closed4_p{k}"] = {"lvl": sha(l), "rec": sha(r), "tu": sha(t)}
        print("closed4", time.time() - t0, flush=True)
        with open(dst, "w") as f:
            json.dump(out, f, indent=1, sort_keys=True)
        return
    with mp.get_context("fork").Pool(procs, initializer=_init, initargs=(ref,)) as pool:
        # config 3, open loop: 1080p YUV420 frame, QP 32
        t0 = time.time()
        planes = FI.cfg3_frame()
        for k, src in enumerate(planes):
            h, w = src.shape
            modes = np.zeros((h // 8, w // 8), np.uint8)
            lvl = np.zeros(src.shape, np.int32)
            rec = np.zeros(src.shape, np.int16)
            total = 0
            for r0, r1, (m, l, r, s) in pool.imap_unordered(_cfg3_band, [(src, FI.CFG3_QP, a, b) for a, b in
                                                                          _bands(h // 8, 4 * procs)]):
                modes[r0:r1] = m[r0:r1]
                lvl[r0 * 8:r1 * 8] = l[r0 * 8:r1 * 8]
                rec[r0 * 8:r1 * 8] = r[r0 * 8:r1 * 8]
                total += s
            out[f"cfg3_p{k}"] = {"modes": sha(modes), "lvl": sha(lvl), "rec": sha(rec), "sse": int(total)}
        print("cfg3", time.time() - t0, flush=True)
        # config 3, closed loop: the same frame, QP 27, one plane per process
        t0 = time.time()
        for k, (m, l, r, s) in enumerate(pool.map(_cfg3_closed_plane, [(src, FI.CLOSED_QP) for src in planes])):
            out[f"closed_p{k}"] = {"modes": sha(m), "lvl": sha(l), "rec": sha(r), "sse": int(s)}
        print("closed", time.time() - t0, flush=True)
        # config 4: 4K YUV420 frame, seeded TU quadtree
        t0 = time.time()
        for k, src in enumerate(FI.cfg4_frame()):
            h, w = src.shape
            ctb = 32 if k == 0 else 16
            lvl = np.zeros(src.shape, np.int32)
            rec = np.zeros(src.shape, np.int16)
            tul = np.zeros((h // 4, w // 4), np.uint8)
            jobs = [(src, ctb, k, FI.CFG4_SEED, FI.CFG4_QP, k == 0, a, b) for a, b in _bands(-(-h // ctb), 4 * procs)]
            for c0, c1, (l, r, t) in pool.imap_unordered(_cfg4_band, jobs):
                y0, y1 = c0 * ctb, min(h, c1 * ctb)
                lvl[y0:y1] = l[y0:y1]
                rec[y0:y1] = r[y0:y1]
                tul[y0 // 4:y1 // 4] = t[y0 // 4:y1 // 4]
            out[f"cfg4_p{k}"] = {"lvl": sha(lvl), "rec": sha(rec), "tu": sha(tul)}
        print("cfg4", time.time() - t0, flush=True)
        # config 5: 8K luma plane, every 32x32 block, QP 4
        t0 = time.time()
        src = FI.cfg5_plane()
        lvl = np.zeros(src.shape, np.int32)
        rec = np.zeros(src.shape, np.int16)
        for r0, r1, l, r in pool.imap_unordered(_cfg5_band, [(src, FI.CFG5_QP, a, b) for a, b in
                                                             _bands(src.shape[0] // 32, 4 * procs)]):
            lvl[r0 * 32:r1 * 32] = l[r0 * 32:r1 * 32]
            rec[r0 * 32:r1 * 32] = r[r0 * 32:r1 * 32]
        out["cfg5_y"] = {"lvl": sha(lvl), "rec": sha(rec)}
        print("cfg5", time.time() - t0, flush=True)
    with open(dst, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

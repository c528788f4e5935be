"""Debug: config-4 closed loop, first luma CTU (a 32x32 TU) at QP 0 -- product lib vs oracle."""
import os, sys, json
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "nano-hevc_amd")); sys.path.insert(0, ROOT)
import torch
from nano_hevc import gpu, _lib
from oracle import oracle as O
if len(sys.argv) > 1 and sys.argv[1] == "ab":
    _lib.use_ab()
_lib.load()
F, W, H, qp = int(os.environ.get("F", 5)), 72, 40, int(os.environ.get("QP", 0))
rng = np.random.default_rng(F * 1000 + W + qp)
fe = gpu.yuv420_frame_elems(W, H)
buf = np.empty(F * fe, np.int16)
off = 0
for f in range(F):
    for pw, ph in ((W, H), (W // 2, H // 2), (W // 2, H // 2)):
        yy, xx = np.mgrid[0:ph, 0:pw]
        p = 255 * rng.integers(0, 2, (ph, pw)) if f == 2 else np.clip(60 + (3 * xx + 2 * yy + 11 * f) % 150 + rng.integers(-30, 31, (ph, pw)), 0, 255)
        buf[off:off + ph * pw] = p.reshape(-1); off += ph * pw
d = torch.from_numpy(buf).cuda()
sy, suv = gpu.yuv420_plane_sets(F, W, H)
lvl = torch.zeros(d.shape, dtype=torch.int32, device="cuda")
rec = torch.zeros(d.shape, dtype=torch.int16, device="cuda")
gpu.tu_pipeline_closed(d, sy, 32, 0, 4242, qp, True, lvl=lvl, rec=rec)
lv, rv = lvl.cpu().numpy(), rec.cpu().numpy()
src = buf[:W * H].reshape(H, W)
el, er, et = O.tu_pipeline_plane_closed(src, 32, 0, 4242, qp, True)
g = lv[:W * H].reshape(H, W)[:32, :32]; e = el[:32, :32]
gr = rv[:W * H].reshape(H, W)[:32, :32]; e2 = er[:32, :32]
print(json.dumps({"lib": _lib.LIB_PATH, "lvl_equal": bool((g == e).all()), "rec_equal": bool((gr == e2).all()),
                  "lvl_diff_rows": np.nonzero((g != e).any(1))[0].tolist(), "lvl_diff_cols": np.nonzero((g != e).any(0))[0].tolist(),
                  "got_col0": g[:, 0].tolist(), "exp_col0": e[:, 0].tolist(), "got_row0": g[0].tolist(), "exp_row0": e[0].tolist(),
                  "rec_diff_n": int((gr != e2).sum())}))

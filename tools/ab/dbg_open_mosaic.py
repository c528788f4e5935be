"""Where the config-4 open loop's chroma output differs from the oracle: mismatching
samples grouped by the TU size of the 4x4 map, and the first mismatching TU of
each size printed (GPU box; debugging aid)."""
import sys, os
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "nano-hevc_amd"))
from oracle import oracle as O   # noqa: E402
from nano_hevc import gpu   # noqa: E402

rng = np.random.default_rng(7 + 68)
h, w = 68, 100
yy, xx = np.mgrid[0:h, 0:w]
src = np.clip(120 + xx - 2 * yy + rng.integers(-25, 26, size=xx.shape), 0, 255).astype(np.int16)
for qp in (22, 37):
    l, r, t = gpu.tu_pipeline_plane(torch.from_numpy(src).cuda(), 16, 1, 7, qp, False)
    el, er, et = O.tu_pipeline_plane(src, 16, 1, 7, qp, False)
    l, r, t = l.cpu().numpy(), r.cpu().numpy(), t.cpu().numpy()
    print("qp", qp, "tu map equal", np.array_equal(t, et), "tu values", np.unique(et))
    tm = np.kron(et, np.ones((4, 4), dtype=et.dtype))[:h, :w]
    for name, a, b in (("lvl", l, el), ("rec", r, er)):
        bad = a != b
        print(name, "mismatches", int(bad.sum()), "by tu value",
              {int(v): int((bad & (tm == v)).sum()) for v in np.unique(et)})
        for v in np.unique(et):
            ys, xs = np.nonzero(bad & (tm == v))
            if len(ys) == 0:
                continue
            y, x = ys[0], xs[0]
            n = 4 << int(v) if v < 4 else int(v)
            by, bx = y // n * n, x // n * n
            print(f"  first {name} mismatch tu={v} at ({y},{x}) block ({by},{bx}) n={n}")
            print("  gpu\n", a[by:by + n, bx:bx + n])
            print("  ref\n", b[by:by + n, bx:bx + n])

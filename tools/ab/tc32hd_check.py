"""A/B parity of config 5's LDS-DMA form (k_tc32_hd, knob NH_TC32H_DMA = blocks
per wave) against the product library's kernel, in one process: the same inputs
through libnanohevc.so and libnanohevc_ab.so, levels and recon compared
element for element.  Set NH_TC32H_DMA before running (read once per process).

Cases: an 8K luma plane (tc32_plane), a ragged 3-frame YUV420 stream with an
int16-extremes frame and a lone wide block (tc32_planes, partial blocks at every
plane's right/bottom edge), and two 8K YUV420 frames with wide blocks sprinkled
in (the bench's config-5 shape).  Prints one JSON line; exit 1 on a mismatch.
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "nano-hevc_amd"))


def main():
    import torch
    from nano_hevc import gpu, _lib
    rng = np.random.default_rng(7)
    out = {"NH_TC32H_DMA": os.environ.get("NH_TC32H_DMA", "0")}
    ok = True

    def both(fn):
        _lib.use_ab(False)
        a = [t.cpu().numpy() for t in fn()]
        _lib.use_ab(True)
        b = [t.cpu().numpy() for t in fn()]
        _lib.use_ab(False)
        return all(np.array_equal(x, y) for x, y in zip(a, b))

    # 8K luma
    yy, xx = np.mgrid[0:4320, 0:7680]
    luma = np.clip(128 + 60 * np.sin(xx / 97.0) * np.cos(yy / 53.0) + rng.integers(-20, 21, xx.shape), 0, 255)
    d = torch.from_numpy(luma.astype(np.int16)).cuda()
    for qp in (4, 30, 51):
        r = both(lambda: gpu.tc32_plane(d, qp, 1))
        out[f"luma8k_qp{qp}"] = r
        ok &= r

    # ragged stream
    nf, w, h = 3, 208, 136
    sets = gpu.yuv420_plane_sets(nf, w, h)
    fe = gpu.yuv420_frame_elems(w, h)
    buf = rng.integers(0, 256, size=nf * fe).astype(np.int16)
    buf[fe:2 * fe] = rng.integers(-32768, 32768, size=fe)
    buf[2 * fe + 5 * w + 40] = 300
    ds = torch.from_numpy(buf).cuda()

    def run_sets(src, ss, qp):
        lvl = torch.full(src.shape, -7, dtype=torch.int32, device="cuda")
        rec = torch.full(src.shape, -7, dtype=torch.int16, device="cuda")
        return gpu.tc32_planes(src, ss, qp, 1, lvl=lvl, rec=rec)

    r = both(lambda: run_sets(ds, sets, 30))
    out["ragged_stream"] = r
    ok &= r

    # two 8K YUV420 frames, wide samples sprinkled (about one block in 200)
    W, H = 7680, 4320
    sets8 = gpu.yuv420_plane_sets(2, W, H)
    fe8 = gpu.yuv420_frame_elems(W, H)
    b8 = rng.integers(0, 256, size=2 * fe8).astype(np.int16)
    idx = rng.integers(0, 2 * fe8, size=2 * fe8 // (32 * 32 * 200))
    b8[idx] = rng.integers(-600, 600, size=idx.size)
    d8 = torch.from_numpy(b8).cuda()
    for qp in (22, 37):
        r = both(lambda: run_sets(d8, sets8, qp))
        out[f"yuv8k_qp{qp}"] = r
        ok &= r
    out["ok"] = bool(ok)
    print(json.dumps(out), flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())

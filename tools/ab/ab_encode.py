#!/usr/bin/env python3
"""A/B of the encode_frame_intra launch structure on a 64-frame 4K YUV420p uint8
stream: the luma (8x8) and chroma (4x4) plane sets back to back on one stream
(the API today), each alone, and the two on two streams at once (the chroma set
forked onto a side stream).  Prints median ms per form (HIP events)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "nano-hevc_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402

from bench_configs import synth_plane, timed  # noqa: E402


def main():
    from nano_hevc import gpu
    torch.cuda.set_device(0)
    W, H, nf = 3840, 2160, 64
    planes = [synth_plane(ph, pw, sd).to(torch.uint8).reshape(-1)
              for pw, ph, sd in ((W, H, 1), (W // 2, H // 2, 2), (W // 2, H // 2, 3))]
    src = torch.cat(planes).repeat(nf)
    rec = torch.empty(src.numel(), dtype=torch.int16, device="cuda")
    stats = torch.zeros((3 * nf, gpu.ENC_STATS), dtype=torch.int64, device="cuda")
    sy, suv = gpu.yuv420_plane_sets(nf, W, H)
    main_s = torch.cuda.current_stream()
    side = torch.cuda.Stream()

    def pair():
        gpu.encode_intra_planes(src, [sy, suv], [8, 4], recon=rec, stats=stats)

    def luma():
        gpu.encode_intra_planes(src, [sy], [8], recon=rec, stats=stats[:nf])

    def chroma():
        gpu.encode_intra_planes(src, [suv], [4], recon=rec, stats=stats[nf:])

    def forked():
        ev = torch.cuda.Event()
        ev.record(main_s)
        side.wait_event(ev)
        with torch.cuda.stream(side):
            gpu.encode_intra_planes(src, [suv], [4], recon=rec, stats=stats[nf:], stream=side)
        gpu.encode_intra_planes(src, [sy], [8], recon=rec, stats=stats[:nf])
        done = torch.cuda.Event()
        done.record(side)
        main_s.wait_event(done)

    res = {}
    for name, fn in (("pair", pair), ("luma", luma), ("chroma", chroma), ("forked", forked)) * 3:
        res.setdefault(name, []).append(timed(fn, 20))
    out = {k: sorted(v)[len(v) // 2] for k, v in res.items()}
    out["bytes"] = src.numel() * 3
    out["GBps_pair"] = out["bytes"] / out["pair"] / 1e6
    out["GBps_forked"] = out["bytes"] / out["forked"] / 1e6
    print(json.dumps(out))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Config 5 batched (nh_tc32_planes) on an 8-frame 8K YUV420 stream, a few
launch sets, for rocprofv3 kernel traces / PMC passes."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nano-hevc_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402


def main():
    from nano_hevc import gpu
    from bench_configs import synth_plane
    torch.cuda.set_device(0)
    W, H, nf = 7680, 4320, 8
    planes = [synth_plane(H, W, 7), synth_plane(H // 2, W // 2, 8), synth_plane(H // 2, W // 2, 9)]
    fe = gpu.yuv420_frame_elems(W, H)
    src = torch.cat([torch.cat([p.flatten() for p in planes]) for _ in range(nf)])
    sets = gpu.yuv420_plane_sets(nf, W, H)
    lvl = torch.zeros_like(src, dtype=torch.int32)
    rec = torch.zeros_like(src)
    for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 5):
        gpu.tc32_planes(src, sets, 4, 1, lvl=lvl, rec=rec)
    torch.cuda.synchronize()
    print("ok", fe)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""The default fused 8x8 DCT+quant launch (variant 4341) on the bench workload
(128 4K YUV420 int16 residual frames in HBM) through the A/B library, so that
NH_CAP_FWD8 (resident workgroups per CU, lds_cap) applies.  Allocates the
output in several buffers in turn (placement regimes) and
prints one JSON line: median kernel ms and TB/s per output buffer."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "nano-hevc_amd"))
import torch  # noqa: E402


def main():
    from nano_hevc import gpu, _lib
    _lib.use_ab()
    _lib.load()
    torch.cuda.set_device(0)
    frames = 128
    sets = gpu.yuv420_plane_sets(frames, 3840, 2160)
    n = frames * gpu.yuv420_frame_elems(3840, 2160)
    g = torch.Generator(device="cuda")
    g.manual_seed(1234)
    res = torch.randint(-255, 256, (n,), dtype=torch.int16, device="cuda", generator=g)
    nblk = gpu.blocks_in(sets)
    outs = [torch.empty(n, dtype=torch.int16, device="cuda") for _ in range(3)]
    st = torch.cuda.current_stream()
    per = []
    for o in outs:
        gpu.fwd8x8_quant(res, sets, 32, True, out=o)
        torch.cuda.synchronize()
        ts = []
        for _ in range(15):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            gpu.fwd8x8_quant(res, sets, 32, True, out=o)
            b.record(st)
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        ms = statistics.median(ts)
        per.append({"ms": ms, "TBps": nblk * 256 / ms / 1e9})
    print(json.dumps({"knobs": {k: v for k, v in os.environ.items() if k.startswith("NH_")}, "buffers": per,
                      "equal": bool(torch.equal(outs[0], outs[1]) and torch.equal(outs[1], outs[2]))}), flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Launch the default hot kernel 5x with output = buffer 1 and 5x with
output = buffer 5 (of 6 same-size torch buffers), for PMC passes that compare
the two placements (tools/ab/ab_bufindex.py showed output placement decides
5.9 vs 6.7 TB/s on some boxes).  Prints the per-launch ms of each group."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "nano-hevc_amd"))
import torch  # noqa: E402


def main():
    from nano_hevc import gpu
    torch.cuda.set_device(0)
    W, H, F = 3840, 2160, 128
    sets = gpu.yuv420_plane_sets(F, W, H)
    nblk = gpu.blocks_in(sets)
    n = F * gpu.yuv420_frame_elems(W, H)
    bufs = [torch.empty(n, dtype=torch.int16, device="cuda") for _ in range(6)]
    bufs[0].copy_(torch.randint(-255, 256, (n,), dtype=torch.int16, device="cuda"))
    st = torch.cuda.current_stream()
    rep = {}
    for o in (1, 5):
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
        for a, b in evs:
            a.record(st)
            gpu.fwd8x8_quant(bufs[0], sets, 32, True, out=bufs[o], stream=st)
            b.record(st)
        torch.cuda.synchronize()
        rep[f"out{o}_GBps"] = round(nblk * 256 / statistics.median([a.elapsed_time(b) for a, b in evs]) / 1e6)
    print(json.dumps(rep), flush=True)


if __name__ == "__main__":
    main()

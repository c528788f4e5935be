#!/usr/bin/env python3
"""Allocation-order A/B for the hot kernel (one case per process, so each case
starts from the same fresh allocator state).  Cases differ only in how the
input and output buffers of the bench's launch are allocated; prints one JSON
line with the buffers' virtual addresses and the median per-launch GB/s of
variants 5 and 4341."""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "nano-hevc_amd"))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", default="adjacent")
    args = ap.parse_args()
    from nano_hevc import gpu
    torch.cuda.set_device(0)
    W, H, F = 3840, 2160, 128
    sets = gpu.yuv420_plane_sets(F, W, H)
    nblk = gpu.blocks_in(sets)
    n = F * gpu.yuv420_frame_elems(W, H)
    keep = []
    c = args.case
    if c.startswith("pre"):          # preN: N GiB allocated before both buffers
        keep.append(torch.empty(int(c[3:]) << 29, dtype=torch.int16, device="cuda"))
    if c == "outfirst":
        out = torch.zeros(n, dtype=torch.int16, device="cuda")
        res = torch.empty(n, dtype=torch.int16, device="cuda")
    else:
        res = torch.empty(n, dtype=torch.int16, device="cuda")
        if c.startswith("gap"):      # gapN: N/4 of the buffer size between input and output
            keep.append(torch.empty(n * int(c[3:]) // 4, dtype=torch.int16, device="cuda"))
        out = torch.zeros(n, dtype=torch.int16, device="cuda")
    g = torch.Generator(device="cuda")
    g.manual_seed(1234)
    res.copy_(torch.randint(-255, 256, (n,), dtype=torch.int16, device="cuda", generator=g))
    st = torch.cuda.current_stream()
    rep = {"case": c, "in": res.data_ptr(), "out": out.data_ptr(), "D": out.data_ptr() - res.data_ptr(),
           "alloc_conf": os.environ.get("PYTORCH_HIP_ALLOC_CONF", "")}
    for v in (5, 4341, 5, 4341):
        for _ in range(3):
            gpu.fwd8x8_quant(res, sets, 32, True, out=out, variant=v, stream=st)
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
        for a, b in evs:
            a.record(st)
            gpu.fwd8x8_quant(res, sets, 32, True, out=out, variant=v, stream=st)
            b.record(st)
        torch.cuda.synchronize()
        med = statistics.median([a.elapsed_time(b) for a, b in evs])
        rep.setdefault(f"v{v}", []).append(round(nblk * 256 / med / 1e6))
    print(json.dumps(rep), flush=True)


if __name__ == "__main__":
    main()

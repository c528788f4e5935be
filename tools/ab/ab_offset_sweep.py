#!/usr/bin/env python3
"""Placement sweep for the hot kernel: input at the start of one allocation,
output at byte offset D = S + delta behind it (S = input bytes rounded to
2 MiB, as torch's allocator places a second same-size buffer).  The
read and write streams of the kernel run at a fixed address distance D, so
D decides how the two streams share HBM channels/banks.  One JSON line per
(delta, variant): median per-launch ms over 25 launches (HIP events)."""
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
    ap.add_argument("--variants", default="5,4341")
    ap.add_argument("--deltas", default="0,4K,16K,64K,256K,1M,2M,4M,8M,16M,32M,64M,128M,256M,512M,1G,2G,S")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--frames", type=int, default=128)
    args = ap.parse_args()
    from nano_hevc import gpu
    torch.cuda.set_device(0)
    W, H, F = 3840, 2160, args.frames
    sets = gpu.yuv420_plane_sets(F, W, H)
    nblk = gpu.blocks_in(sets)
    n = F * gpu.yuv420_frame_elems(W, H)
    S = (n * 2 + (2 << 20) - 1) // (2 << 20) * (2 << 20)
    unit = {"K": 1 << 10, "M": 1 << 20, "G": 1 << 30}
    deltas = []
    for d in args.deltas.split(","):
        deltas.append(S if d == "S" else int(d[:-1]) * unit[d[-1]] if d[-1] in unit else int(d))
    big = torch.empty((2 * S + max(deltas)) // 2, dtype=torch.int16, device="cuda")
    g = torch.Generator(device="cuda")
    g.manual_seed(1234)
    res = big[:n]
    res.copy_(torch.randint(-255, 256, (n,), dtype=torch.int16, device="cuda", generator=g))
    st = torch.cuda.current_stream()
    ref = None
    for r in range(args.rounds):
        for d in deltas:
            o = (S + d) // 2
            out = big[o:o + n]
            for v in [int(x) for x in args.variants.split(",")]:
                gpu.fwd8x8_quant(res, sets, 32, True, out=out, variant=v, stream=st)
                evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(25)]
                for a, b in evs:
                    a.record(st)
                    gpu.fwd8x8_quant(res, sets, 32, True, out=out, variant=v, stream=st)
                    b.record(st)
                torch.cuda.synchronize()
                ts = [a.elapsed_time(b) for a, b in evs]
                if ref is None:
                    ref = out.clone()
                ok = bool(torch.equal(out, ref))
                med = statistics.median(ts)
                print(json.dumps({"round": r, "delta": d, "D": S + d, "variant": v, "ms_median": med,
                                  "GBps_median": nblk * 256 / med / 1e6, "equal": ok}), flush=True)


if __name__ == "__main__":
    main()

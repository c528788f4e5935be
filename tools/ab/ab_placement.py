#!/usr/bin/env python3
"""Why does the interleaved A/B (tools/ab/ab_fwd8x8.py) time the default launch
faster than bench.py on the same box?  Time the bench's exact launch under
controlled differences: a spacer allocation between input and output, bursts
of K launches separated by a sync, and the input's generator.  One JSON line
per case: per-launch ms (HIP events on the launch stream), median / min."""
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
    ap.add_argument("--variant", type=int, default=4341)
    ap.add_argument("--launches", type=int, default=30)
    args = ap.parse_args()
    from nano_hevc import gpu
    torch.cuda.set_device(0)
    W, H, F = 3840, 2160, 128
    sets = gpu.yuv420_plane_sets(F, W, H)
    nblk = gpu.blocks_in(sets)
    n = F * gpu.yuv420_frame_elems(W, H)
    st = torch.cuda.current_stream()
    g = torch.Generator(device="cuda")
    g.manual_seed(1234)
    res = torch.randint(-255, 256, (n,), dtype=torch.int16, device="cuda", generator=g)
    out_adj = torch.zeros_like(res)
    spacer = torch.empty(n, dtype=torch.int16, device="cuda")
    out_far = torch.zeros_like(res)
    outs = [torch.zeros_like(res) for _ in range(3)]

    def timed(out, burst, variant):
        ts = []
        done = 0
        while done < args.launches:
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(burst)]
            for a, b in evs:
                a.record(st)
                gpu.fwd8x8_quant(res, sets, 32, True, out=out, variant=variant, stream=st)
                b.record(st)
            torch.cuda.synchronize()
            ts += [a.elapsed_time(b) for a, b in evs]
            done += burst
        ts = ts[3:]
        return {"ms_median": statistics.median(ts), "ms_min": min(ts),
                "GBps_median": nblk * 256 / statistics.median(ts) / 1e6, "first5": [round(t, 3) for t in ts[:5]]}

    cases = [("adjacent", out_adj, 30), ("adjacent_burst5", out_adj, 5), ("far", out_far, 30),
             ("far_burst5", out_far, 5), ("late0", outs[0], 30), ("late2", outs[2], 30)]
    for r in range(2):
        for v in (5, args.variant):
            for name, o, burst in cases:
                e = timed(o, burst, v)
                e.update({"case": name, "variant": v, "round": r})
                print(json.dumps(e), flush=True)
    del spacer


if __name__ == "__main__":
    main()

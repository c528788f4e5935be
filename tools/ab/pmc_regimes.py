#!/usr/bin/env python3
"""Hot-kernel placement regimes under per-channel memory counters (VERDICT r1
item 5).  One process allocates K same-size buffers in sequence (the torch
allocator, as the bench), fills buffer 0 with the bench's 128-frame 4K YUV420
residual stream, and runs the default k_fwd8x8_quant launch REPS times with
the output in buffer j = 1..K-1, in that order.  It prints per j the median
HIP-event GB/s (one JSON line), so a rocprofv3 --pmc pass of the same command
(dispatch order = j order) gives the memory-side counters of each placement:

    rocprofv3 --pmc TCC_EA0_WRREQ TCC_EA0_RDREQ -- python3 tools/ab/pmc_regimes.py
"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "nano-hevc_amd"))
import torch  # noqa: E402


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    REPS = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    from nano_hevc import gpu
    torch.cuda.set_device(0)
    W, H, F = 3840, 2160, 128
    sets = gpu.yuv420_plane_sets(F, W, H)
    nblk = gpu.blocks_in(sets)
    n = F * gpu.yuv420_frame_elems(W, H)
    bufs = [torch.empty(n, dtype=torch.int16, device="cuda") for _ in range(K)]
    g = torch.Generator(device="cuda")
    g.manual_seed(1234)
    bufs[0].copy_(torch.randint(-255, 256, (n,), dtype=torch.int16, device="cuda", generator=g))
    st = torch.cuda.current_stream()
    torch.cuda.synchronize()
    res = []
    for j in range(1, K):
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(REPS)]
        for a, b in evs:
            a.record(st)
            gpu.fwd8x8_quant(bufs[0], sets, 32, True, out=bufs[j], stream=st)
            b.record(st)
        torch.cuda.synchronize()
        ms = statistics.median(a.elapsed_time(b) for a, b in evs)
        res.append({"out_buffer": j, "ms": ms, "GBps": nblk * 256 / ms / 1e6,
                    "out_va_gb": round(bufs[j].data_ptr() / 2**30, 3)})
    print(json.dumps({"tool": "tools/ab/pmc_regimes.py", "K": K, "reps": REPS, "blocks": nblk, "placements": res}))


if __name__ == "__main__":
    main()

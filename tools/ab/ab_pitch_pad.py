#!/usr/bin/env python3
"""Row-pitch padding vs output placement for the hot kernel: 128 4K YUV420
frames laid out with Y pitch 3840 + pad and chroma pitch 1920 + pad / 2
(samples outside the width untouched).  K buffers are allocated ONCE (sized
for the largest pad), so every pad is measured on the same physical pages:
input = buffer 0, output = buffer j.  Median GB/s (algorithmic bytes of the
unpadded workload) of 20 launches of the default launch; one JSON line per pad."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "nano-hevc_amd"))
import torch  # noqa: E402


def layout(W, H, F, pad, gpu):
    py, pc = W + pad, W // 2 + pad // 2
    fe = py * H + 2 * pc * (H // 2)
    sy = gpu.plane_set(0, W, H, py, 1, F, 0, fe)
    suv = gpu.plane_set(py * H, W // 2, H // 2, pc, 2, F, pc * (H // 2), fe)
    return [sy, suv], F * fe


def main():
    from nano_hevc import gpu
    torch.cuda.set_device(0)
    W, H, F = 3840, 2160, 128
    K = int(os.environ.get("K", "8"))
    variant = int(os.environ.get("VARIANT", "4341"))
    pads = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "0,64,256,1024").split(",")]
    nmax = max(layout(W, H, F, p, gpu)[1] for p in pads)
    bufs = [torch.empty(nmax, dtype=torch.int16, device="cuda") for _ in range(K)]
    bufs[0].copy_(torch.randint(-255, 256, (nmax,), dtype=torch.int16, device="cuda"))
    st = torch.cuda.current_stream()
    for pad in pads:
        sets, n = layout(W, H, F, pad, gpu)
        nblk = gpu.blocks_in(sets)
        res = []
        for j in range(1, K):
            src, dst = bufs[0][:n], bufs[j][:n]
            for _ in range(3):
                gpu.fwd8x8_quant(src, sets, 32, True, out=dst, variant=variant, stream=st)
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
            for a, b in evs:
                a.record(st)
                gpu.fwd8x8_quant(src, sets, 32, True, out=dst, variant=variant, stream=st)
                b.record(st)
            torch.cuda.synchronize()
            res.append(round(nblk * 256 / statistics.median([a.elapsed_time(b) for a, b in evs]) / 1e6))
        print(json.dumps({"pad": pad, "variant": variant, "out_j": res}), flush=True)


if __name__ == "__main__":
    main()

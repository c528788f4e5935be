#!/usr/bin/env python3
"""Placement map for the hot kernel in ONE process: allocate K same-size
buffers in sequence (torch allocator), fill buffer 0 with the input, then time
the default launch for output = buffer j (j = 1..K-1), and for input = buffer
j with output = buffer j+1 (the input copied there first).  Median GB/s of 20
launches per pair."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "nano-hevc_amd"))
import torch  # noqa: E402


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    vs = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "4341").split(",")]
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
    src = bufs[0].clone()
    st = torch.cuda.current_stream()

    def t(i, o, v):
        for _ in range(3):
            gpu.fwd8x8_quant(bufs[i], sets, 32, True, out=bufs[o], variant=v, stream=st)
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
        for a, b in evs:
            a.record(st)
            gpu.fwd8x8_quant(bufs[i], sets, 32, True, out=bufs[o], variant=v, stream=st)
            b.record(st)
        torch.cuda.synchronize()
        return round(nblk * 256 / statistics.median([a.elapsed_time(b) for a, b in evs]) / 1e6)

    import ctypes as C
    from nano_hevc import _lib
    L = _lib.load()

    def tcopy(i, o, pol):   # linear streaming copy probe of the same byte count (policy: see nh_probe_copy_linear)
        args = (bufs[i].data_ptr(), bufs[o].data_ptr(), n // 8 * 8, pol, 0, C.c_void_p(st.cuda_stream))
        for _ in range(3):
            _lib.check(L.nh_probe_copy_linear(*args))
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
        for a, b in evs:
            a.record(st)
            _lib.check(L.nh_probe_copy_linear(*args))
            b.record(st)
        torch.cuda.synchronize()
        return round(nblk * 256 / statistics.median([a.elapsed_time(b) for a, b in evs]) / 1e6)

    rep = {"addr_GB": [round((b.data_ptr() - bufs[0].data_ptr()) / 2**30, 2) for b in bufs]}
    if "--copy" in sys.argv:
        rep["copy_nt_in0_out_j"] = [tcopy(0, j, 1) for j in range(1, K)]
        rep["copy_nt_xcd_in0_out_j"] = [tcopy(0, j, 17) for j in range(1, K)]
    for v in vs:
        rep[f"v{v}_in0_out_j"] = [t(0, j, v) for j in range(1, K)]
    if len(vs) == 1:
        pairs = []
        for j in range(1, K - 1):
            bufs[j].copy_(src)
            pairs.append(t(j, j + 1, vs[0]))
        rep["in_j_out_j1"] = pairs
    rep["again"] = [t(0, j, vs[0]) for j in range(1, K)]
    print(json.dumps(rep), flush=True)


if __name__ == "__main__":
    main()

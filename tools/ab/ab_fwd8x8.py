#!/usr/bin/env python3
"""Interleaved A/B of the fused 8x8 DCT+quant launch variants in ONE process
(cdna_hip_programming.md §5.4 rule 24), on the bench workload (4K YUV420
frame stream resident in HBM), next to two bandwidth references of the same
byte count: torch's copy_ and the same-access-pattern copy probe.

Prints one JSON object: per variant the median / min kernel ms and GB/s
(algorithmic 256 B per block), and whether each variant's output equals v0.
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "nano-hevc_amd"))

import ctypes as C  # noqa: E402

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=128)
    ap.add_argument("--rounds", type=int, default=12)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--variants", default="1,5,9,13")
    ap.add_argument("--epilogue", action="store_true", help="also time the fused level-side epilogue (ex, exnnz)")
    ap.add_argument("--shapes", action="store_true", help="also time the 2-blocks-per-thread pattern probes")
    ap.add_argument("--stripe", action="store_true", help="also time the stripe-form copy probes (LDS-DMA / register staging)")
    ap.add_argument("--rowwave", action="store_true", help="also time the row-per-wave and M-chunks-per-thread linear probes")
    ap.add_argument("--xcd", action="store_true", help="also time the linear copy with the XCD-aware workgroup order")
    args = ap.parse_args()
    from nano_hevc import gpu, _lib
    L = _lib.load()
    torch.cuda.set_device(0)
    W, H = 3840, 2160
    fe = gpu.yuv420_frame_elems(W, H)
    sets = gpu.yuv420_plane_sets(args.frames, W, H)
    nblk = gpu.blocks_in(sets)
    g = torch.Generator(device="cuda")
    g.manual_seed(7)
    res = torch.randint(-255, 256, (args.frames * fe,), dtype=torch.int16, device="cuda", generator=g)
    outs = {}
    st = torch.cuda.current_stream()
    arr = (gpu.PlaneSet * len(sets))(*sets)
    variants = [int(v) for v in args.variants.split(",")]
    bytes_per = nblk * 256

    def run(name):
        o = outs[name]   # preallocated: nothing but the measured kernel runs in the timed region
        if name == "torch_copy":
            o.copy_(res)
        elif name.startswith("linear"):
            pol, grid = name[6:].split("g")
            _lib.check(L.nh_probe_copy_linear(res.data_ptr(), o.data_ptr(), res.numel() // 8 * 8, int(pol), int(grid),
                                              C.c_void_p(st.cuda_stream)))
        elif name.startswith("probe"):
            _lib.check(L.nh_probe_copy8x8_planes(res.data_ptr(), o.data_ptr(), arr, len(sets), int(name[5:]),
                                                 C.c_void_p(st.cuda_stream)))
        elif name.startswith("shape"):     # shapeS_P: pair probe S with cache policy P
            sh, pol = name[5:].split("_")
            _lib.check(L.nh_probe_copy8x8_planes(res.data_ptr(), o.data_ptr(), arr, len(sets), int(pol) + 4 * int(sh),
                                                 C.c_void_p(st.cuda_stream)))
        elif name == "ex":        # + fused count_nonzero / estimate_bits epilogue (261 B/block)
            _lib.check(L.nh_fwd8x8_quant_planes_ex(res.data_ptr(), o.data_ptr(), arr, len(sets), 32, 1,
                                                   ex_nnz.data_ptr(), ex_bits.data_ptr(), C.c_void_p(st.cuda_stream)))
        elif name == "exnnz":     # + count_nonzero only (257 B/block)
            _lib.check(L.nh_fwd8x8_quant_planes_ex(res.data_ptr(), o.data_ptr(), arr, len(sets), 32, 1,
                                                   ex_nnz.data_ptr(), None, C.c_void_p(st.cuda_stream)))
        else:
            gpu.fwd8x8_quant(res, sets, 32, True, out=o, variant=int(name[1:]), stream=st)

    names = (["torch_copy"] + [f"probe{p}" for p in range(4)] + [f"linear{p}g{g}" for p in (0, 1) for g in (0, 4096)]
             + [f"v{v}" for v in variants] + (["ex", "exnnz"] if args.epilogue else [])
             + ([f"shape{sh}_{p}" for sh in (1, 2, 3) for p in (0, 1)] if args.shapes else [])
             + ([f"shape{sh}_{p}" for sh in (4, 5) for p in (0, 1)] if args.stripe else [])
             + ([f"shape{sh}_1" for sh in (6, 7, 8)] + [f"linear{1 + 4 * lm}g0" for lm in (1, 2, 3)] if args.rowwave else [])
             + (["linear16g0", "linear17g0"] if args.xcd else []))
    ex_nnz = torch.empty(nblk, dtype=torch.uint8, device="cuda")
    ex_bits = torch.empty(nblk, dtype=torch.int32, device="cuda")
    for n in names:
        outs[n] = torch.zeros_like(res)
    times = {n: [] for n in names}
    for n in names:      # warm-up + allocation
        run(n)
    torch.cuda.synchronize()
    for r in range(args.rounds):
        order = names if r % 2 == 0 else names[::-1]
        for n in order:
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.reps)]
            for a, b in evs:
                a.record(st)
                run(n)
                b.record(st)
            torch.cuda.synchronize()
            times[n] += [a.elapsed_time(b) for a, b in evs]
    ref = outs["v0"] if "v0" in outs else None
    rep = {"blocks_per_launch": nblk, "bytes_per_launch": bytes_per, "results": {}}
    for n in names:
        med, mn = statistics.median(times[n]), min(times[n])
        e = {"ms_median": med, "ms_min": mn, "GBps_median": bytes_per / med / 1e6, "GBps_best": bytes_per / mn / 1e6}
        if (n.startswith("v") or n.startswith("ex")) and ref is not None:
            e["equal_v0"] = bool(torch.equal(outs[n], ref))
        rep["results"][n] = e
    print(json.dumps(rep, indent=1))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Config-3 closed loop: one launch over F 1080p YUV420 frames vs K launches of F frames
pipelined over D streams (no host round trip between them; one status check per launch
at the end).  Per-frame medians by HIP events; one JSON line.

    python tools/ab/ab_closed3_pipe.py [--frames 64] [--pipe 4] [--depth 2] [--reps 5]
"""
import argparse
import ctypes as C
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "nano-hevc_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=64)
    ap.add_argument("--pipe", type=int, default=4)
    ap.add_argument("--depth", type=int, default=2)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--qp", type=int, default=32)
    args = ap.parse_args()
    from nano_hevc import gpu, _lib
    from nano_hevc._lib import PlaneSet
    from bench_configs import synth_plane
    L = _lib.load()
    W, H, nf = 1920, 1080, args.frames
    planes = []
    for f in range(nf):
        planes += [synth_plane(H, W, 40 + 3 * f).reshape(-1), synth_plane(H // 2, W // 2, 41 + 3 * f).reshape(-1),
                   synth_plane(H // 2, W // 2, 42 + 3 * f).reshape(-1)]
    src = torch.cat(planes)
    del planes
    sets = gpu.yuv420_plane_sets(nf, W, H)
    arr = (PlaneSet * len(sets))(*sets)
    wb = int(L.nh_intra_rdo_closed_workspace_bytes(arr, len(sets)))
    nmodes = sum((s.width // 8) * (s.height // 8) * s.planes_per_group * s.num_groups for s in sets)
    bufs = [(torch.zeros(src.shape, dtype=torch.int32, device="cuda"), torch.zeros(src.shape, dtype=torch.int16, device="cuda"),
             torch.zeros(nmodes, dtype=torch.uint8, device="cuda"), torch.zeros(3 * nf, dtype=torch.int64, device="cuda"))
            for _ in range(args.depth)]
    streams = [torch.cuda.Stream() for _ in range(args.depth)]

    def single():
        lv, rc, _, _ = bufs[0]
        gpu.intra_rdo_closed(src, sets, args.qp, lvl=lv, rec=rc)

    def pipe():
        main = torch.cuda.current_stream()
        ev = torch.cuda.Event()
        ev.record(main)
        works = []
        for s_ in streams:
            s_.wait_event(ev)
        for k in range(args.pipe):
            lv, rc, md, ss = bufs[k % args.depth]
            s_ = streams[k % args.depth]
            with torch.cuda.stream(s_):
                w_ = torch.empty((wb + 3) // 4, dtype=torch.int32, device="cuda")
            works.append(w_)
            _lib.check(L.nh_intra_rdo_planes_closed(src.data_ptr(), arr, len(sets), int(args.qp), md.data_ptr(),
                                                    lv.data_ptr(), rc.data_ptr(), ss.data_ptr(), w_.data_ptr(),
                                                    C.c_void_p(s_.cuda_stream)))
        for s_ in streams:
            j = torch.cuda.Event()
            j.record(s_)
            main.wait_event(j)
        for w_ in works:
            st = C.c_int(0)
            _lib.check(L.nh_intra_rdo_closed_status(w_.data_ptr(), C.byref(st), C.c_void_p(main.cuda_stream)))
            assert st.value == 0

    out = {"frames": nf, "pipe": args.pipe, "depth": args.depth}
    for name, fn, per in (("single", single, nf), (f"pipe{args.pipe}d{args.depth}", pipe, nf * args.pipe)):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        out[name] = {"median_ms": statistics.median(ts), "median_ms_per_frame": statistics.median(ts) / per}
    out["equal"] = all(bool((b[1] == bufs[0][1]).all()) for b in bufs[1:])
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

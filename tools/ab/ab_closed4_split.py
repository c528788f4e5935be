#!/usr/bin/env python3
"""Config-4 closed loop, split timing for A/B: luma alone, chroma alone, and the
two concurrent (gpu.tu_pipeline_closed_yuv420), each launch set timed on its
own with HIP events, REPS times after warm-up; one JSON line with the median and
min of each, plus an output digest (equal digests = equal outputs).

    python tools/ab/ab_closed4_split.py [--lib PATH | --ab] [--frames 64] [--reps 15]

Run several processes alternating the libraries / knob sets being compared
(tools/ab/ab_closed4_split.sh): the concurrent time depends on how the two
launches split the CUs, which varies between processes.
"""
import argparse
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
    ap.add_argument("--lib", default=None)
    ap.add_argument("--ab", action="store_true")
    ap.add_argument("--frames", type=int, default=64)
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--qp", type=int, default=32)
    ap.add_argument("--pipe", type=int, default=0,
                    help="also time K back-to-back launch sets over two stream pairs (two output copies), "
                         "one status check at the end (form pipeK)")
    ap.add_argument("--depth", type=int, default=2, help="stream pairs / output copies of --pipe")
    ap.add_argument("--only-pipe", action="store_true")
    ap.add_argument("--one-stream", action="store_true", help="--pipe: a set's luma then chroma on ONE stream")
    args = ap.parse_args()
    from nano_hevc import gpu, _lib
    from bench_configs import synth_plane
    if args.lib:
        import ctypes
        probe = ctypes.CDLL(os.path.abspath(args.lib))
        for name in [n for n in _lib.SIGNATURES if not hasattr(probe, n)]:
            del _lib.SIGNATURES[name]
        _lib.LIB_PATH = os.path.abspath(args.lib)
    if args.ab:
        _lib.use_ab()
    _lib.load()
    torch.cuda.set_device(0)
    W, H, nf = 3840, 2160, args.frames
    planes = []
    for f in range(nf):
        planes += [synth_plane(H, W, 40 + 3 * f).reshape(-1), synth_plane(H // 2, W // 2, 41 + 3 * f).reshape(-1),
                   synth_plane(H // 2, W // 2, 42 + 3 * f).reshape(-1)]
    stream = torch.cat(planes)
    del planes
    sy, suv = gpu.yuv420_plane_sets(nf, W, H)
    lv = torch.zeros(stream.shape, dtype=torch.int32, device="cuda")
    rc = torch.zeros(stream.shape, dtype=torch.int16, device="cuda")
    tuy = torch.zeros((nf, H // 4, W // 4), dtype=torch.uint8, device="cuda")
    tuc = torch.zeros((2 * nf, H // 8, W // 8), dtype=torch.uint8, device="cuda")
    side = torch.cuda.Stream()

    def luma_first():   # the same two launches, luma submitted before chroma (the product forks chroma first)
        main = torch.cuda.current_stream()
        fork = torch.cuda.Event()
        fork.record(main)
        side.wait_event(fork)
        gpu._tu_closed_launch(stream, sy, 32, 0, 1234, args.qp, True, lv, rc, tuy, main)
        gpu._tu_closed_launch(stream, suv, 16, 1, 1234, args.qp, False, lv, rc, tuc, side)
        join = torch.cuda.Event()
        join.record(side)
        main.wait_event(join)

    def chroma_first():   # the same two launches, chroma submitted first (its waves take their slots first)
        main = torch.cuda.current_stream()
        fork = torch.cuda.Event()
        fork.record(main)
        side.wait_event(fork)
        gpu._tu_closed_launch(stream, suv, 16, 1, 1234, args.qp, False, lv, rc, tuc, side)
        gpu._tu_closed_launch(stream, sy, 32, 0, 1234, args.qp, True, lv, rc, tuy, main)
        join = torch.cuda.Event()
        join.record(side)
        main.wait_event(join)

    pipe_bufs = []
    if args.pipe:   # a second copy of the frames and outputs: consecutive sets alternate between the copies
        pipe_bufs = [(stream, lv, rc, tuy, tuc)] + [
            (stream.clone(), torch.zeros_like(lv), torch.zeros_like(rc), torch.zeros_like(tuy), torch.zeros_like(tuc))
            for _ in range(args.depth - 1)]
        pipe_streams = [(torch.cuda.Stream(), torch.cuda.Stream()) for _ in range(args.depth)]

    def pipe():   # K launch sets, set k on stream pair k % depth, no host round trip between sets
        main = torch.cuda.current_stream()
        fork = torch.cuda.Event()
        fork.record(main)
        for pr in pipe_streams:
            for s_ in pr:
                s_.wait_event(fork)
        works = []
        for k in range(args.pipe):
            src_, lv_, rc_, ty_, tc_ = pipe_bufs[k % args.depth]
            ls, cs = pipe_streams[k % args.depth]
            if args.one_stream:
                cs = ls
            works.append(gpu._tu_closed_launch(src_, sy, 32, 0, 1234, args.qp, True, lv_, rc_, ty_, ls)[3])
            works.append(gpu._tu_closed_launch(src_, suv, 16, 1, 1234, args.qp, False, lv_, rc_, tc_, cs)[3])
        for pr in pipe_streams:
            for s_ in pr:
                j = torch.cuda.Event()
                j.record(s_)
                main.wait_event(j)
        for w_ in works:
            gpu._tu_closed_status(w_, int(main.cuda_stream), "pipe")

    forms = {
        "luma": lambda: gpu.tu_pipeline_closed(stream, sy, 32, 0, 1234, args.qp, True, lvl=lv, rec=rc, tu=tuy),
        "chroma": lambda: gpu.tu_pipeline_closed(stream, suv, 16, 1, 1234, args.qp, False, lvl=lv, rec=rc, tu=tuc),
        "concurrent": lambda: gpu.tu_pipeline_closed_yuv420(stream, sy, suv, 1234, args.qp, lvl=lv, rec=rc,
                                                            tu_luma=tuy, tu_chroma=tuc),
        "luma_first": luma_first,
        "chroma_first": chroma_first,
    }
    if args.only_pipe:
        forms = {}
    if args.pipe:
        forms[f"pipe{args.pipe}d{args.depth}" + ("s" if args.one_stream else "")] = pipe
    out = {"lib": args.lib or ("ab" if args.ab else "product"),
           "knobs": {k: v for k, v in os.environ.items() if k.startswith("NH_")}, "frames": nf}
    for name, fn in forms.items():
        fn()
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
        per = nf * (args.pipe if name.startswith("pipe") else 1)
        out[name] = {"median_ms": statistics.median(ts), "min_ms": min(ts),
                     "median_ms_per_frame": statistics.median(ts) / per}
    out["out_digest"] = [int(lv.to(torch.int64).sum().item()), int(rc.to(torch.int64).sum().item())]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

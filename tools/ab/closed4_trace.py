#!/usr/bin/env python3
"""Config-4 closed loop: which wavefront finishes last when luma and chroma run
concurrently.  Runs gpu.tu_pipeline_closed_yuv420 REPS times (after warm-up);
run it under `rocprofv3 --kernel-trace` and summarise the trace with --summary:
per launch set, the luma / chroma pair kernels' start and end relative to the
set's first kernel start (ms).

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt_x -o run -- python3 tools/ab/closed4_trace.py
    python tools/ab/closed4_trace.py --summary gpurun_out/kt_x
"""
import argparse
import csv
import glob
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "nano-hevc_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def summary(d):
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = [r for r in csv.DictReader(open(f)) if "k_tu_closed_pair" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    sets = []
    for i in range(0, len(rows) - 1, 2):
        a, b = rows[i], rows[i + 1]
        t0 = min(int(a["Start_Timestamp"]), int(b["Start_Timestamp"]))
        rec = {}
        for r in (a, b):
            k = "luma" if ", 32, " in r["Kernel_Name"] or "Li32E" in r["Kernel_Name"] else "chroma"
            rec[k] = ((int(r["Start_Timestamp"]) - t0) / 1e6, (int(r["End_Timestamp"]) - t0) / 1e6)
        sets.append(rec)
    sets = sets[2:]   # warm-up
    out = {k: {"start_ms": statistics.median(s[k][0] for s in sets), "end_ms": statistics.median(s[k][1] for s in sets)}
           for k in ("luma", "chroma")}
    out["sets"] = len(sets)
    print(json.dumps(out))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=64)
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--summary", default=None)
    a = ap.parse_args()
    if a.summary:
        return summary(a.summary)
    import torch
    from nano_hevc import gpu
    from bench_configs import synth_plane
    W, H, nf = 3840, 2160, a.frames
    planes = []
    for f in range(nf):
        planes += [synth_plane(H, W, 40 + 3 * f).reshape(-1), synth_plane(H // 2, W // 2, 41 + 3 * f).reshape(-1),
                   synth_plane(H // 2, W // 2, 42 + 3 * f).reshape(-1)]
    stream = torch.cat(planes)
    sy, suv = gpu.yuv420_plane_sets(nf, W, H)
    lv = torch.zeros(stream.shape, dtype=torch.int32, device="cuda")
    rc = torch.zeros(stream.shape, dtype=torch.int16, device="cuda")
    for _ in range(a.reps + 2):
        gpu.tu_pipeline_closed_yuv420(stream, sy, suv, 1234, 32, lvl=lv, rec=rc)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Headline benchmark: transform-blocks/sec (8x8 DCT+quant, 4K YUV420) on 1..N MI355X.

A "step" = one launch of the fused 8x8 forward DCT + quant (QP 32, intra
offset) over this rank's share of a batch of synthetic 4K YUV420 int16 residual
frames already resident in HBM (BASELINE.json configs[1] kernel on the
metric's 4K YUV420 stream).  Multi-GPU (nano_hevc/shard.py):
every frame is cut into N balanced CTU-row bands, band b of frame f goes to
rank (b - f) mod N, over a global batch of N x frames_per_gpu frames -- every
rank carries exactly frames_per_gpu frames of blocks, no data-path collective,
weak scaling.  With N > 1 a separate, shorter phase also times the path's one
exchange step (RCCL gather of the levels to rank 0) and reports it as
``gather_inclusive``.  Timing: W warmup steps, then K steps between barrier +
synchronize; the max over ranks is reported.  Rank 0 prints one JSON line.

Roofline: algorithmic bytes per 8x8 block = 128 B int16 in + 128 B int16 out
 x blocks per launch / average launch duration (HIP events
on the launch stream), against 8.0 TB/s.  ``traffic`` comes from the rocprofv3
PMC pass committed under profiles/ (tools/pmc_traffic.py) when one matches this
configuration, else null.

cpu_baseline (rank 0, N=1 only): the CPU restatement oracle/ ("port") timed on
a bounded sample of the same workload, on all of the job's host threads
("value", "cores") and on one thread ("value_1thread"); the same sample's GPU
levels are checked bit-exact against it.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "nano-hevc_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "transform-blocks/sec (8×8 DCT+quant, 4K YUV420) at 1/2/4/8 MI355X; % HBM roofline"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
BYTES_PER_BLOCK = 256          # 64 x int16 in + 64 x int16 out
W4K, H4K = 3840, 2160


def load_traffic(cfg_key: str):
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(p):
        return None
    try:
        d = json.load(open(p))
    except Exception:
        return None
    e = d.get(cfg_key)
    return None if e is None else e.get("hbm_bytes_per_launch")


def cpu_threads() -> int:
    """Host threads for the all-cores leg: the job's CPU share (OMP_NUM_THREADS
    on the GPU box = 16), else the affinity mask; nproc there shows the whole
    machine, not this job's share."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    return len(os.sched_getaffinity(0))


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(gpu_out: torch.Tensor, res: torch.Tensor, fe: int, frames: int, qp: int, budget_s: float):
    """Time the oracle (CPU restatement) on whole 4K YUV420 frames: first 1
    thread, then all of the job's host threads, each for
    ~budget_s/2; the GPU levels of every sampled frame are checked bit-exact
    against the single-thread output, and the threaded output against that."""
    from oracle import oracle as O   # checker + CPU baseline only
    O.lib()
    nthr = cpu_threads()
    cw, ch = W4K // 2, H4K // 2
    planes = [(0, H4K, W4K), (W4K * H4K, ch, cw), (W4K * H4K + cw * ch, ch, cw)]
    legs = {}
    exact = True
    for threads in (1, nthr):
        done_blocks, t_cpu, f = 0, 0.0, 0
        while f < frames and (t_cpu < budget_s / 2 or f == 0):
            r = res[f * fe:(f + 1) * fe].cpu().numpy()
            g = gpu_out[f * fe:(f + 1) * fe].cpu().numpy()
            for off, h, w in planes:
                p = r[off:off + h * w].reshape(h, w)
                t0 = time.perf_counter()
                if threads == 1:
                    lv = O.fwd8x8_quant_plane(p, qp, True)
                else:
                    lv = O.fwd8x8_quant_plane_mt(p, qp, True, threads)
                t_cpu += time.perf_counter() - t0
                done_blocks += (h // 8) * (w // 8)
                exact &= bool(np.array_equal(lv, g[off:off + h * w].reshape(h, w)))
            f += 1
        legs[threads] = (done_blocks / t_cpu, f, done_blocks, t_cpu)
    v1, f1, b1, t1 = legs[1]
    vn, fn, bn, tn = legs[nthr]
    return {"value": vn, "unit": "blocks/s", "cores": nthr, "kind": "port",
            "sample": f"{fn} whole 4K YUV420 frames ({bn} 8x8 blocks, QP {qp}) through oracle/nh_oracle.c "
                      f"fwd8x8_quant_plane_mt on {nthr} threads ({tn:.1f} s); single thread: {f1} frames, "
                      f"{b1} blocks, {t1:.1f} s",
            "value_1thread": v1, "cpu_model": cpu_model(), "nproc_machine": os.cpu_count(),
            "gpu_levels_bit_exact_on_sample": exact}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--frames", type=int, default=128, help="4K YUV420 frames per GPU per step")
    ap.add_argument("--qp", type=int, default=32)
    ap.add_argument("--variant", type=int, default=4341, help="launch variant (nanohevc.h); 4341 = default")
    ap.add_argument("--cpu-seconds", type=float, default=20.0, help="CPU baseline budget, split between the 1-thread and all-threads legs")
    ap.add_argument("--gather-steps", type=int, default=3, help="N>1: steps of the gather-inclusive phase")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # NH_DIST_BACKEND / NH_FORCE_DEVICE: rehearsal knobs only (e.g. 2 gloo ranks
        # sharing the one GPU of a test box); the driver's runs use RCCL, 1 GPU/rank.
        backend = os.environ.get("NH_DIST_BACKEND", "nccl")
        local = int(os.environ.get("NH_FORCE_DEVICE", local))
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    else:
        dist = None
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    from nano_hevc import gpu, _lib
    _lib.load()

    from nano_hevc import shard
    frames_global = args.frames * world
    layout = shard.rank_layout(rank, world, frames_global, W4K, H4K)
    sets = layout.plane_sets(gpu)
    nblk = gpu.blocks_in(sets)
    assert nblk == layout.blocks() == args.frames * 194400, (nblk, layout.blocks())
    fe = gpu.yuv420_frame_elems(W4K, H4K)
    # synthetic residual: U[-255,255] (worst-case 8-bit residual magnitude), seeded per rank
    gen = torch.Generator(device=dev)
    gen.manual_seed(1234 + rank)
    res = torch.randint(-255, 256, (layout.total_elems,), dtype=torch.int16, device=dev, generator=gen)
    out = torch.zeros_like(res)
    stream = torch.cuda.current_stream()

    def step():
        gpu.fwd8x8_quant(res, sets, args.qp, True, out=out, variant=args.variant, stream=stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for a, b in ev:
        a.record(stream)
        step()
        b.record(stream)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = sum(a.elapsed_time(b) for a, b in ev) / args.steps

    t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
    blocks_t = torch.tensor([nblk], dtype=torch.float64, device=dev)
    if dist:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(blocks_t, op=dist.ReduceOp.SUM)
    elapsed, kern_ms = float(t[0]), float(t[1])
    total_blocks = float(blocks_t[0]) * args.steps
    value = total_blocks / elapsed

    gather = None
    if dist and args.gather_steps > 0:
        # the path's one exchange step: levels of every rank -> rank 0 (RCCL gather over xGMI)
        sizes = [shard.rank_layout(r, world, frames_global, W4K, H4K).total_elems for r in range(world)]
        dist.barrier()
        torch.cuda.synchronize()
        g0 = time.perf_counter()
        for _ in range(args.gather_steps):
            step()
            shard.gather_to_root(out, sizes, dist)
        torch.cuda.synchronize()
        dist.barrier()
        gt = torch.tensor([time.perf_counter() - g0], dtype=torch.float64, device=dev)
        dist.all_reduce(gt, op=dist.ReduceOp.MAX)
        gv = float(blocks_t[0]) * args.gather_steps / float(gt[0])
        gather = {"value": gv, "unit": "blocks/s", "steps": args.gather_steps,
                  "ms_per_step": float(gt[0]) / args.gather_steps * 1e3,
                  "bytes_gathered_per_step": 2 * sum(sizes[1:]),
                  "note": "compute + torch.distributed.gather (RCCL) of int16 levels to rank 0"}

    if rank == 0:
        achieved = nblk * BYTES_PER_BLOCK / (kern_ms * 1e-3) / 1e9
        cfg_key = f"fwd8x8_qp{args.qp}_4k_yuv420_f{args.frames}_v{args.variant}_n{world}"
        traffic = load_traffic(cfg_key)
        line = {
            "metric": METRIC, "value": value, "unit": "blocks/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "int32",
            "data": "synthetic (seeded U[-255,255] int16 residual frames, resident in HBM)",
            "config": {"workload": "4K YUV420 residual frame stream, fused fwd 8x8 int-DCT + quant QP32 intra "
                                   "(cfg 2 kernel on the metric's 4K stream), CTU-row band sharding",
                       "frames_per_gpu": args.frames, "blocks_per_launch": nblk, "qp": args.qp,
                       "resolution": "3840x2160 YUV420 int16 in / int16 levels out",
                       "parallelism": f"ctu-band{world} (rotated)", "kernel_variant": args.variant},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "bytes_per_block": BYTES_PER_BLOCK, "kernel_ms_avg": kern_ms},
            "cpu_baseline": None,
        }
        if gather:
            line["gather_inclusive"] = gather
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(out, res, fe, frames_global, args.qp, args.cpu_seconds)  # N=1: whole frames
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Config 4 (BASELINE.json configs[3]) sharded across GPUs: 4K YUV420 frames,
mixed 4/8/16/32 TUs per 32x32 CTU, CTU-row bands per rank, RCCL gather of the
reconstructed bands to rank 0.

    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P tools/dist_cfg4.py [--check]

Every rank holds the whole synthetic input stream (the TU chain reads the
source row above its band, block.py:38-50) and runs nh_tu_pipeline_planes on
its bands only: band b of frame f is rank (b - f) mod N's, so the frames of
one band on one rank are evenly strided and form one plane set (2 sets x 4 TU
sizes per band).  Weak scaling: frames_per_gpu frames of work per rank.
Prints one JSON line on rank 0: compute-only samples/s (max over ranks) and
the gather-inclusive rate; with --check rank 0 also recomputes the whole
stream unsharded and compares the gathered reconstruction bit for bit.
NH_DIST_BACKEND=gloo / NH_FORCE_DEVICE=0: rehearsal of N ranks on one GPU.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nano-hevc_amd"))

import torch  # noqa: E402


def synth_stream(nf, w, h, seed, dev):
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    parts = []
    for f in range(nf):
        for pw, ph in ((w, h), (w // 2, h // 2), (w // 2, h // 2)):
            yy = torch.arange(ph, device=dev).view(ph, 1)
            xx = torch.arange(pw, device=dev).view(1, pw)
            base = (50 + (3 * xx + 2 * yy + 13 * f) % 150 + (xx // 97) * 5) % 256
            noise = torch.randint(-15, 16, (ph, pw), device=dev, generator=g)
            parts.append(torch.clamp(base + noise, 0, 255).to(torch.int16).reshape(-1))
    return torch.cat(parts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames-per-gpu", type=int, default=8)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--qp", type=int, default=32)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--check", action="store_true")
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = os.environ.get("NH_DIST_BACKEND", "nccl")
        local = int(os.environ.get("NH_FORCE_DEVICE", local))
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    from nano_hevc import gpu, shard, _lib
    _lib.load()

    W, H = 3840, 2160
    cw, ch = W // 2, H // 2
    fe = gpu.yuv420_frame_elems(W, H)
    nf = args.frames_per_gpu * world
    stream = synth_stream(nf, W, H, args.seed, dev)          # identical on every rank
    lvl = torch.zeros(stream.shape, dtype=torch.int32, device=dev)
    rec = torch.zeros(stream.shape, dtype=torch.int16, device=dev)
    bands = shard.ctu_bands(H, world)
    plan = shard.cfg4_plan(rank, world, nf)
    work = []
    for b, f0, cnt in plan:
        y0, y1 = bands[b]
        r0, r1 = y0 // 32, (y1 + 31) // 32
        sy = gpu.plane_set(f0 * fe, W, H, W, 1, cnt, 0, world * fe)
        suv = gpu.plane_set(f0 * fe + W * H, cw, ch, cw, 2, cnt, cw * ch, world * fe)
        tuy = torch.zeros((cnt, H // 4, W // 4), dtype=torch.uint8, device=dev)
        tuc = torch.zeros((2 * cnt, ch // 4, cw // 4), dtype=torch.uint8, device=dev)
        work.append((sy, suv, r0, r1, tuy, tuc))
    my_samples = sum(cnt * (W * (bands[b][1] - bands[b][0]) + 2 * cw * (bands[b][1] // 2 - bands[b][0] // 2))
                     for b, f0, cnt in plan)

    def step():
        for sy, suv, r0, r1, tuy, tuc in work:
            gpu.tu_pipeline_planes(stream, sy, 32, 0, args.seed, args.qp, True, r0, r1, lvl=lvl, rec=rec, tu=tuy)
            gpu.tu_pipeline_planes(stream, suv, 16, 1, args.seed, args.qp, False, r0, r1, lvl=lvl, rec=rec, tu=tuc)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    el = torch.tensor([time.perf_counter() - t0, my_samples], dtype=torch.float64, device=dev)
    tot = el.clone()
    if dist:
        dist.all_reduce(el[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(tot[1:], op=dist.ReduceOp.SUM)
    elapsed, samples = float(el[0]), float(tot[1])

    # the exchange step: pack this rank's reconstructed bands, gather to rank 0
    sizes = [shard.cfg4_packed_elems(r, world, nf, W, H) for r in range(world)]
    gather = None
    full = None
    if dist:
        dist.barrier()
        torch.cuda.synchronize()
        g0 = time.perf_counter()
        for _ in range(args.steps):
            step()
            got = shard.gather_to_root(shard.cfg4_pack(rec, rank, world, nf, W, H), sizes, dist)
        torch.cuda.synchronize()
        dist.barrier()
        gt = torch.tensor([time.perf_counter() - g0], dtype=torch.float64, device=dev)
        dist.all_reduce(gt, op=dist.ReduceOp.MAX)
        gather = {"frames_per_s": nf * args.steps / float(gt[0]), "ms_per_step": float(gt[0]) / args.steps * 1e3,
                  "bytes_gathered_per_step": 2 * sum(sizes[1:]),
                  "note": "compute + band pack + torch.distributed.gather (RCCL) of int16 recon bands to rank 0"}
        if rank == 0:
            full = torch.zeros_like(rec)
            for r in range(world):
                shard.cfg4_unpack(got[r], r, world, nf, W, H, full)
    else:
        full = rec
    if rank == 0:
        line = {"config": "cfg4 sharded: 4K YUV420, mixed 4/8/16/32 TUs per 32x32 CTU, CTU-row bands per GPU, "
                          "RCCL gather of recon bands",
                "n_gpus": world, "frames_per_gpu": args.frames_per_gpu, "steps": args.steps,
                "compute": {"frames_per_s": nf * args.steps / elapsed, "samples_per_s": samples * args.steps / elapsed,
                            "ms_per_step": elapsed / args.steps * 1e3},
                "scaling": "weak", "gather_inclusive": gather}
        if args.check:
            ref_l = torch.zeros_like(lvl)
            ref_r = torch.zeros_like(rec)
            sy, suv = gpu.yuv420_plane_sets(nf, W, H)
            gpu.tu_pipeline_planes(stream, sy, 32, 0, args.seed, args.qp, True, lvl=ref_l, rec=ref_r)
            gpu.tu_pipeline_planes(stream, suv, 16, 1, args.seed, args.qp, False, lvl=ref_l, rec=ref_r)
            line["gathered_recon_equals_unsharded"] = bool(torch.equal(full, ref_r))
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

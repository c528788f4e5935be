#!/usr/bin/env python3
"""Headline benchmark: transform-blocks/sec (8x8 DCT+quant, 4K YUV420) on 1..N MI355X.

    python bench.py --gpus N --steps K --warmup W            (N > 1: launches N ranks itself)
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Launch: one process per GPU.  When WORLD_SIZE is unset and --gpus N > 1 the
parent process starts `torch.distributed.run --nproc-per-node N` on this same
script and exits with its status -- it never touches the GPU itself.  Under a
launcher, WORLD_SIZE must equal --gpus (else exit 2); n_gpus in the line is the
process group's world size.

--config 2 (default; BASELINE.json configs[1] kernel on the metric's 4K stream):
a "step" = one launch of the fused 8x8 forward DCT + quant (QP 32, intra
offset) over this rank's share of a batch of synthetic 4K YUV420 int16 residual
frames already resident in HBM.  Every frame is cut into N
balanced CTU-row bands, band b of frame f goes to rank (b - f) mod N, over a
global batch of N x frames_per_gpu frames (nano_hevc/shard.py): every rank
carries exactly frames_per_gpu frames of blocks, no data-path collective, weak
scaling.

--config 4 (BASELINE.json configs[3]): 4K YUV420 frames, mixed 4/8/16/32 TUs
per 32x32 CTU, CTU-row bands per rank as above; every rank
holds the whole synthetic input stream (a TU reads the source row above its
band, block.py:38-50) and reconstructs only its bands.

N > 1, both configs: after the compute-only phase, a gather-inclusive phase
runs the path's one exchange step -- an RCCL gather to rank 0 (config 2: a
--gather-frames sample of the int16 levels, 8 of 128 frames by default;
config 4: all reconstructed bands as uint8, clip_to_pixel_range guarantees
[0, 255]) -- on a side stream, the gather of step k overlapped with
the compute of step k+1 (double-buffered outputs).  Reported as
``gather_inclusive`` with the bytes into rank 0 and the achieved xGMI rate.

Timing: W warmup steps, then K steps between barrier + synchronize; the max
over ranks is reported; ``value`` = units of all ranks / that time.  Rank 0
prints one JSON line.

Roofline (config 2): algorithmic bytes per 8x8 block = 128 B int16 in + 128 B
int16 out x blocks per launch / average launch duration
(HIP events on the launch stream), against 8.0 TB/s; ``traffic`` = the PMC
bytes per launch committed in profiles/pmc_traffic.json for this configuration
(tools/pmc_traffic.py), else null.  Config 4: 2 B source + 4 B levels + 2 B
recon + 1/16 B TU map per sample.

cpu_baseline (rank 0, N=1 only): the CPU restatement in oracle/ ("port") on a
bounded sample of the same workload, on all of the job's host threads (config
2) and on one thread; the sample's GPU outputs are checked bit-exact against it.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "nano-hevc_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402   (importing torch does not initialise the GPU)

METRIC = "transform-blocks/sec (8×8 DCT+quant, 4K YUV420) at 1/2/4/8 MI355X; % HBM roofline"
METRIC_CFG4 = "samples/sec (4K YUV420, mixed 4/8/16/32 TUs per 32x32 CTU: pred+DCT+quant+dequant+IDCT+recon)"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
BYTES_PER_BLOCK = 256          # 64 x int16 in + 64 x int16 out
BYTES_PER_SAMPLE_CFG4 = 2 + 4 + 2 + 1 / 16
W4K, H4K = 3840, 2160


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", type=int, default=2, choices=(2, 4), help="2: headline 8x8 DCT+quant; 4: mixed-TU chain")
    ap.add_argument("--frames", type=int, default=None,
                    help="4K YUV420 frames per GPU per step (default 128 for config 2, 16 for config 4)")
    ap.add_argument("--qp", type=int, default=32)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--variant", type=int, default=4341, help="config 2 launch variant (nanohevc.h); 4341 = default")
    ap.add_argument("--cpu-seconds", type=float, default=20.0, help="CPU baseline budget (1-thread + all-threads legs)")
    ap.add_argument("--gather-steps", type=int, default=3, help="N>1: timed steps of the gather-inclusive phase")
    ap.add_argument("--gather-frames", type=int, default=8,
                    help="config 2, N>1: frames' worth of int16 levels each rank ships to rank 0 per gathered step "
                         "(a bounded sample of its output; the whole output would be 3.2 GB per rank at 128 frames)")
    ap.add_argument("--check", action="store_true", help="config 4, N>1: rank 0 compares the gathered recon with "
                                                          "an unsharded run")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--launcher-selftest", action="store_true", help=argparse.SUPPRESS)
    a = ap.parse_args(argv)
    if a.frames is None:
        a.frames = 128 if a.config == 2 else 16
    if a.gpus < 1:
        ap.error("--gpus must be >= 1")
    return a


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_or_check(args, argv):
    """None: run in this process.  An int: exit with it (the launched ranks'
    status, or 2 for a WORLD_SIZE / --gpus mismatch).  The parent never
    initialises the GPU: it only starts the ranks as a child process."""
    ws = os.environ.get("WORLD_SIZE")
    if ws is None:
        if args.gpus == 1:
            return None
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr", "127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + list(argv)
        return subprocess.run(cmd, env=dict(os.environ)).returncode
    if int(ws) != args.gpus:
        print(f"bench.py: WORLD_SIZE={ws} but --gpus {args.gpus}; refusing to report a mislabelled run",
              file=sys.stderr)
        return 2
    return None


def init_dist(world):
    """Process group for world > 1 (RCCL, one GPU per rank).  NH_DIST_BACKEND /
    NH_FORCE_DEVICE are rehearsal knobs of this script only (e.g. 2 gloo ranks
    sharing the one GPU of a test box)."""
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world == 1:
        torch.cuda.set_device(0)
        return None
    import torch.distributed as dist
    backend = os.environ.get("NH_DIST_BACKEND", "nccl")
    local = int(os.environ.get("NH_FORCE_DEVICE", local))
    torch.cuda.set_device(local)
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist.init_process_group(backend)
    return dist


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


def cpu_baseline(gpu_out, res, fe: int, frames: int, qp: int, budget_s: float):
    """Time the oracle (CPU restatement) on whole 4K YUV420 frames: first 1
    thread, then all of the job's host threads, each for
    ~budget_s/2; the GPU levels of every sampled frame are checked bit-exact."""
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


def timed_steps(step, steps, warmup, dist, stream):
    """W warmup steps, then K steps between barrier + synchronize on both sides.
    Returns (wall seconds, mean HIP-event ms per step on the launch stream)."""
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
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
    return elapsed, sum(a.elapsed_time(b) for a, b in ev) / steps


def reduce_max_sum(dist, dev, maxes, sums):
    t = torch.tensor(list(maxes), dtype=torch.float64, device=dev)
    u = torch.tensor(list(sums), dtype=torch.float64, device=dev)
    if dist:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(u, op=dist.ReduceOp.SUM)
    return [float(x) for x in t], [float(x) for x in u]


class OverlappedGather:
    """The exchange step on a side stream: gather(k) waits for compute(k) and
    runs under compute(k+1); the two output buffers alternate, and compute(k+2)
    waits for gather(k) before overwriting its buffer.  ``send_of(k)`` returns
    the flat tensor to send after compute(k) (on the side stream)."""

    def __init__(self, dist, dev, sizes, dtype):
        self.dist, self.dev = dist, dev
        self.gloo = dist.get_backend() == "gloo"
        self.rank, self.world = dist.get_rank(), dist.get_world_size()
        self.n = max(sizes)
        self.side = torch.cuda.Stream(device=dev)
        self.done = [None, None]
        self.recv = None
        if self.rank == 0:
            rdev = "cpu" if self.gloo else dev
            self.recv = [torch.empty(self.n, dtype=dtype, device=rdev) for _ in range(self.world)]

    def wait_free(self, slot, main):
        if self.done[slot] is not None:
            main.wait_event(self.done[slot])

    def gather(self, slot, main, send_fn):
        ready = torch.cuda.Event()
        ready.record(main)
        with torch.cuda.stream(self.side):
            self.side.wait_event(ready)
            send = send_fn()
            if self.gloo:   # gloo gathers host tensors: a synchronous rehearsal of the same call
                send = send.cpu()
            if self.rank == 0:
                self.dist.gather(send, gather_list=self.recv, dst=0)
            else:
                self.dist.gather(send, dst=0)
            done = torch.cuda.Event()
            done.record(self.side)
            self.done[slot] = done


def run_phase_gather(step_into, send_of, og, steps, dist, main):
    """Gather-inclusive phase: one unmeasured round trip (communicator setup),
    then ``steps`` timed steps with the gather of step k overlapped with step k+1."""
    og.wait_free(0, main)
    step_into(0)
    og.gather(0, main, lambda: send_of(0))
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        slot = k % 2
        og.wait_free(slot, main)
        step_into(slot)
        og.gather(slot, main, lambda s=slot: send_of(s))
    torch.cuda.synchronize()
    dist.barrier()
    return time.perf_counter() - t0


# ---------------------------------------------------------------------------
# config 2: the headline kernel
# ---------------------------------------------------------------------------
def run_cfg2(args, dist, world, rank, dev):
    from nano_hevc import gpu, shard, _lib
    _lib.load()
    frames_global = args.frames * world
    layout = shard.rank_layout(rank, world, frames_global, W4K, H4K)
    sets = layout.plane_sets(gpu)
    nblk = gpu.blocks_in(sets)
    assert nblk == layout.blocks() == args.frames * 194400, (nblk, layout.blocks())
    fe = gpu.yuv420_frame_elems(W4K, H4K)
    sizes = [shard.rank_layout(r, world, frames_global, W4K, H4K).total_elems for r in range(world)]
    padded = -(-max(sizes) // 4) * 4       # int16 elements, a whole number of 8-byte words on every rank
    # synthetic residual: U[-255,255] (worst-case 8-bit residual magnitude), seeded per rank
    gen = torch.Generator(device=dev)
    gen.manual_seed(args.seed + rank)
    res = torch.randint(-255, 256, (layout.total_elems,), dtype=torch.int16, device=dev, generator=gen)
    outs = [torch.zeros(padded, dtype=torch.int16, device=dev)]
    stream = torch.cuda.current_stream(dev)

    def step_into(slot):
        gpu.fwd8x8_quant(res, sets, args.qp, True, out=outs[slot], variant=args.variant, stream=stream)

    elapsed, kern_ms = timed_steps(lambda: step_into(0), args.steps, args.warmup, dist, stream)
    (elapsed, kern_ms), (blocks_all,) = reduce_max_sum(dist, dev, (elapsed, kern_ms), (nblk,))
    value = blocks_all * args.steps / elapsed

    gather = None
    if dist and args.gather_steps > 0:
        outs.append(torch.zeros_like(outs[0]))
        frac = min(1.0, args.gather_frames / args.frames)
        words = min(padded, -(-int(padded * frac) // 4) * 4) // 4   # int64 words sent per rank per step
        og = OverlappedGather(dist, dev, [words] * world, torch.int64)
        gt = run_phase_gather(step_into, lambda s: outs[s].view(torch.int64)[:words], og, args.gather_steps, dist,
                              stream)
        (gt,), _ = reduce_max_sum(dist, dev, (gt,), ())
        into_root = 8 * words * (world - 1)
        gather = {"value": blocks_all * args.gather_steps / gt, "unit": "blocks/s", "steps": args.gather_steps,
                  "ms_per_step": gt / args.gather_steps * 1e3, "bytes_into_root_per_step": into_root,
                  "into_root_GBps": into_root * args.gather_steps / gt / 1e9, "overlapped": True,
                  "backend": dist.get_backend(), "levels_fraction_gathered": frac,
                  "note": f"compute + RCCL gather to rank 0 of a {args.gather_frames}-frame sample of every rank's "
                          "int16 levels per step (the head of its output), on a side stream, gather(k) under "
                          "compute(k+1); the exchange is bounded by rank 0's inbound xGMI (SURVEY.md §8e E-2)"}

    if rank != 0:
        return None
    achieved = nblk * BYTES_PER_BLOCK / (kern_ms * 1e-3) / 1e9
    cfg_key = f"fwd8x8_qp{args.qp}_4k_yuv420_f{args.frames}_v{args.variant}_n{world}"
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
                     "frac": achieved / HBM_PEAK_GBS, "traffic": load_traffic(cfg_key),
                     "bytes_per_block": BYTES_PER_BLOCK, "kernel_ms_avg": kern_ms},
        "cpu_baseline": None,
    }
    if gather:
        line["gather_inclusive"] = gather
    if world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(outs[0], res, fe, frames_global, args.qp, args.cpu_seconds)
    return line


# ---------------------------------------------------------------------------
# config 4: mixed 4/8/16/32 TUs per CTU, CTU-row bands, uint8 recon gather
# ---------------------------------------------------------------------------
def synth_stream(nf, w, h, seed, dev):
    """8-bit natural-ish content (gradient + seeded noise), identical on every rank."""
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


def band_views(stream, rank, world, frames, width, height):
    """This rank's reconstructed bands as strided views: per band, the Y / U / V
    rows of the frames f0, f0 + world, ... (one view per plane)."""
    from nano_hevc import shard
    fe = width * height + 2 * (width // 2) * (height // 2)
    cw, ch = width // 2, height // 2
    out = []
    for b, f0, cnt in shard.cfg4_plan(rank, world, frames):
        y0, y1 = shard.ctu_bands(height, world)[b]
        c0, c1 = y0 // 2, y1 // 2
        for off, n in ((width * y0, width * (y1 - y0)), (width * height + cw * c0, cw * (c1 - c0)),
                       (width * height + cw * ch + cw * c0, cw * (c1 - c0))):
            if n:
                out.append(stream.as_strided((cnt, n), (world * fe, 1), f0 * fe + off))
    return out


def run_cfg4(args, dist, world, rank, dev):
    from nano_hevc import gpu, shard, _lib
    _lib.load()
    W, H = W4K, H4K
    cw, ch = W // 2, H // 2
    fe = gpu.yuv420_frame_elems(W, H)
    nf = args.frames * world
    src = synth_stream(nf, W, H, args.seed, dev)          # the whole input stream on every rank
    lvl = torch.zeros(src.shape, dtype=torch.int32, device=dev)
    recs = [torch.zeros(src.shape, dtype=torch.int16, device=dev)]
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
    my_samples = shard.cfg4_packed_elems(rank, world, nf, W, H)
    stream = torch.cuda.current_stream(dev)

    def step_into(slot):
        for sy, suv, r0, r1, tuy, tuc in work:
            gpu.tu_pipeline_planes(src, sy, 32, 0, args.seed, args.qp, True, r0, r1, lvl=lvl, rec=recs[slot], tu=tuy,
                                   stream=stream)
            gpu.tu_pipeline_planes(src, suv, 16, 1, args.seed, args.qp, False, r0, r1, lvl=lvl, rec=recs[slot],
                                   tu=tuc, stream=stream)

    elapsed, kern_ms = timed_steps(lambda: step_into(0), args.steps, args.warmup, dist, stream)
    # TUs per size coded per step (blocks/s per TU size), from the TU maps
    # (one byte per 4x4 unit = log2 of its TU's size; bit 7 marks a group recoded by the wide kernel)
    tu_units = [0, 0, 0, 0]
    for _, _, _, _, tuy, tuc in work:
        for m in (tuy, tuc):
            ls = (m & 0x7F).reshape(-1).to(torch.int64)
            cnt = torch.bincount(ls, minlength=6)
            for k in range(4):
                tu_units[k] += int(cnt[k + 2])
    tu_counts = [tu_units[k] // (1 << (2 * k)) for k in range(4)]   # a TU of 4*2^k samples square = 4^k units
    (elapsed, kern_ms), sums = reduce_max_sum(dist, dev, (elapsed, kern_ms), [my_samples] + tu_counts)
    samples_all, tu_all = sums[0], sums[1:]
    value = samples_all * args.steps / elapsed

    sizes = [shard.cfg4_packed_elems(r, world, nf, W, H) for r in range(world)]
    gather, check = None, None
    if dist and args.gather_steps > 0:
        recs.append(torch.zeros_like(recs[0]))
        packed = [torch.zeros(max(sizes), dtype=torch.uint8, device=dev) for _ in range(2)]
        views = [band_views(r, rank, world, nf, W, H) for r in recs]

        def send_of(slot):   # pack + narrow this rank's recon bands (values in [0, 255]) on the side stream
            o = 0
            for v in views[slot]:
                n = v.numel()
                packed[slot][o:o + n].view(v.shape).copy_(v)
                o += n
            return packed[slot]

        og = OverlappedGather(dist, dev, sizes, torch.uint8)
        gt = run_phase_gather(step_into, send_of, og, args.gather_steps, dist, stream)
        (gt,), _ = reduce_max_sum(dist, dev, (gt,), ())
        into_root = sum(sizes[1:])
        gather = {"value": samples_all * args.gather_steps / gt, "unit": "samples/s", "steps": args.gather_steps,
                  "ms_per_step": gt / args.gather_steps * 1e3, "bytes_into_root_per_step": into_root,
                  "into_root_GBps": into_root * args.gather_steps / gt / 1e9, "overlapped": True,
                  "backend": dist.get_backend(),
                  "note": "compute + band pack + RCCL gather of the reconstructed bands as uint8 to rank 0 on a side "
                          "stream, gather(k) under compute(k+1)"}
        if args.check and rank == 0:   # reassemble the last gather and compare with an unsharded run
            torch.cuda.synchronize()
            full = torch.zeros_like(recs[0])
            for r in range(world):
                got = og.recv[r][:sizes[r]].to(dev)
                o = 0
                for v in band_views(full, r, world, nf, W, H):
                    v.copy_(got[o:o + v.numel()].view(v.shape))
                    o += v.numel()
            ref_l = torch.zeros_like(lvl)
            ref_r = torch.zeros_like(recs[0])
            sy, suv = gpu.yuv420_plane_sets(nf, W, H)
            gpu.tu_pipeline_planes(src, sy, 32, 0, args.seed, args.qp, True, lvl=ref_l, rec=ref_r)
            gpu.tu_pipeline_planes(src, suv, 16, 1, args.seed, args.qp, False, lvl=ref_l, rec=ref_r)
            check = bool(torch.equal(full, ref_r))

    if rank != 0:
        return None
    achieved = my_samples * BYTES_PER_SAMPLE_CFG4 / (kern_ms * 1e-3) / 1e9
    line = {
        "metric": METRIC_CFG4, "value": value, "unit": "samples/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "int32",
        "data": "synthetic 8-bit 4K YUV420 frames (gradient + seeded noise, int16 samples), resident in HBM",
        "config": {"workload": "config 4: 4K YUV420, seeded 4/8/16/32 TU quadtree per 32x32 CTU (16x16 chroma), "
                               "open-loop DC/planar choice, full chain, QP %d" % args.qp,
                   "frames_per_gpu": args.frames, "frames_per_s": value / (W * H + 2 * cw * ch),
                   "samples_per_step_rank0": my_samples, "parallelism": f"ctu-band{world} (rotated)",
                   "tu_blocks_per_step": {f"{4 << k}x{4 << k}": int(tu_all[k]) for k in range(4)},
                   "tu_blocks_per_s": {f"{4 << k}x{4 << k}": tu_all[k] * args.steps / elapsed for k in range(4)}},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": load_traffic(f"cfg4_4k_yuv420_f{args.frames}_n{world}"),
                     "traffic_note": "PMC bytes per step (all 4 launches): reads as the 64-B request tally (a lower "
                                     "bound for 8-B/lane row reads, <= 2x that if every request were 128 B), writes "
                                     "exact; profiles/pmc_traffic.json",
                     "bytes_per_sample": BYTES_PER_SAMPLE_CFG4,
                     "kernel_ms_avg": kern_ms},
        "cpu_baseline": None,
    }
    if gather:
        line["gather_inclusive"] = gather
    if check is not None:
        line["gathered_recon_equals_unsharded"] = check
    if world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline_cfg4(src, lvl, recs[0], args, fe)
    return line


def cpu_baseline_cfg4(src, lvl, rec, args, fe):
    """oracle tu_pipeline_plane (one thread) on whole frames of the same stream
    until ~cpu_seconds; the GPU levels and recon of those frames checked bit-exact."""
    from oracle import oracle as O   # checker + CPU baseline only
    O.lib()
    W, H = W4K, H4K
    cw, ch = W // 2, H // 2
    planes = [(0, H, W, 32, 0, True), (W * H, ch, cw, 16, 1, False), (W * H + cw * ch, ch, cw, 16, 2, False)]
    t_cpu, f, samples, exact = 0.0, 0, 0, True
    while f < args.frames and (t_cpu < args.cpu_seconds or f == 0):
        s = src[f * fe:(f + 1) * fe].cpu().numpy()
        gl = lvl[f * fe:(f + 1) * fe].cpu().numpy()
        gr = rec[f * fe:(f + 1) * fe].cpu().numpy()
        for off, h, w, ctb, pid, luma in planes:
            p = s[off:off + h * w].reshape(h, w)
            t0 = time.perf_counter()
            ol, orc, _ = O.tu_pipeline_plane(p, ctb, pid, args.seed, args.qp, luma)
            t_cpu += time.perf_counter() - t0
            samples += h * w
            exact &= bool(np.array_equal(ol, gl[off:off + h * w].reshape(h, w)) and
                          np.array_equal(orc, gr[off:off + h * w].reshape(h, w)))
        f += 1
    return {"value": samples / t_cpu, "unit": "samples/s", "cores": 1, "kind": "port",
            "sample": f"{f} whole 4K YUV420 frames ({samples} samples) through oracle/nh_oracle.c "
                      f"oh_tu_pipeline_plane on 1 thread ({t_cpu:.1f} s)",
            "cpu_model": cpu_model(), "gpu_outputs_bit_exact_on_sample": exact}


def launcher_selftest(world, rank):
    """CPU-only check of the launch path (tests/test_bench_launch.py): the ranks
    this script started join a gloo group and rank 0 reports the world size."""
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
        t = torch.tensor([rank], dtype=torch.int64)
        dist.all_reduce(t)
        world = dist.get_world_size()
        if rank == 0:
            print(json.dumps({"n_gpus": world, "rank_sum": int(t)}), flush=True)
        dist.destroy_process_group()
    else:
        print(json.dumps({"n_gpus": 1, "rank_sum": 0}), flush=True)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse_args(argv)
    rc = launch_or_check(args, argv)
    if rc is not None:
        return rc
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if args.launcher_selftest:
        launcher_selftest(world, rank)
        return 0
    dist = init_dist(world)
    if dist is not None:
        world = dist.get_world_size()
    dev = torch.device("cuda", torch.cuda.current_device())
    line = (run_cfg2 if args.config == 2 else run_cfg4)(args, dist, world, rank, dev)
    if line is not None:
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())

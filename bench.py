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
synthesises and holds only its bands plus the one source row above each band
(all a TU reads, block.py:38-50; shard.Cfg4Layout) and reconstructs them.

N > 1, both configs: after the compute-only phase, a gather-inclusive phase
runs the path's one exchange step -- an RCCL gather to rank 0 of every rank's
whole output (config 2: all its int16 levels, 3.2 GB per rank at 128 frames,
in --gather-chunk-frames pieces so rank 0's receive buffers stay bounded;
--gather-frames keeps only a sample, as an explicit option; config 4: all
reconstructed bands as uint8, clip_to_pixel_range guarantees [0, 255]) -- on a
side stream, the gather of step k overlapped with the compute of step k+1
(double-buffered outputs).  Reported as ``gather_inclusive`` with the bytes
into rank 0 and the achieved xGMI rate.

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
import ctypes as C
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
BYTES_PER_SAMPLE_CFG4 = 2 + 4 + 2 + 1 / 16   # int16 in, int32 levels + int16 recon out, 1 TU-map byte per 4x4
BYTES_PER_SAMPLE_CFG4_COMPACT = 2 + 2 + 2 + 1 / 16   # --levels int16: the exact compact levels
W4K, H4K = 3840, 2160


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", type=int, default=2, choices=(2, 4), help="2: headline 8x8 DCT+quant; 4: mixed-TU chain")
    ap.add_argument("--frames", type=int, default=None,
                    help="4K YUV420 frames per GPU per step (default 128 for config 2, 64 for config 4)")
    ap.add_argument("--qp", type=int, default=32)
    ap.add_argument("--levels", default="int16", choices=("int16", "int32"),
                    help="config 4: level dtype on the device -- int16 = the exact compact levels (|level| <= 408 "
                         "for an 8-bit TU; int32 spill for the rest, nh_tu_pipeline_planes_compact), int32 = the "
                         "reference's dtype")
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--variant", type=int, default=4341, help="config 2 launch variant (nanohevc.h); 4341 = default")
    ap.add_argument("--cpu-seconds", type=float, default=20.0, help="CPU baseline budget (1-thread + all-threads legs)")
    ap.add_argument("--gather-steps", type=int, default=3, help="N>1: timed steps of the gather-inclusive phase")
    ap.add_argument("--gather-frames", type=int, default=None,
                    help="config 2, N>1: frames' worth of int16 levels each rank ships to rank 0 per gathered step "
                         "(default: all --frames, the whole output; fewer = an explicit sample)")
    ap.add_argument("--gather-chunk-frames", type=int, default=8,
                    help="N>1: frames' worth of output per RCCL gather call (rank 0's receive buffers hold "
                         "one chunk per rank)")
    ap.add_argument("--check", action="store_true", help="config 4, N>1: rank 0 compares the gathered recon with "
                                                          "an unsharded run")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--launcher-selftest", action="store_true", help=argparse.SUPPRESS)
    a = ap.parse_args(argv)
    if a.frames is None:
        a.frames = 128 if a.config == 2 else 64
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


def init_dist(world, force_group=False):
    """Process group for world > 1 (RCCL, one GPU per rank); ``force_group``
    also builds one at world 1 (tests/rccl_world1.py: the RCCL branch and the
    device-tensor gather executed on a one-GPU box).  NH_DIST_BACKEND /
    NH_FORCE_DEVICE are rehearsal knobs of this script only (e.g. 2 gloo ranks
    sharing the one GPU of a test box)."""
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world == 1 and not force_group:
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


# The reference's own numpy path (quantize_block(forward_transform(block), 32) per 8x8 block), timed
# by the survey in the BUILD container: the reference cannot travel to the
# GPU box, so this is a different host's figure, reported beside the box's own C-port legs.
REFERENCE_NUMPY_CFG2 = {"value": 3102.0, "unit": "blocks/s", "cores": 1, "kind": "reference",
                        "host": "build container (8-vCPU Xeon), not the GPU box",
                        "sample": "reference nano_hevc.transform.forward_transform + quant.quantize_block, "
                                  "322 us per 8x8 block at QP 32 (SURVEY.md §6)"}


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
            "gpu_levels_bit_exact_on_sample": exact,
            "reference_numpy": REFERENCE_NUMPY_CFG2}


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
    the flat tensor to send after compute(k) (on the side stream); it goes to
    rank 0 in pieces of at most ``chunk`` elements (one gather call each, in
    order on the side stream), so rank 0 holds one piece per rank, whatever the
    output size.  ``on_chunk(off, n)``, when set, runs on the side stream after
    each piece has landed in ``recv`` (tests: what rank 0 received)."""

    def __init__(self, dist, dev, sizes, dtype, chunk=None):
        self.dist, self.dev = dist, dev
        self.gloo = dist.get_backend() == "gloo"
        self.rank, self.world = dist.get_rank(), dist.get_world_size()
        self.n = max(sizes)
        self.chunk = max(1, min(self.n, chunk or self.n))
        self.side = torch.cuda.Stream(device=dev)
        self.done = [None, None]
        self.recv = None
        self.on_chunk = None
        self.calls = 0
        if self.rank == 0:
            rdev = "cpu" if self.gloo else dev
            self.recv = [torch.empty(self.chunk, dtype=dtype, device=rdev) for _ in range(self.world)]

    def wait_free(self, slot, main):
        if self.done[slot] is not None:
            main.wait_event(self.done[slot])

    def gather(self, slot, main, send_fn):
        ready = torch.cuda.Event()
        ready.record(main)
        with torch.cuda.stream(self.side):
            self.side.wait_event(ready)
            send = send_fn()
            for off in range(0, send.numel(), self.chunk):
                n = min(self.chunk, send.numel() - off)
                piece = send[off:off + n]
                if self.gloo:   # gloo gathers host tensors: a synchronous rehearsal of the same call
                    piece = piece.cpu()
                if self.rank == 0:
                    self.dist.gather(piece, gather_list=[r[:n] for r in self.recv], dst=0)
                else:
                    self.dist.gather(piece, dst=0)
                self.calls += 1
                if self.on_chunk is not None:
                    self.on_chunk(off, n)
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
def _copy_GBps(run, nbytes, stream, reps=10):
    """Median rate (read + write counted) of `run()` enqueued on `stream`, by HIP events."""
    import statistics
    with torch.cuda.stream(stream):
        run()
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
        for a, b in evs:
            a.record(stream)
            run()
            b.record(stream)
    torch.cuda.synchronize()
    ms = statistics.median(a.elapsed_time(b) for a, b in evs)
    return 2 * nbytes / (ms * 1e-3) / 1e9


def device_copy_GBps(src, dst, stream, reps=10):
    """The achievable streaming rate the kernel's HBM fraction is read against
    (VERDICT r4 item 5), on the launch's own input bytes into
    its output buffer: (1) the product library's linear streaming copy
    (nh_probe_copy_linear, 16 B per lane, nontemporal loads and stores, one
    contiguous KiB per wave instruction -- the guide's float4 copy), and (2)
    torch's copy_ (a slower, general copy, for reference only)."""
    from nano_hevc import _lib
    L = _lib.load()
    n = src.numel() - src.numel() % 8
    sp = C.c_void_p(stream.cuda_stream)

    def stream_copy():
        _lib.check(L.nh_probe_copy_linear(src.data_ptr(), dst.data_ptr(), n, 1, 0, sp), "copy")
    nbytes = src.numel() * src.element_size()
    return _copy_GBps(stream_copy, n * src.element_size(), stream, reps), \
        _copy_GBps(lambda: dst.copy_(src), nbytes, stream, reps)


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
    # compute only: each rank's blocks over its own device time, summed over ranks
    (elapsed, kern_ms), (blocks_all, rate_sum) = reduce_max_sum(dist, dev, (elapsed, kern_ms),
                                                                (nblk, nblk / (kern_ms * 1e-3)))
    value = blocks_all * args.steps / elapsed

    gather = None
    if dist and args.gather_steps > 0:
        outs.append(torch.zeros_like(outs[0]))
        gf = args.frames if args.gather_frames is None else args.gather_frames
        frac = min(1.0, gf / args.frames)
        words = min(padded, -(-int(padded * frac) // 4) * 4) // 4   # int64 words sent per rank per step
        chunk = max(1, args.gather_chunk_frames * fe // 4)
        og = OverlappedGather(dist, dev, [words] * world, torch.int64, chunk=chunk)
        gt = run_phase_gather(step_into, lambda s: outs[s].view(torch.int64)[:words], og, args.gather_steps, dist,
                              stream)
        (gt,), _ = reduce_max_sum(dist, dev, (gt,), ())
        into_root = 8 * words * (world - 1)
        what = ("the whole int16 output" if frac >= 1.0 else
                f"a {gf}-frame sample of the int16 levels (the head of the output; --gather-frames)")
        gather = {"value": blocks_all * args.gather_steps / gt, "unit": "blocks/s", "steps": args.gather_steps,
                  "ms_per_step": gt / args.gather_steps * 1e3, "bytes_into_root_per_step": into_root,
                  "into_root_GBps": into_root * args.gather_steps / gt / 1e9, "overlapped": True,
                  "backend": dist.get_backend(), "levels_fraction_gathered": frac,
                  "bytes_per_rank_per_step": 8 * words, "gather_calls_per_step": -(-words // chunk),
                  "chunk_bytes": 8 * chunk,
                  "note": f"compute + RCCL gather to rank 0 of {what} of every rank per step, in "
                          f"{args.gather_chunk_frames}-frame pieces on a side stream, gather(k) under compute(k+1); "
                          "the exchange is bounded by rank 0's inbound xGMI (SURVEY.md §8e E-2)"}

    if rank != 0:
        return None
    achieved = nblk * BYTES_PER_BLOCK / (kern_ms * 1e-3) / 1e9
    tmp = torch.empty_like(res)   # (outs[0] keeps the levels the cpu_baseline leg compares)
    copy_gbs, torch_copy_gbs = device_copy_GBps(res, tmp, stream)   # context, after the timed region
    del tmp
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
                     "bytes_per_block": BYTES_PER_BLOCK, "kernel_ms_avg": kern_ms,
                     "stream_copy_GBps": copy_gbs,
                     "frac_of_achievable_copy": achieved / copy_gbs if copy_gbs else None,
                     "stream_copy": "nh_probe_copy_linear: 16 B/lane nontemporal linear copy of the launch's "
                                    "input bytes into its output buffer (read + write counted)",
                     "torch_copy_GBps": torch_copy_gbs},
        "cpu_baseline": None,
        "compute_only_sum_blocks_per_s": rate_sum,
        "compute_only_note": "sum over ranks of blocks per step / that rank's mean HIP-event time per step "
                             "(device time only: no barrier, no gather); `value` is the wall-clock whole-job rate",
    }
    if gather:
        line["gather_inclusive"] = gather
    if world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(outs[0], res, fe, frames_global, args.qp, args.cpu_seconds)
    return line


# ---------------------------------------------------------------------------
# config 4: mixed 4/8/16/32 TUs per CTU, CTU-row bands, uint8 recon gather
# ---------------------------------------------------------------------------
def synth_rows(f, c, r0, r1, pw, seed, dev):
    """Rows [r0, r1) of plane c (0 Y, 1 U, 2 V) of synthetic frame f: 8-bit
    natural-ish content (gradient + hashed noise in [-15, 15]).  A pure function
    of (seed, f, c, y, x), so a rank synthesises exactly the rows it holds and
    every rank agrees on every sample."""
    yy = torch.arange(r0, r1, device=dev, dtype=torch.int64).view(-1, 1)
    xx = torch.arange(pw, device=dev, dtype=torch.int64).view(1, -1)
    base = (50 + (3 * xx + 2 * yy + 13 * f) % 150 + (xx // 97) * 5) % 256
    m = 0xFFFFFFFF
    h = ((xx * 0x9E3779B1) ^ (yy * 0x85EBCA77) ^ ((3 * f + c + 1) * 0xC2B2AE3D) ^ ((seed * 0x27D4EB2F) & m)) & m
    h = h ^ (h >> 15)
    h = (h * 0x2C1B3C6D) & m
    h = h ^ (h >> 12)
    h = (h * 0x297A2D39) & m
    h = h ^ (h >> 15)
    return torch.clamp(base + h % 31 - 15, 0, 255).to(torch.int16)


def synth_stream(nf, w, h, seed, dev):
    """The whole synthetic stream (frames [Y][U][V] back to back): what every
    rank's bands are cut from (used by --check and the tests, not by the ranks)."""
    parts = []
    for f in range(nf):
        for c, (pw, ph) in enumerate(((w, h), (w // 2, h // 2), (w // 2, h // 2))):
            parts.append(synth_rows(f, c, 0, ph, pw, seed, dev).reshape(-1))
    return torch.cat(parts)


class Cfg4Rank:
    """One rank's share of config 4 (shard.Cfg4Layout): a local buffer holding
    only its bands' rows plus one source row above each band (block.py:38-50 is
    all a TU reads), lvl / recon in the same layout, one luma and one chroma
    plane set per band (rows of the full plane, so the CTU grid, the seeded
    quadtree and the frame-border rule are the unsharded ones), and the packing
    of its reconstructed bands for the gather."""

    def __init__(self, rank, world, frames, width, height, dev, seed):
        from nano_hevc import gpu, shard
        self.gpu, self.dev, self.seed = gpu, dev, seed
        self.lay = shard.cfg4_layout(rank, world, frames, width, height)
        W, H = width, height
        self.work = []
        for b in self.lay.bands:
            r0, r1 = b.ctu_rows()
            tuy = torch.zeros((b.cnt, H // 4, W // 4), dtype=torch.uint8, device=dev)
            tuc = torch.zeros((2 * b.cnt, H // 8, W // 8), dtype=torch.uint8, device=dev)
            self.work.append((self.lay.luma_set(gpu, b), self.lay.chroma_set(gpu, b), r0, r1, tuy, tuc))
        self.total = self.lay.total_elems
        self.packed_elems = self.lay.packed_elems()

    def synth_source(self):
        """The rank's local source buffer, synthesised row range by row range."""
        lay, W = self.lay, self.lay.width
        src = torch.empty(max(1, self.total), dtype=torch.int16, device=self.dev)
        for b in lay.bands:
            for j in range(b.cnt):
                f = b.f0 + j * lay.world
                o = b.off + j * b.slot_elems
                pieces = ((0, b.y0 - b.hy, b.y1, W, 0), (1, b.c0 - b.hc, b.c1, W // 2, b.u_off),
                          (2, b.c0 - b.hc, b.c1, W // 2, b.u_off + b.chroma_elems))
                for c, r0, r1, pw, po in pieces:
                    n = (r1 - r0) * pw
                    src[o + po:o + po + n] = synth_rows(f, c, r0, r1, pw, self.seed, self.dev).reshape(-1)
        return src

    def fill_source(self, stream):
        src = torch.zeros(max(1, self.total), dtype=torch.int16, device=self.dev)
        return self.lay.fill_from_stream(stream, src)

    def new_lvl(self, compact=False):
        """The level buffer: int32, or the int16 compact levels plus their int32 spill plane (self.spill)."""
        if compact:
            self.spill = torch.empty(max(1, self.total), dtype=torch.int32, device=self.dev)
            return torch.zeros(max(1, self.total), dtype=torch.int16, device=self.dev)
        self.spill = None
        return torch.zeros(max(1, self.total), dtype=torch.int32, device=self.dev)

    def widen(self, lvl):
        """int32 levels of the compact ones (outside the timed region: the CPU check)."""
        if lvl.dtype == torch.int32:
            return lvl
        out = torch.zeros(lvl.shape, dtype=torch.int32, device=self.dev)
        for sy, suv, r0, r1, _, _ in self.work:
            self.gpu.tu_levels_widen(lvl, self.spill, sy, 32, r0, r1, out=out)
            self.gpu.tu_levels_widen(lvl, self.spill, suv, 16, r0, r1, out=out)
        return out

    def new_rec(self):
        return torch.zeros(max(1, self.total), dtype=torch.int16, device=self.dev)

    def run(self, src, qp, lvl, rec, stream):
        for sy, suv, r0, r1, tuy, tuc in self.work:
            if lvl.dtype == torch.int16:   # the exact compact levels (int32 spill for strips that are not 8-bit)
                self.gpu.tu_pipeline_planes_compact(src, sy, 32, 0, self.seed, qp, True, r0, r1, lvl=lvl, rec=rec,
                                                    tu=tuy, spill=self.spill, stream=stream)
                self.gpu.tu_pipeline_planes_compact(src, suv, 16, 1, self.seed, qp, False, r0, r1, lvl=lvl, rec=rec,
                                                    tu=tuc, spill=self.spill, stream=stream)
                continue
            self.gpu.tu_pipeline_planes(src, sy, 32, 0, self.seed, qp, True, r0, r1, lvl=lvl, rec=rec, tu=tuy,
                                        stream=stream)
            self.gpu.tu_pipeline_planes(src, suv, 16, 1, self.seed, qp, False, r0, r1, lvl=lvl, rec=rec, tu=tuc,
                                        stream=stream)

    def send_of(self, rec, packed):
        """Pack + narrow the reconstructed band rows (values in [0, 255]) into ``packed``."""
        o = 0
        for v in self.lay.local_views(rec):
            n = v.numel()
            packed[o:o + n].view(v.shape).copy_(v)
            o += n
        return packed

    def tu_counts(self):
        """TUs per size coded per step, from the TU maps (one byte per 4x4 unit =
        log2 of its TU's size; bit 7 marks a group recoded by the wide kernel)."""
        units = [0, 0, 0, 0]
        for *_, tuy, tuc in self.work:
            for m in (tuy, tuc):
                cnt = torch.bincount((m & 0x7F).reshape(-1).to(torch.int64), minlength=6)
                for k in range(4):
                    units[k] += int(cnt[k + 2])
        return [units[k] // (1 << (2 * k)) for k in range(4)]   # a TU of (4*2^k)^2 samples = 4^k units


def unpack_to_stream(packed, rank, world, frames, width, height, stream):
    """Rank ``rank``'s gathered bands (Cfg4Rank.send_of order) into a full stream."""
    from nano_hevc import shard
    o = 0
    for v in shard.cfg4_layout(rank, world, frames, width, height).full_views(stream):
        v.copy_(packed[o:o + v.numel()].view(v.shape))
        o += v.numel()
    return o


def run_cfg4(args, dist, world, rank, dev):
    from nano_hevc import gpu, shard, _lib
    _lib.load()
    W, H = W4K, H4K
    cw, ch = W // 2, H // 2
    fe = gpu.yuv420_frame_elems(W, H)
    nf = args.frames * world
    me = Cfg4Rank(rank, world, nf, W, H, dev, args.seed)
    src = me.synth_source()          # only this rank's bands + one halo row each
    compact = args.levels == "int16"
    lvl = me.new_lvl(compact)
    recs = [me.new_rec()]
    stream = torch.cuda.current_stream(dev)

    def step_into(slot):
        me.run(src, args.qp, lvl, recs[slot], stream)

    elapsed, kern_ms = timed_steps(lambda: step_into(0), args.steps, args.warmup, dist, stream)
    my_samples = me.packed_elems
    (elapsed, kern_ms), sums = reduce_max_sum(dist, dev, (elapsed, kern_ms),
                                              [my_samples, my_samples / (kern_ms * 1e-3)] + me.tu_counts())
    samples_all, rate_sum, tu_all = sums[0], sums[1], sums[2:]
    value = samples_all * args.steps / elapsed

    sizes = [shard.cfg4_packed_elems(r, world, nf, W, H) for r in range(world)]
    gather, check = None, None
    if dist and args.gather_steps > 0:
        recs.append(me.new_rec())
        packed = [torch.zeros(max(sizes), dtype=torch.uint8, device=dev) for _ in range(2)]
        og = OverlappedGather(dist, dev, sizes, torch.uint8)
        gt = run_phase_gather(step_into, lambda s: me.send_of(recs[s], packed[s]), og, args.gather_steps, dist, stream)
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
            full_src = synth_stream(nf, W, H, args.seed, dev)
            full = torch.zeros_like(full_src)
            for r in range(world):
                unpack_to_stream(og.recv[r][:sizes[r]].to(dev), r, world, nf, W, H, full)
            ref_l = torch.zeros(full_src.shape, dtype=torch.int32, device=dev)
            ref_r = torch.zeros_like(full_src)
            sy, suv = gpu.yuv420_plane_sets(nf, W, H)
            gpu.tu_pipeline_planes(full_src, sy, 32, 0, args.seed, args.qp, True, lvl=ref_l, rec=ref_r)
            gpu.tu_pipeline_planes(full_src, suv, 16, 1, args.seed, args.qp, False, lvl=ref_l, rec=ref_r)
            check = bool(torch.equal(full, ref_r))

    if rank != 0:
        return None
    line = {
        "metric": METRIC_CFG4, "value": value, "unit": "samples/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "int32",
        "data": "synthetic 8-bit 4K YUV420 frames (gradient + hashed noise, int16 samples), resident in HBM",
        "config": {"workload": "config 4: 4K YUV420, seeded 4/8/16/32 TU quadtree per 32x32 CTU (16x16 chroma), "
                               "open-loop DC/planar choice, full chain, QP %d" % args.qp,
                   "frames_per_gpu": args.frames, "frames_per_s": value / (W * H + 2 * cw * ch),
                   "samples_per_step_rank0": my_samples, "parallelism": f"ctu-band{world} (rotated)",
                   "source_bytes_rank0": 2 * me.total, "source_bytes_stream": 2 * nf * fe,
                   "source_fraction_rank0": me.total / (nf * fe),
                   "tu_blocks_per_step": {f"{4 << k}x{4 << k}": int(tu_all[k]) for k in range(4)},
                   "tu_blocks_per_s": {f"{4 << k}x{4 << k}": tu_all[k] * args.steps / elapsed for k in range(4)},
                   "levels": ("int16 on the device: the exact compact levels (|level| <= 408 for an 8-bit TU), "
                              "int32 spill + strip markers for the rest, widened to the reference's int32 by "
                              "nh_tu_levels_widen (outside the timed region, for the CPU check)" if compact else
                              "int32 (the reference's dtype)")},
        "roofline": cfg4_roofline(my_samples, kern_ms, args.frames, world, compact),
        "cpu_baseline": None,
        "compute_only_sum_samples_per_s": rate_sum,
        "compute_only_note": "sum over ranks of samples per step / that rank's mean HIP-event time per step "
                             "(device time only: no barrier, no gather); `value` is the wall-clock whole-job rate",
    }
    if gather:
        line["gather_inclusive"] = gather
    if check is not None:
        line["gathered_recon_equals_unsharded"] = check
    if world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline_cfg4(me, src, me.widen(lvl), recs[0], args, fe)
    return line


def valu_sources_match(v) -> bool:
    """Whether a profiles/valu_roofline.json entry was profiled from the kernel
    sources this run executes: tools/pmc_valu.py records the sha256 of the
    config's csrc files (in order); recomputed here."""
    src = (v or {}).get("sources")
    if not src:
        return False
    import hashlib
    h = hashlib.sha256()
    try:
        for f in src["files"]:
            h.update(open(os.path.join(ROOT, "nano-hevc_amd", "csrc", f), "rb").read())
    except OSError:
        return False
    return h.hexdigest() == src.get("sha256")


def load_valu(cfg_key: str):
    """The VALU roofline inputs of a configuration, committed in
    profiles/valu_roofline.json by tools/pmc_valu.py: per kernel of the step the
    SQ_INSTS_VALU wave-instructions per launch (PMC) and the attainable issue
    rate of its static VALU mix priced at the measured per-opcode rates."""
    p = os.path.join(ROOT, "profiles", "valu_roofline.json")
    if not os.path.exists(p):
        return None
    try:
        return json.load(open(p)).get("configs", {}).get(cfg_key)
    except Exception:
        return None


def cfg4_roofline(samples, kern_ms, frames, world, compact=False):
    """Config 4 is VALU-issue-bound: the roofline is the VALU
    issue rate.  achieved = the step's VALU wave-instructions (PMC, per kernel of
    the step, from profiles/valu_roofline.json) / the step's HIP-event time
    measured here; peak = the attainable rate of the step's instruction mix
    (harmonic combination of each kernel's attainable rate, weighted by its
    instructions).  The HBM view (8 B/sample; 6 with compact levels) rides along as ``hbm``."""
    bps = BYTES_PER_SAMPLE_CFG4_COMPACT if compact else BYTES_PER_SAMPLE_CFG4
    gbs = samples * bps / (kern_ms * 1e-3) / 1e9
    hbm = {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
           "traffic": load_traffic(f"cfg4_4k_yuv420_f{frames}_n{world}" + ("_int16" if compact else "")),
           "traffic_note": "PMC bytes per step (all 4 launches): reads as the 64-B request tally (a lower bound for "
                           "8-B/lane row reads, <= 2x that if every request were 128 B), writes exact; "
                           "profiles/pmc_traffic.json",
           "bytes_per_sample": bps}
    v = load_valu("cfg4_4k_yuv420_int16" if compact else "cfg4_4k_yuv420")
    if not v:
        return dict(hbm, kernel_ms_avg=kern_ms)
    if not valu_sources_match(v):   # the committed counts describe another build: the HBM view leads
        return dict(hbm, kernel_ms_avg=kern_ms, valu_profile_stale=True,
                    valu_note="profiles/valu_roofline.json was profiled from other kernel sources (sha256 mismatch); "
                              "re-run the VALU passes (tools/gpu_run.sh valu_kt valu_pmc1..4, tools/pmc_valu.py)")
    nf = samples / (W4K * H4K * 3 // 2)        # frames' worth of samples this rank coded per step
    ks = [k for k in v["kernels"].values() if k.get("valu_per_frame") and k.get("attainable_valu_winst_per_s")]
    instr = sum(k["valu_per_frame"] * nf for k in ks)
    t_att = sum(k["valu_per_frame"] * nf / k["attainable_valu_winst_per_s"] for k in ks)
    peak = instr / t_att / 1e9
    achieved = instr / (kern_ms * 1e-3) / 1e9
    return {"bound": "valu", "achieved": achieved, "peak": peak, "unit": "G VALU wave-instr/s",
            "frac": achieved / peak, "traffic": hbm["traffic"], "valu_instr_per_step": instr,
            "valu_lane_instr_per_sample": instr * 64 / samples,   # wave-instructions x 64 lanes / samples
            "peak_note": "attainable issue rate of the step's executed VALU mix at the measured per-opcode rates: "
                         + v.get("peak_kind", "static mix") + " (tools/ab/valu_rate.hip; profiles/valu_roofline.json)",
            "valu_frac_range": [achieved / peak, achieved / (instr / sum(k["valu_per_frame"] * nf / k["attainable_dynamic_lo"]
                                                                         for k in ks) / 1e9)]
            if all(k.get("attainable_dynamic_lo") for k in ks) else None,
            "valu_profile_matches_build": True, "valu_source": v.get("source"), "kernel_ms_avg": kern_ms, "hbm": hbm}


def cpu_baseline_cfg4(me, src, lvl, rec, args, fe):
    """oracle tu_pipeline_plane on whole frames of the same stream, first on one
    thread, then CTU-row-banded over all of the job's host threads
    (oh_tu_pipeline_plane_mt), each leg ~cpu_seconds/2; the GPU levels and
    recon of every sampled frame are checked bit-exact.  N = 1 only: the rank's
    one band is then the whole frame (slot = frame)."""
    from oracle import oracle as O   # checker + CPU baseline only
    O.lib()
    b = me.lay.bands[0]
    assert len(me.lay.bands) == 1 and b.slot_elems == fe and b.hy == 0
    W, H = W4K, H4K
    cw, ch = W // 2, H // 2
    planes = [(0, H, W, 32, 0, True), (W * H, ch, cw, 16, 1, False), (W * H + cw * ch, ch, cw, 16, 2, False)]
    nthr = cpu_threads()
    legs, exact = {}, True
    for threads in (1, nthr):
        t_cpu, f, samples = 0.0, 0, 0
        while f < args.frames and (t_cpu < args.cpu_seconds / 2 or f == 0):
            s = src[f * fe:(f + 1) * fe].cpu().numpy()
            gl = lvl[f * fe:(f + 1) * fe].cpu().numpy()
            gr = rec[f * fe:(f + 1) * fe].cpu().numpy()
            for off, h, w, ctb, pid, luma in planes:
                p = s[off:off + h * w].reshape(h, w)
                t0 = time.perf_counter()
                if threads == 1:
                    ol, orc, _ = O.tu_pipeline_plane(p, ctb, pid, args.seed, args.qp, luma)
                else:
                    ol, orc, _ = O.tu_pipeline_plane_mt(p, ctb, pid, args.seed, args.qp, luma, threads)
                t_cpu += time.perf_counter() - t0
                samples += h * w
                exact &= bool(np.array_equal(ol, gl[off:off + h * w].reshape(h, w)) and
                              np.array_equal(orc, gr[off:off + h * w].reshape(h, w)))
            f += 1
        legs[threads] = (samples / t_cpu, f, samples, t_cpu)
    v1, f1, s1, t1 = legs[1]
    vn, fn, sn, tn = legs[nthr]
    return {"value": vn, "unit": "samples/s", "cores": nthr, "kind": "port",
            "sample": f"{fn} whole 4K YUV420 frames ({sn} samples) through oracle/nh_oracle.c "
                      f"oh_tu_pipeline_plane_mt on {nthr} threads ({tn:.1f} s); single thread: {f1} frames, "
                      f"{s1} samples, {t1:.1f} s",
            "value_1thread": v1, "cpu_model": cpu_model(), "nproc_machine": os.cpu_count(),
            "gpu_outputs_bit_exact_on_sample": exact}


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

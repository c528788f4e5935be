"""The RCCL exchange path of bench.py executed on a one-GPU box.

Run as its own process by tests/test_rccl_gpu.py (one process group per process):
bench.init_dist(1, force_group=True) takes the ``nccl`` branch
(``dist.init_process_group("nccl", device_id=...)``, RCCL on ROCm), then
bench.OverlappedGather / bench.run_phase_gather drive device-tensor gathers on
the side stream exactly as the N>1 bench does:

* config 2: int64 words of the int16 levels (the --gather-frames sample);
* config 4: the reconstructed bands packed as uint8 (bench.Cfg4Rank.send_of).

Every step writes different outputs into its slot (the QP changes per step and
the first int64 word of a config-2 slot is overwritten with a per-step
sentinel), and after each gather the side stream copies what rank 0 received
into a history buffer.  The history must equal, step by step, what that step's
compute produced: a gather that read its slot after step k+2's compute had
overwritten it (a missing wait_free) shows up as step k+2's sentinel or QP.
Prints one JSON line.
"""
import json
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nano-hevc_amd"))
sys.path.insert(0, ROOT)


def _port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def main():
    for k, v in (("RANK", "0"), ("LOCAL_RANK", "0"), ("WORLD_SIZE", "1"), ("MASTER_ADDR", "127.0.0.1")):
        os.environ[k] = v
    os.environ["MASTER_PORT"] = str(_port())
    os.environ.pop("NH_DIST_BACKEND", None)
    os.environ.pop("NH_FORCE_DEVICE", None)
    import torch
    import bench
    from nano_hevc import gpu, _lib
    _lib.load()
    dist = bench.init_dist(1, force_group=True)
    dev = torch.device("cuda", torch.cuda.current_device())
    out = {"backend": dist.get_backend(), "world": dist.get_world_size()}
    main_s = torch.cuda.current_stream(dev)
    steps = 6
    qps = [22 + 5 * (k % 3) for k in range(steps)]

    # ---- config 2: int64 words of the int16 levels ----
    F, W, H = 2, 3840, 2160
    sets = gpu.yuv420_plane_sets(F, W, H)
    n = F * gpu.yuv420_frame_elems(W, H)
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    res = torch.randint(-255, 256, (n,), dtype=torch.int16, device=dev, generator=g)
    outs = [torch.zeros(n, dtype=torch.int16, device=dev) for _ in range(2)]
    words = n // 4
    og = bench.OverlappedGather(dist, dev, [words], torch.int64)
    hist = [torch.zeros(words, dtype=torch.int64, device=dev) for _ in range(steps + 1)]
    cur = {"k": -1}

    def step_into(slot):
        cur["k"] += 1
        k = cur["k"]
        gpu.fwd8x8_quant(res, sets, qps[k % steps], True, out=outs[slot], stream=main_s)
        outs[slot].view(torch.int64)[0].fill_(1000 + k)   # per-step sentinel word

    og.gather = _wrap(og, og.gather, hist, cur)
    bench.run_phase_gather(step_into, lambda s: outs[s].view(torch.int64)[:words], og, steps, dist, main_s)
    torch.cuda.synchronize()
    ok2 = True
    for k in range(steps + 1):
        exp = gpu.fwd8x8_quant(res, sets, qps[k % steps], True).view(torch.int64)[:words].clone()
        exp[0] = 1000 + k
        ok2 &= bool(torch.equal(hist[k], exp))
    out["cfg2_int64_gathers_equal_sent"] = ok2
    out["cfg2_steps"] = steps + 1

    # ---- config 4: uint8 recon bands ----
    nf = 2
    src = bench.synth_stream(nf, W, H, 1234, dev)
    lay = bench.Cfg4Rank(0, 1, nf, W, H, dev, seed=1234)
    src_local = lay.fill_source(src)
    recs = [lay.new_rec() for _ in range(2)]
    lvl = lay.new_lvl()
    packed = [torch.zeros(lay.packed_elems, dtype=torch.uint8, device=dev) for _ in range(2)]
    og4 = bench.OverlappedGather(dist, dev, [lay.packed_elems], torch.uint8)
    hist4 = [torch.zeros(lay.packed_elems, dtype=torch.uint8, device=dev) for _ in range(steps + 1)]
    cur4 = {"k": -1}

    def step4(slot):
        cur4["k"] += 1
        lay.run(src_local, qps[cur4["k"] % steps], lvl, recs[slot], main_s)

    og4.gather = _wrap(og4, og4.gather, hist4, cur4)
    bench.run_phase_gather(step4, lambda s: lay.send_of(recs[s], packed[s]), og4, steps, dist, main_s)
    torch.cuda.synchronize()
    ok4 = True
    for k in range(steps + 1):
        rr = lay.new_rec()
        lay.run(src_local, qps[k % steps], lay.new_lvl(), rr, main_s)
        exp = torch.zeros(lay.packed_elems, dtype=torch.uint8, device=dev)
        lay.send_of(rr, exp)
        ok4 &= bool(torch.equal(hist4[k], exp))
    out["cfg4_uint8_gathers_equal_sent"] = ok4
    out["cfg4_bytes_per_gather"] = lay.packed_elems
    dist.destroy_process_group()
    print(json.dumps(out), flush=True)
    return 0


def _wrap(og, gather, hist, cur):
    """og.gather plus, on the side stream after the gather, a copy of what rank 0
    received into hist[step] (the slot's done event then covers the copy too)."""
    import torch

    def g(slot, main, send_fn):
        gather(slot, main, send_fn)
        k = cur["k"]
        with torch.cuda.stream(og.side):
            hist[k].copy_(og.recv[0])
            done = torch.cuda.Event()
            done.record(og.side)
            og.done[slot] = done
    return g


if __name__ == "__main__":
    sys.exit(main())

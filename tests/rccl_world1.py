"""The RCCL exchange path of bench.py executed on a one-GPU box.

Run as its own process by tests/test_rccl_gpu.py (one process group per process):
bench.init_dist(1, force_group=True) takes the ``nccl`` branch
(``dist.init_process_group("nccl", device_id=...)``, RCCL on ROCm), then
bench.OverlappedGather / bench.run_phase_gather drive device-tensor gathers on
the side stream exactly as the N>1 bench does:

* config 2: int64 words of the WHOLE int16 output of a 128-frame step (3.2 GB),
  in 8-frame gather calls, as bench.py's default gather-inclusive phase ships it;
* config 4: the reconstructed bands packed as uint8 (bench.Cfg4Rank.send_of).

Every step writes different outputs into its slot (the QP changes per step and
the first int64 word of every config-2 gather piece is overwritten with a
per-step, per-piece sentinel), and after each gather call the side stream
copies what rank 0 received into a history buffer.  The history must equal, step by step, what that step's
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

    # ---- config 2: the WHOLE int16 output of a 128-frame step (bench.py's default gather), in
    #      8-frame RCCL gather calls; every piece of every step carries its own sentinel word ----
    F, W, H = 128, 3840, 2160
    steps2 = 4
    fe = gpu.yuv420_frame_elems(W, H)
    sets = gpu.yuv420_plane_sets(F, W, H)
    n = F * fe
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    res = torch.randint(-255, 256, (n,), dtype=torch.int16, device=dev, generator=g)
    outs = [torch.zeros(n, dtype=torch.int16, device=dev) for _ in range(2)]
    words = n // 4
    chunk = 8 * fe // 4
    og = bench.OverlappedGather(dist, dev, [words], torch.int64, chunk=chunk)
    hist = [torch.zeros(words, dtype=torch.int64, device=dev) for _ in range(steps2 + 1)]
    cur = {"k": -1}
    starts = list(range(0, words, chunk))

    def sentinel(k, c):
        return 1_000_000 * (k + 1) + c

    def step_into(slot):
        cur["k"] += 1
        k = cur["k"]
        gpu.fwd8x8_quant(res, sets, qps[k % steps], True, out=outs[slot], stream=main_s)
        w = outs[slot].view(torch.int64)
        for c, off in enumerate(starts):   # per-step, per-piece sentinel words
            w[off].fill_(sentinel(k, c))

    og.on_chunk = lambda off, m: hist[cur["k"]][off:off + m].copy_(og.recv[0][:m])
    bench.run_phase_gather(step_into, lambda s: outs[s].view(torch.int64)[:words], og, steps2, dist, main_s)
    torch.cuda.synchronize()
    ok2 = True
    for k in range(steps2 + 1):
        exp = gpu.fwd8x8_quant(res, sets, qps[k % steps], True).view(torch.int64)[:words]
        for c, off in enumerate(starts):
            exp[off] = sentinel(k, c)
        ok2 &= bool(torch.equal(hist[k], exp))
        del exp
    out["cfg2_int64_gathers_equal_sent"] = ok2
    out["cfg2_steps"] = steps2 + 1
    out["cfg2_frames"] = F
    out["cfg2_levels_fraction_gathered"] = 1.0
    out["cfg2_bytes_per_step"] = 8 * words
    out["cfg2_gather_calls_per_step"] = len(starts)
    del hist, outs, res
    torch.cuda.empty_cache()

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

#!/usr/bin/env python3
"""Where a config-4 closed-loop CTU step goes: the pair kernel's shader-clock
stamps (A/B build, NH_CLOSED4_STAMPS=1) per (ticket, CTU) -- wait on the row
above (poll), the dataflow rounds, publish + slide -- split by CTU kind (one
32x32 TU vs split).  Luma only, FRAMES frames (2 = the critical-path regime:
one pair per wave, no wave shares a SIMD).  One JSON line.

    NH_CLOSED4_STAMPS=1 python tools/ab/closed4_stamps.py [--frames 2] [--knobs K=V,...]
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
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=2)
    ap.add_argument("--qp", type=int, default=32)
    a = ap.parse_args()
    os.environ["NH_CLOSED4_STAMPS"] = "1"
    from nano_hevc import gpu, _lib
    from bench_configs import synth_plane
    _lib.use_ab()
    L = _lib.load()
    f = L.nh_ab_closed4_stamps
    f.argtypes = [C.c_void_p, C.c_int64]
    f.restype = C.c_int64
    W, H, nf = 3840, 2160, a.frames
    planes = []
    for k in range(nf):
        planes += [synth_plane(H, W, 40 + 3 * k).reshape(-1), synth_plane(H // 2, W // 2, 41 + 3 * k).reshape(-1),
                   synth_plane(H // 2, W // 2, 42 + 3 * k).reshape(-1)]
    stream = torch.cat(planes)
    sy, _ = gpu.yuv420_plane_sets(nf, W, H)
    lv = torch.zeros(stream.shape, dtype=torch.int32, device="cuda")
    rc = torch.zeros(stream.shape, dtype=torch.int16, device="cuda")
    for _ in range(3):
        gpu.tu_pipeline_closed(stream, sy, 32, 0, 1234, a.qp, True, lvl=lv, rec=rc)
    torch.cuda.synchronize()
    buf = np.zeros(1 << 25, np.uint64)
    n = f(buf.ctypes.data, buf.size)
    W16 = 48
    r = buf[:n].reshape(-1, W16).astype(np.int64)
    valid = r[:, 1] != 0
    # consecutive CTUs of one ticket: shader cycles per 100-MHz realtime tick -> clock
    a4, a5 = r[:, 4].reshape(-1, ccols := (W + 31) // 32), r[:, 5].reshape(-1, ccols)
    ok = (a4[:, 1:] != 0) & (a4[:, :-1] != 0)
    ghz = float((a4[:, 1:] - a4[:, :-1])[ok].sum() / (a5[:, 1:] - a5[:, :-1])[ok].sum() * 0.1)
    r = r[valid]
    poll, rounds, tail = r[:, 2] - r[:, 1], r[:, 3] - r[:, 2], r[:, 4] - r[:, 3]
    cnt = np.frombuffer(np.ascontiguousarray(r[:, 8:16]).astype(np.uint64).tobytes(), np.uint8).reshape(-1, 64)
    cnt = cnt.astype(np.int64)
    single = (cnt[:, 0] == 1) & (cnt[:, 1:].sum(1) == 0)
    out = {"frames": nf, "ctus": int(len(r)), "clock_GHz": ghz, "single32_frac": float(single.mean())}
    for name, m in (("all", np.ones(len(r), bool)), ("single32", single), ("split", ~single)):
        out[name] = {k: float(np.median(v[m])) for k, v in (("poll", poll), ("rounds", rounds), ("tail", tail),
                                                          ("step", r[:, 4] - r[:, 1]))}
        out[name]["mean_step"] = float((r[:, 4] - r[:, 1])[m].mean())
        out[name]["mean_rounds"] = float(rounds[m].mean())
    # rounds ~ c0 + per size (chain calls x c_size) + per non-empty (round, size) entry x c_entry
    per_call = {32: 2, 16: 4, 8: 8, 4: 16}   # TUs per chain call (64 / NN), a pair codes 2 x cnt TUs
    X = [np.ones(len(r))]
    names = ["const"]
    for si, nn in enumerate((32, 16, 8, 4)):
        c = cnt[:, si::4]
        X.append(((2 * c + per_call[nn] - 1) // per_call[nn]).sum(1))
        names.append(f"call{nn}")
    X.append((cnt > 0).sum(1))
    names.append("entry")
    X = np.stack(X, 1).astype(np.float64)
    coef, *_ = np.linalg.lstsq(X, rounds.astype(np.float64), rcond=None)
    pred = X @ coef
    r2 = 1 - ((rounds - pred) ** 2).sum() / ((rounds - rounds.mean()) ** 2).sum()
    out["rounds_fit_cycles"] = {k: float(v) for k, v in zip(names, coef)}
    out["rounds_fit_r2"] = float(r2)
    out["mean_per_ctu"] = {k: float(v) for k, v in zip(names, X.mean(0))}
    out["mean_rounds_per_ctu"] = float((cnt > 0).reshape(-1, 16, 4).any(2).sum(1).mean())
    # per TU size: the batch phases' cycles per chain call (packed chains; the 32x32 MFMA chain has none)
    ph = r[:, 16:48].reshape(-1, 4, 8)[:, :, :6].sum(0).astype(np.float64)
    names_ph = ["load+neighbours+mode", "fwd pass 1 + transpose", "fwd pass 2", "quant/dequant + transpose",
                "inv pass 1 + transpose", "inv pass 2 + recon + stores"]
    out["batch_phases_cycles_per_call"] = {}
    for si, nn in enumerate((32, 16, 8, 4)):
        calls = X[:, 1 + si].sum()
        if calls and ph[si].sum():
            out["batch_phases_cycles_per_call"][f"{nn}x{nn}"] = {k: float(v / calls) for k, v in zip(names_ph, ph[si])}
    # where a wave's resident time goes (SQ_WAIT_ANY's structural part): per CTU row (ticket), the wait
    # before its first CTU (the wavefront's ramp: a row starts once the row above is a CTU ahead), then
    # per CTU the poll, the rounds and the publish / slide -- realtime (100 MHz) for the ramp, shader
    # cycles for the rest, all in seconds
    rt = buf[:n].reshape(-1, W16).astype(np.int64)
    tk_of = np.arange(len(rt)) // ccols
    ok = rt[:, 1] != 0
    first = {}
    for i in np.nonzero(ok)[0]:
        k = tk_of[i]
        if k not in first or rt[i, 5] < rt[first[k], 5]:
            first[k] = i
    fi = np.array(list(first.values()))
    t0 = (rt[fi, 5] - (rt[fi, 4] - rt[fi, 1]) / (ghz * 10)).min()          # the first CTU's start (100 MHz ticks)
    ramp = ((rt[fi, 5] - (rt[fi, 4] - rt[fi, 1]) / (ghz * 10)) - t0).sum() * 1e-8
    cyc = 1.0 / (ghz * 1e9)
    tot = ramp + float((r[:, 4] - r[:, 1]).sum()) * cyc
    out["wave_time_split"] = {"ramp": ramp / tot, "poll": float(poll.sum()) * cyc / tot,
                              "rounds": float(rounds.sum()) * cyc / tot, "tail": float(tail.sum()) * cyc / tot}
    out["note"] = "stamps in shader-clock cycles (s_memtime); medians per CTU unless mean_*"
    print(json.dumps(out))


if __name__ == "__main__":
    main()

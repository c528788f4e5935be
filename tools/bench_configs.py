#!/usr/bin/env python3
"""Throughput of the non-headline configs (BASELINE.json configs[2..4]) on one MI355X.

  cfg3  1080p YUV420, 35-mode RDO per 8x8 block (pred+residual+DCT+quant+recon)
  cfg4  4K YUV420, mixed 4/8/16/32 TUs per CTU (plan + per-size chains)
  cfg5  8K YUV420, every 32x32 block through the chain: butterfly vs int8-MFMA,
        plus the frame's Y-PSNR (metrics.psnr semantics) for both variants and,
        with --check, the oracle's PSNR on the same frame.
  enc   encode_frame_intra (__main__.py:142-189, DC vs planar per block, 8x8 luma /
        4x4 chroma) over a stream of 4K YUV420p byte frames -> int16 recon + stats;
        HBM roofline at 3 B/sample (1 B source read + 2 B recon write).
  4b    config 4 batched: --cfg4-frames 4K YUV420 frames in one launch per plane set.
  io    frame I/O casts: YUV420p bytes -> int16 planes and back (3 B/sample each).
  closed4 config 4 in CLOSED loop over a 4K YUV420 stream (TUs in z-order, CTU-row
        wavefront; with --check, frame 0's luma against the oracle).
  3s    config 3 over a --cfg3-frames 1080p YUV420 stream, one launch pair per plane set (intra_rdo_planes)
  closed4s  config 4 closed loop over a 384-frame stream in batches of --closed4s-batch
        frames, --closed4-depth of them in flight (tu_pipeline_closed_yuv420_stream)
  closed4mix  config 4 closed loop on an 8-bit stream vs the same stream with one
        9-bit sample (the stream-wide packed / 32-bit form choice)
  closed  config 3 in CLOSED loop (neighbours from the reconstruction, wavefront
        schedule) over a batch of 1080p YUV420 frames; with --check, frame 0's
        luma against the oracle.

Synthetic 8-bit content (gradient + seeded noise) resident in HBM; HIP events
on the launch stream; one JSON line per config.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nano-hevc_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def synth_plane(h, w, seed):
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    yy = torch.arange(h, device="cuda").view(h, 1)
    xx = torch.arange(w, device="cuda").view(1, w)
    base = (40 + (xx * 3 + yy * 2) % 160 + (xx // 97) * 7) % 256
    noise = torch.randint(-12, 13, (h, w), device="cuda", generator=g)
    return torch.clamp(base + noise, 0, 255).to(torch.int16).contiguous()


def timed(fn, reps):
    st = torch.cuda.current_stream()
    fn()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in evs:
        a.record(st)
        fn()
        b.record(st)
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) for a, b in evs)
    return ts[len(ts) // 2]


def psnr_dev(a, b, peak=255):
    from nano_hevc import _lib
    import ctypes as C
    out = torch.zeros(1, dtype=torch.int64, device="cuda")
    _lib.check(_lib.load().nh_sse_i16(a.data_ptr(), b.data_ptr(), a.numel(), out.data_ptr(),
                                      C.c_void_p(torch.cuda.current_stream().cuda_stream)))
    mse = float(np.float64(int(out.item())) / np.float64(a.numel()))
    return float("inf") if mse == 0 else float(10 * np.log10(peak ** 2 / mse))


def valu_roofline(key, ms_per_frame):
    """`bound: "valu"` roofline of a VALU-bound config, with this run's time.

    achieved = the config's VALU wave-instructions per frame (SQ_INSTS_VALU per
    kernel, profiles/valu_roofline.json by tools/pmc_valu.py) / ms_per_frame
    measured here (wall clock of the timed launches, gaps included); peak = the
    attainable issue rate of the frame's static VALU mix at the measured
    per-opcode rates (harmonic over the kernels, weighted by instructions)."""
    p = os.path.join(ROOT, "profiles", "valu_roofline.json")
    if not os.path.exists(p):
        return None
    v = json.load(open(p)).get("configs", {}).get(key)
    if not v:
        return None
    sys.path.insert(0, ROOT)
    from bench import valu_sources_match
    stale = not valu_sources_match(v)
    ks = [k for k in v["kernels"].values() if k.get("valu_per_frame") and k.get("attainable_valu_winst_per_s")]
    instr = sum(k["valu_per_frame"] for k in ks)
    peak = instr / sum(k["valu_per_frame"] / k["attainable_valu_winst_per_s"] for k in ks) / 1e9
    achieved = instr / (ms_per_frame * 1e-3) / 1e9
    return {"bound": "valu", "achieved": achieved, "peak": peak, "unit": "G VALU wave-instr/s",
            "frac": achieved / peak, "valu_instr_per_frame": instr,
            "profile_kernel_frac": v.get("valu_frac"), "profile_tag": _profile_tag(json.load(open(p)), key),
            "peak_kind": v.get("peak_kind"), "valu_profile_stale": stale}


def _profile_tag(d, key):
    """The profiler pass a config's entry came from (one tag, or one per config)."""
    t = d.get("tag")
    return t.get(key) if isinstance(t, dict) else t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--qp", type=int, default=32)
    ap.add_argument("--qp5", type=int, default=4, help="cfg5 QP (D1 scaling leaves every 32x32 level 0 at QP 32)")
    ap.add_argument("--cfg5-frames", type=int, default=32,
                    help="frames of the batched cfg5 stream (8 until late in round 6: 32 amortise the launch tails)")
    ap.add_argument("--cfg3-frames", type=int, default=16, help="frames of the cfg3 plane-set stream line")
    ap.add_argument("--cfg4-frames", type=int, default=64,
                    help="frames of the batched cfg4 stream (16 until late in round 6)")
    ap.add_argument("--cfg5-levels", default=None,
                    help="5b: level dtypes (default from the configs: 5b int32, 5bc int16, 5bc8 int8 compact levels)")
    ap.add_argument("--cfg4-levels", default=None,
                    help="4b: level dtypes (default from the configs: 4b int32, 4bc int16 compact levels)")
    ap.add_argument("--closed4-frames", type=int, default=64, help="frames of the closed-loop cfg4 stream")
    ap.add_argument("--closed4-seq", action="store_true", help="closed4: luma then chroma (default: concurrent wavefronts)")
    ap.add_argument("--closed4s-batch", default="64,128", help="closed4s: frames per batch (one line each)")
    ap.add_argument("--closed-stream-batches", type=int, default=4,
                    help="closed: also code the frames this many times as a pipelined stream (0: off)")
    ap.add_argument("--closed4s-frames", type=int, default=384, help="closed4s: frames in the stream")
    ap.add_argument("--closed4-depth", type=int, default=3, help="closed4s: batches in flight")
    ap.add_argument("--check", action="store_true", help="oracle PSNR on the cfg5 luma plane (slow, CPU)")
    ap.add_argument("--configs", default="3,4,4b,5,closed,closed4,enc,io")
    ap.add_argument("--enc-frames", type=int, default=64)
    ap.add_argument("--closed-frames", type=int, default=64)
    ap.add_argument("--ab", action="store_true", help="run on the A/B library (libnanohevc_ab.so: NH_* knobs read)")
    ap.add_argument("--lib", default=None, help="A/B: run on another build of libnanohevc.so (e.g. tools/_ab/...)")
    args = ap.parse_args()
    from nano_hevc import gpu, _lib
    if args.lib:
        import ctypes
        probe = ctypes.CDLL(os.path.abspath(args.lib))
        for name in [n for n in _lib.SIGNATURES if not hasattr(probe, n)]:
            del _lib.SIGNATURES[name]
        _lib.LIB_PATH = os.path.abspath(args.lib)
    if args.ab:
        _lib.use_ab()
    _lib.load()
    knobs = {k: v for k, v in os.environ.items() if k.startswith("NH_")}
    torch.cuda.set_device(0)
    cfgs = {int(c) if c.isdigit() else c for c in args.configs.split(",")}
    # the batched configs 4 and 5 by level type: 4b / 5b the reference's int32 levels, 4bc / 5bc the exact
    # int16 compact levels, 5bc8 int8 (each its own kernel instance: one profiler run per config name)
    if args.cfg4_levels is None:
        args.cfg4_levels = ",".join([n for c, n in (("4b", "int32"), ("4bc", "int16")) if c in cfgs])
    if args.cfg5_levels is None:
        args.cfg5_levels = ",".join([n for c, n in (("5b", "int32"), ("5bc", "int16"), ("5bc8", "int8")) if c in cfgs])
    if args.cfg4_levels:
        cfgs.add("4b")
    if args.cfg5_levels:
        cfgs.add("5b")

    if 3 in cfgs:
        W, H = 1920, 1080
        planes = [synth_plane(H, W, 1), synth_plane(H // 2, W // 2, 2), synth_plane(H // 2, W // 2, 3)]
        nblk = sum((p.shape[0] // 8) * (p.shape[1] // 8) for p in planes)
        ms = timed(lambda: [gpu.intra_rdo_plane(p, args.qp) for p in planes], args.reps)
        outs = [gpu.intra_rdo_plane(p, args.qp) for p in planes]
        dig = [int(sum(int(o[0].to(torch.int64).sum().item()) for o in outs)),
               int(sum(int(o[1].to(torch.int64).sum().item()) for o in outs)),
               int(sum(int(o[2].to(torch.int64).sum().item()) for o in outs)),
               int(sum(int(o[3].item()) for o in outs))]
        print(json.dumps({"config": "cfg3 1080p YUV420 35-mode RDO per 8x8 (pred+res+DCT+Q+DQ+IDCT+recon+SSE)",
                          "ms_per_frame": ms, "frames_per_s": 1e3 / ms, "blocks_per_frame": nblk,
                          "blocks_per_s": nblk / ms * 1e3, "mode_evals_per_s": 35 * nblk / ms * 1e3, "knobs": knobs,
                          "roofline": valu_roofline("cfg3_1080p_yuv420", ms),
                          "out_digest": dig}), flush=True)
    if "3s" in cfgs:   # config 3 over a frame stream through the plane-set launch (one launch pair per set)
        W, H = 1920, 1080
        nblk = sum(((h // 8) * (w // 8)) for w, h in ((W, H), (W // 2, H // 2), (W // 2, H // 2)))
        nf3 = args.cfg3_frames
        stream3 = torch.cat([torch.cat([synth_plane(H, W, 1 + 3 * f).reshape(-1), synth_plane(H // 2, W // 2, 2 + 3 * f).reshape(-1),
                                        synth_plane(H // 2, W // 2, 3 + 3 * f).reshape(-1)]) for f in range(nf3)])
        sets3 = gpu.yuv420_plane_sets(nf3, W, H)
        lv3 = torch.zeros(stream3.shape, dtype=torch.int32, device="cuda")
        rc3 = torch.zeros(stream3.shape, dtype=torch.int16, device="cuda")
        ms3 = timed(lambda: gpu.intra_rdo_planes(stream3, sets3, args.qp, lvl=lv3, rec=rc3), args.reps)
        m3, _, _, s3 = gpu.intra_rdo_planes(stream3, sets3, args.qp, lvl=lv3, rec=rc3)
        print(json.dumps({"config": "cfg3 over a 1080p YUV420 frame stream: one launch pair per plane set "
                                    "(intra_rdo_planes)", "frames": nf3, "ms_per_frame": ms3 / nf3,
                          "frames_per_s": nf3 / ms3 * 1e3, "blocks_per_s": nf3 * nblk / ms3 * 1e3,
                          "roofline": valu_roofline("cfg3_1080p_yuv420", ms3 / nf3),
                          "sse_frame0": [int(s3[0].item()), int(s3[nf3].item()), int(s3[nf3 + 1].item())]}), flush=True)
        del stream3, lv3, rc3

    if 4 in cfgs:
        W, H = 3840, 2160
        planes = [(synth_plane(H, W, 4), 32, 0, True), (synth_plane(H // 2, W // 2, 5), 16, 1, False),
                  (synth_plane(H // 2, W // 2, 6), 16, 2, False)]
        bufs = []
        L = _lib.load()
        for p, ctb, pid, luma in planes:
            h, w = p.shape
            bufs.append((torch.zeros((h, w), dtype=torch.int32, device="cuda"),
                         torch.zeros((h, w), dtype=torch.int16, device="cuda"),
                         torch.zeros((h // 4, w // 4), dtype=torch.uint8, device="cuda"),
                         torch.empty(max(1, int(L.nh_tu_workspace_bytes(w, h, ctb))), dtype=torch.uint8, device="cuda")))

        def run4():
            for (p, ctb, pid, luma), (lv, rc, tu, wk) in zip(planes, bufs):
                gpu.tu_pipeline_plane(p, ctb, pid, 1234, args.qp, luma, lvl=lv, rec=rc, tu=tu, work=wk)
        ms = timed(run4, args.reps)
        samples = sum(p.numel() for p, *_ in planes)
        hist = {}
        for (p, *_), (lv, rc, tu, wk) in zip(planes, bufs):
            for lg in (2, 3, 4, 5):
                hist[1 << lg] = hist.get(1 << lg, 0) + int((tu == lg).sum().item()) * 16
        print(json.dumps({"config": "cfg4 4K YUV420 mixed 4/8/16/32 TUs per CTU (DC/planar + full chain)",
                          "ms_per_frame": ms, "frames_per_s": 1e3 / ms, "samples_per_s": samples / ms * 1e3,
                          "samples_by_tu_size": hist, "psnr_y": psnr_dev(planes[0][0], bufs[0][1])}), flush=True)

    if "4b" in cfgs:   # config 4 batched: the whole stream in 2 plane sets x 4 TU sizes = 8 launches
        W, H, nf = 3840, 2160, args.cfg4_frames
        planes = []
        for f in range(nf):
            planes += [synth_plane(H, W, 40 + 3 * f).reshape(-1), synth_plane(H // 2, W // 2, 41 + 3 * f).reshape(-1),
                       synth_plane(H // 2, W // 2, 42 + 3 * f).reshape(-1)]
        stream = torch.cat(planes)
        sy, suv = gpu.yuv420_plane_sets(nf, W, H)
        lv = torch.zeros(stream.shape, dtype=torch.int32, device="cuda")
        rc = torch.zeros(stream.shape, dtype=torch.int16, device="cuda")
        tuy = torch.zeros((nf, H // 4, W // 4), dtype=torch.uint8, device="cuda")
        tuc = torch.zeros((2 * nf, H // 8, W // 8), dtype=torch.uint8, device="cuda")

        spill = None
        for ldt in args.cfg4_levels.split(","):
            # int32: the reference's level dtype; int16: the exact compact levels (|level| <= 408 for an
            # 8-bit TU) plus the int32 spill plane, widened afterwards for the digest
            if ldt == "int32":
                lvx = lv

                def run4b():
                    gpu.tu_pipeline_planes(stream, sy, 32, 0, 1234, args.qp, True, lvl=lv, rec=rc, tu=tuy)
                    gpu.tu_pipeline_planes(stream, suv, 16, 1, 1234, args.qp, False, lvl=lv, rec=rc, tu=tuc)
            else:
                lc = torch.zeros(stream.shape, dtype=torch.int16, device="cuda")
                if spill is None:
                    spill = torch.empty(stream.shape, dtype=torch.int32, device="cuda")

                def run4b():
                    gpu.tu_pipeline_planes_compact(stream, sy, 32, 0, 1234, args.qp, True, lvl=lc, rec=rc, tu=tuy,
                                                   spill=spill)
                    gpu.tu_pipeline_planes_compact(stream, suv, 16, 1, 1234, args.qp, False, lvl=lc, rec=rc, tu=tuc,
                                                   spill=spill)
            ms = timed(run4b, args.reps)
            if ldt != "int32":
                lvx = gpu.tu_levels_widen(lc, spill, sy, 32)
                lvx = gpu.tu_levels_widen(lc, spill, suv, 16, out=lvx)
            samples = stream.numel()
            bps = 8 if ldt == "int32" else 6
            key = "cfg4_4k_yuv420" if ldt == "int32" else "cfg4_4k_yuv420_" + ldt
            print(json.dumps({"config": f"cfg4 batched: {nf} x 4K YUV420 frames, mixed 4/8/16/32 TUs per CTU, 8 launches",
                              "levels": ldt, "frames": nf, "ms_per_launch_set": ms, "ms_per_frame": ms / nf,
                              "frames_per_s": nf / ms * 1e3, "samples_per_s": samples / ms * 1e3,
                              "bytes_per_sample": bps, "achieved_GBps": samples * bps / ms / 1e6,
                              "psnr_y_frame0": psnr_dev(stream[:W * H], rc[:W * H]), "knobs": knobs,
                              "roofline": valu_roofline(key, ms / nf),
                              "out_digest": [int(lvx.to(torch.int64).sum().item()), int(rc.to(torch.int64).sum().item()),
                                             int((lvx.to(torch.int64) * torch.arange(lvx.numel(), device="cuda") % 1000003)
                                                 .sum().item())]}), flush=True)

    if "closed4" in cfgs:   # config 4 in closed loop: 64 4K YUV420 frames, 2 concurrent launches (CTU-row wavefronts)
        W, H, nf = 3840, 2160, args.closed4_frames
        planes = []
        for f in range(nf):
            planes += [synth_plane(H, W, 40 + 3 * f).reshape(-1), synth_plane(H // 2, W // 2, 41 + 3 * f).reshape(-1),
                       synth_plane(H // 2, W // 2, 42 + 3 * f).reshape(-1)]
        stream = torch.cat(planes)
        sy, suv = gpu.yuv420_plane_sets(nf, W, H)
        lv = torch.zeros(stream.shape, dtype=torch.int32, device="cuda")
        rc = torch.zeros(stream.shape, dtype=torch.int16, device="cuda")
        tuy = torch.zeros((nf, H // 4, W // 4), dtype=torch.uint8, device="cuda")
        tuc = torch.zeros((2 * nf, H // 8, W // 8), dtype=torch.uint8, device="cuda")

        def run4c():
            if args.closed4_seq:
                gpu.tu_pipeline_closed(stream, sy, 32, 0, 1234, args.qp, True, lvl=lv, rec=rc, tu=tuy)
                gpu.tu_pipeline_closed(stream, suv, 16, 1, 1234, args.qp, False, lvl=lv, rec=rc, tu=tuc)
            else:   # luma and chroma wavefronts concurrent (two streams)
                gpu.tu_pipeline_closed_yuv420(stream, sy, suv, 1234, args.qp, lvl=lv, rec=rc, tu_luma=tuy, tu_chroma=tuc)
        ms = timed(run4c, max(3, args.reps // 4))
        line = {"config": "cfg4 closed loop: 4K YUV420 frames, mixed TUs in z-order, neighbours from the reconstruction, "
                          "CTU-row wavefront on the device", "frames": nf,
                "luma_chroma": "sequential" if args.closed4_seq else "concurrent", "ms_per_launch_set": ms, "ms_per_frame": ms / nf,
                "frames_per_s": nf / ms * 1e3, "samples_per_s": stream.numel() / ms * 1e3,
                "psnr_y_frame0": psnr_dev(stream[:W * H], rc[:W * H]), "knobs": knobs,
                "roofline": valu_roofline("cfg4_closed_4k_yuv420", ms / nf),
                "out_digest": [int(lv.to(torch.int64).sum().item()), int(rc.to(torch.int64).sum().item())]}
        if args.check:   # frames 0 and 1: the two planes of the first luma pair
            from oracle import oracle as O   # checker only
            fe = gpu.yuv420_frame_elems(W, H)
            for f in range(min(2, nf)):
                y = stream[f * fe:f * fe + W * H].view(H, W).cpu().numpy()
                el, er, _ = O.tu_pipeline_plane_closed(y, 32, 0, 1234, args.qp, True)
                line[f"frame{f}_luma_equals_oracle"] = bool(
                    np.array_equal(er, rc[f * fe:f * fe + W * H].view(H, W).cpu().numpy()) and
                    np.array_equal(el, lv[f * fe:f * fe + W * H].view(H, W).cpu().numpy()))
        print(json.dumps(line), flush=True)

    if "closed4s" in cfgs:   # config 4 closed loop over a frame stream: batches of frames, `depth` of them in flight
        W, H, nf = 3840, 2160, args.closed4s_frames
        depth = args.closed4_depth
        batches = [int(x) for x in args.closed4s_batch.split(",")]
        nd = max(batches)   # distinct frames; the stream repeats them (disjoint outputs per frame)
        planes = []
        for f in range(nd):
            planes += [synth_plane(H, W, 40 + 3 * f).reshape(-1), synth_plane(H // 2, W // 2, 41 + 3 * f).reshape(-1),
                       synth_plane(H // 2, W // 2, 42 + 3 * f).reshape(-1)]
        one = torch.cat(planes)
        del planes
        assert nf % nd == 0
        stream = one.repeat(nf // nd)
        del one
        fe = gpu.yuv420_frame_elems(W, H)
        lv = torch.zeros(stream.shape, dtype=torch.int32, device="cuda")
        rc = torch.zeros(stream.shape, dtype=torch.int16, device="cuda")
        tuy = torch.zeros((nf, H // 4, W // 4), dtype=torch.uint8, device="cuda")
        tuc = torch.zeros((2 * nf, H // 8, W // 8), dtype=torch.uint8, device="cuda")
        for bf in batches:
            run4s = lambda: gpu.tu_pipeline_closed_yuv420_stream(stream, W, H, nf, 1234, args.qp, batch_frames=bf,
                                                                   depth=depth, lvl=lv, rec=rc, tu_luma=tuy, tu_chroma=tuc)
            ms = timed(run4s, max(3, args.reps // 5))
            rep = nf // nd
            print(json.dumps({"config": "cfg4 closed loop over a frame stream: 4K YUV420, batches of frames coded as "
                                        "concurrent luma + chroma CTU-row wavefronts, `depth` batches in flight "
                                        "(tu_pipeline_closed_yuv420_stream)",
                              "frames": nf, "batch_frames": bf, "depth": depth, "ms_per_stream": ms,
                              "ms_per_frame": ms / nf, "frames_per_s": nf / ms * 1e3,
                              "samples_per_s": stream.numel() / ms * 1e3, "knobs": knobs,
                              "roofline": valu_roofline("cfg4_closed_4k_yuv420", ms / nf),
                              "repeats_equal": bool((lv.view(rep, -1) == lv.view(rep, -1)[:1]).all() and
                                                    (rc.view(rep, -1) == rc.view(rep, -1)[:1]).all()),
                              "out_digest": [int(lv[:64 * fe].to(torch.int64).sum().item()),
                                             int(rc[:64 * fe].to(torch.int64).sum().item())]}), flush=True)
        del stream, lv, rc, tuy, tuc

    if "closed4mix" in cfgs:   # the stream-wide wide flag: one 9-bit sample in the last frame
        W, H, nf = 3840, 2160, args.closed4_frames
        planes = []
        for f in range(nf):
            planes += [synth_plane(H, W, 40 + 3 * f).reshape(-1), synth_plane(H // 2, W // 2, 41 + 3 * f).reshape(-1),
                       synth_plane(H // 2, W // 2, 42 + 3 * f).reshape(-1)]
        stream = torch.cat(planes)
        sy, suv = gpu.yuv420_plane_sets(nf, W, H)
        fe = gpu.yuv420_frame_elems(W, H)
        lv = torch.zeros(stream.shape, dtype=torch.int32, device="cuda")
        rc = torch.zeros(stream.shape, dtype=torch.int16, device="cuda")
        tuy = torch.zeros((nf, H // 4, W // 4), dtype=torch.uint8, device="cuda")
        tuc = torch.zeros((2 * nf, H // 8, W // 8), dtype=torch.uint8, device="cuda")
        res = {}
        for name in ("8bit", "one_sample_300"):
            if name != "8bit":
                stream[(nf - 1) * fe + 1234] = 300   # one luma sample of the last frame
            ms = timed(lambda: gpu.tu_pipeline_closed_yuv420(stream, sy, suv, 1234, args.qp, lvl=lv, rec=rc,
                                                              tu_luma=tuy, tu_chroma=tuc), max(3, args.reps // 4))
            res[name] = {"ms_per_frame": ms / nf}
        print(json.dumps({"config": "cfg4 closed loop, the stream-wide form choice: an 8-bit stream vs the same "
                                    "stream with one luma sample at 300 (whole luma set on the 32-bit form)",
                          "frames": nf, **res, "ratio": res["one_sample_300"]["ms_per_frame"] / res["8bit"]["ms_per_frame"]}),
              flush=True)

    if "5b" in cfgs:   # config 5 batched only (the product launch), for per-config profiler runs
        W, H, nf = 7680, 4320, args.cfg5_frames
        fe = gpu.yuv420_frame_elems(W, H)
        stream5 = torch.cat([torch.cat([synth_plane(H, W, 7 + 3 * f).flatten(), synth_plane(H // 2, W // 2, 8 + 3 * f).flatten(),
                                        synth_plane(H // 2, W // 2, 9 + 3 * f).flatten()]) for f in range(nf)])
        sets5 = gpu.yuv420_plane_sets(nf, W, H)
        rc5 = torch.zeros_like(stream5)
        nblk = nf * sum((h // 32) * (w // 32) for w, h in ((W, H), (W // 2, H // 2), (W // 2, H // 2)))
        spill = None
        for ldt in args.cfg5_levels.split(","):
            # int32: the reference's level dtype; int16 / int8: the exact compact levels (|level| <= 51 for an
            # 8-bit 32x32 block) plus the int32 spill plane, widened afterwards for the digest
            dt = getattr(torch, ldt)
            lv = torch.zeros_like(stream5, dtype=dt)
            if ldt == "int32":
                ms = timed(lambda: gpu.tc32_planes(stream5, sets5, args.qp5, 1, lvl=lv, rec=rc5), args.reps)
                lv5 = lv
            else:
                if spill is None:
                    spill = torch.empty_like(stream5, dtype=torch.int32)
                ms = timed(lambda: gpu.tc32_planes_compact(stream5, sets5, args.qp5, dt, lvl=lv, rec=rc5, spill=spill),
                           args.reps)
                lv5 = gpu.tc32_levels_widen(lv, spill, sets5)
            bps = 4 + lv.element_size()
            key = "cfg5_8k_yuv420" if ldt == "int32" else "cfg5_8k_yuv420_" + ldt
            print(json.dumps({"config": "cfg5 batched: 8K YUV420 frame stream, f16 MFMA launch + int8 fix-up per plane set",
                              "levels": ldt, "frames": nf, "ms_per_launch_set": ms, "ms_per_frame": ms / nf,
                              "blocks_per_s": nblk / ms * 1e3,
                              "samples_per_s": nf * fe / ms * 1e3, "bytes_per_sample": bps,
                              "achieved_GBps": nf * fe * bps / ms / 1e6,
                              "psnr_y_frame0": psnr_dev(stream5[:W * H], rc5[:W * H]),
                              "knobs": knobs, "roofline": valu_roofline(key, ms / nf),
                              "out_digest": [int(lv5.to(torch.int64).sum().item()), int(rc5.to(torch.int64).sum().item()),
                                             int((lv5.to(torch.int64) * torch.arange(lv5.numel(), device="cuda") % 1000003)
                                                 .sum().item())]}),
                  flush=True)
            del lv, lv5

    if 5 in cfgs:
        W, H = 7680, 4320
        planes = [synth_plane(H, W, 7), synth_plane(H // 2, W // 2, 8), synth_plane(H // 2, W // 2, 9)]
        nblk = sum((p.shape[0] // 32) * (p.shape[1] // 32) for p in planes)
        outs = [(torch.zeros(p.shape, dtype=torch.int32, device="cuda"),
                 torch.zeros(p.shape, dtype=torch.int16, device="cuda")) for p in planes]
        res = {}
        for v, name in ((0, "butterfly"), (1, "mfma_f16"), (2, "mfma_i8")):
            ms = timed(lambda: [gpu.tc32_plane(p, args.qp5, v, lvl=o[0], rec=o[1]) for p, o in zip(planes, outs)],
                       args.reps)
            res[name] = {"ms_per_frame": ms, "blocks_per_s": nblk / ms * 1e3,
                         "samples_per_s": sum(p.numel() for p in planes) / ms * 1e3,
                         "psnr_y": psnr_dev(planes[0], outs[0][1])}
            lv = outs[0][0].to(torch.int64).flatten()
            wts = torch.arange(1, lv.numel() + 1, device="cuda", dtype=torch.int64) % 1000003
            res[name]["levels_checksum"] = int(torch.sum(lv * wts).item())
            res[name]["nonzero_levels_y"] = int(torch.count_nonzero(lv).item())
        line = {"config": "cfg5 8K YUV420, every 32x32 block through the chain: butterfly vs f16 MFMA (8-bit blocks; "
                          "int8 fix-up for the rest) vs int8 MFMA",
                "blocks_per_frame": nblk, **res,
                "qp": args.qp5,
                "variants_identical": all(res[k]["levels_checksum"] == res["butterfly"]["levels_checksum"]
                                          and res[k]["psnr_y"] == res["butterfly"]["psnr_y"] for k in res)}
        if args.check:
            from oracle import oracle as O   # checker only
            y = planes[0].cpu().numpy()
            t0 = time.perf_counter()
            _, er = O.tc32_plane(y, args.qp5)
            line["oracle_seconds_luma"] = time.perf_counter() - t0
            d = y.astype(np.float64) - er.astype(np.float64)
            mse = float(np.mean(d ** 2))
            line["psnr_y_oracle"] = float(10 * np.log10(255 ** 2 / mse))
            line["psnr_matches_oracle"] = line["psnr_y_oracle"] == res["mfma_f16"]["psnr_y"]
        print(json.dumps(line), flush=True)
        # the same over a stream of frames: one MFMA launch per plane set (nh_tc32_planes)
        nf = args.cfg5_frames
        fe = gpu.yuv420_frame_elems(W, H)
        stream5 = torch.empty(nf * fe, dtype=torch.int16, device="cuda")
        for f in range(nf):
            stream5[f * fe:(f + 1) * fe] = torch.cat([p.flatten() for p in planes])
        sets5 = gpu.yuv420_plane_sets(nf, W, H)
        lv5 = torch.zeros_like(stream5, dtype=torch.int32)
        rc5 = torch.zeros_like(stream5)
        for v, name in ((1, "f16 MFMA launch + int8 fix-up"), (2, "int8-MFMA launch")):
            ms = timed(lambda: gpu.tc32_planes(stream5, sets5, args.qp5, v, lvl=lv5, rec=rc5), args.reps)
            same = bool(torch.equal(rc5[:W * H].view(H, W), outs[0][1])) and bool(torch.equal(lv5[:W * H].view(H, W), outs[0][0]))
            samples = nf * fe
            print(json.dumps({"config": "cfg5 batched: 8K YUV420 frame stream, one %s per plane set" % name,
                              "variant": v, "frames": nf, "ms_per_launch_set": ms, "ms_per_frame": ms / nf,
                              "blocks_per_s": nf * nblk / ms * 1e3, "samples_per_s": samples / ms * 1e3,
                              "bytes_per_sample": 8, "achieved_GBps": samples * 8 / ms / 1e6,
                              "frame0_equals_per_plane": same,
                              # the product form (variant 1) is the one profiled for the VALU roofline (§6a)
                              **({"roofline": valu_roofline("cfg5_8k_yuv420", ms / nf)} if v == 1 else {})}),
                  flush=True)

    if "enc" in cfgs or "io" in cfgs:
        W, H = 3840, 2160
        nf = args.enc_frames
        fe = gpu.yuv420_frame_elems(W, H)
        g = torch.Generator(device="cuda")
        g.manual_seed(17)
        planes = []
        for pw, ph, sd in ((W, H, 1), (W // 2, H // 2, 2), (W // 2, H // 2, 3)):
            planes.append(synth_plane(ph, pw, sd).to(torch.uint8).reshape(-1))
        frame = torch.cat(planes)
        stream_u8 = frame.repeat(nf)
        samples = stream_u8.numel()
        if "enc" in cfgs:
            rec = torch.empty(samples, dtype=torch.int16, device="cuda")
            stats = torch.zeros((2 * nf + nf, gpu.ENC_STATS), dtype=torch.int64, device="cuda")
            sets = gpu.yuv420_plane_sets(nf, W, H)

            def run_enc():
                gpu.encode_intra_planes(stream_u8, sets, [8, 4], recon=rec, stats=stats)
            ms = timed(run_enc, args.reps)
            stats.zero_()
            st = gpu.encode_intra_yuv420(stream_u8[:fe], W, H, 8).cpu().numpy()
            mse = np.float64(st[0, 0, 5]) / np.float64(W * H)
            gbs = samples * 3 / ms / 1e6
            print(json.dumps({"config": "enc: encode_frame_intra (DC vs planar, 8x8 luma / 4x4 chroma) over a 4K "
                                        "YUV420p uint8 stream -> int16 recon + per-plane stats",
                              "frames": nf, "ms_per_launch": ms, "frames_per_s": nf / ms * 1e3,
                              "blocks_per_s": int(st[0, :, 0].sum()) * nf / ms * 1e3,
                              "roofline": {"bound": "hbm", "bytes_per_sample": 3, "achieved_GBps": gbs,
                                           "peak_GBps": 8000.0, "frac": gbs / 8000.0},
                              "frame0": {"blocks": int(st[0, :, 0].sum()), "dc": int(st[0, :, 1].sum()),
                                         "planar": int(st[0, :, 2].sum()),
                                         "psnr_y": float(10 * np.log10(255 ** 2 / mse))}}), flush=True)
        if "io" in cfgs:
            wide = torch.empty(samples, dtype=torch.int16, device="cuda")
            back = torch.empty(samples, dtype=torch.uint8, device="cuda")
            ms_w = timed(lambda: gpu.widen_u8(stream_u8, out=wide), args.reps)
            ms_n = timed(lambda: gpu.narrow_u8(wide, out=back), args.reps)
            ok = bool(torch.equal(back, stream_u8))
            print(json.dumps({"config": "io: YUV420p bytes <-> int16 planes (frame.py astype casts), 4K stream",
                              "frames": nf, "widen_ms": ms_w, "narrow_ms": ms_n,
                              "widen_GBps": samples * 3 / ms_w / 1e6, "narrow_GBps": samples * 3 / ms_n / 1e6,
                              "frac_widen": samples * 3 / ms_w / 1e6 / 8000.0,
                              "frac_narrow": samples * 3 / ms_n / 1e6 / 8000.0, "round_trip_exact": ok}), flush=True)

    if "closed" in cfgs:
        W, H = 1920, 1080
        nf = args.closed_frames
        planes = []
        for f in range(nf):
            planes += [synth_plane(H, W, 11 + 3 * f).reshape(-1), synth_plane(H // 2, W // 2, 12 + 3 * f).reshape(-1),
                       synth_plane(H // 2, W // 2, 13 + 3 * f).reshape(-1)]
        stream = torch.cat(planes)
        sets = gpu.yuv420_plane_sets(nf, W, H)
        lvl = torch.zeros(stream.shape, dtype=torch.int32, device="cuda")
        rec = torch.zeros(stream.shape, dtype=torch.int16, device="cuda")
        ms = timed(lambda: gpu.intra_rdo_closed(stream, sets, args.qp, lvl=lvl, rec=rec), max(2, args.reps // 3))
        modes, _, rec, sse = gpu.intra_rdo_closed(stream, sets, args.qp, lvl=lvl, rec=rec)
        nblk = modes.numel()
        line = {"config": "cfg3 closed loop: 35-mode RDO per 8x8, neighbours from the reconstruction, "
                          "row wavefront on the device, 1080p YUV420 frames",
                "frames": nf, "ms_per_launch": ms, "ms_per_frame": ms / nf, "frames_per_s": nf / ms * 1e3,
                "blocks_per_s": nblk / ms * 1e3, "sse_y_frame0": int(sse[0].item()),
                "note": "one wave per block row; a frame's latency is ~(W/8 + 2*H/8) block steps",
                "roofline": valu_roofline("cfg3_closed_1080p_yuv420", ms / nf)}
        if args.check:
            from oracle import oracle as O   # checker only
            y = stream[:W * H].view(H, W).cpu().numpy()
            t0 = time.perf_counter()
            em, _, er, es = O.intra_rdo_plane(y, args.qp, closed=True)
            line["oracle_seconds_luma"] = time.perf_counter() - t0
            line["luma0_matches_oracle"] = bool(np.array_equal(rec[:W * H].view(H, W).cpu().numpy(), er)
                                                and int(sse[0].item()) == es)
        print(json.dumps(line), flush=True)
        if args.closed_stream_batches:   # the same frames, coded `batches` times as a stream of 64-frame batches
            nb_ = args.closed_stream_batches
            big = stream.repeat(nb_)
            lvl2 = torch.zeros(big.shape, dtype=torch.int32, device="cuda")
            rec2 = torch.zeros(big.shape, dtype=torch.int16, device="cuda")
            run = lambda: gpu.intra_rdo_closed_yuv420_stream(big, W, H, nf * nb_, args.qp, batch_frames=nf,
                                                               depth=args.closed4_depth, lvl=lvl2, rec=rec2)
            ms2 = timed(run, max(2, args.reps // 4))
            _, _, rec2, sse2 = run()
            print(json.dumps({"config": "cfg3 closed loop over a frame stream: batches of 1080p YUV420 frames, "
                                        "`depth` in flight (intra_rdo_closed_yuv420_stream)",
                              "frames": nf * nb_, "batch_frames": nf, "depth": args.closed4_depth,
                              "ms_per_stream": ms2, "ms_per_frame": ms2 / (nf * nb_),
                              "roofline": valu_roofline("cfg3_closed_1080p_yuv420", ms2 / (nf * nb_)),
                              "repeats_equal_single_call": bool((rec2.view(nb_, -1) == rec.view(1, -1)).all()) and
                              int(sse2[0].item()) == int(sse[0].item())}), flush=True)
            del big, lvl2, rec2


if __name__ == "__main__":
    main()

"""Per-call cost of the drop-in API (SURVEY.md §6's table).

    python tools/percall.py                          # the MI355X shim (nano-hevc_amd/nano_hevc), on a GPU box
    python tools/percall.py --impl /root/reference   # the reference numpy package (build container only)
    python tools/percall.py --lib tools/_ab/libnanohevc_r01_staging.so   # the shim over another build (A/B)
    python tools/percall.py --server-idle-us 0       # without the block-call server (a launch per call)

Times every compute function the reference exports (nano_hevc/__init__.py:50-91)
one block per call, as the reference's callers use them, at sizes 4 / 8 / 16 / 32
where a size applies: median microseconds per call over ``--reps`` calls after
warm-up.  Prints one JSON object {"impl": ..., "us_per_call": {name: {size: us}}}.
Inputs are the same seeded arrays for both implementations.

--phases (shim only): also splits each call's median into
  python   -- the shim's numpy conversions + the Python/ctypes call overhead
              (total minus the time spent inside the C function),
  marshal / launch / wait / finish -- the C library's host phases of the call
              (nh_last_call_times: inputs into the argument block, the launch
              API, launch-return -> completion word seen, outputs copied back).
"""
from __future__ import annotations

import json
import os
import platform
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _load(impl):
    if impl == "shim":
        sys.path.insert(0, os.path.join(ROOT, "nano-hevc_amd"))
    else:
        sys.path.insert(0, impl)
    import nano_hevc as nh
    return nh


def _time(fn, reps):
    for _ in range(5):
        fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return round(statistics.median(ts) * 1e6, 2)


def cases(nh, rng):
    """(name, size, thunk) for every timed call."""
    out = []
    for n in (4, 8, 16, 32):
        top = rng.integers(0, 256, n).astype(np.int16)
        left = rng.integers(0, 256, n).astype(np.int16)
        topa = rng.integers(0, 256, 2 * n).astype(np.int16)
        lefta = rng.integers(0, 256, 2 * n).astype(np.int16)
        orig = rng.integers(0, 256, (n, n)).astype(np.int16)
        pred = rng.integers(0, 256, (n, n)).astype(np.int16)
        res = rng.integers(-255, 256, (n, n)).astype(np.int16)
        coeff = nh.forward_transform(res)
        lvl = nh.quantize_block(coeff, 22)
        if n == 4:
            out.append(("intra_dc_predict_4x4", n, lambda t=top, l=left: nh.intra_dc_predict_4x4(t, l)))
            out.append(("satd_4x4", n, lambda a=orig.astype(np.int32), b=pred.astype(np.int32): nh.satd_4x4(a, b)))
        out += [
            ("intra_dc_predict", n, lambda t=top, l=left, n=n: nh.intra_dc_predict(t, l, n)),
            ("intra_planar_predict", n, lambda t=top, l=left, n=n: nh.intra_planar_predict(t, l, int(t[-1]), int(l[-1]), n)),
            ("intra_angular_predict", n, lambda t=topa, l=lefta, n=n: nh.intra_angular_predict(t, l, int(l[0]), 23, n)),
            ("residual_block", n, lambda o=orig, p=pred: nh.residual_block(o, p)),
            ("reconstruct_block", n, lambda p=pred, r=res: nh.reconstruct_block(p, r)),
            ("clip_to_pixel_range", n, lambda p=pred, r=res: nh.clip_to_pixel_range(p.astype(np.int32) + r, 8)),
            ("forward_transform", n, lambda r=res: nh.forward_transform(r, use_dst=False)),
            ("inverse_transform", n, lambda c=coeff: nh.inverse_transform(c, use_dst=False)),
            ("quantize_block", n, lambda c=coeff: nh.quantize_block(c, 22)),
            ("dequantize_block", n, lambda l=lvl: nh.dequantize_block(l, 22)),
            ("quantize", n, lambda c=coeff, n=n: nh.quantize(c, 22, n)),
            ("dequantize", n, lambda l=lvl, n=n: nh.dequantize(l, 22, n)),
            ("mse", n, lambda o=orig, p=pred: nh.mse(o, p)),
            ("psnr", n, lambda o=orig.astype(np.uint8), p=pred.astype(np.uint8): nh.psnr(o, p)),
            ("sad", n, lambda o=orig, p=pred: nh.sad(o, p)),
            ("residual_energy", n, lambda r=res: nh.residual_energy(r)),
        ]
        wrap = {4: "4x4", 8: "8x8", 16: "16x16", 32: "32x32"}[n]
        out.append((f"forward_transform_{wrap}", n, lambda r=res, f=getattr(nh, f"forward_transform_{wrap}"): f(r)))
        out.append((f"inverse_transform_{wrap}", n, lambda c=coeff, f=getattr(nh, f"inverse_transform_{wrap}"): f(c)))
    return out


class _Timed:
    """Proxy over the ctypes library: records the wall time of each C call."""

    def __init__(self, lib):
        self._lib = lib
        self.last = 0.0

    def __getattr__(self, name):
        f = getattr(self._lib, name)
        if not name.startswith("nh_") or name == "nh_last_call_times":
            return f

        def call(*a):
            t0 = time.perf_counter()
            r = f(*a)
            self.last = time.perf_counter() - t0
            return r
        return call


def phases(nh, fn, reps):
    """Median split of one call (see --phases)."""
    import ctypes
    from nano_hevc import _lib
    real = _lib.load()
    prox = _Timed(real)
    load0 = _lib.load
    _lib.load = lambda: prox
    ns = (ctypes.c_int64 * 4)()
    rows = []
    try:
        for _ in range(5):
            fn()
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            tot = time.perf_counter() - t0
            real.nh_last_call_times(ns)
            rows.append((tot, prox.last, ns[0] * 1e-9, ns[1] * 1e-9, ns[2] * 1e-9, ns[3] * 1e-9))
    finally:
        _lib.load = load0
    med = [statistics.median(r[i] for r in rows) * 1e6 for i in range(6)]
    c_internal = med[2] + med[3] + med[4] + med[5]
    return {"total_with_proxy": round(med[0], 2), "in_c_call": round(med[1], 2),
            "python_and_ctypes": round(med[0] - med[1], 2), "ctypes_entry_exit": round(med[1] - c_internal, 2),
            "marshal": round(med[2], 2), "launch": round(med[3], 2), "wait": round(med[4], 2),
            "finish": round(med[5], 2)}


def main():
    impl = "shim"
    if "--impl" in sys.argv:
        impl = sys.argv[sys.argv.index("--impl") + 1]
    reps = int(sys.argv[sys.argv.index("--reps") + 1]) if "--reps" in sys.argv else 200
    nh = _load(impl)
    dev = None
    if impl == "shim":
        import torch
        assert torch.cuda.is_available(), "the shim's per-call cost is measured on an MI355X"
        dev = torch.cuda.get_device_name(0)
        from nano_hevc import _lib
        if "--lib" in sys.argv:   # A/B: an older build of the library (symbols it lacks are skipped)
            import ctypes
            path = os.path.abspath(sys.argv[sys.argv.index("--lib") + 1])
            probe = ctypes.CDLL(path)
            for name in [n for n in _lib.SIGNATURES if not hasattr(probe, n)]:
                del _lib.SIGNATURES[name]
            _lib.LIB_PATH = path
        L = _lib.load()
        if "--server-idle-us" in sys.argv and hasattr(L, "nh_block_server_set_idle_us"):   # 0: launch per call
            _lib.check(L.nh_block_server_set_idle_us(int(sys.argv[sys.argv.index("--server-idle-us") + 1])))
    rng = np.random.default_rng(7)
    res, ph = {}, {}
    want_phases = impl == "shim" and "--phases" in sys.argv
    for name, n, fn in cases(nh, rng):
        r = reps if (impl == "shim" or n <= 16) else max(10, reps // 10)
        res.setdefault(name, {})[n] = _time(fn, r)
        if want_phases:
            ph.setdefault(name, {})[n] = phases(nh, fn, r)
    lib = sys.argv[sys.argv.index("--lib") + 1] if "--lib" in sys.argv else "nano_hevc/libnanohevc.so"
    print(json.dumps({"impl": f"nano-hevc_amd shim (MI355X), {lib}" if impl == "shim" else "reference numpy",
                      "device": dev, "cpu": platform.processor() or platform.machine(), "reps": reps,
                      "us_per_call": res, **({"phases_us": ph} if ph else {})}))


if __name__ == "__main__":
    main()

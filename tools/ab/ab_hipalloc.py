#!/usr/bin/env python3
"""Hot kernel on buffers from hipExtMallocWithFlags (flags: 0 default,
4 = hipDeviceMallocContiguous) instead of torch's allocator: does physically
contiguous backing remove the per-process placement lottery seen with
tools/ab/ab_alloc.py?  One JSON line per process."""
import argparse
import ctypes as C
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "nano-hevc_amd"))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--flags", type=int, default=4)
    args = ap.parse_args()
    from nano_hevc import gpu, _lib
    L = _lib.load()
    torch.cuda.set_device(0)
    hip = C.CDLL("libamdhip64.so")
    W, H, F = 3840, 2160, 128
    sets = gpu.yuv420_plane_sets(F, W, H)
    arr = (gpu.PlaneSet * len(sets))(*sets)
    nblk = gpu.blocks_in(sets)
    n = F * gpu.yuv420_frame_elems(W, H)
    pin, pout = C.c_void_p(), C.c_void_p()
    for p in (pin, pout):
        rc = hip.hipExtMallocWithFlags(C.byref(p), C.c_size_t(n * 2), C.c_uint(args.flags))
        assert rc == 0, rc
    g = torch.Generator(device="cuda")
    g.manual_seed(1234)
    src = torch.randint(-255, 256, (n,), dtype=torch.int16, device="cuda", generator=g)
    assert hip.hipMemcpy(pin, C.c_void_p(src.data_ptr()), C.c_size_t(n * 2), 3) == 0
    ref = torch.empty_like(src)
    gpu.fwd8x8_quant(src, sets, 32, True, out=ref)
    del src
    st = torch.cuda.current_stream()
    sp = C.c_void_p(st.cuda_stream)
    rep = {"flags": args.flags, "in": pin.value, "out": pout.value, "D": pout.value - pin.value}
    for v in (5, 4341, 5, 4341):
        for _ in range(3):
            _lib.check(L.nh_fwd8x8_quant_planes_variant(pin, pout, arr, len(sets), 32, 1, v, sp))
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
        for a, b in evs:
            a.record(st)
            _lib.check(L.nh_fwd8x8_quant_planes_variant(pin, pout, arr, len(sets), 32, 1, v, sp))
            b.record(st)
        torch.cuda.synchronize()
        med = statistics.median([a.elapsed_time(b) for a, b in evs])
        rep.setdefault(f"v{v}", []).append(round(nblk * 256 / med / 1e6))
    chk = torch.empty_like(ref)
    assert hip.hipMemcpy(C.c_void_p(chk.data_ptr()), pout, C.c_size_t(n * 2), 3) == 0
    rep["equal"] = bool(torch.equal(chk, ref))
    hip.hipFree(pin)
    hip.hipFree(pout)
    print(json.dumps(rep), flush=True)


if __name__ == "__main__":
    main()

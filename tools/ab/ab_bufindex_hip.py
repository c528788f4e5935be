#!/usr/bin/env python3
"""tools/ab/ab_bufindex.py with buffers from hipExtMallocWithFlags(flags) instead
of torch's allocator (flags 0 default, 4 hipDeviceMallocContiguous): input =
buffer 0, output = buffer j.  Median GB/s of 20 launches of the default
launch per j."""
import ctypes as C
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "nano-hevc_amd"))
import torch  # noqa: E402


def main():
    K = int(sys.argv[1])
    flags = int(sys.argv[2])
    v = int(sys.argv[3]) if len(sys.argv) > 3 else 4341
    from nano_hevc import gpu, _lib
    L = _lib.load()
    torch.cuda.set_device(0)
    hip = C.CDLL("libamdhip64.so")
    W, H, F = 3840, 2160, 128
    sets = gpu.yuv420_plane_sets(F, W, H)
    arr = (gpu.PlaneSet * len(sets))(*sets)
    nblk = gpu.blocks_in(sets)
    n = F * gpu.yuv420_frame_elems(W, H)
    bufs = []
    for _ in range(K):
        p = C.c_void_p()
        rc = hip.hipExtMallocWithFlags(C.byref(p), C.c_size_t(n * 2), C.c_uint(flags))
        assert rc == 0, rc
        bufs.append(p)
    g = torch.Generator(device="cuda")
    g.manual_seed(1234)
    src = torch.randint(-255, 256, (n,), dtype=torch.int16, device="cuda", generator=g)
    assert hip.hipMemcpy(bufs[0], C.c_void_p(src.data_ptr()), C.c_size_t(n * 2), 3) == 0
    del src
    st = torch.cuda.current_stream()
    sp = C.c_void_p(st.cuda_stream)

    def t(i, o):
        for _ in range(3):
            _lib.check(L.nh_fwd8x8_quant_planes_variant(bufs[i], bufs[o], arr, len(sets), 32, 1, v, sp))
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
        for a, b in evs:
            a.record(st)
            _lib.check(L.nh_fwd8x8_quant_planes_variant(bufs[i], bufs[o], arr, len(sets), 32, 1, v, sp))
            b.record(st)
        torch.cuda.synchronize()
        return round(nblk * 256 / statistics.median([a.elapsed_time(b) for a, b in evs]) / 1e6)

    rep = {"flags": flags, "variant": v, "addr_GB": [round((b.value - bufs[0].value) / 2**30, 2) for b in bufs]}
    rep["in0_out_j"] = [t(0, j) for j in range(1, K)]
    rep["in0_out_j_again"] = [t(0, j) for j in range(1, K)]
    for b in bufs:
        hip.hipFree(b)
    print(json.dumps(rep), flush=True)


if __name__ == "__main__":
    main()

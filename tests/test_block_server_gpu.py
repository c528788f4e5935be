"""The block-call server (nh_blocks.hip k_srv) on the GPU.

Per-block calls are taken by one resident workgroup from mapped host memory
while calls keep coming; it leaves after its idle time and is relaunched by the
next call.  These tests check that (i) a long mixed sequence of served calls and
calls that run as their own kernel (inputs over 8 KB: stop request, then the
staged form) is bit-exact against the oracle, (ii) a call after the server left is served by
a relaunched one, (iii) torch work and other threads are not held up, and (iv)
the launch-per-call form (nh_block_server_set_idle_us(0)) gives the same answers."""
import ctypes as C
import os
import subprocess
import sys
import threading
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from oracle import oracle as O  # noqa: E402  (checker only)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def nh():
    import nano_hevc
    from nano_hevc import _lib
    assert _lib.device_count() > 0, "no HIP device: the gpu tests need an MI355X"
    return nano_hevc


def stats():
    from nano_hevc import _lib
    out = (C.c_int64 * 4)()
    _lib.check(_lib.load().nh_block_server_stats(0, out))
    return list(out)


def one_round(nh, rng, n):
    """One block through the reference's chain, every step checked against the oracle."""
    top = rng.integers(0, 256, 2 * n).astype(np.int16)
    left = rng.integers(0, 256, 2 * n).astype(np.int16)
    orig = rng.integers(0, 256, (n, n)).astype(np.int16)
    mode = int(rng.integers(2, 35))
    dc = nh.intra_dc_predict(top[:n], left[:n], n)
    assert np.array_equal(dc, O.intra_dc(top[:n], left[:n], n))
    pl = nh.intra_planar_predict(top[:n], left[:n], int(top[n]), int(left[n]), n)
    assert np.array_equal(pl, O.intra_planar(top[:n], left[:n], int(top[n]), int(left[n]), n))
    an = nh.intra_angular_predict(top, left, int(left[0]), mode, n)
    assert np.array_equal(an, O.intra_angular(top, left, int(left[0]), mode, n)), mode
    res = nh.residual_block(orig, an)
    assert np.array_equal(res, O.residual(orig, an))
    coeff = nh.forward_transform(res)          # served, tile in the server's LDS scratch
    assert np.array_equal(coeff, O.forward_transform(res))
    qp = int(rng.integers(0, 52))
    lvl = nh.quantize_block(coeff, qp)
    assert np.array_equal(lvl, O.quantize(coeff, qp, n))
    dq = nh.dequantize_block(lvl, qp)
    assert np.array_equal(dq, O.dequantize(lvl, qp))
    rr = nh.inverse_transform(dq)
    rec = nh.reconstruct_block(an, rr.astype(np.int16))
    assert np.array_equal(rec, O.reconstruct(an, rr.astype(np.int16)))
    clipped = nh.clip_to_pixel_range(an.astype(np.int32) + rr, 8)
    assert np.array_equal(clipped, O.clip(an.astype(np.int32) + rr, 8))
    d = orig.astype(np.float64) - clipped.astype(np.float64)
    assert nh.mse(orig, clipped) == float(np.mean(d ** 2))     # metrics.py:7-10


def test_mixed_sequence_served_and_kernel_calls(nh):
    rng = np.random.default_rng(20261017)
    s0 = stats()
    for i in range(120):
        one_round(nh, rng, (4, 8, 16, 32)[i % 4])
    s1 = stats()
    if s1[3] > 0:   # server enabled (default)
        assert s1[0] - s0[0] >= 120 * 10, (s0, s1)       # served calls (transforms on the LDS scratch too)
        assert s1[2] - s0[2] >= 30, (s0, s1)             # 32x32 mse (16 KB of int64 inputs) is staged
        assert s1[1] - s0[1] >= 2, (s0, s1)              # relaunched after each stop


def test_call_after_idle_exit_is_served_by_a_new_server(nh):
    s = stats()
    if s[3] == 0:
        pytest.skip("server disabled (idle time 0)")
    top = np.arange(8, dtype=np.int16)
    left = np.arange(8, 16, dtype=np.int16)
    want = O.intra_dc(top, left, 8)
    for k in range(5):
        a = stats()
        assert np.array_equal(nh.intra_dc_predict(top, left, 8), want)
        time.sleep(max(0.005, 5 * s[3] * 1e-6))       # well past the idle time: the server has left
        assert np.array_equal(nh.intra_dc_predict(top, left, 8), want)
        b = stats()
        assert b[1] - a[1] >= 1, (k, a, b)


def test_torch_work_not_blocked(nh):
    import torch
    x = torch.arange(1 << 20, device="cuda", dtype=torch.float32)
    rng = np.random.default_rng(3)
    o = rng.integers(0, 256, (8, 8)).astype(np.int16)
    p = rng.integers(0, 256, (8, 8)).astype(np.int16)
    t0 = time.perf_counter()
    for _ in range(50):
        r = nh.residual_block(o, p)
        y = (x * 2).sum()
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    assert np.array_equal(r, O.residual(o, p))
    assert float(y.item()) == float((x * 2).sum().item())
    assert dt < 5.0, dt      # 50 rounds; each waits at most one idle time


def test_device_sync_after_calls_waits_at_most_the_idle_time(nh):
    """a device-wide synchronize right after per-block calls waits
    for the resident server's idle exit -- bounded by the idle time (100 us by
    default), and not at all after block_server_stop()."""
    import statistics
    import torch
    from nano_hevc import gpu
    idle_us = gpu.block_server_stats()["idle_us"]
    assert 0 < idle_us <= 100
    rng = np.random.default_rng(4)
    o = rng.integers(0, 256, (8, 8)).astype(np.int16)
    p = rng.integers(0, 256, (8, 8)).astype(np.int16)
    torch.cuda.synchronize()
    base, after, stopped = [], [], []
    for _ in range(40):
        t0 = time.perf_counter()
        torch.cuda.synchronize()                 # nothing resident: the bare cost of the call
        base.append(time.perf_counter() - t0)
        nh.residual_block(o, p)
        t0 = time.perf_counter()
        torch.cuda.synchronize()                 # waits for the server's idle exit
        after.append(time.perf_counter() - t0)
        nh.residual_block(o, p)
        gpu.block_server_stop()
        t0 = time.perf_counter()
        torch.cuda.synchronize()
        stopped.append(time.perf_counter() - t0)
    b, a, s = (statistics.median(v) * 1e6 for v in (base, after, stopped))
    assert a - b < idle_us + 150, (b, a, s)     # the idle time + a PCIe poll round, no more
    assert s - b < 100, (b, a, s)


def test_threads_share_the_server(nh):
    errs = []

    def worker(seed):
        try:
            rng = np.random.default_rng(seed)
            for i in range(60):
                n = (4, 8, 16, 32)[i % 4]
                a = rng.integers(0, 256, (n, n)).astype(np.int16)
                b = rng.integers(0, 256, (n, n)).astype(np.int16)
                assert np.array_equal(nh.residual_block(a, b), O.residual(a, b))
                c = rng.integers(-5000, 5000, (n, n)).astype(np.int32)
                qp = int(rng.integers(0, 52))
                assert np.array_equal(nh.quantize_block(c, qp), O.quantize(c, qp, n))
        except Exception as e:   # pragma: no cover - reported below
            errs.append(repr(e))
    ts = [threading.Thread(target=worker, args=(s,)) for s in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(60)
    assert not errs, errs


def test_launch_per_call_form_agrees():
    code = (
        "import sys, numpy as np, ctypes as C\n"
        f"sys.path[:0] = [{os.path.join(ROOT, 'nano-hevc_amd')!r}, {ROOT!r}]\n"
        "import nano_hevc as nh\n"
        "from nano_hevc import _lib\n"
        "from oracle import oracle as O\n"
        "_lib.check(_lib.load().nh_block_server_set_idle_us(0))\n"
        "rng = np.random.default_rng(9)\n"
        "for n in (4, 8, 16, 32):\n"
        "    a = rng.integers(0, 256, (n, n)).astype(np.int16); b = rng.integers(0, 256, (n, n)).astype(np.int16)\n"
        "    assert np.array_equal(nh.residual_block(a, b), O.residual(a, b))\n"
        "    t = rng.integers(0, 256, n).astype(np.int16); l = rng.integers(0, 256, n).astype(np.int16)\n"
        "    assert np.array_equal(nh.intra_dc_predict(t, l, n), O.intra_dc(t, l, n))\n"
        "out = (C.c_int64 * 4)(); _lib.load().nh_block_server_stats(0, out)\n"
        "assert out[0] == 0 and out[1] == 0 and out[2] >= 8 and out[3] == 0, list(out)\n"
        "print('ok')\n")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=100)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr

"""Parity at BASELINE.json's full sizes (configs 2-5), against the pinned CPU
restatement (oracle/, checker only) on the same seeded frames.

The small-size tests in test_gpu_parity.py cover edge cases; these run every
config once at the size its metric is quoted on: a 4K YUV420 frame for the
fused 8x8 path (cfg 2, bench workload) and the mixed-TU pipeline (cfg 4), a
1080p YUV420 frame for the 35-mode RDO in open and closed loop (cfg 3), an 8K
luma plane for the 32x32 chain (cfg 5, both the int8-MFMA and the butterfly
kernels, plus the size-independent property that their Y-PSNRs -- metrics.psnr
semantics -- equal the oracle's).  CPU side: ~25 s of oracle time here, 8 s on the GPU box.
"""
import math

import numpy as np
import pytest

from oracle import oracle as O   # checker only

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    assert torch.cuda.is_available(), "the gpu tests need an MI355X"
    torch.cuda.set_device(0)
    return torch


def natural(h, w, seed):
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w]
    return np.clip(90 + (xx // 3 + yy // 2) % 120 + rng.integers(-12, 13, (h, w)), 0, 255).astype(np.int16)


def yuv420(w, h, seed):
    return [natural(h, w, seed), natural(h // 2, w // 2, seed + 1), natural(h // 2, w // 2, seed + 2)]


def psnr(orig, recon):
    """metrics.psnr (metrics.py:13-21): float64 MSE over the compared region."""
    mse = np.mean((orig.astype(np.float64) - recon.astype(np.float64)) ** 2)
    return float("inf") if mse == 0 else 10 * math.log10(255.0 ** 2 / mse)


def test_cfg2_4k_frame(torch_dev):
    """The bench kernel on one 4K YUV420 int16 residual frame (U[-255,255])."""
    torch = torch_dev
    from nano_hevc import gpu
    W, H = 3840, 2160
    fe = gpu.yuv420_frame_elems(W, H)
    buf = np.random.default_rng(2).integers(-255, 256, size=fe).astype(np.int16)
    out = gpu.fwd8x8_quant(torch.from_numpy(buf).cuda(), gpu.yuv420_plane_sets(1, W, H), 32).cpu().numpy()
    off = 0
    for w, h in ((W, H), (W // 2, H // 2), (W // 2, H // 2)):
        p = buf[off:off + w * h].reshape(h, w)
        assert np.array_equal(out[off:off + w * h].reshape(h, w), O.fwd8x8_quant_plane(p, 32))
        off += w * h


def test_cfg3_1080p_frame_open_loop(torch_dev):
    torch = torch_dev
    from nano_hevc import gpu
    for k, src in enumerate(yuv420(1920, 1080, 30)):
        m, l, r, sse = gpu.intra_rdo_plane(torch.from_numpy(src).cuda(), 32)
        em, el, er, es = O.intra_rdo_plane(src, 32)
        assert np.array_equal(m.cpu().numpy(), em), k
        assert np.array_equal(l.cpu().numpy(), el), k
        assert np.array_equal(r.cpu().numpy(), er), k
        assert int(sse.item()) == es, k


def test_cfg3_1080p_frame_closed_loop(torch_dev):
    torch = torch_dev
    from nano_hevc import gpu
    W, H = 1920, 1080
    planes = yuv420(W, H, 40)
    buf = np.concatenate([p.reshape(-1) for p in planes])
    modes, lvl, rec, sse = gpu.intra_rdo_closed(torch.from_numpy(buf).cuda(), gpu.yuv420_plane_sets(1, W, H), 27)
    modes, lvl, rec, sse = modes.cpu().numpy(), lvl.cpu().numpy(), rec.cpu().numpy(), sse.cpu().numpy()
    off = moff = 0
    for k, p in enumerate(planes):
        h, w = p.shape
        em, el, er, es = O.intra_rdo_plane(p, 27, closed=True)
        nb = (h // 8) * (w // 8)
        assert np.array_equal(modes[moff:moff + nb].reshape(h // 8, w // 8), em), k
        assert np.array_equal(rec[off:off + h * w].reshape(h, w), er), k
        assert np.array_equal(lvl[off:off + h * w].reshape(h, w), el), k
        assert int(sse[k]) == es, k
        off += h * w
        moff += nb


def test_cfg4_4k_frame(torch_dev):
    """Mixed 4/8/16/32 TUs over a whole 4K YUV420 frame (2160 = 67.5 CTU rows:
    a partial last CTU row), batched launch per plane set."""
    torch = torch_dev
    from nano_hevc import gpu
    W, H = 3840, 2160
    planes = yuv420(W, H, 50)
    buf = np.concatenate([p.reshape(-1) for p in planes])
    d = torch.from_numpy(buf).cuda()
    sy, suv = gpu.yuv420_plane_sets(1, W, H)
    lvl = torch.zeros(d.shape, dtype=torch.int32, device="cuda")
    rec = torch.zeros(d.shape, dtype=torch.int16, device="cuda")
    _, _, tuy = gpu.tu_pipeline_planes(d, sy, 32, 0, 4242, 30, True, lvl=lvl, rec=rec)
    _, _, tuc = gpu.tu_pipeline_planes(d, suv, 16, 1, 4242, 30, False, lvl=lvl, rec=rec)
    lvl, rec, tuy, tuc = lvl.cpu().numpy(), rec.cpu().numpy(), tuy.cpu().numpy(), tuc.cpu().numpy()
    off = 0
    for c, p in enumerate(planes):
        h, w = p.shape
        el, er, et = O.tu_pipeline_plane(p, 32 if c == 0 else 16, c, 4242, 30, c == 0)
        assert np.array_equal(lvl[off:off + h * w].reshape(h, w), el), c
        assert np.array_equal(rec[off:off + h * w].reshape(h, w), er), c
        assert np.array_equal(tuy[0] if c == 0 else tuc[c - 1], et), c
        off += h * w


def test_cfg5_8k_luma_mfma_and_butterfly(torch_dev):
    torch = torch_dev
    from nano_hevc import gpu
    src = natural(4320, 7680, 60)
    d = torch.from_numpy(src).cuda()
    el, er = O.tc32_plane(src, 4)
    full = (slice(0, 4320 // 32 * 32), slice(0, 7680 // 32 * 32))
    p_ref = psnr(src[full], er[full])
    for v in (1, 2, 0):   # f16 MFMA (8-bit blocks), int8 MFMA, butterfly
        l, r = gpu.tc32_plane(d, 4, v)
        r = r.cpu().numpy()
        assert np.array_equal(l.cpu().numpy(), el), v
        assert np.array_equal(r, er), v
        assert psnr(src[full], r[full]) == p_ref

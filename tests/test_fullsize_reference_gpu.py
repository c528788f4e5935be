"""Reference parity at BASELINE.json's full sizes: the GPU outputs hash to the
REFERENCE's own outputs on the same seeded frames.

tests/golden/fullsize.json holds sha256 hashes of what the reference's
functions, composed as DESIGN.md §3.3-3.5 / §3.7 define the drivers, produce
on the frames of tests/golden/fullsize_inputs.py (generated in the build
container by tests/golden/make_fullsize.py; the reference never travels here):
config 2 (the headline 8x8 DCT+quant) on a 4K YUV420 residual frame, config 3
on a 1080p YUV420 frame in open and closed loop, config 4 on a 4K YUV420 frame
in open and closed loop, config 5 on the three planes of an 8K YUV420 frame
(int8-MFMA and butterfly kernels).
"""
import hashlib
import json
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import fullsize_inputs as FI  # noqa: E402

pytestmark = pytest.mark.gpu
FIX = os.path.join(HERE, "golden", "fullsize.json")


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.fixture(scope="module")
def ref():
    with open(FIX) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    assert torch.cuda.is_available(), "the gpu tests need an MI355X"
    torch.cuda.set_device(0)
    return torch


def test_cfg3_1080p_open_loop_equals_reference(ref, torch_dev):
    torch = torch_dev
    from nano_hevc import gpu
    for k, src in enumerate(FI.cfg3_frame()):
        m, l, r, s = gpu.intra_rdo_plane(torch.from_numpy(src).cuda(), FI.CFG3_QP)
        e = ref[f"cfg3_p{k}"]
        assert sha(m.cpu().numpy()) == e["modes"], k
        assert sha(l.cpu().numpy()) == e["lvl"], k
        assert sha(r.cpu().numpy()) == e["rec"], k
        assert int(s.item()) == e["sse"], k


def test_cfg3_1080p_planes_equals_reference(ref, torch_dev):
    """Config 3 through the plane-set launch (intra_rdo_planes): 3 copies of the
    1080p YUV420 frame in one launch pair per set; every copy's planes equal the
    reference's hashes."""
    torch = torch_dev
    from nano_hevc import gpu
    planes = FI.cfg3_frame()
    h, w = planes[0].shape
    one = np.concatenate([p.reshape(-1) for p in planes])
    F, fe = 3, one.size
    d = torch.from_numpy(one).cuda().repeat(F)
    m, l, r, s = gpu.intra_rdo_planes(d, gpu.yuv420_plane_sets(F, w, h), FI.CFG3_QP)
    m, l, r, s = m.cpu().numpy(), l.cpu().numpy(), r.cpu().numpy(), s.cpu().numpy()
    ny, nc = (h // 8) * (w // 8), (h // 16) * (w // 16)
    for f in range(F):
        off = f * fe
        for k, p in enumerate(planes):
            ph, pw = p.shape
            e = ref[f"cfg3_p{k}"]
            mo = f * ny if k == 0 else F * ny + (2 * f + k - 1) * nc
            n = (ph // 8) * (pw // 8)
            assert sha(m[mo:mo + n].reshape(ph // 8, pw // 8)) == e["modes"], (f, k)
            assert sha(l[off:off + ph * pw].reshape(ph, pw)) == e["lvl"], (f, k)
            assert sha(r[off:off + ph * pw].reshape(ph, pw)) == e["rec"], (f, k)
            assert int(s[f if k == 0 else F + 2 * f + k - 1]) == e["sse"], (f, k)
            off += ph * pw


def test_cfg3_1080p_closed_loop_equals_reference(ref, torch_dev):
    torch = torch_dev
    from nano_hevc import gpu
    planes = FI.cfg3_frame()
    h, w = planes[0].shape
    buf = np.concatenate([p.reshape(-1) for p in planes])
    modes, lvl, rec, sse = gpu.intra_rdo_closed(torch.from_numpy(buf).cuda(), gpu.yuv420_plane_sets(1, w, h),
                                                FI.CLOSED_QP)
    modes, lvl, rec, sse = modes.cpu().numpy(), lvl.cpu().numpy(), rec.cpu().numpy(), sse.cpu().numpy()
    off = moff = 0
    for k, p in enumerate(planes):
        ph, pw = p.shape
        nb = (ph // 8) * (pw // 8)
        e = ref[f"closed_p{k}"]
        assert sha(modes[moff:moff + nb].reshape(ph // 8, pw // 8)) == e["modes"], k
        assert sha(lvl[off:off + ph * pw].reshape(ph, pw)) == e["lvl"], k
        assert sha(rec[off:off + ph * pw].reshape(ph, pw)) == e["rec"], k
        assert int(sse[k]) == e["sse"], k
        off += ph * pw
        moff += nb


def test_cfg4_4k_equals_reference(ref, torch_dev):
    torch = torch_dev
    from nano_hevc import gpu
    planes = FI.cfg4_frame()
    h, w = planes[0].shape
    buf = np.concatenate([p.reshape(-1) for p in planes])
    d = torch.from_numpy(buf).cuda()
    sy, suv = gpu.yuv420_plane_sets(1, w, h)
    lvl = torch.zeros(d.shape, dtype=torch.int32, device="cuda")
    rec = torch.zeros(d.shape, dtype=torch.int16, device="cuda")
    _, _, tuy = gpu.tu_pipeline_planes(d, sy, 32, 0, FI.CFG4_SEED, FI.CFG4_QP, True, lvl=lvl, rec=rec)
    _, _, tuc = gpu.tu_pipeline_planes(d, suv, 16, 1, FI.CFG4_SEED, FI.CFG4_QP, False, lvl=lvl, rec=rec)
    lvl, rec, tuy, tuc = lvl.cpu().numpy(), rec.cpu().numpy(), tuy.cpu().numpy(), tuc.cpu().numpy()
    off = 0
    for k, p in enumerate(planes):
        ph, pw = p.shape
        e = ref[f"cfg4_p{k}"]
        assert sha(lvl[off:off + ph * pw].reshape(ph, pw)) == e["lvl"], k
        assert sha(rec[off:off + ph * pw].reshape(ph, pw)) == e["rec"], k
        assert sha(tuy[0] if k == 0 else tuc[k - 1]) == e["tu"], k
        off += ph * pw


def test_cfg4_4k_compact_levels_equal_reference(ref, torch_dev):
    """Config 4 with compact int16 levels (tu_pipeline_planes_compact), widened back
    to int32: every plane of the 4K frame hashes to the reference's levels, recon
    and TU map."""
    torch = torch_dev
    from nano_hevc import gpu
    planes = FI.cfg4_frame()
    h, w = planes[0].shape
    buf = np.concatenate([p.reshape(-1) for p in planes])
    d = torch.from_numpy(buf).cuda()
    sy, suv = gpu.yuv420_plane_sets(1, w, h)
    lc = torch.zeros(d.shape, dtype=torch.int16, device="cuda")
    rec = torch.zeros(d.shape, dtype=torch.int16, device="cuda")
    spill = torch.empty(d.shape, dtype=torch.int32, device="cuda")
    _, _, tuy, _ = gpu.tu_pipeline_planes_compact(d, sy, 32, 0, FI.CFG4_SEED, FI.CFG4_QP, True, lvl=lc, rec=rec,
                                                  spill=spill)
    _, _, tuc, _ = gpu.tu_pipeline_planes_compact(d, suv, 16, 1, FI.CFG4_SEED, FI.CFG4_QP, False, lvl=lc, rec=rec,
                                                  spill=spill)
    lvl = gpu.tu_levels_widen(lc, spill, sy, 32)
    lvl = gpu.tu_levels_widen(lc, spill, suv, 16, out=lvl)
    lvl, rec, tuy, tuc = lvl.cpu().numpy(), rec.cpu().numpy(), tuy.cpu().numpy(), tuc.cpu().numpy()
    off = 0
    for k, p in enumerate(planes):
        ph, pw = p.shape
        e = ref[f"cfg4_p{k}"]
        assert sha(lvl[off:off + ph * pw].reshape(ph, pw)) == e["lvl"], k
        assert sha(rec[off:off + ph * pw].reshape(ph, pw)) == e["rec"], k
        assert sha(tuy[0] if k == 0 else tuc[k - 1]) == e["tu"], k
        off += ph * pw


def test_cfg2_4k_yuv420_equals_reference(ref, torch_dev):
    """The metric's own workload: every 8x8 block of a 4K YUV420 residual frame
    through forward_transform + quantize_block (transform.py:154-196,
    quant.py:126-137), all three planes hashed against the reference."""
    torch = torch_dev
    from nano_hevc import gpu
    planes = FI.cfg2_frame()
    h, w = planes[0].shape
    buf = np.concatenate([p.reshape(-1) for p in planes])
    out = gpu.fwd8x8_quant(torch.from_numpy(buf).cuda(), gpu.yuv420_plane_sets(1, w, h), qp=FI.CFG2_QP)
    out = out.cpu().numpy()
    off = 0
    for k, p in enumerate(planes):
        ph, pw = p.shape
        assert sha(out[off:off + ph * pw].reshape(ph, pw)) == ref[f"cfg2_4k_p{k}"]["lvl"], k
        off += ph * pw


@pytest.mark.parametrize("variant", [1, 2, 0])   # f16 MFMA (8-bit blocks), int8 MFMA, butterfly
def test_cfg5_8k_chroma_equals_reference(ref, torch_dev, variant):
    torch = torch_dev
    from nano_hevc import gpu
    for name, src in zip("uv", FI.cfg5_chroma()):
        l, r = gpu.tc32_plane(torch.from_numpy(src).cuda(), FI.CFG5_QP, variant)
        assert sha(l.cpu().numpy()) == ref[f"cfg5_{name}"]["lvl"], name
        assert sha(r.cpu().numpy()) == ref[f"cfg5_{name}"]["rec"], name


@pytest.mark.parametrize("variant", [1, 2, 0])   # f16 MFMA (8-bit blocks), int8 MFMA, butterfly
def test_cfg5_8k_luma_equals_reference(ref, torch_dev, variant):
    torch = torch_dev
    from nano_hevc import gpu
    src = FI.cfg5_plane()
    l, r = gpu.tc32_plane(torch.from_numpy(src).cuda(), FI.CFG5_QP, variant)
    assert sha(l.cpu().numpy()) == ref["cfg5_y"]["lvl"]
    assert sha(r.cpu().numpy()) == ref["cfg5_y"]["rec"]


@pytest.mark.parametrize("ldt", ["int16", "int8"])
def test_cfg5_8k_yuv420_compact_levels_equal_reference(ref, torch_dev, ldt):
    """Config 5's compact levels (tc32_planes_compact: int16 / int8 levels, int32
    spill for blocks that are not 8-bit) over the 8K YUV420 frame, widened back to
    int32: every plane hashes to the reference's levels and recon."""
    torch = torch_dev
    from nano_hevc import gpu
    planes = [FI.cfg5_plane()] + list(FI.cfg5_chroma())
    h, w = planes[0].shape
    buf = np.concatenate([p.reshape(-1) for p in planes])
    d = torch.from_numpy(buf).cuda()
    sets = gpu.yuv420_plane_sets(1, w, h)
    lc, rec, spill = gpu.tc32_planes_compact(d, sets, FI.CFG5_QP, getattr(torch, ldt))
    lvl = gpu.tc32_levels_widen(lc, spill, sets).cpu().numpy()
    rec = rec.cpu().numpy()
    off = 0
    for name, p in zip("yuv", planes):
        ph, pw = p.shape
        assert sha(lvl[off:off + ph * pw].reshape(ph, pw)) == ref[f"cfg5_{name}"]["lvl"], name
        assert sha(rec[off:off + ph * pw].reshape(ph, pw)) == ref[f"cfg5_{name}"]["rec"], name
        off += ph * pw


@pytest.mark.parametrize("conc", [False, True])
def test_cfg4_4k_closed_loop_equals_reference(ref, torch_dev, conc):
    """Config 4 in closed loop on the 4K YUV420 frame, luma and
    chroma in sequence or as concurrent wavefronts (tu_pipeline_closed_yuv420)."""
    torch = torch_dev
    from nano_hevc import gpu
    planes = FI.cfg4_frame()
    h, w = planes[0].shape
    buf = np.concatenate([p.reshape(-1) for p in planes])
    d = torch.from_numpy(buf).cuda()
    sy, suv = gpu.yuv420_plane_sets(1, w, h)
    lvl = torch.zeros(d.shape, dtype=torch.int32, device="cuda")
    rec = torch.zeros(d.shape, dtype=torch.int16, device="cuda")
    if conc:
        _, _, tuy, tuc = gpu.tu_pipeline_closed_yuv420(d, sy, suv, FI.CFG4_SEED, FI.CFG4_QP, lvl=lvl, rec=rec)
    else:
        _, _, tuy = gpu.tu_pipeline_closed(d, sy, 32, 0, FI.CFG4_SEED, FI.CFG4_QP, True, lvl=lvl, rec=rec)
        _, _, tuc = gpu.tu_pipeline_closed(d, suv, 16, 1, FI.CFG4_SEED, FI.CFG4_QP, False, lvl=lvl, rec=rec)
    lvl, rec, tuy, tuc = lvl.cpu().numpy(), rec.cpu().numpy(), tuy.cpu().numpy(), tuc.cpu().numpy()
    off = 0
    for k, p in enumerate(planes):
        ph, pw = p.shape
        e = ref[f"closed4_p{k}"]
        assert sha(lvl[off:off + ph * pw].reshape(ph, pw)) == e["lvl"], k
        assert sha(rec[off:off + ph * pw].reshape(ph, pw)) == e["rec"], k
        assert sha(tuy[0] if k == 0 else tuc[k - 1]) == e["tu"], k
        off += ph * pw


def test_cfg4_4k_closed_loop_64_frames_equals_reference(ref, torch_dev):
    """64 copies of the 4K YUV420 frame in one closed-loop launch pair: enough
    CTU rows (>= 4096 per launch) that the pair kernel leaves each whole CTU's
    packed-chain recon from its LDS reconstruction as row pieces at the CTU's
    end (Closed4Args::rec_ctu).  Frame 0 equals the reference's hashes and every
    other frame equals frame 0 (the quadtree depends on the plane, not the frame)."""
    torch = torch_dev
    from nano_hevc import gpu
    F = 64
    planes = FI.cfg4_frame()
    h, w = planes[0].shape
    one = np.concatenate([p.reshape(-1) for p in planes])
    fe = one.size
    d = torch.from_numpy(one).cuda().repeat(F)
    sy, suv = gpu.yuv420_plane_sets(F, w, h)
    lvl = torch.zeros(d.shape, dtype=torch.int32, device="cuda")
    rec = torch.zeros(d.shape, dtype=torch.int16, device="cuda")
    _, _, tuy, tuc = gpu.tu_pipeline_closed_yuv420(d, sy, suv, FI.CFG4_SEED, FI.CFG4_QP, lvl=lvl, rec=rec)
    lvl, rec = lvl.view(F, fe), rec.view(F, fe)
    assert bool((lvl == lvl[:1]).all()) and bool((rec == rec[:1]).all())
    assert bool((tuy == tuy[:1]).all()) and bool((tuc.view(F, 2, -1) == tuc.view(F, 2, -1)[:1]).all())
    l0, r0, tuy, tuc = lvl[0].cpu().numpy(), rec[0].cpu().numpy(), tuy[0].cpu().numpy(), tuc[:2].cpu().numpy()
    off = 0
    for k, p in enumerate(planes):
        ph, pw = p.shape
        e = ref[f"closed4_p{k}"]
        assert sha(l0[off:off + ph * pw].reshape(ph, pw)) == e["lvl"], k
        assert sha(r0[off:off + ph * pw].reshape(ph, pw)) == e["rec"], k
        assert sha(tuy if k == 0 else tuc[k - 1]) == e["tu"], k
        off += ph * pw


def test_cfg4_4k_closed_loop_stream_equals_reference(ref, torch_dev):
    """8 copies of the 4K YUV420 frame through tu_pipeline_closed_yuv420_stream in
    batches of 3 frames over 3 stream pairs (batches in flight together, a
    ragged last batch): frame 0 equals the reference's hashes and every other
    frame equals frame 0."""
    torch = torch_dev
    from nano_hevc import gpu
    F = 8
    planes = FI.cfg4_frame()
    h, w = planes[0].shape
    one = np.concatenate([p.reshape(-1) for p in planes])
    fe = one.size
    d = torch.from_numpy(one).cuda().repeat(F)
    lvl, rec, tuy, tuc = gpu.tu_pipeline_closed_yuv420_stream(d, w, h, F, FI.CFG4_SEED, FI.CFG4_QP, batch_frames=3,
                                                              depth=3)
    lvl, rec = lvl.view(F, fe), rec.view(F, fe)
    assert bool((lvl == lvl[:1]).all()) and bool((rec == rec[:1]).all())
    assert bool((tuy == tuy[:1]).all()) and bool((tuc.view(F, 2, -1) == tuc.view(F, 2, -1)[:1]).all())
    l0, r0, tuy, tuc = lvl[0].cpu().numpy(), rec[0].cpu().numpy(), tuy[0].cpu().numpy(), tuc[:2].cpu().numpy()
    off = 0
    for k, p in enumerate(planes):
        ph, pw = p.shape
        e = ref[f"closed4_p{k}"]
        assert sha(l0[off:off + ph * pw].reshape(ph, pw)) == e["lvl"], k
        assert sha(r0[off:off + ph * pw].reshape(ph, pw)) == e["rec"], k
        assert sha(tuy if k == 0 else tuc[k - 1]) == e["tu"], k
        off += ph * pw

"""Frame-level intra driver of the reference CLI, device-backed.

Drop-in for the functions the reference keeps in ``nano_hevc/__main__.py``:

  encode_frame_intra(frame, block_size, output_path=None) -> (recon, stats)
      __main__.py:142-189.  Per block (luma max(4, block_size), chroma
      max(4, block_size // 2); any size): DC vs planar from the source plane's
      neighbours, smaller residual energy wins (DC on ties), recon =
      clip_to_pixel_range(best prediction); partial blocks stay 0.
  create_test_frame(height, width) -> Frame
      __main__.py:26-52 (host data generation: the demo's test pattern).
  prediction_stats(plane, block_size) -> dict
      the numbers demo_predictions prints (__main__.py:55-139): block count,
      DC / planar wins, total DC / planar residual energies, Y-PSNR of the
      best-mode reconstruction.

The per-block work runs in one gfx950 kernel launch per plane set
(nh_encode_intra_planes); there is no CPU fallback.
"""
from __future__ import annotations

import numpy as np

from . import gpu
from .frame import Frame, Plane

__all__ = ["encode_frame_intra", "create_test_frame", "prediction_stats"]


def _device_planes(planes):
    """Pack host planes (all uint8 or all int16) into one device buffer; returns
    (tensor, plane sets with one plane each, offsets)."""
    import torch
    dts = {np.dtype(p.dtype) for p in planes}
    if len(dts) != 1 or next(iter(dts)) not in (np.dtype(np.uint8), np.dtype(np.int16)):
        raise NotImplementedError(f"encode_frame_intra: planes must all be uint8 or all int16, got {sorted(map(str, dts))}")
    host = np.concatenate([np.ascontiguousarray(p).reshape(-1) for p in planes])
    dev = torch.from_numpy(host).to("cuda")
    sets, offs, o = [], [], 0
    for p in planes:
        h, w = p.shape
        sets.append(gpu.plane_set(o, w, h, w))
        offs.append(o)
        o += h * w
    return dev, sets, offs


def encode_frame_intra(frame: Frame, block_size: int, output_path: str | None = None):
    """__main__.py:142-189 on the device.  Returns (recon Frame of int16 planes,
    {"dc": .., "planar": .., "blocks": ..})."""
    planes = [frame.y.data, frame.u.data, frame.v.data]
    dev, sets, offs = _device_planes(planes)
    import torch
    rec = torch.empty(dev.numel(), dtype=torch.int16, device=dev.device)
    bs = [gpu.luma_block_size(block_size), gpu.chroma_block_size(block_size), gpu.chroma_block_size(block_size)]
    st = gpu.encode_intra_planes(dev, sets, bs, recon=rec).sum(0).cpu().numpy()
    rec_h = rec.cpu().numpy()
    recon = Frame.zeros(frame.height, frame.width, dtype=np.int16)
    for dst, p, o in zip((recon.y, recon.u, recon.v), planes, offs):
        h, w = p.shape
        hh, ww = min(h, dst.height), min(w, dst.width)   # the reference writes source-plane blocks into Frame.zeros planes
        dst.data[:hh, :ww] = rec_h[o:o + h * w].reshape(h, w)[:hh, :ww]
    stats = {"dc": int(st[1]), "planar": int(st[2]), "blocks": int(st[0])}
    if output_path:
        with open(output_path, "wb") as f:
            f.write(recon.to_yuv420p())
        print(f"Wrote: {output_path}")
    return recon, stats


def prediction_stats(plane: Plane, block_size: int) -> dict:
    """The totals demo_predictions reports (__main__.py:55-139) for one plane."""
    dev, sets, _ = _device_planes([plane.data])
    st = gpu.encode_intra_planes(dev, sets, [block_size]).cpu().numpy()[0]
    mse = np.float64(st[5]) / np.float64(plane.data.size)   # metrics.mse of integer-valued samples
    return {"blocks": int(st[0]), "dc_wins": int(st[1]), "planar_wins": int(st[2]),
            "dc_energy": int(st[3]), "planar_energy": int(st[4]),
            "psnr": float("inf") if mse == 0 else float(10 * np.log10(255 ** 2 / mse))}


def create_test_frame(height: int, width: int) -> Frame:
    """The demo's synthetic frame (__main__.py:26-52): four quadrants --
    horizontal ramp, vertical ramp, flat 128, diagonal ramp -- with flat chroma."""
    y = np.zeros((height, width), dtype=np.uint8)
    h2, w2 = height // 2, width // 2
    y[:h2, :w2] = np.linspace(50, 200, w2, dtype=np.uint8)[None, :]
    y[:h2, w2:] = np.linspace(50, 200, h2, dtype=np.uint8)[:, None]
    y[h2:, :w2] = 128
    ii, jj = np.mgrid[0:height - h2, 0:width - w2]
    y[h2:, w2:] = np.minimum(255, 50 + ii + jj)
    u = np.full((h2, w2), 128, dtype=np.uint8)
    v = np.full((h2, w2), 128, dtype=np.uint8)
    return Frame(Plane(y.astype(np.int16)), Plane(u.astype(np.int16)), Plane(v.astype(np.int16)))

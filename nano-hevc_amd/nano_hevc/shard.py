"""CTU-row band sharding of a YUV420 frame stream across ranks.

Every 8x8 block (and every CTU) is independent in the reference's open-loop
model (block.py:38-55 reads neighbours from the SOURCE plane; __main__.py:160-163),
so a frame can be cut into CTU-row bands with no halo exchange for the
transform path.  Bands are balanced to whole CTU rows; band b of frame f goes
to rank (b - f) mod N ("rotation"), so over any N consecutive frames every rank
processes every band once and all ranks carry exactly the same number of
blocks.  A rank stores its bands grouped by band height, which makes each
group one uniform nh_plane_set (Y) plus one (U+V).

The only exchange step is the optional gather of per-rank results to rank 0
(RCCL ``gather`` over xGMI through torch.distributed), used for the
gather-inclusive number and for reassembling frames.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Tuple

CTU_LUMA = 32
CTU_CHROMA = 16


def ctu_bands(height: int, nbands: int, ctu: int = CTU_LUMA) -> List[Tuple[int, int]]:
    """Split [0, height) into nbands runs of whole CTU rows, sizes differing by at
    most one CTU row (the last CTU row may be partial)."""
    rows = (height + ctu - 1) // ctu
    base, extra = divmod(rows, nbands)
    out, r = [], 0
    for b in range(nbands):
        n = base + (1 if b < extra else 0)
        y0, y1 = min(r * ctu, height), min((r + n) * ctu, height)
        out.append((y0, y1))
        r += n
    return out


def band_of(rank: int, frame: int, world: int) -> int:
    """Band index rank ``rank`` processes in global frame ``frame`` (rotation)."""
    return (rank + frame) % world


@dataclass
class LocalGroup:
    """Frames whose band for this rank has the same luma height."""
    y_rows: int
    frames: List[Tuple[int, int]]          # (global frame, band index)
    base: int                              # element offset of the group in the local buffer
    frame_elems: int                       # local elements per frame slot (Y band + U band + V band)


@dataclass
class RankLayout:
    width: int
    height: int
    world: int
    rank: int
    groups: List[LocalGroup]
    total_elems: int

    def plane_sets(self, gpu):
        """nh_plane_set list (<= 2 per distinct band height) for this rank's buffer."""
        sets = []
        cw = self.width // 2
        for g in self.groups:
            c_rows = g.y_rows // 2
            n = len(g.frames)
            sets.append(gpu.plane_set(g.base, self.width, g.y_rows, self.width, 1, n, 0, g.frame_elems))
            if c_rows:
                sets.append(gpu.plane_set(g.base + self.width * g.y_rows, cw, c_rows, cw, 2, n, cw * c_rows,
                                          g.frame_elems))
        return sets

    def blocks(self) -> int:
        cw = self.width // 2
        return sum(len(g.frames) * ((self.width // 8) * (g.y_rows // 8) + 2 * (cw // 8) * ((g.y_rows // 2) // 8))
                   for g in self.groups)


def rank_layout(rank: int, world: int, frames_global: int, width: int = 3840, height: int = 2160) -> RankLayout:
    """Local buffer layout of ``rank`` for a global batch of ``frames_global`` frames."""
    bands = ctu_bands(height, world)
    by_h: Dict[int, List[Tuple[int, int]]] = {}
    for f in range(frames_global):
        b = band_of(rank, f, world)
        y0, y1 = bands[b]
        if y1 > y0:
            by_h.setdefault(y1 - y0, []).append((f, b))
    groups, base = [], 0
    cw = width // 2
    for h in sorted(by_h, reverse=True):
        fe = width * h + 2 * cw * (h // 2)
        groups.append(LocalGroup(h, by_h[h], base, fe))
        base += fe * len(by_h[h])
    return RankLayout(width, height, world, rank, groups, base)


def fill_from_frames(layout: RankLayout, frames_yuv, out):
    """Copy this rank's bands out of full frames (indexable by global frame id,
    each a flat [Y][U][V] array/tensor of one frame) into ``out`` (local buffer)."""
    w, h = layout.width, layout.height
    cw, ch = w // 2, h // 2
    bands = ctu_bands(h, layout.world)
    for g in layout.groups:
        for slot, (f, b) in enumerate(g.frames):
            y0, y1 = bands[b]
            src = frames_yuv[f]
            dst = g.base + slot * g.frame_elems
            out[dst:dst + w * (y1 - y0)] = src[w * y0:w * y1]
            d = dst + w * (y1 - y0)
            c0, c1 = y0 // 2, y1 // 2
            for c in range(2):
                o = w * h + c * cw * ch
                out[d:d + cw * (c1 - c0)] = src[o + cw * c0:o + cw * c1]
                d += cw * (c1 - c0)


def scatter_to_frames(layout: RankLayout, local, frames_yuv):
    """Inverse of fill_from_frames: write this rank's bands back into full frames."""
    w, h = layout.width, layout.height
    cw, ch = w // 2, h // 2
    bands = ctu_bands(h, layout.world)
    for g in layout.groups:
        for slot, (f, b) in enumerate(g.frames):
            y0, y1 = bands[b]
            dst = frames_yuv[f]
            s = g.base + slot * g.frame_elems
            dst[w * y0:w * y1] = local[s:s + w * (y1 - y0)]
            s += w * (y1 - y0)
            c0, c1 = y0 // 2, y1 // 2
            for c in range(2):
                o = w * h + c * cw * ch
                dst[o + cw * c0:o + cw * c1] = local[s:s + cw * (c1 - c0)]
                s += cw * (c1 - c0)


def gather_to_root(local, layouts_total_elems: List[int], dist, group=None):
    """RCCL/gloo gather of every rank's local buffer to rank 0 (the path's one
    exchange step).  Buffers travel as raw 8-byte words (neither NCCL/RCCL nor
    gloo has an int16 type, and 8-byte words keep element counts < 2^31 for
    multi-GB buffers), padded to the largest rank's size."""
    import torch
    es = local.element_size()
    if local.is_cuda and dist.get_backend(group) == "gloo":   # gloo gathers host tensors only
        out = gather_to_root(local.cpu(), layouts_total_elems, dist, group)
        return None if out is None else [o.to(local.device) for o in out]
    nbytes = -(-max(layouts_total_elems) * es // 8) * 8
    raw = local.contiguous().view(torch.uint8)
    if raw.numel() != nbytes:
        raw = torch.nn.functional.pad(raw, (0, nbytes - raw.numel()))
    send = raw.view(torch.int64)
    rank = dist.get_rank(group)
    if rank == 0:
        bufs = [torch.empty(nbytes // 8, dtype=torch.int64, device=local.device) for _ in layouts_total_elems]
        dist.gather(send, gather_list=bufs, dst=0, group=group)
        return [b.view(torch.uint8)[:m * es].view(local.dtype) for b, m in zip(bufs, layouts_total_elems)]
    dist.gather(send, dst=0, group=group)
    return None


# ---------------------------------------------------------------------------
# Config 4 (mixed TUs): CTU-row bands of full frames.  The
# TU chain reads the source row above its band (block.py:38-50), so every rank
# holds the whole input stream and computes only its bands (rotation as
# above); reconstructed bands are packed, gathered to rank 0 and unpacked.
# ---------------------------------------------------------------------------

def cfg4_plan(rank: int, world: int, frames: int) -> List[Tuple[int, int, int]]:
    """(band, first frame, count) per band this rank processes: the frames
    f = first, first + world, ... (band_of(rank, f, world) == band)."""
    plan = []
    for b in range(world):
        f0 = (b - rank) % world
        cnt = len(range(f0, frames, world))
        if cnt:
            plan.append((b, f0, cnt))
    return plan


def _band_views(stream, f: int, y0: int, y1: int, width: int, height: int):
    """Flat slices [Y rows y0..y1, U rows y0/2..y1/2, V rows ...] of frame f."""
    cw, ch = width // 2, height // 2
    fe = width * height + 2 * cw * ch
    base = f * fe
    c0, c1 = y0 // 2, y1 // 2
    u = base + width * height
    v = u + cw * ch
    return [stream[base + width * y0:base + width * y1], stream[u + cw * c0:u + cw * c1],
            stream[v + cw * c0:v + cw * c1]]


def cfg4_pack(stream, rank: int, world: int, frames: int, width: int, height: int):
    """This rank's reconstructed bands of a full-frame stream, packed band-major
    (frames in plan order, Y then U then V rows of each) into one flat tensor."""
    import torch
    bands = ctu_bands(height, world)
    parts = []
    for b, f0, cnt in cfg4_plan(rank, world, frames):
        y0, y1 = bands[b]
        for f in range(f0, frames, world):
            parts += _band_views(stream, f, y0, y1, width, height)
    return torch.cat(parts) if parts else stream[:0].clone()


def cfg4_unpack(packed, rank: int, world: int, frames: int, width: int, height: int, stream):
    """Inverse of cfg4_pack: write rank ``rank``'s bands into the full stream."""
    bands = ctu_bands(height, world)
    o = 0
    for b, f0, cnt in cfg4_plan(rank, world, frames):
        y0, y1 = bands[b]
        for f in range(f0, frames, world):
            for view in _band_views(stream, f, y0, y1, width, height):
                view.copy_(packed[o:o + view.numel()])
                o += view.numel()
    return o


def cfg4_packed_elems(rank: int, world: int, frames: int, width: int, height: int) -> int:
    bands = ctu_bands(height, world)
    cw = width // 2
    n = 0
    for b, f0, cnt in cfg4_plan(rank, world, frames):
        y0, y1 = bands[b]
        n += cnt * (width * (y1 - y0) + 2 * cw * (y1 // 2 - y0 // 2))
    return n

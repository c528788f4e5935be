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
# Config 4 (mixed TUs): CTU-row bands of full frames.  A TU
# reads the source row above it and the column to its left (block.py:38-50),
# so a band needs its own rows plus ONE source row above it (the halo) and
# nothing else.  Each rank holds only those rows (Cfg4Layout), computes its
# bands (rotation as above), and its reconstructed bands are packed, gathered
# to rank 0 and unpacked.
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


@dataclass
class Cfg4Band:
    """One band of one rank in its local buffer: ``cnt`` frame slots (frames f0,
    f0 + world, ...) of ``slot_elems`` elements each, a slot holding the band's
    Y rows [y0 - hy, y1), then U and V rows [c0 - hc, c1) (hy / hc = 1: the
    halo row above the band, 0 for the top band)."""
    band: int
    f0: int
    cnt: int
    y0: int
    y1: int
    hy: int
    hc: int
    off: int            # local element offset of the band's first slot
    slot_elems: int
    u_off: int          # offset of the U rows inside a slot (V follows at u_off + chroma_elems)
    chroma_elems: int   # elements of one chroma plane's rows in a slot (halo included)

    @property
    def c0(self):
        return self.y0 // 2

    @property
    def c1(self):
        return self.y1 // 2

    def ctu_rows(self, ctu: int = CTU_LUMA) -> Tuple[int, int]:
        """CTU rows [r0, r1) of the band (luma CTB 32 and chroma CTB 16 number
        the same rows in 4:2:0)."""
        return self.y0 // ctu, (self.y1 + ctu - 1) // ctu


@dataclass
class Cfg4Layout:
    """A rank's local config-4 buffer: its bands, nothing else of the stream."""
    width: int
    height: int
    world: int
    rank: int
    frames: int
    bands: List[Cfg4Band]
    total_elems: int

    def luma_set(self, gpu, b: Cfg4Band):
        """nh_plane_set of the band's Y planes as rows of the FULL plane: the base
        is the element where full-plane row 0 would sit (negative offsets are
        fine: the kernels touch rows [y0 - 1, y1) only; gpu.tu_pipeline_planes
        checks exactly those rows against the buffer)."""
        w = self.width
        return gpu.plane_set(b.off - (b.y0 - b.hy) * w, w, self.height, w, 1, b.cnt, 0, b.slot_elems)

    def chroma_set(self, gpu, b: Cfg4Band):
        cw = self.width // 2
        return gpu.plane_set(b.off + b.u_off - (b.c0 - b.hc) * cw, cw, self.height // 2, cw, 2, b.cnt,
                             b.chroma_elems, b.slot_elems)

    def local_views(self, local):
        """The band rows (halo excluded) of a local-layout tensor, as (cnt, n)
        strided views: per band, Y then U then V (the order of full_views)."""
        out = []
        w, cw = self.width, self.width // 2
        for b in self.bands:
            for off, n in ((b.off + b.hy * w, w * (b.y1 - b.y0)),
                           (b.off + b.u_off + b.hc * cw, cw * (b.c1 - b.c0)),
                           (b.off + b.u_off + b.chroma_elems + b.hc * cw, cw * (b.c1 - b.c0))):
                if n:
                    out.append(local.as_strided((b.cnt, n), (b.slot_elems, 1), local.storage_offset() + off))
        return out

    def full_views(self, stream):
        """The same band rows of a FULL-frame stream (frames [Y][U][V] back to
        back), as (cnt, n) strided views in local_views' order."""
        w, h = self.width, self.height
        cw, ch = w // 2, h // 2
        fe = w * h + 2 * cw * ch
        out = []
        for b in self.bands:
            for off, n in ((w * b.y0, w * (b.y1 - b.y0)), (w * h + cw * b.c0, cw * (b.c1 - b.c0)),
                           (w * h + cw * ch + cw * b.c0, cw * (b.c1 - b.c0))):
                if n:
                    out.append(stream.as_strided((b.cnt, n), (self.world * fe, 1),
                                                 stream.storage_offset() + b.f0 * fe + off))
        return out

    def held_views(self, stream, local):
        """Every row this rank holds (bands + halos) as pairs (view of a FULL
        stream, view of the local buffer), (cnt, n) each."""
        w, h = self.width, self.height
        cw, ch = w // 2, h // 2
        fe = w * h + 2 * cw * ch
        out = []
        for b in self.bands:
            for foff, loff, n in ((w * (b.y0 - b.hy), 0, w * (b.y1 - b.y0 + b.hy)),
                                  (w * h + cw * (b.c0 - b.hc), b.u_off, b.chroma_elems),
                                  (w * h + cw * ch + cw * (b.c0 - b.hc), b.u_off + b.chroma_elems, b.chroma_elems)):
                if n:
                    out.append((stream.as_strided((b.cnt, n), (self.world * fe, 1),
                                                  stream.storage_offset() + b.f0 * fe + foff),
                                local.as_strided((b.cnt, n), (b.slot_elems, 1), local.storage_offset() + b.off + loff)))
        return out

    def fill_from_stream(self, stream, local):
        """Copy every row this rank holds (bands + halos) out of a full stream."""
        for full, loc in self.held_views(stream, local):
            loc.copy_(full)
        return local

    def packed_elems(self) -> int:
        cw = self.width // 2
        return sum(b.cnt * (self.width * (b.y1 - b.y0) + 2 * cw * (b.c1 - b.c0)) for b in self.bands)


def cfg4_layout(rank: int, world: int, frames: int, width: int = 3840, height: int = 2160) -> Cfg4Layout:
    """Local buffer of ``rank``: for each band it codes, its frame slots of band
    rows + one halo row per plane (none for the top band)."""
    bands_y = ctu_bands(height, world)
    cw = width // 2
    out, off = [], 0
    for b, f0, cnt in cfg4_plan(rank, world, frames):
        y0, y1 = bands_y[b]
        if y1 <= y0:
            continue
        hy = 1 if y0 > 0 else 0
        c0, c1 = y0 // 2, y1 // 2
        hc = 1 if c0 > 0 else 0
        u_off = width * (y1 - y0 + hy)
        ce = cw * (c1 - c0 + hc)
        slot = u_off + 2 * ce
        out.append(Cfg4Band(b, f0, cnt, y0, y1, hy, hc, off, slot, u_off, ce))
        off += cnt * slot
    return Cfg4Layout(width, height, world, rank, frames, out, off)


def cfg4_pack(stream, rank: int, world: int, frames: int, width: int, height: int):
    """This rank's reconstructed bands of a FULL-frame stream, packed in
    Cfg4Layout.full_views order into one flat tensor."""
    import torch
    views = cfg4_layout(rank, world, frames, width, height).full_views(stream)
    return torch.cat([v.reshape(-1) for v in views]) if views else stream[:0].clone()


def cfg4_unpack(packed, rank: int, world: int, frames: int, width: int, height: int, stream):
    """Inverse of cfg4_pack: write rank ``rank``'s bands into the full stream."""
    o = 0
    for view in cfg4_layout(rank, world, frames, width, height).full_views(stream):
        view.copy_(packed[o:o + view.numel()].view(view.shape))
        o += view.numel()
    return o


def cfg4_packed_elems(rank: int, world: int, frames: int, width: int, height: int) -> int:
    return cfg4_layout(rank, world, frames, width, height).packed_elems()

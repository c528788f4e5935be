"""Multi-rank path on CPU: CTU-band sharding invariants and the gather step
with the gloo backend at world_size 2 (the RCCL path on the GPU box is the same
torch.distributed.gather call).  Per-rank "compute" here is the oracle standing
in for the device kernel -- this file tests the sharding/gather plumbing only;
kernel parity is covered by tests/test_gpu_parity.py."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from nano_hevc import gpu, shard


@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_bands_cover_frame_once_and_balance(world):
    h = 2160
    bands = shard.ctu_bands(h, world)
    assert bands[0][0] == 0 and bands[-1][1] == h
    assert all(a[1] == b[0] for a, b in zip(bands, bands[1:]))
    assert all(y0 % 32 == 0 for y0, _ in bands)
    frames = 2 * world
    per_rank = [shard.rank_layout(r, world, frames).blocks() for r in range(world)]
    assert len(set(per_rank)) == 1 and sum(per_rank) == frames * 194400
    # every (frame, band) is owned by exactly one rank
    owned = {}
    for r in range(world):
        for g in shard.rank_layout(r, world, frames).groups:
            for f, b in g.frames:
                assert (f, b) not in owned
                owned[(f, b)] = r
    assert len(owned) == frames * world
    sets = shard.rank_layout(0, world, frames).plane_sets(gpu)
    assert len(sets) <= 8   # NH_MAX_PLANE_SETS


def _frames(n, w, h, seed):
    rng = np.random.default_rng(seed)
    fe = gpu.yuv420_frame_elems(w, h)
    return [rng.integers(-255, 256, size=fe).astype(np.int16) for _ in range(n)]


def test_fill_scatter_roundtrip():
    w, h, world, n = 128, 160, 3, 6
    frames = _frames(n, w, h, 1)
    back = [np.zeros_like(f) for f in frames]
    for r in range(world):
        L = shard.rank_layout(r, world, n, w, h)
        loc = np.zeros(L.total_elems, np.int16)
        shard.fill_from_frames(L, frames, loc)
        shard.scatter_to_frames(L, loc, back)
    for a, b in zip(frames, back):
        assert np.array_equal(a, b)


def _oracle_levels_local(L, loc):
    """Apply the 8x8 DCT+quant oracle to every plane of every band in a local buffer."""
    from oracle import oracle as O
    out = np.zeros_like(loc)
    w, cw = L.width, L.width // 2
    for g in L.groups:
        for slot in range(len(g.frames)):
            s = g.base + slot * g.frame_elems
            planes = [(s, g.y_rows, w), (s + w * g.y_rows, g.y_rows // 2, cw),
                      (s + w * g.y_rows + cw * (g.y_rows // 2), g.y_rows // 2, cw)]
            for off, hh, ww in planes:
                p = loc[off:off + hh * ww].reshape(hh, ww)
                out[off:off + hh * ww] = O.fwd8x8_quant_plane(p, 32).ravel()
    return out


def _worker(rank, world, port, w, h, n, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    frames = _frames(n, w, h, 5)
    L = shard.rank_layout(rank, world, n, w, h)
    loc = np.zeros(L.total_elems, np.int16)
    shard.fill_from_frames(L, frames, loc)
    lv = torch.from_numpy(_oracle_levels_local(L, loc))
    sizes = [shard.rank_layout(r, world, n, w, h).total_elems for r in range(world)]
    got = shard.gather_to_root(lv, sizes, dist)
    if rank == 0:
        from oracle import oracle as O
        full = [np.zeros_like(f) for f in frames]
        for r in range(world):
            shard.scatter_to_frames(shard.rank_layout(r, world, n, w, h), got[r].numpy(), full)
        ok = True
        cw, ch = w // 2, h // 2
        for f, fr in enumerate(frames):
            exp = np.concatenate([O.fwd8x8_quant_plane(fr[:w * h].reshape(h, w), 32).ravel(),
                                  O.fwd8x8_quant_plane(fr[w * h:w * h + cw * ch].reshape(ch, cw), 32).ravel(),
                                  O.fwd8x8_quant_plane(fr[w * h + cw * ch:].reshape(ch, cw), 32).ravel()])
            ok &= bool(np.array_equal(full[f], exp))
        q.put(ok)
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_gloo_world2_band_shard_and_gather():
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    w, h, n = 128, 96, 4        # 3 CTU rows -> bands of 2 and 1 CTU rows
    procs = [ctx.Process(target=_worker, args=(r, 2, port, w, h, n, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    assert q.get() is True


# ---------------------------------------------------------------- config 4: bands of full frames

def _cfg4_worker(rank, world, port, w, h, n, q):
    """Each rank holds the full stream, computes only its CTU-row bands (the
    oracle stands in for the device kernel: same row0/row1 contract as
    nh_tu_pipeline_planes), packs them, gathers to rank 0; rank 0 unpacks and
    must get exactly the unsharded reconstruction."""
    from oracle import oracle as O
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    frames = _frames(n, w, h, 11)
    cw, ch = w // 2, h // 2
    stream = np.concatenate(frames)
    rec = np.zeros_like(stream)
    bands = shard.ctu_bands(h, world)

    def planes_of(f):
        base = f * (w * h + 2 * cw * ch)
        return [(base, h, w, 32, 0), (base + w * h, ch, cw, 16, 1), (base + w * h + cw * ch, ch, cw, 16, 2)]

    for b, f0, cnt in shard.cfg4_plan(rank, world, n):
        y0, y1 = bands[b]
        r0, r1 = y0 // 32, (y1 + 31) // 32
        for f in range(f0, n, world):
            for off, ph, pw, ctb, pid in planes_of(f):
                _, r, _ = O.tu_pipeline_plane(stream[off:off + ph * pw].reshape(ph, pw), ctb, pid, 77, 30, pid == 0, r0, r1)
                rows = slice(y0, y1) if pid == 0 else slice(y0 // 2, y1 // 2)
                rec[off:off + ph * pw].reshape(ph, pw)[rows] = r[rows]
    packed = shard.cfg4_pack(torch.from_numpy(rec), rank, world, n, w, h)
    assert packed.numel() == shard.cfg4_packed_elems(rank, world, n, w, h)
    sizes = [shard.cfg4_packed_elems(r, world, n, w, h) for r in range(world)]
    got = shard.gather_to_root(packed, sizes, dist)
    if rank == 0:
        full = torch.zeros(stream.size, dtype=torch.int16)
        for r in range(world):
            assert shard.cfg4_unpack(got[r], r, world, n, w, h, full) == sizes[r]
        exp = np.zeros_like(stream)
        for f in range(n):
            for off, ph, pw, ctb, pid in planes_of(f):
                _, r, _ = O.tu_pipeline_plane(stream[off:off + ph * pw].reshape(ph, pw), ctb, pid, 77, 30, pid == 0)
                exp[off:off + ph * pw] = r.ravel()
        q.put(bool(np.array_equal(full.numpy(), exp)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 4), (3, 5)])
def test_gloo_cfg4_band_shard_pack_gather(world, n):
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    w, h = 96, 112        # 4 luma CTU rows (3.5 -> partial), ragged chroma
    procs = [ctx.Process(target=_cfg4_worker, args=(r, world, port, w, h, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
        assert p.exitcode == 0
    assert q.get() is True


def test_cfg4_plan_covers_every_band_once():
    for world in range(1, 9):
        for n in (1, world, 3 * world + 1):
            seen = {}
            for r in range(world):
                for b, f0, cnt in shard.cfg4_plan(r, world, n):
                    for f in range(f0, n, world):
                        assert (f, b) not in seen
                        seen[(f, b)] = r
                        assert shard.band_of(r, f, world) == b
            assert len(seen) == n * world

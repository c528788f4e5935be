"""bench.py's multi-GPU launch path on CPU (no GPU): `--gpus N` without a
launcher starts N ranks itself (torch.distributed.run), a WORLD_SIZE that
disagrees with --gpus is refused, and the config-4 band layout (input sharded
to bands + one halo row) tiles every frame exactly once and holds all a band's
TUs read."""
import json
import os
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(kw)
    return env


def _last_json(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert lines, out
    return json.loads(lines[-1])


@pytest.mark.parametrize("n", [1, 2, 3])
def test_gpus_flag_launches_that_many_ranks(n):
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--launcher-selftest"], env=_env(),
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    d = _last_json(r.stdout)
    assert d["n_gpus"] == n and d["rank_sum"] == n * (n - 1) // 2


def test_world_size_mismatch_is_refused():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launcher-selftest"],
                       env=_env(WORLD_SIZE="3", RANK="0", LOCAL_RANK="0"), capture_output=True, text=True, timeout=120)
    assert r.returncode == 2
    assert "WORLD_SIZE=3" in r.stderr


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_cfg4_layout_views_tile_the_stream(world):
    """Every band row of every frame is packed by exactly one rank, and a rank's
    local buffer holds its bands plus one halo row per band and plane: about
    1/N of the stream."""
    from nano_hevc import shard
    W, H, frames = 64, 200, 2 * world      # 200 rows: 7 CTU rows, the last one partial
    fe = W * H + 2 * (W // 2) * (H // 2)
    stream = torch.arange(frames * fe, dtype=torch.int64)
    seen = torch.zeros(frames * fe, dtype=torch.int64)
    held = 0
    for r in range(world):
        lay = shard.cfg4_layout(r, world, frames, W, H)
        views = lay.full_views(stream)
        packed = torch.cat([v.reshape(-1) for v in views]) if views else torch.zeros(0, dtype=torch.int64)
        assert packed.numel() == lay.packed_elems() == shard.cfg4_packed_elems(r, world, frames, W, H)
        seen[packed] += 1
        local = lay.fill_from_stream(stream, torch.full((max(1, lay.total_elems),), -1, dtype=torch.int64))
        assert bool((local[:lay.total_elems] >= 0).all())          # every local element comes from the stream
        lp = torch.cat([v.reshape(-1) for v in lay.local_views(local)]) if views else packed
        assert torch.equal(lp, packed)                               # local and full views agree element by element
        halo = sum(b.cnt * (b.hy * W + 2 * b.hc * (W // 2)) for b in lay.bands)
        assert lay.total_elems == lay.packed_elems() + halo
        held += lay.total_elems
    assert bool((seen == 1).all())
    assert held - frames * fe == sum(b.cnt * (b.hy * W + 2 * b.hc * (W // 2))
                                     for r in range(world) for b in shard.cfg4_layout(r, world, frames, W, H).bands)


@pytest.mark.parametrize("world", [2, 3])
def test_cfg4_band_local_planes_need_only_the_halo(world):
    """The launch contract of a band-local plane set, checked with the oracle:
    a full-height plane that holds ONLY the rank's local rows (band + halo row)
    and poison everywhere else gives the band exactly the unsharded result;
    gpu.sets_fit_rows accepts the layout's sets for exactly those rows."""
    import numpy as np
    from oracle import oracle as O
    from nano_hevc import gpu, shard
    W, H, frames = 96, 200, world
    fe = W * H + 2 * (W // 2) * (H // 2)
    rng = np.random.default_rng(3)
    stream = torch.from_numpy(rng.integers(0, 256, frames * fe).astype(np.int16))
    for r in range(world):
        lay = shard.cfg4_layout(r, world, frames, W, H)
        local = lay.fill_from_stream(stream, torch.zeros(lay.total_elems, dtype=torch.int16)).numpy()
        for b in lay.bands:
            r0, r1 = b.ctu_rows()
            for sset, ctb, ppg in ((lay.luma_set(gpu, b), 32, 1), (lay.chroma_set(gpu, b), 16, 2)):
                gpu.sets_fit_rows([sset], lay.total_elems, r0 * ctb - 1, r1 * ctb, "t")
                if b is lay.bands[0] and b.y0 > 0 and ctb == 32:   # its halo row is the buffer's first row
                    with pytest.raises(ValueError):
                        gpu.sets_fit_rows([sset], lay.total_elems, r0 * ctb - 2, r1 * ctb, "t")
                for j in range(b.cnt):
                    f = b.f0 + j * world
                    for c in range(ppg):
                        pid = c + (0 if ctb == 32 else 1)
                        h, w = sset.height, sset.width
                        base = sset.base + j * sset.group_stride + c * sset.plane_stride
                        lo, hi = max(0, r0 * ctb - 1), min(h, r1 * ctb)
                        plane = np.full((h, w), 30000, np.int16)         # poison: any read outside changes results
                        plane[lo:hi] = local[base + lo * w:base + hi * w].reshape(hi - lo, w)
                        full_off = f * fe + (0 if pid == 0 else W * H + (pid - 1) * (W // 2) * (H // 2))
                        ref = stream[full_off:full_off + h * w].numpy().reshape(h, w)
                        got = O.tu_pipeline_plane(plane, ctb, pid, 77, 30, pid == 0, r0, r1)
                        exp = O.tu_pipeline_plane(ref, ctb, pid, 77, 30, pid == 0)
                        rows = slice(r0 * ctb, hi)
                        assert np.array_equal(got[0][rows], exp[0][rows]) and np.array_equal(got[1][rows], exp[1][rows])


def test_bench_inputs_travel_to_the_gpu_box():
    """bench.py reads profiles/pmc_traffic.json for roofline.traffic: no
    .gpurunignore pattern may keep it (or the built library) off the GPU box."""
    import fnmatch
    pats = [p.strip() for p in open(os.path.join(ROOT, ".gpurunignore")) if p.strip() and not p.startswith("#")]
    for rel in ("profiles/pmc_traffic.json", "nano-hevc_amd/nano_hevc/libnanohevc.so", "bench.py"):
        parts = rel.split("/")
        for p in pats:
            if p.startswith("./"):
                anchored = p[2:].rstrip("/")
                assert not (rel == anchored or rel.startswith(anchored + "/")), (rel, p)
            else:
                assert not any(fnmatch.fnmatch(x, p) for x in parts) and not fnmatch.fnmatch(rel, p), (rel, p)
    assert os.path.exists(os.path.join(ROOT, "profiles", "pmc_traffic.json"))

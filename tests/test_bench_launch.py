"""bench.py's multi-GPU launch path on CPU (no GPU): `--gpus N` without a
launcher starts N ranks itself (torch.distributed.run), a WORLD_SIZE that
disagrees with --gpus is refused, and the config-4 band views used by the
uint8 recon gather tile every frame exactly once."""
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
def test_cfg4_band_views_tile_the_stream(world):
    sys.path.insert(0, ROOT)
    import bench
    from nano_hevc import shard
    W, H, frames = 64, 72, 2 * world      # 72 rows: a partial last CTU row
    fe = W * H + 2 * (W // 2) * (H // 2)
    stream = torch.arange(frames * fe, dtype=torch.int64)
    seen = torch.zeros(frames * fe, dtype=torch.int64)
    for r in range(world):
        views = bench.band_views(stream, r, world, frames, W, H)
        packed = torch.cat([v.reshape(-1) for v in views]) if views else torch.zeros(0, dtype=torch.int64)
        assert packed.numel() == shard.cfg4_packed_elems(r, world, frames, W, H)
        seen[packed] += 1
    assert bool((seen == 1).all())


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

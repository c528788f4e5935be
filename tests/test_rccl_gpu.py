"""The RCCL branch of bench.py executed on the one-GPU box:
tests/rccl_world1.py builds an ``nccl`` (RCCL) process group at world size 1
through bench.init_dist and drives bench.OverlappedGather / run_phase_gather
with device tensors -- config 2's int64 words and config 4's packed uint8 recon
bands -- checking every gathered step against what that step computed (a slot
overwritten before its gather completed would show the wrong step)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_rccl_world1_overlapped_gathers_match_their_steps():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "rccl_world1.py")], env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert lines, r.stdout[-2000:] + r.stderr[-2000:]
    d = json.loads(lines[-1])
    assert d["backend"] == "nccl" and d["world"] == 1
    assert d["cfg2_int64_gathers_equal_sent"] is True and d["cfg2_steps"] >= 5
    assert d["cfg2_frames"] == 128 and d["cfg2_levels_fraction_gathered"] == 1.0
    assert d["cfg2_gather_calls_per_step"] == 16
    assert d["cfg4_uint8_gathers_equal_sent"] is True and d["cfg4_bytes_per_gather"] > 0

"""The multi-rank device path executed across real ranks:
bench.py launches 2 ranks itself (--gpus 2), each running the HIP kernels on
its CTU-row bands; on the one-GPU box both ranks share device 0 and talk over
gloo (NH_DIST_BACKEND / NH_FORCE_DEVICE, the script's rehearsal knobs), on an
8-GPU node the same code runs one rank per GPU over RCCL.

* config 4: rank 0 reassembles the gathered uint8 recon bands and compares
  them with an unsharded run of the whole stream (``--check``);
* config 2: the line reports both ranks' blocks and the gather phase.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(NH_DIST_BACKEND="gloo", NH_FORCE_DEVICE="0")
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--no-cpu-baseline"] + args, env=env,
                       capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert lines, r.stdout[-2000:] + r.stderr[-2000:]
    return json.loads(lines[-1])


def test_cfg4_two_ranks_gathered_recon_equals_unsharded():
    d = _run(["--config", "4", "--frames", "2", "--steps", "2", "--warmup", "1", "--gather-steps", "1", "--check"])
    assert d["n_gpus"] == 2
    assert d["gathered_recon_equals_unsharded"] is True
    assert d["gather_inclusive"]["bytes_into_root_per_step"] > 0
    # the input is sharded: rank 0 holds its bands + one halo row per band and plane, ~1/2 of the stream
    assert 0.5 <= d["config"]["source_fraction_rank0"] < 0.51


def test_cfg2_two_ranks_report_the_whole_job():
    d = _run(["--frames", "4", "--steps", "2", "--warmup", "1", "--gather-steps", "1", "--gather-frames", "2"])
    assert d["n_gpus"] == 2 and d["config"]["frames_per_gpu"] == 4
    g = d["gather_inclusive"]
    assert g["levels_fraction_gathered"] == 0.5
    assert g["bytes_into_root_per_step"] > 0

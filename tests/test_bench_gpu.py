"""bench.py's one-GPU line against the driver's contract: every key the
contract names, the roofline object (achieved / peak = frac, bound, unit) and
the cpu_baseline object (value, unit, cores, kind, sample), with the sampled
GPU outputs bit-exact against the CPU restatement -- for the headline
configuration and for --config 4 (blocks/s per TU size)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"}


def _run(args):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, BENCH] + args, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def _check_common(d, steps):
    assert KEYS <= set(d), KEYS - set(d)
    assert d["n_gpus"] == 1 and d["steps"] == steps and d["higher_is_better"] is True and d["scaling"] == "weak"
    assert d["value"] > 0 and d["ms_per_step"] > 0 and "workload" in d["config"]
    rf = d["roofline"]
    assert rf["bound"] in ("hbm", "mfma", "valu")
    if rf["bound"] == "valu":   # config 4: VALU issue against the attainable rate of its instruction mix
        assert rf["unit"] == "G VALU wave-instr/s" and rf["valu_instr_per_step"] > 0 and rf["hbm"]["peak"] == 8000.0
    else:
        assert rf["unit"] in ("GB/s", "TFLOP/s") and rf["peak"] == 8000.0
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-9 and 0 < rf["frac"] < 1
    assert rf["kernel_ms_avg"] <= d["ms_per_step"] * 1.05
    cb = d["cpu_baseline"]
    assert {"value", "unit", "cores", "kind", "sample"} <= set(cb) and cb["kind"] == "port" and cb["value"] > 0


def test_bench_headline_line():
    d = _run(["--frames", "2", "--steps", "3", "--warmup", "1", "--cpu-seconds", "0.5"])
    _check_common(d, 3)
    assert d["unit"] == "blocks/s" and d["config"]["blocks_per_launch"] == 2 * 194400
    assert d["cpu_baseline"]["gpu_levels_bit_exact_on_sample"] is True
    # the achievable streaming-copy rate beside the kernel's (context for the HBM fraction): the
    # product's 16-B/lane nontemporal linear copy, not torch's slower copy_
    rf = d["roofline"]
    assert rf["stream_copy_GBps"] > 0 and rf["torch_copy_GBps"] > 0
    assert abs(rf["frac_of_achievable_copy"] - rf["achieved"] / rf["stream_copy_GBps"]) < 1e-9
    # value is the whole job's blocks over the timed wall clock
    assert abs(d["value"] * d["ms_per_step"] / 1e3 - 2 * 194400) / (2 * 194400) < 1e-6
    # device-time-only rate (one rank: blocks / HIP-event time) beside it, and the reference's numpy
    # figure, labelled as another host's
    assert abs(d["compute_only_sum_blocks_per_s"] - 2 * 194400 / (rf["kernel_ms_avg"] * 1e-3)) < 1e-3 * d["value"]
    rn = d["cpu_baseline"]["reference_numpy"]
    assert rn["kind"] == "reference" and rn["value"] > 0 and "not the GPU box" in rn["host"]


def test_bench_config4_line():
    d = _run(["--config", "4", "--frames", "2", "--steps", "2", "--warmup", "1", "--cpu-seconds", "0.5"])
    _check_common(d, 2)
    assert d["unit"] == "samples/s" and d["cpu_baseline"]["gpu_outputs_bit_exact_on_sample"] is True
    assert d["cpu_baseline"]["cores"] > 1 and d["cpu_baseline"]["value_1thread"] > 0
    assert d["config"]["source_fraction_rank0"] == 1.0
    assert d["compute_only_sum_samples_per_s"] >= d["value"] * 0.95
    # the default: exact compact int16 levels on the device (widened for the CPU check above)
    rf = d["roofline"]
    assert d["config"]["levels"].startswith("int16") and rf.get("hbm", rf)["bytes_per_sample"] == 6.0625
    if os.path.exists(os.path.join(ROOT, "profiles", "valu_roofline.json")):   # committed VALU roofline inputs
        # the VALU view leads, from counts of THIS build's kernel sources (strict; the CPU
        # suite's test_valu_profile_matches_the_tree fails first when the sources moved on)
        assert d["roofline"]["bound"] == "valu" and not d["roofline"].get("valu_profile_stale"), d["roofline"]
    tu = d["config"]["tu_blocks_per_step"]
    # every sample of the two frames lies in exactly one TU
    area = sum(n * (4 << k) ** 2 for k, n in enumerate(tu[f"{4 << k}x{4 << k}"] for k in range(4)))
    assert area == d["config"]["samples_per_step_rank0"] == 2 * (3840 * 2160 * 3 // 2)

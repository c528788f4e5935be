"""The VALU-roofline tooling on the CPU: the dynamic-mix LP of
tools/valu_dyn.py on a control-flow graph whose execution counts the counters
pin, and the internal consistency of the committed profiles/valu_roofline.json
(achieved = VALU per frame / busy time, frac = achieved / attainable, the
dynamic bracket ordered).  Recomputing the committed file from its committed
inputs (`tools/pmc_valu.py --tag r04zg --dir profiles/r04/valu --cal r04zg`,
then `--tag r04zq --rates-tag r04zk --cal r04zk --configs 3,closed,closed4 --merge`) takes
minutes of hipcc disassembly and is not repeated here."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def test_dynamic_mix_lp_brackets_the_pinned_execution():
    pytest.importorskip("scipy")
    import valu_dyn as vd
    # entry -> loop body (taken back-edge or fall through) -> exit
    blocks = [(["v_add_u32", "s_cbranch_execz"], [1]),
              (["v_mov_b32", "v_dot2_i32_i16", "s_cbranch_scc1"], [1, 2]),
              (["v_lshlrev_b32", "s_endpgm"], [])]
    rates = {"v_add_u32": 1e12, "v_mov_b32": 1e12, "v_dot2_i32_i16": 5e11, "v_lshlrev_b32": 5e11,
             "v_add3_u32": 5e11}
    waves, trips = 10000, 5
    meas = {"SQ_WAVES": waves, "SQ_INSTS_VALU": waves * (1 + 2 * trips + 1)}
    r = vd.solve(blocks, meas, rates, tol=0.005)
    assert r["feasible"], r
    exact = waves * (1 / 1e12 + trips * (1 / 1e12 + 1 / 5e11) + 1 / 5e11)
    lo, hi = r["min"]["T_s"], r["max"]["T_s"]
    assert lo <= exact <= hi and (hi - lo) / exact < 0.02
    # a counter the CFG cannot reproduce makes the program infeasible rather than mispriced
    bad = dict(meas, SQ_INSTS_VALU=waves * 1)
    assert not vd.solve(blocks, bad, rates, tol=0.005)["feasible"]


def test_committed_valu_roofline_is_self_consistent():
    path = os.path.join(ROOT, "profiles", "valu_roofline.json")
    d = json.load(open(path))
    assert set(d["configs"]) >= {"cfg3_1080p_yuv420", "cfg3_closed_1080p_yuv420", "cfg4_4k_yuv420",
                                 "cfg4_closed_4k_yuv420", "cfg5_8k_yuv420"}
    for key, e in d["configs"].items():
        ach = e["valu_per_frame"] / (e["busy_ms_per_frame"] * 1e-3)
        assert abs(ach / e["achieved_valu_winst_per_s"] - 1) < 1e-9, key
        assert abs(e["valu_frac"] - ach / e["attainable_valu_winst_per_s"]) < 1e-9, key
        lo, hi = e["valu_frac_range"]
        assert lo <= hi and abs(lo - e["valu_frac"]) < 1e-12, key
        alo, ahi = e["attainable_dynamic_range"]
        assert alo <= ahi and abs(ahi - e["attainable_valu_winst_per_s"]) < 1e-3 * ahi, key
        assert e["peak_kind"].startswith("dynamic mix"), key
        # every kernel input the file cites is committed
        for src in e["source"].values():
            assert src is None or os.path.exists(os.path.join(ROOT, src)), (key, src)


def test_valu_profile_matches_the_tree():
    """The committed VALU roofline (profiles/valu_roofline.json) was measured on THESE kernel
    sources: every config's recorded sha256 over its source files equals the tree's.
    A kernel change must be re-profiled (TAG=x tools/gpu_run.sh valu_rate pmc_cal valu_kt
    valu_pmc1 valu_pmc2 valu_pmc3 valu_pmc4; tools/pmc_valu.py --tag x --cal x --rates-tag x)."""
    import json
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import pmc_valu
    d = json.load(open(os.path.join(ROOT, "profiles", "valu_roofline.json")))
    keys = {v[0]: c for c, v in pmc_valu.CONFIGS.items()}
    stale = {}
    for key, ent in d["configs"].items():
        src = ent["sources"]
        assert src["files"] == pmc_valu.SOURCES[keys[key]], key
        now = pmc_valu.sources_digest(src["files"])
        if now != src["sha256"]:
            stale[key] = (src["sha256"][:12], now[:12])
    assert not stale, f"profiles/valu_roofline.json is stale for {stale}"

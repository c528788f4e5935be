#!/usr/bin/env python3
"""VALU roofline of the VALU-bound configs from committed profiles.

    python tools/pmc_valu.py --tag r03a [--dir gpurun_out] [--out profiles/valu_roofline.json]

Inputs, all written by `TAG=... tools/gpu_run.sh valu_rate valu_kt valu_pmc1 valu_pmc2`
(one profiler run per config of tools/bench_configs.py, so every CSV holds one
config's kernels):
  * valu_rate_<tag>.jsonl: chip-wide issue rate of each VALU opcode class
    (tools/ab/valu_rate.hip, 8 waves/SIMD, on the clock the chip holds);
  * valu_kt_<tag>_<cfg>/: kernel trace (average duration, calls per kernel);
  * valu_pmc1_<tag>_<cfg>/: SQ_INSTS_VALU, SQ_WAVES, SQ_WAVE_CYCLES,
    SQ_BUSY_CYCLES, SQ_ACTIVE_INST_VALU, SQ_WAIT_ANY, SQ_INSTS_SALU, SQ_INSTS_LDS
    per dispatch;
  * valu_pmc2_<tag>_<cfg>/: SQ_VALU_MFMA_BUSY_CYCLES, SQ_ACTIVE_INST_ANY,
    SQ_WAIT_INST_ANY, SQ_INSTS_VMEM_RD/WR, SQ_ACTIVE_INST_LDS, GRBM_GUI_ACTIVE,
    GRBM_COUNT per dispatch;
  * the static VALU mix of each kernel (tools/valu_mix.py, compiled here).

Per kernel: achieved = SQ_INSTS_VALU per dispatch / average duration (chip-wide
VALU wave-instructions per second); attainable = the kernel's static VALU mix
priced at the measured per-opcode rates, N / sum(n_i / r_i); frac = achieved /
attainable.  Per config: the same over one frame's worth of its kernels
(instructions summed, attainable combined harmonically, time = the union of the
kernels' trace intervals per frame, so concurrent launches count once).  SQ ratios say where the rest goes:
valu_active = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES, wait_any = SQ_WAIT_ANY /
SQ_WAVE_CYCLES, clock = GRBM_GUI_ACTIVE / duration.
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# kernels of the measuring harness, not of a config (bench_configs' PSNR reduction)
HARNESS = ("k_sse_i16", "k_tc32_widen", "k_tu_widen")   # (+ the compact levels' widen, run once for the digest)

# bench_configs config -> (profile key, anchor kernel, anchor dispatches per frame)
CONFIGS = {
    "3": ("cfg3_1080p_yuv420", "k_intra_rdo8<1, true, 1>", 3.0),
    "closed": ("cfg3_closed_1080p_yuv420", "k_intra_rdo8_closed_tag<1, 1>", 1 / 64),
    "4b": ("cfg4_4k_yuv420", "k_ctu_open<32", 1 / 16),
    "closed4": ("cfg4_closed_4k_yuv420", "k_tu_closed_pair<3, true, 32", 1 / 64),   # (luma instance: one per launch set)
    "5b": ("cfg5_8k_yuv420", "k_tc32_hd<2", 2 / 8),
    # round 6: the compact-level instances (int16 levels, int32 spill; one profiler run each)
    "4bc": ("cfg4_4k_yuv420_int16", "k_ctu_open<32", 1 / 16),
    "5bc": ("cfg5_8k_yuv420_int16", "k_tc32_hd<2", 2 / 8),
}
# the sources a config's kernels are compiled from: their digest goes into the
# entry, and bench.py / tools/bench_configs.py recompute it to tell whether the
# committed instruction counts still describe the build they run
_HDRS = ["nh_common.hpp", "nh_internal.hpp", "nh_packed.hpp", "nh_tree.hpp", "nh_mfma.hpp", "nh_f16mma.hpp", "nh_mosaic.hpp",
         "nh_ldsdma.hpp"]
SOURCES = {
    "3": ["nh_intraloop.hip"] + _HDRS,
    "closed": ["nh_intraloop.hip"] + _HDRS,
    "4b": ["nh_ctu.hip"] + _HDRS,
    "closed4": ["nh_intraloop.hip"] + _HDRS,
    "5b": ["nh_ctu.hip", "nh_tc32.hip"] + _HDRS,
    "4bc": ["nh_ctu.hip"] + _HDRS,
    "5bc": ["nh_ctu.hip", "nh_tc32.hip"] + _HDRS,
}


def sources_digest(files):
    """sha256 over the listed nano-hevc_amd/csrc files, in order (bench.py: same rule)."""
    import hashlib
    h = hashlib.sha256()
    for f in files:
        h.update(open(os.path.join(ROOT, "nano-hevc_amd", "csrc", f), "rb").read())
    return h.hexdigest()


def _find(d, pattern):
    hits = sorted(glob.glob(os.path.join(d, "**", pattern), recursive=True))
    return hits[0] if hits else None


def kernel_times(d):
    p = _find(d, "*kernel_stats.csv")
    out = {}
    if p:
        for r in csv.DictReader(open(p)):
            if "nh::" in r["Name"] and not any(k in r["Name"] for k in HARNESS):
                out[r["Name"]] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"])}
    return out, p


def busy_ns(d):
    """Union of the config's kernel intervals in the trace (ns): concurrent launches
    (config 4's closed loop runs its luma and chroma wavefronts side by side)
    count once."""
    p = _find(d, "*kernel_trace.csv")
    if not p:
        return None
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(p))
                if "nh::" in r["Kernel_Name"] and not any(k in r["Kernel_Name"] for k in HARNESS))
    tot, cur_s, cur_e = 0, None, None
    for a, b in iv:
        if cur_e is None or a > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = a, b
        else:
            cur_e = max(cur_e, b)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def counters(d):
    p = _find(d, "*counter_collection.csv")
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    if p:
        for r in csv.DictReader(open(p)):
            if "nh::" in r["Kernel_Name"] and not any(k in r["Kernel_Name"] for k in HARNESS):
                per[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, d2 in per.items():
        e = {c: statistics.mean(v) for c, v in d2.items()}
        e["_dispatches"] = max(len(v) for v in d2.values())
        out[k] = e
    return out, p


def static_mix(rates_path):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "valu_mix.py"), "--rates", rates_path, "--kernels", "nh::"],
                       capture_output=True, text=True, check=True)
    return {d["kernel"]: d for d in (json.loads(x) for x in r.stdout.splitlines() if x.startswith("{"))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("--dir", default=os.path.join(ROOT, "gpurun_out"))
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "valu_roofline.json"))
    ap.add_argument("--configs", default=",".join(CONFIGS))
    ap.add_argument("--cal", default=None, help="tag of the tools/ab/_pmc_cal passes (pmc_cal3_<tag>, pmc_cal4_<tag>, "
                                                "pmc_cal_<tag>.log in --cal-dir): dynamic mix from valu_pmc3/4")
    ap.add_argument("--cal-dir", default=None)
    ap.add_argument("--rates-tag", default=None, help="tag of the valu_rate_<tag>.jsonl issue-rate probe in --dir "
                    "(default: --tag; the rates are the chip's, not the build's)")
    ap.add_argument("--merge", action="store_true",
                    help="keep the other configs of an existing --out file (per-config tags)")
    ap.add_argument("--refresh-digests", default=None, metavar="REASON",
                    help="only re-record the source digests of --out's configs (after a source change that leaves "
                         "the device code objects identical; REASON says how that was checked)")
    a = ap.parse_args()
    if a.refresh_digests:
        res = json.load(open(a.out))
        for key, ent in res["configs"].items():
            c = next(k for k, v in CONFIGS.items() if v[0] == key)
            new = {"files": SOURCES[c], "sha256": sources_digest(SOURCES[c])}
            if new != ent.get("sources"):
                ent.setdefault("sources_history", []).append({"previous": ent.get("sources"), "reason": a.refresh_digests})
                ent["sources"] = new
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1, sort_keys=True)
            f.write("\n")
        return 0
    rates_path = os.path.join(a.dir, f"valu_rate_{a.rates_tag or a.tag}.jsonl")
    rates = [json.loads(x) for x in open(rates_path) if x.startswith("{")]
    mix = static_mix(rates_path)
    dyn = None
    if a.cal:
        import valu_dyn
        cd = a.cal_dir or a.dir
        valu_dyn.load_membership(os.path.join(cd, f"pmc_cal3_{a.cal}"), os.path.join(cd, f"pmc_cal4_{a.cal}"),
                                 os.path.join(cd, f"pmc_cal_{a.cal}.log"))
        dyn = valu_dyn
    res = {"tag": a.tag, "rates_chip_winst_per_s": {r["op"]: r["chip_winst_per_s"] for r in rates},
           "method": "achieved = SQ_INSTS_VALU per dispatch / kernel-trace average duration; attainable = static "
                     "VALU mix (tools/valu_mix.py) priced at the measured per-opcode rates (tools/ab/valu_rate.hip)",
           "configs": {}}
    for c in a.configs.split(","):
        key, anchor, anchor_pf = CONFIGS[c]
        times, kt_path = kernel_times(os.path.join(a.dir, f"valu_kt_{a.tag}_{c}"))
        c1, p1_path = counters(os.path.join(a.dir, f"valu_pmc1_{a.tag}_{c}"))
        c2, p2_path = counters(os.path.join(a.dir, f"valu_pmc2_{a.tag}_{c}"))
        if not times or not c1:
            print(f"{c}: missing profiles", file=sys.stderr)
            continue
        f_pmc = next(v["_dispatches"] for k, v in c1.items() if anchor in k) / anchor_pf
        f_kt = next(v["calls"] for k, v in times.items() if anchor in k) / anchor_pf
        kernels, instr, t_att, t_ms, t_lo = {}, 0.0, 0.0, 0.0, 0.0
        for name in sorted(set(times) | set(c1)):
            t, p, q, m = times.get(name), c1.get(name, {}), c2.get(name, {}), mix.get(name)
            e = {"calls_traced": t["calls"] if t else 0, "avg_ms": t["avg_ns"] / 1e6 if t else None,
                 "dispatches_counted": p.get("_dispatches", 0)}
            for k in ("SQ_INSTS_VALU", "SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_ACTIVE_INST_VALU",
                      "SQ_WAIT_ANY", "SQ_INSTS_SALU", "SQ_INSTS_LDS"):
                if k in p:
                    e[k] = p[k]
            for k in ("SQ_VALU_MFMA_BUSY_CYCLES", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_INSTS_VMEM_RD",
                      "SQ_INSTS_VMEM_WR", "SQ_ACTIVE_INST_LDS", "GRBM_GUI_ACTIVE", "GRBM_COUNT"):
                if k in q:
                    e[k] = q[k]
            wc = p.get("SQ_WAVE_CYCLES", 0)
            if wc:
                e["valu_active_of_wave_cycles"] = p.get("SQ_ACTIVE_INST_VALU", 0) / wc
                e["wait_any_of_wave_cycles"] = p.get("SQ_WAIT_ANY", 0) / wc
                if "SQ_WAIT_INST_ANY" in q:
                    e["wait_inst_any_of_wave_cycles"] = q["SQ_WAIT_INST_ANY"] / wc
                if "SQ_ACTIVE_INST_ANY" in q:
                    e["active_any_of_wave_cycles"] = q["SQ_ACTIVE_INST_ANY"] / wc
            if t and "GRBM_GUI_ACTIVE" in q:
                e["clock_GHz_held"] = q["GRBM_GUI_ACTIVE"] / t["avg_ns"]
            if m:
                e["valu_static"] = m["valu_static"]
                e["valu_by_rate_class"] = m["valu_by_rate_class"]
                e["attainable_valu_winst_per_s"] = m.get("attainable_valu_winst_per_s")
                e["attainable_vs_plain_32bit"] = m.get("attainable_vs_plain_32bit")
            if t and "SQ_INSTS_VALU" in p:
                e["achieved_valu_winst_per_s"] = p["SQ_INSTS_VALU"] / (t["avg_ns"] * 1e-9)
                if e.get("attainable_valu_winst_per_s"):
                    e["valu_frac"] = e["achieved_valu_winst_per_s"] / e["attainable_valu_winst_per_s"]
            # one frame's worth of this kernel
            if "SQ_INSTS_VALU" in p:
                e["valu_per_frame"] = p["SQ_INSTS_VALU"] * p["_dispatches"] / f_pmc
                instr += e["valu_per_frame"]
                if e.get("attainable_valu_winst_per_s"):
                    t_att += e["valu_per_frame"] / e["attainable_valu_winst_per_s"]
            if t:
                e["ms_per_frame"] = t["avg_ns"] * t["calls"] / f_kt / 1e6
                t_ms += e["ms_per_frame"]
            kernels[name] = e
        if dyn is not None:   # the dynamic mix: LP bounds per kernel from the instruction counters (valu_dyn)
            d3, d4 = (os.path.join(a.dir, f"valu_pmc{i}_{a.tag}_{c}") for i in (3, 4))
            dr = dyn.run_config([d3, d4], rates_path)
            t_att = 0.0
            for name, e in kernels.items():
                r = dr.get(name)
                if not r or not r.get("feasible") or not e.get("valu_per_frame"):
                    continue
                e["attainable_dynamic_lo"] = r["attainable_lo"]
                e["attainable_dynamic_hi"] = r["attainable_hi"]
                e["dynamic_counter_tol"] = r["tol"]   # the counters' agreement the LP needed (0.005 unless widened)
                e["attainable_static"] = e.get("attainable_valu_winst_per_s")
                e["attainable_valu_winst_per_s"] = r["attainable_hi"]   # the peak: the most the executed mix allows
                e["valu_priced_measured_frac"] = r.get("valu_priced_measured_frac")
                if e.get("achieved_valu_winst_per_s"):
                    e["valu_frac"] = e["achieved_valu_winst_per_s"] / r["attainable_hi"]
                    e["valu_frac_range"] = [e["achieved_valu_winst_per_s"] / r["attainable_hi"],
                                            e["achieved_valu_winst_per_s"] / r["attainable_lo"]]
            t_att = sum(e["valu_per_frame"] / e["attainable_valu_winst_per_s"] for e in kernels.values()
                        if e.get("valu_per_frame") and e.get("attainable_valu_winst_per_s"))
            t_lo = sum(e["valu_per_frame"] / e["attainable_dynamic_lo"] for e in kernels.values()
                       if e.get("valu_per_frame") and e.get("attainable_dynamic_lo"))
        busy = busy_ns(os.path.join(a.dir, f"valu_kt_{a.tag}_{c}"))
        busy_ms = busy / f_kt / 1e6 if busy else t_ms
        ent = {"kernels": kernels, "frames_counted": f_pmc, "frames_traced": f_kt,
               "valu_per_frame": instr, "kernel_ms_per_frame": t_ms, "busy_ms_per_frame": busy_ms,
               "source": {"kernel_trace": os.path.relpath(kt_path, ROOT) if kt_path else None,
                          "pmc1": os.path.relpath(p1_path, ROOT) if p1_path else None,
                          "pmc2": os.path.relpath(p2_path, ROOT) if p2_path else None, "rates": os.path.relpath(rates_path, ROOT)}}
        if busy_ms and t_att:   # over the time the GPU was running the config's kernels (union of intervals)
            ent["achieved_valu_winst_per_s"] = instr / (busy_ms * 1e-3)
            ent["attainable_valu_winst_per_s"] = instr / t_att
            ent["valu_frac"] = ent["achieved_valu_winst_per_s"] / ent["attainable_valu_winst_per_s"]
            if dyn is not None and t_lo:
                ent["attainable_dynamic_range"] = [instr / t_lo, instr / t_att]
                ent["valu_frac_range"] = [ent["valu_frac"], ent["achieved_valu_winst_per_s"] / (instr / t_lo)]
                ent["peak_kind"] = "dynamic mix (LP upper bound, tools/valu_dyn.py)"
            else:
                ent["peak_kind"] = "static mix (tools/valu_mix.py)"
        ent["sources"] = {"files": SOURCES[c], "sha256": sources_digest(SOURCES[c])}
        res["configs"][key] = ent
        print(f"{key:28s} frac {ent.get('valu_frac', float('nan')):.3f}  {busy_ms:.4f} ms/frame busy ({t_ms:.4f} kernel sum)  "
              f"VALU/frame {instr:.4g}", flush=True)
        for name, e in kernels.items():
            if e.get("valu_per_frame", 0) > 0.01 * instr:
                print(f"    {e.get('valu_frac', float('nan')):6.3f} act {e.get('valu_active_of_wave_cycles', float('nan')):.3f} "
                      f"wait {e.get('wait_any_of_wave_cycles', float('nan')):.3f} {name[:90]}")
    if a.merge and os.path.exists(a.out):   # per-config tags: configs re-profiled after a change
        old = json.load(open(a.out))
        tags = old.get("tag") if isinstance(old.get("tag"), dict) else {k: old.get("tag") for k in old.get("configs", {})}
        tags.update({k: a.tag for k in res["configs"]})
        res = {**old, "configs": {**old.get("configs", {}), **res["configs"]}, "tag": tags}
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
        f.write("\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())

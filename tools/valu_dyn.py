#!/usr/bin/env python3
"""Dynamic VALU mix of the product kernels and their attainable VALU rate
(price the executed mix, not the static disassembly).

    python tools/valu_dyn.py --rates RATES.jsonl --pmc DIR [DIR ...] [--json OUT]

Method:
1. Compile the product sources for gfx950 with the product flags and
   disassemble every kernel (tools/valu_mix.py); split each kernel into basic
   blocks at branch targets and after branches, and build its control-flow
   graph (fall-through and taken edges; s_endpgm ends a path).
2. Unknowns: the execution count of every CFG edge (wave executions).  Flow
   conservation at every block (in = out; the entry block receives SQ_WAVES
   waves), and the block counts must reproduce the kernel's MEASURED
   instruction counters (rocprofv3 --pmc, summed over its dispatches):
   SQ_INSTS_VALU / SALU / LDS / SMEM / BRANCH / MFMA / VMEM_RD / VMEM_WR and the
   VALU class counters INT32 / INT64 / CVT / ADD_F32 / MUL_F32 / FMA_F32.  Which
   counter counts which instruction was measured (tools/ab/pmc_cal.hip,
   profiles/r04/valu/pmc_cal_*): an instruction whose membership was not
   measured counts as "0 or 1" (it only widens the bounds).
3. The time the kernel's VALU stream needs at the measured per-opcode issue
   rates (tools/ab/valu_rate.hip, 8 waves/SIMD) is T = sum_b x_b * sum_{i in b}
   1 / r(i); it is minimised and maximised over every execution-count vector
   the constraints allow (two linear programs, scipy HiGHS), so the attainable
   VALU rate N / T of the DYNAMIC mix is bracketed -- [lo, hi] -- with no
   assumption about which branch ran how often beyond what the counters pin.

The rate of a VALU opcode is its own measurement when the probe measured it;
an unmeasured opcode takes its class's (RATE_CLASS of tools/valu_mix.py) and
the fraction of dynamic VALU priced that way is reported.  MFMA instructions
are priced at their VALU-issue cost (an MFMA holds the SIMD's vector issue for
8 cycles, MI355X_MICROARCH.md: 4x a full-rate VALU op).
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import json
import os
import re
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
import valu_mix as vm  # noqa: E402

csv.field_size_limit(1 << 30)

COUNTERS = ["SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_SMEM", "SQ_INSTS_BRANCH", "SQ_INSTS_MFMA",
            "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_INT64",
            "SQ_INSTS_VALU_CVT", "SQ_INSTS_VALU_ADD_F32", "SQ_INSTS_VALU_MUL_F32", "SQ_INSTS_VALU_FMA_F32"]

# ---- counter membership (measured by tools/ab/pmc_cal.hip; 1 = counted, 0 = not, None = not measured)
_SALU_NOT = re.compile(r"^s_(nop|waitcnt|setprio|sleep|branch|cbranch|load|buffer_load|endpgm|barrier)")
_SALU_UNKNOWN = re.compile(r"^s_(barrier|endpgm|getpc|setpc|swappc|getreg|setreg|sendmsg|icache|dcache|memtime|"
                           r"memrealtime|trap|sethalt|ttrace)")
INT32_YES = {"v_add_u32", "v_dot2_i32_i16", "v_dot2c_i32_i16", "v_mad_i32_i24", "v_mul_lo_u32", "v_cmp_gt_i32",
             "v_max_i32", "v_bfe_u32", "v_add_co_u32"}
INT32_NO = {"v_mov_b32", "v_pk_add_u16", "v_cndmask_b32", "v_perm_b32", "v_lshlrev_b64", "v_readfirstlane_b32",
            "v_readlane_b32", "v_accvgpr_read_b32", "v_accvgpr_write_b32", "v_permlane32_swap_b32", "v_pk_mad_u16",
            "v_cvt_f32_i32", "v_cvt_rpi_i32_f32", "v_add_f32", "v_fma_f32", "v_mul_f32", "v_floor_f32",
            "v_mad_u64_u32"}


MEMBERSHIP = {}   # measured: {mnemonic: {counter: count per instruction}} (load_membership)
_CLASS_COUNTERS = ("SQ_INSTS_VALU", "SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_INT64", "SQ_INSTS_VALU_CVT",
                   "SQ_INSTS_VALU_ADD_F32", "SQ_INSTS_VALU_MUL_F32", "SQ_INSTS_VALU_FMA_F32")


def load_membership(cal3, cal4, log):
    """Per-opcode counter membership from tools/ab/pmc_cal.hip's kop<OP> kernels
    (REP copies of one opcode each): (counter - the smallest value of that
    counter over all opcodes) / waves / REP; SQ_INSTS_VALU per opcode is its own
    count per op (2 for v_permlane32_swap)."""
    meta = json.loads(next(line for line in open(log) if line.startswith("{") and '"ops"' in line))
    ops, rep, waves = meta["ops"], meta["rep"], meta["waves_per_variant"]
    per = collections.defaultdict(dict)
    for d in (cal3, cal4):
        for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(p)):
                mm = re.search(r"kop<(\d+)>", r["Kernel_Name"])
                if mm:
                    per[int(mm.group(1))][r["Counter_Name"]] = float(r["Counter_Value"])
    cnts = {c for k in per for c in per[k]}
    base = {c: min(per[k][c] for k in per if c in per[k]) for c in cnts}
    out = {}
    for k, op in enumerate(ops):
        if k not in per or not re.match(r"^v_[a-z0-9_]+$", op) or op.endswith(("_vamt", "_rot", "_vcc", "_init", "_s", "_vv")):
            continue
        e = {c: round((per[k][c] - (0.0 if c == "SQ_INSTS_VALU" else base[c])) / waves / rep) for c in per[k]
             if c in _CLASS_COUNTERS}
        if "SQ_INSTS_VALU" in e:
            e["SQ_INSTS_VALU"] = round((per[k]["SQ_INSTS_VALU"] - base["SQ_INSTS_VALU"]) / waves / rep + 1)
        out[vm.base_mnemonic(op)] = e
        if op == "v_permlane32_swap":   # the probe's name for v_permlane32_swap_b32
            out["v_permlane32_swap_b32"] = e
    MEMBERSHIP.clear()
    MEMBERSHIP.update(out)
    return out


def membership(m: str, counter: str):
    """(known, unknown) contribution of one instruction to one counter."""
    b = vm.base_mnemonic(m)
    if b in MEMBERSHIP and counter in MEMBERSHIP[b]:
        return (MEMBERSHIP[b][counter], 0)
    if counter == "SQ_INSTS_VALU":
        return (1, 0) if m.startswith("v_") else (0, 0)
    if counter == "SQ_INSTS_MFMA":
        return (1, 0) if re.match(r"^v_(mfma|smfmac)", m) else (0, 0)
    if counter == "SQ_INSTS_LDS":
        if m.startswith("ds_"):
            return (1, 0)
        return (0, 1) if re.match(r"^(global|buffer)_load_lds", m) else (0, 0)
    if counter == "SQ_INSTS_SMEM":
        if re.match(r"^s_(load|buffer_load)", m):
            return (1, 0)
        return (0, 1) if re.match(r"^s_(memtime|memrealtime|dcache)", m) else (0, 0)
    if counter == "SQ_INSTS_BRANCH":
        if re.match(r"^s_(branch|cbranch)", m):
            return (1, 0)
        return (0, 1) if re.match(r"^s_(setpc|swappc)", m) else (0, 0)
    if counter == "SQ_INSTS_SALU":
        if not m.startswith("s_"):
            return (0, 0)
        if _SALU_UNKNOWN.match(m):
            return (0, 1)
        return (0, 0) if _SALU_NOT.match(m) else (1, 0)
    if counter in ("SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR"):
        if re.match(r"^(global|buffer|flat|scratch)_atomic", m):
            return (0, 1)
        rd = re.match(r"^(global|buffer|flat|scratch)_load", m)
        wr = re.match(r"^(global|buffer|flat|scratch)_store", m)
        return (1, 0) if (rd if counter.endswith("RD") else wr) else (0, 0)
    if not m.startswith("v_"):
        return (0, 0)
    if counter == "SQ_INSTS_VALU_INT32":
        if b in INT32_YES:
            return (1, 0)
        return (0, 0) if b in INT32_NO or re.match(r"^v_(mfma|smfmac|accvgpr|pk_)", b) else (0, 1)
    if counter == "SQ_INSTS_VALU_INT64":
        if b == "v_mad_u64_u32":
            return (1, 0)
        return (0, 1) if re.search(r"(64|i64|u64)", b) and b != "v_lshlrev_b64" else (0, 0)
    if counter == "SQ_INSTS_VALU_CVT":
        if b in ("v_cvt_f32_i32", "v_cvt_rpi_i32_f32"):
            return (1, 0)
        return (0, 1) if b.startswith("v_cvt") else (0, 0)
    for cn, op in (("SQ_INSTS_VALU_ADD_F32", "v_add_f32"), ("SQ_INSTS_VALU_MUL_F32", "v_mul_f32"),
                   ("SQ_INSTS_VALU_FMA_F32", "v_fma_f32")):
        if counter == cn:
            if b == op:
                return (1, 0)
            return (0, 1) if re.search(r"_f32$", b) and not b.startswith("v_cvt") and b != "v_floor_f32" else (0, 0)
    return (0, 0)


# ---- disassembly -> basic blocks
_LINE = re.compile(r"^\s+([a-z_0-9]+)(.*?)//\s*([0-9A-F]+):")


def kernels_text(obj: str):
    txt = subprocess.run([vm.OBJDUMP, "-d", "--mcpu=gfx950", obj], check=True, capture_output=True, text=True).stdout
    out, cur, base = {}, None, 0
    for line in txt.splitlines():
        mm = re.match(r"^([0-9a-f]+) <(.+)>:$", line)
        if mm:
            cur = out.setdefault(mm.group(2), [])
            base = int(mm.group(1), 16)
            continue
        if cur is None:
            continue
        m = _LINE.match(line)
        if not m:
            continue
        mn, rest, addr = m.group(1), m.group(2), int(m.group(3), 16)
        tgt = None
        t = re.search(r"<(.+?)\+0x([0-9a-f]+)>", line)
        if t and mn.startswith(("s_branch", "s_cbranch")):
            tgt = ("sym", t.group(1), int(t.group(2), 16))
        cur.append((addr, mn, tgt))
    return out


def build_cfg(insts):
    """insts: [(addr, mnemonic, target)] of one kernel -> blocks [(start, [mn...], succs)]."""
    if not insts:
        return []
    base = insts[0][0]
    addrs = [a for a, _, _ in insts]
    idx = {a: i for i, a in enumerate(addrs)}
    leaders = {0}
    for i, (a, mn, tgt) in enumerate(insts):
        if mn.startswith(("s_branch", "s_cbranch")) and tgt:
            ta = base + tgt[2]
            if ta in idx:
                leaders.add(idx[ta])
            if i + 1 < len(insts):
                leaders.add(i + 1)
        elif mn.startswith(("s_endpgm", "s_setpc", "s_swappc")) and i + 1 < len(insts):
            leaders.add(i + 1)
    ls = sorted(leaders)
    blocks = []
    for k, s in enumerate(ls):
        e = ls[k + 1] if k + 1 < len(ls) else len(insts)
        body = insts[s:e]
        last = body[-1]
        succ = []
        mn = last[1]
        if mn.startswith("s_endpgm"):
            pass
        elif mn.startswith("s_branch") and last[2]:
            succ = [idx.get(base + last[2][2])]
        elif mn.startswith("s_cbranch") and last[2]:
            succ = [idx.get(base + last[2][2])] + ([e] if e < len(insts) else [])
        elif e < len(insts):
            succ = [e]
        blocks.append((s, [m for _, m, _ in body], [x for x in succ if x is not None]))
    start_to_block = {b[0]: j for j, b in enumerate(blocks)}
    return [(b[1], [start_to_block[x] for x in b[2]]) for b in blocks]


# ---- rates
def load_rates(path):
    rates = {}
    for line in open(path):
        if line.startswith("{"):
            d = json.loads(line)
            if d.get("waves_per_simd", 8) == 8 and d["op"] not in rates:
                rates[d["op"]] = d["chip_winst_per_s"]
    return rates


def price(m: str, rates):
    """(seconds per chip wave-instruction, measured?)"""
    b = vm.base_mnemonic(m)
    if re.match(r"^v_(mfma|smfmac)", b):
        return 4.0 / rates["v_add_u32"], False
    if b in rates:
        return 1.0 / rates[b], True
    if m in rates:
        return 1.0 / rates[m], True
    return 1.0 / rates.get(vm.rate_class(m), rates["v_add3_u32"]), False


# ---- measured counters
def load_counters(dirs):
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for d in dirs:
        for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(p)):
                if "nh::" not in r["Kernel_Name"] or "k_sse_i16" in r["Kernel_Name"]:
                    continue
                key = (r["Counter_Name"], r["Dispatch_Id"])
                tot[r["Kernel_Name"]][key] = float(r["Counter_Value"])
                disp[r["Kernel_Name"]].add(r["Dispatch_Id"])
    out = {}
    for k, d in tot.items():
        agg = collections.defaultdict(float)
        for (c, _), v in d.items():
            agg[c] += v
        out[k] = dict(agg)
    return out


def solve(blocks, meas, rates, tol=0.005):
    """LP bounds of the VALU issue time over every execution-count vector the CFG
    and the measured counters allow; returns a dict (None if infeasible)."""
    from scipy.optimize import linprog
    nb = len(blocks)
    edges = [(i, j) for i, (_, su) in enumerate(blocks) for j in su]
    exits = [i for i, (_, su) in enumerate(blocks) if not su]
    nv = len(edges) + len(exits)
    # block count x_b = sum of out-edges (+ exit); flow: in-edges (+ entry) = x_b
    Aeq, beq = [], []
    waves = meas.get("SQ_WAVES")
    out_of = collections.defaultdict(list)
    in_of = collections.defaultdict(list)
    for k, (i, j) in enumerate(edges):
        out_of[i].append(k)
        in_of[j].append(k)
    for k, i in enumerate(exits):
        out_of[i].append(len(edges) + k)
    for b in range(nb):
        row = np.zeros(nv)
        for k in out_of[b]:
            row[k] += 1
        for k in in_of[b]:
            row[k] -= 1
        Aeq.append(row)
        beq.append(waves if b == 0 else 0.0)
    # x_b as a linear map of the variables
    X = np.zeros((nb, nv))
    for b in range(nb):
        for k in out_of[b]:
            X[b, k] = 1
    Aub, bub = [], []
    used = []
    for c in COUNTERS:
        if c not in meas:
            continue
        known = np.array([sum(membership(m, c)[0] for m in blocks[b][0]) for b in range(nb)], float)
        unk = np.array([sum(membership(m, c)[1] for m in blocks[b][0]) for b in range(nb)], float)
        M = meas[c]
        slack = tol * M + 1.0
        Aub.append(known @ X)               # known part <= M + slack
        bub.append(M + slack)
        Aub.append(-((known + unk) @ X))    # known + unknown >= M - slack
        bub.append(-(M - slack))
        used.append(c)
    cost_b = np.zeros(nb)
    valu_b = np.zeros(nb)
    meas_b = np.zeros(nb)
    for b in range(nb):
        for m in blocks[b][0]:
            if m.startswith("v_"):
                t, ok = price(m, rates)
                cost_b[b] += t
                valu_b[b] += 1
                meas_b[b] += ok
    cvec = cost_b @ X
    res = {}
    for sense, sgn in (("min", 1.0), ("max", -1.0)):
        r = linprog(sgn * cvec, A_ub=np.array(Aub), b_ub=np.array(bub), A_eq=np.array(Aeq), b_eq=np.array(beq),
                    bounds=(0, None), method="highs")
        if r.status != 0:
            return {"feasible": False, "status": r.message, "counters": used}
        xb = X @ r.x
        res[sense] = {"T_s": float(cost_b @ xb), "valu": float(valu_b @ xb), "valu_priced_measured": float(meas_b @ xb)}
    return {"feasible": True, "counters": used, "tol": tol, **res}


_TEXT = None


def _kernel_text():
    global _TEXT
    if _TEXT is None:
        srcs = sorted(glob.glob(os.path.join(vm.CSRC, "*.hip")))
        with tempfile.TemporaryDirectory() as tmp:
            objs = vm.compile_objects(tmp, srcs)
            text = {}
            for o in objs:
                text.update(kernels_text(o))
        dm = vm.demangle(list(text))
        _TEXT = {dm.get(s, s): text[s] for s in text}
    return _TEXT


def run_config(pmc_dirs, rates_path, tol=0.005):
    """{demangled kernel: LP result} for one config's counter directories."""
    rates = load_rates(rates_path)
    meas = load_counters(pmc_dirs)
    text = _kernel_text()
    out = {}
    for kname, m in meas.items():
        if kname not in text or not m.get("SQ_WAVES") or not m.get("SQ_INSTS_VALU"):
            continue
        cfg = build_cfg(text[kname])
        r = solve(cfg, m, rates, tol)
        t = tol
        while not r["feasible"] and t < 0.04:
            # counters from separate passes disagree beyond tol when a kernel's work varies run to run
            # (the closed loops' spin waits on the row above): widen, and record the tolerance used
            t *= 2
            r = solve(cfg, m, rates, t)
        if r["feasible"]:
            r["attainable_lo"] = m["SQ_INSTS_VALU"] / r["max"]["T_s"]
            r["attainable_hi"] = m["SQ_INSTS_VALU"] / r["min"]["T_s"]
            r["valu_priced_measured_frac"] = r["min"]["valu_priced_measured"] / max(1.0, r["min"]["valu"])
        out[kname] = r
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rates", required=True)
    ap.add_argument("--pmc", nargs="+", required=True, help="rocprofv3 --pmc output dirs of ONE config")
    ap.add_argument("--kernels", default="nh::")
    ap.add_argument("--tol", type=float, default=0.005)
    ap.add_argument("--cal", nargs=3, default=None, metavar=("CAL3", "CAL4", "LOG"),
                    help="tools/ab/_pmc_cal outputs: the measured counter membership of every probe opcode")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    rates = load_rates(a.rates)
    if a.cal:
        load_membership(*a.cal)
    meas = load_counters(a.pmc)
    srcs = sorted(glob.glob(os.path.join(vm.CSRC, "*.hip")))
    with tempfile.TemporaryDirectory() as tmp:
        objs = vm.compile_objects(tmp, srcs)
        text = {}
        for o in objs:
            text.update(kernels_text(o))
    dm = vm.demangle(list(text))
    by_name = {dm.get(s, s): s for s in text}
    out = {"rates": a.rates, "pmc": a.pmc, "kernels": {}}
    N_tot, Tmin_tot, Tmax_tot, ok = 0.0, 0.0, 0.0, True
    for kname, m in sorted(meas.items()):
        sym = by_name.get(kname)
        if sym is None or not m.get("SQ_WAVES") or not m.get("SQ_INSTS_VALU"):
            continue
        blocks = build_cfg(text[sym])
        r = solve(blocks, m, rates, a.tol)
        static = collections.Counter(mn for body, _ in blocks for mn in body)
        r["blocks"] = len(blocks)
        r["SQ_INSTS_VALU"] = m["SQ_INSTS_VALU"]
        r["SQ_WAVES"] = m["SQ_WAVES"]
        if r["feasible"]:
            N = m["SQ_INSTS_VALU"]
            r["attainable_lo"] = N / r["max"]["T_s"]
            r["attainable_hi"] = N / r["min"]["T_s"]
            r["valu_priced_measured_frac"] = r["min"]["valu_priced_measured"] / max(1.0, r["min"]["valu"])
            N_tot += N
            Tmin_tot += r["min"]["T_s"]
            Tmax_tot += r["max"]["T_s"]
        else:
            ok = False
        st = vm.summarize(kname, static, {k: {"chip_winst_per_s": v} for k, v in rates.items()})
        r["attainable_static"] = st.get("attainable_valu_winst_per_s")
        out["kernels"][kname] = r
        print(json.dumps({"kernel": kname[:70], **{k: r.get(k) for k in ("feasible", "blocks", "attainable_lo",
                                                                          "attainable_hi", "attainable_static")}}))
    if N_tot and ok:
        out["config"] = {"valu": N_tot, "attainable_lo": N_tot / Tmax_tot, "attainable_hi": N_tot / Tmin_tot}
        print(json.dumps(out["config"]))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())

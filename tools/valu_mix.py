#!/usr/bin/env python3
"""Static instruction mix of the product kernels, and their attainable VALU rate.

    python tools/valu_mix.py [--rates profiles/r05/valu/valu_rate_r05w.jsonl] [--json out.json] [--kernels REGEX]

1. Compiles every nano-hevc_amd/csrc/*.hip for gfx950 with the product flags
   (device code only, unbundled ELF) and disassembles it (llvm-objdump).
2. Splits the text per kernel symbol and counts instructions per mnemonic and
   per unit: VALU (v_*, without MFMA / AccVGPR moves), MFMA, ACC (v_accvgpr_*),
   SALU, SMEM, VMEM (global_/buffer_/flat_), LDS (ds_), branch / wait / misc.
3. With --rates (tools/ab/valu_rate.hip output, one JSON line per measured
   opcode: chip-wide wave-instructions per second at 8 waves/SIMD), prices every
   VALU mnemonic by its measured opcode (RATE_CLASS below maps the rest onto a
   measured opcode of the same issue class) and gives the kernel's ATTAINABLE
   VALU rate = N_valu / sum_i(n_i / r_i): the wave-instructions per second the
   chip can issue for that static mix.  That rate, not a 4-cycles-per-op
   guess, is the roofline peak of a VALU-bound kernel.

Static counts weight every instruction once; loops weight their body by the
trip count at run time.  The dynamic count comes from SQ_INSTS_VALU (PMC), the
mix from here: the two agree to the extent the hot loop's mix is the kernel's.
"""
from __future__ import annotations

import argparse
import collections
import glob
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "nano-hevc_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "--cuda-device-only", "--no-gpu-bundle-output"]

# VALU mnemonic (regex, first match wins) -> the measured opcode whose rate it takes,
# for the (few) mnemonics tools/ab/valu_rate.hip does not measure itself.  The
# round-4 probe (interleaved rounds, SIMD cycles per instruction from s_memtime
# spans per SIMD) splits gfx950's VALU into a 2-cycle class (32-bit add / sub /
# logic / lshrrev / ashrrev / mov, f32 add / mul / fma, non-packed 16-bit add /
# sub / mul / shifts, bitop3, accvgpr moves: ~0.93-1.02 T wave-instr/s) and a
# 4-cycle class (everything else: packed 16-bit, dot2, 24-bit multiplies, cmp,
# cndmask, perm, bfe / bfi, 3-input ops, min / max, lshlrev_b32, cvt, 64-bit
# ops: ~0.52-0.58 T/s), plus 8-cycle transcendentals.
RATE_CLASS = [
    (r"^v_dot2", "v_dot2c_i32_i16"),
    (r"^v_(mad|mul)_(i32_i24|u32_u24)$", "v_mad_i32_i24"),
    (r"^v_mul_(lo|hi)_(u32|i32)$|^v_mad_(u64_u32|i64_i32)$|^v_mul_hi_(i32|u32)_(i24|u24)$", "v_mul_lo_u32"),
    (r"^v_pk_(mad|mul|fma)", "v_pk_mad_u16"),
    (r"^v_pk_", "v_pk_add_u16"),
    (r"^v_(lshlrev|lshrrev|ashrrev)_(b|i)64$|^v_lshl_add_u64$|^v_(add|sub)_(co|u64)|^v_mov_b64", "v_lshlrev_b64"),
    (r"^v_cmp|^v_cmpx", "v_cmp_gt_i32"),
    (r"^v_cndmask", "v_cndmask_b32"),
    (r"^v_perm", "v_perm_b32"),
    (r"^v_bfe|^v_bfi|^v_alignbit|^v_alignbyte", "v_bfe_i32"),
    (r"^v_(add3|lshl_add|add_lshl|lshl_or|and_or|or3|xad|xor3|mad_u32_u16|max3|min3|med3)", "v_add3_u32"),
    (r"^v_readfirstlane|^v_readlane|^v_writelane", "v_readfirstlane_b32"),
    (r"^v_permlane", "v_permlane32_swap"),
    (r"^v_(rcp|rsq|sqrt|exp|log|sin|cos)_", "v_rcp_iflag_f32"),
    (r"^v_(add|sub|subrev|mul|fma|mac)_f32$", "v_add_f32"),
    (r"^v_(max|min)_f32|^v_floor|^v_cvt|^v_rndne|^v_trunc|^v_fract", "v_floor_f32"),
    (r"^v_(add|sub|subrev|and|or|xor|not)_(u32|b32)$|^v_(lshrrev_b32|ashrrev_i32)$", "v_add_u32"),
    (r"^v_(add|sub|mul_lo|lshlrev|lshrrev)_(u16|b16)$", "v_add_u16"),
    (r"^v_accvgpr", "v_accvgpr_read_b32"),
    (r"^v_mov", "v_mov_b32"),
    (r"^v_", "v_add3_u32"),   # unmeasured: priced at the 4-cycle class, not the 2-cycle one
]

UNIT_RULES = [
    ("MFMA", r"^v_mfma|^v_smfmac"),
    ("ACC", r"^v_accvgpr"),
    ("VALU", r"^v_"),
    ("LDS", r"^ds_"),
    ("VMEM", r"^(global|buffer|flat|scratch)_"),
    ("SMEM", r"^s_(load|buffer_load|store|dcache|memtime|memrealtime)"),
    ("BRANCH", r"^s_(branch|cbranch|setpc|swappc|getpc|call)"),
    ("WAIT", r"^s_(waitcnt|barrier|sleep|nop|endpgm|setprio|sethalt|trap|wait_idle|icache|sendmsg)"),
    ("SALU", r"^s_"),
]


def base_mnemonic(m: str) -> str:
    """v_mul_i32_i24_e32 -> v_mul_i32_i24 (encoding suffixes do not change the issue class)."""
    return re.sub(r"_(e32|e64|sdwa|dpp)$", "", m)


def rate_class(m: str) -> str:
    m = base_mnemonic(m)
    for pat, cls in RATE_CLASS:
        if re.search(pat, m):
            return cls
    return "v_add3_u32"


def unit_of(m: str) -> str:
    for u, pat in UNIT_RULES:
        if re.search(pat, m):
            return u
    return "OTHER"


def compile_objects(outdir: str, sources):
    objs = []
    for src in sources:
        obj = os.path.join(outdir, os.path.basename(src).replace(".hip", ".co"))
        subprocess.run([HIPCC] + FLAGS + ["-c", src, "-o", obj], check=True)
        objs.append(obj)
    return objs


def kernels_of(obj: str):
    """{symbol: Counter(mnemonic)} for every function in the code object."""
    txt = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", obj], check=True, capture_output=True, text=True).stdout
    out, cur = {}, None
    for line in txt.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            cur = out.setdefault(m.group(1), collections.Counter())
            continue
        if cur is None:
            continue
        s = line.strip()
        if not s or s.startswith(";") or s.endswith(":"):
            continue
        mn = s.split()[0]
        if re.match(r"^[a-z_0-9]+$", mn) and (mn.startswith(("v_", "s_", "ds_", "global_", "buffer_", "flat_", "scratch_"))):
            cur[mn] += 1
    return out


def demangle(names):
    try:
        r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True, check=True)
        return dict(zip(names, r.stdout.splitlines()))
    except Exception:
        return {n: n for n in names}


def load_rates(path):
    rates = {}
    for line in open(path):
        line = line.strip()
        if line.startswith("{"):
            d = json.loads(line)
            if d.get("waves_per_simd", 8) == 8 and d["op"] not in rates:   # the all-opcode block at 8 waves/SIMD
                rates[d["op"]] = d
    return rates


def summarize(sym, cnt, rates):
    units = collections.Counter()
    valu = collections.Counter()
    for m, n in cnt.items():
        u = unit_of(m)
        units[u] += n
        if u == "VALU":
            valu[m] += n
    nv = sum(valu.values())
    res = {"kernel": sym, "units": dict(units), "valu_static": nv}
    by_class = collections.Counter()
    for m, n in valu.items():   # a measured opcode prices itself; the rest take their class's measured opcode
        b = base_mnemonic(m)
        by_class[b if rates and b in rates else rate_class(m)] += n
    res["valu_by_rate_class"] = dict(by_class.most_common())
    res["valu_top"] = dict(valu.most_common(25))
    if rates and nv:
        missing = [c for c in by_class if c not in rates]
        t = 0.0
        for c, n in by_class.items():
            r = rates.get(c, rates.get("v_add3_u32", rates.get("v_add_u32")))
            t += n / r["chip_winst_per_s"]
        att = nv / t
        res["attainable_valu_winst_per_s"] = att
        # the same per SIMD and clock cycle at the nominal 2.4 GHz (1,024 SIMDs)
        res["attainable_per_simd_cycle_2p4GHz"] = att / (1024 * 2.4e9)
        res["rate_classes_unmeasured"] = missing
        full = rates.get("v_add_u32")
        if full:
            res["attainable_vs_plain_32bit"] = att / full["chip_winst_per_s"]
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rates", default=None, help="valu_rate.jsonl (chip-wide wave-instr/s per opcode)")
    ap.add_argument("--kernels", default=r"k_ctu_open|k_tc32_h|k_tc32_mfma|k_intra_rdo8|k_tu_closed|k_fwd8x8_quant",
                    help="regex over demangled kernel names")
    ap.add_argument("--sources", default=None, help="comma-separated csrc files (default: all)")
    ap.add_argument("--json", default=None)
    ap.add_argument("--objdir", default=None, help="keep the device objects here")
    a = ap.parse_args()
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    if a.sources:
        srcs = [os.path.join(CSRC, s) for s in a.sources.split(",")]
    rates = load_rates(a.rates) if a.rates else None
    with tempfile.TemporaryDirectory() as tmp:
        od = a.objdir or tmp
        os.makedirs(od, exist_ok=True)
        objs = compile_objects(od, srcs)
        allk = {}
        for o in objs:
            for sym, cnt in kernels_of(o).items():
                allk[sym] = (os.path.basename(o), cnt)
    dm = demangle(list(allk))
    out = []
    for sym, (obj, cnt) in sorted(allk.items()):
        name = dm.get(sym, sym)
        if not re.search(a.kernels, name):
            continue
        r = summarize(name, cnt, rates)
        r["object"] = obj
        out.append(r)
        print(json.dumps(r), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())

#!/usr/bin/env python3
"""Mechanical checks of hand-counted hardware assumptions in the SHIPPED code
object (nano-hevc_amd/nano_hevc/libnanohevc.so), run on the CPU.

    python tools/isa_check.py [--lib PATH] [--narrow N] [--wide N]

1. k_tc32_hd<2> (nh_ctu.hip, config 5) retires block k's LDS-DMA image with a
   hand-counted `s_waitcnt vmcnt(4 + stores of block k-1)` (kTc32hdStoresNarrow /
   kTc32hdStoresWide).  That is only right if the compiler emits exactly that many
   VMEM instructions between the DMA bursts.  `check_dma_waits` runs the kernel's
   control-flow graph as an explicit-state model of the in-order vmcnt queue:
   every VMEM instruction enters the queue (LDS-DMA loads tagged with their
   burst: the 4 loads of one issue() call), every `s_waitcnt vmcnt(n)` retires
   the oldest until n remain, the scalar register holding `prev` and the SCC /
   VCC tests of the kernel's uniform decisions are evaluated (constant
   propagation over the SALU lane-mask booleans), SCC / VCC tests on unknown
   values are explored both ways.  Forward exec-mask branches are taken as "some
   lane is active": the kernel's wave-uniform decisions are scalar branches (its
   wave index is read into an SGPR), so an exec-masked region is a lane subset
   (lane < 4 / < 32 / == 0) that always holds for some lane of a full wave;
   only after a loop's exit masking (s_andn2_b64 exec, exec, x) may exec be
   empty, and exec branches there are explored both ways.  At the w-th block wait it requires that burst w-1 (the block about to
   be read) has fully retired (SAFETY) and that the wait retired nothing issued
   after it (TIGHT: the count equals the VMEM instructions really issued since).
   Any other VMEM instruction, scratch use or call in the loop fails the check.
2. `check_mfma_hazard`: every v_cvt_rpi/flr_i32_f32 (inline asm, invisible to the
   compiler's hazard recognizer) whose source register was last written by an
   MFMA has the mfma_result_ready s_nop run (>= 24 wait states, nh_f16mma.hpp)
   between the MFMA and itself.
3. `check_no_scratch`: the kernels use no private segment (scratch).

tests/test_isa_checks.py runs all three on the built library (and shows that
a miscounted constant is caught).
"""
from __future__ import annotations

import argparse
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "nano-hevc_amd", "nano_hevc", "libnanohevc.so")
LLVM = "/opt/rocm/lib/llvm/bin"
TRIPLE = "hipv4-amdgcn-amd-amdhsa--gfx950"
TC32HD = "_ZN2nh9k_tc32_hdILi2EiLb1ELi4ELb0EEEvNS_7CtuArgsEi"   # k_tc32_hd<2, int32_t, ILV, 4, !NT>: int32 levels
# the three level types and the store instructions a narrow block issues (4 / 2 / 1 level rows + 2 recon)
TC32HD_LEVELS = {"int32": (TC32HD, 6), "int16": ("_ZN2nh9k_tc32_hdILi2EsLb1ELi4ELb0EEEvNS_7CtuArgsEi", 4),
                 "int8": ("_ZN2nh9k_tc32_hdILi2EaLb1ELi4ELb0EEEvNS_7CtuArgsEi", 3)}


# ---------------------------------------------------------------------------
# code object extraction and parsing
# ---------------------------------------------------------------------------
def code_objects(lib: str, workdir: str) -> list[str]:
    """The gfx950 code objects of every HIP translation unit linked into lib."""
    fb = os.path.join(workdir, "fatbin.bin")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", lib, os.path.join(workdir, "x.o")],
                   check=True, capture_output=True)
    data = open(fb, "rb").read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    starts = [m.start() for m in re.finditer(re.escape(magic), data)]
    out = []
    for i, s in enumerate(starts):
        e = starts[i + 1] if i + 1 < len(starts) else len(data)
        b = os.path.join(workdir, f"b{i}.bin")
        co = os.path.join(workdir, f"b{i}.co")
        open(b, "wb").write(data[s:e])
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o", f"--input={b}", f"--targets={TRIPLE}",
                        f"--output={co}", "--unbundle"], check=True, capture_output=True)
        out.append(co)
    return out


class Insn:
    __slots__ = ("addr", "mn", "ops", "target")

    def __init__(self, addr, mn, ops, target):
        self.addr, self.mn, self.ops, self.target = addr, mn, ops, target

    def __repr__(self):
        return f"{self.addr:x}: {self.mn} {self.ops}"


_LINE = re.compile(r"^\s+([a-z_0-9]+)\s*(.*?)\s*//\s*([0-9A-Fa-f]+):")
_TGT = re.compile(r"<([^>+]+)\+0x([0-9a-f]+)>")


def disassemble(co: str) -> dict[str, list[Insn]]:
    txt = subprocess.run([f"{LLVM}/llvm-objdump", "-d", co], check=True, capture_output=True, text=True).stdout
    funcs, cur, name = {}, None, None
    for line in txt.splitlines():
        m = re.match(r"^([0-9a-f]+) <(.+)>:$", line)
        if m:
            name, cur = m.group(2), []
            funcs[name] = cur
            continue
        if cur is None:
            continue
        m = _LINE.match(line)
        if not m:
            continue
        mn, ops, addr = m.group(1), m.group(2), int(m.group(3), 16)
        t = _TGT.search(line)
        target = None
        if t and mn.startswith("s_") and ("branch" in mn):
            target = ("+", t.group(1), int(t.group(2), 16))
        cur.append(Insn(addr, mn, ops, target))
    for name, ins in funcs.items():   # resolve branch targets to absolute addresses
        base = ins[0].addr if ins else 0
        for i in ins:
            if i.target:
                i.target = base + i.target[2]
    return funcs


def kernel_metadata(co: str) -> str:
    return subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True, text=True).stdout


def compile_device(src: str, out: str, defines=()) -> str:
    """Device-only gfx950 ELF of one source with the product flags (plus -D defines)."""
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "--cuda-device-only",
           "--no-gpu-bundle-output", "-c", src, "-o", out] + [f"-D{d}" for d in defines]
    subprocess.run(cmd, check=True, capture_output=True)
    return out


def load(lib: str = LIB):
    """({function name: instructions}, metadata text) over every code object of lib."""
    with tempfile.TemporaryDirectory() as d:
        funcs, meta = {}, ""
        for co in code_objects(lib, d):
            funcs.update(disassemble(co))
            meta += kernel_metadata(co)
    return funcs, meta


# ---------------------------------------------------------------------------
# 1. the vmcnt model of k_tc32_hd's LDS-DMA pipeline
# ---------------------------------------------------------------------------
_SREG = re.compile(r"^s(\d+)$")
_SPAIR = re.compile(r"^s\[(\d+):(\d+)\]$")


def _imm(tok: str):
    tok = tok.strip()
    try:
        return int(tok, 0)
    except ValueError:
        return None


def _ops(ins: Insn) -> list[str]:
    return [o.strip() for o in ins.ops.split(",")] if ins.ops else []


def _sgpr_writes(ins: Insn) -> list[str]:
    """Scalar destinations of an instruction (conservative: the first operand of
    any SALU / readlane / v_cmp-with-sgpr-dst instruction)."""
    mn = ins.mn
    ops = _ops(ins)
    if not ops:
        return []
    if mn.startswith(("s_cmp", "s_bitcmp", "s_cbranch", "s_branch", "s_waitcnt", "s_nop", "s_barrier", "s_setprio",
                      "s_sleep", "s_endpgm", "s_dcache", "s_icache", "s_sethalt", "s_trap", "s_setreg",
                      "s_store", "s_buffer_store", "s_atomic")):
        return []
    if mn.startswith("s_") or mn.startswith(("v_readfirstlane", "v_readlane", "v_cmp", "v_cmpx", "v_div_scale",
                                            "v_add_co", "v_sub_co", "v_addc", "v_subb", "v_mad_u64", "v_mad_i64")):
        d = [ops[0]]
        if mn.startswith(("v_add_co", "v_sub_co", "v_addc", "v_subb", "v_mad_u64", "v_mad_i64", "v_div_scale")) \
                and len(ops) > 1:
            d.append(ops[1])
        return d
    return []


def _regs(tok: str) -> list[str]:
    m = _SREG.match(tok)
    if m:
        return [f"s{m.group(1)}"]
    m = _SPAIR.match(tok)
    if m:
        return [f"s{i}" for i in range(int(m.group(1)), int(m.group(2)) + 1)]
    if tok in ("vcc", "vcc_lo", "vcc_hi"):
        return ["vcc"]
    if tok.startswith("exec"):
        return ["exec"]
    if tok == "scc":
        return ["scc"]
    return []


def _vmcnt(ins: Insn):
    m = re.search(r"vmcnt\((\d+)\)", ins.ops)
    return int(m.group(1)) if m else None


def _vmem_kind(mn: str):
    if mn.startswith(("global_", "buffer_", "flat_", "scratch_")):
        if "load_lds" in mn:
            return "D"
        if "store" in mn or "atomic" in mn:
            return "S"
        return "L"
    return None


class DmaModelError(AssertionError):
    pass


def _fail(msg, hist):
    raise DmaModelError(msg + ("\n  path: " + "\n  ".join(hist) if hist else ""))


def _salu(i: Insn, cd: dict, scc, vcc, tracked: set):
    """Constant propagation over the SALU instructions that carry the kernel's
    uniform decisions: 32-bit moves of immediates, and 64-bit lane-mask booleans
    (0 / -1) built by s_mov / s_cselect / s_and / s_or / s_xor / s_andn2 / s_not
    (exec counts as -1: inside any region the wave runs, some lane is active).
    Returns the new (scc, vcc); cd is updated in place."""
    mn, ops = i.mn, _ops(i)
    if ops and ops[0] == "exec":   # exec may be empty only after a loop's exit masking (s_andn2_b64 exec, exec, x)
        if mn == "s_andn2_b64" and ops[1] == "exec":
            cd["execmz"] = True
        else:
            cd.pop("execmz", None)
    elif mn.endswith("saveexec_b64"):
        cd.pop("execmz", None)

    def get64(tok):
        if tok.startswith("exec"):
            return -1
        if tok == "vcc":
            return {"zero": 0, "nz": -1}.get(vcc)
        v = _imm(tok)
        if v is not None:
            return -1 if v == -1 else 0 if v == 0 else None
        rs = _regs(tok)
        vals = [cd.get(r) for r in rs]
        return vals[0] if rs and None not in vals and len(set(vals)) == 1 else None

    def put64(tok, v):
        nonlocal vcc
        if tok == "vcc":
            vcc = None if v is None else ("zero" if v == 0 else "nz")
            return
        for r in _regs(tok):
            if v is None:
                cd.pop(r, None)
            else:
                cd[r] = v

    if mn in ("s_mov_b32", "s_movk_i32") and ops and _SREG.match(ops[0]):
        v = _imm(ops[1])
        if v is None:
            cd.pop(ops[0], None)
        else:
            cd[ops[0]] = v
        return scc, vcc
    if mn.endswith("_b64") and mn.startswith(("s_mov_", "s_cselect_", "s_and_", "s_or_", "s_xor_", "s_andn2_",
                                               "s_orn2_", "s_not_")) and not mn.endswith("saveexec_b64"):
        d = ops[0]
        a = [get64(o) for o in ops[1:]]
        op = mn[2:].split("_")[0]
        v = None
        if op == "mov":
            v = a[0]
        elif op == "cselect":
            v = None if scc is None else (a[0] if scc else a[1])
        elif op == "not":
            v = None if a[0] is None else ~a[0]
        elif None not in a:
            x, y = a
            v = {"and": x & y, "or": x | y, "xor": x ^ y, "andn2": x & ~y, "orn2": x | ~y}[op]
        if op in ("and", "andn2") and v is None and 0 in a[:1] + (a[1:] if op == "and" else []):
            v = 0
        if not d.startswith("exec"):
            put64(d, v)
        if op != "mov":
            scc = None if v is None else v != 0
        return scc, vcc
    for dst in _sgpr_writes(i):
        for r in _regs(dst):
            if r == "vcc":
                vcc = None
            cd.pop(r, None)
    if mn.startswith("v_cmp") and ops[:1] == ["vcc"]:
        vcc = None
    if mn.startswith("s_") and not mn.startswith(("s_nop", "s_waitcnt", "s_barrier", "s_setprio", "s_mov_b32",
                                                  "s_movk_i32")):
        scc = None   # SALU arithmetic / logic rewrites SCC
    return scc, vcc


def check_dma_waits(ins: list[Insn], max_waits: int = 5, max_states: int = 200000, trace: bool = False) -> dict:
    """Explore every path of the kernel through `max_waits` block waits (see the
    module docstring).  Returns a summary; raises DmaModelError on a violation."""
    by_addr = {i.addr: k for k, i in enumerate(ins)}
    for i in ins:
        if i.mn.startswith(("s_swappc", "s_setpc", "s_call")):
            raise DmaModelError(f"call in the kernel: {i}")
        if i.mn.startswith(("scratch_", "buffer_")):
            raise DmaModelError(f"scratch / buffer access: {i}")
    # registers whose constant values decide branches: those compared with an immediate
    tracked = set()
    for i in ins:
        if i.mn.startswith("s_cmp"):
            for o in _ops(i):
                tracked.update(r for r in _regs(o) if r.startswith("s"))
        if i.mn.endswith("_b64") and i.mn.startswith(("s_and", "s_or", "s_xor", "s_cselect", "s_mov", "s_not")):
            for o in _ops(i):
                tracked.update(r for r in _regs(o) if r.startswith("s"))
    summary = {"block_waits": 0, "wait_imms": set(), "paths_cut": 0, "stores_per_segment": set(), "states": 0}

    # state: (pc index, queue of (kind, burst), consts (frozenset), scc, vcc, waits, bursts issued,
    #         in_burst, stores since the last block wait)
    start = (0, (), frozenset(), None, None, 0, 0, False, 0, ())
    stack, seen = [start], set()
    while stack:
        st = stack.pop()
        pc, q, consts, scc, vcc, w, nb, inb, nst, hist = st
        if trace and (i_ := ins[pc]).mn.startswith(('s_cbranch', 's_branch', 's_waitcnt', 'global', 's_cmp', 's_mov_b32')):
            hist = (hist + (f"{i_!r} scc={scc} vcc={vcc}",))[-400:]
        key = (pc, tuple((k, b - w if b is not None else None) for k, b in q), consts, scc, vcc, min(w, 1),
               nb - w, inb, nst)
        if key in seen:
            continue
        seen.add(key)
        summary["states"] += 1
        if summary["states"] > max_states:
            raise DmaModelError("state space too large: the kernel's structure changed; revisit tools/isa_check.py")
        if pc >= len(ins):
            raise DmaModelError("fell off the end of the kernel")
        i = ins[pc]
        mn = i.mn
        cd = dict(consts)
        nxt = [pc + 1]
        kind = _vmem_kind(mn)
        if kind:
            if kind == "D":
                if not inb:
                    nb += 1
                q = q + (("D", nb - 1),)
                inb = True
            else:
                if nb > 0 and kind == "L":
                    raise DmaModelError(f"a VMEM load into registers after the LDS-DMA started: {i}")
                q = q + ((kind, None),)
                inb = False
                if kind == "S":
                    nst += 1
        elif mn == "s_waitcnt":
            n = _vmcnt(i)
            inb = False
            if n is not None:
                if nb > 0:   # a block wait: retires block w's burst
                    cur = w
                    last = max((k for k, (t, b) in enumerate(q) if t == "D" and b <= cur), default=None)
                    if last is not None and len(q) - last - 1 != n:
                        rest = [t for t, _ in q[last + 1:]]
                        if len(q) - last - 1 < n:
                            _fail(
                                f"UNSAFE wait at {i}: block {cur}'s DMA not retired (vmcnt({n}), only "
                                f"{len(q) - last - 1} VMEM ops issued after it: {rest})", hist)
                        _fail(
                            f"LOOSE wait at {i}: vmcnt({n}) but {len(q) - last - 1} VMEM ops issued after block "
                            f"{cur}'s DMA ({rest}): the hand count does not match the code", hist)
                    summary["block_waits"] += 1
                    summary["wait_imms"].add(n)
                    if w > 0:
                        summary["stores_per_segment"].add(nst)
                    nst = 0
                    w += 1
                while len(q) > n:
                    q = q[1:]
                if any(t == "D" and b < w for t, b in q):
                    raise DmaModelError(f"block {w - 1}'s DMA outstanding after {i}")
        elif mn.startswith("ds_"):
            inb = False
        elif mn == "s_endpgm":
            continue
        elif mn == "s_branch":
            nxt = [by_addr[i.target]]
        elif mn.startswith("s_cbranch"):
            cond = mn[len("s_cbranch_"):]
            tgt = by_addr[i.target]
            mz = cd.get("execmz", False)
            val = {"scc0": None if scc is None else not scc, "scc1": scc,
                   "vccz": None if vcc is None else vcc == "zero", "vccnz": None if vcc is None else vcc == "nz",
                   # some lane is active (lane-subset regions), except after a loop's exit masking
                   "execz": None if mz else False, "execnz": None if mz else True}[cond]
            nxt = [tgt] if val is True else [pc + 1] if val is False else [tgt, pc + 1]
            if val is None and cond.startswith(("vcc", "scc")):   # remember the outcome on each side
                for n2, taken in ((tgt, True), (pc + 1, False)):
                    truth = taken if cond in ("scc1", "vccz") else not taken
                    v_scc = truth if cond.startswith("scc") else scc
                    v_vcc = ("zero" if truth else "nz") if cond.startswith("vcc") else vcc
                    stack.append((n2, q, frozenset((k, v) for k, v in cd.items() if k in tracked or k == "execmz"), v_scc, v_vcc,
                                  w, nb, inb, nst, hist))
                continue
        elif mn.startswith("s_cmp_"):
            a, b = _ops(i)[:2]
            av = cd.get(a, _imm(a))
            bv = cd.get(b, _imm(b))
            if av is None or bv is None:
                scc = None
            else:
                op = mn.split("_")[2]
                signed = mn.endswith("i32")
                if not signed:
                    av, bv = av & 0xffffffff, bv & 0xffffffff
                scc = {"gt": av > bv, "ge": av >= bv, "lt": av < bv, "le": av <= bv, "eq": av == bv,
                       "lg": av != bv}[op]
        if not mn.startswith(("s_cmp_", "s_cbranch", "s_branch")) and kind is None:
            scc, vcc = _salu(i, cd, scc, vcc, tracked)
        cst = frozenset((k, v) for k, v in cd.items() if k in tracked or k == "execmz")
        if w > max_waits:
            summary["paths_cut"] += 1
            continue
        for n2 in nxt:
            stack.append((n2, q, cst, scc, vcc, w, nb, inb, nst, hist))
    summary["wait_imms"] = sorted(summary["wait_imms"])
    summary["stores_per_segment"] = sorted(summary["stores_per_segment"])
    if summary["block_waits"] == 0:
        raise DmaModelError("no block wait found: the kernel's structure changed")
    return summary


# ---------------------------------------------------------------------------
# 2. MFMA result reads by inline asm
# ---------------------------------------------------------------------------
_VREG = re.compile(r"^([va])(\d+)$|^([va])\[(\d+):(\d+)\]$")


def _vregs(tok: str) -> set[str]:
    m = _VREG.match(tok.strip())
    if not m:
        return set()
    if m.group(1):
        return {f"{m.group(1)}{m.group(2)}"}
    return {f"{m.group(3)}{k}" for k in range(int(m.group(4)), int(m.group(5)) + 1)}


def _wait_states(i: Insn) -> int:
    if i.mn == "s_nop":
        return int(_ops(i)[0], 0) + 1
    return 1


def check_mfma_hazard(funcs: dict[str, list[Insn]], need: int = 24, need16: int = 8) -> int:
    """Every v_cvt_{rpi,flr}_i32_f32 whose source was last written (in program
    order) by an MFMA has >= `need` wait states of s_nop between them (`need16`
    after a 16x16 MFMA: the 8 the compiler itself inserts before a VALU read of a
    v_mfma_f32_16x16x16_f16 result on gfx950).  Returns the number of such reads checked."""
    checked = 0
    for name, ins in funcs.items():
        for k, i in enumerate(ins):
            if i.mn not in ("v_cvt_rpi_i32_f32_e32", "v_cvt_flr_i32_f32_e32", "v_cvt_rpi_i32_f32_e64",
                            "v_cvt_flr_i32_f32_e64"):
                continue
            src = _vregs(_ops(i)[1])
            nops = 0
            for j in range(k - 1, max(-1, k - 400), -1):
                p = ins[j]
                if p.mn.startswith(("s_cbranch", "s_branch", "s_endpgm")):
                    break
                dst = _vregs(_ops(p)[0]) if _ops(p) else set()
                if p.mn == "s_nop":
                    nops += _wait_states(p)
                if dst & src:
                    if p.mn.startswith("v_mfma"):
                        checked += 1
                        req = need16 if "16x16" in p.mn else need
                        if nops < req:
                            raise AssertionError(
                                f"{name}: {i} reads {sorted(dst & src)[0]} of {p} after only {nops} s_nop wait "
                                f"states (mfma_result_ready needs {req})")
                    break
    return checked


# ---------------------------------------------------------------------------
# 3. scratch
# ---------------------------------------------------------------------------
def private_segment_sizes(meta: str) -> dict[str, int]:
    """Kernel name -> .private_segment_fixed_size from the code objects' metadata."""
    out, name = {}, None
    for line in meta.splitlines():
        m = re.search(r"\.name:\s+(\S+)", line)
        if m:
            name = m.group(1)
        m = re.search(r"\.private_segment_fixed_size:\s+(\d+)", line)
        if m and name:
            out[name] = int(m.group(1))
    return out


def lds_sizes(meta: str) -> dict[str, int]:
    """Kernel name -> static LDS (.group_segment_fixed_size; listed before .name in each kernel's map)."""
    out, pending = {}, None
    for line in meta.splitlines():
        m = re.search(r"\.group_segment_fixed_size:\s+(\d+)", line)
        if m:
            pending = int(m.group(1))
        m = re.search(r"\.name:\s+(\S+)", line)
        if m and pending is not None:
            out[m.group(1)] = pending
            pending = None
    return out


# ---------------------------------------------------------------------------
# 4. source lint
# ---------------------------------------------------------------------------
# __builtin_bit_cast of an ext-vector ELEMENT (v.x / v.y / ...) read element 0 on hipcc 7.2 (round 5:
# the mosaics' pass-2 initial accumulator silently became pass 1's); read the element as a value first
BITCAST_ELEMENT = re.compile(r"__builtin_bit_cast\(\s*[\w:<> ]+,\s*[\w\[\]]+\.[xyzw]\s*\)")


def bitcast_element_uses(paths) -> list[str]:
    hits = []
    for p in paths:
        with open(p) as f:
            for n, line in enumerate(f, 1):
                code = line.split("//", 1)[0]
                if BITCAST_ELEMENT.search(code):
                    hits.append(f"{p}:{n}: {line.strip()}")
    return hits


# readfirstlane returns int: widening its result straight to 64 bits sign-extends a low address word
# with bit 31 set, so a pointer rebuilt from two readfirstlanes (sgpr_ptr, nh_ldsdma.hpp) got an all-ones
# high word -- the round-5 hipErrorIllegalAddress in k_tc32_hd, seen only for buffers whose address had
# bit 31 set; widen through uint32_t
RFL_WIDEN = re.compile(r"\(\s*(?:u?int64_t|uintptr_t|intptr_t|size_t|(?:unsigned\s+)?long(?:\s+long)?)\s*\)"
                       r"\s*__builtin_amdgcn_readfirstlane\b")


def readfirstlane_widen_uses(paths) -> list[str]:
    hits = []
    for p in paths:
        with open(p) as f:
            for n, line in enumerate(f, 1):
                code = line.split("//", 1)[0]
                if RFL_WIDEN.search(code):
                    hits.append(f"{p}:{n}: {line.strip()}")
    return hits


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=LIB)
    a = ap.parse_args()
    funcs, meta = load(a.lib)
    for lv, (name, narrow) in sorted(TC32HD_LEVELS.items()):
        s = check_dma_waits(funcs[name])
        print(f"k_tc32_hd<2, {lv}> (narrow block: {narrow} stores):", s)
    print("MFMA results read by inline asm, checked:", check_mfma_hazard(funcs))
    ps = private_segment_sizes(meta)
    print("scratch:", {k: v for k, v in ps.items() if v}, "of", len(ps), "kernels")


if __name__ == "__main__":
    sys.exit(main())

#!/usr/bin/env python3
"""Which files under profiles/ the documentation and code cite.

    python tools/profile_refs.py            # report: cited patterns, tracked files kept / uncited
    python tools/profile_refs.py --prune    # git rm the tracked profiles/ files nothing cites

A citation is (a) a path starting with profiles/ (a file, a directory -- all of it --,
or a glob with * / {a,b}) or (b) a bare profile file name or stem in DESIGN.md /
README.md (e.g. `ab_closed4_split_r05z_f64.jsonl`, `stamps_r05zh.json`,
`ab_libs_5b_r05*`, `_r05r_*`), matched against the basenames under profiles/.
tests/test_profile_refs.py checks that every (a) citation names an existing file.
"""
from __future__ import annotations

import fnmatch
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SOURCES = ["DESIGN.md", "README.md", "INTEGRATION.md", "bench.py", "profiles/valu_roofline.json",
           "profiles/pmc_traffic.json"]
SOURCE_DIRS = [("tools", (".py", ".sh")), ("tests", (".py",)), ("nano-hevc_amd/csrc", (".hip", ".hpp"))]
FULL = re.compile(r"profiles/[A-Za-z0-9_./*{},-]+")
# bare names: a round tag r0N plus letters, as a file name, stem or glob; or any file name with a
# record's extension (e.g. `ab_variants*.json`, `not_kept_srclds.diff`)
BARE = re.compile(r"(?<![/A-Za-z0-9])_?[A-Za-z0-9_]*_r0\d[a-z0-9]*[A-Za-z0-9_*.]*"
                  r"|(?<![/A-Za-z0-9])[A-Za-z0-9_*{},-]+\.(?:jsonl|json|csv|diff|log)\b")


def source_files():
    out = [os.path.join(ROOT, p) for p in SOURCES if os.path.exists(os.path.join(ROOT, p))]
    for d, exts in SOURCE_DIRS:
        for dp, _, fs in os.walk(os.path.join(ROOT, d)):
            if "__pycache__" in dp or "/_ab" in dp:
                continue
            out += [os.path.join(dp, f) for f in fs if f.endswith(exts) and f not in ("profile_refs.py", "test_profile_refs.py")]
    return out


def expand_braces(p: str) -> list[str]:
    m = re.search(r"\{([^{}]*)\}", p)
    if not m:
        return [p]
    return [q for alt in m.group(1).split(",") for q in expand_braces(p[:m.start()] + alt + p[m.end():])]


def citations():
    full, bare = set(), set()
    for f in source_files():
        txt = open(f, errors="replace").read()
        for m in FULL.finditer(txt):
            p = m.group(0).rstrip(".,);:")
            if re.fullmatch(r"profiles/r0\d/?", p):   # a whole round's directory names no record
                continue
            full.update(expand_braces(p))
        if f.endswith(".md"):
            for m in BARE.finditer(txt):
                t = m.group(0).rstrip(".,);:")
                if len(t) >= 6:
                    bare.update(expand_braces(t))
    return sorted(full), sorted(bare)


def tracked_profiles() -> list[str]:
    out = subprocess.run(["git", "ls-files", "profiles"], cwd=ROOT, capture_output=True, text=True, check=True).stdout
    return [ln for ln in out.splitlines() if ln]


def full_matches(pat: str, files: list[str]) -> list[str]:
    pat = pat.rstrip("/")
    return [f for f in files if f == pat or f.startswith(pat + "/") or fnmatch.fnmatch(f, pat) or
            fnmatch.fnmatch(f, pat + "/*")]


def bare_matches(tok: str, files: list[str]) -> list[str]:
    t = tok if "*" in tok else tok + "*"
    if t.startswith("_"):
        t = "*" + t
    out = []
    for f in files:
        parts = f.split("/")[1:]
        # a bare name may name a file or a directory of a profiler pass (valu_kt_r05w_5b/...)
        if any(fnmatch.fnmatch(p, t) for p in parts):
            out.append(f)
    return out


def main():
    files = tracked_profiles()
    full, bare = citations()
    keep, missing = set(), []
    for p in full:
        m = full_matches(p, files)
        if not m:
            missing.append(p)
        keep.update(m)
    for t in bare:
        keep.update(bare_matches(t, files))
    # a profiler pass directory is kept whole when any of its files is cited
    dirs = {os.path.dirname(f) for f in keep if os.path.basename(os.path.dirname(f)).startswith(("valu_", "prof_", "pmc_", "kt_"))}
    keep.update(f for f in files if os.path.dirname(f) in dirs)
    drop = [f for f in files if f not in keep]
    print(f"{len(files)} tracked, {len(keep)} cited, {len(drop)} uncited; {len(missing)} citations name no file")
    for p in missing:
        print("  missing:", p)
    if "--list" in sys.argv:
        for f in drop:
            print("  uncited:", f)
    if "--prune" in sys.argv and drop:
        for i in range(0, len(drop), 200):
            subprocess.run(["git", "rm", "-q", "--"] + drop[i:i + 200], cwd=ROOT, check=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())

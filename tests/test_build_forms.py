"""Host-side compile check of both library forms (CPU, seconds): every HIP source
under the product flags and under the A/B build's -DNH_AB=1 (which
__graft_entry__.build() also makes).  The A/B-only dispatch branches are host
code, so a break in them shows here without building device code."""
import glob
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "nano-hevc_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="no hipcc")
@pytest.mark.parametrize("ab", [False, True])
def test_host_code_compiles(ab):
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    if ab:
        srcs += sorted(glob.glob(os.path.join(CSRC, "ab", "*.hip")))
    assert srcs
    bad = []
    for src in srcs:
        cmd = [HIPCC, "--offload-arch=gfx950", "-std=c++17", "--cuda-host-only", "-fsyntax-only", "-Wall",
               "-Werror=unused-variable", src] + (["-DNH_AB=1"] if ab else [])
        r = subprocess.run(cmd, capture_output=True, text=True, cwd=CSRC)
        if r.returncode != 0:
            bad.append((os.path.basename(src), r.stderr[-800:]))
    assert not bad, bad

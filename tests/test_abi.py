"""C-ABI boundary checks that need no GPU: the in-tree libnanohevc.so loads,
exports every function include/nanohevc.h declares, the ctypes signature table
covers exactly that set, and compute entry points fail LOUDLY without a device
(no CPU fallback)."""
import ctypes as C
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "nanohevc.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(nh_[a-z0-9_]+)\s*\(", src)))


def test_header_parses():
    names = declared_functions()
    assert "nh_fwd8x8_quant_planes" in names and len(names) >= 20


def test_library_exports_every_declared_symbol():
    from nano_hevc import _lib
    L = _lib.load()
    for name in declared_functions():
        assert hasattr(L, name), name


def test_signature_table_matches_header():
    from nano_hevc import _lib
    assert sorted(_lib.SIGNATURES) == declared_functions()


def test_plane_set_struct_layout():
    from nano_hevc._lib import PlaneSet
    assert C.sizeof(PlaneSet) == 48          # 3 x int64 + 6 x int32, as in nanohevc.h
    assert PlaneSet.width.offset == 24 and PlaneSet.num_groups.offset == 40


def test_version_and_device_count():
    from nano_hevc import _lib
    assert b"gfx950" in _lib.load().nh_version()
    assert _lib.device_count() >= 0


@pytest.mark.skipif(bool(os.environ.get("HIP_VISIBLE_DEVICES_FORCE")), reason="forced device")
def test_compute_without_device_fails_loudly():
    from nano_hevc import _lib
    if _lib.device_count() > 0:
        pytest.skip("a device is visible here")
    import nano_hevc as nh
    with pytest.raises(_lib.NanoHevcUnavailable):
        nh.forward_transform(np.zeros((4, 4), np.int16))
    with pytest.raises(_lib.NanoHevcUnavailable):
        nh.intra_dc_predict(np.zeros(4, np.int16), np.zeros(4, np.int16), 4)


def test_oracle_not_imported_by_product():
    """The product package must never reach into oracle/ (test infrastructure)."""
    pkg = os.path.join(ROOT, "nano-hevc_amd")
    for dp, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".hpp", ".cpp", ".h")):
                txt = open(os.path.join(dp, f), errors="replace").read()
                assert "import oracle" not in txt and "from oracle" not in txt and "nh_oracle" not in txt, f


def _undefined_symbols(path):
    import subprocess
    out = subprocess.run(["nm", "-D", "--undefined-only", path], capture_output=True, text=True, check=True).stdout
    return {ln.split()[-1].split("@")[0] for ln in out.splitlines() if ln.strip()}


def test_product_library_reads_no_environment():
    """The shipped library has no A/B knobs: no getenv import and no NH_* knob
    names (they exist only in the -DNH_AB=1 build, libnanohevc_ab.so)."""
    from nano_hevc import _lib
    assert "getenv" not in _undefined_symbols(_lib.LIB_PATH)
    blob = open(_lib.LIB_PATH, "rb").read()
    for knob in (b"NH_RDO_FORM", b"NH_TU32_BUTTERFLY", b"NH_TU_CLOSED_WAVES", b"NH_CLOSED_WAVES",
                 b"NH_CLOSED_FORM", b"NH_CLOSED_ORDER", b"NH_CLOSED_PROBE", b"NH_ENC_TUNE", b"NH_XCD_ORDER"):
        assert knob not in blob, knob
    # the losing fwd8x8 launch forms and memory probes are not compiled in either
    for kern in (b"k_fwd8x8_quant_h2", b"k_fwd8x8_quant_v2", b"k_fwd8x8_quant_stripe", b"k_probe_rowwave",
                 b"k_intra_rdo8_closed_pair"):
        assert kern not in blob, kern


def test_ab_library_exports_the_same_abi():
    from nano_hevc import _lib
    if not os.path.exists(_lib.LIB_AB_PATH):
        pytest.skip("A/B build absent (make -C nano-hevc_amd ab)")
    L = _lib.load_ab()
    for name in declared_functions():
        assert hasattr(L, name), name
    assert "getenv" in _undefined_symbols(_lib.LIB_AB_PATH)


def test_tc32_layout_checks_precede_any_device_call():
    """nh_tc32_planes / nh_tc32_planes_compact refuse, on the host and before any
    HIP call, the layouts their kernels' address arithmetic does not cover: pitches
    beyond 2^24 samples (k_tc32_hd's 32-bit per-lane offsets), int8 levels on rows
    that are not 16-element aligned, compact levels without a spill plane."""
    from nano_hevc import _lib
    from nano_hevc._lib import PlaneSet
    L = _lib.load()
    fake = C.c_void_p(1 << 20)   # never dereferenced: the checks return first
    big = PlaneSet(0, 0, 0, 64, 64, (1 << 24) + 8, 1, 1, 0)
    assert L.nh_tc32_planes(fake, C.byref(big), 1, 30, fake, fake, 1, None) == _lib.NH_EARG
    assert b"2^24" in L.nh_last_error()
    odd = PlaneSet(0, 0, 0, 104, 64, 104, 1, 1, 0)   # 8- but not 16-element aligned rows
    assert L.nh_tc32_planes_compact(fake, C.byref(odd), 1, 30, fake, 1, fake, fake, None) == _lib.NH_EARG
    assert L.nh_tc32_planes_compact(fake, C.byref(odd), 1, 30, fake, 2, None, fake, None) == _lib.NH_EARG
    assert L.nh_tc32_planes_compact(fake, C.byref(odd), 1, 30, fake, 4, fake, fake, None) == _lib.NH_EARG


def test_tu_compact_layout_checks_precede_any_device_call():
    """nh_tu_pipeline_planes_compact refuses CTB sizes other than 16 / 32 and rows
    that are not 8-sample aligned on the host, before any HIP call."""
    from nano_hevc import _lib
    from nano_hevc._lib import PlaneSet
    L = _lib.load()
    fake = C.c_void_p(1 << 20)
    ok = PlaneSet(0, 0, 0, 64, 64, 64, 1, 1, 0)
    assert L.nh_tu_pipeline_planes_compact(fake, C.byref(ok), 8, 0, 1, 30, 1, 0, 99, fake, fake, fake, fake,
                                           None) == _lib.NH_EARG
    odd = PlaneSet(0, 0, 0, 100, 64, 100, 1, 1, 0)
    assert L.nh_tu_pipeline_planes_compact(fake, C.byref(odd), 32, 0, 1, 30, 1, 0, 99, fake, fake, fake, fake,
                                           None) == _lib.NH_EARG
    assert L.nh_tu_levels_widen(fake, fake, C.byref(ok), 8, 0, 99, fake, None) == _lib.NH_EARG

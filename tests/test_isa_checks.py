"""Hand-counted hardware assumptions of the product kernels, checked on the CPU
against the SHIPPED code object (tools/isa_check.py):

* k_tc32_hd<2> (config 5) retires block k's LDS-DMA image with a hand-counted
  vmcnt (nh_ctu.hip kTc32hdStoresNarrow / kTc32hdStoresWide): an explicit-state
  model of the in-order vmcnt queue over the kernel's control flow proves every
  block wait retires exactly that block's DMA -- and a build with a miscounted
  constant is caught;
* every inline-asm v_cvt_rpi / v_cvt_flr that reads an MFMA result directly has
  the 24 wait states of mfma_result_ready (nh_f16mma.hpp) after the MFMA;
* the hot kernels use no scratch, and config 4's open-loop kernels keep their
  static LDS (a struct copy of the mosaic lane words once added 5 KB per
  chroma workgroup);
* no source bit_casts an ext-vector element (hipcc read element 0).
"""
import os
import sys
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import isa_check as ic  # noqa: E402

HOT = ("k_fwd8x8_quant", "k_tc32_hd", "k_tc32_mfma", "k_ctu_open", "k_ctu_wide", "k_tu_closed_pair",
       "k_intra_rdo8", "k_encode_u8", "k_encode_dcpl", "k_widen", "k_narrow")


@pytest.fixture(scope="module")
def product():
    if not os.path.exists(ic.LIB):
        pytest.skip("libnanohevc.so not built (python -c 'import __graft_entry__ as g; g.build()')")
    return ic.load(ic.LIB)


@pytest.mark.parametrize("levels", sorted(ic.TC32HD_LEVELS))
def test_tc32hd_dma_waits_match_the_code(product, levels):
    """Every level type's instance (int32, and the compact int16 / int8 levels)."""
    funcs, _ = product
    name, narrow = ic.TC32HD_LEVELS[levels]
    s = ic.check_dma_waits(funcs[name])
    # both block kinds reached a wait, with exactly the counted stores behind them
    assert s["stores_per_segment"] == [2, narrow], s
    assert {0, 4}.issubset(s["wait_imms"]) and s["block_waits"] >= 3, s


@pytest.mark.parametrize("define", ["NH_TC32HD_STORES_NARROW=7", "NH_TC32HD_STORES_NARROW=5",
                                    "NH_TC32HD_STORES_WIDE=1"])
def test_tc32hd_miscounted_constant_is_caught(define):
    """The same kernels built with a wrong store count (UNSAFE for an over-count:
    the wait leaves the block's DMA in flight; LOOSE for an under-count) -- every
    level type's instance."""
    src = os.path.join(ROOT, "nano-hevc_amd", "csrc", "nh_ctu.hip")
    with tempfile.TemporaryDirectory() as d:
        elf = ic.compile_device(src, os.path.join(d, "ctu.o"), [define])
        funcs = ic.disassemble(elf)
    for name, _ in ic.TC32HD_LEVELS.values():
        with pytest.raises(ic.DmaModelError):
            ic.check_dma_waits(funcs[name])


def test_mfma_results_read_by_inline_asm_wait(product):
    funcs, _ = product
    assert ic.check_mfma_hazard(funcs) > 0   # config 4 / 5 / closed-loop 32x32 chains


def test_mfma_hazard_checker_catches_a_short_wait():
    mk = ic.Insn
    body = [mk(0, "v_mfma_f32_32x32x16_f16", "v[0:15], v[16:19], v[20:23], 0", None),
            mk(8, "s_nop", "7", None), mk(12, "s_nop", "7", None),
            mk(16, "v_cvt_rpi_i32_f32_e32", "v30, v3", None)]
    with pytest.raises(AssertionError):
        ic.check_mfma_hazard({"k": body})
    body.insert(3, mk(14, "s_nop", "7", None))
    assert ic.check_mfma_hazard({"k": body}) == 1


def test_hot_kernels_use_no_scratch(product):
    _, meta = product
    sizes = ic.private_segment_sizes(meta)
    hot = {k: v for k, v in sizes.items() if any(h in k for h in HOT) and "ILi8ELi1ELb1ELi4E" not in k}
    assert len(hot) >= 20, sorted(hot)
    assert not {k: v for k, v in hot.items() if v}, "scratch in a hot kernel"


def test_ctu_open_static_lds(product):
    _, meta = product
    lds = {k: v for k, v in ic.lds_sizes(meta).items() if "k_ctu_open" in k}
    assert len(lds) >= 8, sorted(lds)
    # CTB 4 / 8 / 16 groups: the strip images, lists, output images and tiles (45,568 B at most);
    # CTB 32: 31,200 B
    assert max(lds.values()) <= 45568, {k: v for k, v in lds.items() if v > 45568}


def test_no_bitcast_of_a_vector_element():
    import glob
    srcs = glob.glob(os.path.join(ROOT, "nano-hevc_amd", "csrc", "*.hip")) + \
        glob.glob(os.path.join(ROOT, "nano-hevc_amd", "csrc", "*.hpp"))
    assert len(srcs) > 10
    assert not ic.bitcast_element_uses(srcs)
    with tempfile.TemporaryDirectory() as d:   # the lint itself
        p = os.path.join(d, "x.hpp")
        with open(p, "w") as f:
            f.write("const float c2 = __builtin_bit_cast(float, mw1.y);\n"
                    "const float ok = __uint_as_float((uint32_t)mw1.y);\n")
        assert len(ic.bitcast_element_uses([p])) == 1


def test_no_readfirstlane_widened_to_64_bits():
    """readfirstlane returns int: (uint64_t)readfirstlane(lo) sign-extends an address
    word with bit 31 set (the round-5 illegal address in k_tc32_hd's SGPR-base
    pointers).  Every such widening goes through uint32_t."""
    import glob
    srcs = glob.glob(os.path.join(ROOT, "nano-hevc_amd", "csrc", "*.hip")) + \
        glob.glob(os.path.join(ROOT, "nano-hevc_amd", "csrc", "*.hpp"))
    assert not ic.readfirstlane_widen_uses(srcs)
    with tempfile.TemporaryDirectory() as d:   # the lint itself
        p = os.path.join(d, "x.hpp")
        with open(p, "w") as f:
            f.write("return (uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)v) | hi;\n"
                    "return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v) | hi;\n")
        assert len(ic.readfirstlane_widen_uses([p])) == 1

"""ctypes binding of include/nanohevc.h (libnanohevc.so, built in-tree for gfx950).

There is no CPU fallback: if the library or a HIP device is missing, every
compute call raises ``NanoHevcUnavailable`` (a RuntimeError) -- loudly.
"""
from __future__ import annotations

import atexit
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libnanohevc.so")
# The A/B build (make ab, -DNH_AB=1): losing launch forms, memory probes and the
# NH_* environment knobs of tools/.  Never loaded unless asked for explicitly
# (use_ab(), or a fwd8x8 launch variant that only exists there).
LIB_AB_PATH = os.path.join(HERE, "libnanohevc_ab.so")

NH_OK, NH_EVALUE, NH_EINDEX, NH_EOVERFLOW, NH_EZERODIV, NH_EARG, NH_ETYPE = 0, -1, -2, -3, -4, -5, -6
NH_ENODEV, NH_EHIP = -10, -11


class NanoHevcUnavailable(RuntimeError):
    """The HIP library or an MI355X is not available (no CPU fallback exists)."""


class PlaneSet(C.Structure):
    """nh_plane_set (include/nanohevc.h)."""
    _fields_ = [("base", C.c_int64), ("plane_stride", C.c_int64), ("group_stride", C.c_int64),
                ("width", C.c_int32), ("height", C.c_int32), ("pitch", C.c_int32),
                ("planes_per_group", C.c_int32), ("num_groups", C.c_int32), ("reserved", C.c_int32)]


P, I64, I32, U32, VP = C.c_void_p, C.c_int64, C.c_int, C.c_uint32, C.c_void_p

# every symbol declared in include/nanohevc.h, with its argument types
SIGNATURES = {
    "nh_version": ([], C.c_char_p),
    "nh_last_error": ([], C.c_char_p),
    "nh_device_count": ([P], I32),
    "nh_staging_bytes": ([I32, P], I32),
    "nh_release_staging": ([], I32),
    "nh_last_call_times": ([P], I32),
    "nh_block_server_set_idle_us": ([I64], I32),
    "nh_block_server_stop": ([], I32),
    "nh_block_server_stats": ([I32, P], I32),
    "nh_intra_dc": ([P, I64, P, I64, I64, I32, P], I32),
    "nh_intra_planar": ([P, I64, P, I64, I64, I32, I64, I32, I64, I64, P], I32),
    "nh_intra_angular": ([P, I64, P, I64, I64, I32, I64, P], I32),
    "nh_residual": ([P, P, I64, P], I32),
    "nh_reconstruct": ([P, P, I64, P], I32),
    "nh_clip": ([P, I64, I64, P], I32),
    "nh_forward_transform": ([P, I64, I32, P], I32),
    "nh_inverse_transform": ([P, I64, I32, P], I32),
    "nh_quantize": ([P, I64, I32, I64, I32, I32, P], I32),
    "nh_quantize_abs": ([P, I64, I32, I64, I32, P], I32),
    "nh_dequantize": ([P, I64, I32, P], I32),
    "nh_count_nonzero": ([P, I64, P], I32),
    "nh_estimate_bits": ([P, I64, I32, P], I32),
    "nh_sum_sq_diff": ([P, P, I64, P], I32),
    "nh_sum_sq_diff_f64": ([P, P, I64, P], I32),
    "nh_sad": ([P, P, I64, P], I32),
    "nh_satd_4x4": ([P, P, P], I32),
    "nh_residual_energy": ([P, I64, P], I32),
    "nh_sse_i16": ([P, P, I64, P, VP], I32),
    "nh_fwd8x8_quant_planes": ([P, P, C.POINTER(PlaneSet), I32, I32, I32, VP], I32),
    "nh_fwd8x8_quant_planes_variant": ([P, P, C.POINTER(PlaneSet), I32, I32, I32, I32, VP], I32),
    "nh_fwd8x8_quant_planes_ex": ([P, P, C.POINTER(PlaneSet), I32, I32, I32, P, P, VP], I32),
    "nh_probe_copy8x8_planes": ([P, P, C.POINTER(PlaneSet), I32, I32, VP], I32),
    "nh_probe_copy_linear": ([P, P, I64, I32, I32, VP], I32),
    "nh_fwd_transform_batch": ([P, P, I64, I32, I32, VP], I32),
    "nh_inv_transform_batch": ([P, P, I64, I32, I32, VP], I32),
    "nh_quant_batch": ([P, P, I64, I32, I32, I32, VP], I32),
    "nh_dequant_batch": ([P, P, I64, I32, VP], I32),
    "nh_intra_rdo_plane": ([P, I32, I32, I32, I32, P, P, P, P, VP], I32),
    "nh_intra_rdo_planes": ([P, C.POINTER(PlaneSet), I32, I32, P, P, P, P, VP], I32),
    "nh_tu_workspace_bytes": ([I32, I32, I32], I64),
    "nh_tu_pipeline_plane": ([P, I32, I32, I32, I32, I32, U32, I32, I32, I32, I32, P, P, P, P, VP], I32),
    "nh_tu_pipeline_planes": ([P, C.POINTER(PlaneSet), I32, I32, U32, I32, I32, I32, I32, P, P, P, VP], I32),
    "nh_tu_pipeline_planes_compact": ([P, C.POINTER(PlaneSet), I32, I32, U32, I32, I32, I32, I32, P, P, P, P, VP], I32),
    "nh_tu_levels_widen": ([P, P, C.POINTER(PlaneSet), I32, I32, I32, P, VP], I32),
    "nh_tc32_plane": ([P, I32, I32, I32, I32, P, P, I32, VP], I32),
    "nh_tc32_planes": ([P, C.POINTER(PlaneSet), I32, I32, P, P, I32, VP], I32),
    "nh_tc32_planes_compact": ([P, C.POINTER(PlaneSet), I32, I32, P, I32, P, P, VP], I32),
    "nh_tc32_levels_widen": ([P, I32, P, C.POINTER(PlaneSet), I32, P, VP], I32),
    "nh_tu_pipeline_closed_workspace_bytes": ([C.POINTER(PlaneSet), I32], I64),
    "nh_tu_pipeline_planes_closed": ([P, C.POINTER(PlaneSet), I32, I32, C.c_uint32, I32, I32, P, P, P, P, VP], I32),
    "nh_probe_mfma_i8": ([P, P, P, VP], I32),
    "nh_intra_rdo_closed_workspace_bytes": ([C.POINTER(PlaneSet), I32], I64),
    "nh_intra_rdo_planes_closed": ([P, C.POINTER(PlaneSet), I32, I32, P, P, P, P, P, VP], I32),
    "nh_intra_rdo_closed_status": ([P, P, VP], I32),
    "nh_widen_u8_i16": ([P, P, I64, VP], I32),
    "nh_narrow_i16_u8": ([P, P, I64, VP], I32),
    "nh_encode_intra_planes": ([P, I32, C.POINTER(PlaneSet), I32, P, P, P, P, P, VP], I32),
}

_libs = {}
_use_ab = False


def use_ab(on: bool = True):
    """Route every later call of this process to the A/B library (tools/ only)."""
    global _use_ab
    _use_ab = bool(on)


def load_ab():
    """The A/B library (raises NanoHevcUnavailable if `make ab` was not run)."""
    return _open(LIB_AB_PATH, "make -C nano-hevc_amd ab")


def load():
    """Load libnanohevc.so (raises NanoHevcUnavailable if it was not built)."""
    if _use_ab:
        return load_ab()
    return _open(LIB_PATH, "python -c 'import __graft_entry__ as g; g.build()'")


def _open(path, how):
    L = _libs.get(path)
    if L is not None:
        return L
    # One HIP runtime per process: torch wheels bundle their own libamdhip64
    # (SONAME libamdhip64.so.7).  Importing torch first makes that copy the
    # process's runtime, and our DT_NEEDED libamdhip64.so.7 then binds to it
    # (loading /opt/rocm's copy first would leave torch with a second runtime
    # that cannot see the device).  Without torch, /opt/rocm's runtime is used.
    try:
        import torch  # noqa: F401
    except Exception:  # pragma: no cover - torch is optional for the C-ABI path
        pass
    if not os.path.exists(path):
        raise NanoHevcUnavailable(
            f"{path} not built: run `{how}` (hipcc --offload-arch=gfx950); nano_hevc has no CPU fallback")
    try:
        L = C.CDLL(path)
    except OSError as e:  # pragma: no cover
        raise NanoHevcUnavailable(f"cannot load {path}: {e}") from e
    for name, (args, res) in SIGNATURES.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _libs[path] = L
    # a resident block-call server leaves on its own within its idle time; at
    # interpreter exit it is asked to leave at once (while the runtime is up)
    atexit.register(L.nh_block_server_stop)
    return L


def device_count() -> int:
    n = C.c_int(0)
    load().nh_device_count(C.byref(n))
    return n.value


def check(rc: int, what: str = "", lib=None):
    """Map an NH_E* code to the exception the reference raises in that case
    (``lib``: the library that returned it, for its last-error text)."""
    if rc == NH_OK:
        return
    msg = f"{what}: " if what else ""
    if rc == NH_EVALUE:
        raise ValueError(msg + "unsupported value")
    if rc == NH_EINDEX:
        raise IndexError(msg + "index out of range")
    if rc == NH_EOVERFLOW:
        raise OverflowError(msg + "Python integer out of bounds for int16")
    if rc == NH_EZERODIV:
        raise ZeroDivisionError(msg + "integer division or modulo by zero")
    if rc == NH_ETYPE:
        raise TypeError(msg + "ufunc 'right_shift' not supported for the input types")
    if rc == NH_ENODEV:
        raise NanoHevcUnavailable(msg + "no HIP device visible: nano_hevc (MI355X) has no CPU fallback")
    err = (lib or load()).nh_last_error().decode(errors="replace")
    if rc == NH_EARG:
        raise ValueError(msg + "bad argument: " + err)
    raise RuntimeError(msg + f"HIP error {rc}: {err}")


try:   # in-tree host glue (nano_hevc/_nhaddr.c, built by the Makefile): ~0.15 us per address
    from ._nhaddr import addr as _addr
except ImportError:  # pragma: no cover - numpy's ctypes route (1-4 us per address)
    _addr = None


def ptr(a: np.ndarray):
    """Data address of a C-contiguous host array for a c_void_p argument (the
    array must stay referenced for the duration of the call)."""
    return _addr(a) if _addr is not None else a.ctypes.data_as(C.c_void_p)

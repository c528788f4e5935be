"""Quality metrics (reference metrics.py:7-48).

Planned as device reductions ("next"); until then these names
exist for import compatibility and raise loudly instead of silently computing
on the CPU.
"""
from __future__ import annotations


def _pending(name):
    def f(*args, **kwargs):
        raise NotImplementedError(f"nano_hevc.{name}: device metric reduction not built yet (SURVEY §8f-2)")
    f.__name__ = name
    return f


mse = _pending("mse")
psnr = _pending("psnr")
sad = _pending("sad")
satd_4x4 = _pending("satd_4x4")
residual_energy = _pending("residual_energy")

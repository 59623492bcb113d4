"""MI355X-native Reed-Solomon engine behind the reference's internal/ec surface.

Public surface:
  ec.NewService / ec.Service  -- IEcDriver mirror (Split / Encode / Reconstruct)
  batch.BatchEngine           -- batched device-resident and pinned-host entry points
The arithmetic lives in librsgpu.so (csrc/, gfx950 HIP kernels, C-ABI include/rsgpu.h).
"""
from . import _lib  # noqa: F401

__all__ = ["ec", "batch", "xoshiro"]

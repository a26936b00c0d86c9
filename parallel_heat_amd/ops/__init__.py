"""Tensor-level stencil kernels (gfx950 HIP on ROCm tensors, OpenMP oracle on CPU tensors)."""
from .stencil import (Field, Geom, init_field, lds_step, mfma_step, naive_step, pack, residual, resid_value, tb_stamps, tb_step,
                      unpack)

__all__ = ["Field", "Geom", "init_field", "lds_step", "mfma_step", "naive_step", "tb_step", "tb_stamps", "pack", "unpack", "residual",
           "resid_value"]

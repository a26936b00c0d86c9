"""Tensor-level stencil kernels (gfx950 HIP on ROCm tensors, OpenMP oracle on CPU tensors)."""
from .stencil import (Field, Geom, TbTuning, TbVariant, init_field, lds_step, mfma_step,
                      naive_step, pack, residual, resid_value, set_tb_tuning, tb_stamps, tb_step,
                      tb_tuning, unpack)

__all__ = ["Field", "Geom", "TbTuning", "TbVariant", "init_field", "lds_step", "mfma_step",
           "naive_step", "tb_step", "tb_stamps", "tb_tuning", "set_tb_tuning", "pack", "unpack",
           "residual", "resid_value"]

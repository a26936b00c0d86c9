"""parallel_heat_amd — MI355X-native 2-D heat-diffusion framework.

Capabilities of manospits/parallel_heat (5-point Jacobi heat plate, reference
initial condition, convergence test, ``prtdat`` text output, CUDA single-GPU and
MPI/OpenMP distributed programs), rebuilt for AMD Instinct MI355X (gfx950):
hand-written CDNA4 HIP kernels (register-streaming temporal blocking), a native
C++ runtime (``csrc/``, ``libheat.so``) with hipGraph-captured passes, and RCCL
halo exchange over xGMI with one process per GPU.

Layout:
    models/    HeatConfig, HeatSolver (the heat-plate model), NumPy/PyTorch reference
    ops/       tensor-level kernels (naive step, temporally blocked step, pack, residual)
    parallel/  topology/decomposition, torch.distributed plumbing, transports
    utils/     .dat/.bin I/O, timing, reporting
"""
import torch  # noqa: F401  (load torch's HIP runtime before libheat)

from . import _native
from ._native import NativeError, build_native
from .models.config import HeatConfig
from .models.heat2d import HeatSolver, RunResult

__version__ = "0.1.0"

__all__ = ["HeatConfig", "HeatSolver", "RunResult", "NativeError", "build_native", "_native"]

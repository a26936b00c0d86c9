"""Heat-plate model: configuration, native-engine solver, NumPy/PyTorch reference."""
from .config import HeatConfig
from .heat2d import BlockInfo, HeatSolver, RunResult
from . import reference

__all__ = ["HeatConfig", "HeatSolver", "RunResult", "BlockInfo", "reference"]

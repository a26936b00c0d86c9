"""Run configuration of the 2-D heat-diffusion model.

Every field replaces one of the reference's compile-time macros
(``cuda/cuda_heat.cu:7-23``, ``mpi/mpi_heat_improved_persistent_stat.c:7-32``,
``mpi/Makefile:1-25``); defaults reproduce the reference source defaults.
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass
from typing import Optional

from .. import _native

INIT_MODES = {"ref-wrap": 0, "exact": 1, "ref64": 1, "random": 2, "zero": 3}
BACKENDS = {"cpu": 0, "hip": 1}
KERNELS = {"auto": 0, "naive": 1, "tb": 2, "lds": 3, "mfma": 4}
DECOMPS = {"auto": 0, "rows": 1, "1d": 1, "2d": 2}
COMPATS = {"none": 0, "mpi": 1, "cuda": 2}
SCHEDULES = {"auto": 0, "sync": 1, "overlap": 2, "pipeline": 3}
NUMERICS = {"fp32": 0, "mpi": 1}


@dataclass
class HeatConfig:
    nx: int = 20                  # NXPROB (rows, slow index)
    ny: int = 20                  # NYPROB (columns, contiguous index)
    steps: int = 10000            # STEPS
    cx: float = 0.1               # PARMS_CX / parms.cx
    cy: float = 0.1               # PARMS_CY / parms.cy
    converge: bool = False        # -DCONVERGE
    check_interval: int = 20      # CHECK_INTERVAL / STEP
    eps: float = 1e-3             # threshold literal 1e-3
    init: str = "ref-wrap"        # inidat semantics (ref-wrap | exact | random | zero)
    seed: int = 0
    backend: str = "hip"          # hip | cpu
    kernel: str = "auto"          # auto | naive | tb
    tb_depth: int = 0             # fused steps per pass / halo depth (0 = tuned default)
    threads: int = 0              # CPU threads (THREAD_COUNT); 0 = runtime default
    decomp: str = "auto"          # auto (MPI_Dims_create 2-D) | rows | 2d
    px: int = 0
    py: int = 0
    use_graph: bool = True
    overlap: bool = True
    compat: str = "none"          # none | mpi | cuda  
    device: int = -1
    schedule: str = "auto"        # multi-rank pass schedule: auto(=sync) | sync | overlap | pipeline
    halo_passes: int = 0          # sync: passes per halo exchange (ghost depth m*K); 0 = auto
    numerics: str = "fp32"        # fp32 (canonical FMA) | mpi (reference MPI double arithmetic)
    phase_timing: bool = False    # per-phase times (exchange/compute/reduce) in RunResult; eager

    def replace(self, **kw) -> "HeatConfig":
        return dataclasses.replace(self, **kw)

    def validate(self) -> None:
        if self.nx < 1 or self.ny < 1:
            raise ValueError(f"grid {self.nx}x{self.ny}")
        for name, table in (("init", INIT_MODES), ("backend", BACKENDS), ("kernel", KERNELS),
                            ("decomp", DECOMPS), ("compat", COMPATS),
                            ("schedule", SCHEDULES), ("numerics", NUMERICS)):
            if getattr(self, name) not in table:
                raise ValueError(f"{name}={getattr(self, name)!r}; expected one of {sorted(table)}")
        if self.check_interval < 1:
            raise ValueError("check_interval must be >= 1")
        if self.halo_passes < 0:
            raise ValueError("halo_passes must be >= 0")

    def total_steps(self) -> int:
        """Updates a full run performs (compat=mpi runs STEPS+1)."""
        return self.steps + 1 if self.compat == "mpi" else self.steps

    def to_native(self, device: Optional[int] = None) -> _native.HeatParams:
        self.validate()
        p = _native.HeatParams()
        p.nx, p.ny = int(self.nx), int(self.ny)
        p.cx, p.cy = float(self.cx), float(self.cy)
        p.converge = int(bool(self.converge))
        p.check_interval = int(self.check_interval)
        p.eps = float(self.eps)
        p.init = INIT_MODES[self.init]
        p.seed = int(self.seed)
        p.backend = BACKENDS[self.backend]
        p.kernel = KERNELS[self.kernel]
        p.tb_depth = int(self.tb_depth)
        p.threads = int(self.threads)
        p.decomp = DECOMPS[self.decomp]
        p.px, p.py = int(self.px), int(self.py)
        p.use_graph = int(bool(self.use_graph))
        p.overlap = int(bool(self.overlap))
        p.compat = COMPATS[self.compat]
        p.device = int(self.device if device is None else device)
        p.schedule = SCHEDULES[self.schedule]
        p.halo_passes = int(self.halo_passes)
        p.numerics = NUMERICS[self.numerics]
        p.phase_timing = int(bool(self.phase_timing))
        return p

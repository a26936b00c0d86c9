"""The 2-D heat-plate model: a Python handle on one rank of the native engine.

This is the user-facing equivalent of the reference's two ``main`` programs
(``cuda/cuda_heat.cu:166-269`` single GPU, ``mpi/mpi_heat_improved_persistent_stat.c:35-310``
distributed).  One ``HeatSolver`` per process; with ``world > 1`` every rank
constructs one with the same config and they cooperate through the chosen
transport (see ``parallel.comm``).

    cfg = HeatConfig(nx=8192, ny=8192, steps=1000, init="random")
    s = HeatSolver(cfg)                # hip backend, rank 0 of 1
    stats = s.run()                    # cfg.total_steps() steps (or until converged)
    grid = s.gather()                  # full grid on rank 0 (numpy)
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Optional

import numpy as np

from .. import _native
from ..parallel import comm as pcomm
from .config import HeatConfig


@dataclass
class RunResult:
    steps_done: int
    total_steps: int
    converged: bool
    converged_at: int
    last_resid: float
    seconds: float
    passes: int
    exchanges: int
    checks: int
    cells: int  # nx*ny
    t_exchange: float = 0.0  # seconds in halo exchanges (phase_timing)
    t_compute: float = 0.0   # seconds in stencil kernels
    t_reduce: float = 0.0    # seconds in residual all-reduce + read-back
    resident_passes: int = 0  # passes run inside resident-tile launches (tiles kept in VGPRs)
    # 1: a resident launch gave up a neighbour wait (results invalid); only
    # returned with HEAT_TB_RES_GIVEUP=defer, otherwise run() raises.
    resident_giveups: int = 0
    # passes run inside chained level-split launches (one-rank runs of the
    # streaming depth-12 pipelines, no grid-wide boundary between passes)
    chained_passes: int = 0

    @property
    def mcells_per_s(self) -> float:
        return self.cells * self.steps_done / self.seconds / 1e6 if self.seconds > 0 else 0.0

    @property
    def s_per_1000_iters(self) -> float:
        return self.seconds * 1000.0 / self.steps_done if self.steps_done else 0.0

    def as_dict(self) -> dict:
        d = dict(self.__dict__)
        d["mcells_per_s"] = self.mcells_per_s
        d["s_per_1000_iters"] = self.s_per_1000_iters
        return d


@dataclass
class BlockInfo:
    rank: int
    world: int
    px: int
    py: int
    cx: int
    cy: int
    ox: int
    oy: int
    lx: int
    ly: int
    nbr: tuple
    pitch: int
    rows: int
    hx: int
    hy: int
    halo: int
    tb_depth: int
    bytes_per_field: int
    schedule: str


class HeatSolver:
    """One rank of a heat-diffusion run on the native MI355X engine."""

    def __init__(self, config: HeatConfig, transport: str = "auto",
                 dist_info: Optional[pcomm.DistInfo] = None, device: Optional[int] = None,
                 hub: Optional[pcomm.LoopbackHub] = None, group=None,
                 shared: Optional[pcomm.EngineTransport] = None,
                 rccl_uid: Optional[bytes] = None):
        """`shared`: an existing EngineTransport (e.g. the run's one RCCL
        communicator) instead of building a new transport.  `rccl_uid`: the
        RCCL unique id shared by ranks that are threads of one process."""
        self.config = config
        config.validate()
        if config.backend == "hip":
            _native.require_gpu_native()
        self.dist = dist_info or pcomm.env_info()
        if shared is not None:
            transport = shared.kind
        if transport == "auto":
            if self.dist.world == 1:
                transport = "local"
            elif config.backend == "hip":
                transport = "rccl"
            else:
                transport = "torch"
        if device is None:
            if config.device >= 0:
                device = config.device
            elif config.backend == "hip":
                n = max(1, _native.device_count())
                device = self.dist.local_rank % n
            else:
                device = -1
        self.device = device
        self.transport = transport
        params = config.to_native(device=device)
        h = ctypes.c_void_p()
        if shared is not None:
            self._comm, self._keep = None, shared
            _native.call("heat_solver_create_shared", ctypes.byref(params), shared.handle,
                         ctypes.byref(h))
        else:
            self._comm, self._keep = pcomm.make_comm(transport, self.dist, device=max(device, 0),
                                                     hub=hub, group=group, rccl_uid=rccl_uid)
            _native.call("heat_solver_create", ctypes.byref(params), ctypes.byref(self._comm),
                         ctypes.byref(h))
        self._h = h
        self.info = self._info()

    # -- lifecycle -----------------------------------------------------------
    def abort(self) -> None:
        """Give up this rank: abort its transport (ncclCommAbort) so that its
        peers stop waiting for it; a wait of this solver on another thread
        raises.  Thread-safe; the solver is unusable afterwards."""
        if getattr(self, "_h", None):
            _native.call("heat_solver_abort", self._h)

    def close(self) -> None:
        if getattr(self, "_h", None):
            _native.call("heat_solver_destroy", self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # -- queries ---------------------------------------------------------------
    def _info(self) -> BlockInfo:
        i = _native.HeatBlockInfo()
        _native.call("heat_solver_info", self._h, ctypes.byref(i))
        return BlockInfo(i.rank, i.world, i.px, i.py, i.cx, i.cy, i.ox, i.oy, i.lx, i.ly,
                         tuple(i.nbr), i.pitch, i.rows, i.hx, i.hy, i.halo, i.tb_depth,
                         i.bytes_per_field,
                         {1: "sync", 2: "overlap", 3: "pipeline"}.get(i.schedule, "?"))

    @property
    def step(self) -> int:
        v = ctypes.c_int64()
        _native.call("heat_solver_step", self._h, ctypes.byref(v))
        return v.value

    @property
    def rank(self) -> int:
        return self.info.rank

    @property
    def world(self) -> int:
        return self.info.world

    # -- running ----------------------------------------------------------------
    def run(self, steps: Optional[int] = None, wait: bool = True) -> RunResult:
        """Advance `steps` steps (default: the config's full run, minus steps done).

        wait=False enqueues them and returns at once (plain GPU runs; gated
        convergence checks, phase timing and host-staged halos still wait):
        back-to-back calls keep the device busy, and the next run() -- run(0)
        to just complete -- waits for every enqueued step and reports
        errors and resident give-ups.  seconds is 0 for an enqueued run."""
        if steps is None:
            steps = self.config.total_steps() - self.step
        st = _native.HeatRunStats()
        _native.call("heat_solver_run" if wait else "heat_solver_enqueue", self._h, int(steps),
                     ctypes.byref(st))
        return RunResult(st.steps_done, st.total_steps, bool(st.converged), st.converged_at,
                         st.last_resid, st.seconds, st.passes, st.exchanges, st.checks,
                         self.config.nx * self.config.ny, st.t_exchange, st.t_compute,
                         st.t_reduce, st.resident_passes, st.resident_giveups, st.chained_passes)

    def time_exchange(self, depth: int, iters: int = 20) -> tuple:
        """(seconds per grouped halo exchange of `depth` rows/columns on this
        rank, its largest message in bytes).  Collective over the ranks."""
        t = ctypes.c_double()
        b = ctypes.c_int64()
        _native.call("heat_solver_time_exchange", self._h, int(depth), int(iters),
                     ctypes.byref(t), ctypes.byref(b))
        return t.value, b.value

    def reset(self) -> None:
        _native.call("heat_solver_reset", self._h)

    def barrier(self) -> None:
        _native.call("heat_solver_barrier", self._h)

    # -- state --------------------------------------------------------------------
    def local(self) -> np.ndarray:
        """This rank's owned block of the current state (lx, ly) float32."""
        a = np.empty((self.info.lx, self.info.ly), np.float32)
        _native.call("heat_solver_copy_owned", self._h, a.ctypes.data, self.info.ly)
        return a

    def load_local(self, block: np.ndarray, step: int = 0) -> None:
        a = np.ascontiguousarray(block, dtype=np.float32)
        if a.shape != (self.info.lx, self.info.ly):
            raise ValueError(f"block shape {a.shape} != {(self.info.lx, self.info.ly)}")
        _native.call("heat_solver_load_owned", self._h, a.ctypes.data, self.info.ly, int(step))

    def gather(self) -> Optional[np.ndarray]:
        """Full (nx, ny) grid on rank 0; None on other ranks.  Collective."""
        if self.rank == 0:
            g = np.empty((self.config.nx, self.config.ny), np.float32)
            _native.call("heat_solver_gather", self._h, g.ctypes.data)
            return g
        _native.call("heat_solver_gather", self._h, None)
        return None

    def scatter(self, grid: Optional[np.ndarray] = None, step: int = 0) -> None:
        """Distribute a full (nx, ny) grid held by rank 0 to every rank's block
        (the reference's master scatter, mpi/...c:100-127).  Collective; other
        ranks pass None."""
        if self.rank == 0:
            if grid is None:
                raise ValueError("rank 0 must pass the full grid")
            g = np.ascontiguousarray(grid, dtype=np.float32)
            if g.shape != (self.config.nx, self.config.ny):
                raise ValueError(f"grid shape {g.shape} != {(self.config.nx, self.config.ny)}")
            _native.call("heat_solver_scatter", self._h, g.ctypes.data, int(step))
        else:
            _native.call("heat_solver_scatter", self._h, None, int(step))

    def checksum(self) -> dict:
        c = _native.HeatChecksum()
        _native.call("heat_solver_checksum", self._h, ctypes.byref(c))
        return {"hash": f"{c.hash:016x}", "sum": c.sum, "min": c.min, "max": c.max,
                "count": c.count}

    def save(self, path: str) -> None:
        """Binary grid / checkpoint (header + nx*ny fp32); collective."""
        _native.call("heat_solver_write_bin", self._h, str(path).encode())

    def load(self, path: str) -> None:
        """Resume from a binary checkpoint written by save(); collective."""
        _native.call("heat_solver_read_bin", self._h, str(path).encode())

    def device_ptr(self) -> int:
        p = ctypes.c_void_p()
        _native.call("heat_solver_current_ptr", self._h, ctypes.byref(p))
        return p.value or 0

"""Runtime autotuning of the multi-rank layout: decomposition x pass schedule.

The reference fixes its decomposition with ``MPI_Dims_create``
(``mpi/mpi_heat_improved_persistent_stat.c:51-75``) and its overlap scheme in
source.  On an MI355X node the best choice depends on things that are only
known on the machine: per-rank block shape vs. the temporally blocked
kernel's chunk ramp, RCCL point-to-point bandwidth per xGMI link (1-D slabs
put all halo bytes on two links, 2-D blocks spread fewer bytes over four),
and how well an exchange overlaps the interior launch.  ``autotune`` times a
short run of every candidate on the real ranks (collectively, max over
ranks), and returns the fastest configuration plus the measured table.

    best, table = autotune(cfg, DistInfo(rank, world, local_rank))
    solver = HeatSolver(best, dist_info=info)

Every rank must call it with the same arguments (it builds and destroys one
solver per candidate; with ``shared`` they all use one RCCL communicator).  A candidate the
engine rejects (e.g. a block thinner than its halo) is skipped on every rank
(the rejection is decided from global quantities, so all ranks agree).
"""
from __future__ import annotations

import time
from typing import Callable, Dict, List, Optional, Sequence, Tuple

from .. import _native
from ..models.config import HeatConfig
from .comm import DistInfo
from .topology import dims_create


def _layout_key(cfg: HeatConfig, world: int) -> Tuple[int, int]:
    """(px, py) the engine will use for cfg on `world` ranks."""
    if cfg.px > 0 and cfg.py > 0:
        return cfg.px, cfg.py
    if cfg.decomp in ("rows", "1d"):
        return world, 1
    d = dims_create(world, 2)
    return d[0], d[1]


def default_candidates(cfg: HeatConfig, world: int, schedules: Sequence[str] = ("sync",),
                       halo_passes: Sequence[int] = (0,)) -> List[HeatConfig]:
    """Rows slabs and the MPI_Dims_create 2-D grid (when different), times the
    given pass schedules and passes-per-exchange values (0 = engine default)."""
    layouts: List[HeatConfig] = []
    seen = set()
    for decomp in ("rows", "auto"):
        c = cfg.replace(decomp=decomp, px=0, py=0)
        key = _layout_key(c, world)
        if key not in seen:
            seen.add(key)
            layouts.append(c)
    out = []
    for c in layouts:
        for s in schedules:
            for m in halo_passes:
                if s != "sync" and m:
                    continue  # passes per exchange only apply to the sync schedule
                out.append(c.replace(schedule=s, halo_passes=m))
    return out


def describe(cfg: HeatConfig, world: int) -> Dict[str, object]:
    px, py = _layout_key(cfg, world)
    return {"px": px, "py": py, "schedule": cfg.schedule, "halo_passes": cfg.halo_passes}


def autotune(cfg: HeatConfig, info: DistInfo, candidates: Optional[List[HeatConfig]] = None,
             steps: int = 1000, repeats: int = 3,
             make: Optional[Callable[[HeatConfig], object]] = None,
             log: Optional[Callable[[str], None]] = None,
             shared=None) -> Tuple[HeatConfig, List[dict]]:
    """Time every candidate (steps x repeats, after one untimed run of `steps`
    that captures the graphs) and return (fastest config, table).

    `make(cfg)` builds the solver (default: HeatSolver(cfg, dist_info=info,
    shared=shared)); pass `shared` (a parallel.comm.EngineTransport) so every
    candidate rides the same communicator instead of one ncclCommInitRank per
    candidate.  Collective over torch.distributed's default group when
    info.world > 1: every rank takes the same sequence of agreements, so a
    candidate that any rank rejects at construction is skipped on all
    of them together instead of leaving the ranks in mismatched collectives.
    That holds for failures at construction only: a candidate that fails
    while it runs aborts the (shared) transport and the whole autotune on
    that rank (NativeError); its peers end in their watchdog."""
    import torch
    import torch.distributed as dist

    from ..models.heat2d import HeatSolver

    world = info.world
    if candidates is None:
        candidates = default_candidates(cfg, world)
    if make is None:
        def make(c):
            return HeatSolver(c, dist_info=info, shared=shared)

    gpu = cfg.backend == "hip"

    def agree_all(flag: float, op) -> float:
        if world == 1:
            return flag
        t = torch.tensor([flag], dtype=torch.float64, device="cuda" if gpu else "cpu")
        dist.all_reduce(t, op=op)
        return float(t.item())

    MIN = dist.ReduceOp.MIN if world > 1 else None
    MAX = dist.ReduceOp.MAX if world > 1 else None

    def sync():
        if gpu:
            torch.cuda.synchronize()

    def barrier():
        if world > 1:
            dist.barrier()

    table: List[dict] = []
    best, best_ms = None, float("inf")
    for c in candidates:
        row = describe(c, world)
        solver = None
        try:
            solver = make(c)
            ok = 1.0
        except _native.NativeError as e:
            ok = 0.0
            row["error"] = str(e).splitlines()[0][:200]
        if agree_all(ok, MIN) < 1.0:
            if solver is not None:
                solver.close()
            row.setdefault("error", "rejected on another rank")
            table.append(row)
            if log:
                log(f"autotune: {row} skipped")
            continue
        dt = 0.0
        try:
            solver.run(steps)  # graph capture, RCCL connections
            barrier()
            sync()
            t0 = time.perf_counter()
            for _ in range(repeats):
                solver.run(steps)
            sync()
            dt = time.perf_counter() - t0
            row["halo"] = solver.info.halo
            row["tb_depth"] = solver.info.tb_depth
        except _native.NativeError as e:
            # A run-time failure can leave this rank's peers inside a send /
            # recv / all-reduce that will never match, and unmatched ops queued
            # on the shared communicator: no later candidate may use it.
            # Abort it (ncclCommAbort: the peers' pending waits end in their
            # watchdog, HEAT_WATCHDOG_S) and end the whole autotune.
            try:
                solver.abort()
            finally:
                solver.close()
            raise _native.NativeError(
                f"autotune aborted: candidate {row} failed at run time on rank "
                f"{info.rank}: {str(e).splitlines()[0][:200]}") from e
        solver.close()
        dt = agree_all(dt, MAX)
        ms = dt * 1e3 * 1000.0 / (steps * repeats)
        row["ms_per_1000_iters"] = round(ms, 4)
        row["repeats"] = repeats
        table.append(row)
        if log:
            log(f"autotune: {row}")
        if ms < best_ms:
            best, best_ms = c, ms
    if best is None:
        raise _native.NativeError("autotune: every candidate was rejected: %r" % table)
    return best, table

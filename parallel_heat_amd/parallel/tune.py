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


def exchange_depths(halo: int) -> List[int]:
    """Three (or more) distinct probe depths up to `halo`: H, H/2, H/4."""
    return sorted({max(1, halo), max(1, halo // 2), max(1, halo // 4)})


def measure_exchange(solver, depths: Sequence[int], iters: int = 20, reps: int = 5,
                     agree_max: Optional[Callable[[float], float]] = None) -> List[tuple]:
    """(largest message bytes, seconds per grouped exchange) samples of
    `solver`'s halo exchange at each depth (<= its halo): `reps` samples of
    `iters` exchanges each, interleaved over the depths (a slow phase of the
    machine hits every size), timed on the real ranks; `agree_max` reduces a
    float to its max over the ranks (the slowest rank sets the pace).
    Collective.  Feed the samples to parallel.model.fit_exchange, which takes
    the median per size."""
    out = []
    ds = [max(1, min(int(d), solver.info.halo)) for d in depths]
    for _ in range(reps):
        for d in ds:
            t, b = solver.time_exchange(d, iters)
            if agree_max is not None:
                t = agree_max(t)
            out.append((b, t))
    return out


def is_clean_failure(e: BaseException) -> bool:
    """A run-time failure after which the rank's queued work completed and its
    communicator was kept (the native run() says "[clean]", only for
    heat::GlobalError, e.g. a non-finite all-reduced residual): every rank
    meets it at the same point, so the ranks can agree and go on."""
    return "[clean]" in str(e)


def autotune(cfg: HeatConfig, info: DistInfo, candidates: Optional[List[HeatConfig]] = None,
             steps: int = 1000, repeats: int = 3,
             make: Optional[Callable[[HeatConfig], object]] = None,
             log: Optional[Callable[[str], None]] = None,
             shared=None, vote_timeout_s: float = 180.0) -> Tuple[HeatConfig, List[dict]]:
    """Time every candidate (steps x repeats, after one untimed run of `steps`
    that captures the graphs) and return (fastest config, table).

    `make(cfg)` builds the solver (default: HeatSolver(cfg, dist_info=info,
    shared=shared)); pass `shared` (a parallel.comm.EngineTransport) so every
    candidate rides the same communicator instead of one ncclCommInitRank per
    candidate.  Collective over torch.distributed when info.world > 1: the
    ranks agree after construction, after the untimed run and after the timed
    runs (a gloo group with a `vote_timeout_s` timeout), so a candidate is
    skipped on every rank together when any rank

    * rejects it at construction,
    * fails at run time "cleanly" (the native run() drained its queued work
      and kept the communicator: an error class every rank meets at the same
      point, heat::GlobalError -- a non-finite all-reduced residual), or
    * reports a resident-tile give-up (HEAT_TB_RES_GIVEUP=defer: the run's
      results are invalid, its transport calls all matched).

    Any other run-time failure aborts the transport and the autotune (its
    peers may be waiting inside a send/recv that will never match); so does
    an agreement that times out (a peer stuck in such a wait)."""
    import datetime

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
    # Agreements go over a gloo group with a timeout: a rank whose peer is
    # stuck in an engine collective gives up instead of waiting forever.
    group = None
    if world > 1:
        group = dist.new_group(backend="gloo",
                               timeout=datetime.timedelta(seconds=vote_timeout_s))

    def agree_all(flag: float, op) -> float:
        if world == 1:
            return flag
        t = torch.tensor([flag], dtype=torch.float64)
        dist.all_reduce(t, op=op, group=group)
        return float(t.item())

    MIN = dist.ReduceOp.MIN if world > 1 else None
    MAX = dist.ReduceOp.MAX if world > 1 else None

    def sync():
        if gpu:
            torch.cuda.synchronize()

    table: List[dict] = []
    best, best_ms = None, float("inf")

    def attempt(solver, row, fn):
        """Run fn(); returns 1.0, or 0.0 after a clean failure / a resident
        give-up (recorded in row); raises after any other failure."""
        try:
            gave_up = fn()
            if gave_up:
                row["error"] = "resident tiles gave up a neighbour wait (results invalid)"
                return 0.0
            return 1.0
        except _native.NativeError as e:
            if is_clean_failure(e):
                row["error"] = str(e).splitlines()[0][:200]
                return 0.0
            # Peers may be inside a send / recv / all-reduce that will never
            # match, with unmatched ops queued on the shared communicator: no
            # later candidate may use it.  Abort it (their pending waits end
            # in their watchdog, HEAT_WATCHDOG_S) and end the autotune.
            try:
                solver.abort()
            finally:
                solver.close()
            raise _native.NativeError(
                f"autotune aborted: candidate {row} failed at run time on rank "
                f"{info.rank}: {str(e).splitlines()[0][:200]}") from e

    def agree_ok(solver, row, ok: float) -> bool:
        try:
            ok = agree_all(ok, MIN)
        except RuntimeError as e:  # the gloo agreement timed out
            try:
                solver.abort()
            finally:
                solver.close()
            raise _native.NativeError(f"autotune aborted: ranks did not agree on {row}: {e}") \
                from e
        if ok < 1.0:
            solver.close()
            row.setdefault("error", "failed on another rank")
            table.append(row)
            if log:
                log(f"autotune: {row} skipped")
            return False
        return True

    # The gloo group is destroyed on every exit (a raise included: bench.py
    # may call autotune again after a failure).
    try:
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
            # Untimed run (graph capture, RCCL connections); the agreement after
            # it is also the barrier before the timed runs.
            ok = attempt(solver, row, lambda: solver.run(steps).resident_giveups > 0)
            if not agree_ok(solver, row, ok):
                continue
            sync()
            t0 = time.perf_counter()

            def timed():
                g = 0
                for _ in range(repeats):
                    g += solver.run(steps).resident_giveups
                return g > 0

            ok = attempt(solver, row, timed)
            sync()
            dt = time.perf_counter() - t0
            if not agree_ok(solver, row, ok):
                continue
            row["halo"] = solver.info.halo
            row["tb_depth"] = solver.info.tb_depth
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
    finally:
        if group is not None:
            dist.destroy_process_group(group)
    if best is None:
        raise _native.NativeError("autotune: every candidate was rejected: %r" % table)
    return best, table

"""Timing and reporting.

Replaces ``cuda/timestamp.h`` (gettimeofday ms timer) and ``MPI_Wtime``
(``mpi/...c:88, :298``).  Timing here is always synchronised (the reference's
CUDA timer stops without a device sync).  Output lines reproduce the
reference's (``mpi/...c:90-96, :300-306``; ``cuda/cuda_heat.cu:254-260``), and
``metrics_json`` is the machine-readable line.
"""
from __future__ import annotations

import json
import time
from contextlib import contextmanager
from typing import Dict, Optional

import torch


class Timer:
    """Wall-clock timer that synchronises the GPU at start and stop."""

    def __init__(self, sync_cuda: bool = True):
        self.sync = sync_cuda and torch.cuda.is_available()
        self.t0 = 0.0
        self.elapsed = 0.0

    def __enter__(self):
        if self.sync:
            torch.cuda.synchronize()
        self.t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        if self.sync:
            torch.cuda.synchronize()
        self.elapsed = time.perf_counter() - self.t0


class PhaseTimes:
    """Accumulate named phase durations (init / run / output ...)."""

    def __init__(self):
        self.t: Dict[str, float] = {}

    @contextmanager
    def phase(self, name: str, sync_cuda: bool = False):
        if sync_cuda and torch.cuda.is_available():
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        try:
            yield
        finally:
            if sync_cuda and torch.cuda.is_available():
                torch.cuda.synchronize()
            self.t[name] = self.t.get(name, 0.0) + time.perf_counter() - t0


def mpi_banner(world: int, nx: int, ny: int, steps: int, converge: bool) -> str:
    s = f"Starting mpi_heat2D with {world} worker tasks.\n"
    if converge:
        s += f"Grid size: X= {nx}  Y= {ny}  Time steps= - \n"
    else:
        s += f"Grid size: X= {nx}  Y= {ny}  Time steps= {steps}\n"
    return s


def convergence_line(naming: str, converged: bool, converged_at: int, steps: int) -> str:
    if naming == "mpi":
        return f"Converged after {converged_at - 1} steps\n" if converged else "Didn't converged\n"
    if naming == "cuda":
        return f"Converged at {converged_at - 1} steps\n" if converged else "Did not converge\n"
    return (f"Converged after {converged_at} steps\n" if converged
            else f"Did not converge after {steps} steps\n")


def elapsed_line(naming: str, seconds: float) -> str:
    if naming == "cuda":
        ms = seconds * 1e3
        return ("Elapsed time: %.3f %ssecs\n" % (ms / 1000, "") if ms / 1000 > 1.0
                else "Elapsed time: %.3f %ssecs\n" % (ms, "m"))
    return "Elapsed time %f secs\n" % seconds


def metrics_json(**kw) -> str:
    return json.dumps(kw, sort_keys=False)


def cuda_output_name(nx: int, ny: int, steps: int) -> str:
    """out_cuda_<TPB>_<NB>_<STEPS>.dat with the reference's T=32 geometry (cuda/cuda_heat.cu:17-21)."""
    t = 32
    rb = (nx - 2) // t + (1 if (nx - 2) % t else 0)
    cb = (ny - 2) // t + (1 if (ny - 2) % t else 0)
    return f"out_cuda_{t * t}_{rb * cb}_{steps}.dat"


def roctx_range(name: str):
    """A roctx range if roctx is reachable through torch, else a no-op context."""
    try:
        from torch.cuda import nvtx  # routed to roctx on ROCm builds
        return nvtx.range(name)
    except Exception:  # pragma: no cover
        from contextlib import nullcontext
        return nullcontext()


def optional(v: Optional[float]) -> Optional[float]:
    return None if v is None else float(v)

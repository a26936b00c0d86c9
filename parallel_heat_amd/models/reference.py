"""Pure NumPy / PyTorch reference of the heat model (the test oracle).

Mirrors the reference programs' semantics:
  * ``inidat``  (``cuda/cuda_heat.cu:274-280``): u = ix*(nx-ix-1)*iy*(ny-iy-1) in int32
  * the 5-point update with fixed boundary (``cuda/cuda_heat.cu:57-65``,
    ``mpi/mpi_heat_improved_persistent_stat.c:166-174``)
  * the convergence test every C steps (``cuda/cuda_heat.cu:219-236``,
    ``mpi/...c:235-262``) with the canonical / mpi / cuda schedules.

The update here is evaluated in plain float32 (NumPy has no fused
multiply-add); the native engine evaluates the same expression with FMA, so
the two agree to within a few float32 ulps per step, not bitwise.
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np
import torch

_U64 = np.uint64


def _mix64(z: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = z + _U64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> _U64(30))) * _U64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> _U64(27))) * _U64(0x94D049BB133111EB)
        return z ^ (z >> _U64(31))


def init_grid(nx: int, ny: int, mode: str = "ref-wrap", seed: int = 0,
              ox: int = 0, oy: int = 0, lx: Optional[int] = None,
              ly: Optional[int] = None) -> np.ndarray:
    """Initial condition for the block [ox, ox+lx) x [oy, oy+ly) of an nx x ny plate."""
    lx = nx - ox if lx is None else lx
    ly = ny - oy if ly is None else ly
    ix = np.arange(ox, ox + lx, dtype=np.int64)[:, None]
    iy = np.arange(oy, oy + ly, dtype=np.int64)[None, :]
    if mode == "ref-wrap":
        with np.errstate(over="ignore"):
            a = (ix.astype(np.uint32) * (nx - ix - 1).astype(np.uint32))
            a = a * iy.astype(np.uint32)
            a = a * (ny - iy - 1).astype(np.uint32)
        return a.astype(np.uint32).view(np.int32).astype(np.float32)
    if mode in ("exact", "ref64"):
        return (ix.astype(np.float64) * (nx - ix - 1) * iy * (ny - iy - 1)).astype(np.float32)
    if mode == "random":
        s = _U64(seed)
        with np.errstate(over="ignore"):
            inner = _mix64(ix.astype(np.uint64) * _U64(0x9E3779B97F4A7C15) ^ iy.astype(np.uint64))
            h = _mix64(s * _U64(0xD1B54A32D192ED03) ^ inner)
        v = (h >> _U64(40)).astype(np.float32) * np.float32(1.0 / 16777216.0) * np.float32(100.0)
        return v.astype(np.float32)
    if mode == "zero":
        return np.zeros((lx, ly), np.float32)
    raise ValueError(mode)


def step_np(u: np.ndarray, cx: float = 0.1, cy: float = 0.1) -> np.ndarray:
    """One Jacobi step in float32; boundary ring unchanged."""
    u = np.asarray(u, np.float32)
    out = u.copy()
    if u.shape[0] < 3 or u.shape[1] < 3:
        return out
    c = u[1:-1, 1:-1]
    n, s = u[:-2, 1:-1], u[2:, 1:-1]
    w, e = u[1:-1, :-2], u[1:-1, 2:]
    two = np.float32(2.0)
    tx = (s + n) - two * c
    ty = (e + w) - two * c
    out[1:-1, 1:-1] = (c + np.float32(cx) * tx) + np.float32(cy) * ty
    return out


def step_np_mpi(u: np.ndarray, cx: float = 0.1, cy: float = 0.1) -> np.ndarray:
    """One step with the reference MPI program's arithmetic
    (mpi/mpi_heat_improved_persistent_stat.c:168-174): the two neighbour sums
    in float32 (float + float in C), the rest in float64 because of the 2.0
    literal, evaluated left to right, rounded to float32 once.  NumPy float64
    ops are IEEE and never fused, so this is the exact oracle of
    `numerics="mpi"`."""
    u = np.asarray(u, np.float32)
    out = u.copy()
    if u.shape[0] < 3 or u.shape[1] < 3:
        return out
    c = u[1:-1, 1:-1].astype(np.float64)
    ns = (u[2:, 1:-1] + u[:-2, 1:-1]).astype(np.float64)   # float32 add, then widen
    ew = (u[1:-1, 2:] + u[1:-1, :-2]).astype(np.float64)
    fcx, fcy = float(np.float32(cx)), float(np.float32(cy))  # parms are float
    a = c + fcx * (ns - 2.0 * c)
    out[1:-1, 1:-1] = (a + fcy * (ew - 2.0 * c)).astype(np.float32)
    return out


def step_torch(u: torch.Tensor, cx: float = 0.1, cy: float = 0.1) -> torch.Tensor:
    """The same step as plain PyTorch fp32 ops (any device)."""
    out = u.clone()
    if u.shape[0] < 3 or u.shape[1] < 3:
        return out
    c = u[1:-1, 1:-1]
    tx = (u[2:, 1:-1] + u[:-2, 1:-1]) - 2.0 * c
    ty = (u[1:-1, 2:] + u[1:-1, :-2]) - 2.0 * c
    out[1:-1, 1:-1] = (c + cx * tx) + cy * ty
    return out


def check_points(total: int, interval: int, compat: str = "none"):
    """Completed-step counts after which a convergence check happens."""
    if compat == "cuda":
        return [c for c in range(1, total + 1) if (c - 1) % interval == 0]
    return [c for c in range(1, total + 1) if c % interval == 0]


def run_np(nx: int, ny: int, steps: int, cx: float = 0.1, cy: float = 0.1,
           converge: bool = False, check_interval: int = 20, eps: float = 1e-3,
           compat: str = "none", init: str = "ref-wrap", seed: int = 0,
           u0: Optional[np.ndarray] = None,
           numerics: str = "fp32") -> Tuple[np.ndarray, int, int]:
    """Run the model; returns (grid, steps_done, converged_at or -1)."""
    step = step_np_mpi if numerics == "mpi" else step_np
    u = init_grid(nx, ny, init, seed) if u0 is None else np.array(u0, np.float32)
    total = steps + 1 if compat == "mpi" else steps
    checks = set(check_points(total, check_interval, compat)) if converge else set()
    for k in range(1, total + 1):
        v = step(u, cx, cy)
        if k in checks:
            r = float(np.max(np.abs(v - u))) if v.size else 0.0
            ok = r <= eps if compat == "mpi" else r < np.float32(eps)
            if ok:
                return v, k, k
        u = v
    return u, total, -1

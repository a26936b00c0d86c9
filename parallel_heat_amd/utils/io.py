"""Grid files.

* ``.dat`` text, byte-compatible with the reference's ``prtdat``
  (``cuda/cuda_heat.cu:285-300``, ``mpi/mpi_heat_improved_persistent_stat.c:326-341``):
  ``"%6.1f"`` values, one line per iy from ny-1 down to 0 (transposed and
  y-flipped), single spaces, newline at line end.
* ``.bin``: 72-byte header (magic ``HEATF32``, version, parity, nx, ny, step,
  cx, cy) + nx*ny float32 row-major; written by ``HeatSolver.save`` and used
  for checkpoints.
"""
from __future__ import annotations

import ctypes
import struct
from typing import Tuple

import numpy as np

from .. import _native

BIN_HEADER = struct.Struct("<8sIIqqqff24x")
assert BIN_HEADER.size == 72


def format_value(v: float) -> str:
    """Python rendering of printf("%6.1f", v) (used to cross-check the native formatter)."""
    return "%6.1f" % float(np.float32(v))


def write_dat(path: str, grid: np.ndarray) -> None:
    """Write an (nx, ny) grid in prtdat format with the native writer."""
    g = np.ascontiguousarray(grid, dtype=np.float32)
    nx, ny = g.shape
    _native.call("heat_write_dat", str(path).encode(), nx, ny, g.ctypes.data)


def write_dat_py(path: str, grid: np.ndarray) -> None:
    """Pure-Python prtdat writer (independent oracle for tests)."""
    g = np.asarray(grid, dtype=np.float32)
    nx, ny = g.shape
    with open(path, "w") as f:
        for iy in range(ny - 1, -1, -1):
            f.write(" ".join("%6.1f" % float(g[ix, iy]) for ix in range(nx)) + "\n")


def read_dat(path: str) -> np.ndarray:
    """Read a prtdat file back into an (nx, ny) grid of the printed values."""
    with open(path) as f:
        rows = [list(map(float, line.split())) for line in f if line.strip()]
    a = np.array(rows, dtype=np.float32)  # (ny, nx), iy descending
    return np.ascontiguousarray(a[::-1].T)


def native_format(v: float) -> str:
    buf = ctypes.create_string_buffer(64)
    _native.call("heat_format_6_1f", ctypes.c_float(v), buf, 64)
    return buf.value.decode()


def read_bin_header(path: str) -> dict:
    with open(path, "rb") as f:
        magic, ver, parity, nx, ny, step, cx, cy = BIN_HEADER.unpack(f.read(72))
    if magic != b"HEATF32\0" or ver != 1:
        raise ValueError(f"{path} is not a heat binary grid")
    return {"nx": nx, "ny": ny, "step": step, "parity": parity, "cx": cx, "cy": cy}


def read_bin(path: str, mmap: bool = True) -> Tuple[np.ndarray, dict]:
    """(grid, header) of a binary grid file; memory-mapped by default."""
    h = read_bin_header(path)
    if mmap:
        g = np.memmap(path, dtype=np.float32, mode="r", offset=72, shape=(h["nx"], h["ny"]))
    else:
        g = np.fromfile(path, dtype=np.float32, offset=72).reshape(h["nx"], h["ny"])
    return g, h


def write_bin(path: str, grid: np.ndarray, step: int = 0, cx: float = 0.1,
              cy: float = 0.1) -> None:
    g = np.ascontiguousarray(grid, dtype=np.float32)
    with open(path, "wb") as f:
        f.write(BIN_HEADER.pack(b"HEATF32\0", 1, 0, g.shape[0], g.shape[1], step, cx, cy))
        g.tofile(f)

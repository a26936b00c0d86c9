"""ctypes binding of ``libheat.so`` (the native C++/HIP engine, ``csrc/``).

The shared library is built in-tree by ``make`` (see ``Makefile`` or
``parallel_heat_amd.build_native()``) into ``parallel_heat_amd/_lib/``.  It is
loaded after ``torch`` so that it binds to the HIP runtime and RCCL that torch
already loaded (same sonames ``libamdhip64.so.7`` / ``librccl.so.1``): one HIP
runtime per process.

On a machine with a GPU a missing library is a hard error (no silent
fallback); on a CPU-only machine the package still imports, and only the
functions that need the library raise.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import threading
from ctypes import (POINTER, Structure, c_char_p, c_double, c_float, c_int, c_int32, c_int64,
                    c_uint, c_uint8, c_uint64, c_void_p)
from pathlib import Path

import torch  # noqa: F401  (must be imported before libheat: shared HIP runtime)

ABI_VERSION = 5  # must match HEAT_ABI_VERSION in csrc/include/heat/capi.h

PKG_DIR = Path(__file__).resolve().parent
REPO_DIR = PKG_DIR.parent
# HEAT_LIB: another build of the engine (kernel A/B timing in one tree).
LIB_PATH = Path(os.environ["HEAT_LIB"]) if os.environ.get("HEAT_LIB") else PKG_DIR / "_lib" / "libheat.so"
CLI_PATH = REPO_DIR / "build" / "heat"

_lock = threading.Lock()
_lib = None


class NativeError(RuntimeError):
    """An error reported by the native engine."""


class HeatParams(Structure):
    _fields_ = [
        ("nx", c_int64), ("ny", c_int64),
        ("cx", c_float), ("cy", c_float),
        ("converge", c_int32), ("check_interval", c_int32),
        ("eps", c_double),
        ("init", c_int32),
        ("seed", c_uint64),
        ("backend", c_int32), ("kernel", c_int32), ("tb_depth", c_int32), ("threads", c_int32),
        ("decomp", c_int32), ("px", c_int32), ("py", c_int32),
        ("use_graph", c_int32), ("overlap", c_int32),
        ("compat", c_int32), ("device", c_int32),
        ("schedule", c_int32), ("halo_passes", c_int32),
        ("numerics", c_int32), ("phase_timing", c_int32),
    ]


SENDRECV_CB = ctypes.CFUNCTYPE(c_int, c_void_p, c_void_p, c_int)
ALLREDUCE_CB = ctypes.CFUNCTYPE(c_int, c_void_p, c_void_p, c_int, c_int)
BARRIER_CB = ctypes.CFUNCTYPE(c_int, c_void_p)


class HeatComm(Structure):
    _fields_ = [
        ("kind", c_int32), ("rank", c_int32), ("world", c_int32), ("device", c_int32),
        ("unique_id", c_uint8 * 128),
        ("addr", c_char_p), ("port", c_int32),
        ("ctx", c_void_p),
        ("sendrecv", SENDRECV_CB), ("allreduce", ALLREDUCE_CB), ("barrier", BARRIER_CB),
    ]


class HeatMsg(Structure):
    _fields_ = [("peer", c_int), ("sbuf", c_void_p), ("sbytes", ctypes.c_size_t),
                ("rbuf", c_void_p), ("rbytes", ctypes.c_size_t)]


class HeatRunStats(Structure):
    _fields_ = [
        ("steps_done", c_int64), ("total_steps", c_int64),
        ("converged", c_int32), ("converged_at", c_int64),
        ("last_resid", c_float), ("seconds", c_double),
        ("passes", c_int64), ("exchanges", c_int64), ("checks", c_int64),
        ("t_exchange", c_double), ("t_compute", c_double), ("t_reduce", c_double),
        ("resident_passes", c_int64), ("resident_giveups", c_int64),
        ("chained_passes", c_int64),
    ]


class HeatBlockInfo(Structure):
    _fields_ = [
        ("rank", c_int32), ("world", c_int32), ("px", c_int32), ("py", c_int32),
        ("cx", c_int32), ("cy", c_int32),
        ("ox", c_int64), ("oy", c_int64), ("lx", c_int64), ("ly", c_int64),
        ("nbr", c_int32 * 4),
        ("pitch", c_int64), ("rows", c_int64),
        ("hx", c_int32), ("hy", c_int32), ("halo", c_int32), ("tb_depth", c_int32),
        ("bytes_per_field", c_int64),
        ("schedule", c_int32), ("pad_", c_int32),
    ]


class HeatTransportInfo(Structure):
    _fields_ = [("nranks", c_int32), ("device", c_int32), ("user_rank", c_int32),
                ("bus_id", ctypes.c_char * 32), ("name", ctypes.c_char * 16)]


class HeatTbTuning(Structure):
    _fields_ = [("variant", c_int32), ("rounds", c_int32), ("min_len", c_int32),
                ("waves", c_int32), ("edge_frac", c_double), ("n_weights", c_int32),
                ("tile_rows", c_int32), ("weights", c_double * 4), ("tile_waves", c_int32),
                ("tile_xl", c_int32), ("nt", c_int32), ("pad_", c_int32)]


class HeatChecksum(Structure):
    _fields_ = [("hash", c_uint64), ("sum", c_double), ("min", c_double), ("max", c_double),
                ("count", c_int64)]


_SIGS = {
    "heat_last_error": (c_char_p, []),
    "heat_abi_version": (c_int, []),
    "heat_build_info": (c_char_p, []),
    "heat_rccl_unique_id": (c_int, [POINTER(c_uint8)]),
    "heat_device_count": (c_int, [POINTER(c_int)]),
    "heat_solver_create": (c_int, [POINTER(HeatParams), POINTER(HeatComm), POINTER(c_void_p)]),
    "heat_solver_destroy": (c_int, [c_void_p]),
    "heat_transport_create": (c_int, [POINTER(HeatComm), POINTER(c_void_p)]),
    "heat_transport_destroy": (c_int, [c_void_p]),
    "heat_transport_info_get": (c_int, [c_void_p, POINTER(HeatTransportInfo)]),
    "heat_solver_create_shared": (c_int, [POINTER(HeatParams), c_void_p, POINTER(c_void_p)]),
    "heat_solver_run": (c_int, [c_void_p, c_int64, POINTER(HeatRunStats)]),
    "heat_solver_enqueue": (c_int, [c_void_p, c_int64, POINTER(HeatRunStats)]),
    "heat_loopback_hub_create": (c_int, [c_int, POINTER(c_void_p)]),
    "heat_rccl_self_test": (c_int, [c_int, c_int64, c_int, c_int, POINTER(c_double)]),
    "heat_rccl_abort_race_test": (c_int, [c_int, c_int, POINTER(c_int)]),
    "heat_loopback_hub_destroy": (c_int, [c_void_p]),
    "heat_loopback_hub_fail": (c_int, [c_void_p]),
    "heat_solver_reset": (c_int, [c_void_p]),
    "heat_solver_info": (c_int, [c_void_p, POINTER(HeatBlockInfo)]),
    "heat_solver_step": (c_int, [c_void_p, POINTER(c_int64)]),
    "heat_solver_copy_owned": (c_int, [c_void_p, c_void_p, c_int64]),
    "heat_solver_load_owned": (c_int, [c_void_p, c_void_p, c_int64, c_int64]),
    "heat_solver_gather": (c_int, [c_void_p, c_void_p]),
    "heat_solver_checksum": (c_int, [c_void_p, POINTER(HeatChecksum)]),
    "heat_solver_scatter": (c_int, [c_void_p, c_void_p, c_int64]),
    "heat_solver_write_bin": (c_int, [c_void_p, c_char_p]),
    "heat_solver_read_bin": (c_int, [c_void_p, c_char_p]),
    "heat_solver_barrier": (c_int, [c_void_p]),
    "heat_solver_current_ptr": (c_int, [c_void_p, POINTER(c_void_p)]),
    "heat_write_dat": (c_int, [c_char_p, c_int64, c_int64, c_void_p]),
    "heat_format_6_1f": (c_int, [c_float, c_char_p, c_int]),
    "heat_dims_create": (c_int, [c_int, c_int, POINTER(c_int)]),
    "heat_block_span": (c_int, [c_int64, c_int, c_int, POINTER(c_int64), POINTER(c_int64)]),
    "heat_init_value": (c_int, [c_int, c_int64, c_int64, c_int64, c_int64, c_uint64,
                                POINTER(c_float)]),
    "heat_cpu_step": (c_int, [c_void_p, c_void_p, c_int64, c_int64, c_int64, c_int64, c_int64,
                              c_float, c_float, c_int64, c_int64, c_int64, c_int64,
                              POINTER(c_float)]),
    "heat_op_naive_step": (c_int, [c_void_p, c_void_p, c_int64, c_int64, c_int64, c_int64,
                                   c_int64, c_float, c_float, c_int64, c_int64, c_int64, c_int64,
                                   c_void_p, c_void_p]),
    "heat_op_lds_step": (c_int, [c_void_p, c_void_p, c_int64, c_int64, c_int64, c_int64,
                                 c_int64, c_float, c_float, c_int64, c_int64, c_int64, c_int64,
                                 c_void_p, c_void_p, c_int]),
    "heat_op_mfma_step": (c_int, [c_void_p, c_void_p, c_int64, c_int64, c_int64, c_int64,
                                  c_int64, c_float, c_float, c_int64, c_int64, c_int64, c_int64,
                                  c_void_p, c_void_p]),
    "heat_op_tb_step": (c_int, [c_void_p, c_void_p, c_int64, c_int64, c_int64, c_int64, c_int64,
                                c_float, c_float, POINTER(c_int64), c_int, c_int, c_void_p,
                                c_void_p, c_int, c_int, c_int]),
    "heat_tb_get_tuning": (c_int, [POINTER(HeatTbTuning)]),
    "heat_tb_set_tuning": (c_int, [POINTER(HeatTbTuning)]),
    "heat_op_tb_stamps": (c_int, [c_void_p, c_int64]),
    "heat_op_init": (c_int, [c_void_p, c_int64, c_int64, c_int, c_int64, c_int64, c_int64,
                             c_int64, c_int, c_uint64, c_void_p]),
    "heat_op_pack": (c_int, [c_void_p, c_int64, c_int64, c_int64, c_int64, c_int64, c_void_p,
                             c_void_p]),
    "heat_op_unpack": (c_int, [c_void_p, c_void_p, c_int64, c_int64, c_int64, c_int64, c_int64,
                               c_void_p]),
    "heat_op_residual": (c_int, [c_void_p, c_void_p, c_int64, c_int64, c_int64, c_int64,
                                 c_int64, c_void_p, c_void_p]),
    "heat_layout": (c_int, [c_int64, c_int64, c_int, POINTER(c_int64), POINTER(c_int64),
                            POINTER(c_int), POINTER(c_int)]),
    "heat_tb_supported": (c_int, [c_int]),
    "heat_tb_exp_loaded": (c_int, []),
    "heat_register_exp_kernels": (None, [c_void_p]),
    "heat_resident_shape": (c_int, [c_int64, c_int64, c_int, c_int, POINTER(c_int32)]),
    "heat_tb_mid_residual": (c_int, [c_int]),
    "heat_group_transport": (c_int, [ctypes.c_char_p, c_int, POINTER(c_int32), POINTER(c_int32)]),
    "heat_solver_abort": (c_int, [c_void_p]),
    "heat_solver_time_exchange": (c_int, [c_void_p, c_int, c_int, POINTER(c_double),
                                          POINTER(c_int64)]),
}


def build_native(jobs: int = 8, quiet: bool = True) -> None:
    """Compile libheat.so, the ``heat`` CLI and the experiment kernels
    (libheat_exp.so) for gfx950 with hipcc (``make all exp``)."""
    cmd = ["make", f"-j{jobs}", "-C", str(REPO_DIR), "all", "exp"]
    res = subprocess.run(cmd, capture_output=quiet, text=True)
    if res.returncode != 0:
        raise NativeError("native build failed:\n" + (res.stdout or "") + (res.stderr or ""))


def _gpu_present() -> bool:
    try:
        return torch.cuda.device_count() > 0
    except Exception:  # pragma: no cover
        return False


def lib():
    """Return the loaded native library (building it on first use if absent)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not LIB_PATH.exists():
            if os.environ.get("HEAT_NO_AUTOBUILD"):
                raise NativeError(f"{LIB_PATH} is missing (HEAT_NO_AUTOBUILD set)")
            build_native()
        if not LIB_PATH.exists():
            raise NativeError(f"{LIB_PATH} is missing and could not be built")
        L = ctypes.CDLL(str(LIB_PATH))
        for name, (res, args) in _SIGS.items():
            # An older build (HEAT_LIB A/Bs) may lack a newer entry point: it
            # stays unbound, and only calling it fails.
            fn = getattr(L, name, None)
            if fn is None:
                continue
            fn.restype = res
            fn.argtypes = args
        if L.heat_abi_version() != ABI_VERSION:
            raise NativeError("libheat ABI mismatch; rebuild with `make`")
        _lib = L
    if os.environ.get("HEAT_EXP", "") not in ("", "0"):
        load_exp()
    return _lib


# The experiment kernels (csrc/kernels/tb_exp.hpp; `make exp`): TB builds
# measured slower than the defaults, kept out of the product library and
# registered with it when this one is loaded (HEAT_EXP=1, or load_exp()).
EXP_PATH = LIB_PATH.parent / "libheat_exp.so"
_exp = None


def load_exp():
    """Load libheat_exp.so next to the product library: its kernels (packed
    and float2 single-wave builds, mixed-shift and packed split builds,
    chained passes) become available to tb_step and the solver."""
    global _exp
    lib()
    with _lock:
        if _exp is None:
            if not EXP_PATH.exists():
                raise NativeError(f"{EXP_PATH} is missing: build it with `make exp`")
            _exp = ctypes.CDLL(str(EXP_PATH))
        _exp.heat_exp_register()  # (again, after an unload_exp())
    return _exp


def unload_exp() -> None:
    """Unregister the experiment kernels (the library stays mapped): launches
    that need one fail again, as in a process that never loaded them."""
    L = lib()
    L.heat_register_exp_kernels(None)


def available() -> bool:
    try:
        lib()
        return True
    except Exception:
        return False


def check(rc: int) -> None:
    if rc != 0:
        msg = lib().heat_last_error()
        raise NativeError(msg.decode() if msg else "native error")


def call(name: str, *args):
    check(getattr(lib(), name)(*args))


def loaded_path() -> str:
    lib()
    return str(LIB_PATH)


def device_count() -> int:
    n = c_int(0)
    call("heat_device_count", ctypes.byref(n))
    return n.value


def require_gpu_native() -> None:
    """On a GPU machine the HIP path must be the one that runs: fail loudly."""
    if _gpu_present():
        lib()


def rccl_unique_id() -> bytes:
    buf = (c_uint8 * 128)()
    call("heat_rccl_unique_id", buf)
    return bytes(buf)


__all__ = [
    "HeatParams", "HeatComm", "HeatMsg", "HeatTransportInfo", "HeatTbTuning", "HeatRunStats", "HeatBlockInfo", "HeatChecksum",
    "SENDRECV_CB", "ALLREDUCE_CB", "BARRIER_CB", "NativeError", "lib", "call", "check",
    "available", "build_native", "loaded_path", "device_count", "rccl_unique_id",
    "require_gpu_native", "LIB_PATH", "CLI_PATH", "c_uint", "EXP_PATH", "load_exp", "unload_exp",
]

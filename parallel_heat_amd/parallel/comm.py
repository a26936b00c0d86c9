"""Process-group plumbing: one process per GPU with ``torch.distributed``.

The reference bootstraps with ``MPI_Init`` / ``MPI_Comm_size`` /
``MPI_Comm_rank`` (``mpi/mpi_heat_improved_persistent_stat.c:48-50``).  Here
the launcher is ``python -m torch.distributed.run`` (or anything that sets
RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR / MASTER_PORT) and the native
engine gets one of these transports:

* ``local``     single rank, no messages.
* ``rccl``      the native engine's own RCCL communicator over xGMI (GPU fast
                path: grouped ncclSend/ncclRecv halos and ncclAllReduce(max),
                stream-ordered and captured in hipGraphs).  Its 128-byte unique
                id is created on rank 0 and broadcast with torch.distributed.
* ``torch``     the native engine calls back into Python and the messages go
                through ``torch.distributed`` (gloo on CPU).  Used for CPU
                multi-process runs and tests, and for GPU runs whose halos are
                staged through pinned host memory (several ranks sharing one GPU).
* ``tcp``       the engine's own TCP transport (what the standalone ``heat``
                binary uses for CPU ranks).
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np
import torch
import torch.distributed as dist

from .. import _native


@dataclass
class DistInfo:
    rank: int = 0
    world: int = 1
    local_rank: int = 0

    @property
    def is_root(self) -> bool:
        return self.rank == 0


def env_info() -> DistInfo:
    return DistInfo(int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
                    int(os.environ.get("LOCAL_RANK", os.environ.get("RANK", 0))))


def init_distributed(backend: Optional[str] = None) -> DistInfo:
    """Initialise torch.distributed from the launcher's environment (idempotent)."""
    info = env_info()
    if info.world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            torch.cuda.set_device(info.local_rank % max(1, torch.cuda.device_count()))
        dist.init_process_group(backend=backend)
    if dist.is_initialized():
        info = DistInfo(dist.get_rank(), dist.get_world_size(), info.local_rank)
    return info


def _np_view(ptr: int, nbytes: int, dtype=np.uint8) -> np.ndarray:
    buf = (ctypes.c_uint8 * nbytes).from_address(ptr)
    return np.frombuffer(buf, dtype=dtype)


class TorchDistTransport:
    """Callback transport: the native engine's messages over torch.distributed.

    Works with any backend that supports CPU tensors for send/recv and
    all_reduce (gloo).  Buffers are host memory owned by the engine.
    """

    def __init__(self, group=None):
        if not dist.is_initialized():
            raise RuntimeError("torch.distributed is not initialised")
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self._error: Optional[BaseException] = None
        # Keep the ctypes callbacks alive as long as this object.
        self._cb_sendrecv = _native.SENDRECV_CB(self._sendrecv)
        self._cb_allreduce = _native.ALLREDUCE_CB(self._allreduce)
        self._cb_barrier = _native.BARRIER_CB(self._barrier)

    def _sendrecv(self, ctx, msgs_ptr, n):
        try:
            msgs = ctypes.cast(msgs_ptr, ctypes.POINTER(_native.HeatMsg))
            reqs = []
            for i in range(n):
                m = msgs[i]
                if m.rbytes:
                    t = torch.from_numpy(_np_view(m.rbuf, m.rbytes))
                    reqs.append(dist.irecv(t, src=m.peer, group=self.group))
            for i in range(n):
                m = msgs[i]
                if m.sbytes:
                    t = torch.from_numpy(_np_view(m.sbuf, m.sbytes).copy())
                    reqs.append(dist.isend(t, dst=m.peer, group=self.group))
            for r in reqs:
                r.wait()
            return 0
        except BaseException as e:  # never let an exception cross the C boundary
            self._error = e
            return -1

    def _allreduce(self, ctx, buf, count, dtype):
        try:
            if dtype == 0:
                a = _np_view(buf, 4 * count, np.float32)
                op = dist.ReduceOp.MAX
            elif dtype == 1:
                a = _np_view(buf, 8 * count, np.float64)
                op = dist.ReduceOp.SUM
            else:  # uint64 sum == int64 sum bit pattern (two's complement)
                a = _np_view(buf, 8 * count, np.int64)
                op = dist.ReduceOp.SUM
            t = torch.from_numpy(a)
            dist.all_reduce(t, op=op, group=self.group)
            return 0
        except BaseException as e:
            self._error = e
            return -1

    def _barrier(self, ctx):
        try:
            dist.barrier(group=self.group)
            return 0
        except BaseException as e:
            self._error = e
            return -1

    def fill(self, comm: _native.HeatComm) -> None:
        comm.kind = 3
        comm.rank = self.rank
        comm.world = self.world
        comm.sendrecv = self._cb_sendrecv
        comm.allreduce = self._cb_allreduce
        comm.barrier = self._cb_barrier


def group_transport(requested: str, devices: Sequence[int]) -> str:
    """Transport of a single-process multi-rank run with rank r on devices[r]:
    "rccl" when every rank has a GPU of its own, "loopback" when ranks share
    one ("auto"); "rccl" / "loopback" force one.  The native rule
    (heat::choose_group_transport) that `heat --gpus N` uses too."""
    arr = (ctypes.c_int32 * len(devices))(*[int(d) for d in devices])
    kind = ctypes.c_int32(0)
    _native.call("heat_group_transport", requested.encode(), len(devices), arr,
                 ctypes.byref(kind))
    return {1: "rccl", 4: "loopback"}[kind.value]


def broadcast_bytes(data: Optional[bytes], src: int = 0) -> bytes:
    """Broadcast a small byte string from `src` over the default process group."""
    obj = [data]
    dist.broadcast_object_list(obj, src=src)
    return obj[0]


class LoopbackHub:
    """Native hub of the loopback transport: `world` ranks that are threads of
    this process (see csrc/src/transport_loopback.cpp)."""

    def __init__(self, world: int):
        h = ctypes.c_void_p()
        _native.call("heat_loopback_hub_create", int(world), ctypes.byref(h))
        self.world = world
        self.handle = h

    def fail(self) -> None:
        """A rank failed: its peers' pending and future exchanges raise."""
        if self.handle:
            _native.call("heat_loopback_hub_fail", self.handle)

    def close(self) -> None:
        if self.handle:
            _native.call("heat_loopback_hub_destroy", self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def make_comm(kind: str, info: DistInfo, device: int = 0, addr: Optional[str] = None,
              port: Optional[int] = None, hub: Optional[LoopbackHub] = None, group=None,
              rccl_uid: Optional[bytes] = None):
    """Build a native HeatComm (and the Python object that must outlive it).

    `group`: torch.distributed process group of the ``torch`` transport
    (default: the default group; it must support CPU tensors, e.g. gloo).
    `rccl_uid`: the RCCL unique id, when the ranks are threads of one process
    that already share it (parallel.group.run_group); otherwise rank 0 makes
    one and torch.distributed broadcasts it."""
    comm = _native.HeatComm()
    keep = None
    if kind == "loopback":
        if hub is None:
            raise ValueError("the loopback transport needs a LoopbackHub")
        comm.kind = 4
        comm.rank, comm.world, comm.device = info.rank, hub.world, device
        comm.ctx = hub.handle
        keep = hub
    elif info.world == 1 or kind == "local":
        comm.kind = 0
        comm.rank, comm.world = 0, 1
    elif kind == "rccl":
        if rccl_uid is not None:
            uid = rccl_uid
        else:
            uid = _native.rccl_unique_id() if info.rank == 0 else None
            uid = broadcast_bytes(uid)
        comm.kind = 1
        comm.rank, comm.world, comm.device = info.rank, info.world, device
        ctypes.memmove(comm.unique_id, uid, 128)
    elif kind == "torch":
        keep = TorchDistTransport(group)
        keep.fill(comm)
    elif kind == "tcp":
        comm.kind = 2
        comm.rank, comm.world = info.rank, info.world
        a = addr or os.environ.get("MASTER_ADDR", "127.0.0.1")
        keep = a.encode()
        comm.addr = keep
        comm.port = int(port or int(os.environ.get("MASTER_PORT", 29599)) + 1)
    else:
        raise ValueError(f"unknown transport {kind!r}")
    return comm, keep


class EngineTransport:
    """One native transport that several solvers use in turn.

    ``bench.py``'s multi-GPU autotune builds a solver per candidate layout;
    with a shared transport they all ride ONE RCCL communicator (one
    ncclCommInitRank per rank per run, its P2P connections made once) instead
    of one per candidate.  Collective: every rank constructs it with the same
    kind.  Each solver keeps its own reference to the native object, so
    ``close()`` is safe while solvers are alive."""

    def __init__(self, kind: str, info: DistInfo, device: int = 0, hub: Optional[LoopbackHub] = None,
                 group=None):
        self.kind = kind
        self.device = device
        self._comm, self._keep = make_comm(kind, info, device=device, hub=hub, group=group)
        h = ctypes.c_void_p()
        _native.call("heat_transport_create", ctypes.byref(self._comm), ctypes.byref(h))
        self.handle = h

    def info(self) -> dict:
        """The transport's own view: for RCCL ncclCommCount / ncclCommCuDevice /
        ncclCommUserRank and the device's PCI bus id."""
        i = _native.HeatTransportInfo()
        _native.call("heat_transport_info_get", self.handle, ctypes.byref(i))
        return {"name": i.name.decode(), "nranks": i.nranks, "device": i.device,
                "user_rank": i.user_rank, "bus_id": i.bus_id.decode()}

    def close(self) -> None:
        if getattr(self, "handle", None):
            _native.call("heat_transport_destroy", self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

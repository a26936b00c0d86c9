"""Several ranks in one process: one host thread per rank.

This is the single-process multi-GPU mode (one process owning N
GPUs, the reference's ``MPI_Init`` world of ``mpi/mpi_heat_improved_persistent_stat.c:48-69``)
and the way the device-memory exchange path runs with real concurrency on ONE
GPU.  The transport follows the native rule that ``heat --gpus N`` uses too
(``heat::choose_group_transport``, ``parallel.comm.group_transport``):

* every rank on a GPU of its own: **RCCL**, one communicator rank per thread
  from one unique id (the ``ncclCommInitAll`` model), hipGraph-captured
  exchanges;
* ranks sharing a device: the **loopback** transport (device buffers,
  stream-ordered D2D / peer copies), since RCCL refuses two ranks per device.

    results = run_group(HeatConfig(nx=8192, ny=8192, steps=1000), world=4,
                        fn=lambda s: (s.run(), s.gather()))
"""
from __future__ import annotations

import threading
from typing import Callable, List, Optional, Sequence

from .. import _native
from ..models.config import HeatConfig
from ..models.heat2d import HeatSolver
from . import comm as pcomm


def default_devices(config: HeatConfig, world: int) -> List[int]:
    """Rank r's GPU: config.device for every rank if set, else r % visible GPUs."""
    if config.device >= 0:
        return [config.device] * world
    n = max(1, _native.device_count())
    return [r % n for r in range(world)]


def run_group(config: HeatConfig, world: int, fn: Callable[[HeatSolver], object],
              devices: Optional[Sequence[int]] = None,
              transport: str = "auto") -> List[object]:
    """Run `fn(solver)` on `world` ranks (threads); returns the per-rank results.

    `devices[r]` is rank r's GPU (default: default_devices).  `transport`:
    "auto" (RCCL with a GPU per rank, else loopback), "rccl" or "loopback".
    Every rank must make the same sequence of collective calls (run, gather,
    checksum, ...), as with one process per rank."""
    if config.backend != "hip":
        raise ValueError("single-process groups need backend='hip'")
    devices = list(devices) if devices is not None else default_devices(config, world)
    if len(devices) != world:
        raise ValueError(f"{len(devices)} devices for {world} ranks")
    kind = pcomm.group_transport(transport, devices)
    hub = pcomm.LoopbackHub(world) if kind == "loopback" else None
    uid = _native.rccl_unique_id() if kind == "rccl" else None
    results: List[object] = [None] * world
    errors: List[Optional[BaseException]] = [None] * world
    solvers: List[Optional[HeatSolver]] = [None] * world
    # One lock per rank guards that rank's slot for the whole of an abort: a
    # rank clears its slot (under its lock) before its solver is closed, so
    # an abort from a failing peer never runs on a solver being destroyed
    # (ctypes drops the GIL in both native calls).
    locks = [threading.Lock() for _ in range(world)]

    def fail_peers(rank: int) -> None:
        # Unblock the peers, which would wait forever for this rank's
        # messages: loopback peers raise "a peer rank failed"; RCCL peers have
        # their communicators aborted (their waits raise "run aborted").  The
        # native abort takes no lock a blocked peer call holds.
        if hub is not None:
            hub.fail()
            return
        for r in range(world):
            if r == rank:
                continue
            with locks[r]:
                s = solvers[r]
                if s is None:
                    continue
                try:
                    s.abort()
                except Exception:  # noqa: BLE001 - best effort
                    pass

    def body(rank: int) -> None:
        try:
            info = pcomm.DistInfo(rank, world, rank)
            with HeatSolver(config, transport=kind, dist_info=info, device=devices[rank],
                            hub=hub, rccl_uid=uid) as s:
                with locks[rank]:
                    solvers[rank] = s
                try:
                    results[rank] = fn(s)
                finally:
                    with locks[rank]:
                        solvers[rank] = None
        except BaseException as e:  # noqa: BLE001 - re-raised in the caller
            errors[rank] = e
            fail_peers(rank)

    threads = [threading.Thread(target=body, args=(r,), name=f"heat-rank{r}")
               for r in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    if hub is not None:
        hub.close()
    # Report the first failure, not the peers' echoes.
    failed = [(r, e) for r, e in enumerate(errors) if e is not None]
    if failed:
        echo = ("a peer rank failed", "run aborted", "communicator was aborted")
        own = [(r, e) for r, e in failed if not any(x in str(e) for x in echo)]
        r, e = (own or failed)[0]
        raise RuntimeError(f"rank {r} failed: {e}") from e
    return results

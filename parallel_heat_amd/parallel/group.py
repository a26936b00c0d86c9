"""Several ranks in one process: one host thread per rank over the loopback
transport (device buffers, stream-ordered D2D / peer copies).

This is the single-process multi-GPU mode (ranks on devices 0..N-1) and the
way the device-memory exchange path runs with real concurrency on ONE GPU,
where RCCL refuses two ranks ("decomposition invariance (1 GPU)").

    results = run_group(HeatConfig(nx=8192, ny=8192, steps=1000), world=4,
                        fn=lambda s: (s.run(), s.gather()))
"""
from __future__ import annotations

import threading
from typing import Callable, List, Optional, Sequence

from ..models.config import HeatConfig
from ..models.heat2d import HeatSolver
from . import comm as pcomm


def run_group(config: HeatConfig, world: int, fn: Callable[[HeatSolver], object],
              devices: Optional[Sequence[int]] = None) -> List[object]:
    """Run `fn(solver)` on `world` ranks (threads); returns the per-rank results.

    `devices[r]` is rank r's GPU (default: all on device 0, or config.device).
    Every rank must make the same sequence of collective calls (run, gather,
    checksum, ...), as with one process per rank."""
    if config.backend != "hip":
        raise ValueError("the loopback transport needs backend='hip'")
    hub = pcomm.LoopbackHub(world)
    if devices is None:
        devices = [max(config.device, 0)] * world
    results: List[object] = [None] * world
    errors: List[Optional[BaseException]] = [None] * world

    def body(rank: int) -> None:
        try:
            info = pcomm.DistInfo(rank, world, rank)
            with HeatSolver(config, transport="loopback", dist_info=info,
                            device=devices[rank], hub=hub) as s:
                results[rank] = fn(s)
        except BaseException as e:  # noqa: BLE001 - re-raised in the caller
            errors[rank] = e
            # Unblock the peers (they would wait forever for this rank's
            # messages); they raise "a peer rank failed" in turn.
            hub.fail()

    threads = [threading.Thread(target=body, args=(r,), name=f"heat-rank{r}")
               for r in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    hub.close()
    # Report the first failure, not the peers' "a peer rank failed" echoes.
    failed = [(r, e) for r, e in enumerate(errors) if e is not None]
    if failed:
        own = [(r, e) for r, e in failed if "a peer rank failed" not in str(e)]
        r, e = (own or failed)[0]
        raise RuntimeError(f"rank {r} failed: {e}") from e
    return results

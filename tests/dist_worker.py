"""Multi-process worker used by the distributed tests (gloo on CPU, or one
shared GPU with host-staged halos)."""
import os
import socket
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def rccl_host_per_rank(rank):
    """Let several RCCL ranks share one GPU: each rank claims its own host id,
    so RCCL's duplicate-device check passes and the ranks talk over its socket
    transport on loopback (same hook as bench.py's HEAT_RCCL_HOST_PER_RANK)."""
    os.environ.update(NCCL_HOSTID=f"heat-rank-{rank}", NCCL_SOCKET_IFNAME="lo",
                      NCCL_IB_DISABLE="1")


def worker(rank, world, port, cfg_kwargs, steps, out_path, transport, chunks, env=None):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    os.environ.update(env or {})
    if transport == "rccl":
        rccl_host_per_rank(rank)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from parallel_heat_amd import HeatConfig, HeatSolver
    from parallel_heat_amd.parallel.comm import DistInfo

    cfg = HeatConfig(**cfg_kwargs)
    group = None
    if transport == "torch_subgroup":  # bench.py's fallback: an explicit gloo group
        transport, group = "torch", dist.new_group(backend="gloo")
    s = HeatSolver(cfg, transport=transport, dist_info=DistInfo(rank, world, rank),
                   device=0 if cfg.backend == "hip" else None, group=group)
    if cfg_kwargs.get("init") == "zero":  # start from a grid scattered by rank 0
        from parallel_heat_amd.models import reference as R
        s.scatter(R.init_grid(cfg.nx, cfg.ny, "random", 77) if rank == 0 else None)
    conv, conv_at, done, res_passes, giveups = False, -1, 0, 0, 0
    for n in (chunks or [steps]):
        r = s.run(n)
        done += r.steps_done
        res_passes += r.resident_passes
        giveups += r.resident_giveups
        if r.converged:
            conv, conv_at = True, r.converged_at
            break
    g = s.gather()
    cs = s.checksum()
    every = [None] * world
    dist.all_gather_object(every, [res_passes, giveups, s.info.halo])
    if rank == 0:
        np.savez(out_path, grid=g, conv=conv, conv_at=conv_at, done=done, hash=cs["hash"],
                 px=s.info.px, py=s.info.py, exchanges=r.exchanges, schedule=s.info.schedule,
                 resident_passes=np.array([e[0] for e in every]),
                 resident_giveups=np.array([e[1] for e in every]),
                 halo=np.array([e[2] for e in every]))
    s.close()
    dist.barrier()
    dist.destroy_process_group()


def run_world(world, cfg_kwargs, steps, tmp_path, transport="torch", chunks=None, env=None):
    import torch.multiprocessing as mp

    out = str(tmp_path / f"out_{world}_{os.getpid()}.npz")
    mp.spawn(worker, args=(world, free_port(), cfg_kwargs, steps, out, transport, chunks, env),
             nprocs=world, join=True)
    return dict(np.load(out))


def tune_worker(rank, world, port, cfg_kwargs, out_path, transport):
    """Runs parallel.tune.autotune on every rank; rank 0 saves the choice."""
    import json

    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    if transport == "rccl":
        rccl_host_per_rank(rank)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from parallel_heat_amd import HeatConfig
    from parallel_heat_amd.parallel.comm import DistInfo
    from parallel_heat_amd.parallel.tune import autotune, default_candidates

    cfg = HeatConfig(**cfg_kwargs)
    cands = default_candidates(cfg, world, schedules=["sync", "overlap"], halo_passes=[0, 2])
    info = DistInfo(rank, world, rank)
    make = None
    shared = None
    if transport == "shared":  # one engine transport for every candidate and the final run
        from parallel_heat_amd.parallel.comm import EngineTransport
        shared = EngineTransport("torch", info)
    elif transport != "auto":  # e.g. GPU ranks sharing one device: host-staged halos
        from parallel_heat_amd import HeatSolver

        def make(c):
            return HeatSolver(c, transport=transport, dist_info=info,
                              device=0 if c.backend == "hip" else None)
    best, table = autotune(cfg, info, cands, steps=20, repeats=1, make=make, shared=shared)
    choice = [best.decomp, best.schedule, best.halo_passes]
    if shared is not None:
        from parallel_heat_amd import HeatSolver
        with HeatSolver(best, dist_info=info, shared=shared) as s:
            s.run(29)
            g = s.gather()
        if rank == 0:
            np.save(out_path + ".npy", g)
        shared.close()
    got = [None] * world
    dist.all_gather_object(got, choice)
    if rank == 0:
        with open(out_path, "w") as f:
            json.dump({"choices": got, "table": table}, f)
    dist.barrier()
    dist.destroy_process_group()


def run_tune(world, cfg_kwargs, tmp_path, transport="auto"):
    import json

    import torch.multiprocessing as mp

    out = str(tmp_path / f"tune_{world}_{os.getpid()}.json")
    mp.spawn(tune_worker, args=(world, free_port(), cfg_kwargs, out, transport), nprocs=world,
             join=True)
    with open(out) as f:
        return json.load(f)

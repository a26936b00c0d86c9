#!/usr/bin/env python3
"""Headline benchmark: Mcells/s (whole node) and s/1000 iters on an 8192^2 fp32 grid.

BASELINE.json metric: "Mcells/sec (whole node) + sec/1000 iters, 8192^2 grid at
1/2/4/8 MI355X".  One benchmark *step* = 1000 Jacobi iterations of the full
8192 x 8192 plate (BASELINE config "8192x8192 grid fp32 on 1 MI355X, 1000
iters"), i.e. ms_per_step is directly ms per 1000 iterations.  The grid is
fixed as N grows (strong scaling); every rank owns an 8192/N-row slab (1-D
decomposition: contiguous halo rows over RCCL/xGMI).

    python bench.py                                  # 1 GPU
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
        --master-addr 127.0.0.1 --master-port 29500 bench.py --gpus 8

Data: synthetic random-init temperature grid (--init random), no files.
Timing: W untimed warmup steps, then barrier + synchronize, K timed steps,
synchronize + barrier; the max over ranks is reported.  Everything the model
does per iteration (halo exchange, all kernels) is inside the timed region.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

BASELINE_MCELLS = 3556.2  # reference best single-GPU throughput (Heat.pdf p.11 Table 6, 1000^2 T=8)
METRIC = "Mcells/sec (whole node) + sec/1000 iters, 8192^2 grid at 1/2/4/8 MI355X"


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--nx", type=int, default=8192)
    ap.add_argument("--weak", action="store_true",
                    help="weak scaling: nx rows PER GPU (the grid grows with N); not the headline")
    ap.add_argument("--ny", type=int, default=8192)
    ap.add_argument("--iters-per-step", type=int, default=1000)
    ap.add_argument("--tb-depth", type=int, default=0)
    ap.add_argument("--kernel", default="auto")
    ap.add_argument("--decomp", default="rows")
    ap.add_argument("--converge", action="store_true",
                    help="also run the convergence check (never converges on random data)")
    ap.add_argument("--check-interval", type=int, default=50)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--schedule", default="auto", help="multi-rank pass schedule")
    ap.add_argument("--halo-passes", type=int, default=0)
    ap.add_argument("--phase-timing", action="store_true",
                    help="diagnostic: eager run with per-phase device times (not the headline)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.weak:
        args.nx *= world
    if world != args.gpus and rank == 0:
        print(f"[bench] note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE",
              file=sys.stderr)
    if not torch.cuda.is_available():
        print("[bench] no GPU visible", file=sys.stderr)
        return 1
    torch.cuda.set_device(local_rank % torch.cuda.device_count())
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl")

    from parallel_heat_amd import HeatConfig, HeatSolver, _native
    from parallel_heat_amd.parallel.comm import DistInfo

    cfg = HeatConfig(nx=args.nx, ny=args.ny, steps=args.iters_per_step, init="random", seed=1234,
                     backend="hip", kernel=args.kernel, tb_depth=args.tb_depth,
                     decomp=args.decomp, converge=args.converge,
                     check_interval=args.check_interval, use_graph=not args.no_graph,
                     overlap=not args.no_overlap, device=local_rank % torch.cuda.device_count(),
                     schedule=args.schedule, halo_passes=args.halo_passes,
                     phase_timing=args.phase_timing)
    info = DistInfo(rank, world, local_rank)
    try:
        solver = HeatSolver(cfg, dist_info=info)
    except Exception as e:  # noqa: BLE001
        if world == 1:
            raise
        # The engine's own RCCL communicator failed to come up on every rank:
        # fall back, loudly, to halos staged through host memory over a gloo
        # group (the transport name lands in config.parallelism).
        print(f"[bench] rank {rank}: RCCL transport failed ({e}); "
              "falling back to the staged torch/gloo transport", file=sys.stderr, flush=True)
        solver = HeatSolver(cfg, transport="torch", dist_info=info,
                            group=dist.new_group(backend="gloo"))

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        solver.run(args.iters_per_step)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    done = 0
    phases = [0.0, 0.0, 0.0]
    for _ in range(args.steps):
        r = solver.run(args.iters_per_step)
        done += r.steps_done
        phases = [phases[0] + r.t_exchange, phases[1] + r.t_compute, phases[2] + r.t_reduce]
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())

    cells = args.nx * args.ny * done
    mcells = cells / elapsed / 1e6
    ms_per_step = elapsed * 1e3 / max(1, args.steps)
    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(mcells, 3),
            "unit": "Mcells/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "sec_per_1000_iters": round(elapsed * 1000.0 / max(1, done), 6),
            "higher_is_better": True,
            "scaling": "weak" if args.weak else "strong",
            "vs_baseline": round(mcells / BASELINE_MCELLS, 3),
            "dtype": "fp32",
            "data": "synthetic (random-init temperature grid, seed 1234)",
            "config": {
                "model": "heat2d 5-point Jacobi (fixed boundary)",
                "grid": f"{args.nx}x{args.ny}",
                "global_batch": 1,
                "seq_len": args.nx * args.ny,
                "iters_per_step": args.iters_per_step,
                "parallelism": f"domain-decomp {solver.info.px}x{solver.info.py} "
                               f"({solver.transport}), tb_depth {solver.info.tb_depth}, "
                               f"halo {solver.info.halo}, schedule {solver.info.schedule}",
                "converge_check": bool(args.converge),
            },
        }
        if args.verbose:
            line["native"] = _native.loaded_path()
        if args.phase_timing:
            line["phase_seconds_rank0"] = {"exchange": round(phases[0], 6),
                                           "compute": round(phases[1], 6),
                                           "reduce": round(phases[2], 6)}
        print(json.dumps(line), flush=True)
    solver.close()
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())

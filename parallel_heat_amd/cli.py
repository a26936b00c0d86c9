"""``python -m parallel_heat_amd`` — the Python front end of the ``heat`` CLI.

Same flags as the native ``build/heat`` binary (tests/test_cli.py pins the
two flag sets and their reference output lines against each other).
Multi-rank runs are launched with ``python -m torch.distributed.run
--nproc-per-node N -m parallel_heat_amd ...``: GPU ranks talk over the
engine's RCCL communicator, CPU ranks over torch.distributed (gloo).  The
single-process native modes -- ``--gpus N`` (N GPU ranks as threads of one
process) and ``--plan`` (the per-GPU memory plan) -- run the native binary
with the same arguments.  ``--transport torch`` is the one Python-only value.  Replaces the reference's -D macro builds
(``cuda/Makefile``, ``mpi/Makefile:12-22``) with run-time flags.
"""
from __future__ import annotations

import argparse
import json
import subprocess
import sys

import torch

from . import _native
from .models.config import HeatConfig
from .models.heat2d import HeatSolver
from .parallel import comm as pcomm
from .utils import io as hio
from .utils import report


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(prog="python -m parallel_heat_amd",
                                description="2-D heat diffusion on MI355X (5-point Jacobi)")
    a = p.add_argument
    a("--nx", type=int, default=20)
    a("--ny", type=int, default=20)
    a("--steps", type=int, default=10000)
    a("--cx", type=float, default=0.1)
    a("--cy", type=float, default=0.1)
    a("--converge", action="store_true")
    a("--check-interval", type=int, default=20)
    a("--eps", type=float, default=1e-3)
    a("--backend", choices=["cpu", "hip"], default=None)
    a("--threads", type=int, default=0)
    a("--kernel", choices=["auto", "naive", "tb", "lds", "mfma"], default="auto")
    a("--tb-depth", type=int, default=0)
    a("--decomp", choices=["auto", "rows", "1d", "2d"], default="auto")
    a("--px", type=int, default=0)
    a("--py", type=int, default=0)
    a("--init", choices=["ref-wrap", "exact", "ref64", "random", "zero"], default="ref-wrap")
    a("--seed", type=int, default=0)
    a("--out", default=None)
    a("--out-format", choices=["dat", "bin", "checksum"], default="dat")
    a("--naming", choices=["plain", "mpi", "cuda"], default="plain")
    a("--dump-initial", action="store_true")
    a("--compat", choices=["none", "mpi", "cuda"], default=None)
    a("--no-graph", action="store_true")
    a("--no-overlap", action="store_true")
    a("--schedule", choices=["auto", "sync", "overlap", "pipeline"], default="auto")
    a("--halo-passes", type=int, default=0)
    a("--numerics", choices=["fp32", "mpi"], default="fp32")
    a("--phase-timing", action="store_true")
    a("--transport", choices=["auto", "local", "rccl", "torch", "tcp", "loopback"], default="auto",
      help="loopback: --gpus ranks sharing a device (native binary)")
    a("--port", type=int, default=0, help="tcp transport rendezvous port (0: MASTER_PORT+1)")
    a("--gpus", type=int, default=0,
      help="one process, N GPU ranks as threads (native binary): RCCL with a GPU per rank, "
           "else loopback copies")
    a("--watchdog", type=float, default=None,
      help="multi-rank GPU runs: abort and exit 1 after this many seconds without device "
           "progress (HEAT_WATCHDOG_S, default 300, 0 = never)")
    a("--plan", action="store_true", help="print the per-GPU memory plan and exit (native)")
    a("--checkpoint", default=None)
    a("--checkpoint-every", type=int, default=0)
    a("--resume", default=None)
    a("--warmup", type=int, default=0,
      help="N untimed steps first (graph capture), then the initial state is restored")
    a("--json", action="store_true")
    return p


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    args = build_parser().parse_args(argv)
    if args.gpus > 0 or args.plan:
        # Single-process native modes: the `heat` binary owns the threads
        # and the planner; same flags, same output.
        return subprocess.run([str(_native.CLI_PATH)] + argv).returncode
    if args.watchdog is not None:
        import os
        os.environ["HEAT_WATCHDOG_S"] = str(args.watchdog)  # read by the native solver
    if args.transport == "loopback":
        raise SystemExit("--transport loopback is the --gpus mode of ranks sharing a device")
    backend = args.backend or ("hip" if torch.cuda.is_available() else "cpu")
    compat = args.compat or {"mpi": "mpi", "cuda": "cuda"}.get(args.naming, "none")
    cfg = HeatConfig(nx=args.nx, ny=args.ny, steps=args.steps, cx=args.cx, cy=args.cy,
                     converge=args.converge, check_interval=args.check_interval, eps=args.eps,
                     init=args.init, seed=args.seed, backend=backend, kernel=args.kernel,
                     tb_depth=args.tb_depth, threads=args.threads, decomp=args.decomp,
                     px=args.px, py=args.py, use_graph=not args.no_graph,
                     overlap=not args.no_overlap, compat=compat, schedule=args.schedule,
                     halo_passes=args.halo_passes, numerics=args.numerics,
                     phase_timing=args.phase_timing)
    info = pcomm.init_distributed("nccl" if backend == "hip" else "gloo")
    root = info.is_root
    out = sys.stdout
    if root and args.naming == "mpi":
        out.write(report.mpi_banner(info.world, cfg.nx, cfg.ny, cfg.steps, cfg.converge))
        out.flush()
    if args.port and args.transport == "tcp":
        import os
        os.environ["MASTER_PORT"] = str(args.port - 1)  # make_comm uses MASTER_PORT + 1
    solver = HeatSolver(cfg, transport=args.transport, dist_info=info)
    if args.resume:
        solver.load(args.resume)

    small = cfg.nx * cfg.ny <= (1 << 24)
    if args.naming == "mpi":
        init_path, final_path = "initial_im.dat", "final_im.dat"
    elif args.naming == "cuda":
        init_path, final_path = None, report.cuda_output_name(cfg.nx, cfg.ny, cfg.steps)
    else:
        init_path, final_path = "initial.dat", ("final.dat" if small else None)
    if args.out is not None:
        final_path = None if args.out == "none" else args.out

    def emit(path):
        if not path:
            return
        if args.out_format == "bin":
            solver.save(path)
        elif args.out_format == "checksum":
            c = solver.checksum()
            if root:
                with open(path, "w") as f:
                    f.write(json.dumps({"nx": cfg.nx, "ny": cfg.ny, "step": solver.step, **c}) + "\n")
        else:
            g = solver.gather()
            if root:
                hio.write_dat(path, g)

    if args.warmup > 0:
        # Untimed warm-up (graph capture, first touch), then the initial
        # state again: the timed run and the output are a cold run's.
        if args.resume:
            raise SystemExit("--warmup with --resume")
        solver.run(args.warmup)
        solver.reset()
    if args.dump_initial or args.naming == "mpi":
        emit(init_path)
    total = cfg.total_steps()
    todo = total - solver.step
    acc = dict(steps_done=0, seconds=0.0, passes=0, exchanges=0, checks=0, t_exchange=0.0,
               t_compute=0.0, t_reduce=0.0)
    converged, converged_at, last = False, -1, -1.0
    while todo > 0:
        chunk = min(args.checkpoint_every, todo) if args.checkpoint_every > 0 else todo
        r = solver.run(chunk)
        for k in acc:
            acc[k] += getattr(r, k)
        last = r.last_resid
        todo -= r.steps_done
        if args.checkpoint and args.checkpoint_every > 0:
            solver.save(args.checkpoint)
        if r.converged:
            converged, converged_at = True, r.converged_at
            break
    emit(final_path)
    if root:
        if cfg.converge:
            out.write(report.convergence_line(args.naming, converged, converged_at, solver.step))
        out.write(report.elapsed_line(args.naming, acc["seconds"]))
        if args.json:
            cells = cfg.nx * cfg.ny * acc["steps_done"]
            out.write(report.metrics_json(
                nx=cfg.nx, ny=cfg.ny, steps=total, steps_done=acc["steps_done"],
                ranks=info.world, backend=backend,
                decomp=f"{solver.info.px}x{solver.info.py}", tb_depth=solver.info.tb_depth,
                seconds=acc["seconds"],
                mcells_per_s=cells / acc["seconds"] / 1e6 if acc["seconds"] > 0 else 0.0,
                s_per_1000_iters=acc["seconds"] * 1000 / max(1, acc["steps_done"]),
                converged=converged, converged_at=converged_at, last_resid=last,
                passes=acc["passes"], exchanges=acc["exchanges"],
                transport=solver.transport, schedule=solver.info.schedule,
                halo=solver.info.halo, t_exchange=acc["t_exchange"],
                t_compute=acc["t_compute"], t_reduce=acc["t_reduce"],
                native=_native.loaded_path()) + "\n")
        out.flush()
    solver.barrier()
    solver.close()
    return 0


if __name__ == "__main__":  # pragma: no cover
    sys.exit(main())

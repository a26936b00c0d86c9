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

Verification (after the timed region, `--no-verify` skips it): the global
checksum of the final state is compared with the same number of steps of a
single-rank run of the independent LDS-tiled single-step kernel on rank 0's GPU
(bitwise-equal numerics): `"verified": true` in the JSON line means the
benchmarked (multi-GPU, graph-captured, temporally blocked) run computed
exactly the reference field.  A mismatch prints `"verified": false` and exits
non-zero.

Multi-GPU autotune (`--no-autotune` skips it): before the warmup, every
decomposition candidate (rows slabs, the 2-D MPI_Dims_create grid) x pass
schedule (deep-halo sync with the default and a halved exchange interval,
boundary-first pipeline overlapping the exchange with the interior) that the
scaling model (parallel/model.py) does not rule out (predicted > 1.3x the
best) is timed on the real ranks (max over ranks) and the fastest is
benchmarked; the table is in the JSON line ("autotune", the ruled-out ones
in "autotune_pruned") and the choice in config.parallelism.

Multi-GPU explanation (after verification, untimed): "predicted" is the
model's time per 1000 iterations and node Tcells/s for the chosen layout
(per-rank plate rate measured on one GPU + a stated xGMI exchange model,
parameters in "model"), and "phase_seconds_per_1000" the per-rank exchange /
compute / reduce device time of one eager phase-timed run of the same
configuration (Heat.pdf p.8-11 Paraver phases, as numbers).

Failure handling: RCCL must come up on every rank (the ranks agree through
torch.distributed before going on); if it fails anywhere the run exits
non-zero, unless `--allow-fallback` lets ALL ranks switch together to halos
staged through host memory (named in config.parallelism).  A resident-tile
launch that gives up a neighbour wait (tiles not co-resident) invalidates its
run: the ranks agree on that after the warmup and after the timed steps
(outside the timed region), rebuild the solver with one launch per pass and
measure again.  The autotune skips a candidate that fails cleanly at run time
(every rank at the same point, communicator intact) instead of aborting.
Every such step is listed in "fallbacks" (empty when none was taken).  A
watchdog ends a hung run with a stack dump instead of letting it hang
(`--watchdog-s`).

Exchange model (multi-GPU): before pruning autotune candidates, grouped halo
exchanges of the first candidate are timed at three depths (5 samples of 20
exchanges each) on the real ranks; a fit with a positive slope and R^2 >= 0.8
over the per-size medians replaces the stated latency and per-link GB/s of
parallel/model.py in the pruning and in "predicted" / "model"; a fit that
fails those checks (model.xgmi.fit_ok false) prunes nothing.  The pruning
always keeps the best-predicted candidate of every (layout, halo passes).
"""
from __future__ import annotations

import argparse
import faulthandler
import json
import os
import re
import sys
import tempfile
import time

import torch
import torch.distributed as dist

BASELINE_MCELLS = 3556.2  # reference best single-GPU throughput (Heat.pdf p.11 Table 6, 1000^2 T=8)
METRIC = "Mcells/sec (whole node) + sec/1000 iters, 8192^2 grid at 1/2/4/8 MI355X"


def log(rank: int, msg: str) -> None:
    print(f"[bench] rank {rank}: {msg}", file=sys.stderr, flush=True)


_LINK = re.compile(r"(\d+)\[[^\]]*\] -> (\d+)\[[^\]]*\] (?:\[\w+\] )?via (\S+)")


def rccl_links(path: str) -> list:
    """Distinct 'src->dst via TRANSPORT' channel connections RCCL logged
    (NCCL_DEBUG=INFO, subsystems INIT,P2P) for this rank's communicators."""
    seen = set()
    try:
        with open(path, errors="replace") as f:
            for line in f:
                m = _LINK.search(line)
                if m:
                    seen.add(f"{m.group(1)}->{m.group(2)} via {m.group(3)}")
    except OSError:
        return []
    return sorted(seen)


def main() -> int:
    # The JSON line is the only thing on stdout: native libraries (RCCL's
    # version banner under NCCL_DEBUG=VERSION, ...) print there too, so fd 1
    # is pointed at stderr and the JSON goes to a saved copy of it.
    sys.stdout.flush()
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
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
                    help="also run the convergence check every --check-interval steps (a run "
                         "stops at its converging check; random data converges within a few "
                         "hundred steps, --init ref-wrap does not within a bench run)")
    ap.add_argument("--check-interval", type=int, default=50)
    ap.add_argument("--eps", type=float, default=1e-3)
    ap.add_argument("--init", default="random",
                    help="initial condition: random (synthetic, default) | ref-wrap (the "
                         "reference's inidat, int32-wrapped)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--schedule", default="auto", help="multi-rank pass schedule")
    ap.add_argument("--halo-passes", type=int, default=0)
    ap.add_argument("--phase-timing", action="store_true",
                    help="diagnostic: eager run with per-phase device times (not the headline)")
    ap.add_argument("--no-verify", action="store_true",
                    help="skip the post-run check against a single-rank LDS-kernel run")
    ap.add_argument("--allow-fallback", action="store_true",
                    help="if RCCL fails on every rank, run with host-staged halos over gloo")
    ap.add_argument("--no-autotune", action="store_true",
                    help="multi-GPU: skip timing the decomposition/schedule candidates "
                         "(use --decomp/--schedule as given)")
    ap.add_argument("--autotune-schedules", default="sync,pipeline",
                    help="comma list of pass schedules the multi-GPU autotune tries")
    ap.add_argument("--autotune-halo-passes", default="0,4",
                    help="comma list of sync-schedule passes per exchange (0 = engine default)")
    ap.add_argument("--watchdog-s", type=float, default=900.0,
                    help="abort (stack dump, exit 1) if one phase takes longer than this")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.weak:
        args.nx *= world
    if world != args.gpus and rank == 0:
        log(rank, f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    if not torch.cuda.is_available():
        log(rank, "no GPU visible")
        return 1

    def watchdog(phase: str, seconds: float) -> None:
        # A hung collective (a peer that died, a stuck exchange) ends the
        # process with every thread's stack instead of hanging the job.
        faulthandler.cancel_dump_traceback_later()
        if seconds > 0:
            if args.verbose:
                log(rank, f"phase {phase} (watchdog {seconds:.0f} s)")
            faulthandler.dump_traceback_later(seconds, exit=True)

    watchdog("init", args.watchdog_s)
    # A resident-tile give-up (tiles not co-resident) is reported by the run
    # instead of raised: the ranks agree on it and redo the work without
    # resident spans ("fallbacks" in the JSON line).
    os.environ.setdefault("HEAT_TB_RES_GIVEUP", "defer")
    fallbacks = []
    device = local_rank % torch.cuda.device_count()
    torch.cuda.set_device(device)
    rccl_log = None
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if os.environ.get("NCCL_DEBUG", "").upper() not in ("INFO", "TRACE"):
            # Record which transport RCCL picks for each neighbour pair (xGMI
            # P2P on a node) in a per-rank file, reported in the JSON line.
            rccl_log = os.path.join(tempfile.gettempdir(),
                                    f"heat_rccl_{os.getpid()}_r{rank}.log")
            os.environ.update(NCCL_DEBUG="INFO", NCCL_DEBUG_SUBSYS="INIT,P2P",
                              NCCL_DEBUG_FILE=rccl_log)
        if os.environ.get("HEAT_RCCL_HOST_PER_RANK") == "1":
            # Rehearsal hook for a 1-GPU box (tools/rccl_rehearsal.sh): RCCL
            # refuses two ranks on one device of one host, so each rank claims
            # its own host id and the ranks talk over RCCL's socket transport.
            # The API path (grouped send/recv captured in hipGraphs, the
            # all-reduces, torch's own nccl group) is the one a real node runs.
            os.environ["NCCL_HOSTID"] = f"heat-rank-{rank}"
        dist.init_process_group("nccl")

    from parallel_heat_amd import HeatConfig, HeatSolver, _native
    from parallel_heat_amd.parallel.comm import DistInfo

    cfg = HeatConfig(nx=args.nx, ny=args.ny, steps=args.iters_per_step, init=args.init, seed=1234,
                     backend="hip", kernel=args.kernel, tb_depth=args.tb_depth,
                     decomp=args.decomp, converge=args.converge,
                     check_interval=args.check_interval, eps=args.eps,
                     use_graph=not args.no_graph,
                     overlap=not args.no_overlap, device=device,
                     schedule=args.schedule, halo_passes=args.halo_passes,
                     phase_timing=args.phase_timing)
    info = DistInfo(rank, world, local_rank)

    def vote(ok: bool) -> bool:
        """True on every rank iff ok on every rank (torch's own group)."""
        if world == 1:
            return ok
        t = torch.tensor([1 if ok else 0], dtype=torch.int32, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return bool(t.item())

    # ONE engine transport per rank for the whole run: the autotune
    # candidates and the benchmarked solver all use this RCCL communicator.
    shared = None
    if world > 1:
        from parallel_heat_amd.parallel.comm import EngineTransport
        err = None
        try:
            shared = EngineTransport("rccl", info, device=device)
        except _native.NativeError as e:
            err = e
        if not vote(shared is not None):
            log(rank, f"RCCL transport failed on some rank ({err})")
            if shared is not None:
                shared.close()
                shared = None
            if not args.allow_fallback:
                log(rank, "RCCL transport unavailable on some rank; exiting "
                          "(--allow-fallback runs host-staged halos over gloo instead)")
                return 1
            log(rank, "falling back to host-staged halos over gloo (all ranks)")
            shared = EngineTransport("torch", info, group=dist.new_group(backend="gloo"))
            fallbacks.append({"what": f"RCCL transport failed on some rank ({err})",
                              "action": "host-staged halos over gloo (--allow-fallback)"})

    tuning = None
    pruned = []
    xgmi = None
    if world > 1 and not args.no_autotune:
        # The fastest decomposition (rows slabs vs the 2-D dims_create grid)
        # and pass schedule depend on xGMI link bandwidth and the per-rank
        # block shape: time each on the real ranks before the timed region.
        from parallel_heat_amd.parallel.model import fit_exchange, predict, prune
        from parallel_heat_amd.parallel.tune import (autotune, default_candidates, describe,
                                                     exchange_depths, measure_exchange)

        watchdog("autotune", args.watchdog_s)
        all_cands = default_candidates(cfg, world,
                                       schedules=[x for x in args.autotune_schedules.split(",") if x],
                                       halo_passes=[int(x) for x in
                                                    args.autotune_halo_passes.split(",") if x])
        # The exchange model's latency and bandwidth, measured on these ranks
        # (grouped exchanges of the first candidate's messages at two depths)
        # before they prune anything.
        xgmi = exchange_probe(all_cands[0], info, shared, world, HeatSolver, measure_exchange,
                              exchange_depths, fit_exchange, rank)
        cands = prune(all_cands, world, xgmi=xgmi)
        pruned = [dict(describe(c, world),
                       predicted_ms_per_1000=predict(c, world, xgmi=xgmi)["ms_per_1000"])
                  for c in all_cands if c not in cands]
        try:
            cfg, tuning = autotune(cfg, info, cands, steps=args.iters_per_step, repeats=3,
                                   log=(lambda m: log(rank, m)) if args.verbose else None,
                                   shared=shared)
        except _native.NativeError as e:
            # Every candidate rejected (the ranks agree inside autotune).
            log(rank, f"autotune failed ({e}); using --decomp {args.decomp}")
            fallbacks.append({"what": f"autotune failed ({str(e)[:160]})",
                              "action": f"--decomp {args.decomp} as given"})

    solver = None
    err = None
    try:
        solver = HeatSolver(cfg, dist_info=info, shared=shared)
    except _native.NativeError as e:
        if world == 1:
            raise
        err = e
    if not vote(solver is not None):
        log(rank, f"solver construction failed on some rank ({err})")
        return 1

    def barrier():
        if world > 1:
            dist.barrier()

    # Plain runs are enqueued back to back (HeatSolver.run(wait=False)): the
    # device goes from one 1000-iteration step to the next without a host
    # round trip in between; run(0) completes them (and reports errors).
    # Convergence checks and phase timing run step by step.
    wait = args.converge or args.phase_timing

    def measure():
        """Warmup, then the timed region.  None if a resident launch gave up
        on any rank (the ranks agree outside the timed region)."""
        watchdog("warmup", args.watchdog_s)
        gave = 0
        for _ in range(args.warmup):
            gave += solver.run(args.iters_per_step, wait=wait).resident_giveups
        gave += solver.run(0).resident_giveups
        if not vote(gave == 0):
            return None
        barrier()
        torch.cuda.synchronize()
        watchdog("timed", args.watchdog_s)
        t0 = time.perf_counter()
        done = 0
        phases = [0.0, 0.0, 0.0]
        for _ in range(args.steps):
            r = solver.run(args.iters_per_step, wait=wait)
            done += r.steps_done
            gave += r.resident_giveups
            phases = [phases[0] + r.t_exchange, phases[1] + r.t_compute, phases[2] + r.t_reduce]
        gave += solver.run(0).resident_giveups
        torch.cuda.synchronize()
        barrier()
        elapsed = time.perf_counter() - t0
        if not vote(gave == 0):
            return None
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item()), done, phases

    res = measure()
    if res is None:
        # Resident tiles were not co-resident somewhere (another process on a
        # GPU, ...): the state is invalid.  Every rank rebuilds its solver
        # with one launch per pass and measures again from the initial state.
        log(rank, "a resident launch gave up on some rank: measuring again without resident spans")
        fallbacks.append({"what": "resident tiles gave up a neighbour wait on some rank "
                                  "(state invalid)",
                          "action": "solver rebuilt with HEAT_TB_RESIDENT=0 (one launch per "
                                    "pass), warmup and timed steps run again"})
        solver.close()
        os.environ["HEAT_TB_RESIDENT"] = "0"
        solver = HeatSolver(cfg, dist_info=info, shared=shared)
        res = measure()
        if res is None:
            log(rank, "resident give-up with resident spans off: giving up")
            return 1
    elapsed, done, phases = res

    verified = None
    check = {}
    if not args.no_verify:
        watchdog("verify", args.watchdog_s)
        verified, check = verify(solver, cfg, rank, world, device, HeatSolver, DistInfo)
    explain = None
    if world > 1:
        # Untimed: the model's prediction for the chosen layout and the
        # measured per-rank phase split of one eager phase-timed run.
        watchdog("explain", args.watchdog_s)
        explain = explain_run(cfg, info, shared, world, args.iters_per_step, HeatSolver, xgmi)
    rccl = None
    if shared is not None:
        # What the engine's communicator saw, from every rank: its rank count
        # and device (ncclCommCount / ncclCommCuDevice), the PCI bus id, and
        # the transport RCCL logged for each channel connection.
        mine = dict(shared.info(), rank=rank, local_rank=local_rank,
                    links=rccl_links(rccl_log) if rccl_log else None)
        every = [None] * world
        dist.all_gather_object(every, mine)
        links = sorted({l for r in every for l in (r.get("links") or [])})
        rccl = {"transport": mine["name"], "nranks": mine["nranks"],
                "ranks": [{k: r[k] for k in ("rank", "user_rank", "device", "bus_id")}
                          for r in every],
                "distinct_devices": len({r["bus_id"] or r["device"] for r in every}),
                "links": links if rccl_log else "not recorded (NCCL_DEBUG=INFO/TRACE set by the caller)"}
    faulthandler.cancel_dump_traceback_later()

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
            "data": ("synthetic (random-init temperature grid, seed 1234)" if args.init == "random"
                     else f"synthetic ({args.init} initial condition of the reference)"),
            "config": {
                "model": "heat2d 5-point Jacobi (fixed boundary)",
                "grid": f"{args.nx}x{args.ny}",
                "global_batch": 1,
                "seq_len": args.nx * args.ny,
                "iters_per_step": args.iters_per_step,
                "parallelism": f"domain-decomp {solver.info.px}x{solver.info.py} "
                               f"({solver.transport}), tb_depth {solver.info.tb_depth}, "
                               f"halo {solver.info.halo}, schedule {solver.info.schedule}",
                "converge_check": (f"every {args.check_interval} steps, eps {args.eps:g}"
                                   if args.converge else False),
            },
            "verified": verified,
            "fallbacks": fallbacks,
        }
        if tuning is not None:
            line["autotune"] = tuning
            if pruned:
                line["autotune_pruned"] = pruned
        if explain is not None:
            line.update(explain)
        if rccl is not None:
            line["rccl"] = rccl
        if check:
            line["verification"] = check
        if args.verbose:
            line["native"] = _native.loaded_path()
        if args.phase_timing:
            line["phase_seconds_rank0"] = {"exchange": round(phases[0], 6),
                                           "compute": round(phases[1], 6),
                                           "reduce": round(phases[2], 6)}
        print(json.dumps(line), file=json_out, flush=True)
    solver.close()
    if shared is not None:
        shared.close()
    if world > 1:
        dist.destroy_process_group()
    return 0 if verified is not False else 2


def exchange_probe(cfg, info, shared, world, HeatSolver, measure_exchange, exchange_depths,
                   fit_exchange, rank):
    """Measured exchange parameters (latency, GB/s per link) from grouped halo
    exchanges of cfg's layout at three depths (H, H/2, H/4), 5 interleaved
    samples of 20 exchanges each, max over the ranks (collective); the fit
    takes medians and says whether it may prune (fit_ok).  None (the stated
    model) if the probe fails on any rank."""
    pts = None
    try:
        with HeatSolver(cfg, dist_info=info, shared=shared) as s:
            H = s.info.halo
            def agree_max(x):
                t = torch.tensor([x], dtype=torch.float64, device="cuda")
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                return float(t.item())
            pts = measure_exchange(s, exchange_depths(H), iters=20, reps=5, agree_max=agree_max)
    except Exception as e:  # noqa: BLE001 - diagnostics; the stated model stays
        log(rank, f"exchange probe failed ({e})")
    ok = torch.tensor([1 if pts else 0], dtype=torch.int32, device="cuda")
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    return fit_exchange(pts) if ok.item() else None


def explain_run(cfg, info, shared, world, iters, HeatSolver, xgmi=None):
    """Model prediction + measured per-rank phase split (collective)."""
    from parallel_heat_amd.parallel.model import model_params, predict
    phases = {"exchange": None, "compute": None, "reduce": None}
    try:
        with HeatSolver(cfg.replace(phase_timing=True), dist_info=info, shared=shared) as s:
            r = s.run(iters)
            scale = 1000.0 / max(1, r.steps_done)
            phases = {"exchange": round(r.t_exchange * scale, 6),
                      "compute": round(r.t_compute * scale, 6),
                      "reduce": round(r.t_reduce * scale, 6),
                      "wall": round(r.seconds * scale, 6),
                      "resident_passes": r.resident_passes,
                      "chained_passes": r.chained_passes}
    except Exception as e:  # noqa: BLE001 - diagnostics only; every rank still gathers
        phases["error"] = str(e)[:200]
    every = [None] * world
    dist.all_gather_object(every, dict(phases, rank=info.rank))
    return {"predicted": predict(cfg, world, xgmi=xgmi), "model": model_params(xgmi),
            "phase_seconds_per_1000": every}


def verify(solver, cfg, rank, world, device, HeatSolver, DistInfo):
    """Global checksum of the benchmarked state vs rank 0's single-rank run of
    the same steps with the LDS-tiled single-step kernel (an independent
    kernel, bitwise equal to the CPU oracle).  Collective; returns the verdict
    on every rank and a small record for the JSON line."""
    steps = solver.step
    got = solver.checksum()  # collective (all-reduced over the ranks)
    ok = torch.zeros(1, dtype=torch.int32, device="cuda")
    rec = {}
    if rank == 0:
        t0 = time.perf_counter()
        ref_cfg = cfg.replace(kernel="lds", tb_depth=0, converge=False, phase_timing=False)
        with HeatSolver(ref_cfg, transport="local", dist_info=DistInfo(0, 1, 0),
                        device=device) as ref:
            left = steps
            while left > 0:  # 1000-step segments: one captured graph, replayed
                left -= ref.run(min(1000, left)).steps_done
            want = ref.checksum()
        ok[0] = int(got["hash"] == want["hash"] and got["count"] == want["count"])
        rec = {"steps": steps, "hash": got["hash"], "reference_hash": want["hash"],
               "reference": "1 rank, lds kernel", "seconds": round(time.perf_counter() - t0, 3)}
        if not ok[0]:
            print(f"[bench] VERIFICATION FAILED after {steps} steps: hash {got['hash']} "
                  f"(sum {got['sum']}) vs single-rank lds {want['hash']} (sum {want['sum']})",
                  file=sys.stderr, flush=True)
    if world > 1:
        dist.broadcast(ok, src=0)
    return bool(ok.item()), rec


if __name__ == "__main__":
    sys.exit(main())

"""Candidate set of the multi-GPU autotune (parallel/tune.py) as bench.py
builds it: rows slabs and the MPI_Dims_create grid, x deep-halo sync with the
default and a doubled exchange interval, x the boundary-first pipeline."""
import pytest

from parallel_heat_amd import HeatConfig, _native
from parallel_heat_amd.parallel.tune import default_candidates, describe


def _keys(world, **kw):
    cfg = HeatConfig(nx=8192, ny=8192, steps=0, backend="cpu")
    return [tuple(describe(c, world).values())
            for c in default_candidates(cfg, world, **kw)]


def test_bench_candidates_8_ranks():
    keys = _keys(8, schedules=["sync", "pipeline"], halo_passes=[0, 4])
    assert keys == [(8, 1, "sync", 0), (8, 1, "sync", 4), (8, 1, "pipeline", 0),
                    (4, 2, "sync", 0), (4, 2, "sync", 4), (4, 2, "pipeline", 0)]


def test_bench_candidates_2_ranks_one_layout():
    # dims_create(2) = [2, 1] = the rows slabs: one layout only.
    keys = _keys(2, schedules=["sync", "pipeline"], halo_passes=[0, 16])
    assert keys == [(2, 1, "sync", 0), (2, 1, "sync", 16), (2, 1, "pipeline", 0)]


def test_halo_passes_only_for_sync():
    keys = _keys(4, schedules=["overlap"], halo_passes=[0, 4, 16])
    assert keys == [(4, 1, "overlap", 0), (2, 2, "overlap", 0)]


def test_model_prunes_overlap_schedules_at_8_ranks():
    # The scaling model (parallel/model.py) rules out the boundary-first
    # pipeline on the 8-GPU blocks (per-pass band launches and joins, no
    # resident spans) and keeps every deep-halo sync candidate.
    from parallel_heat_amd.parallel.model import predict, prune
    cfg = HeatConfig(nx=8192, ny=8192, steps=0, backend="cpu")
    cands = default_candidates(cfg, 8, schedules=["sync", "pipeline"], halo_passes=[0, 4])
    kept = [tuple(describe(c, 8).values()) for c in prune(cands, 8)]
    assert kept == [(8, 1, "sync", 0), (8, 1, "sync", 4), (4, 2, "sync", 0), (4, 2, "sync", 4)]
    p = predict(cands[0], 8)
    # Resident-aware m = 7 (1168-row span boxes keep the 12 x 16 tiles).
    assert p["layout"] == "8x1" and p["block"] == "1024x8192" and p["halo"] == 84
    assert p["exchanges_per_1000"] == 12 and p["message_bytes"] == 84 * (8192 + 2 * 84) * 4
    assert abs(p["ms_per_1000"] - (p["compute_ms"] + p["exchange_ms"])) < 1e-3
    assert 0 < p["tcells_per_s"] < 8 * 5.5


def test_model_single_gpu_is_the_plate_rate():
    from parallel_heat_amd.parallel.model import RATE_POINTS, predict
    cfg = HeatConfig(nx=8192, ny=8192, steps=0, backend="cpu")
    p = predict(cfg, 1)
    assert p["exchanges_per_1000"] == 0 and p["exchange_ms"] == 0
    assert p["tcells_per_s"] == RATE_POINTS[-1][1]


def test_model_more_ranks_never_slower_per_rank_block():
    from parallel_heat_amd.parallel.model import rate_tcells
    # Within a family, rates are monotone in work per SIMD over the measured range.
    assert (rate_tcells(8192, 8192, False) >= rate_tcells(4096, 8192, False)
            >= rate_tcells(2048, 8192, False) >= rate_tcells(1024, 8192, False))
    assert rate_tcells(2048, 8192, True) >= rate_tcells(1024, 8192, True) > rate_tcells(512, 8192, True)


def test_model_resident_fits_mirrors_the_planner():
    from parallel_heat_amd.parallel.model import predict, resident_fits
    assert resident_fits(1024, 8192) and resident_fits(2048, 4096)        # 12 x 16: 252 / 234 tiles
    assert resident_fits(1192, 8192)                                      # 14 x 8, two per CU
    assert resident_fits(2048, 8192) and resident_fits(4096, 4096)        # 20 x 16: 252 tiles
    assert resident_fits(4096 + 36, 4096 + 36)                            # 2 x 2, m = 4 box
    assert not resident_fits(2048 + 2 * 84, 8192)                         # 1-D middle rank, m = 8
    assert not resident_fits(8192, 8192) and not resident_fits(4096, 8192)
    cfg = HeatConfig(nx=8192, ny=8192, steps=0, backend="cpu")
    two_by_two = predict(cfg.replace(px=2, py=2, halo_passes=4), 4)
    slabs = predict(cfg.replace(decomp="rows", halo_passes=8), 4)
    assert two_by_two["resident"] and not slabs["resident"]
    assert two_by_two["ms_per_1000"] < slabs["ms_per_1000"]


class _FakeSolver:
    """Stands in for HeatSolver: construction outcome and run outcome chosen
    per candidate schedule."""
    aborted = []

    def __init__(self, cfg, fail_make=False, fail_run=False, clean=False, giveup=False):
        if fail_make:
            raise _native.NativeError("block thinner than its halo")
        self.cfg, self.fail_run, self.clean, self.giveup = cfg, fail_run, clean, giveup
        self.info = type("I", (), {"halo": 12, "tb_depth": 12})()

    def run(self, n):
        if self.fail_run:
            # The native run() prefixes "[clean]" when the rank's queued work
            # completed and the communicator was kept.
            raise _native.NativeError(("[clean] " if self.clean else "") +
                                      "planner check failed mid-run")
        return type("R", (), {"resident_giveups": int(self.giveup)})()

    def abort(self):
        _FakeSolver.aborted.append(self.cfg.schedule)

    def close(self):
        pass


def _tune(fails):
    from parallel_heat_amd.parallel.comm import DistInfo
    from parallel_heat_amd.parallel.tune import autotune
    cfg = HeatConfig(nx=64, ny=64, backend="cpu")
    cands = [cfg.replace(schedule=s) for s in ("sync", "pipeline", "overlap")]
    make = lambda c: _FakeSolver(c, **fails.get(c.schedule, {}))  # noqa: E731
    return autotune(cfg, DistInfo(0, 1, 0), candidates=cands, steps=2, repeats=1, make=make)


def test_autotune_skips_a_candidate_rejected_at_construction():
    best, table = _tune({"sync": dict(fail_make=True)})
    assert "error" in table[0] and "ms_per_1000_iters" in table[1]
    assert best.schedule in ("pipeline", "overlap")


def test_autotune_aborts_on_a_run_time_failure():
    # The shared communicator may hold unmatched ops after a mid-run failure:
    # the transport is aborted and no later candidate runs.
    _FakeSolver.aborted.clear()
    with pytest.raises(_native.NativeError, match="autotune aborted"):
        _tune({"pipeline": dict(fail_run=True)})
    assert _FakeSolver.aborted == ["pipeline"]


def test_autotune_skips_a_clean_run_time_failure():
    # A failure every rank meets at the same point with the communicator
    # intact ("[clean]") skips the candidate instead of ending the autotune.
    _FakeSolver.aborted.clear()
    best, table = _tune({"pipeline": dict(fail_run=True, clean=True)})
    assert _FakeSolver.aborted == []
    assert "[clean]" in table[1]["error"] and "ms_per_1000_iters" not in table[1]
    assert best.schedule in ("sync", "overlap")


def test_autotune_skips_a_resident_giveup():
    # HEAT_TB_RES_GIVEUP=defer: a run whose resident tiles gave up returns
    # resident_giveups = 1 (results invalid); the candidate is not timed.
    _FakeSolver.aborted.clear()
    best, table = _tune({"sync": dict(giveup=True)})
    assert "gave up" in table[0]["error"] and _FakeSolver.aborted == []
    assert best.schedule in ("pipeline", "overlap")


def _tune_worker(rank, world, port, out):
    import os
    import torch.distributed as dist
    from parallel_heat_amd.parallel.comm import DistInfo
    from parallel_heat_amd.parallel.tune import autotune
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = HeatConfig(nx=64, ny=64, backend="cpu")
    cands = [cfg.replace(schedule=s) for s in ("sync", "pipeline", "overlap")]
    # Rank 1 alone gives up on "sync"; both ranks fail cleanly on "pipeline".
    fails = {"pipeline": dict(fail_run=True, clean=True)}
    if rank == 1:
        fails["sync"] = dict(giveup=True)
    make = lambda c: _FakeSolver(c, **fails.get(c.schedule, {}))  # noqa: E731
    best, table = autotune(cfg, DistInfo(rank, world, rank), candidates=cands, steps=2,
                           repeats=1, make=make)
    with open(out, "w") as f:
        f.write(best.schedule + "\n" + "|".join(str("error" in r) for r in table))
    dist.destroy_process_group()


def test_autotune_two_ranks_agree_on_skips(tmp_path):
    import torch.multiprocessing as mp
    from .dist_worker import free_port
    port = free_port()
    outs = [str(tmp_path / f"r{r}.txt") for r in range(2)]
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=_tune_worker, args=(r, 2, port, outs[r])) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(120)
        assert p.exitcode == 0
    got = [open(o).read().split("\n") for o in outs]
    assert got[0] == got[1] == ["overlap", "True|True|False"]


def test_fit_exchange_and_prune_from_measurements():
    # Latency and link bandwidth fitted from measured (bytes, seconds) samples
    # (median per size) replace the stated constants in predict() and prune().
    from parallel_heat_amd.parallel.model import XGMI, fit_exchange, predict, prune
    sizes = (3_000_000, 1_500_000, 750_000)
    pts = [(b, 12e-6 + b / 20e9) for b in sizes for _ in range(4)]
    pts.append((750_000, 5e-3))  # one outlier sample: the median ignores it
    x = fit_exchange(pts)
    assert x["fit_ok"] and x["fit_r2"] > 0.999
    assert abs(x["link_gbps"] - 20.0) < 0.01 and abs(x["latency_us"] - 12.0) < 0.01
    assert x["measured"][-1] == [3_000_000, round(pts[0][1] * 1e6, 3)]
    assert XGMI["link_gbps"] == 50.0  # the stated model is untouched
    cfg = HeatConfig(nx=8192, ny=8192, steps=0, backend="cpu")
    cands = default_candidates(cfg, 8, schedules=["sync", "pipeline"], halo_passes=[0, 4])
    p_stated, p_meas = predict(cands[0], 8), predict(cands[0], 8, xgmi=x)
    assert p_meas["exchange_ms"] > p_stated["exchange_ms"]
    # Very slow links (1 GB/s) make the 1-D slabs' 3 MB messages the cost:
    # the 2-D grid's smaller messages win; the slabs' candidates fall outside
    # the slack, but the best one of each (layout, halo passes) is still timed.
    slow = fit_exchange([(b, b / 1e9 + 1e-6) for b in sizes])
    assert slow["fit_ok"]
    kept = [tuple(describe(c, 8).values()) for c in prune(cands, 8, xgmi=slow)]
    assert {(k[0], k[1], k[3]) for k in kept} == {(8, 1, 0), (8, 1, 4), (4, 2, 0), (4, 2, 4)}
    assert len(kept) < len(cands)


def test_fit_exchange_rejects_round5_rehearsal_points():
    # The round-5 8-rank rehearsal (8 RCCL ranks on one GPU over sockets)
    # measured 19,942 us at 0.83 MB and 17,799 us at 3.3 MB: a negative
    # slope.  Its fit then kept 50 GB/s, set the latency to 20.6 ms and
    # pruned four candidates untimed.  Now: not trusted, nothing pruned.
    from parallel_heat_amd.parallel.model import XGMI, fit_exchange, prune
    pts = [(829440, 19942.334e-6), (3317760, 17799.033e-6)]
    x = fit_exchange(pts)
    assert not x["fit_ok"] and "sizes" in x["fit_reason"]
    assert x["latency_us"] == XGMI["latency_us"] and x["link_gbps"] == XGMI["link_gbps"]
    three = fit_exchange(pts + [(1658880, 21000e-6)])
    assert not three["fit_ok"] and three["fit_reason"] == "non-positive slope"
    noisy = fit_exchange([(1e6, 50e-6), (2e6, 20e-6), (3e6, 90e-6), (4e6, 60e-6)])
    assert not noisy["fit_ok"] and noisy["fit_reason"].startswith("R^2")
    cfg = HeatConfig(nx=8192, ny=8192, steps=0, backend="cpu")
    cands = default_candidates(cfg, 8, schedules=["sync", "pipeline"], halo_passes=[0, 4])
    for bad in (x, three, noisy):
        assert prune(cands, 8, xgmi=bad) == cands


def test_measure_exchange_interleaves_three_sizes():
    from parallel_heat_amd.parallel.tune import exchange_depths, measure_exchange
    assert exchange_depths(96) == [24, 48, 96] and exchange_depths(2) == [1, 2]
    calls = []

    class S:
        info = type("I", (), {"halo": 96})()

        def time_exchange(self, d, iters):
            calls.append((d, iters))
            return 1e-5 * d, d * 1000

    pts = measure_exchange(S(), exchange_depths(96), iters=20, reps=5)
    assert len(pts) == 15 and calls[:3] == [(24, 20), (48, 20), (96, 20)]
    assert {b for b, _ in pts} == {24000, 48000, 96000}


def test_resident_aware_halo_passes_model():
    # The solver's resident-aware m (topology.cpp resident_halo_passes,
    # mirrored by the model): 2 x 2 at 8192^2 -> m = 5 (4144-cell span boxes
    # in 20 x 16 tiles; m = 8 gives 4180, which has no one-round plan); the
    # 1-D 4-rank slabs fit only at m = 2 (< RES_MIN_PASSES: m = 8 streaming);
    # 8 ranks take m = 7: at m = 8 the 1192-row (1-D) / 2216 x 4180 (4 x 2)
    # boxes fall from 12 x 16 tiles to 14 x 8 ones, -10 % per owned cell.
    from parallel_heat_amd.parallel.model import RES_MIN_PASSES, predict, resident_halo_passes
    assert resident_halo_passes(8192, 8192, 2, 2) == 5
    assert resident_halo_passes(8192, 8192, 4, 1) == 2 < RES_MIN_PASSES
    assert resident_halo_passes(8192, 8192, 8, 1) == 7
    assert resident_halo_passes(8192, 8192, 4, 2) == 7
    assert resident_halo_passes(8192, 8192, 2, 1) == 0  # 4096 x 8192 has no resident plan
    cfg = HeatConfig(nx=8192, ny=8192, steps=0, backend="cpu")
    p = predict(cfg.replace(decomp="auto"), 4)
    assert p["layout"] == "2x2" and p["halo"] == 60 and p["resident"]
    assert p["tcells_per_s"] > 15.0  # m = 5 spans: 5.29 / (1 + 0.7 / 5) per rank
    rows = predict(cfg.replace(decomp="rows"), 4)
    assert rows["halo"] == 96 and not rows["resident"]

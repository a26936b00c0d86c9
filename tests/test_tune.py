"""Candidate set of the multi-GPU autotune (parallel/tune.py) as bench.py
builds it: rows slabs and the MPI_Dims_create grid, x deep-halo sync with the
default and a doubled exchange interval, x the boundary-first pipeline."""
from parallel_heat_amd import HeatConfig
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

"""Chained level-split passes (tb_chain.hip, tb_chain_kernel): one launch runs
the unchecked depth-12 passes of a one-rank segment with per-unit flags
instead of a grid-wide boundary between passes.  Every case is bitwise
against the same run with one launch per pass (HEAT_TB_CHAIN=0), which the
kernel tests hold bitwise against the CPU oracle.  Needs an MI355X."""
import os

import numpy as np
import pytest

from parallel_heat_amd import HeatConfig, HeatSolver, ops

pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("exp_kernels")]


def _run(cfg, chain, nt=-1):  # chain: HEAT_TB_CHAIN=1 (opt-in) or 0
    old = os.environ.get("HEAT_TB_CHAIN")
    os.environ["HEAT_TB_CHAIN"] = "1" if chain else "0"
    saved = ops.tb_tuning()
    try:
        if nt >= 0:
            t = ops.tb_tuning()
            t.nt = nt
            ops.set_tb_tuning(t)
        with HeatSolver(cfg) as s:
            r = s.run()
            return r, s.checksum(), s.gather()
    finally:
        ops.set_tb_tuning(saved)
        if old is None:
            del os.environ["HEAT_TB_CHAIN"]
        else:
            os.environ["HEAT_TB_CHAIN"] = old


def _same(a, b):
    ra, ca, ga = a
    rb, cb, gb = b
    assert ra.steps_done == rb.steps_done and ra.converged_at == rb.converged_at
    assert ca["hash"] == cb["hash"]  # (the double sum's order varies; the hash is exact)
    assert np.array_equal(ga, gb)


@pytest.mark.parametrize("steps", [120, 132, 1000])
def test_chain_8192_bitwise(gpu, steps):
    # 8192^2 (268 MB: streaming rows): 10 / 11 chained passes, and the
    # bench's 1000 = 82 x 12 + 8 + 8 (the two depth-8 passes per launch).
    cfg = HeatConfig(nx=8192, ny=8192, steps=steps, init="random", seed=5, backend="hip", device=0)
    on = _run(cfg, True)
    assert on[0].chained_passes >= steps // 12 - 2
    off = _run(cfg, False)
    assert off[0].chained_passes == 0
    _same(on, off)


def test_chain_forced_streaming_small_plate(gpu):
    # 4096 x 8192 with the streaming build forced (TbTuning.nt = 1): an odd
    # pass count (the last pass writes the other field) and a plate-edge mix.
    cfg = HeatConfig(nx=4096, ny=8192, steps=7 * 12, init="random", seed=9, backend="hip", device=0)
    on = _run(cfg, True, nt=1)
    assert on[0].chained_passes == 7
    _same(on, _run(cfg, False, nt=1))


def test_chain_with_checks_converges_alike(gpu):
    # Convergence checks every 50 steps (device-judged): the check passes run
    # alone, the passes between them chained; same converging step, field.
    cfg = HeatConfig(nx=8192, ny=8192, steps=600, init="ref-wrap", converge=True, check_interval=50,
                     eps=1e30, backend="hip", device=0)
    on = _run(cfg, True)
    off = _run(cfg, False)
    assert on[0].converged and on[0].converged_at == off[0].converged_at
    _same(on, off)
    cfg2 = cfg.replace(eps=1e-3, steps=300)
    on2, off2 = _run(cfg2, True), _run(cfg2, False)
    assert on2[0].chained_passes > 0
    _same(on2, off2)


def test_chain_l2_sized_plate_stale_lines(gpu, monkeypatch):
    # a chained unit reads rows another unit (maybe on another
    # XCD) wrote in the same launch; the smallest plate the chained
    # level-split passes run on (2048 x 8192, 64 MB: 72 strip-rows per SIMD,
    # the split pipelines' threshold; resident spans off) with the streaming
    # build forced and 24 passes per launch, where lines an XCD's L2 kept
    # from an earlier pass are most likely to be hit.  The chain build's row
    # loads are sc1 now (tb_stream.inl ld_in).
    monkeypatch.setenv("HEAT_TB_RESIDENT", "0")
    cfg = HeatConfig(nx=2048, ny=8192, steps=24 * 12, init="random", seed=13, backend="hip",
                     device=0)
    on = _run(cfg, True, nt=1)
    assert on[0].chained_passes > 0
    _same(on, _run(cfg, False, nt=1))
